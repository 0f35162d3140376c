# round-3 (d) GPU session: full GPU suite, config-5 kernel profile, default bench
mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03d_pytest_gpu.txt 2>&1 && \
timeout -k 10 120 python -u tools/cg_ab.py --grid 128 --option cg_par --values 0,1 --rounds 4 > gpurun_out/r03d_cg_ab_par128.log 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 --output-format csv -- python3 tools/bench_nonlinear.py --grid 128 --ts 3 > gpurun_out/r03d_c5_prof.json 2>&1 && \
timeout -k 10 400 python -u bench.py > gpurun_out/r03d_bench.json 2> gpurun_out/r03d_bench.log
