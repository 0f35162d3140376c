mkdir -p gpurun_out && export TMPDIR=/tmp && \
timeout -k 10 180 python -u tools/cg_ab.py --grid 256 --option cg_par --values 0,1 --rounds 4 > gpurun_out/r03d_cg_ab_par.log 2>&1 && \
timeout -k 10 180 python -u tools/cg_ab.py --grid 256 --option cg_fold --values 0,1 --rounds 4 --set cg_par=1 > gpurun_out/r03d_cg_ab_fold.log 2>&1 && \
timeout -k 10 120 python -u tools/cg_ab.py --grid 128 --option cg_fold --values 0,1 --rounds 4 --set cg_par=1 > gpurun_out/r03d_cg_ab_fold128.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -k "pdb" -x -v --timeout 120 --timeout-method thread > gpurun_out/r03d_pytest_pdb.txt 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 -- python3 tools/bench_nonlinear.py --grid 128 --ts 3 > gpurun_out/r03d_c5_prof.json 2>&1 && \
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03d_pytest_gpu.txt 2>&1
