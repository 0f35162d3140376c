# round-3 (g): cg_rev A/B + pdb tests, then final-code measurements — bench, bench under rocprofv3,
# PMC traffic of the SpMV, config 5 under rocprofv3
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python -u tools/cg_ab.py --grid 256 --option cg_rev --values 0,1 --rounds 4 > gpurun_out/r03g_cg_ab_rev256.log 2>&1
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "pdb" -x -v --timeout 120 --timeout-method thread > gpurun_out/r03g_pytest_pdb.txt 2>&1
bash tools/profile_round.sh r03g
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r03g_prof_c5 -o c5 --output-format csv -- \
  python3 tools/bench_nonlinear.py --grid 128 --ts 3 > gpurun_out/r03g_config5_under_rocprof.json 2> gpurun_out/r03g_config5_rocprof.log
