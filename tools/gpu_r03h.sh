# round-3 (h): cg_rev A/B at 256^3 and 128^3 + the p-update bitwise tests
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 180 python -u tools/cg_ab.py --grid 256 --option cg_rev --values 0,1 --rounds 4 > gpurun_out/r03h_cg_ab_rev256.log 2>&1
timeout -k 10 120 python -u tools/cg_ab.py --grid 128 --option cg_rev --values 0,1 --rounds 4 > gpurun_out/r03h_cg_ab_rev128.log 2>&1
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -k "pdb" -x -v --timeout 120 --timeout-method thread > gpurun_out/r03h_pytest_pdb.txt 2>&1
