#!/bin/bash
# tools/gpu_session.sh TAG STEP [STEP ...] — the GPU-box steps of a session, one script for all
# rounds (replaces the per-session tools/gpu_r0x*.sh of rounds 1-4).  Run on the box through
#   gpurun --timeout 1200 -- 'bash tools/gpu_session.sh r05a suite smoke bench'
# Steps:
#   suite          the whole GPU test suite (pytest -m gpu), -s: C-level stderr (HIP / ROCr
#                  messages, std::terminate text) goes to the log instead of pytest's fd capture
#   tests:<expr>   pytest -m gpu -k <expr>
#   smoke          __graft_entry__.smoke()
#   bench          the driver's command: python bench.py --steps 20 --warmup 5 (+ its wall time)
#   bench-default  python bench.py
#   rocprof        the headline under rocprofv3 --kernel-trace --stats (no variants / legs / CPU baseline)
#   pmc            PMC HBM-traffic passes of the headline SpMV (tools/pmc_spmv.sh) + SQ passes (tools/pmc_vibm.sh)
#   py:<script>    python tools/<script> (an A/B script; its arguments after a second colon, separated
#                  by @: py:spmv_ab.py:--grid@256)
#   kprof:<script> the same under rocprofv3 --kernel-trace --stats (per-kernel averages in
#                  gpurun_out/<TAG>_kprof<step>/)
# Every step has its own timeout and its own log, named with the step and the box's clock, so a
# failing attempt is never overwritten by a later one (gpurun merges gpurun_out/ back by name).
# The session stops at the first failing step: nothing more runs on the GPU after a fault, an abort
# or a timeout.
set -uo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:?usage: gpu_session.sh TAG STEP...}
shift
STAMP=$(date +%H%M%S)

run() {  # run NAME TIMEOUT OUTFILE CMD...  (stdout to OUTFILE, stderr to the .log beside it)
  local name=$1 to=$2 out=$3
  shift 3
  local t0=$SECONDS rc
  echo "[$(date +%T)] $name: $*" | tee -a "gpurun_out/${TAG}_${STAMP}_session.log"
  timeout -k 10 "$to" "$@" > "$out" 2> "${out%.*}.err"
  rc=$?
  echo "[$(date +%T)] $name: rc=$rc, $((SECONDS - t0)) s" | tee -a "gpurun_out/${TAG}_${STAMP}_session.log"
  if [ $rc -ne 0 ]; then
    tail -n 30 "$out" "${out%.*}.err"
    exit $rc
  fi
}

idx=0
for step in "$@"; do
  idx=$((idx + 1))
  name=${step%%@*}
  base="gpurun_out/${TAG}_${STAMP}_${idx}_${name//[:,\/ ]/_}"
  case "$step" in
    suite)
      AMD_LOG_LEVEL=1 run suite 1100 "$base.log" python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider \
        --timeout 400 --timeout-method thread ;;
    tests:*)
      AMD_LOG_LEVEL=1 run tests 900 "$base.log" python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider \
        --timeout 400 --timeout-method thread -k "${step#tests:}" ;;
    smoke)
      run smoke 180 "$base.log" python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    bench)
      t0=$SECONDS
      run bench 700 "$base.json" python bench.py --steps 20 --warmup 5
      echo "$((SECONDS - t0)) s wall (python bench.py --steps 20 --warmup 5)" > "$base.wall" ;;
    bench-default)
      run bench-default 600 "$base.json" python bench.py ;;
    rocprof)
      run rocprof 600 "$base.json" rocprofv3 --kernel-trace --stats -d "gpurun_out/${TAG}_prof" -o run \
        --output-format csv -- python3 bench.py --variants '' --config5 0 --bending 0 --cpu-grid 0 ;;
    kprof:*)  # kprof:<script>:<args @-separated>: the script under rocprofv3 --kernel-trace --stats
      spec=${step#kprof:}
      script=${spec%%:*}
      args=""
      [ "$spec" != "$script" ] && args=${spec#*:}
      run "kprof-$script" 600 "$base.log" rocprofv3 --kernel-trace --stats -d "gpurun_out/${TAG}_kprof${idx}" -o run \
        --output-format csv -- python3 "tools/$script" ${args//@/ } ;;
    pmc)
      run pmc-hbm 600 "$base.log" bash tools/pmc_spmv.sh aij-vi 256
      run pmc-sq 600 "${base}_sq.log" bash tools/pmc_vibm.sh ;;
    py:*)
      spec=${step#py:}
      script=${spec%%:*}
      args=""
      [ "$spec" != "$script" ] && args=${spec#*:}
      run "$script" 900 "$base.log" python -u "tools/$script" ${args//@/ } ;;
    *)
      echo "unknown step $step" >&2
      exit 2 ;;
  esac
done
