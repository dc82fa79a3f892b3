#!/bin/bash
# One GPU-box session: each GPU step under its own time limit; a crash / abort / timeout
# (exit status other than 0 = pass or 1 = test failures) stops the session immediately.
# usage: tools/gpu_session.sh <step> [<step> ...]   steps: kernels encoder gpu bench smoke instep prof
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "=== [$name] $(date +%T) start" | tee -a gpurun_out/session.log
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== [$name] $(date +%T) rc=$rc" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping session after rc=$rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
}
for step in "$@"; do
  case $step in
    kernels) run kernels 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -rA ;;
    w8a8)    run w8a8 600 python -m pytest tests/test_w8a8.py -q -m gpu -s -rA ;;
    w4a8)    run w4a8 600 python -m pytest tests/test_w4a8.py -q -m gpu -s -rA ;;
    encoder) run encoder 700 python -m pytest tests/test_gpu_encoder.py -q -m gpu -s -rA ;;
    gpu)     run gputests 900 python -m pytest tests -q -m gpu -s -rA ;;
    smoke)   run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   run bench 500 python bench.py --steps 20 --warmup 5 ;;
    bench48) run bench_w4a8 600 python bench.py --mode w4a8 --steps 10 --warmup 3 ;;
    bench88) run bench_w8a8 600 python bench.py --mode w8a8 --steps 20 --warmup 5 ;;
    b48q)    run b48q 400 python bench.py --mode w4a8 --steps 10 --warmup 3 --no-cpu-baseline ;;
    b88q)    run b88q 400 python bench.py --mode w8a8 --steps 20 --warmup 5 --no-cpu-baseline ;;
    benchq)  run benchq 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    instep)  run instep 500 bash tools/instep_profile.sh w4a16 ;;
    benchg)  run benchg 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --groupsize 128 ;;
    instepg) run instepg 500 bash tools/instep_profile.sh w4a16 --groupsize 128 ;;
    grouped) run grouped 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -rA -k "grouped or auto_pick or configs" ;;
    instep48) run instep48 500 bash tools/instep_profile.sh w4a8 ;;
    instepb8) run instepb8 500 bash tools/instep_profile.sh w4a16 --batch 8 ;;
    instep88) run instep88 500 bash tools/instep_profile.sh w8a8 ;;
    prof)    run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
