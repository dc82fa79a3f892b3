set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu -rA > gpurun_out/r3_gputests_a52412a85860.log 2>&1; rc=$?; tail -3 gpurun_out/r3_gputests_a52412a85860.log; exit $rc
