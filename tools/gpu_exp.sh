set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests/test_w8a8.py -q -x -m gpu > gpurun_out/g11_tests.log 2>&1 || exit $?
BENCH_ARGS="--mode w8a8 --steps 40 --warmup 5" timeout -k 10 600 bash tools/bench_variants.sh build_ab/old_q8.so build_ab/new.so > gpurun_out/g11_var88.log 2>&1 || exit $?
BENCH_ARGS="--mode w8a8 --steps 40 --warmup 5" timeout -k 10 600 bash tools/bench_variants.sh build_ab/old_q8.so build_ab/new.so >> gpurun_out/g11_var88.log 2>&1
