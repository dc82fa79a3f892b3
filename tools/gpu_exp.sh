set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_w4a8.py -q -x -m gpu -k "patch or conv or embed or neck" > gpurun_out/g18_tests.log 2>&1 || exit $?
for lib in old_conv new; do
  for mode in w4a8 w4a16; do
    SAMQ_LIB=$PWD/sam-quantization_amd/build_ab/$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/g18_${lib}_$mode -o run --output-format csv -- python3 bench.py --mode $mode --steps 5 --warmup 2 --no-cpu-baseline --no-isolated > gpurun_out/g18_${lib}_$mode.log 2>&1 || exit $?
  done
done
