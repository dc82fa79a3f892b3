set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py tests/test_w4a8.py -q -x -m gpu > gpurun_out/g8_tests.log 2>&1 || exit $?
for lib in old new; do
  SAMQ_LIB=$PWD/sam-quantization_amd/build_ab/$lib.so timeout -k 10 200 python tools/bench_gemm.py --m 8192 --cfgs 57 --shapes lin1,qkv --iters 20 > gpurun_out/g8_$lib.log 2>&1 || exit $?
done
timeout -k 10 600 bash tools/bench_variants.sh build_ab/old.so build_ab/new.so > gpurun_out/g8_var.log 2>&1 || exit $?
BENCH_ARGS="--mode w4a8 --steps 10 --warmup 3" timeout -k 10 600 bash tools/bench_variants.sh build_ab/old_i8.so build_ab/new.so > gpurun_out/g8_var48.log 2>&1
