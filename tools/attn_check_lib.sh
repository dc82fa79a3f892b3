# attention parity tests against a variant library: tools/attn_check_lib.sh build_ab/x.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
SAMQ_LIB=$PWD/sam-quantization_amd/$1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -m gpu -k "attention" --timeout 120 --timeout-method thread > gpurun_out/attn_tests_lib.log 2>&1 || { tail -30 gpurun_out/attn_tests_lib.log; exit 1; }
tail -1 gpurun_out/attn_tests_lib.log
