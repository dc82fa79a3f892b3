set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 240 python tools/bench_gemm.py --m 8192 --cfgs 57,52,64,53 --iters 20 > gpurun_out/g12_m8192.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_gemm.py --m 65536 --cfgs 57,52,64,53 --iters 5 > gpurun_out/g12_m65536.log 2>&1 || exit $?
timeout -k 10 400 python tools/bench_cfg_ab.py 2 8 "te_all:qkv=52,lin1=52,proj=53,lin2=53;te_wide:qkv=52,lin1=52;te_narrow:proj=53,lin2=53" > gpurun_out/g12_ab.log 2>&1
