set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python tools/bench_cfg_ab.py 2 14 "all59:qkv=59,lin1=59,proj=59,lin2=59;all64:qkv=64,lin1=64,proj=64,lin2=64;wide59:qkv=59,lin1=59" > gpurun_out/g15_ab.log 2>&1
