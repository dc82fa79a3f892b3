set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 240 python tools/bench_gemm.py --m 8192 --cfgs 57,64,32,33 --iters 20 > gpurun_out/g4_m8192.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_gemm.py --m 65536 --cfgs 57,64,32,33 --iters 5 > gpurun_out/g4_m65536.log 2>&1 || exit $?
