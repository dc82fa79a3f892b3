set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/g19_pmc -o p1 -- python3 tools/bench_gemm.py --m 65536 --cfgs 57,64 --shapes qkv,lin1,lin2,proj --iters 2 > gpurun_out/g19_pmc.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/bench_gemm.py --m 65536 --cfgs 57,64 --shapes qkv,lin1,lin2,proj --iters 5 > gpurun_out/g19_time.log 2>&1
