set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/g20_pmc -o p1 -- python3 tools/bench_attn.py --batch 2 --iters 5 > gpurun_out/g20_pmc.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/g20_pmc2 -o p2 -- python3 tools/bench_attn.py --batch 2 --iters 5 > gpurun_out/g20_pmc2.log 2>&1 || true
timeout -k 10 120 python3 tools/bench_attn.py --batch 2 --iters 20 > gpurun_out/g20_time.log 2>&1
