#!/bin/bash
# PMC passes (one counter group per rocprofv3 run) over the GEMM micro-benchmark.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CFG=${1:-22}; SHAPE=${2:-qkv}
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_INSTS_SALU GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum FETCH_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_$CFG_$SHAPE -o pass$i -- python3 tools/bench_gemm.py --cfgs $CFG --shapes $SHAPE --iters 3 > gpurun_out/pmc_pass$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 gpurun_out/pmc_pass$i.log; exit 1; }
done
echo pmc done
