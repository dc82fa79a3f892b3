#!/bin/bash
# PMC counter groups of the W8A8 attention kernels (tools/bench_attn_q8.py), one rocprofv3 --pmc pass
# per group under its own limit -> gpurun_out/pmc_attn_q8.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp
d=gpurun_out/pmc_attn_q8
rm -rf $d
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $d -o p$i -- python3 tools/bench_attn_q8.py --iters 2 \
    > gpurun_out/pmc_attn_q8_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_attn_q8_$i.log; exit 1; }
done
python3 tools/pmc_kernel_counters.py $d > gpurun_out/pmc_attn_q8.txt && cat gpurun_out/pmc_attn_q8.txt
