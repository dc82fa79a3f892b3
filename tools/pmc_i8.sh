#!/bin/bash
# PMC counter breakdown of the W4A8 int8 ping-pong GEMM (i8_gemm_pp2, cfg 86) and its timing-only
# no-epilogue twin (cfg 94, tuning build) on the ViT-H shapes at M = 16384 (tools/bench_i8.py):
# one rocprofv3 --pmc pass per counter group, no traces -> gpurun_out/pmc_i8_summary.txt
# usage: tools/pmc_i8.sh [cfgs, default 86,94]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export SAMQ_LIB=tuning
d=gpurun_out/pmc_i8
rm -rf $d
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $d -o pass$i -- python3 tools/bench_i8.py --m 16384 --cfgs ${1:-86,94} --iters 3 > $d.pass$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 $d.pass$i.log; exit 1; }
done
python3 tools/pmc_kernel_counters.py $d i8_gemm_pp2 > gpurun_out/pmc_i8_summary.txt || exit 1
head -80 gpurun_out/pmc_i8_summary.txt
