#!/bin/bash
# round 4: swizzled epilogue staging (int8 + f16 outputs of the int8 GEMMs, f16 outputs of the
# W4A16 ping-pong): exactness tests, PMC conflicts, bench A/B vs the build before; global attention
# DMA-between-Q.K^T variant
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
o=gpurun_out/r4_p
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_w8a8.py tests/test_w4a8.py tests/test_gpu_kernels.py -m gpu -k "w8a8 or w4a8_gemm or stage_local or (pingpong and (57 or 64 or 111)) or persistent_matches or w4a16_gemm" > $o.tests.log 2>&1 || { tail -40 $o.tests.log; exit 1; }
tail -2 $o.tests.log
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $o.pmc -o p -- python3 tools/bench_i8.py --m 16384 --cfgs 86 --iters 3 > $o.pmc.log 2>&1 || { tail -5 $o.pmc.log; exit 1; }
python3 tools/pmc_kernel_counters.py $o.pmc i8_gemm_pp2 | grep -E "i8_gemm|CONFLICT|GRBM"
SAMQ_LIB=tuning timeout -k 10 200 python -u tools/attn_variant_ab.py 0,4096 2 8 > $o.gvar.log 2>&1 || { tail -20 $o.gvar.log; exit 1; }
cat $o.gvar.log
for r in 1 2; do
  for lib in tools/ab/libsamq_pre_swz.so new; do
    if [ $lib = new ]; then unset SAMQ_LIB; else export SAMQ_LIB=$lib; fi
    for m in w4a16 w4a8 w8a8; do
      st=20; [ $m = w4a8 ] && st=10
      timeout -k 10 300 python -u bench.py --mode $m --steps $st --warmup 3 --no-cpu-baseline --no-isolated > $o.b.$m.$r.$(basename $lib).log 2>&1 || exit 1
      echo "$m $lib $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" $o.b.$m.$r.$(basename $lib).log)"
    done
  done
done
