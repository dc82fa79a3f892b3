#!/bin/bash
# One GPU-box session (the single runner for every gpurun call): each GPU step under its own time
# limit; a crash / abort / timeout (exit status other than 0 = pass or 1 = test failures) stops
# the session immediately, and no step is retried.
# usage: tools/gpu_session.sh <tag> <step> [<step> ...]       logs: gpurun_out/<tag>.<step>.log
# steps:
#   gpu                    whole GPU suite (-s -rA: the [parity] lines are kept)
#   kernels|w8a8|w4a8|encoder|decoder   one GPU test file
#   k=<pytest -k expr>     GPU tests selected by -k
#   smoke                  __graft_entry__.smoke()
#   bench | bench48 | bench88 | benchg       full bench lines (w4a16 / w4a8 / w8a8 / G=128)
#   benchq | b48q | b88q   bench lines without CPU baseline
#   instep | instep48 | instep88 | instepg   rocprofv3 in-step kernel traces (tools/instep_profile.sh)
#   instep8                the same for config 4's per-GPU geometry (B = 8, 4 lanes: the N > 1 line's roofline)
#   rehearse               the N = 2 bench line on this one GPU (gloo, both ranks on cuda:0)
#   pmc                    PMC HBM traffic of every mode (tools/pmc_all.sh)
#   publish=<round>        copy this build's in-step traces and the PMC summaries (wrapped with their
#                          source line as profiles/<round>_pmc_traffic_<mode>_m<rows>.json) into
#                          profiles/, so later bench steps in the same call quote them; copies of
#                          them come back in gpurun_out/publish_<round>/ (raw trace dirs removed)
#   attnpmc                attention counters (tools/attn_pmc.sh)
#   pmci8[=<cfgs>]         int8 GEMM counters (tools/pmc_i8.sh; default cfgs 86,94)
#   i8=<cfgs>@<m>          int8 GEMM tile configs (tools/bench_i8.py, tuning library)
#   w4=<cfgs>@<m>          W4A16 GEMM tile configs (tools/bench_gemm.py, tuning library)
#   w4g=<cfgs>@<m>         the same with G = 128 grouped weights
#   ab48=<variants>        in-graph W4A8 per-layer cfg A/B (tools/bench_cfg_ab_w4a8.py, tuning library)
#   ab16=<variants>        in-graph W4A16 per-layer cfg A/B (tools/bench_cfg_ab.py, tuning library)
#   ab16g=<variants>       the same with G = 128 grouped weights (product library)
#   ab88=<variants>        in-graph W8A8 per-layer cfg A/B (tools/bench_cfg_ab_w8a8.py, tuning library)
#   abl=<mode>@<lib.so>    bench <mode> alternating this build and <lib.so> (SAMQ_LIB), 2 rounds each
#   ablg=<lib.so>          W4A16 G = 128 bench alternating this build and <lib.so>, 3 rounds each
#   lanes=<mode>@<l1,l2..> bench <mode> at each lane count (2 rounds each, alternating)
#   attn                   attention kernels isolated (tools/bench_attn.py)
#   attnq8                 W8A8 attention kernels isolated (tools/bench_attn_q8.py)
#   attnq8pmc              W8A8 attention counters (tools/attn_q8_pmc.sh)
#   attnq8prof             W8A8 attention kernel trace (per-kernel durations, rocprofv3 --stats)
#   probe                  v_cvt_pk_u8_f32 semantics (tools/probe_cvt_u8.hip, built on the box)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:?tag}
shift
run() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  local log="gpurun_out/$tag.$name.log"
  echo "=== [$name] $(date +%T) start" | tee -a "gpurun_out/$tag.session.log"
  timeout -k 10 "$secs" "$@" > "$log" 2>&1
  local rc=$?
  echo "=== [$name] $(date +%T) rc=$rc" | tee -a "gpurun_out/$tag.session.log"
  tail -n 25 "$log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping session after rc=$rc" | tee -a "gpurun_out/$tag.session.log"
    exit $rc
  fi
}
PYT="python -u -m pytest -x --timeout 200 --timeout-method thread -m gpu -s -rA"
for step in "$@"; do
  arg=${step#*=}
  case $step in
    gpu)      run gputests 1100 $PYT -q tests ;;
    kernels)  run kernels 600 $PYT -q tests/test_gpu_kernels.py ;;
    w8a8)     run w8a8 600 $PYT -q tests/test_w8a8.py ;;
    w4a8)     run w4a8 600 $PYT -q tests/test_w4a8.py ;;
    encoder)  run encoder 700 $PYT -q tests/test_gpu_encoder.py ;;
    decoder)  run decoder 600 $PYT -q tests/test_sam_decoder.py ;;
    k=*)      run k_$(echo "$arg" | tr -c 'a-zA-Z0-9' '_') 900 $PYT -q tests -k "$arg" ;;
    smoke)    run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)    run bench 600 python bench.py --steps 20 --warmup 5 ;;
    bench48)  run bench48 600 python bench.py --mode w4a8 --steps 10 --warmup 3 ;;
    bench88)  run bench88 600 python bench.py --mode w8a8 --steps 20 --warmup 5 ;;
    benchg)   run benchg 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --groupsize 128 ;;
    benchq)   run benchq 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    b48q)     run b48q 400 python bench.py --mode w4a8 --steps 10 --warmup 3 --no-cpu-baseline ;;
    b88q)     run b88q 400 python bench.py --mode w8a8 --steps 20 --warmup 5 --no-cpu-baseline ;;
    instep)   run instep 500 bash tools/instep_profile.sh w4a16 ;;
    instep48) run instep48 500 bash tools/instep_profile.sh w4a8 ;;
    instep88) run instep88 500 bash tools/instep_profile.sh w8a8 ;;
    instepg)  run instepg 500 bash tools/instep_profile.sh w4a16 --groupsize 128 ;;
    instep8)  run instep8 500 bash tools/instep_profile.sh w4a16 --batch 8 ;;
    rehearse) run rehearse 600 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 ;;
    pmc)      run pmc 900 bash tools/pmc_all.sh ;;
    publish=*) H=$(python3 -c "import bench; print(bench.source_hash())")
              cp gpurun_out/instep_*_"$H".json gpurun_out/instep_*_"$H"_wholerun_stats.csv profiles/ || exit 1
              for mr in w4a16:8192 w4a8:16384 w8a8:4096; do
                python3 - "${mr%:*}" "${mr#*:}" "$H" "$arg" <<'PY' || exit 1
import json, sys
m, r, h, rnd = sys.argv[1:]
src = (f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, tools/pmc_all.sh via tools/gpu_session.sh) "
       f"over `python3 bench.py --mode {m} --steps 2 --warmup 1 --no-cpu-baseline --no-graph` (GEMM M = {r} per "
       f"launch) on MI355X, build {h}; hbm = 2*FETCH_SIZE + WRITE_SIZE per dispatch (MI355X_MICROARCH.md HBM "
       f"section: gfx950 FETCH_SIZE counts half of 16-B/lane streaming reads; Infinity-Cache hits included)")
out = {"source": src, "kernels": json.load(open(f"gpurun_out/pmc_{m}.json"))}
for d in ("gpurun_out", "profiles"):
    json.dump(out, open(f"{d}/{rnd}_pmc_traffic_{m}_m{r}.json", "w"), indent=1)
PY
              done
              # the raw rocprofv3 directories would push gpurun_out/ past what comes back from the box
              find gpurun_out -mindepth 1 -maxdepth 1 -type d \( -name 'instep_*' -o -name 'pmc_*' \) -exec rm -rf {} +
              mkdir -p gpurun_out/publish_"$arg"
              cp profiles/instep_*_"$H"* profiles/"$arg"_pmc_traffic_* gpurun_out/publish_"$arg"/
              ls -l gpurun_out/publish_"$arg" ;;
    attnpmc)  run attnpmc 400 bash tools/attn_pmc.sh ;;
    pmci8)    run pmci8 400 bash tools/pmc_i8.sh ;;
    pmci8=*)  run pmci8_$(echo "$arg" | tr -c 'a-zA-Z0-9' '_') 400 bash tools/pmc_i8.sh "$arg" ;;
    i8=*)     run i8_$(echo "$arg" | tr -c 'a-zA-Z0-9' '_') 400 env SAMQ_LIB=tuning python -u tools/bench_i8.py \
                --cfgs "${arg%@*}" --m "${arg#*@}" --iters 10 ;;
    w4=*)     run w4_$(echo "$arg" | tr -c 'a-zA-Z0-9' '_') 400 env SAMQ_LIB=tuning python -u tools/bench_gemm.py \
                --cfgs "${arg%@*}" --m "${arg#*@}" --iters 10 ;;
    w4g=*)    run w4g_$(echo "$arg" | tr -c 'a-zA-Z0-9' '_') 400 env SAMQ_LIB=tuning python -u tools/bench_gemm.py \
                --cfgs "${arg%@*}" --m "${arg#*@}" --iters 10 --groupsize 128 ;;
    ab48=*)   run ab48 500 env SAMQ_LIB=tuning python -u tools/bench_cfg_ab_w4a8.py 2 6 "$arg" ;;
    ab16g=*)  run ab16g 500 env SAMQ_AB_GS=128 python -u tools/bench_cfg_ab.py 2 6 "$arg" ;;
    ab88=*)   run ab88 500 env SAMQ_LIB=tuning python -u tools/bench_cfg_ab_w8a8.py 10 "$arg" ;;
    ab16=*)   run ab16 500 env SAMQ_LIB=tuning python -u tools/bench_cfg_ab.py 2 6 "$arg" ;;
    abl=*)    m=${arg%@*}; lib=${arg#*@}
              for r in 1 2; do
                run abl_${m}_new_$r 400 python bench.py --mode "$m" --steps 10 --warmup 3 --no-cpu-baseline --no-isolated
                run abl_${m}_lib_$r 400 env SAMQ_LIB="$lib" python bench.py --mode "$m" --steps 10 --warmup 3 --no-cpu-baseline --no-isolated
              done
              for f in gpurun_out/$tag.abl_${m}_*.log; do
                echo "$f $(grep -h '"value"' "$f" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
              done ;;
    ablg=*)   for r in 1 2 3; do
                run ablg_new_$r 400 python bench.py --groupsize 128 --steps 10 --warmup 3 --no-cpu-baseline --no-isolated --no-modes
                run ablg_lib_$r 400 env SAMQ_LIB="$arg" python bench.py --groupsize 128 --steps 10 --warmup 3 --no-cpu-baseline --no-isolated --no-modes
              done
              for f in gpurun_out/$tag.ablg_*.log; do
                echo "$f $(grep -h '"value"' "$f" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
              done ;;
    lanes=*)  m=${arg%@*}; ls=${arg#*@}
              for r in 1 2; do
                for l in ${ls//,/ }; do
                  run lanes_${m}_${l}_$r 400 python bench.py --mode "$m" --lanes "$l" --steps 10 --warmup 3 --no-cpu-baseline --no-isolated
                done
              done
              for f in gpurun_out/$tag.lanes_${m}_*.log; do
                echo "$f $(grep -h '"value"' "$f" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
              done ;;
    attn)     run attn 300 python -u tools/bench_attn.py ;;
    attnq8)   run attnq8 300 python -u tools/bench_attn_q8.py ;;
    attnq8pmc) run attnq8pmc 300 bash tools/attn_q8_pmc.sh ;;
    attnq8prof) run attnq8prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag.attnq8prof -o run --output-format csv \
                -- python3 tools/bench_attn_q8.py
              python3 -c "import csv,sys; [print(r['Name'][:90], r['Calls'], r['AverageNs']) for r in csv.DictReader(open(sys.argv[1]))]" \
                gpurun_out/$tag.attnq8prof/run_kernel_stats.csv ;;
    probe)    run probe 120 bash -c "hipcc --offload-arch=gfx950 -O2 -o gpurun_out/probe_cvt_u8 tools/probe_cvt_u8.hip && gpurun_out/probe_cvt_u8" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
exit 0
