"""Per-kernel stats of the dispatches inside bench.py's roctx-marked timed window.

    python tools/instep_window.py <rocprofv3 output dir> <steps> <out.json> [mode]
Reads <dir>/**/*kernel_trace.csv and *marker_api_trace.csv (rocprofv3 --kernel-trace
--marker-trace --output-format csv); keeps the dispatches that start inside the
"samq_timed_steps" range; writes {"steps", "window_ms", "kernels": {name: {calls, total_ns,
avg_ns, min_ns, max_ns}}, "busy_ns", "gemm_union_ns"} -- busy_ns / gemm_union_ns are the lengths
of the UNION of the dispatch intervals (all kernels / the mode's projection GEMMs,
bench.is_proj_gemm): with concurrent lanes the summed durations count overlapped time twice.
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def union(spans):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(spans):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    return tot + (cur_e - cur_s if cur_e is not None else 0)


def main():
    d, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    mode = sys.argv[4] if len(sys.argv) > 4 else "w4a16"
    sys.path.insert(0, ".")
    from bench import is_proj_gemm
    win = None
    for f in glob.glob(f"{d}/**/*marker_api_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if any("samq_timed_steps" in str(v) for v in r.values()):
                win = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    if win is None:
        sys.exit("no samq_timed_steps marker range in the trace")
    ker = defaultdict(list)
    spans, gspans = [], []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if win[0] <= s <= win[1]:
                ker[r["Kernel_Name"]].append(e - s)
                spans.append((s, e))
                if is_proj_gemm(mode, r["Kernel_Name"]):
                    gspans.append((s, e))
    res = {k: dict(calls=len(v), total_ns=sum(v), avg_ns=sum(v) / len(v), min_ns=min(v), max_ns=max(v))
           for k, v in sorted(ker.items(), key=lambda kv: -sum(kv[1]))}
    json.dump(dict(steps=steps, window_ms=(win[1] - win[0]) / 1e6, busy_ns=union(spans), gemm_union_ns=union(gspans),
                   kernels=res), open(out, "w"), indent=1)
    print(f"{out}: {sum(len(v) for v in ker.values())} dispatches of {len(ker)} kernels in "
          f"{(win[1] - win[0]) / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
