"""Per-kernel stats of the dispatches inside bench.py's roctx-marked timed window.

    python tools/instep_window.py <rocprofv3 output dir> <steps> <out.json>
Reads <dir>/**/*kernel_trace.csv and *marker_api_trace.csv (rocprofv3 --kernel-trace
--marker-trace --output-format csv); keeps the dispatches that start inside the
"samq_timed_steps" range; writes {"steps", "window_ms", "kernels": {name: {calls, total_ns,
avg_ns, min_ns, max_ns}}} sorted by total time.
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def main():
    d, steps, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    win = None
    for f in glob.glob(f"{d}/**/*marker_api_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if any("samq_timed_steps" in str(v) for v in r.values()):
                win = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    if win is None:
        sys.exit("no samq_timed_steps marker range in the trace")
    ker = defaultdict(list)
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if win[0] <= s <= win[1]:
                ker[r["Kernel_Name"]].append(e - s)
    res = {k: dict(calls=len(v), total_ns=sum(v), avg_ns=sum(v) / len(v), min_ns=min(v), max_ns=max(v))
           for k, v in sorted(ker.items(), key=lambda kv: -sum(kv[1]))}
    json.dump(dict(steps=steps, window_ms=(win[1] - win[0]) / 1e6, kernels=res), open(out, "w"), indent=1)
    print(f"{out}: {sum(len(v) for v in ker.values())} dispatches of {len(ker)} kernels in "
          f"{(win[1] - win[0]) / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
