"""Average every PMC counter per kernel over rocprofv3 --pmc counter_collection CSVs.

    python tools/pmc_kernel_counters.py <dir> [kernel-substring]

Counter values are summed over the dimensions rocprofv3 reports (per XCD / SE) for each
dispatch, then averaged over dispatches."""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
per = defaultdict(lambda: defaultdict(float))   # (kernel, dispatch) -> counter -> value
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row["Kernel_Name"]
            if sub and sub not in k:
                continue
            per[(k, f, row.get("Dispatch_Id", row.get("Correlation_Id", "")))][row["Counter_Name"]] += float(
                row["Counter_Value"])
agg = defaultdict(lambda: defaultdict(list))
for (k, _, _), cs in per.items():
    for c, v in cs.items():
        agg[k][c].append(v)
for k, cs in agg.items():
    print(k[:100])
    for c in sorted(cs):
        v = cs[c]
        print(f"   {c:28s} n={len(v):3d} avg={sum(v) / len(v):18.1f}")
