"""Per-kernel averages of every counter in rocprofv3 --pmc output directories.

    python tools/pmc_kernels.py gpurun_out/pmc_attn [name-filter]
"""
import csv
import glob
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if len(sys.argv) > 2 and sys.argv[2] not in r["Kernel_Name"]:
            continue
        agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} n={len(v):3d} avg={sum(v) / len(v):16.1f}")
