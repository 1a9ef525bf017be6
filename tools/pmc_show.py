"""Per-dispatch averages of the PMC passes written by tools/pmc_compare.sh, for the
FULL apply kernel (the 19-seed pass; KERNEL=fks_apply_bs_kernel for the 32-seed slice
kernel), one column per variant."""
import csv
import os
import glob
import sys
from collections import defaultdict


def load(v):
    acc = defaultdict(list)
    for f in glob.glob(f"gpurun_out/pmc_{v}_*/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if os.environ.get("KERNEL", "fks_apply_kernel") + "<" in row["Kernel_Name"] and "true>" in row["Kernel_Name"]:
                acc[(row["Counter_Name"], row["Dispatch_Id"])].append(float(row["Counter_Value"]))
    per = defaultdict(list)
    for (name, _), vals in acc.items():
        per[name].append(sum(vals))
    return {k: sum(x) / len(x) for k, x in per.items()}


vs = sys.argv[1:]
data = {v: load(v) for v in vs}
names = sorted({k for d in data.values() for k in d})
print("counter".ljust(28) + "".join(v.rjust(16) for v in vs))
for n in names:
    print(n.ljust(28) + "".join(f"{data[v].get(n, float('nan')):16.4g}" for v in vs))
