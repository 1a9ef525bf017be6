"""Per-dispatch averages of tools/gpu_pmc2.sh passes: one column per variant for the
full 32-seed slice kernel launch (KERNEL env overrides), and, if present, per-kernel rows
of the issue2 ubench."""
import collections
import csv
import glob
import os
import sys


def load(v, match):
    acc = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob(f"gpurun_out/pmc2_{v}_*/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if match(row["Kernel_Name"]):
                acc[row["Counter_Name"]] += float(row["Counter_Value"])
                disp[row["Counter_Name"]].add(row["Dispatch_Id"])
    return {k: acc[k] / len(disp[k]) for k in acc}


def main():
    kern = os.environ.get("KERNEL", "fks_apply_bs_kernel")
    vs = sys.argv[1:]
    data = {v: load(v, lambda n: (kern + "<") in n and "true>" in n) for v in vs}
    names = sorted({k for d in data.values() for k in d})
    print("counter".ljust(26) + "".join(v.rjust(16) for v in vs))
    for n in names:
        print(n.ljust(26) + "".join(f"{data[v].get(n, float('nan')):16.5g}" for v in vs))
    if glob.glob("gpurun_out/pmc2_ub_*"):
        ks = set()
        for f in glob.glob("gpurun_out/pmc2_ub_*/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                ks.add(row["Kernel_Name"].split("(")[0])
        for k in sorted(ks):
            d = load("ub", lambda n, k=k: n.split("(")[0] == k)
            print(k, {n: f"{x:.4g}" for n, x in sorted(d.items())})


if __name__ == "__main__":
    main()
