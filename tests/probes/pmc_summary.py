"""Average PMC counter values per dispatch of the conv kernel (development probe).

    python tests/probes/pmc_summary.py gpurun_out/pmc_conv/22 [kernel-substring]
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "conv"
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
    for k in sorted(agg):
        print(f"{k:40s} {agg[k] / max(1, len(disp[k])):16.1f}")


if __name__ == "__main__":
    main()
