"""Per-op kernel durations of one forward from a rocprofv3 --kernel-trace run of bench.py
(development tool): matches the last complete forward's dispatches to the plan ops in
gpurun_out/pmc_ops.json (written by tools/pmc_workload.py) by order.

    python tools/op_times.py gpurun_out/tr [pmc_ops.json]
"""
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    st = [i for i, r in enumerate(rows) if "stem2_fused" in r["Kernel_Name"]]
    i0 = st[-2]
    q = rows[i0]["Queue_Id"]
    fw = []
    for r in rows[i0:]:
        if r["Queue_Id"] != q:
            continue
        if fw and "stem2_fused" in r["Kernel_Name"]:
            break
        fw.append(r)
    tot = 0.0
    out = []
    for k, r in enumerate(fw):
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += dur
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        out.append((dur, k, name[:70]))
    print(f"{len(fw)} dispatches, sum {tot:.1f} us, span {(int(fw[-1]['End_Timestamp']) - int(fw[0]['Start_Timestamp'])) / 1e3:.1f} us")
    for dur, k, name in sorted(out, reverse=True)[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
        print(f"{dur:8.1f} us  #{k:3d}  {name}")


if __name__ == "__main__":
    main()
