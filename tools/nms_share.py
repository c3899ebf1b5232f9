"""NMS kernels' share of GPU time from a rocprofv3 --stats kernel_stats.csv (development tool).

    python tools/nms_share.py <dir with *kernel_stats.csv>
"""
import csv
import glob
import sys


def main():
    f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    nms = [r for r in rows if "nms_" in r["Name"]]
    print(f"NMS kernels {100 * sum(float(r['TotalDurationNs']) for r in nms) / tot:.2f} % of GPU time")
    for r in sorted(nms, key=lambda r: -float(r["TotalDurationNs"])):
        name = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        print(f"  {name:22s} calls {int(r['Calls']):5d}  avg {float(r['AverageNs']) / 1e3:8.1f} us  "
              f"{100 * float(r['TotalDurationNs']) / tot:5.2f} % of GPU time")


if __name__ == "__main__":
    main()
