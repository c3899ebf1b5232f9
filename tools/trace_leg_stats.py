"""Per-kernel duration statistics of one leg of a rocprofv3 kernel trace (development tool).

bench.py runs three legs on the GPU: the warm-up + timed loop (three batches in
flight on three streams, so kernels of different batches overlap and each
kernel's wall duration includes the time it shares the GPU), then the roofline
leg (``--roofline-steps`` serial eager forwards of one plan on one stream, the
launches ``roofline.avg_launch_ms`` is measured on). This script splits the
trace of that same command into the two legs and prints, per kernel name, the
calls and the average / min / max duration of each, so the roofline kernel's
average can be checked against the profiler's own clock.

    python tools/trace_leg_stats.py gpurun_out/r01/trace/run_kernel_trace.csv 91 3 [out.csv]
(91 = ops of the plan, 3 = roofline steps: the roofline leg is the last 91 x 3
conv/pool/copy dispatches of the trace.)
"""
import csv
import sys


def main():
    path, n_ops, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else None
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    fwd = [r for r in rows if not r["Kernel_Name"].startswith(("__amd", "void at::", "at::"))
           and not any(k in r["Kernel_Name"] for k in ("nms_", "decode_filter", "FillFunc", "reduce_kernel"))]
    leg = fwd[-n_ops * steps:]
    ids = {r["Dispatch_Id"] for r in leg}
    legs = {"roofline_leg": leg, "timed_loop_and_warmup": [r for r in rows if r["Dispatch_Id"] not in ids]}
    table = []
    for name, rs in legs.items():
        per = {}
        for r in rs:
            per.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
            table.append(dict(leg=name, Name=k, Calls=len(v), TotalDurationNs=sum(v),
                              AverageNs=round(sum(v) / len(v), 1), MinNs=min(v), MaxNs=max(v)))
    for t in table[:12] + [t for t in table if t["leg"] == "timed_loop_and_warmup"][:6]:
        print(t["leg"], t["Name"][:80], t["Calls"], t["AverageNs"])
    if out:
        with open(out, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(table[0]))
            w.writeheader()
            w.writerows(table)


if __name__ == "__main__":
    main()
