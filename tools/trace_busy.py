"""GPU occupancy of the concurrent bench loop from a rocprofv3 kernel trace (development tool).

    python tools/trace_busy.py gpurun_out/r05/busy/.../run_kernel_trace.csv [skip_frac]

Takes the kernels of the timed loop of `bench.py --latency-steps 0 --image-in-steps 0
--cpu-seconds 0 --fp16-steps 0 --pipelined-steps 0 --roofline-steps 1`: the longest run of dispatches with no
kernel on the default stream (the slot streams of the concurrent detector only; set-up
copies, graph capture and the serial roofline leg run on the default stream), less its
first and last `skip_frac` so the warm-up / drain edges do not count, and prints: the fraction of wall time at least one
kernel runs (union busy), the time-weighted number of kernels in flight, the idle gaps
by length, and the kernels' summed durations by name (each kernel's wall duration counts
the time it shares the GPU with other streams' kernels).
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    best, cur = (0, 0), 0
    for i, r in enumerate(rows + [{"Stream_Id": "0"}]):
        if r["Stream_Id"] == "0":
            if i - cur > best[1] - best[0]:
                best = (cur, i)
            cur = i + 1
    rows = rows[best[0]:best[1]]
    n = len(rows)
    rows = rows[int(n * skip):int(n * (1 - skip))]
    ev = []
    for r in rows:
        ev.append((int(r["Start_Timestamp"]), 1))
        ev.append((int(r["End_Timestamp"]), -1))
    ev.sort()
    t0, t1 = ev[0][0], ev[-1][0]
    busy = 0
    conc = collections.Counter()
    gaps = []
    cur, last = 0, t0
    for t, d in ev:
        if t > last:
            conc[cur] += t - last
            if cur > 0:
                busy += t - last
            else:
                gaps.append(t - last)
        cur += d
        last = t
    wall = t1 - t0
    print(f"kernels {len(rows)}  wall {wall / 1e6:.3f} ms  union busy {busy / wall:.4f}")
    print("time-weighted kernels in flight:", round(sum(k * v for k, v in conc.items()) / wall, 3))
    for k in sorted(conc):
        print(f"  {k} in flight: {conc[k] / wall:.4f}")
    gaps.sort(reverse=True)
    print(f"idle gaps: {len(gaps)}, total {sum(gaps) / 1e3:.1f} us, largest {[round(g / 1e3, 1) for g in gaps[:8]]} us")
    per = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        per[r["Kernel_Name"][:70]][0] += 1
        per[r["Kernel_Name"][:70]][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = sum(v[1] for v in per.values())
    print(f"summed kernel durations {tot / 1e6:.3f} ms ({tot / wall:.2f} x wall)")
    for k, v in sorted(per.items(), key=lambda kv: -kv[1][1])[:14]:
        print(f"  {v[1] / tot:6.3f}  {v[0]:6d}  {k}")


if __name__ == "__main__":
    main()
