"""Render bench.py's per-op roofline gap table (YCX_BENCH_KERNELS=<file>) as markdown.

    YCX_BENCH_KERNELS=gpurun_out/ops.json python bench.py ...
    python tools/op_gap.py gpurun_out/ops.json > profiles/r04/op_gap.md

Each row: the op's measured time (HIP events around every op of a serial forward), its
algorithmic FLOPs and HBM bytes (input once, weights once, residual once, output once), the
bound (MFMA above the peak/HBM ridge, else HBM), the floor that bound implies, the achieved
fraction of it and the gap. Rows are sorted by gap; a per-kernel and per-bound summary follows.
"""
import json
import sys


def main(path, top=None):
    d = json.load(open(path))
    ops = d['ops']
    print(f"# Per-op roofline gaps — {d.get('precision')} {d.get('shape')}\n")
    print(f"Peaks: {d.get('peak_tflops')} TFLOP/s MFMA, {d.get('hbm_peak_gbs')} GB/s HBM. "
          f"Forward {d['forward_kernel_ms']:.3f} ms, floor {d['forward_floor_ms']:.3f} ms, "
          f"gap {d['forward_gap_ms']:.3f} ms.")
    if d.get('forward_graph_ms'):
        print(f"Per-op times: HIP events around every op of serial forwards ({d['forward_events_ms']:.3f} ms in all), "
              f"less the event-record overhead spread evenly, so that they sum to the HIP-graph replay forward "
              f"({d['forward_graph_ms']:.3f} ms).")
    print()
    by = {}
    for o in ops:
        s = by.setdefault(o['bound'], [0.0, 0.0, 0])
        s[0] += o['ms']
        s[1] += o['floor_ms']
        s[2] += 1
    print("| bound | ops | ms | floor ms | gap ms | frac |")
    print("|---|---|---|---|---|---|")
    for b, (ms, fl, n) in sorted(by.items()):
        print(f"| {b} | {n} | {ms:.3f} | {fl:.3f} | {ms - fl:.3f} | {fl / ms:.3f} |")
    kern = {}
    for o in ops:
        k = kern.setdefault((o['name'], o['bound']), [0.0, 0.0, 0])
        k[0] += o['ms']
        k[1] += o['floor_ms']
        k[2] += 1
    print("\n| kernel | bound | launches | ms | floor ms | gap ms | frac |")
    print("|---|---|---|---|---|---|---|")
    for (name, b), (ms, fl, n) in sorted(kern.items(), key=lambda kv: -(kv[1][0] - kv[1][1])):
        print(f"| {name} | {b} | {n} | {ms:.4f} | {fl:.4f} | {ms - fl:.4f} | {fl / ms:.3f} |")
    print("\n| op | kernel | shape (n,h,w,cin,cout,k,s) | bound | FLOP/B | ms | floor ms | gap ms | frac | TFLOP/s | GB/s |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    rows = sorted(ops, key=lambda o: -o['gap_ms'])
    for o in rows[:top] if top else rows:
        print(f"| {o['i']} | {o['name']} | {o.get('shape')} | {o['bound']} | {o.get('intensity')} | {o['ms']:.4f} | "
              f"{o['floor_ms']:.4f} | {o['gap_ms']:.4f} | {o['frac']} | {o.get('tflops')} | {o.get('gbs')} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
