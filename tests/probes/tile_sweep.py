"""Tile-picker audit (development probe): every conv shape of a bench plan (bench.py
YCX_BENCH_KERNELS ops.json; fused-pool, head, stem and pair ops excluded) timed in
isolation with the picker's own choice (tile 0) and with every tile that accepts it.

    python tests/probes/tile_sweep.py gpurun_out/r05/ops.json [tile ...]
Prints one line per shape: the auto pick's time, the fastest tile and its time.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import conv_bench  # noqa: E402

TILES = [16, 18, 15, 9, 10, 11, 12, 13, 14, 17, 19, 20, 21, 22, 23, 24, 25, 26, 48, 49, 50, 1, 2, 3, 4]


def main():
    ops = json.load(open(sys.argv[1]))["ops"]
    tiles = [int(t) for t in sys.argv[2:]] or TILES
    seen = []
    for o in ops:
        if o["kind"] != "conv" or "+" in o["name"] or o["name"].startswith(("head", "wres1x1_pair", "stem")):
            continue
        sh = tuple(o["shape"])
        if sh in seen:
            continue
        seen.append(sh)
        auto = conv_bench.run(sh, 0)
        res = []
        for t in tiles:
            try:
                r = conv_bench.run(sh, t)
            except Exception:  # noqa: BLE001 (a tile the shape does not fit)
                r = None
            if r is not None:
                res.append((r[0], t))
        res.sort()
        best = " ".join(f"t{t}:{ms * 1e3:.1f}" for ms, t in res[:4])
        gain = (auto[0] - res[0][0]) / auto[0] if res and auto else 0.0
        print(f"{sh} plan {o['name']} auto {auto[0] * 1e3:.1f} us | best {best} | gain {gain:+.1%}", flush=True)


if __name__ == "__main__":
    main()
