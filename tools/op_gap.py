"""Per-op gap to the roofline floor (development tool).

    python tools/op_gap.py gpurun_out/r02/k_base.json
Floor per conv = max(FLOP / 2.0 PF, algorithmic bytes / 6.0 TB/s): the bf16 MFMA rate at the
clock the chip holds under load and the achievable HBM rate (MI355X_MICROARCH.md). Bytes = input
map once + output map once + weights, bf16.
"""
import json
import sys

PF, BW = 2.0e15, 6.0e12
d = json.load(open(sys.argv[1]))
rows, tot, tot_floor = [], 0.0, 0.0
for o in d['ops']:
    ms = o['ms']
    tot += ms
    sh = o.get('shape')
    if not sh:
        rows.append((ms * 1e3, ms * 1e3, 0.0, o['i'], o['name'], None))
        continue
    n, h, w, ci, co, k, s = sh
    ho, wo = (h + 2 * (k // 2) - k) // s + 1, (w + 2 * (k // 2) - k) // s + 1
    fl = 2.0 * n * ho * wo * co * ci * k * k
    by = 2.0 * (n * h * w * ci + n * ho * wo * co + co * ci * k * k)
    if o['name'].startswith('head'):
        by = 2.0 * n * h * w * ci
    fl_t, by_t = fl / PF * 1e6, by / BW * 1e6
    floor = max(fl_t, by_t)
    tot_floor += floor / 1e3
    rows.append((ms * 1e3 - floor, ms * 1e3, floor, o['i'], o['name'], ('mfma' if fl_t > by_t else 'hbm', sh)))
rows.sort(key=lambda r: -r[0])
for g, t, f, i, name, extra in rows:
    print(f"{i:3d} {name[:26]:26s} {t:7.1f} us floor {f:6.1f} gap {g:6.1f} eff {f / t:4.2f} {extra}")
print(f"total {tot:.3f} ms, floor {tot_floor:.3f} ms")
