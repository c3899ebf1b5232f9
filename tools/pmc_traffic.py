"""HBM bytes per kernel launch from the rocprofv3 PMC passes of tools/pmc_workload.py.

    python3 tools/pmc_traffic.py --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write \
        --ops gpurun_out/pmc_ops.json --out profiles/r01/traffic.json

Counters are corrected as MI355X_MICROARCH.md's HBM section prescribes:
FETCH_SIZE and WRITE_SIZE come from separate passes. rocprofv3 reports them in
KiB. On gfx950 FETCH_SIZE counts half the bytes of wide coalesced streaming
reads, so it is doubled. The first ycx dispatch of the workload is a copy with
a known byte count (512 MiB read, 512 MiB written, past the Infinity Cache).
Its corrected counters are reported as `calibration` so the correction can be
checked on this access pattern. The other ycx dispatches are matched, in
order, to the plan's ops and then to the post-processing kernels.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re

KIB = 1024


def _short(name):
    """Base name of one of our kernels (all live in anonymous namespaces), else None.
    Names arrive demangled ("void (anonymous namespace)::conv1x1_wres<8, ...>(...)") or, when
    the demangler gives up on __bf16 template arguments, mangled ("_ZN12_GLOBAL__N_111copy_kernelI...")."""
    if "(anonymous namespace)::" in name:
        return re.split(r"[<(]", name.split("(anonymous namespace)::", 1)[1], 1)[0]
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)", name)
    if m:
        n = int(m.group(1))
        return name[m.end():m.end() + n]
    return None


def load(d, counter):
    """Per ycx dispatch, in dispatch order: (short name, full name, summed counter value)."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    agg, names = collections.defaultdict(float), {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            key = (f, int(r["Dispatch_Id"]))
            agg[key] += float(r["Counter_Value"])
            names[key] = r["Kernel_Name"]
    out = []
    for key in sorted(agg, key=lambda k: (k[0], k[1])):
        s = _short(names[key])
        if s:
            out.append((s, names[key], agg[key]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--ops", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    meta = json.load(open(a.ops))
    fetch, write = load(a.fetch, "FETCH_SIZE"), load(a.write, "WRITE_SIZE")
    if [f[0] for f in fetch] != [w[0] for w in write]:
        raise SystemExit("FETCH_SIZE and WRITE_SIZE passes saw different dispatch sequences")
    ops = meta["ops"]
    if len(fetch) < 1 + len(ops):
        raise SystemExit(f"expected >= {1 + len(ops)} ycx dispatches, found {len(fetch)}")
    rd = [2.0 * f[2] * KIB for f in fetch]   # gfx950: FETCH_SIZE counts half of streaming reads
    wr = [w[2] * KIB for w in write]
    cal = meta["calibration"]
    calibration = dict(kernel=fetch[0][0], known_read=cal["read_bytes"], known_write=cal["write_bytes"],
                       fetch_corrected=rd[0], write=wr[0], read_ratio=rd[0] / cal["read_bytes"],
                       write_ratio=wr[0] / cal["write_bytes"])
    per_op = []
    for i, op in enumerate(ops):
        k = 1 + i
        per_op.append(dict(i=i, name=op["name"], kernel=fetch[k][0], shape=op.get("shape"), flops=op.get("flops", 0),
                           read_bytes=rd[k], write_bytes=wr[k], hbm_bytes=rd[k] + wr[k]))
    post = [dict(kernel=fetch[k][0], read_bytes=rd[k], write_bytes=wr[k], hbm_bytes=rd[k] + wr[k])
            for k in range(1 + len(ops), len(fetch))]
    per_name = {}
    for o in per_op:
        d = per_name.setdefault(o["name"], dict(launches=0, hbm_bytes=0.0, read_bytes=0.0, write_bytes=0.0))
        d["launches"] += 1
        for f in ("hbm_bytes", "read_bytes", "write_bytes"):
            d[f] += o[f]
    for d in per_name.values():
        d["hbm_bytes_per_launch"] = d["hbm_bytes"] / d["launches"]
    res = dict(source="rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), tools/pmc_workload.py",
               correction="bytes = FETCH_SIZE*2*1024 + WRITE_SIZE*1024 (KiB; gfx950 FETCH_SIZE halving)",
               shape=meta["shape"], calibration=calibration, per_name=per_name, per_op=per_op, post=post,
               forward_hbm_bytes=sum(o["hbm_bytes"] for o in per_op))
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(dict(calibration=calibration, forward_hbm_GB=res["forward_hbm_bytes"] / 1e9,
                          n_ops=len(per_op), post=len(post))))


if __name__ == "__main__":
    main()
