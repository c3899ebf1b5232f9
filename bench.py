"""Benchmark: YOLOv7 (COCO-80) 640x640 inference, bs=32 per GPU, on MI355X.

One step = one batch through the whole hot path, device resident:
  Model.forward (static plan of HIP kernels, one HIP graph replay)
  -> fused decode + filter (ycx_decode_filter) -> sort + per-class NMS (ycx_sort_nms)
  -> (N > 1) one RCCL all_gather of the padded detections over xGMI.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--global-batch B]
--gpus N > 1 starts N rank processes by itself (one per GPU, before any GPU
call in the parent); a launch under torch.distributed.run (WORLD_SIZE set) is
used as is. Images are sharded by rank (weak scaling: 32 images per GPU per
step; --global-batch B: strong scaling, B images per step split over the ranks,
"scaling": "strong").

Prints ONE JSON line (rank 0) with images/s for the whole job, p50 step
latency, the dominant kernel's roofline, and the CPU-oracle baseline.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "yolo-continuous_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

ANCHORS = [[12, 16, 19, 36, 40, 28], [36, 75, 76, 55, 72, 146], [142, 110, 192, 243, 459, 401]]
MASK = [[6, 7, 8], [3, 4, 5], [0, 1, 2]]
METRIC = "images/sec (whole node) + p50 end-to-end latency, 640×640 bs=32, 1/2/4/8 MI355X"
PEAK = {"bf16": 2500.0, "fp16": 2500.0, "f32": 157.3, "fp8": 5000.0}  # dense MFMA TFLOP/s (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0  # HBM3E peak (MI355X_MICROARCH.md)


def _current_round():
    """profiles/<round>/ of the newest round that holds a PMC traffic summary
    (``--round`` overrides): roofline.traffic is read from there."""
    base = os.path.join(REPO, "profiles")
    try:
        rounds = sorted(d for d in os.listdir(base)
                        if d[:1] == "r" and d[1:].isdigit() and os.path.isfile(os.path.join(base, d, "traffic.json")))
    except OSError:
        rounds = []
    return rounds[-1] if rounds else None


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 100 timed steps (≈ 0.5 s): with three batches in flight the pipeline fill and the final
    # drain inside the timed region cost ≈ 4 % of a 20-step run
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=32, help="images per GPU per step (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="strong scaling (SURVEY.md 8(e)): this many images per step over all ranks, "
                         "split evenly (32 over 1/2/4/8 GPUs = 32/16/8/4 each); overrides --batch")
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--net", default="yolov7")
    ap.add_argument("--nc", type=int, default=80)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp16", "f32", "fp8"],
                    help="fp16: the north_star-conforming mode (1e-3 on box/confidence tensors) at the bf16 rate")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--mode", default="concurrent", choices=["concurrent", "pipelined", "serial"],
                    help="concurrent: 3 batches in flight on 3 streams (default); pipelined: forward and "
                         "decode+NMS on two streams; serial: one stream")
    ap.add_argument("--depth", type=int, default=3, help="batches in flight in concurrent mode")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="run each batch's forward and post back to back on one stream")
    ap.add_argument("--conf", type=float, default=0.3)
    ap.add_argument("--iou", type=float, default=0.3)
    ap.add_argument("--max-det", type=int, default=300)
    ap.add_argument("--cpu-seconds", type=float, default=15.0,
                    help="0: skip the CPU baseline; --post-micro: time budget of its CPU leg")
    ap.add_argument("--cpu-batch", type=int, default=32, help="CPU baseline batch (BASELINE.md §4: 32)")
    ap.add_argument("--cpu-iters", type=int, default=3, help="CPU baseline timed iterations (after 1 warm-up)")
    ap.add_argument("--no-fuse-heads", action="store_true",
                    help="diagnostic: decode in a separate ycx_decode_filter pass over stored fp32 heads")
    ap.add_argument("--keep-heads", action="store_true",
                    help="diagnostic: the fused head convs also store the raw fp32 NCHW logits")
    ap.add_argument("--roofline-steps", type=int, default=3)
    ap.add_argument("--dist", action="store_true",
                    help="run the N > 1 code path (process group + RCCL all-gather) even at one rank")
    ap.add_argument("--latency-steps", type=int, default=10,
                    help="unloaded latency leg: batches run one at a time (0: skip)")
    ap.add_argument("--post-micro", action="store_true",
                    help="fixed-load decode + NMS micro-bench on G3-recipe head logits (SURVEY 8(d)) instead of "
                         "the network bench; prints its own JSON line")
    ap.add_argument("--obj-shift", type=float, default=-3.0, help="--post-micro: objectness logit shift")
    ap.add_argument("--diag-forward-only", action="store_true",
                    help="DIAGNOSTIC (not the metric): time the forwards alone, no decode / NMS")
    ap.add_argument("--image-in-steps", type=int, default=30,
                    help="image-in leg (SURVEY 8(d) H2D-inclusive variant): seeded 512x773 uint8 BGR host images "
                         "in pinned memory -> H2D -> ycx_letterbox_batch -> the same path; 0: skip")
    ap.add_argument("--fp16-steps", type=int, default=None,
                    help="the north_star-conforming fp16 plan (1e-3 on box / confidence tensors) timed in the same "
                         "run after the headline leg, same mode (default: min(--steps, 30) when --precision is "
                         "bf16; 0: skip); reported as value_fp16 / ms_per_step_fp16 / roofline_fp16")
    ap.add_argument("--pipelined-steps", type=int, default=None,
                    help="the low-latency point of the same workload and precision timed in the same run: mode "
                         "pipelined (two slots, forward and post on two streams) instead of the concurrent "
                         "throughput mode (default: min(--steps, 30) in concurrent mode; 0: skip); reported as "
                         "value_pipelined / ms_per_step_pipelined / p50_ms_pipelined")
    ap.add_argument("--round", default=None,
                    help="profiles/<round>/traffic.json for roofline.traffic (default: the newest round that has one)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: every rank joins a gloo process group, all-gathers "
                         "fabricated padded detections and rank 0 prints one JSON line (no GPU legs)")
    return ap.parse_args(argv)


def op_gap_table(op_info, per_op_ms, peak_tflops, hbm_gbs=HBM_PEAK_GBS):
    """One row per plan op: its algorithmic FLOPs and HBM bytes (engine op_info:
    input once, weights once, residual once, output once), the bound it sits
    under (MFMA when FLOP / peak exceeds bytes / HBM peak, i.e. above the
    peak / HBM ridge, 312 FLOP/B for bf16), the floor time that bound implies,
    the achieved fraction of it (floor / measured) and the gap in ms."""
    rows = []
    for i, info in enumerate(op_info):
        ms = per_op_ms[i]
        fl, by = int(info.get('flops', 0)), int(info.get('bytes', 0))
        t_mfma = fl / (peak_tflops * 1e12) * 1e3
        t_hbm = by / (hbm_gbs * 1e9) * 1e3
        floor = max(t_mfma, t_hbm)
        rows.append(dict(i=i, name=info['name'], kind=info.get('kind'), shape=info.get('shape'), ms=round(ms, 5),
                         flops=fl, bytes=by, bound='mfma' if t_mfma > t_hbm else 'hbm',
                         intensity=round(fl / by, 1) if by else None,
                         floor_ms=round(floor, 5), frac=round(floor / ms, 4) if ms > 0 else None,
                         gap_ms=round(max(0.0, ms - floor), 5),
                         tflops=round(fl / (ms * 1e-3) / 1e12, 1) if fl and ms > 0 else None,
                         gbs=round(by / (ms * 1e-3) / 1e9, 1) if by and ms > 0 else None))
    return rows


def roofline(det, steps, precision, replays=10):
    """Per-op HIP events around every op of the plan (recorded on the plan's
    stream by ycx_run_ops) for `steps` extra forwards; returns the dominant
    conv kernel's achieved TFLOP/s and a per-kernel table.

    Every event record costs the stream ~6 us between two kernels (measured
    against the rocprofv3 trace of the same leg: 508 us of gaps over 82
    boundaries, r04), which the raw event intervals charge to the ops. So the
    forward is also timed as `replays` HIP-graph replays (the bench's own
    launch path, ~1 us kernel boundaries) and the difference, spread evenly
    over the ops, is taken off each op: the corrected per-op times sum to the
    graph-replay forward time and match the profiler's per-kernel durations."""
    eng = det.engine
    n = eng.n_ops
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    for e in evs:  # materialise the underlying hipEvent_t
        e.record()
    per_op = [0.0] * n
    for _ in range(steps):
        det.forward(events=evs)  # counts reset first: the fused heads append this forward's candidates
        torch.cuda.synchronize()
        for i in range(n):
            per_op[i] += evs[i].elapsed_time(evs[i + 1]) / steps
    raw_ms = sum(per_op)
    graph_ms = None
    if getattr(eng, 'graph_exec', None) is not None and replays > 0:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        eng.replay()
        torch.cuda.synchronize()
        e0.record()
        for _ in range(replays):
            eng.replay()
        e1.record()
        torch.cuda.synchronize()
        graph_ms = e0.elapsed_time(e1) / replays
        overhead = max(0.0, (raw_ms - graph_ms) / n)
        per_op = [max(0.0, t - overhead) for t in per_op]
    per = {}
    for i, info in enumerate(eng.op_info):
        d = per.setdefault(info['name'], dict(ms=0.0, launches=0, flops=0))
        d['ms'] += per_op[i]
        d['launches'] += 1
        d['flops'] += info.get('flops', 0)
    convs = {k: v for k, v in per.items() if v['flops'] > 0 and k != 'stem'}
    dom = max(convs, key=lambda k: convs[k]['ms'])
    dd = convs[dom]
    avg_ms = dd['ms'] / dd['launches']
    flops_per_launch = dd['flops'] / dd['launches']
    achieved = flops_per_launch / (avg_ms * 1e-3) / 1e12
    all_conv_ms = sum(v['ms'] for v in per.values() if v['flops'] > 0)
    all_conv_tf = sum(v['flops'] for v in per.values()) / (all_conv_ms * 1e-3) / 1e12
    fwd_ms = sum(v['ms'] for v in per.values())
    ops = op_gap_table(eng.op_info, per_op, PEAK[precision])
    # the dominant kernel's launches split by the bound each one sits under (its frac above mixes them)
    split = {}
    for o in ops:
        if o['name'] == dom:
            s = split.setdefault(o['bound'], dict(launches=0, ms=0.0, flops=0, bytes=0, floor_ms=0.0))
            s['launches'] += 1
            s['ms'] += o['ms']
            s['flops'] += o['flops']
            s['bytes'] += o['bytes']
            s['floor_ms'] += o['floor_ms']
    for b, s in split.items():
        s['frac_of_bound'] = round(s['floor_ms'] / s['ms'], 4) if s['ms'] else None
        s['tflops'] = round(s['flops'] / (s['ms'] * 1e-3) / 1e12, 1) if s['ms'] else None
        s['ms'] = round(s['ms'], 5)
        s['floor_ms'] = round(s['floor_ms'], 5)
    return dict(kernel=dom, avg_launch_ms=avg_ms, ops=ops, flops_per_launch=flops_per_launch, achieved=achieved,
                dominant_by_bound=split, forward_floor_ms=sum(o['floor_ms'] for o in ops),
                forward_events_ms=raw_ms, forward_graph_ms=graph_ms,
                forward_gap_ms=sum(o['gap_ms'] for o in ops),
                all_conv_tflops=all_conv_tf, all_conv_ms=all_conv_ms, forward_kernel_ms=fwd_ms,
                per_kernel={k: dict(ms=round(v['ms'], 4), launches=v['launches'],
                                    tflops=(round(v['flops'] / (v['ms'] * 1e-3) / 1e12, 1)
                                            if v['flops'] and v['ms'] > 0 else None))
                            for k, v in sorted(per.items(), key=lambda kv: -kv[1]['ms'])})


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _cgroup_cpus():
    """CPUs granted by the cgroup quota (cpu.max), or None when unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            return max(1, int(int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(args, sd, model_cfg):
    """the oracle (CPU fp32 restatement of the reference path:
    forward + decode_box + non_max_suppression, torch.no_grad, eval) on the
    bench's own workload shape (yolov7 nc=80, bs=32 at 640x640, seeded U[0,1)
    images), 1 warm-up + 3 timed iterations, with
    torch.set_num_threads(len(os.sched_getaffinity(0))) -- capped at the cgroup
    CPU quota when one is set, since threads past the quota only time-slice."""
    import numpy as np
    from oracle import ref_forward, ref_post
    from ycx.utils.synth import synthetic_images
    affinity = len(os.sched_getaffinity(0))
    quota = _cgroup_cpus()
    threads = min(affinity, quota) if quota else affinity
    torch.set_num_threads(threads)
    fwd = ref_forward.build(model_cfg, ANCHORS, args.nc, sd)
    anchors = np.asarray(ANCHORS).reshape(-1, 2)
    n = args.cpu_batch
    x = synthetic_images(n, 3, args.size, args.size, seed=1000)

    def one():
        with torch.no_grad():
            heads = fwd(x)
            dec = torch.cat(ref_post.decode_box(heads, anchors, MASK, args.nc, (args.size, args.size)), 1)
            ref_post.non_max_suppression(dec, args.nc, (args.size, args.size), np.array([args.size, args.size]),
                                         True, args.conf, args.iou)
    one()  # warm-up
    times = []
    for _ in range(args.cpu_iters):
        t0 = time.perf_counter()
        one()
        times.append(time.perf_counter() - t0)
    per_batch = statistics.median(times)
    model = _cpu_model()
    return dict(value=round(n / per_batch, 4), unit="images/s", cores=threads, threads=threads,
                affinity_cpus=affinity, cgroup_cpus=quota, cpu_model=model, batch=n, kind="port",
                p50_batch_s=round(per_batch, 3), iterations=args.cpu_iters, warmup=1,
                sample=f"oracle forward + decode_box + non_max_suppression (fp32, eval, no_grad; C greedy NMS "
                       f"restatement), yolov7 nc={args.nc}, {n} images {args.size}x{args.size} per batch, "
                       f"1 warm-up + {args.cpu_iters} timed batches (p50 {per_batch:.2f} s), {threads} threads "
                       f"(affinity {affinity}, cgroup quota {quota}), {model}, torch {torch.__version__}")


def setup(args, dev, rank=0, use_graph=None, pipeline=False):
    """The bench workload on ``dev``: yolov7 with seeded synthetic weights, a
    Detector (pipeline False), a 2-slot PipelinedDetector ('pipelined') or a
    ConcurrentDetector ('concurrent' / True) for (batch, 3, size, size) and this
    rank's synthetic images already resident in HBM."""
    from ycx.detect import ConcurrentDetector, Detector, PipelinedDetector
    from ycx.nets.yolo import Model
    from ycx.utils.helper_io import cvt_cfg
    from ycx.utils.synth import synthetic_images, synthetic_state_dict

    cfg = cvt_cfg(args.net)
    model = Model(cfg, ANCHORS, args.nc, precision=args.precision).eval()
    sd = synthetic_state_dict(model, seed=0)
    model.load_state_dict(sd)
    model.to(dev)
    shape = (args.batch, 3, args.size, args.size)
    kw = dict(conf_thres=args.conf, nms_thres=args.iou, max_det=args.max_det,
              use_graph=(not args.no_graph) if use_graph is None else use_graph,
              fuse_heads=not getattr(args, 'no_fuse_heads', False), keep_heads=getattr(args, 'keep_heads', False))
    images = synthetic_images(*shape, seed=1000 + rank).to(dev)
    if pipeline:
        if pipeline == 'pipelined':
            det = PipelinedDetector(model, shape, dev, ANCHORS, MASK, depth=2, **kw)
        else:
            det = ConcurrentDetector(model, shape, dev, ANCHORS, MASK, depth=getattr(args, 'depth', 3), **kw)
        for d in det.slots:
            d.x.copy_(images)
    else:
        det = Detector(model, shape, dev, ANCHORS, MASK, **kw)
        det.x.copy_(images)
    return model, det, sd, cfg, shape


def pmc_traffic(kernel, shape, rnd):
    """HBM bytes per launch of ``kernel`` from round ``rnd``'s PMC passes
    (tools/pmc_traffic.py -> profiles/<rnd>/traffic.json), or None."""
    if rnd is None:
        return None
    path = os.path.join(REPO, "profiles", rnd, "traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if list(t.get("shape", [])) != list(shape) or kernel not in t.get("per_name", {}):
        return None
    return round(t["per_name"][kernel]["hbm_bytes_per_launch"])


def post_micro(args, dev):
    """decode_box + non_max_suppression alone at a fixed load: the G3 recipe's
    N(0, 1) head logits with the objectness logit shifted by --obj-shift (-3:
    about 280 candidates per image at conf 0.3), [bs, 3*(5+nc), s/k, s/k] for
    k = 32, 16, 8 (Detect order), resident in HBM; one step = ycx_decode_filter
    + ycx_sort_nms of the batch on one stream. The CPU leg runs the oracle's
    decode_box + non_max_suppression on the same batch. Both GPU legs are timed
    as HIP-graph replays (10 steps per graph) so host launch cost is excluded."""
    import ctypes
    import numpy as np
    from ycx import _lib as L
    from ycx.detect import DevicePost
    from ycx.utils.synth import synthetic_head_logits
    bs, s = args.batch, args.size
    shapes = [(bs, s // k, s // k) for k in (32, 16, 8)]
    heads_cpu = synthetic_head_logits(shapes, args.nc, seed=11, obj_shift=args.obj_shift)
    heads = [h.to(dev) for h in heads_cpu]
    post = DevicePost(heads, args.nc, ANCHORS, MASK, (s, s), dev, args.conf, args.iou, args.max_det)

    def decode_only():
        st = L.stream_handle(dev)  # the capturing stream inside graphed()
        post.counts.zero_()
        L.check(L.lib.ycx_decode_filter(ctypes.byref(post.df_desc), post.heads_arr, post.cand.data_ptr(),
                                        post.cand_rows.data_ptr(), post.counts.data_ptr(), st), "ycx_decode_filter")

    def timed(fn, k):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(k):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k

    def graphed(fn, reps=10):  # host launch cost out of the timing: reps calls in one HIP graph
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        return lambda: g.replay(), reps

    for _ in range(args.warmup):
        post()
    g_post, reps = graphed(post)
    g_dec, _ = graphed(decode_only)
    ms = timed(g_post, args.steps) / reps
    dec_ms = timed(g_dec, args.steps) / reps  # decode_filter + the 4-byte-per-image counts memset
    post()
    torch.cuda.synchronize()
    cands = post.counts.sum().item() / bs
    kept = post.kc.clamp(max=args.max_det).sum().item() / bs
    rows = post.rows
    dec_bytes = bs * rows * (args.nc + 5) * 4  # fp32 logits read once (algorithmic)
    out = dict(metric="decode+NMS images/s at a fixed load (G3 recipe)", value=round(bs / (ms * 1e-3), 1),
               unit="images/s", n_gpus=1, steps=args.steps, warmup=args.warmup, ms_per_step=round(ms, 4),
               higher_is_better=True, dtype="f32", data="synthetic G3-recipe head logits",
               config=dict(workload=f"decode_box + non_max_suppression, nc={args.nc}, {s}x{s} heads, bs={bs}, "
                                    f"obj shift {args.obj_shift}", batch=bs, image_size=s, conf_thres=args.conf,
                           iou_thres=args.iou, max_det=args.max_det),
               candidates_per_image=round(cands, 1), kept_per_image=round(kept, 1),
               roofline=dict(bound="hbm", kernel="decode_filter_kernel", achieved=round(dec_bytes / (dec_ms * 1e-3) / 1e9, 1),
                             peak=8000.0, unit="GB/s", frac=round(dec_bytes / (dec_ms * 1e-3) / 1e9 / 8000.0, 4),
                             traffic=None, avg_launch_ms=round(dec_ms, 4), bytes_per_launch=dec_bytes))
    if args.cpu_seconds > 0:
        from oracle import ref_post
        cores = min(16, len(os.sched_getaffinity(0)))
        torch.set_num_threads(cores)
        anchors = np.asarray(ANCHORS).reshape(-1, 2)
        times = []
        t_start = time.perf_counter()
        while not times or (time.perf_counter() - t_start < args.cpu_seconds and len(times) < 5):
            t0 = time.perf_counter()
            dec = torch.cat(ref_post.decode_box(heads_cpu, anchors, MASK, args.nc, (s, s)), 1)
            ref_post.non_max_suppression(dec, args.nc, (s, s), np.array([s, s]), True, args.conf, args.iou)
            times.append(time.perf_counter() - t0)
        per = statistics.median(times)
        out["cpu_baseline"] = dict(value=round(bs / per, 2), unit="images/s", cores=cores, kind="port",
                                   sample=f"oracle decode_box + non_max_suppression of the same {bs}-image batch, "
                                          f"{len(times)} timed runs (median {per:.3f} s), {cores} threads")
    print(json.dumps(out), flush=True)


def image_in_leg(args, det, dev, dist_on, gather):
    """SURVEY 8(d) "H2D-inclusive variant" / 8(f)1: the step starts from host
    images, as detect.py:16-26 does (cv2 image -> letterbox -> tensor): seeded
    512x773x3 uint8 BGR images in pinned host memory; on each batch's slot stream
    one async H2D copy into a device staging buffer, one ycx_letterbox_batch into
    the slot's input, then the same forward + decode + NMS (+ gather). Returns
    the loaded rate (batches in flight, copies overlapping other batches'
    kernels) and the unloaded host-to-detections latency of one batch alone."""
    from ycx.utils.letterbox import letterbox_batch_gpu
    n, h0, w0 = args.batch, 512, 773
    g = torch.Generator().manual_seed(2024)
    host = torch.randint(0, 256, (n, h0, w0, 3), dtype=torch.uint8, generator=g).pin_memory()
    slots = det.slots if hasattr(det, 'slots') else [det]
    stage = [torch.empty((n, h0, w0, 3), dtype=torch.uint8, device=dev) for _ in slots]

    def pre(k, d):
        stage[k].copy_(host, non_blocking=True)
        letterbox_batch_gpu(stage[k], d.x)

    def step():
        if hasattr(det, 'slots'):
            return det.submit(pre=pre, then=gather if dist_on else None)[2]
        pre(0, det)
        return det()[2]

    def drain():
        if hasattr(det, 'slots'):
            det.synchronize()
        torch.cuda.synchronize()

    for _ in range(3):
        step()
    drain()
    if dist_on:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.image_in_steps):
        step()
    drain()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    lat = []
    for _ in range(max(3, min(10, args.image_in_steps))):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        step()
        drain()
        lat.append((time.perf_counter() - t1) * 1e3)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist_on:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    world = dist.get_world_size() if dist_on else 1
    return dict(value_image_in=round(world * n * args.image_in_steps / float(t.item()), 2),
                ms_per_step_image_in=round(float(t.item()) / args.image_in_steps * 1e3, 4),
                p50_ms_image_in_unloaded=round(statistics.median(lat), 4),
                image_in=f"{n} seeded {h0}x{w0}x3 uint8 BGR images per GPU per step in pinned host memory "
                         f"({host.numel() / 1e6:.1f} MB): async H2D + ycx_letterbox_batch to {args.size}x{args.size} "
                         f"inside the step; {args.image_in_steps} timed steps")


def visible_gpus(env=None, kfd_nodes="/sys/class/kfd/kfd/topology/nodes"):
    """GPUs a child process may use, found WITHOUT any HIP / torch.cuda call (the
    launcher parent must never initialise the GPU runtime): the shortest of the
    HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES lists when
    one is set, else the KFD topology nodes with SIMDs (CPU nodes have none);
    None when neither is readable (each rank then checks LOCAL_RANK itself)."""
    env = os.environ if env is None else env
    lists = [env[k] for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES") if k in env]
    if lists:
        return min(len([t for t in v.split(",") if t.strip()]) for v in lists)
    try:
        nodes = os.listdir(kfd_nodes)
    except OSError:
        return None
    n = 0
    for d in nodes:
        try:
            with open(os.path.join(kfd_nodes, d, "properties")) as f:
                props = dict(ln.split()[:2] for ln in f if len(ln.split()) >= 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0")) > 0:
            n += 1
    return n


def launch_ranks(args, argv):
    """``--gpus N`` (N > 1) without WORLD_SIZE in the environment: start N rank
    processes of this same script, one per GPU (RANK = LOCAL_RANK = i,
    WORLD_SIZE = N, rendezvous on 127.0.0.1 at a free port), and return the
    worst exit code. The parent never touches the GPU (visible_gpus reads the
    environment / sysfs, no HIP or torch.cuda call) and starts the ranks as
    child processes, never by exec. If a rank fails the others are stopped instead
    of waiting at a barrier forever."""
    import socket
    import subprocess
    have = None if args.dry_run else visible_gpus()  # the dry run uses no GPU
    if have is not None and have < args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but only {have} GPU(s) are visible")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   YCX_BENCH_LAUNCHED="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    codes = [None] * len(procs)
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
        if any(c not in (None, 0) for c in codes):
            for i, p in enumerate(procs):
                if codes[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if codes[i] is None:
                    try:
                        codes[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        codes[i] = p.wait()
            break
        time.sleep(0.05)
    return max((abs(c) for c in codes), default=0)


def dry_run(args, world, rank):
    """The N-rank launcher path without a GPU: a gloo process group, the bench's
    one collective on fabricated padded detections [batch, max_det, 7] (+ counts,
    keep rows), max-over-ranks timing; rank 0 prints one JSON line."""
    from ycx.dist import gather_detections
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = args.batch
        dets = torch.full((n, args.max_det, 7), float(rank))
        keep = torch.full((n, args.max_det), rank, dtype=torch.int32)
        kc = torch.full((n,), rank, dtype=torch.int32)
        dist.barrier()
        t0 = time.perf_counter()
        g_dets, g_kc, g_keep = gather_detections(dets, kc, keep)
        dist.barrier()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ok = bool(torch.equal(g_kc, torch.arange(world, dtype=torch.int32).repeat_interleave(n)))
        if rank == 0:
            print(json.dumps({"dry_run": True, "n_gpus": args.gpus, "rccl_world_size": dist.get_world_size(),
                              "backend": dist.get_backend(), "gathered_dets": list(g_dets.shape),
                              "gathered_keep": list(g_keep.shape), "rank_major_order": ok,
                              "gather_s": float(t.item())}), flush=True)
        if not ok:
            raise SystemExit("dry run: gathered counts are not in rank-major order")
    finally:
        dist.destroy_process_group()


def timed_leg(args, det, mode, dist_on, gather, lat_ev, steps=None, latency_steps=None):
    """W untimed warm-up steps, then exactly ``steps`` timed steps between a barrier +
    device synchronise on both sides (host wall clock), then the unloaded latency leg.
    Returns (elapsed s, loaded per-batch latencies ms, unloaded latencies ms, last kc)."""
    from ycx.dist import gather_detections
    steps = args.steps if steps is None else steps
    latency_steps = args.latency_steps if latency_steps is None else latency_steps
    pipeline = mode != "serial"

    def step(i=None):
        timing = lat_ev[i] if i is not None else None
        if mode == "concurrent":  # the collective on the batch's own stream, issued in batch order on every rank
            dets, keep, kc, done = det.submit(timing=timing, then=gather if dist_on else None,
                                              post=not args.diag_forward_only)
            return kc
        if pipeline:
            dets, keep, kc, _ = det.submit(timing=timing)
            if dist_on:  # the single collective, on the post stream after this batch's NMS
                with torch.cuda.stream(det.s_post):
                    dets, kc, keep = gather_detections(dets, kc, keep)
            return kc
        if timing is not None:
            timing[0].record()
        dets, keep, kc = det()
        if dist_on:  # the single collective: all-gather of padded detections (+ counts, keep rows)
            dets, kc, keep = gather_detections(dets, kc, keep)
        if timing is not None:
            timing[1].record()
        return kc

    def drain():
        if pipeline:
            det.synchronize()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    drain()
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        kc = step(i)
    drain()
    if dist_on:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    det.check()  # outside the timed region: no batch left the plan's range (fp16: |a| <= 65504)
    lat = [a.elapsed_time(b) for a, b in lat_ev]
    # unloaded latency: one batch in flight at a time (input resident -> detections, + gather)
    lat1 = []
    for _ in range(latency_steps):
        if dist_on:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        step()
        drain()
        lat1.append((time.perf_counter() - t1) * 1e3)
    return elapsed, lat, lat1, kc


def precision_leg(args, dev, rank, world, dist_on, gather, mode, precision, steps, sfx=None, with_roofline=True):
    """A second plan of the same workload in another precision (or mode), timed exactly as
    the headline leg (warm-up, ``steps`` timed steps between barriers, max over ranks) in the
    same run: the fp16 plan is the one that holds north_star's 1e-3 on box / confidence
    tensors (detect.py:227-231 compares the reference's fp32 outputs); the pipelined mode is
    the low-latency point (BASELINE's p50 end-to-end latency). Returns the ``*<sfx>`` keys
    of the JSON line (default suffix: ``_<precision>``)."""
    import copy
    a = copy.copy(args)
    a.precision = precision
    a.mode = mode
    pipeline = False if mode == "serial" else mode
    _, det, _, _, _ = setup(a, dev, rank, pipeline=pipeline)
    lat_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    elapsed, lat, _, _ = timed_leg(a, det, mode, dist_on, gather, lat_ev, steps=steps, latency_steps=0)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist_on:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    value = world * args.batch * steps / elapsed
    det1 = det.slots[0] if pipeline else det
    rl = roofline(det1, args.roofline_steps, precision) if rank == 0 and with_roofline else None
    det.close()
    sfx = sfx or "_" + precision
    out = {"value" + sfx: round(value, 2), "ms_per_step" + sfx: round(elapsed / steps * 1e3, 4),
           "steps" + sfx: steps, "p50_ms" + sfx: round(statistics.median(lat), 4),
           "p90_ms" + sfx: round(sorted(lat)[int(0.9 * (len(lat) - 1))], 4)}
    if rl is not None:
        peak = PEAK[precision]
        out["roofline" + sfx] = {"bound": "mfma", "kernel": rl['kernel'], "achieved": round(rl['achieved'], 2),
                                 "peak": peak, "unit": "TFLOP/s", "frac": round(rl['achieved'] / peak, 4),
                                 "avg_launch_ms": round(rl['avg_launch_ms'], 5),
                                 "flops_per_launch": int(rl['flops_per_launch']),
                                 "forward_kernel_ms": round(rl['forward_kernel_ms'], 4),
                                 "forward_floor_ms": round(rl['forward_floor_ms'], 4)}
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.post_micro:
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        return post_micro(args, dev)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        return dry_run(args, world, rank)
    rnd = args.round or _current_round()
    if local >= torch.cuda.device_count():  # the launcher could not count devices: the rank checks its own
        raise SystemExit(f"LOCAL_RANK {local} but only {torch.cuda.device_count()} GPU(s) are visible")
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    dist_on = world > 1 or args.dist  # --dist: the N > 1 code path (RCCL gather) on a single rank
    if args.global_batch:
        if args.global_batch % world:
            raise SystemExit(f"--global-batch {args.global_batch} does not split over {world} ranks")
        args.batch = args.global_batch // world
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)

    mode = "serial" if args.no_pipeline else args.mode
    pipeline = False if mode == "serial" else mode
    model, det, sd, cfg, shape = setup(args, dev, rank, pipeline=pipeline)
    from ycx.dist import gather_detections
    lat_ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]

    def gather(dets, keep, kc):  # the single collective: all-gather of padded detections (+ counts, keep rows)
        g_dets, g_kc, g_keep = gather_detections(dets, kc, keep)
        return g_dets, g_keep, g_kc

    elapsed, lat, lat1, kc = timed_leg(args, det, mode, dist_on, gather, lat_ev)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist_on:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    images = world * args.batch * args.steps
    value = images / elapsed
    det1 = det.slots[0] if pipeline else det

    img_in = image_in_leg(args, det, dev, dist_on, gather) if args.image_in_steps > 0 else None
    rl = roofline(det1, args.roofline_steps, args.precision) if rank == 0 else None
    flops_per_image = det1.engine.flops_per_image
    detections_last_step = int(kc.sum().item())
    # the fp16 (north_star 1e-3) leg: at most 30 timed steps by default, so a long headline run
    # does not double the bench's wall time
    n16 = args.fp16_steps if args.fp16_steps is not None else (min(args.steps, 30) if args.precision == "bf16" else 0)
    npl = args.pipelined_steps if args.pipelined_steps is not None else (min(args.steps, 30) if mode == "concurrent"
                                                                          else 0)
    fp16 = pipelined = None
    legs = not args.diag_forward_only and ((n16 > 0 and args.precision != "fp16") or (npl > 0 and mode == "concurrent"))
    if legs:
        det.close()  # the headline plan's HBM back before another plan is built
        del det, det1, model
    if n16 > 0 and args.precision != "fp16" and not args.diag_forward_only:
        fp16 = precision_leg(args, dev, rank, world, dist_on, gather, mode, "fp16", n16)
    if npl > 0 and mode == "concurrent" and not args.diag_forward_only:
        pipelined = precision_leg(args, dev, rank, world, dist_on, gather, "pipelined", args.precision, npl,
                                  sfx="_pipelined", with_roofline=False)
    cpu = None
    if rank == 0 and world == 1 and args.cpu_seconds > 0:
        cpu = cpu_baseline(args, sd, cfg)
    if rank == 0:
        peak = PEAK[args.precision]
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "p50_ms": round(statistics.median(lat), 4), "p90_ms": round(sorted(lat)[int(0.9 * (len(lat) - 1))], 4),
            "p50_ms_unloaded": round(statistics.median(lat1), 4) if lat1 else None,
            "higher_is_better": True, "scaling": "strong" if args.global_batch else "weak", "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic U[0,1) images, seeded synthetic weights (no checkpoint exists)",
            "config": {"workload": f"{args.net} COCO-{args.nc} {args.size}x{args.size}, {args.batch} images per GPU "
                                   f"per step: forward + decode + NMS (+ all-gather)",
                       "global_batch": world * args.batch, "per_gpu_batch": args.batch, "image_size": args.size,
                       "parallelism": f"dp{world}", "hip_graph": not args.no_graph,
                       "mode": mode, "batches_in_flight": (args.depth if mode == "concurrent" else
                                                           2 if mode == "pipelined" else 1),
                       "latency": "p50_ms: submit -> detections of a batch in the timed loop (batches_in_flight "
                                  "queued); p50_ms_unloaded: host wall time of one batch alone, synchronised",
                       "conf_thres": args.conf, "iou_thres": args.iou, "max_det": args.max_det},
            "mfma_fraction_whole_step": round(flops_per_image * value /
                                              (world * peak * 1e12), 4),
            "roofline": {"bound": "mfma", "kernel": rl['kernel'], "achieved": round(rl['achieved'], 2), "peak": peak,
                         "unit": "TFLOP/s", "frac": round(rl['achieved'] / peak, 4),
                         "traffic": pmc_traffic(rl['kernel'], shape, rnd),
                         "traffic_unit": "bytes/launch (HBM, PMC)", "traffic_round": rnd,
                         "avg_launch_ms": round(rl['avg_launch_ms'], 5),
                         "flops_per_launch": int(rl['flops_per_launch']),
                         "all_conv_tflops": round(rl['all_conv_tflops'], 2),
                         "forward_kernel_ms": round(rl['forward_kernel_ms'], 4),
                         "forward_floor_ms": round(rl['forward_floor_ms'], 4),
                         "forward_events_ms": round(rl['forward_events_ms'], 4),
                         "per_op_timing": "HIP events around every op of 3 serial forwards, less the event-record "
                                          "overhead (events minus the HIP-graph replay forward, spread evenly)",
                         "forward_gap_ms": round(rl['forward_gap_ms'], 4),
                         "dominant_by_bound": rl['dominant_by_bound'],
                         "top_gaps": [[o['i'], o['name'], o['bound'], o['ms'], o['floor_ms'], o['gap_ms']]
                                      for o in sorted(rl['ops'], key=lambda o: -o['gap_ms'])[:8]]},
            "cpu_baseline": cpu,
            "rccl_world_size": dist.get_world_size() if dist_on else 1,
            **(img_in or {}),
            **(fp16 or {}),
            **(pipelined or {}),
            "detections_last_step": detections_last_step,
        }
        print(json.dumps(out), flush=True)
        if os.environ.get("YCX_BENCH_KERNELS"):  # the per-op roofline gap table (serial leg, HIP events)
            with open(os.environ["YCX_BENCH_KERNELS"], "w") as f:
                json.dump(dict(precision=args.precision, shape=list(shape), peak_tflops=peak,
                               hbm_peak_gbs=HBM_PEAK_GBS, forward_kernel_ms=rl['forward_kernel_ms'],
                               forward_floor_ms=rl['forward_floor_ms'], forward_gap_ms=rl['forward_gap_ms'],
                               forward_events_ms=rl['forward_events_ms'], forward_graph_ms=rl['forward_graph_ms'],
                               per_kernel=rl['per_kernel'], ops=rl['ops']), f, indent=1)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
