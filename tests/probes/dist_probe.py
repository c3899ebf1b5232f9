"""Why does the N > 1 code path serialise the concurrent detector? (development probe)

    python tests/probes/dist_probe.py
One rank, process group over RCCL; the bench's concurrent loop with the
detections all-gather done in several ways; prints ms per step for each.
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "yolo-continuous_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29512")
    args = bench.parse(["--cpu-seconds", "0"])
    first = os.environ.get("PROBE_PG_FIRST") == "1"  # the bench's order: process group before the plan
    pg_kw = {}
    if os.environ.get("PROBE_HIPRIO") == "1":  # communicator stream from the high-priority pool
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        pg_kw = dict(pg_options=opts)
    if first:
        dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1, **pg_kw)
        if os.environ.get("PROBE_WARM_COLL") == "1":  # create the communicator's stream now
            w = torch.zeros(8, device=dev)
            dist.all_gather_into_tensor(torch.empty_like(w), w)
            torch.cuda.synchronize()
    _, det, _, _, _ = bench.setup(args, dev, pipeline="concurrent")
    if not first and os.environ.get("PROBE_NO_PG") != "1":
        dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)
    print("process group first:", first, flush=True)
    s_coll = torch.cuda.Stream(dev, priority=-1 if os.environ.get("PROBE_HIPRIO") == "1" else 0)

    def gather_plain(t):
        out = t.new_empty(t.shape)
        dist.all_gather_into_tensor(out, t.contiguous())
        return out

    def gather_async(t):
        out = t.new_empty(t.shape)
        dist.all_gather_into_tensor(out, t.contiguous(), async_op=True)
        return out

    def gather_copy(t):  # what a 1-rank gather computes, without RCCL
        return t.clone()

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    from ycx.dist import gather_detections
    held = [None]
    order = [("gd_keep", "gd"), ("none", None), ("rccl", gather_plain), ("gd_keep2", "gd"), ("none2", None)]
    for name, fn in order:
        if name.startswith("rccl") and not dist.is_initialized():
            continue
        use_ev = name.endswith("_ev")
        it = [0]

        def step():
            ev = evs[it[0] % 20] if use_ev else None
            it[0] += 1
            dets, keep, kc, done = det.submit(timing=(ev[0], None) if ev else None)
            if fn == "gd":
                with torch.cuda.stream(s_coll):
                    s_coll.wait_event(done)
                    g = gather_detections(dets, kc, keep)
                    if name.startswith("gd_keep"):
                        held[0] = g[1]  # the bench keeps the gathered counts until the next step
            elif fn is not None:
                with torch.cuda.stream(s_coll):
                    s_coll.wait_event(done)
                    fn(dets), fn(kc), fn(keep)
                    if ev:
                        ev[1].record(s_coll)
            elif ev:
                ev[1].record(s_coll)
        for _ in range(5):
            step()
        det.synchronize()
        torch.cuda.current_stream().wait_stream(s_coll)
        torch.cuda.synchronize()
        if os.environ.get("PROBE_BARRIER") == "1" and dist.is_initialized():
            dist.barrier()  # the bench's barrier between warm-up and the timed loop
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            step()
        det.synchronize()
        torch.cuda.current_stream().wait_stream(s_coll)
        torch.cuda.synchronize()
        print(f"{name:12s} {(time.perf_counter() - t0) / 20 * 1e3:.3f} ms/step", flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
