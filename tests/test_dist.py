"""N > 1 data-parallel path on CPU: world_size 2 over gloo.

Each rank fabricates its shard's padded detections; after the single
all-gather every rank must hold all images in rank-major (= original image)
order, and the host conversion must reproduce the reference's output list
shape (np.float32 (K, 7) or None per image)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ycx.dist import gather_detections, shard, to_output_list

MAX_DET = 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _fake_shard(images):
    """Deterministic padded detections for global image ids ``images``."""
    n = len(images)
    dets = torch.full((n, MAX_DET, 7), -1.0)
    keep = torch.full((n, MAX_DET), -1, dtype=torch.int32)
    cnt = torch.zeros(n, dtype=torch.int32)
    for i, g in enumerate(images):
        k = g % (MAX_DET + 1)  # image 0 and 6 keep nothing
        cnt[i] = k
        for j in range(k):
            dets[i, j] = torch.tensor([g, j, g + 1, j + 1, 0.5, 0.25, g % 3], dtype=torch.float32)
            keep[i, j] = 100 * g + j
    return dets, keep, cnt


def _worker(rank, world, port, global_batch, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sl = shard(global_batch, rank, world)
        dets, keep, cnt = _fake_shard(list(range(sl.start, sl.stop)))
        g_dets, g_cnt, g_keep = gather_detections(dets, cnt, keep)
        q.put((rank, g_dets.numpy(), g_cnt.numpy(), g_keep.numpy()))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_shard_is_a_partition():
    for gb in (1, 7, 32, 256):
        for world in (1, 2, 3, 8):
            ids = [i for r in range(world) for i in range(gb)[shard(gb, r, world)]]
            assert ids == list(range(gb))


@pytest.mark.parametrize("global_batch", [8, 64])
def test_gather_world2_gloo(global_batch):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, global_batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want_dets, want_keep, want_cnt = _fake_shard(list(range(global_batch)))
    for rank, g_dets, g_cnt, g_keep in results:
        np.testing.assert_array_equal(g_dets, want_dets.numpy())
        np.testing.assert_array_equal(g_cnt, want_cnt.numpy())
        np.testing.assert_array_equal(g_keep, want_keep.numpy())
    out = to_output_list(torch.from_numpy(results[0][1]), torch.from_numpy(results[0][2]))
    assert len(out) == global_batch
    for g, o in enumerate(out):
        k = g % (MAX_DET + 1)
        if k == 0:
            assert o is None
        else:
            assert o.dtype == np.float32 and o.shape == (k, 7) and o[0, 0] == g


def test_to_output_list_truncation_is_explicit():
    """count > max_det: the list holds max_det rows for that image, and the
    result says so (raw counts + truncated flags + a warning), never a silent
    slice that disagrees with the count."""
    max_det = 4
    dets = torch.arange(3 * max_det * 7, dtype=torch.float32).reshape(3, max_det, 7)
    counts = torch.tensor([2, 9, 0], dtype=torch.int32)
    with pytest.warns(RuntimeWarning, match="truncated"):
        out = to_output_list(dets, counts)
    assert out[0].shape == (2, 7) and out[1].shape == (max_det, 7) and out[2] is None
    assert out.truncated == [False, True, False] and out.any_truncated
    assert out.counts.tolist() == [2, 9, 0]
    np.testing.assert_array_equal(out[1], dets[1].numpy())
    import warnings
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        ok = to_output_list(dets, torch.tensor([1, 4, 0], dtype=torch.int32))
    assert not ok.any_truncated and ok[1].shape == (4, 7)


def test_bench_launches_n_ranks_itself():
    """``python bench.py --gpus 2`` (no torchrun, no WORLD_SIZE)
    starts its own 2 rank processes; --dry-run takes the launcher path with a
    gloo group instead of the GPU legs. Exactly one JSON line (rank 0) comes out,
    and it reports the process group's world size."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dry-run", "--batch", "4"],
                       env=env, capture_output=True, text=True, timeout=180, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["rccl_world_size"] == 2 and out["n_gpus"] == 2 and out["rank_major_order"]
    assert out["gathered_dets"] == [8, 300, 7] and out["gathered_keep"] == [8, 300]


def test_launcher_parent_never_initialises_the_gpu(tmp_path):
    """the rank launcher counts GPUs from the environment /
    KFD sysfs only. In a child interpreter every torch.cuda entry that could
    reach HIP is made to raise; the 2-rank dry run must still succeed, leave
    torch.cuda uninitialised in the parent, and refuse --gpus 2 when only one
    device is visible."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prog = f"""
import sys, torch
sys.path.insert(0, {repo!r})
def boom(*a, **k):
    raise AssertionError("launcher parent touched torch.cuda")
for name in ("device_count", "init", "_lazy_init", "is_available", "set_device", "synchronize"):
    setattr(torch.cuda, name, boom)
import bench
rc = bench.main(["--gpus", "2", "--dry-run", "--batch", "2"])
assert not torch.cuda.is_initialized()
print("RC", rc)
"""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["HIP_VISIBLE_DEVICES"] = "0,1"
    r = subprocess.run([sys.executable, "-c", prog], env=env, capture_output=True, text=True, timeout=180, cwd=repo)
    assert r.returncode == 0 and "RC 0" in r.stdout, r.stderr[-2000:]
    env["HIP_VISIBLE_DEVICES"] = "0"  # the real (non-dry) launcher refuses before it starts any rank
    prog = prog.replace('"--dry-run", ', "")
    r = subprocess.run([sys.executable, "-c", prog], env=env, capture_output=True, text=True, timeout=180, cwd=repo)
    assert r.returncode != 0 and "only 1 GPU(s) are visible" in r.stderr


def test_visible_gpus_from_kfd_topology(tmp_path):
    """visible_gpus without *_VISIBLE_DEVICES: KFD nodes with SIMDs are GPUs."""
    import bench
    for i, simds in enumerate((0, 1024, 1024, 0)):
        d = tmp_path / str(i)
        d.mkdir()
        (d / "properties").write_text(f"cpu_cores_count 8\nsimd_count {simds}\n")
    assert bench.visible_gpus(env={}, kfd_nodes=str(tmp_path)) == 2
    assert bench.visible_gpus(env={}, kfd_nodes=str(tmp_path / "missing")) is None
    assert bench.visible_gpus(env={"ROCR_VISIBLE_DEVICES": "0,1,2", "HIP_VISIBLE_DEVICES": "1"}) == 1
