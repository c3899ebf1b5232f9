"""Achievable HBM bandwidth on the box (development probe): torch copy of a 419 MB / 1 GB bf16
tensor (read + write), the practical ceiling the memory-bound layers are compared with.

    python tools/hbm_probe.py
"""
import torch, time
dev = torch.device("cuda:0")
for mb in (419, 1024):
    n = mb * 1024 * 1024 // 2
    a = torch.randn(n, device=dev).to(torch.bfloat16)
    b = torch.empty_like(a)
    for _ in range(3): b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): b.copy_(a)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"copy {mb} MB: {ms:.4f} ms, {2 * a.numel() * 2 / ms / 1e6:.0f} GB/s (read + write)")
    e0.record()
    for _ in range(20): a.max()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"max-reduce {mb} MB: {ms:.4f} ms, {a.numel() * 2 / ms / 1e6:.0f} GB/s (read)")
