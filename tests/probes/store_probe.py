"""Store-pattern microbenchmark (development probe): see store_probe.hip.

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tests/probes/store_probe.hip -o tests/probes/build/store_probe.so
    python tests/probes/store_probe.py
"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "build", "store_probe.so"))
    dev = torch.device("cuda:0")
    rows = 32 * 160 * 160  # 819200 rows x 512 B = 419 MB
    y = torch.empty(rows * 512, dtype=torch.uint8, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    tiles = rows // 64
    for pat in (0, 1, 2):
        for blocks in (256, 512, 1024, tiles):
            tpb = -(-tiles // blocks)
            f = lambda: lib.store_probe(pat, ctypes.c_void_p(y.data_ptr()), rows, blocks, tpb, st)
            for _ in range(3):
                f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                f()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 20
            print(f"pattern {pat} blocks {blocks:6d} x {tpb:3d} tiles: {ms:.4f} ms {rows * 512 / ms / 1e6:.0f} GB/s",
                  flush=True)


if __name__ == "__main__":
    main()
