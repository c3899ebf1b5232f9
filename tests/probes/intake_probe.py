"""L2 -> CU intake microbenchmark (development probe): see intake_probe.hip.

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC tests/probes/intake_probe.hip -o tests/probes/build/intake_probe.so
    python tests/probes/intake_probe.py
"""
import ctypes
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "build", "intake_probe.so"))
    dev = torch.device("cuda:0")
    src = torch.randint(0, 255, (64 << 20,), dtype=torch.uint8, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    steps = 1000
    cases = []
    for src_mb in (2, 32):
        for stride in (2048, 128):
            for mode, lds, infl, bar, bpc in [(0, 64, 1, 1, 2), (0, 64, 2, 1, 2), (0, 64, 1, 0, 2), (0, 64, 2, 0, 2),
                                              (0, 64, 4, 0, 2), (0, 32, 1, 1, 4), (0, 32, 2, 1, 4), (0, 32, 4, 0, 4),
                                              (0, 128, 2, 0, 1), (0, 128, 4, 0, 1),
                                              (1, 64, 1, 1, 2), (1, 64, 1, 0, 2), (1, 32, 1, 0, 4),
                                              (2, 64, 1, 0, 2), (2, 32, 1, 0, 4)]:
                cases.append((src_mb, stride, mode, lds, infl, bar, bpc))
    for src_mb, stride, mode, lds, infl, bar, bpc in cases:
        blocks = 256 * bpc
        mask = (src_mb << 20) - 1
        f = lambda: lib.intake_probe(mode, lds, infl, bar, ctypes.c_void_p(src.data_ptr()), mask, stride, steps,
                                     blocks, ctypes.c_void_p(sink.data_ptr()), st)
        for _ in range(2):
            f()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 5
        gbs = blocks * steps * 32768 / (ms * 1e-3) / 1e9
        print(f"src {src_mb:3d} MB stride {stride:5d} mode {mode} lds {lds:3d}K infl {infl} bar {bar} blocks/CU {bpc}: "
              f"{ms:.3f} ms  {gbs / 1e3:.2f} TB/s  {gbs / 256:.1f} GB/s per CU", flush=True)


if __name__ == "__main__":
    main()
