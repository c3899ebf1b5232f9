"""Library GEMM timings (torch -> hipBLASLt/rocBLAS) for the yolov7 1x1-conv shapes, as a
reference point for the hand-written kernels (development probe)."""
import torch

SHAPES = [(819200, 256, 256), (819200, 128, 128), (204800, 512, 512), (204800, 256, 256), (51200, 1024, 1024),
          (819200, 256, 128), (204800, 512, 256)]


def main():
    dev = torch.device("cuda:0")
    for m, k, n in SHAPES:
        a = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
        w = torch.randn(n, k, device=dev, dtype=torch.bfloat16)
        out = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        for _ in range(3):
            torch.mm(a, w.t(), out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            torch.mm(a, w.t(), out=out)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(f"M={m} K={k} N={n}: {ms:.4f} ms  {2 * m * n * k / ms / 1e9:.0f} TF  "
              f"{2 * (m * k + m * n + n * k) / ms / 1e9:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
