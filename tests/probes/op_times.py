"""Per-op times of one serial forward (bench.py's roofline leg: HIP events around every op of
the plan), largest first (development probe).

    python tests/probes/op_times.py [bench args, e.g. --precision fp8 --batch 64]
Prints op index, kernel tile, shape (n, h, w, cin, cout, k, s), ms and TFLOP/s, then the total.
"""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, '..', '..'), os.path.join(HERE, '..', '..', 'yolo-continuous_amd')]
import bench  # noqa: E402


def main():
    args = bench.parse(["--cpu-seconds", "0"] + sys.argv[1:])
    dev = torch.device("cuda:0")
    _, det, _, _, _ = bench.setup(args, dev)
    for _ in range(3):
        det()
    torch.cuda.synchronize()
    rl = bench.roofline(det, 5, args.precision)
    ops = sorted(rl['ops'], key=lambda o: -o['ms'])
    for o in ops[:int(os.environ.get("OP_TOP", "40"))]:
        print(f"op{o['i']:3d} {o['ms']:8.4f} ms {str(o['tflops']):>7} TF  {o['name']:<36} {o['shape']}")
    print(f"forward kernels {rl['forward_kernel_ms']:.3f} ms, convs {rl['all_conv_tflops']:.0f} TF")


if __name__ == "__main__":
    main()
