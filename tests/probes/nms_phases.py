"""Per-phase cycle counts of nms_big on the bench workload (development probe).

    make -C yolo-continuous_amd/csrc prof
    python tests/probes/nms_phases.py
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("YCX_LIB", os.path.join(REPO, "yolo-continuous_amd", "ycx", "libycx_hip_prof.so"))
sys.path[:0] = [REPO, os.path.join(REPO, "yolo-continuous_amd")]

import torch  # noqa: E402

import bench  # noqa: E402
from ycx import _lib as L  # noqa: E402

PHASES = ["sort", "spatial", "suppressors", "rounds", "compact"]


def main():
    args = bench.parse(["--cpu-seconds", "0"] + os.environ.get("NMS_PROBE_ARGS", "").split())
    dev = torch.device("cuda:0")
    _, det, _, _, _ = bench.setup(args, dev, use_graph=False)
    det()
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * 32)()
    prof = hasattr(L.lib, "ycx_nms_prof_read")  # False on the release library: post time only
    if not prof:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        det.forward()
        e0.record()
        for _ in range(5):
            det.post()
        e1.record()
        torch.cuda.synchronize()
        print(f"release library: post ms {e0.elapsed_time(e1) / 5:.3f}")
        return
    L.lib.ycx_nms_prof_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.lib.ycx_nms_prof_read(buf, 1)
    reps = 3
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    det.forward()  # zeroes the candidate counts when the heads decode in the convs
    e0.record()
    for _ in range(reps):
        det.post()
    e1.record()
    torch.cuda.synchronize()
    L.lib.ycx_nms_prof_read(buf, 1)
    tasks = buf[7] // reps
    print(f"post ms {e0.elapsed_time(e1) / reps:.3f}  big tasks/step {tasks}")
    for i, n in enumerate(PHASES):
        print(f"  {n:12s} {buf[i] / max(1, buf[7]) / 1e3:9.1f} kcycles/task")
    print(f"  rounds/task {buf[5] / max(1, buf[7]):.1f}   boxes with > kSlots suppressors/task {buf[6] / max(1, buf[7]):.1f}")
    nt = max(1, buf[7])
    print(f"  candidate visits/task {buf[8] / nt:.0f}  sum of per-wave max visits x64/task {64 * buf[9] / nt:.0f}  "
          f"suppressor pairs/task {buf[10] / nt:.0f}")
    print(f"  search: mean wave {buf[11] / (16 * nt) / 1e3:.1f} kcycles, slowest wave {buf[12] / nt / 1e3:.1f} kcycles, "
          f"slowest wave's visits {buf[13] / nt:.0f} (mean {buf[8] / (16 * nt):.0f})")
    wt = buf[16 + 7]
    if wt:
        print(f"  nms_wide: {wt // reps} tasks/step; " + "  ".join(
            f"{n} {buf[16 + i] / wt / 1e3:.1f}" for i, n in enumerate(PHASES)) + f" kcycles/task; rounds/task {buf[21] / wt:.1f}; "
              f"positions visited in rounds/task {buf[22] / wt:.0f}")
        print(f"  wide sort: key build {buf[24] / wt / 1e3:.1f}  passes {buf[25] / wt / 1e3:.1f} kcycles/task over "
              f"{buf[26] / wt:.1f} passes")
    cnt = det.counts.cpu()
    print("candidates/img", cnt.float().mean().item())
    ws = det.ws.view(torch.int32).cpu()  # header (ntasks) then the task table {img, cls, off, S} at byte 256
    nt = int(ws[0])
    S = ws[64:64 + 4 * nt].view(nt, 4)[:, 3].sort().values
    lds_cap = (159744 - 22016 - 32) // 19
    print(f"big classes {nt}: S min {int(S[0])} median {int(S[nt // 2])} max {int(S[-1])}, "
          f"{int((S > lds_cap).sum())} over the LDS capacity {lds_cap}")


if __name__ == "__main__":
    main()
