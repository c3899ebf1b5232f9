import sys, time, numpy as np, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/yolo-continuous_amd')
from ycx.detect import Detector
from ycx.nets.yolo import Model
from ycx.utils.helper_io import cvt_cfg
from ycx.utils.synth import synthetic_images, synthetic_state_dict
A = [[12, 16, 19, 36, 40, 28], [36, 75, 76, 55, 72, 146], [142, 110, 192, 243, 459, 401]]
M = [[6, 7, 8], [3, 4, 5], [0, 1, 2]]
dev = torch.device('cuda:0')
m = Model(cvt_cfg('yolov7'), A, 80).eval(); m.load_state_dict(synthetic_state_dict(m, 0)); m.to(dev)
det = Detector(m, (32, 3, 640, 640), dev, A, M, conf_thres=0.3, nms_thres=0.3)
det.x.copy_(synthetic_images(32, 3, 640, 640, seed=1000).to(dev))
det(); torch.cuda.synchronize()
cnt = det.counts.cpu()
print('candidates/img', cnt.tolist()[:8], 'kept', det.kc.cpu().tolist()[:8], flush=True)
cls = det.cand[0, :, 6].view(torch.int32)
rows = det.cand_rows[0, :int(cnt[0])].long()
h = torch.bincount(cls[rows].cpu(), minlength=80)
print('class hist img0 (sorted desc)', sorted(h.tolist(), reverse=True)[:12], flush=True)
for name, fn in [('replay', lambda: det.engine.replay()), ('post', det.post)]:
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5): fn()
    e1.record(); torch.cuda.synchronize(); print(name, 'ms', e0.elapsed_time(e1) / 5, flush=True)
