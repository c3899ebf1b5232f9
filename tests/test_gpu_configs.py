"""BASELINE.json configs other than the headline bench line, as parity cases.

C4: yolov7 COCO-80 at 1280x1280, bs=8, bf16 on one GPU (head grids
40^2/80^2/160^2, 100,800 candidates per image). The whole batch runs on the GPU; the
oracle (fp32 CPU restatement, pinned to the reference's goldens) recomputes the first
and the last image only, which is what keeps this test to seconds on the host.

Tolerances: bf16 forward 5e-2 of max |ref| per head (as tests/test_gpu_model.py);
the fused decode+NMS path is decomposed by helpers.fused_keep_report against the
oracle chain on the same heads: decoded boxes <= 2e-6, membership flips only at
conf_thres, keep rows bit-exact on the device's own candidates, and the
end-to-end keep-set difference pinned to its measured value (KEEP_FLIPS_PIN).
"""
import numpy as np
import pytest
import torch

from helpers import ANCHORS, MASK, fused_keep_report, make_model, rel_err
from oracle import ref_forward
from ycx.detect import ConcurrentDetector, Detector, device_nms
from ycx.utils.helper_io import cvt_cfg
from ycx.utils.synth import synthetic_images

pytestmark = pytest.mark.gpu
A = np.asarray(ANCHORS).reshape(-1, 2)
C2_BAR, C5_BAR = 1e-2, 0.10   # heads: max |gpu - oracle| / max |oracle| (bf16, fp8 e4m3); measured r02: 0.0045, 0.088
# end-to-end keep-set differences over the FULL survivor lists (images 0 / n-1), all from
# sigmoid/exp ulps in the device decode (nms_exact holds on the device's own candidates);
# measured r03 on MI355X: c2 3 / 0 of 9725 / 9754 kept, c5 0 / 0 of 9685 / 9659, c4 6 of 38781
KEEP_FLIPS_PIN = {'c2': 6, 'c5': 4, 'c4': 12, 'c2h': 6}


@pytest.fixture(scope='module')
def c4(device):
    m, sd = make_model('yolov7', 80, 0, 'bf16')
    m.to(device)
    shape = (8, 3, 1280, 1280)
    x = synthetic_images(*shape, seed=11)
    det = Detector(m, shape, device, ANCHORS, MASK, conf_thres=0.3, nms_thres=0.3, max_det=50000)
    dets, keep, kc = det(x.to(device))
    torch.cuda.synchronize()
    heads = [h.cpu() for h in det.heads]
    ref = ref_forward.build(cvt_cfg('yolov7'), ANCHORS, 80, sd)(x[[0, 7]])
    return dict(m=m, heads=heads, keep=keep.cpu(), kc=kc.cpu(), dets=dets.cpu(), ref=ref, cand=det.cand.cpu(),
                cand_rows=det.cand_rows.cpu(), counts=det.counts.cpu())


def test_c4_1280_forward_vs_oracle(c4):
    assert [tuple(h.shape) for h in c4['heads']] == [(8, 255, 40, 40), (8, 255, 80, 80), (8, 255, 160, 160)]
    for h, r in zip(c4['heads'], c4['ref']):
        for gi, ri in ((0, 0), (7, 1)):
            assert rel_err(h[gi], r[ri]) < 5e-2, (tuple(h.shape), gi, rel_err(h[gi], r[ri]))


def test_c4_1280_decode_nms_vs_oracle(c4):
    assert all(int(c) > 0 for c in c4['kc'])  # every image of the batch produced detections
    for b in (0, 7):  # the first and the last image of the batch (verdict r05 item 8)
        rep = fused_keep_report(c4['cand'], c4['cand_rows'], c4['counts'], c4['keep'], c4['kc'], b,
                                [h[b] for h in c4['heads']], 80, 0.3, 0.3, 1280, 50000)
        print(f"\nc4 image {b}: {rep}")
        assert rep['cls_same'] and rep['nms_exact'], rep
        assert rep['box_maxdiff'] <= 2e-6 and rep['member_max_dist'] <= 1e-6, rep
        assert rep['keep_flips'] <= KEEP_FLIPS_PIN['c4'] and rep['unexplained_flips'] == 0, rep
        k = int(c4['kc'][b])
        assert 0 < k <= 50000 and (k == 50000 or int(c4['keep'][b, k:].max()) == -1)


# ---------------------------------------------------------------------------
# The benchmarked plans themselves (the conv tile picker depends on
# M = n*Ho*Wo, so bs=2 tests do not run the kernels bench.py times). C2 and C5
# are built exactly as bench.py builds them -- same Model, weights recipe,
# ConcurrentDetector (3 slots on 3 HIP streams, HIP graphs), shape and
# precision, hence the same conv descriptors and tiles -- with three batches in
# flight; the last one is checked against the oracle.
# ---------------------------------------------------------------------------


def _bench_config(device, precision, bs, seed):
    m, sd = make_model('yolov7', 80, 0, precision)
    m.to(device)
    shape = (bs, 3, 640, 640)
    cd = ConcurrentDetector(m, shape, device, ANCHORS, MASK, depth=3, conf_thres=0.3, nms_thres=0.3, max_det=300)
    x = synthetic_images(*shape, seed=seed)
    for i in range(3):  # three batches in flight; the third (slot 2) is the one checked
        cd.submit(x.to(device) if i == 2 else synthetic_images(*shape, seed=seed + 1 + i).to(device))
    cd.synchronize()
    torch.cuda.synchronize()
    det = cd.slots[2]
    tiles = {}
    for info in det.engine.op_info:
        tiles[info['name']] = tiles.get(info['name'], 0) + 1
    print(f"\n{precision} bs={bs} plan tiles: {tiles}")
    # the bench slot keeps max_det = 300 rows per image; for the parity check the same
    # device candidates go through ycx_sort_nms again with room for every survivor
    # (max_det = rows_total), and the bench's 300 rows must be that list's prefix
    rows_total = det.cand.shape[1]
    _, keep_full, kc_full = device_nms(det.cand, det.cand_rows, det.counts, 80, 0.3, rows_total)
    torch.cuda.synchronize()
    keep_full, kc_full = keep_full.cpu(), kc_full.cpu()
    keep300, kc300 = det.keep.cpu(), det.kc.cpu()
    assert torch.equal(kc_full, kc300), "the uncapped survivor counts depend on max_det"
    assert torch.equal(keep_full[:, :300], keep300), "the bench's 300 rows are not the full list's prefix"
    out = dict(heads=[h.cpu() for h in det.heads], cand=det.cand.cpu(), cand_rows=det.cand_rows.cpu(),
               counts=det.counts.cpu(), keep=keep_full, kc=kc_full, tiles=tiles, bs=bs, rows_total=rows_total)
    ref = ref_forward.build(cvt_cfg('yolov7'), ANCHORS, 80, sd)(x[[0, bs - 1]])
    out['ref'] = ref
    del cd, det
    m.invalidate()
    torch.cuda.empty_cache()
    return out


@pytest.fixture(scope='module')
def c2(device):
    return _bench_config(device, 'bf16', 32, 50)


@pytest.fixture(scope='module')
def c5(device):
    return _bench_config(device, 'fp8', 64, 60)


@pytest.fixture(scope='module')
def c2h(device):
    return _bench_config(device, 'fp16', 32, 50)


def _check_heads(cfg, bar):
    bs = cfg['bs']
    errs = []
    for h, r in zip(cfg['heads'], cfg['ref']):
        for gi, ri in ((0, 0), (bs - 1, 1)):
            errs.append(rel_err(h[gi], r[ri]))
    print(f"\nheads rel err (img 0, img {bs - 1}) per level: {[round(e, 4) for e in errs]}")
    assert max(errs) < bar, errs


def _check_keep(cfg, name):
    """Every survivor's keep row of images 0 and n-1 (not the first 300)."""
    for b in (0, cfg['bs'] - 1):
        assert int(cfg['kc'][b]) > 300  # the bench load: thousands of survivors per image
        rep = fused_keep_report(cfg['cand'], cfg['cand_rows'], cfg['counts'], cfg['keep'], cfg['kc'], b,
                                [h[b] for h in cfg['heads']], 80, 0.3, 0.3, 640, cfg['rows_total'])
        print(f"\n{name} image {b}: {rep}")
        assert rep['cls_same'], "class ids differ on common candidates"
        assert rep['box_maxdiff'] <= 2e-6, rep          # device decode vs oracle decode, normalised xyxy
        assert rep['member_max_dist'] <= 1e-6, rep      # membership flips only at conf_thres
        assert rep['nms_exact'], rep                    # keep rows bit-exact on the device's own candidates
        assert rep['keep_flips'] <= KEEP_FLIPS_PIN[name] and rep['unexplained_flips'] == 0, rep


def test_c2_bs32_bf16_forward_vs_oracle(c2):
    assert [tuple(h.shape) for h in c2['heads']] == [(32, 255, 20, 20), (32, 255, 40, 40), (32, 255, 80, 80)]
    _check_heads(c2, C2_BAR)


def test_c2_bs32_bf16_keep_vs_oracle(c2):
    _check_keep(c2, 'c2')


def test_c5_bs64_fp8_forward_vs_oracle(c5):
    assert [tuple(h.shape) for h in c5['heads']] == [(64, 255, 20, 20), (64, 255, 40, 40), (64, 255, 80, 80)]
    assert any(k.startswith('f8_') for k in c5['tiles'])
    _check_heads(c5, C5_BAR)


def test_c5_bs64_fp8_keep_vs_oracle(c5):
    _check_keep(c5, 'c5')


# ---------------------------------------------------------------------------
# C2 in the fp16 plan (precision='fp16'): the bench's own ConcurrentDetector at bs=32,
# held to north_star's 1e-3 on the raw heads and on the decoded box, objectness and
# class-confidence tensors (decode_box, detect.py:29-87), images 0 and 31.
# ---------------------------------------------------------------------------
F16_BAR = 1e-3


def test_c2_bs32_fp16_heads_vs_oracle(c2h):
    assert [tuple(h.shape) for h in c2h['heads']] == [(32, 255, 20, 20), (32, 255, 40, 40), (32, 255, 80, 80)]
    assert all(bool(torch.isfinite(h).all()) for h in c2h['heads'])
    _check_heads(c2h, F16_BAR)


def test_c2_bs32_fp16_decoded_vs_oracle(c2h):
    from oracle import ref_post
    dev = torch.cat(ref_post.decode_box([h[[0, 31]] for h in c2h['heads']], A, MASK, 80, (640, 640)), 1)
    ref = torch.cat(ref_post.decode_box(c2h['ref'], A, MASK, 80, (640, 640)), 1)
    errs = {k: rel_err(dev[..., sl], ref[..., sl]) for k, sl in
            (('box', slice(0, 4)), ('obj', slice(4, 5)), ('cls', slice(5, 85)))}
    print(f"\nfp16 C2 decoded rel err (images 0, 31): {errs}")
    assert max(errs.values()) < F16_BAR, errs


def test_c2_bs32_fp16_keep_vs_oracle(c2h):
    _check_keep(c2h, 'c2h')
