"""decode_box / non_max_suppression / fused Detector on the GPU vs the golden
fixtures and the oracle.

  decode          : <= 1e-6 relative (fp32; GPU expf vs CPU vectorised exp may differ by ~1 ulp)
  NMS keep rows   : bit-exact on identical decoded inputs (G3 fixtures)
  final (K, 7)    : bit-exact (same fp32 xyxy ops, same numpy yolo_correct_boxes)
"""
import numpy as np
import pytest
import torch

from helpers import ANCHORS, MASK, fused_keep_report, g3_heads, make_model, rel_err
from oracle import ref_forward, ref_post
from ycx.detect import (ConcurrentDetector, Detector, DevicePost, PipelinedDetector, decode_box, nms_device,
                        non_max_suppression)
from ycx.utils.helper_io import cvt_cfg
from ycx.utils.synth import synthetic_images

pytestmark = pytest.mark.gpu
CASES = ['coco80_bs4', 'nc1_bs2', 'nc3_dense']
# end-to-end keep-set differences of the fused path (device sigmoid ulps at the
# thresholds), pinned to the values measured on MI355X
FLIPS_PIN = {'g3': 0, 'tiny320': 0}   # measured: 0 everywhere
A = np.asarray(ANCHORS).reshape(-1, 2)


def _oracle_decoded(e):
    heads = g3_heads(e)
    return heads, torch.cat(ref_post.decode_box(heads, A, MASK, e['nc'], (e['size'], e['size'])), 1)


@pytest.mark.parametrize('name', CASES)
def test_decode_box(device, manifest, name):
    e = manifest['g3'][name]
    heads, ref = _oracle_decoded(e)
    outs = decode_box([h.to(device) for h in heads], A, MASK, e['nc'], (e['size'], e['size']))
    got = torch.cat(outs, 1).cpu()
    assert got.shape == ref.shape
    d = (got.double() - ref.double()).abs()
    assert float((d / ref.double().abs().clamp_min(1e-3)).max()) < 1e-5
    assert float(d.max()) < 1e-5


@pytest.mark.parametrize('name', CASES)
def test_nms_keep_rows_bit_exact(device, manifest, g3, name):
    e = manifest['g3'][name]
    _, dec = _oracle_decoded(e)
    pred = dec.clone().to(device)
    dets, keep, kc = nms_device(pred, e['nc'], e['conf'], e['iou'])
    torch.cuda.synchronize()
    xyxy_ref = dec.clone()
    ref_post.nms_keep_rows(xyxy_ref, e['nc'], e['conf'], e['iou'])
    assert torch.equal(pred.cpu(), xyxy_ref), "xywh->xyxy in-place mutation differs (detect.py:98-103)"
    for b in range(e['bs']):
        k = int(kc[b])
        gold = g3[f'{name}/keep_rows/{b}']
        assert k == len(gold) == e['n_keep'][b]
        np.testing.assert_array_equal(keep[b, :k].cpu().numpy(), gold)
        assert (keep[b, k:] == -1).all()


def misaligned(h):
    """The same values at a 4-byte (not 16-byte) aligned address: ycx_decode_filter then
    takes its one-row-per-thread kernel (decode_filter_kernel), as it does for heads with
    h*w % 4 != 0 or unaligned pointers."""
    buf = torch.empty(h.numel() + 4, dtype=h.dtype, device=h.device)
    v = buf[1:1 + h.numel()].view(h.shape)
    v.copy_(h)
    assert v.data_ptr() % 16 != 0 and v.is_contiguous()
    return v


@pytest.mark.parametrize('scalar', [False, True])
@pytest.mark.parametrize('name', CASES)
def test_device_post_g3(device, manifest, g3, name, scalar):
    """DevicePost (fused ycx_decode_filter + ycx_sort_nms, the Detector's post and
    bench.py --post-micro) on the G3 head logits vs the golden keep rows. The
    fused filter evaluates the sigmoids on the GPU, so a candidate at the conf
    boundary may flip by an ulp; no systematic difference is allowed."""
    e = manifest['g3'][name]
    heads = [h.to(device).contiguous() for h in g3_heads(e)]
    if scalar:  # the one-row-per-thread kernel (heads with h*w % 4 != 0 or unaligned take it)
        heads = [misaligned(h) for h in heads]
    post = DevicePost(heads, e['nc'], ANCHORS, MASK, (e['size'], e['size']), device, e['conf'], e['iou'],
                      max_det=8192)  # nc3_dense keeps ~1.9k rows per image
    dets, keep, kc = post()
    torch.cuda.synchronize()
    cpu = [t.cpu() for t in (post.cand, post.cand_rows, post.counts, keep, kc)]
    heads_cpu = [h.cpu() for h in heads]
    for b in range(e['bs']):
        k = int(kc[b])
        assert k <= 8192
        rep = fused_keep_report(*cpu, b, [h[b] for h in heads_cpu], e['nc'], e['conf'], e['iou'], e['size'], 8192)
        print(f"\n{name} image {b} scalar={scalar}: {rep}")
        assert rep['cls_same'] and rep['nms_exact'], rep
        assert rep['box_maxdiff'] <= 2e-6 and rep['member_max_dist'] <= 1e-6, rep
        assert rep['keep_flips'] <= FLIPS_PIN['g3'] and rep['unexplained_flips'] == 0, rep
        assert rep['n_keep_ref'] == len(g3[f'{name}/keep_rows/{b}'])  # the oracle chain = the golden
        assert (keep[b, k:] == -1).all()
        assert np.isfinite(dets[b, :k].cpu().numpy()).all()


@pytest.mark.parametrize('scalar', [False, True])
def test_device_post_sparse_class_ties(device, scalar):
    """Sparse rows through both decode_filter kernels (four rows per thread; one
    row per thread with the wave-cooperative class scan for <= 8 rows per wave): ties resolve to the first class (torch.max,
    detect.py:108), a maximum past class 63 is found, and the kept rows and
    classes equal the oracle's."""
    nc, bs, size = 80, 2, 640
    g = torch.Generator().manual_seed(5)
    shapes = [(size // k, size // k) for k in (32, 16, 8)]
    heads = [torch.randn(bs, 3, 5 + nc, h, w, generator=g) for h, w in shapes]
    for hd in heads:
        hd[:, :, 4] = -10.0
    rng = np.random.default_rng(3)
    for b in range(bs):
        for l, hd in enumerate(heads):
            h, w = shapes[l]
            for t in range(12):
                a, y, x = int(rng.integers(3)), int(rng.integers(h)), int(rng.integers(w))
                hd[b, a, 4, y, x] = 5.0
                kind = t % 4
                if kind == 0:
                    hd[b, a, 5:, y, x] = 1.5                 # all tie -> class 0
                elif kind == 1:
                    hd[b, a, 5:, y, x] = 0.0
                    hd[b, a, 5 + np.array([70, 7, 3]), y, x] = 2.0   # tie -> class 3
                elif kind == 2:
                    hd[b, a, 5:, y, x] = -1.0
                    hd[b, a, 5 + 79, y, x] = 3.0             # past the first 64 lanes
    heads = [hd.reshape(bs, 3 * (5 + nc), h, w).contiguous() for hd, (h, w) in zip(heads, shapes)]
    post = DevicePost([misaligned(h.to(device)) if scalar else h.to(device) for h in heads], nc, ANCHORS, MASK,
                      (size, size), device, 0.3, 0.45, 1000)
    dets, keep, kc = post()
    torch.cuda.synchronize()
    dec = torch.cat(ref_post.decode_box(heads, A, MASK, nc, (size, size)), 1)
    ref_keep, ref_dets = ref_post.nms_keep_rows(dec, nc, 0.3, 0.45)
    for b in range(bs):
        k = int(kc[b])
        assert k == len(ref_keep[b]) > 20
        np.testing.assert_array_equal(keep[b, :k].cpu().numpy(), ref_keep[b].numpy())
        np.testing.assert_array_equal(dets[b, :k, 6].cpu().numpy(), ref_dets[b][:, 6].numpy())
    assert {0, 3, 79} <= set(dets[0, :int(kc[0]), 6].cpu().long().tolist())


def test_sigmoid_monotone_every_float(device):
    """The decoders' sigmoid is monotone non-decreasing over all 2^32 floats
    (ycx_check_sigmoid_monotone): the premise of the exact class argmax
    (ycx_internal.h ycx_class_argmax) that reads nc logits and a few sigmoids."""
    import ctypes
    from ycx import _lib as L
    bad = torch.zeros(1, dtype=torch.int64, device=device)
    L.check(L.lib.ycx_check_sigmoid_monotone(ctypes.c_void_p(bad.data_ptr()), L.stream_handle(device)),
            "ycx_check_sigmoid_monotone")
    torch.cuda.synchronize()
    assert int(bad) == 0


@pytest.mark.parametrize('scalar', [True, False])
def test_device_post_dense_class_scan(device, scalar):
    """Dense waves (every row passes on objectness) with crafted class logits:
    saturated ties (several logits past ~17 give sigmoid 1.0: first such class),
    exact ties, near-ties one float apart, +inf, -inf and NaN (class 0 NaN sticks,
    later NaNs never win). Every candidate's (cls, cls_conf) equals the
    sequential strict-'>' scan over the device's own sigmoids (ycx_decode),
    i.e. the exact class argmax is the scan bit for bit."""
    nc, bs, size = 80, 2, 320
    g = torch.Generator().manual_seed(11)
    shapes = [(size // k, size // k) for k in (32, 16, 8)]
    heads = [torch.randn(bs, 3, 5 + nc, h, w, generator=g) * 3.0 for h, w in shapes]
    rng = np.random.default_rng(7)
    for hd in heads:
        hd[:, :, 4] = 6.0
        flat = hd.permute(0, 1, 3, 4, 2).reshape(-1, 5 + nc)   # view: rows x channels
        for r in rng.choice(flat.shape[0], size=flat.shape[0] // 2, replace=False):
            kind = int(rng.integers(9))
            ks = rng.choice(nc, size=3, replace=False)
            if kind == 0:
                flat[r, 5 + ks] = torch.tensor([18.0, 25.0, 40.0])          # saturated: all 1.0
            elif kind == 1:
                flat[r, 5 + ks] = 4.25                                       # exact tie
            elif kind == 2:
                v = np.float32(2.5)
                flat[r, 5 + ks[0]] = float(v)
                flat[r, 5 + ks[1]] = float(np.nextafter(v, np.float32(0)))   # one float below
                flat[r, 5 + ks[2]] = float(np.nextafter(v, np.float32(9)))   # one float above
            elif kind == 3:
                flat[r, 5 + ks[0]] = float('inf')
                flat[r, 5 + ks[1]] = 30.0
            elif kind == 4:
                flat[r, 5 + ks[0]] = float('-inf')
            elif kind == 5:
                flat[r, 5 + ks[0]] = float('nan')
                flat[r, 5 + ks[1]] = 9.0
            elif kind == 6:
                flat[r, 5] = float('nan')                                    # class 0 NaN sticks
            elif kind == 7:
                flat[r, 5 + ks] = torch.tensor([16.5, 16.6, 16.7])           # edge of saturation
            else:   # every sigmoid 0: -inf before the largest logit ties it (the scan keeps class 0)
                j = int(ks[0]) % 8 + 1
                flat[r, 5:5 + j] = float('-inf')
                flat[r, 5 + j] = -200.0
                flat[r, 5 + j + 1:] = -250.0
        hd.copy_(flat.reshape(hd.shape[0], hd.shape[1], hd.shape[3], hd.shape[4], 5 + nc).permute(0, 1, 4, 2, 3))
    heads = [hd.reshape(bs, 3 * (5 + nc), h, w).contiguous() for hd, (h, w) in zip(heads, shapes)]
    dh = [misaligned(h.to(device)) if scalar else h.to(device) for h in heads]
    post = DevicePost(dh, nc, ANCHORS, MASK, (size, size), device, 0.0, 0.45, 100)
    post.counts.zero_()
    post()
    dec = torch.cat(decode_box(dh, A, MASK, nc, (size, size)), 1).cpu().numpy()
    torch.cuda.synchronize()
    cls_sig = dec[..., 5:]
    for b in range(bs):
        n = int(post.counts[b])
        rows = np.sort(post.cand_rows[b, :n].cpu().numpy())
        cand = post.cand[b].cpu().numpy()[rows]
        sig = cls_sig[b, rows]
        want_i = np.zeros(len(rows), dtype=np.int64)
        want_v = sig[:, 0].copy()
        for k in range(1, nc):   # the sequential scan of detect.py:109 as the kernels define it
            upd = sig[:, k] > want_v
            want_v[upd] = sig[upd, k]
            want_i[upd] = k
        got_i = cand[:, 6].view(np.int32)
        np.testing.assert_array_equal(got_i, want_i)
        np.testing.assert_array_equal(cand[:, 5].view(np.uint32), want_v.view(np.uint32))
        assert n > 0.4 * dec.shape[1]


@pytest.mark.parametrize('name', CASES)
def test_non_max_suppression_final(device, manifest, g3, name):
    e = manifest['g3'][name]
    _, dec = _oracle_decoded(e)
    res = non_max_suppression(dec.clone().to(device), e['nc'], (e['size'], e['size']), np.array(e['image_shape']),
                              True, e['conf'], e['iou'])
    for b in range(e['bs']):
        np.testing.assert_array_equal(res[b], g3[f'{name}/final/{b}'])


def test_nms_edge_cases(device):
    # no candidate passes -> None, count 0
    pred = torch.zeros(2, 100, 6, device=device)
    pred[..., 4] = 0.1
    pred[..., 5] = 0.5
    assert non_max_suppression(pred.clone(), 1, (64, 64), np.array([64, 64]), False, 0.3, 0.5) == [None, None]
    # identical boxes and scores: stable order keeps the lowest row only
    pred = torch.zeros(1, 8, 7, device=device)
    pred[0, :, :4] = torch.tensor([0.5, 0.5, 0.2, 0.2])
    pred[0, :, 4] = 0.9
    pred[0, :, 5] = 1.0
    _, keep, kc = nms_device(pred.clone(), 2, 0.25, 0.5)
    assert int(kc[0]) == 1 and int(keep[0, 0]) == 0
    # two classes never suppress each other; output grouped by class ascending
    pred[0, 3, 5], pred[0, 3, 6] = 0.0, 1.0  # row 3 -> class 1
    _, keep, kc = nms_device(pred.clone(), 2, 0.25, 0.5)
    assert int(kc[0]) == 2 and keep[0, :2].tolist() == [0, 3]
    # the '>' boundary: a threshold equal to the fp32 IoU keeps both boxes, the
    # next double below suppresses (also exercises the division-free compare)
    pred = torch.zeros(1, 2, 6, device=device)
    pred[0, 0, :4] = torch.tensor([5.0, 5.0, 10.0, 10.0])   # xywh -> xyxy (0, 0, 10, 10)
    pred[0, 1, :4] = torch.tensor([5.5, 5.5, 10.0, 10.0])   # -> (0.5, 0.5, 10.5, 10.5)
    pred[0, :, 4] = torch.tensor([0.9, 0.8])
    pred[0, :, 5] = 1.0
    inter, a0, a1 = np.float32(90.25), np.float32(100.0), np.float32(100.0)
    iou = float(inter / (a0 + a1 - inter))
    for thr, want in ((iou, 2), (np.nextafter(iou, 0.0), 1), (np.nextafter(iou, 1.0), 2)):
        _, keep, kc = nms_device(pred.clone(), 1, 0.1, thr)
        assert int(kc[0]) == want, (thr, int(kc[0]))
    # every row passes (the conf_thres=0.001 evaluation regime): 3 classes of
    # ~5.5k (bitmask path, LDS sort) and one class of 16384 (workspace sort)
    for nc in (3, 1):
        g = torch.Generator().manual_seed(nc)
        pred = torch.rand(1, 16384, 5 + nc, generator=g)
        pred[..., 2:4] *= 0.05
        pred[..., 4] = 0.5 + 0.5 * pred[..., 4]
        pred = pred.to(device)
        ref_keep, _ = ref_post.nms_keep_rows(pred.cpu().clone(), nc, 0.0, 0.3)
        _, keep, kc = nms_device(pred.clone(), nc, 0.0, 0.3)
        k = int(kc[0])
        np.testing.assert_array_equal(keep[0, :k].cpu().numpy(), ref_keep[0].numpy())


def _sorted_cands(det, b):
    n = int(det.counts[b])
    rows = torch.sort(det.cand_rows[b, :n].cpu()).values
    return rows, det.cand[b].cpu()[rows.long()]   # ycx_cand is indexed by row, cand_rows lists the rows


@pytest.mark.parametrize('precision', ['bf16', 'fp8'])
@pytest.mark.parametrize('cfg,nc,shape', [('yolov7-tiny', 1, (3, 3, 224, 224)), ('yolov7-tiny', 80, (2, 3, 320, 256)),
                                          ('yolov7', 80, (2, 3, 256, 256))])
def test_head_decode_fused_in_conv(device, cfg, nc, shape, precision):
    """ycx_conv2d_head (decode + filter in the Detect-head conv epilogue) vs the
    unfused chain (head conv -> fp32 NCHW heads -> ycx_decode_filter) on the
    same model and images: raw heads, candidate rows and values, keep rows and
    dets are all bit-identical, with and without the raw-head store. 224 and
    320x256 put 64-pixel head tiles across image boundaries (7x7, 10x8 grids)."""
    m, _ = make_model(cfg, nc, 0, precision)
    m.to(device)
    x = synthetic_images(*shape, seed=31).to(device)
    conf = 0.3 if nc == 1 else 0.05   # random-init nc=80 scores are ~0.5*0.5; keep the filter busy
    kw = dict(conf_thres=conf, nms_thres=0.45, max_det=1000)
    ref = Detector(m, shape, device, ANCHORS, MASK, fuse_heads=False, **kw)
    fz = Detector(m, shape, device, ANCHORS, MASK, keep_heads=True, **kw)
    fn = Detector(m, shape, device, ANCHORS, MASK, keep_heads=False, **kw)
    assert not ref.fused and fz.fused and fn.fused
    assert sum(i['kind'] == 'head' for i in fz.engine.op_info) == 3
    want = [t.clone() for t in ref(x)]
    for det in (fz, fn):
        for rep in range(2):   # replays reset the counts
            got = [t.clone() for t in det(x)]
            torch.cuda.synchronize()
            assert torch.equal(det.counts, ref.counts)
            for b in range(shape[0]):
                r1, c1 = _sorted_cands(ref, b)
                r2, c2 = _sorted_cands(det, b)
                assert torch.equal(r1, r2) and torch.equal(c1, c2)
            for w, g in zip(want, got):
                assert torch.equal(w, g)
    for h1, h2 in zip(ref.heads, fz.heads):
        assert torch.equal(h1, h2)
    assert int(ref.counts.sum()) > 0


@pytest.mark.parametrize('precision', ['f32', 'bf16'])
def test_detector_idetect_model(device, precision):
    """The fused Detector on an IDetect-headed network (yolov7-tiny with its head
    swapped for IDetect, nets/idetect.py:7-50; ImplicitA/M folded into the head
    convs): the head convs decode in their epilogue (bf16) or through
    ycx_decode_filter (f32), then NMS; vs the oracle chain (decode_box -> nms,
    detect.py:29-144) on the same GPU heads. IDetect's outputs are [P3, P4, P5]
    with anchor rows 0, 1, 2, hence the mask."""
    import copy
    from helpers import make_model_cfg
    cfg = copy.deepcopy(cvt_cfg('yolov7-tiny'))
    assert cfg['head'][-1][2] == 'Detect'
    cfg['head'][-1][2] = 'IDetect'
    m, sd = make_model_cfg(cfg, 1, 0, precision)
    m.to(device)
    imask = [[0, 1, 2], [3, 4, 5], [6, 7, 8]]
    shape = (2, 3, 320, 320)
    det = Detector(m, shape, device, ANCHORS, imask, conf_thres=0.3, nms_thres=0.45, max_det=1000)
    assert det.fused == (precision == 'bf16')
    x = synthetic_images(*shape, seed=19).to(device)
    dets, keep, kc = det(x)
    torch.cuda.synchronize()
    heads = [h.cpu() for h in det.heads]
    assert [h.shape[2] for h in heads] == [40, 20, 10]
    # the head maps are the network's own (oracle forward of the same weights, raw IDetect x_i)
    ref = ref_forward.build(cfg, ANCHORS, 1, sd)(x.cpu())
    ref = ref[1] if isinstance(ref, tuple) else ref
    for h, r in zip(heads, ref):
        r = r if r.dim() == 4 else r.permute(0, 1, 4, 2, 3).reshape(h.shape)
        assert rel_err(h, r) < (1e-3 if precision == 'f32' else 5e-2)
    cpu = [t.cpu() for t in (det.cand, det.cand_rows, det.counts, keep, kc)]
    for b in range(2):
        rep = fused_keep_report(*cpu, b, [h[b] for h in heads], 1, 0.3, 0.45, 320, 1000, mask=imask)
        print(f"\n{precision} image {b}: {rep}")
        assert rep['cls_same'] and rep['nms_exact'], rep
        assert rep['box_maxdiff'] <= 2e-6 and rep['member_max_dist'] <= 1e-6, rep
        assert rep['keep_flips'] <= FLIPS_PIN['tiny320'] and rep['unexplained_flips'] == 0, rep
        assert int(kc[b]) > 0


@pytest.mark.parametrize('precision', ['f32', 'bf16'])
def test_detector_fused_path(device, precision):
    """Fused decode+filter+sort+NMS from the model's own heads vs the oracle
    chain (decode_box -> nms) run on the same GPU heads."""
    m, sd = make_model('yolov7-tiny', 1, 0, precision)
    m.to(device)
    shape = (2, 3, 320, 320)
    det = Detector(m, shape, device, ANCHORS, MASK, conf_thres=0.3, nms_thres=0.45, max_det=1000)
    x = synthetic_images(*shape, seed=9).to(device)
    dets, keep, kc = det(x)
    torch.cuda.synchronize()
    heads = [h.cpu() for h in det.heads]
    cpu = [t.cpu() for t in (det.cand, det.cand_rows, det.counts, keep, kc)]
    for b in range(2):
        rep = fused_keep_report(*cpu, b, [h[b] for h in heads], 1, 0.3, 0.45, 320, 1000)
        print(f"\n{precision} image {b}: {rep}")
        assert rep['cls_same'] and rep['nms_exact'], rep
        assert rep['box_maxdiff'] <= 2e-6 and rep['member_max_dist'] <= 1e-6, rep
        assert rep['keep_flips'] <= FLIPS_PIN['tiny320'] and rep['unexplained_flips'] == 0, rep
        assert int(kc[b]) > 0


def test_detector_graph_matches_eager(device):
    m, _ = make_model('yolov7-tiny', 1, 0, 'bf16')
    m.to(device)
    shape = (2, 3, 256, 256)
    x = synthetic_images(*shape, seed=4).to(device)
    g = Detector(m, shape, device, ANCHORS, MASK, use_graph=True)
    d1, k1, c1 = [t.clone() for t in g(x)]   # HIP graph replay + post
    g.counts.zero_()                          # the fused heads append this forward's candidates
    g.engine.run_static()                     # eager ycx_run_ops on the same static buffers
    d2, k2, c2 = [t.clone() for t in g.post()]
    torch.cuda.synchronize()
    assert torch.equal(c1, c2) and torch.equal(k1, k2) and torch.equal(d1, d2)


def test_fused_append_bounded_without_reset(device):
    """A caller that replays the fused forward without resetting the candidate counts
    keeps appending past rows_total: the counts grow, the row list stays in bounds
    (the writes past it are dropped) and a reset restores the exact result."""
    m, _ = make_model('yolov7-tiny', 1, 0, 'bf16')
    m.to(device)
    shape = (2, 3, 256, 256)
    x = synthetic_images(*shape, seed=4).to(device)
    g = Detector(m, shape, device, ANCHORS, MASK, use_graph=False)
    assert g.fused
    d1, k1, c1 = [t.clone() for t in g(x)]
    n1 = g.counts.clone()
    guard = torch.full((1 << 16,), 7, dtype=torch.int32, device=device)  # allocated after the row list
    reps = g.rows // max(1, int(n1.min())) + 2  # enough replays to pass rows_total
    assert int(n1.min()) > 0 and reps <= 64, (n1, g.rows)
    for _ in range(reps):
        g.engine.run_static()
    torch.cuda.synchronize()
    assert bool((g.counts > g.rows).all()) and bool((guard == 7).all())
    d2, k2, c2 = [t.clone() for t in g(x)]  # forward() resets the counts
    torch.cuda.synchronize()
    assert torch.equal(g.counts, n1) and torch.equal(k1, k2) and torch.equal(c1, c2) and torch.equal(d1, d2)


def test_pipelined_detector_matches_serial(device):
    """Two slots on two streams, five batches in flight back to back: every
    batch's detections equal the single-stream Detector's on the same images."""
    m, _ = make_model('yolov7-tiny', 1, 0, 'bf16')
    m.to(device)
    shape = (2, 3, 256, 256)
    ref = Detector(m, shape, device, ANCHORS, MASK, use_graph=True)
    pd = PipelinedDetector(m, shape, device, ANCHORS, MASK, depth=2, use_graph=True)
    xs = [synthetic_images(*shape, seed=20 + i).to(device) for i in range(5)]
    want = [[t.clone() for t in ref(x)] for x in xs]
    got = []
    for x in xs:
        dets, keep, kc, done = pd.submit(x)
        torch.cuda.current_stream().wait_event(done)
        got.append([dets.clone(), keep.clone(), kc.clone()])
    pd.synchronize()
    torch.cuda.synchronize()
    for (d1, k1, c1), (d2, k2, c2) in zip(want, got):
        assert torch.equal(c1, c2) and torch.equal(k1, k2) and torch.equal(d1, d2)


def test_concurrent_detector_matches_serial(device):
    """Three slots on three streams, seven batches back to back (every slot
    reused): each batch's detections equal the single-stream Detector's."""
    m, _ = make_model('yolov7-tiny', 1, 0, 'bf16')
    m.to(device)
    shape = (2, 3, 256, 256)
    ref = Detector(m, shape, device, ANCHORS, MASK, use_graph=True)
    cd = ConcurrentDetector(m, shape, device, ANCHORS, MASK, depth=3, use_graph=True)
    xs = [synthetic_images(*shape, seed=40 + i).to(device) for i in range(7)]
    want = [[t.clone() for t in ref(x)] for x in xs]
    got = []
    for x in xs:
        dets, keep, kc, done = cd.submit(x)
        torch.cuda.current_stream().wait_event(done)
        got.append([dets.clone(), keep.clone(), kc.clone()])
    cd.synchronize()
    torch.cuda.synchronize()
    for (d1, k1, c1), (d2, k2, c2) in zip(want, got):
        assert torch.equal(c1, c2) and torch.equal(k1, k2) and torch.equal(d1, d2)


def _check_keep(pred, nc, conf, thr):
    ref_keep, _ = ref_post.nms_keep_rows(pred.clone(), nc, conf, thr)
    _, keep, kc = nms_device(pred.clone().to('cuda'), nc, conf, thr)
    keep, kc = keep.cpu().numpy(), kc.cpu().numpy()
    for b in range(pred.shape[0]):
        assert int(kc[b]) == len(ref_keep[b]), (b, int(kc[b]), len(ref_keep[b]))
        np.testing.assert_array_equal(keep[b, :int(kc[b])], ref_keep[b].numpy())


def _random_pred(n, rows, nc, seed, scale=1.0, size_lo=-4.0, size_hi=0.0):
    """Boxes with log-uniform sizes over 10^size_lo..10^size_hi (aspect up to
    ~10:1) at uniform centres, every row passing the threshold."""
    g = torch.Generator().manual_seed(seed)
    pred = torch.zeros(n, rows, 5 + nc)
    pred[..., 0:2] = torch.rand(n, rows, 2, generator=g) * scale
    logs = size_lo + (size_hi - size_lo) * torch.rand(n, rows, 2, generator=g)
    pred[..., 2:4] = (10.0 ** logs) * scale
    pred[..., 4] = 0.5 + 0.5 * torch.rand(n, rows, generator=g)
    pred[..., 5:] = torch.rand(n, rows, nc, generator=g)
    return pred


@pytest.mark.parametrize('rows', [6000, 24000])  # two classes each: LDS-resident fast path / nms_wide
@pytest.mark.parametrize('thr', [0.0, 0.3, 0.65, 1.0])
def test_nms_spatial_wide_sizes(device, thr, rows):
    """Large classes (spatial-grid path) with sizes spanning four octaves of
    ten, down to far below one grid cell: every level/window bound is used."""
    _check_keep(_random_pred(2, rows, 2, seed=11), 2, 0.0, thr)


def test_nms_many_big_classes_unsplit(device):
    """More big classes per batch than the split threshold (64): the fast classes then run
    whole on a workgroup each inside nms_fast (the C2 regime), beside one wide class whose
    search and fixed point run in nms_search / nms_resolve. Every other big-class test here
    has few classes and takes the split path."""
    pred = _random_pred(2, 40000, 40, seed=18, size_lo=-2.5, size_hi=-1.0)  # ~1000 rows per class
    pred[0, :9000, 5] = 2.0  # class 0 of image 0: ~9.5k rows, past the LDS-resident size
    _check_keep(pred, 40, 0.0, 0.45)


def test_nms_wide_class_past_u16_ranks(device):
    """One class of 60k boxes: past the u16 rank range the wide path stages in LDS (~52.5k),
    so its search and fixed point keep 16 int ranks per box and read the ranks from L2."""
    _check_keep(_random_pred(1, 60000, 1, seed=19, size_lo=-2.0, size_hi=-1.0), 1, 0.0, 0.45)


def test_nms_spatial_pixel_coords_and_clusters(device):
    # pixel units (class extent normalisation) and tight clusters of near-duplicates
    pred = _random_pred(1, 5000, 1, seed=12, scale=640.0, size_lo=-2.5, size_hi=-0.5)
    g = torch.Generator().manual_seed(13)
    centers = torch.rand(40, 2, generator=g) * 640
    idx = torch.randint(0, 40, (2500,), generator=g)
    pred[0, :2500, 0:2] = centers[idx] + torch.randn(2500, 2, generator=g) * 3.0
    pred[0, :2500, 2:4] = 40.0 + torch.randn(2500, 2, generator=g) * 4.0
    _check_keep(pred, 1, 0.0, 0.45)


@pytest.mark.parametrize('rows', [3000, 12000])  # fast path / nms_wide
def test_nms_spatial_degenerate_and_identical(device, rows):
    pred = _random_pred(1, rows, 1, seed=14, size_lo=-2.0, size_hi=-1.0)
    pred[0, 0:200, 2] = 0.0                      # zero width
    pred[0, 200:400, 3] = -0.01                  # negative height (x2 < x1 after conversion)
    pred[0, 400:420, 0] = float('nan')           # NaN centre
    pred[0, 420:440, 2] = float('inf')           # infinite width
    pred[0, 1000:1800, :4] = torch.tensor([0.5, 0.5, 0.1, 0.1])  # 800 identical boxes
    pred[0, 1000:1800, 4] = 0.9
    for thr in (0.5, -0.1):                      # negative threshold: every pair compared
        _check_keep(pred, 1, 0.0, thr)


def test_nms_spatial_long_chain(device):
    """A staircase where each box suppresses only its successor: greedy keeps
    every other box, and the fixed point needs one round per link."""
    rows = 1500
    pred = torch.zeros(1, rows, 6)
    i = torch.arange(rows, dtype=torch.float32)
    pred[0, :, 0] = 0.1 + i * 0.0004          # centre steps 0.4 of a box width
    pred[0, :, 1] = 0.5
    pred[0, :, 2] = 0.001
    pred[0, :, 3] = 0.001
    pred[0, :, 4] = 1.0 - i * 1e-4            # scores descend along the chain
    pred[0, :, 5] = 1.0
    _check_keep(pred, 1, 0.0, 0.3)


def test_nms_big_class_score_ties(device):
    """A large class (the LDS-resident fast path: radix rank sort) whose 4000 scores take
    only 8 values: nearly every rank decision is the row tie-break of the stable
    descending order (torchvision's sort), and the digits the keys share are skipped."""
    pred = _random_pred(2, 4000, 1, seed=15, size_lo=-2.0, size_hi=-1.0)
    g = torch.Generator().manual_seed(16)
    pred[..., 4] = 0.5 + 0.0625 * torch.randint(0, 8, (2, 4000), generator=g).float()
    pred[..., 5] = 1.0
    _check_keep(pred, 1, 0.0, 0.3)
    pred[..., 4] = 0.75  # one score for every box: the order is the row order alone
    _check_keep(pred, 1, 0.0, 0.3)
    wide = _random_pred(1, 20000, 1, seed=17, size_lo=-2.5, size_hi=-1.5)  # a wide class: bins of ~2500
    wide[..., 4] = 0.5 + 0.0625 * torch.randint(0, 8, (1, 20000), generator=g).float()  # ties: the radix sort
    wide[..., 5] = 1.0
    _check_keep(wide, 1, 0.0, 0.3)
    wide[..., 4] = 0.75  # one score: the keys differ in the row bits only, the bin rank orders by row
    _check_keep(wide, 1, 0.0, 0.3)


def test_nms_row_ordered_buckets_many_classes(device):
    """The class bucketing walks row slices in ascending order with a per-wave class match (ten
    ballots at nc = 600): every class bucket lists its rows in ascending order, so the score
    sorts (score digits only) keep equal scores in row order. Hundreds of small classes, one
    LDS-resident and one wide class with few distinct scores, a row count that splits unevenly
    over the slices."""
    pred = _random_pred(2, 30001, 600, seed=21, size_lo=-2.5, size_hi=-1.0)
    g = torch.Generator().manual_seed(22)
    pred[0, :7000, 5 + 17] = 2.0                                  # class 17 of image 0: ~7k rows
    pred[1, 5:20005, 5 + 599] = 2.0                               # class 599 of image 1: 20k rows
    pred[1, 5:20005, 4] = 0.5 + 0.0625 * torch.randint(0, 8, (20000,), generator=g).float()
    _check_keep(pred, 600, 0.0, 0.45)
