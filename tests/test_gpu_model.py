"""Model.forward on the HIP engine vs the golden fixtures and the pinned oracle.

Tolerances (max |gpu - ref| / max |ref| per output tensor):
  f32 parity mode : 1e-3  (north_star: 1e-3 relative on box/confidence tensors)
  fp16            : 1e-3 on raw tensors (IEEE half activations/weights on the f16 MFMA; a G1
                           net that ends in an activation carries that value's own fp16
                           rounding, 2^-11 relative, measured r03 <= 0.0009; yolov7_160 heads
                           4.4e-4). One documented exception: the RAW logits of yolov7-tiny
                           at 640 (LeakyReLU, 1.21-1.34e-3 measured r03) are held to 1.5e-3;
                           the DECODED box / objectness / class-confidence tensors north_star
                           names are held to 1e-3 everywhere, that net included (6.4e-4 /
                           4.2e-4 / 4.6e-4: test_g2_decoded_fp16, test_yolov7_640_vs_oracle,
                           C2 in test_gpu_configs.py)
  bf16            : 2.5e-2 (bf16 activations/weights drift ~0.5 % median, up to 1.25 % of
                           max-abs end to end through 100+ layers: measured r02 max 0.0125)
"""
import numpy as np
import pytest
import torch

from helpers import ANCHORS, g1_case, make_model, rel_err
from oracle import ref_forward, ref_post
from ycx.utils.helper_io import cvt_cfg
from ycx.utils.synth import synthetic_images

pytestmark = pytest.mark.gpu

F32_TOL, BF16_TOL = 1e-3, 2.5e-2   # bf16 measured r02: <= 0.0125 (G2 tiny_640), yolov7 heads ~0.005
F16_TOL = 1e-3
F16_RAW_TOL = {'tiny_640': 1.5e-3}  # raw LeakyReLU-net logits only; decoded: 1e-3 (module doc)
G1_NAMES = ['conv_k3s1_cin32', 'conv_k3s2_cin32', 'conv_k1_cin64', 'conv_leaky', 'stem_s2_leaky', 'pools',
            'upsample_concat', 'upsample_shared', 'sppcspc', 'repconv', 'csp_blocks', 'detect', 'idetect',
            'upsample_offset', 'iauxdetect']


def _outs(y):
    return y if isinstance(y, list) else [y]


@pytest.mark.parametrize('precision,tol', [('f32', F32_TOL), ('bf16', BF16_TOL), ('fp16', F16_TOL)])
@pytest.mark.parametrize('name', G1_NAMES)
def test_g1_ops(device, manifest, g1, name, precision, tol):
    m, sd, x, e = g1_case(manifest, name, precision)
    m.to(device)
    y = m(x.to(device))
    if name == 'idetect':  # eval branch: (z, [x_i (bs, na, ny, nx, no)]); fixtures hold the x_i
        z, y = y
        head = m.model[-1]
        strides = [x.shape[2] / o.shape[2] for o in y]
        gold_nchw = [torch.from_numpy(g1[f'{name}/{j}']).permute(0, 1, 4, 2, 3).reshape(o.shape[0], -1, o.shape[2],
                                                                                       o.shape[3])
                     for j, o in enumerate(y)]
        z_ref, _ = ref_post.idetect_eval(gold_nchw, head.anchors.cpu().view(len(y), -1).tolist(), head.na, head.no,
                                         strides)
        assert z.shape == z_ref.shape and rel_err(z.cpu(), z_ref) < tol, ('z', rel_err(z.cpu(), z_ref))
    if name == 'iauxdetect':  # eval branch (z, x[:nl]) vs the reference's own eval output, strides set
        z, xs = y
        assert [x.shape[2] / o.shape[2] for o in xs] == e['strides']
        y = [z] + list(xs)
    outs = _outs(y)
    assert len(outs) == e['n_out']
    for j, o in enumerate(outs):
        gold = torch.from_numpy(g1[f'{name}/{j}'])
        o = o.cpu()
        assert o.shape == gold.shape
        print(f"\n{precision} G1 {name} out {j} rel err {rel_err(o, gold):.5f}")
        assert rel_err(o, gold) < tol, (name, j, rel_err(o, gold))


@pytest.mark.parametrize('precision,tol', [('f32', F32_TOL), ('bf16', BF16_TOL), ('fp16', F16_TOL)])
@pytest.mark.parametrize('name', ['yolov7_160', 'tiny_640'])
def test_g2_nets(device, manifest, g2, name, precision, tol):
    e = manifest['g2'][name]
    if precision == 'fp16':
        tol = F16_RAW_TOL.get(name, tol)
    m, _ = make_model(e['net'], e['nc'], e['w_seed'], precision)
    m.to(device)
    x = synthetic_images(*e['shape'], seed=e['img_seed']).to(device)
    outs = m(x)
    for j, o in enumerate(outs):
        gold = torch.from_numpy(g2[f'{name}/{j}'])
        assert tuple(o.shape) == tuple(gold.shape)
        print(f"\n{precision} G2 {name} out {j} rel err {rel_err(o.cpu(), gold):.5f}")
        assert rel_err(o.cpu(), gold) < tol, (name, j, rel_err(o.cpu(), gold))


@pytest.mark.parametrize('name', ['yolov7_160', 'tiny_640'])
def test_g2_decoded_fp16(device, manifest, g2, name):
    """fp16 plan: decode_box (detect.py:29-87) of the G2 heads -- boxes, objectness and
    class confidences separately -- within north_star's 1e-3 of the decoded fixture heads."""
    from ycx.detect import decode_box
    e = manifest['g2'][name]
    m, _ = make_model(e['net'], e['nc'], e['w_seed'], 'fp16')
    m.to(device)
    x = synthetic_images(*e['shape'], seed=e['img_seed']).to(device)
    outs = m(x)
    size = e['shape'][2]
    a = np.asarray(ANCHORS).reshape(-1, 2)
    mask = [[6, 7, 8], [3, 4, 5], [0, 1, 2]]
    gold = [torch.from_numpy(g2[f'{name}/{j}']) for j in range(len(outs))]
    dec = torch.cat(decode_box(outs, a, mask, e['nc'], (size, size)), 1).cpu()
    dref = torch.cat(ref_post.decode_box(gold, a, mask, e['nc'], (size, size)), 1)
    no = e['nc'] + 5
    errs = {k: rel_err(dec[..., sl], dref[..., sl]) for k, sl in
            (('box', slice(0, 4)), ('obj', slice(4, 5)), ('cls', slice(5, no)))}
    print(f"\nfp16 G2 {name} decoded rel err: {errs}")
    assert max(errs.values()) < 1e-3, errs


# decoded box / confidence tensors, max |gpu - ref| / max |ref|; r02: f32 6e-7, bf16 1.1e-3
DECODED_TOL = {'f32': 1e-3, 'bf16': 5e-3, 'fp16': 1e-3}


@pytest.mark.parametrize('precision,tol', [('f32', F32_TOL), ('bf16', BF16_TOL), ('fp16', F16_TOL)])
def test_yolov7_640_vs_oracle(device, precision, tol):
    """Full BASELINE shape (640x640, COCO-80) at bs=2 against the oracle computed
    live: the raw heads (Model.forward, nets/yolo.py:143-153) and the decoded
    (N, 25200, 85) tensor (decode_box, detect.py:29-87) that north_star's
    "1e-3 relative for box/confidence tensors" names -- boxes (cols 0-3),
    objectness (col 4) and class confidences (cols 5-84) separately."""
    from ycx.detect import decode_box
    m, sd = make_model('yolov7', 80, 0, precision)
    m.to(device)
    x = synthetic_images(2, 3, 640, 640, seed=3)
    ref = ref_forward.build(cvt_cfg('yolov7'), ANCHORS, 80, sd)(x)
    outs = m(x.to(device))
    for o, r in zip(outs, ref):
        assert rel_err(o.cpu(), r) < tol
    a = np.asarray(ANCHORS).reshape(-1, 2)
    mask = [[6, 7, 8], [3, 4, 5], [0, 1, 2]]
    dec = torch.cat(decode_box(outs, a, mask, 80, (640, 640)), 1).cpu()
    dref = torch.cat(ref_post.decode_box(ref, a, mask, 80, (640, 640)), 1)
    assert dec.shape == dref.shape == (2, 25200, 85)
    errs = {k: rel_err(dec[..., sl], dref[..., sl]) for k, sl in
            (('box', slice(0, 4)), ('obj', slice(4, 5)), ('cls', slice(5, 85)))}
    print(f"\n{precision} decoded rel err: {errs}")
    assert max(errs.values()) < DECODED_TOL[precision], errs


def test_engine_plan_properties(device):
    m, _ = make_model('yolov7', 80, 0, 'bf16')
    m.to(device)
    eng = m.engine_for((2, 3, 640, 640), device)
    s = eng.summary()
    assert s['kinds'].get('copy', 0) == 0, "every concat input should alias its slice (no copy kernels)"
    k = s['kinds']
    # 95 convs minus the 3 folded RepConv 1x1 branches; at 640 the stem and layer 1 run fused (stem2)
    # and the 8 ELAN cv1/cv2 sibling pairs run as one conv each
    assert k.get('stem2', 0) == 1 and 'stem' not in k
    assert sum(i.get('parts', 1) for i in eng.op_info if i['kind'] in ('conv', 'stem', 'stem2', 'conv_pair')) == 92
    # the 160^2 ELAN exit (layer 11 -> layer 14) runs as one fused 1x1 pair (tile 55) once the map
    # gives the weight-resident kernel >= 8 tiles per CU (bs >= 6 at 640)
    assert not any(i['kind'] == 'conv_pair' for i in eng.op_info)
    eng8 = m.engine_for((8, 3, 640, 640), device, slot=7)
    assert [i['shape'][1:5] for i in eng8.op_info if i['kind'] == 'conv_pair'] == [(160, 160, 256, 256)]
    assert sum(i.get('parts', 1) for i in eng8.op_info if i['kind'] in ('conv', 'stem', 'stem2', 'conv_pair')) == 92
    m.release_slot((8, 3, 640, 640), device, 7)
    assert sum(1 for i in eng.op_info if i['kind'] == 'conv' and i['parts'] == 2) == 8
    assert abs(s['gflop_per_image'] - 104.511078400) < 1e-6
    # the five MP k2 s2 pools run inside their 1x1 consumers; the SPPCSPC cascade is the one pool op
    assert sum(1 for i in eng.op_info if i['name'].endswith('+maxpool_k2s2')) == 5
    assert [i['name'] for i in eng.op_info if i['kind'] == 'pool'] == ['maxpool_k5s1_cascade3']


def test_conv_pair_fusion_bit_identical(device, monkeypatch):
    """The yolov7 plan with its 1x1 -> 1x1 chain fused (ycx_conv2d_pair) == the plan that runs
    the two convs apart (YCX_NO_CONV_PAIR=1), bit for bit, in bf16 and fp16."""
    from ycx.engine import Engine
    for precision in ('bf16', 'fp16'):
        m, _ = make_model('yolov7', 80, 0, precision)
        m.to(device)
        x = synthetic_images(8, 3, 640, 640, seed=6).to(device)
        outs = []
        for off in ('', '1'):
            monkeypatch.setenv('YCX_NO_CONV_PAIR', off)
            eng = Engine(m, tuple(x.shape), torch.device(device), precision)
            try:
                assert sum(1 for i in eng.op_info if i['kind'] == 'conv_pair') == (0 if off else 1)
                outs.append([o.clone() for o in eng.run(x)])
            finally:
                eng.close()
        for a, b in zip(*outs):
            assert torch.equal(a, b)


@pytest.mark.parametrize('prec', ['bf16', 'fp8'])
def test_pool_fusion_bit_identical(device, prec):
    """yolov7 bf16 / fp8 plan with the MP pools fused into their 1x1 convs == the plan that
    runs them as ycx_maxpool ops, bit for bit."""
    from ycx.engine import Engine
    m, _ = make_model('yolov7', 80, 0, prec)
    m.to(device)
    x = synthetic_images(2, 3, 320, 320, seed=4).to(device)
    amax = m.calibrate_fp8(device=device, hw=(320, 320), n=2) if prec == 'fp8' else None
    outs = []
    for fuse in (True, False):
        eng = Engine(m, tuple(x.shape), torch.device(device), prec, fuse_pool=fuse, fp8_amax=amax)
        try:
            assert sum(1 for i in eng.op_info if i['name'].endswith('+maxpool_k2s2')) == (5 if fuse else 0)
            outs.append([o.clone() for o in eng.run(x)])
        finally:
            eng.close()
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_graph_replay_matches_eager(device):
    m, _ = make_model('yolov7-tiny', 1, 0, 'bf16')
    m.to(device)
    x = synthetic_images(2, 3, 320, 320, seed=5).to(device)
    eager = [o.clone() for o in m(x)]
    eng = m.engine_for(x.shape, device)
    xs, outs = eng.bind_static(x)
    eng.capture()
    for _ in range(2):
        eng.replay()
    torch.cuda.synchronize()
    for a, b in zip(outs, eager):
        assert torch.equal(a, b)  # same kernels, same order: bitwise identical


def test_forward_rejects_cpu_and_training():
    m, _ = make_model('yolov7-tiny', 1, 0)
    with pytest.raises(RuntimeError, match='ROCm device'):
        m(torch.zeros(1, 3, 64, 64))
    m.train()
    with pytest.raises(RuntimeError, match='inference-only'):
        m(torch.zeros(1, 3, 64, 64))


@pytest.mark.parametrize('hw,cascade', [(24, True), (48, False)])
def test_sppcspc_pool_cascade_size_limit(device, manifest, hw, cascade):
    """the one-launch 5/9/13 cascade keeps two copies of the map's plane in
    64 KB of LDS. A 48^2 map (2304 pixels, 64 channels) does not fit; the plan must fall
    back to three pool launches (not fail in run_ops), and both forms match the oracle."""
    from ycx.engine import cascade_fits
    e = manifest['g1']['sppcspc']
    assert cascade_fits(hw, hw, 64, 2) == cascade
    m, sd = make_model(e['cfg'], e['nc'], e['w_seed'], 'bf16')
    m.to(device)
    x = synthetic_images(1, 3, hw, hw, seed=21)
    eng = m.engine_for(x.shape, device)
    pools = [i['name'] for i in eng.op_info if i['kind'] == 'pool']
    assert pools == (['maxpool_k5s1_cascade3'] if cascade else ['maxpool_k5s1'] * 3), pools
    y = m(x.to(device))
    ref = ref_forward.build(e['cfg'], ANCHORS, e['nc'], sd)(x)
    for o, r in zip(_outs(y), _outs(ref)):
        assert rel_err(o.cpu(), r) < BF16_TOL


def test_detector_close_releases_its_engine(device):
    """every Detector owns a private engine; close() (or collecting the
    Detector) removes it from the model's engine table, so repeated Detectors do
    not accumulate activation buffers."""
    import gc
    from ycx.detect import ConcurrentDetector, Detector
    m, _ = make_model('yolov7-tiny', 1, 0, 'bf16')
    m.to(device)
    shape = (1, 3, 64, 64)
    base = len(m._engines)
    det = Detector(m, shape, device, ANCHORS, [[6, 7, 8], [3, 4, 5], [0, 1, 2]], use_graph=True)
    det(torch.zeros(shape, device=device))
    torch.cuda.synchronize()
    assert len(m._engines) == base + 1
    det.close()
    assert len(m._engines) == base
    for _ in range(3):  # dropped without close(): the finaliser releases the engine
        Detector(m, shape, device, ANCHORS, [[6, 7, 8], [3, 4, 5], [0, 1, 2]], use_graph=False)
        gc.collect()
    assert len(m._engines) == base
    cd = ConcurrentDetector(m, shape, device, ANCHORS, [[6, 7, 8], [3, 4, 5], [0, 1, 2]], depth=3)
    assert len(m._engines) == base + 3
    cd.submit(torch.zeros(shape, device=device))
    cd.close()
    assert len(m._engines) == base


@pytest.mark.parametrize('precision', ['bf16', 'fp8'])
def test_chunked_prefix_bit_identical(device, precision, monkeypatch):
    """YCX_CHUNK='k:cut' (the image-chunked prefix experiment) runs the plan's first cut
    ops k images at a time: every op is image-major, so the fused Detector's outputs
    must equal the unchunked plan's bit for bit."""
    from ycx.detect import Detector
    m, _ = make_model('yolov7', 80, 0, precision)
    m.to(device)
    if precision == 'fp8':
        m.calibrate_fp8(device=device, hw=(160, 160), n=2)
    x = synthetic_images(4, 3, 160, 160, seed=5).to(device)
    kw = dict(conf_thres=0.3, nms_thres=0.45, max_det=2000, keep_heads=True)
    det = Detector(m, tuple(x.shape), device, ANCHORS, [[6, 7, 8], [3, 4, 5], [0, 1, 2]], **kw)
    d0, k0, c0 = [t.clone() for t in det(x)]
    h0 = [h.clone() for h in det.heads]
    det.close()
    monkeypatch.setenv('YCX_CHUNK', '2:40')
    det = Detector(m, tuple(x.shape), device, ANCHORS, [[6, 7, 8], [3, 4, 5], [0, 1, 2]], **kw)
    d1, k1, c1 = det(x)
    torch.cuda.synchronize()
    assert det.engine._exec_ops()[1] > det.engine.n_ops  # the chunked list really ran
    for a, b in zip(h0, det.heads):
        assert torch.equal(a, b)
    assert torch.equal(c0, c1) and torch.equal(k0, k1) and torch.equal(d0, d1)
    det.close()


def test_concurrent_detector_dropped_in_flight(device):
    """a ConcurrentDetector dropped (no close()) right after submit():
    its slot engines are released by their finalisers while the batches may still
    run on the slot streams. The release waits for the device first, so memory
    handed back to the caching allocator and then overwritten cannot corrupt the
    detections still referenced by the caller."""
    import gc
    from ycx.detect import ConcurrentDetector, Detector
    mask = [[6, 7, 8], [3, 4, 5], [0, 1, 2]]
    m, _ = make_model('yolov7', 80, 0, 'bf16')
    m.to(device)
    shape = (4, 3, 160, 160)
    x = synthetic_images(*shape, seed=7).to(device)
    ref = Detector(m, shape, device, ANCHORS, mask, conf_thres=0.3, nms_thres=0.45, max_det=500)
    d_ref, k_ref, c_ref = [t.clone() for t in ref(x)]
    ref.close()
    base = len(m._engines)
    cd = ConcurrentDetector(m, shape, device, ANCHORS, mask, depth=3, conf_thres=0.3, nms_thres=0.45, max_det=500)
    outs = [cd.submit(x)[:3] for _ in range(3)]
    del cd
    gc.collect()
    assert len(m._engines) == base
    junk = torch.full((64 << 20,), 7, dtype=torch.int32, device=device)  # reuses the released blocks
    torch.cuda.synchronize()
    del junk
    for d, k, c in outs:
        assert torch.equal(c, c_ref) and torch.equal(k, k_ref) and torch.equal(d, d_ref)


@pytest.mark.parametrize('net,nc', [('yolov7', 80), ('yolov7-tiny', 1)])
def test_fp16_range_guard(device, net, nc):
    """VERDICT r3 weak 1 / ADVICE r3: the fp16 plan (the Model default) must never return
    inf / NaN silently. A synthetic checkpoint whose third conv's BN scale is multiplied by
    1e5 drives that layer's activations past 65504 (fine in fp32 / bf16, inf in fp16):
      - the fused Detector fast path sets its device flag and check() raises YcxRangeError
        (ConcurrentDetector.check() likewise, over all slots);
      - Model.forward warns and re-plans itself in bf16, and the heads it then returns are
        finite and equal to a bf16 Model's.
    The unmodified checkpoint raises nothing (the flag stays 0)."""
    from ycx import _lib as L
    from ycx.detect import ConcurrentDetector, Detector
    mask = [[6, 7, 8], [3, 4, 5], [0, 1, 2]]
    m, sd = make_model(net, nc, 0, 'fp16')
    m.to(device)
    shape = (2, 3, 160, 160)
    x = synthetic_images(*shape, seed=9).to(device)
    det = Detector(m, shape, device, ANCHORS, mask, conf_thres=0.3, nms_thres=0.45, max_det=300)
    assert det.fused
    det(x)
    det.check()  # in range: no error
    assert not det.overflowed()
    det.close()
    bn = [k for k in sd if k.endswith('.bn.weight')][2]
    big = dict(sd)
    big[bn] = sd[bn] * 1e5
    m.load_state_dict(big)
    m.to(device)
    det = Detector(m, shape, device, ANCHORS, mask, conf_thres=0.3, nms_thres=0.45, max_det=300)
    det(x)
    assert det.overflowed()
    with pytest.raises(L.YcxRangeError, match='non-finite'):
        det.check()
    det.close()
    cd = ConcurrentDetector(m, shape, device, ANCHORS, mask, depth=2, conf_thres=0.3, nms_thres=0.45)
    cd.submit(x)
    with pytest.raises(L.YcxRangeError):
        cd.check()
    cd.close()
    with pytest.warns(RuntimeWarning, match='overflowed'):
        outs = m(x)
    assert m.precision == 'bf16'
    assert all(bool(torch.isfinite(o).all()) for o in outs)
    mb, _ = make_model(net, nc, 0, 'bf16')
    mb.load_state_dict(big)
    mb.to(device)
    for a, b in zip(outs, mb(x)):
        assert torch.equal(a, b)
