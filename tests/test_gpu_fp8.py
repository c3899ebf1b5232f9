"""fp8 (OCP e4m3fn) path: BASELINE.json config C5 (640x640, fp8 MFMA conv).

Oracle levels:
  * the e4m3 cast itself (ycx_quantize_fp8) vs torch's float8_e4m3fn cast of the
    same clamped fp32 values: bit-exact;
  * one conv (tiles 34/35) vs a float64 CPU conv of the SAME dequantised e4m3
    operands, then torch's e4m3 cast of the result: the fp32 accumulation order
    differs, so a value within ~1e-6 relative of a rounding midpoint may land on
    the neighbouring code. Bar: >= 99.5 % of bytes identical, every other byte
    one code away; fp32 head outputs within 1e-4 of max |ref|;
  * the whole network vs the fp32 oracle (the reference's own forward restated):
    e4m3 keeps 3 mantissa bits per activation and weight, so per-head error is
    bounded at FP8_TOL of max |ref| (measured on MI355X, r02: 0.054-0.095 over the G1 nets,
    0.062-0.086 on yolov7 640 bs 2).
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import ANCHORS, MASK, make_model, rel_err
from oracle import ref_forward, ref_post
from ycx.detect import Detector
from ycx.utils.helper_io import cvt_cfg
from ycx.utils.synth import synthetic_images

pytestmark = pytest.mark.gpu
L = pytest.importorskip("ycx._lib")
E4M3 = torch.float8_e4m3fn
FP8_TOL = 0.12   # 1.26x the largest measured error (G1 csp_blocks 0.095)


def _q(x, s=1.0):
    """torch's e4m3 cast of clamp(x * s) (the encoding the kernels must produce)."""
    return (x.float() * s).clamp(-448.0, 448.0).to(E4M3)


def _codes_close(got_u8, ref_u8, min_exact=0.995):
    g = got_u8.to(torch.int32)
    r = ref_u8.to(torch.int32)
    same = g == r
    frac = float(same.float().mean())
    # e4m3 is sign-magnitude: neighbouring values are +-1 in the low 7 bits, same sign,
    # or +0 / -0 / smallest subnormals across zero
    mag_g, mag_r = g & 0x7F, r & 0x7F
    near = same | (((g ^ r) & 0x80) == 0) & ((mag_g - mag_r).abs() <= 1) | ((mag_g <= 1) & (mag_r <= 1))
    return frac, bool(near.all())


def test_quantize_matches_torch_cast(device):
    g = torch.Generator().manual_seed(0)
    x = torch.cat([torch.randn(100000, generator=g) * 50, torch.randn(1000, generator=g) * 1e-3,
                   torch.tensor([0.0, -0.0, 448.0, -448.0, 500.0, -1e9, 1e9, 0.0625, 0.5625, 0.59375, 2 ** -9,
                                 3 * 2 ** -10, 240.0, 232.0, 248.0])])
    for s in (1.0, 8.0, 0.25):
        xd = x.to(device)
        y = torch.empty(x.numel(), dtype=torch.uint8, device=device)
        L.check(L.lib.ycx_quantize_fp8(xd.data_ptr(), y.data_ptr(), x.numel(), ctypes.c_float(s),
                                       L.stream_handle(device)))
        torch.cuda.synchronize()
        ref = _q(x, s).view(torch.uint8)
        assert torch.equal(y.cpu(), ref), int((y.cpu() != ref).sum())


def _pow2_scale(amax, target=224.0):
    return 2.0 ** np.floor(np.log2(target / amax))


def _run_fp8_conv(device, n, h, w, cin, cout, k, s, act, tile=0, in_extra=0, out_extra=0, residual=False,
                  layout=L.OUT_NHWC, seed=0):
    from ycx.engine import pack_fp8_weights
    g = torch.Generator().manual_seed(seed)
    p = k // 2
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    sx = 16.0
    xq = _q(torch.randn(n, h, w, cin + in_extra, generator=g), sx)  # NHWC e4m3 of x * sx
    wt = torch.randn(cout, cin, k, k, generator=g, dtype=torch.float64) / (cin * k * k) ** 0.5
    b = torch.randn(cout, generator=g, dtype=torch.float64) * 0.1
    cpad = -(-cout // 64) * 64
    wp = torch.zeros(cpad, cin, k, k, dtype=torch.float64)
    wp[:cout] = wt
    wq, sw = pack_fp8_weights(wp)
    bp = torch.zeros(cpad, dtype=torch.float64)
    bp[:cout] = b
    bias = torch.cat([bp, 1.0 / (sw * sx)]).float()
    up = 2 if layout == L.OUT_NHWC_UP2 else 1
    so, sr = 32.0, 8.0
    rq = _q(torch.randn(n, ho, wo, cout, generator=g), sr) if residual else None
    if layout == L.OUT_NCHW_F32:
        y = torch.zeros(n, cout, ho, wo, dtype=torch.float32)
    else:
        y = torch.zeros(n, ho * up, wo * up, cout + out_extra, dtype=torch.uint8)
    d = L.ConvDesc()
    d.n, d.h, d.w, d.cin, d.in_c_off, d.in_c_stride = n, h, w, cin, in_extra, cin + in_extra
    d.ho, d.wo, d.cout, d.cout_pad = ho, wo, cout, cpad
    d.out_c_off, d.out_c_stride = (0, cout) if layout == L.OUT_NCHW_F32 else (out_extra, cout + out_extra)
    d.kh = d.kw = k
    d.stride, d.pad, d.act, d.leaky_slope = s, p, act, 0.1
    d.dtype, d.out_layout = L.DT_FP8, layout
    d.res_c_off, d.res_c_stride = 0, cout
    d.tile = tile
    d.out_scale, d.res_scale = (1.0 if layout == L.OUT_NCHW_F32 else so), 1.0 / sr
    xd, wd, bd, yd = xq.view(torch.uint8).to(device), wq.view(torch.uint8).to(device), bias.to(device), y.to(device)
    rd = rq.view(torch.uint8).to(device) if residual else None
    L.check(L.lib.ycx_conv2d(ctypes.byref(d), xd.data_ptr(), wd.data_ptr(), bd.data_ptr(), yd.data_ptr(),
                             rd.data_ptr() if rd is not None else None, L.stream_handle(device)), "fp8 conv")
    torch.cuda.synchronize()
    # oracle: float64 conv of the dequantised operands
    x64 = xq[..., in_extra:].to(torch.float64).permute(0, 3, 1, 2) / sx
    kt = k * k * cin
    w64 = (wq[:cout, :kt].to(torch.float64) / sw[:cout].reshape(-1, 1)).reshape(cout, k, k, cin).permute(0, 3, 1, 2)
    ref = F.conv2d(x64, w64, b, s, p)
    if act == L.ACT_SILU:
        ref = F.silu(ref)
    elif act == L.ACT_LEAKY:
        ref = F.leaky_relu(ref, 0.1)
    if residual:
        ref = ref + rq.to(torch.float64).permute(0, 3, 1, 2) / sr
    got = yd.cpu()
    if layout == L.OUT_NCHW_F32:
        return got.double(), ref, None
    ref_q = _q(ref.permute(0, 2, 3, 1), so).view(torch.uint8)
    if layout == L.OUT_NHWC_UP2:
        ref_q = ref_q.repeat_interleave(2, 1).repeat_interleave(2, 2)
    assert torch.all(got[..., :out_extra] == 0), "wrote outside the output channel slice"
    return got[..., out_extra:], ref_q, True


CASES = [  # n, h, w, cin, cout, k, s, act, extras
    (2, 20, 20, 128, 128, 3, 1, L.ACT_SILU, {}),
    (2, 20, 20, 256, 256, 1, 1, L.ACT_SILU, {}),
    (2, 40, 24, 64, 128, 3, 1, L.ACT_SILU, {}),      # 2 taps per K step, ragged pixel tail
    (2, 40, 40, 32, 64, 3, 2, L.ACT_SILU, {}),       # 4 taps per K step, stride 2
    (1, 33, 17, 64, 64, 1, 1, L.ACT_LEAKY, {}),
    (2, 16, 16, 128, 192, 3, 2, L.ACT_NONE, {}),
    (2, 16, 16, 128, 128, 3, 1, L.ACT_SILU, dict(in_extra=64, out_extra=64)),
    (2, 16, 16, 128, 128, 1, 1, L.ACT_SILU, dict(residual=True)),
    (2, 10, 10, 256, 128, 1, 1, L.ACT_SILU, dict(layout=L.OUT_NHWC_UP2)),
    (2, 20, 20, 256, 255, 1, 1, L.ACT_NONE, dict(layout=L.OUT_NCHW_F32)),
    (2, 12, 12, 96, 64, 3, 1, L.ACT_SILU, {}),       # generic K walk: chunks cross taps at any cin % 16
    (2, 12, 12, 48, 128, 3, 2, L.ACT_SILU, {}),
    (2, 12, 12, 160, 128, 1, 1, L.ACT_SILU, {}),
    (2, 24, 20, 512, 256, 1, 1, L.ACT_SILU, {}),     # weight-resident 1x1 (tile 36) cases
    (1, 33, 17, 128, 64, 1, 1, L.ACT_LEAKY, {}),
    (2, 16, 16, 256, 128, 1, 1, L.ACT_SILU, dict(in_extra=128, out_extra=64)),
    (3, 20, 20, 256, 200, 1, 1, L.ACT_SILU, {}),     # cout < cout_pad
    (2, 96, 96, 256, 256, 1, 1, L.ACT_SILU, {}),     # several tiles per block: deferred epilogues
    (3, 70, 70, 512, 128, 1, 1, L.ACT_SILU, {}),
    (2, 90, 90, 128, 64, 1, 1, L.ACT_NONE, {}),
    (2, 32, 32, 64, 64, 3, 1, L.ACT_SILU, {}),       # weight-stationary 3x3 64 -> 64 (tile 37) cases
    (1, 16, 48, 64, 48, 3, 1, L.ACT_LEAKY, {}),
    (2, 32, 16, 64, 64, 3, 1, L.ACT_NONE, dict(in_extra=64, out_extra=64)),
]


@pytest.mark.parametrize('tile', [34, 35, 36, 37])
@pytest.mark.parametrize('case', range(len(CASES)))
def test_fp8_conv_vs_dequantised_oracle(device, tile, case):
    n, h, w, cin, cout, k, s, act, kw = CASES[case]
    if tile == 34 and -(-cout // 64) * 64 % 128:
        pytest.skip("tile 34 needs cout_pad % 128 == 0")
    cpad = -(-cout // 64) * 64
    if tile == 36 and not (k == 1 and s == 1 and cin in (128, 256, 512) and not kw.get('residual') and
                           kw.get('layout', L.OUT_NHWC) == L.OUT_NHWC and (cpad in (64, 128) or cpad % 256 == 0)):
        pytest.skip("tile 36: 1x1/s1, cin 128/256/512, NHWC without residual")
    if tile == 37 and not (k == 3 and s == 1 and cin == 64 and cpad == 64 and h % 16 == 0 and w % 16 == 0 and
                           not kw.get('residual') and kw.get('layout', L.OUT_NHWC) == L.OUT_NHWC):
        pytest.skip("tile 37: 3x3/s1 64 -> 64 on 16-aligned maps, NHWC without residual")
    got, ref, q = _run_fp8_conv(device, n, h, w, cin, cout, k, s, act, tile=tile, seed=case, **kw)
    if q is None:  # fp32 heads: the fp8 MFMA's fp32 accumulation (measured ~2e-5 of max at K = 256)
        assert rel_err(got, ref) < 1e-4
        return
    frac, near = _codes_close(got, ref)
    assert near and frac >= 0.995, (frac, near)


@pytest.mark.parametrize('tile', [34, 35])
@pytest.mark.parametrize('n,hw,cin,cout,ex', [(2, (20, 20), 256, 128, 0), (3, (9, 13), 128, 128, 128),
                                              (2, (10, 10), 512, 256, 0), (1, (7, 5), 128, 64, 0)])
def test_fp8_conv_pool_fused(device, tile, n, hw, cin, cout, ex):
    """MP fused into the fp8 1x1 conv (ycx_conv_desc.in_pool: the k2 s2 max-pool of the (2h, 2w)
    e4m3 map formed in the operand staging, tiles 34 / 35) vs ycx_maxpool (fp8) then the same
    tile on the pooled map: bit for bit. Ragged pixel tails, channel-sliced input, negative
    and zero activations in the windows."""
    from ycx.engine import pack_fp8_weights
    cpad = -(-cout // 64) * 64
    if tile == 34 and cpad % 128:
        pytest.skip("tile 34 is 128 output channels wide")
    g = torch.Generator().manual_seed(17)
    h, w = hw
    x = torch.randn(n, 2 * h, 2 * w, cin + ex, generator=g)
    x[x.abs() < 0.05] = 0.0
    xq = _q(x, 16.0)
    wt = torch.randn(cpad, cin, 1, 1, generator=g, dtype=torch.float64) / cin ** 0.5
    wt[cout:] = 0
    wq, sw = pack_fp8_weights(wt)
    bias = torch.cat([torch.randn(cpad, generator=g, dtype=torch.float64) * 0.1, 1.0 / (sw * 16.0)]).float()
    xd, wd, bd = xq.view(torch.uint8).to(device), wq.view(torch.uint8).to(device), bias.to(device)
    pooled = torch.zeros(n, h, w, cin, dtype=torch.uint8, device=device)
    pd = L.PoolDesc()
    pd.n, pd.h, pd.w, pd.c, pd.in_c_off, pd.in_c_stride = n, 2 * h, 2 * w, cin, ex, cin + ex
    pd.ho, pd.wo, pd.out_c_off, pd.out_c_stride, pd.k, pd.stride, pd.pad, pd.dtype = h, w, 0, cin, 2, 2, 0, L.DT_FP8
    pd.levels = 1
    L.check(L.lib.ycx_maxpool(ctypes.byref(pd), xd.data_ptr(), pooled.data_ptr(), L.stream_handle(device)))

    def conv(src, in_off, in_stride, in_pool):
        y = torch.zeros(n, h, w, cout + 8, dtype=torch.uint8, device=device)
        d = L.ConvDesc()
        d.n, d.h, d.w, d.cin, d.in_c_off, d.in_c_stride = n, h, w, cin, in_off, in_stride
        d.ho, d.wo, d.cout, d.cout_pad, d.out_c_off, d.out_c_stride = h, w, cout, cpad, 8, cout + 8
        d.kh = d.kw = d.stride = 1
        d.pad, d.act, d.dtype, d.out_layout, d.tile, d.in_pool = 0, L.ACT_SILU, L.DT_FP8, L.OUT_NHWC, tile, in_pool
        d.out_scale = 32.0
        L.check(L.lib.ycx_conv2d(ctypes.byref(d), src.data_ptr(), wd.data_ptr(), bd.data_ptr(), y.data_ptr(), None,
                                 L.stream_handle(device)), "fp8 conv")
        return y

    fused = conv(xd, ex, cin + ex, 1)
    ref = conv(pooled, 0, cin, 0)
    torch.cuda.synchronize()
    assert torch.equal(fused.cpu(), ref.cpu())
    assert torch.all(fused[..., :8] == 0)


def test_fp8_tile_choice_and_rejects(device):
    d = L.ConvDesc()
    d.n, d.h, d.w, d.cin, d.in_c_off, d.in_c_stride = 32, 80, 80, 256, 0, 256
    d.ho, d.wo, d.cout, d.cout_pad, d.out_c_off, d.out_c_stride = 80, 80, 128, 128, 0, 128
    d.kh = d.kw = 3
    d.stride, d.pad, d.act, d.dtype = 1, 1, L.ACT_SILU, L.DT_FP8
    assert L.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 34
    d.n = 1
    assert L.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 35
    d.cin, d.in_c_stride = 40, 48  # cin % 16 != 0
    z = torch.zeros(1 << 20, dtype=torch.uint8, device=device)
    st = L.lib.ycx_conv2d(ctypes.byref(d), z.data_ptr(), z.data_ptr(), z.data_ptr(), z.data_ptr(), None,
                          L.stream_handle(device))
    assert st == L.YCX_ERR_UNSUPPORTED


@pytest.fixture(scope='module')
def v7_fp8(device):
    m, sd = make_model('yolov7', 80, 0, 'fp8')
    m.to(device)
    x = synthetic_images(2, 3, 640, 640, seed=3)
    ref = ref_forward.build(cvt_cfg('yolov7'), ANCHORS, 80, sd)(x)
    return m, sd, x, ref


def test_yolov7_640_fp8_vs_oracle(device, v7_fp8):
    m, _, x, ref = v7_fp8
    outs = m(x.to(device))
    errs = [rel_err(o.cpu(), r) for o, r in zip(outs, ref)]
    print("fp8 yolov7 640 rel err per head", errs)
    assert max(errs) < FP8_TOL, errs
    eng = m.engine_for(x.shape, device)
    assert eng.dt == L.DT_FP8 and all(t.dtype == torch.float8_e4m3fn for t in eng.buffers)
    names = {i['name'].split('+')[0] for i in eng.op_info if i['kind'] == 'conv'}  # '+maxpool_k2s2': MP fused
    assert sum(1 for i in eng.op_info if i['name'].endswith('+maxpool_k2s2')) == 5
    assert names <= {'f8_co128_px128_k128_s2', 'f8_co64_px128_k128_s2', 'f8_wres1x1', 'f8_halo3x3_ws_co64'}, names
    # every scale is a power of two and the calibrated maxima sit in [224, 448)
    assert all(float(s).hex().startswith(('0x1.0000000000000p', '0x1p')) for s in eng.scales.values())


@pytest.mark.parametrize('name', ['conv_k3s1_cin32', 'conv_k1_cin64', 'conv_leaky', 'pools', 'upsample_concat',
                                  'sppcspc', 'repconv', 'csp_blocks', 'detect'])
def test_g1_ops_fp8(device, manifest, g1, name):
    from helpers import g1_case
    m, sd, x, e = g1_case(manifest, name, 'fp8')
    m.to(device)
    y = m(x.to(device))
    outs = y if isinstance(y, list) else [y]
    for j, o in enumerate(outs):
        gold = torch.from_numpy(g1[f'{name}/{j}'])
        assert o.shape == gold.shape
        print(f"\nfp8 G1 {name} out {j} rel err {rel_err(o.cpu(), gold):.4f}")
        assert rel_err(o.cpu(), gold) < FP8_TOL, (name, j, rel_err(o.cpu(), gold))


def test_fp8_detector_decode_nms(device):
    """C5 shape class at small batch: the fused decode + NMS on the fp8 model's
    heads equals the oracle chain on the same heads (the post path is fp32)."""
    m, _ = make_model('yolov7', 80, 0, 'fp8')
    m.to(device)
    shape = (2, 3, 640, 640)
    det = Detector(m, shape, device, ANCHORS, MASK, conf_thres=0.3, nms_thres=0.3, max_det=30000)
    x = synthetic_images(*shape, seed=21).to(device)
    dets, keep, kc = det(x)
    torch.cuda.synchronize()
    heads = [h.cpu() for h in det.heads]
    from helpers import fused_keep_report
    cpu = [t.cpu() for t in (det.cand, det.cand_rows, det.counts, keep, kc)]
    rep = fused_keep_report(*cpu, 0, [h[0] for h in heads], 80, 0.3, 0.3, 640, 30000)
    print(f"\nfp8 bs=2 image 0: {rep}")
    assert rep['n_keep'] > 0 and rep['cls_same'] and rep['nms_exact'], rep
    assert rep['box_maxdiff'] <= 2e-6 and rep['member_max_dist'] <= 1e-6, rep
    assert rep['keep_flips'] <= 4 and rep['unexplained_flips'] == 0, rep   # measured on MI355X: 0


def test_fp8_calibration_record(device):
    m, _ = make_model('yolov7-tiny', 1, 0, 'fp8')
    m.to(device)
    rec = m.calibrate_fp8(device=device, hw=(320, 320), n=2)
    assert all(r['amax'] > 0 for r in rec)
    eng = m.engine_for((2, 3, 320, 320), device)
    assert len(eng.buffers) == len(rec)
    # a weight update drops the stale calibration
    m.load_state_dict(m.state_dict())
    assert m._fp8_amax == {}
