"""Kernel-level numerics through the C ABI vs a plain PyTorch fp32 (CPU, float64
accumulate) reference of the same op on the same (bf16-rounded) operands."""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

L = pytest.importorskip("ycx._lib")


def _ref_conv(x_nchw, w, b, s, p, act, slope=0.1):
    y = F.conv2d(x_nchw.double(), w.double(), b.double(), s, p)
    if act in (L.ACT_SILU, L.ACT_SILU_PS):
        y = F.silu(y)
    elif act == L.ACT_LEAKY:
        y = F.leaky_relu(y, slope)
    return y


def _run_conv(device, n, h, w, cin, cout, k, s, act, tile, dtype, in_extra=0, out_extra=0, residual=False,
              layout=L.OUT_NHWC, seed=0, k_split=0):
    g = torch.Generator().manual_seed(seed)
    tdt = {L.DT_BF16: torch.bfloat16, L.DT_F16: torch.float16}.get(dtype, torch.float32)
    p = k // 2
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    x = torch.randn(n, h, w, cin + in_extra, generator=g).to(tdt)           # NHWC, slice at in_extra
    wt = (torch.randn(cout, cin, k, k, generator=g) / (cin * k * k) ** 0.5).to(tdt)
    b = torch.randn(cout, generator=g) * 0.1
    cpad = -(-cout // 64) * 64 if dtype == L.DT_F32 else (32 if cout <= 32 else 64 if cout <= 64 else -(-cout // 128) * 128)
    ks = L.SILU_PS_K if act == L.ACT_SILU_PS else 1.0  # YCX_ACT_SILU_PS: weights and bias packed x -log2(e)
    wp = torch.zeros(cpad, k, k, cin, dtype=tdt)
    wp[:cout] = (wt.double() * ks).to(tdt).permute(0, 2, 3, 1)
    bp = torch.zeros(cpad)
    bp[:cout] = b * ks
    up = 2 if layout == L.OUT_NHWC_UP2 else 1
    if layout == L.OUT_NCHW_F32:
        y = torch.zeros(n, cout, ho, wo, dtype=torch.float32)
    else:
        y = torch.zeros(n, ho * up, wo * up, cout + out_extra, dtype=tdt)
    r = torch.randn(n, ho, wo, cout, generator=g).to(tdt) if residual else None
    d = L.ConvDesc()
    d.n, d.h, d.w, d.cin, d.in_c_off, d.in_c_stride = n, h, w, cin, in_extra, cin + in_extra
    d.ho, d.wo, d.cout, d.cout_pad = ho, wo, cout, cpad
    d.out_c_off, d.out_c_stride = (0, cout) if layout == L.OUT_NCHW_F32 else (out_extra, cout + out_extra)
    d.kh = d.kw = k
    d.stride, d.pad, d.act, d.leaky_slope = s, p, act, 0.1
    d.dtype, d.out_layout = dtype, layout
    d.res_c_off, d.res_c_stride = 0, cout
    d.tile = tile
    d.k_split = k_split
    xd, wd, bd, yd = x.to(device), wp.contiguous().to(device), bp.to(device), y.to(device)
    rd = r.to(device) if r is not None else None
    if k_split > 1:
        nws = int(L.lib.ycx_conv_workspace_size(ctypes.byref(d)))
        assert nws == k_split * n * ho * wo * cpad * 4
        ws = torch.full((nws // 4,), float('nan'), device=device)  # every partial must be overwritten
        L.check(L.lib.ycx_conv2d_ws(ctypes.byref(d), xd.data_ptr(), wd.data_ptr(), bd.data_ptr(), yd.data_ptr(),
                                    rd.data_ptr() if rd is not None else None, ws.data_ptr(), nws,
                                    L.stream_handle(device)))
    else:
        L.check(L.lib.ycx_conv2d(ctypes.byref(d), xd.data_ptr(), wd.data_ptr(), bd.data_ptr(), yd.data_ptr(),
                                 rd.data_ptr() if rd is not None else None, L.stream_handle(device)))
    torch.cuda.synchronize()
    ref = _ref_conv(x[..., in_extra:].permute(0, 3, 1, 2).float(), wt.float(), b, s, p, act)
    if residual:
        ref = ref + r.permute(0, 3, 1, 2).double()
    got = yd.cpu()
    if layout == L.OUT_NCHW_F32:
        got = got.double()
    elif layout == L.OUT_NHWC_UP2:
        got = got[..., out_extra:].permute(0, 3, 1, 2).double()
        ref = ref.repeat_interleave(2, 2).repeat_interleave(2, 3)
    else:
        got = got[..., out_extra:].permute(0, 3, 1, 2).double()
        assert torch.all(yd.cpu()[..., :out_extra] == 0), "wrote outside the output channel slice"
    return got, ref


TILES_BF16 = [(1, 128, 64), (2, 64, 64), (3, 64, 64), (4, 128, 64), (5, 32, 32), (6, 64, 32), (7, 128, 32),
              (9, 128, 64), (10, 64, 64), (11, 256, 128), (12, 128, 64), (13, 64, 32), (14, 128, 32), (14, 256, 32),
              (15, 64, 64), (16, 128, 64), (17, 64, 32), (18, 64, 128), (56, 64, 128), (56, 192, 64)]


@pytest.mark.parametrize('tile,cout,cin', TILES_BF16)
@pytest.mark.parametrize('k,s', [(3, 1), (1, 1), (3, 2), (5, 1)])
def test_conv_bf16_tiles(device, tile, cout, cin, k, s):
    got, ref = _run_conv(device, 2, 13, 11, cin, cout, k, s, L.ACT_SILU, tile, L.DT_BF16, in_extra=8, out_extra=16)
    # bf16 output rounding (2^-8 relative) on top of exact products of bf16 inputs
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize('tile,cout,cin,k,s', [(16, 128, 64, 3, 1), (16, 256, 128, 1, 1), (18, 64, 128, 3, 2),
                                               (17, 64, 32, 3, 1), (5, 32, 32, 3, 1), (7, 128, 32, 3, 2),
                                               (1, 128, 64, 3, 1), (11, 256, 128, 3, 1)])
def test_conv_fp16_tiles(device, tile, cout, cin, k, s):
    """The same tiles built with IEEE half elements (YCX_DT_F16, v_mfma_f32_16x16x32_f16):
    fp16 output rounding (2^-11 relative) on top of exact products of fp16 inputs."""
    got, ref = _run_conv(device, 2, 13, 11, cin, cout, k, s, L.ACT_SILU, tile, L.DT_F16, in_extra=8, out_extra=16)
    torch.testing.assert_close(got, ref, rtol=2e-3, atol=2e-3)


@pytest.mark.parametrize('tile,args', [(19, (2, 16, 16, 64, 64, 3, 1)), (20, (2, 32, 48, 128, 256, 3, 1)),
                                       (22, (2, 13, 11, 256, 248, 1, 1)), (23, (2, 32, 48, 64, 64, 3, 1)),
                                       (0, (3, 20, 20, 256, 255, 1, 1))])
def test_conv_fp16_special_kernels(device, tile, args):
    """fp16 halo (19, 20), weight-resident 1x1 (22), weight-stationary 3x3 (23) and the
    fp32 NCHW head store."""
    n, h, w, cin, cout, k, s = args
    layout = L.OUT_NCHW_F32 if cout == 255 else L.OUT_NHWC
    extra = 0 if layout == L.OUT_NCHW_F32 else 16
    got, ref = _run_conv(device, n, h, w, cin, cout, k, s, L.ACT_SILU if cout != 255 else L.ACT_NONE, tile,
                         L.DT_F16, in_extra=8, out_extra=extra, layout=layout)
    torch.testing.assert_close(got, ref, rtol=2e-3, atol=2e-3)


@pytest.mark.parametrize('tile,cout', [(16, 128), (18, 64), (56, 64), (56, 192)])
@pytest.mark.parametrize('k_split', [2, 3, 4])
@pytest.mark.parametrize('cin,k,s', [(256, 3, 1), (512, 1, 1), (128, 3, 2), (256, 3, 2)])
def test_conv_splitk(device, tile, cout, k_split, cin, k, s):
    """Split-K (ycx_conv_desc.k_split, r06): K ranges on separate workgroups, fp32 partials in the
    workspace, one ordered reduce launch with bias + act; ragged pixel tail (13 x 11), input and
    output channel slices, the chunk-major stride-2 K order at cin 128 (tile 16)."""
    got, ref = _run_conv(device, 2, 13, 11, cin, cout, k, s, L.ACT_SILU, tile, L.DT_BF16, in_extra=8, out_extra=16,
                         k_split=k_split)
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize('dtype,layout,residual,act', [(L.DT_BF16, L.OUT_NHWC, True, L.ACT_LEAKY),
                                                       (L.DT_BF16, L.OUT_NHWC_UP2, False, L.ACT_NONE),
                                                       (L.DT_F16, L.OUT_NHWC, True, L.ACT_SILU),
                                                       (L.DT_F16, L.OUT_NHWC_UP2, False, L.ACT_SILU)])
@pytest.mark.parametrize('tile', [16, 18])
def test_conv_splitk_residual_up2(device, dtype, layout, residual, act, tile):
    """The split-K reduce's store is the unsplit epilogue's (store8): residual added after the
    activation, x2 nearest upsample, fp16 elements."""
    cout = 128 if tile == 16 else 64
    got, ref = _run_conv(device, 3, 20, 20, 512, cout, 3, 1, act, tile, dtype, in_extra=0, out_extra=8 if
                         layout == L.OUT_NHWC else 0, residual=residual, layout=layout, k_split=2)
    tol = 1e-2 if dtype == L.DT_BF16 else 2e-3
    torch.testing.assert_close(got, ref, rtol=tol, atol=tol)


@pytest.mark.parametrize('tile,cout,cin,k,s', [(16, 128, 64, 3, 1), (18, 64, 128, 3, 2), (16, 128, 128, 3, 2),
                                               (22, 256, 256, 1, 1), (22, 128, 128, 1, 1), (23, 64, 64, 3, 1),
                                               (20, 128, 64, 3, 1), (50, 128, 64, 3, 2), (5, 32, 32, 3, 1),
                                               (7, 128, 32, 3, 1), (17, 64, 32, 3, 1)])
@pytest.mark.parametrize('dtype', [L.DT_BF16, L.DT_F16])
def test_conv_silu_prescaled(device, tile, cout, cin, k, s, dtype):
    """YCX_ACT_SILU_PS (r06): weights and bias packed x -log2(e), the epilogue's SiLU one multiply
    shorter; against torch's silu of the unscaled conv on the same operands, every tile family
    (LDS-DMA, register-staged, weight-resident 1x1, weight-stationary 3x3, halo, tile 50)."""
    h, w = (32, 32) if tile in (23, 20, 50) else (13, 11)
    got, ref = _run_conv(device, 2, h, w, cin, cout, k, s, L.ACT_SILU_PS, tile, dtype, in_extra=0 if tile in (22, 23, 50) else 8,
                         out_extra=0 if tile in (22, 23, 50) else 16)
    tol = 1e-2 if dtype == L.DT_BF16 else 2e-3
    torch.testing.assert_close(got, ref, rtol=tol, atol=tol)


def test_conv_silu_prescaled_rejects_f32(device):
    """The fp32 parity path keeps torch's silu: YCX_ACT_SILU_PS is refused there."""
    with pytest.raises(L.YcxError, match='unsupported'):
        _run_conv(device, 2, 13, 11, 64, 128, 3, 1, L.ACT_SILU_PS, 8, L.DT_F32)


def test_conv_splitk_rejects(device):
    """k_split > 1 needs a workspace (YCX_ERR_CAPACITY without one) and one of the LDS-DMA
    tiles 16 / 18 / 56 (the weight-resident, halo and fp32 tiles refuse it)."""
    with pytest.raises(L.YcxError, match='capacity'):
        d = L.ConvDesc()
        d.n, d.h, d.w, d.cin, d.in_c_stride, d.ho, d.wo, d.cout, d.cout_pad, d.out_c_stride = \
            1, 8, 8, 64, 64, 8, 8, 128, 128, 128
        d.kh = d.kw = 1
        d.stride, d.dtype, d.tile, d.k_split = 1, L.DT_BF16, 16, 2
        x = torch.zeros(1, 8, 8, 64, dtype=torch.bfloat16, device=device)
        wt = torch.zeros(128, 64, dtype=torch.bfloat16, device=device)
        b = torch.zeros(128, device=device)
        y = torch.zeros(1, 8, 8, 128, dtype=torch.bfloat16, device=device)
        L.check(L.lib.ycx_conv2d(ctypes.byref(d), x.data_ptr(), wt.data_ptr(), b.data_ptr(), y.data_ptr(), None,
                                 L.stream_handle(device)))
    for tile in (22, 20, 8):
        with pytest.raises(L.YcxError, match='unsupported'):
            _run_conv(device, 2, 16, 16, 64, 128, 3 if tile == 20 else 1, 1, L.ACT_SILU, tile,
                      L.DT_F32 if tile == 8 else L.DT_BF16, k_split=2)


@pytest.mark.parametrize('tile', [27, 31, 33, 40, 41, 42, 43, 44, 47, 57])
def test_retired_tiles_are_not_dispatched(device, tile):
    """Tiles 27-33 (rejected experiments) exist only in a
    -DYCX_EXPERIMENTAL_TILES build; tiles 40-47 (conv_bigt, r03) only with
    tools/experiments/conv_bigt_tiles40_47.patch applied, tile 57 (warp-specialised,
    r06) only with tools/experiments/wsp_tile57.patch: the product library refuses them."""
    with pytest.raises(L.YcxError, match='unsupported'):
        _run_conv(device, 2, 13, 11, 64, 128, 3, 1, L.ACT_SILU, tile, L.DT_BF16)


@pytest.mark.parametrize('tile,cin,cout', [(19, 64, 64), (19, 128, 192), (20, 64, 128), (20, 128, 256),
                                           (21, 192, 128), (21, 64, 256)])
@pytest.mark.parametrize('hw', [(16, 16), (32, 48)])
def test_conv_halo3x3(device, tile, cin, cout, hw):
    """LDS halo-tile 3x3/s1 kernel: image borders are the halo's zero padding,
    several 64-channel chunks re-fill the halo, channel-sliced input/output."""
    got, ref = _run_conv(device, 2, hw[0], hw[1], cin, cout, 3, 1, L.ACT_SILU, tile, L.DT_BF16, in_extra=8,
                         out_extra=16)
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize('cin', [64, 128, 256, 512])
@pytest.mark.parametrize('cout', [64, 128, 248, 256, 512])
def test_conv1x1_wres(device, cin, cout):
    """Weight-resident 1x1 kernel (tile 22): ragged pixel tail, more ranges than
    tiles, channel-sliced input/output, cout < cout_pad."""
    got, ref = _run_conv(device, 2, 13, 11, cin, cout, 1, 1, L.ACT_SILU, 22, L.DT_BF16, in_extra=8, out_extra=16)
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize('act', [L.ACT_LEAKY, L.ACT_SILU, L.ACT_NONE])
@pytest.mark.parametrize('n,hw,cin,cout', [(2, 128, 256, 256), (1, 128, 256, 512), (4, 128, 128, 128),
                                           (2, 96, 64, 64), (3, 72, 512, 256), (3, 70, 256, 248)])
def test_conv1x1_wres_multi_tile(device, n, hw, cin, cout, act):
    """Several tiles per persistent block: the LDS ring wraps across tile
    boundaries with the epilogue stores counted into the next waits; at cin <= 256 each
    tile's epilogue runs in the next tile's first K step (one instance per activation), the
    last one after the loop; a ragged last tile and cout < cout_pad (uncounted stores)."""
    got, ref = _run_conv(device, n, hw, hw, cin, cout, 1, 1, act, 22, L.DT_BF16, in_extra=8, out_extra=8)
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize('n,hw,cout,act', [(2, (40, 40), 128, L.ACT_SILU), (1, (33, 47), 120, L.ACT_LEAKY),
                                           (3, (64, 48), 256, L.ACT_NONE), (2, (160, 160), 128, L.ACT_SILU)])
def test_tile16_s2_cin128_chunk_major(device, n, hw, cout, act):
    """Tile 16 on a 3x3/s2 conv at cin 128 walks K channel-chunk-major with paired taps (its
    KCM template instance): odd map sizes (taps outside the image), several pixel and channel
    tiles, cout < cout_pad, channel-sliced input/output."""
    got, ref = _run_conv(device, n, hw[0], hw[1], 128, cout, 3, 2, act, 16, L.DT_BF16, in_extra=8, out_extra=16)
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize('n,hw,cout,act', [(2, (16, 16), 64, L.ACT_SILU), (2, (32, 48), 64, L.ACT_LEAKY),
                                           (3, (64, 80), 48, L.ACT_SILU), (1, (16, 32), 64, L.ACT_NONE)])
def test_conv3x3_ws64(device, n, hw, cout, act):
    """Weight-stationary 3x3 64->64 kernel (tile 23): image borders as halo zeros,
    several tiles per persistent block (double-buffered halo), sliced channels."""
    got, ref = _run_conv(device, n, hw[0], hw[1], 64, cout, 3, 1, act, 23, L.DT_BF16, in_extra=8, out_extra=16)
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize('n,hw,cout,act,dt', [(2, (32, 64), 128, L.ACT_SILU, L.DT_BF16),
                                              (1, (31, 63), 96, L.ACT_LEAKY, L.DT_BF16),
                                              (3, (256, 160), 128, L.ACT_SILU, L.DT_BF16),
                                              (2, (64, 32), 128, L.ACT_NONE, L.DT_F16),
                                              (3, (256, 160), 120, L.ACT_SILU, L.DT_F16)])
def test_conv3x3s2_wsr(device, n, hw, cout, act, dt):
    """3x3/s2 64 -> 128 with weights in registers (tile 50): parity-split halo columns, image
    borders (odd input sizes too), several tiles per persistent block (480 tiles on <= 256
    blocks), cout < cout_pad, channel-sliced input/output."""
    got, ref = _run_conv(device, n, hw[0], hw[1], 64, cout, 3, 2, act, 50, dt, in_extra=8, out_extra=16)
    tol = 1e-2 if dt == L.DT_BF16 else 2e-3
    torch.testing.assert_close(got, ref, rtol=tol, atol=tol)


def test_conv3x3s2_wsr_rejects(device):
    """Tile 50 needs cin 64, cout_pad 128, stride 2 and Wo % 16 == Ho % 4 == 0."""
    for args in ((2, 32, 40, 64, 128, 3, 2), (2, 32, 64, 128, 128, 3, 2), (2, 32, 64, 64, 256, 3, 2),
                 (2, 30, 64, 64, 128, 3, 2), (2, 32, 64, 64, 128, 3, 1)):
        n, h, w, cin, cout, k, s = args
        with pytest.raises(L.YcxError, match='unsupported'):
            _run_conv(device, n, h, w, cin, cout, k, s, L.ACT_SILU, 50, L.DT_BF16)


@pytest.mark.parametrize('tile,cin,cout', [(48, 64, 64), (48, 128, 192), (48, 256, 128), (49, 64, 128),
                                           (49, 128, 256), (49, 256, 384)])
def test_conv_halo3x3_band(device, tile, cin, cout):
    """Band halo tiles (48: 8 x 40, 49: 4 x 40 output rows of a 40-wide map): each lane finds
    its fragment pixel's (row, column) in the halo; image borders, several 64-channel chunks,
    channel slices; then a residual and the x2 upsample store."""
    got, ref = _run_conv(device, 2, 40, 40, cin, cout, 3, 1, L.ACT_SILU, tile, L.DT_BF16, in_extra=8, out_extra=16)
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-2)
    got, ref = _run_conv(device, 1, 40, 40, cin, cout, 3, 1, L.ACT_LEAKY, tile, L.DT_BF16, residual=True, seed=1)
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=2e-2)
    got, ref = _run_conv(device, 1, 40, 40, cin, cout, 3, 1, L.ACT_SILU, tile, L.DT_F16, layout=L.OUT_NHWC_UP2,
                         seed=2)
    torch.testing.assert_close(got, ref, rtol=2e-3, atol=2e-3)


def test_conv_halo3x3_band_rejects(device):
    """Band tiles need the map's full width (40) and whole bands of rows."""
    for tile, hw in ((48, (40, 32)), (48, (36, 40)), (49, (42, 40))):
        with pytest.raises(L.YcxError, match='unsupported'):
            _run_conv(device, 1, hw[0], hw[1], 64, 64 if tile == 48 else 128, 3, 1, L.ACT_SILU, tile, L.DT_BF16)


def test_conv_halo3x3_residual_up2(device):
    got, ref = _run_conv(device, 1, 32, 16, 64, 64, 3, 1, L.ACT_LEAKY, 19, L.DT_BF16, residual=True)
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=2e-2)
    got, ref = _run_conv(device, 1, 16, 32, 128, 128, 3, 1, L.ACT_SILU, 20, L.DT_BF16, layout=L.OUT_NHWC_UP2)
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize('cin,cout,k,s', [(32, 64, 3, 1), (64, 128, 3, 2), (128, 255, 1, 1), (64, 32, 1, 1)])
def test_conv_f32(device, cin, cout, k, s):
    layout = L.OUT_NCHW_F32 if cout == 255 else L.OUT_NHWC
    got, ref = _run_conv(device, 2, 9, 10, cin, cout, k, s, L.ACT_LEAKY, 0, L.DT_F32, layout=layout)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


def test_conv_heads_nchw_bf16(device):
    got, ref = _run_conv(device, 3, 20, 20, 256, 255, 1, 1, L.ACT_NONE, 0, L.DT_BF16, layout=L.OUT_NCHW_F32)
    torch.testing.assert_close(got, ref, rtol=1e-3, atol=1e-3)  # fp32 output: only accumulation order differs


def test_conv_residual_and_up2(device):
    got, ref = _run_conv(device, 2, 8, 8, 64, 64, 3, 1, L.ACT_SILU, 0, L.DT_BF16, residual=True)
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=2e-2)
    got, ref = _run_conv(device, 2, 5, 7, 128, 128, 1, 1, L.ACT_SILU, 0, L.DT_BF16, layout=L.OUT_NHWC_UP2,
                         out_extra=8)
    torch.testing.assert_close(got, ref, rtol=1e-2, atol=1e-2)
    got, ref = _run_conv(device, 2, 5, 7, 64, 64, 1, 1, L.ACT_NONE, 0, L.DT_F32, layout=L.OUT_NHWC_UP2, residual=False)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)


def test_conv_rejects_bad_shapes(device):
    d = L.ConvDesc()
    d.n, d.h, d.w, d.cin, d.in_c_stride, d.ho, d.wo, d.cout, d.cout_pad = 1, 8, 8, 24, 24, 8, 8, 64, 64
    d.out_c_stride, d.kh, d.kw, d.stride, d.pad, d.dtype = 64, 3, 3, 1, 1, L.DT_BF16
    t = torch.zeros(1 << 16, device=device)
    s = L.lib.ycx_conv2d(ctypes.byref(d), t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr(), None,
                         L.stream_handle(device))
    assert s == L.YCX_ERR_UNSUPPORTED  # cin 24 is not a multiple of the 32-wide K step
    d.cin, d.in_c_stride, d.ho = 32, 32, 7
    assert L.lib.ycx_conv2d(ctypes.byref(d), t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr(), None,
                            L.stream_handle(device)) == L.YCX_ERR_BAD_ARG
    assert L.lib.ycx_conv2d(None, None, None, None, None, None, None) == L.YCX_ERR_BAD_ARG


@pytest.mark.parametrize('dtype', [L.DT_BF16, L.DT_F32])
@pytest.mark.parametrize('k,s,p', [(2, 2, 0), (5, 1, 2), (9, 1, 4), (13, 1, 6), (3, 2, 1)])
def test_maxpool(device, dtype, k, s, p):
    tdt = torch.bfloat16 if dtype == L.DT_BF16 else torch.float32
    n, h, w, c = 2, 11, 13, 32
    x = torch.randn(n, h, w, c + 8).to(tdt)
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    y = torch.zeros(n, ho, wo, c + 16, dtype=tdt)
    d = L.PoolDesc()
    d.n, d.h, d.w, d.c, d.in_c_off, d.in_c_stride = n, h, w, c, 8, c + 8
    d.ho, d.wo, d.out_c_off, d.out_c_stride, d.k, d.stride, d.pad, d.dtype = ho, wo, 16, c + 16, k, s, p, dtype
    xd, yd = x.to(device), y.to(device)
    L.check(L.lib.ycx_maxpool(ctypes.byref(d), xd.data_ptr(), yd.data_ptr(), L.stream_handle(device)))
    ref = F.max_pool2d(x[..., 8:].permute(0, 3, 1, 2).float(), k, s, p).permute(0, 2, 3, 1)
    assert torch.equal(yd.cpu()[..., 16:].float(), ref)  # max is exact


@pytest.mark.parametrize('hw,c,k', [((20, 20), 512, 5), ((11, 13), 48, 5), ((40, 40), 256, 3), ((7, 9), 16, 7)])
@pytest.mark.parametrize('fp8', [False, True])
def test_maxpool_cascade(device, hw, c, k, fp8):
    """levels = 3 (SPPCSPC's 5 / 9 / 13 as a k5 cascade, one launch, the plane in LDS) vs
    torch max_pool2d applied level after level; level i lands at out_c_off + i*c. Max is exact:
    bf16 bit for bit, e4m3 bytes bit for bit (values go through float and back unchanged)."""
    n, (h, w) = 2, hw
    g = torch.Generator().manual_seed(3)
    xf = torch.randn(n, h, w, c + 16, generator=g) * 4
    if fp8:
        x = xf.to(torch.float8_e4m3fn)
        xv, dt = x.float(), L.DT_FP8
        y = torch.zeros(n, h, w, 3 * c + 32, dtype=torch.uint8)
        xd = x.view(torch.uint8).to(device)
    else:
        x = xf.to(torch.bfloat16)
        xv, dt = x.float(), L.DT_BF16
        y = torch.zeros(n, h, w, 3 * c + 32, dtype=torch.bfloat16)
        xd = x.to(device)
    d = L.PoolDesc()
    d.n, d.h, d.w, d.c, d.in_c_off, d.in_c_stride = n, h, w, c, 16, c + 16
    d.ho, d.wo, d.out_c_off, d.out_c_stride = h, w, 32, 3 * c + 32
    d.k, d.stride, d.pad, d.dtype, d.levels = k, 1, k // 2, dt, 3
    yd = y.to(device)
    L.check(L.lib.ycx_maxpool(ctypes.byref(d), xd.data_ptr(), yd.data_ptr(), L.stream_handle(device)))
    got = yd.cpu()
    cur = xv[..., 16:].permute(0, 3, 1, 2)
    for lv in range(3):
        cur = F.max_pool2d(cur, k, 1, k // 2)
        sl = got[..., 32 + lv * c:32 + (lv + 1) * c]
        sl = sl.view(torch.float8_e4m3fn).float() if fp8 else sl.float()
        assert torch.equal(sl, cur.permute(0, 2, 3, 1)), lv
    assert not got[..., :32].any()  # channels before out_c_off untouched


@pytest.mark.parametrize('tile', [0, 16, 18])
@pytest.mark.parametrize('n,hw,cin,cout', [(2, (13, 11), 64, 128), (3, (20, 20), 256, 128), (1, (8, 40), 128, 256),
                                           (2, (10, 10), 512, 256), (1, (5, 7), 64, 64)])
def test_conv_pool_fused(device, tile, n, hw, cin, cout):
    """MP fused into the 1x1 conv (ycx_conv_desc.in_pool: the k2 s2 max-pool of the (2h, 2w)
    map formed in the operand staging) vs ycx_maxpool then the same tile on the pooled map:
    bit for bit (the max is exact, the MFMA sees identical operands in the same order), and
    vs the float64 reference of pool + conv. Ragged pixel tails, channel-sliced input."""
    g = torch.Generator().manual_seed(11)
    (h, w), ex = hw, 16
    x = (torch.randn(n, 2 * h, 2 * w, cin + ex, generator=g) * 2).to(torch.bfloat16)
    wt = (torch.randn(cout, cin, generator=g) / cin ** 0.5).to(torch.bfloat16)
    b = torch.randn(cout, generator=g) * 0.1
    cpad = 64 if cout <= 64 else -(-cout // 128) * 128
    if tile == 16 and cpad % 128:
        pytest.skip("tile 16 is 128 output channels wide")
    wp = torch.zeros(cpad, cin, dtype=torch.bfloat16)
    wp[:cout] = wt
    bp = torch.zeros(cpad)
    bp[:cout] = b
    xd, wd, bd = x.to(device), wp.to(device), bp.to(device)
    pooled = torch.zeros(n, h, w, cin, dtype=torch.bfloat16, device=device)
    pd = L.PoolDesc()
    pd.n, pd.h, pd.w, pd.c, pd.in_c_off, pd.in_c_stride = n, 2 * h, 2 * w, cin, ex, cin + ex
    pd.ho, pd.wo, pd.out_c_off, pd.out_c_stride, pd.k, pd.stride, pd.pad, pd.dtype = h, w, 0, cin, 2, 2, 0, L.DT_BF16
    pd.levels = 1
    L.check(L.lib.ycx_maxpool(ctypes.byref(pd), xd.data_ptr(), pooled.data_ptr(), L.stream_handle(device)))

    def conv(src, in_off, in_stride, in_pool):
        y = torch.zeros(n, h, w, cout + 8, dtype=torch.bfloat16, device=device)
        d = L.ConvDesc()
        d.n, d.h, d.w, d.cin, d.in_c_off, d.in_c_stride = n, h, w, cin, in_off, in_stride
        d.ho, d.wo, d.cout, d.cout_pad, d.out_c_off, d.out_c_stride = h, w, cout, cpad, 8, cout + 8
        d.kh = d.kw = d.stride = 1
        d.pad, d.act, d.leaky_slope, d.dtype, d.out_layout = 0, L.ACT_SILU, 0.1, L.DT_BF16, L.OUT_NHWC
        d.in_pool = in_pool
        d.tile = tile if tile else int(L.lib.ycx_conv_pick_tile(ctypes.byref(d)))
        L.check(L.lib.ycx_conv2d(ctypes.byref(d), src.data_ptr(), wd.data_ptr(), bd.data_ptr(), y.data_ptr(), None,
                                 L.stream_handle(device)))
        return y, d.tile

    fused, tile = conv(xd, ex, cin + ex, 1)  # auto: the unfused call runs the tile the fused one picked
    assert tile in (16, 18)
    unfused = conv(pooled, 0, cin, 0)[0]
    torch.cuda.synchronize()
    assert torch.equal(fused.cpu(), unfused.cpu())
    assert not fused.cpu()[..., :8].any()
    ref = F.silu(F.conv2d(F.max_pool2d(x[..., ex:].permute(0, 3, 1, 2).double(), 2, 2), wt.double()[..., None, None],
                          b.double()))
    torch.testing.assert_close(fused.cpu()[..., 8:].permute(0, 3, 1, 2).double(), ref, rtol=1e-2, atol=1e-2)


def test_conv_pool_fused_rejects(device):
    """in_pool is a bf16 1x1 / s1 / p0 feature of tiles 16 / 18 / 25."""
    d = L.ConvDesc()
    d.n, d.h, d.w, d.cin, d.in_c_stride, d.ho, d.wo, d.cout, d.cout_pad = 1, 8, 8, 64, 64, 8, 8, 128, 128
    d.out_c_stride, d.kh, d.kw, d.stride, d.pad, d.dtype, d.in_pool = 128, 1, 1, 1, 0, L.DT_BF16, 1
    t = torch.zeros(1 << 16, device=device)
    call = lambda: L.lib.ycx_conv2d(ctypes.byref(d), t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr(), None,
                                    L.stream_handle(device))
    d.tile = 22
    assert call() == L.YCX_ERR_UNSUPPORTED
    d.tile, d.dtype = 0, L.DT_F32
    assert call() == L.YCX_ERR_UNSUPPORTED
    d.dtype, d.kh, d.kw, d.pad = L.DT_BF16, 3, 3, 1
    assert call() == L.YCX_ERR_UNSUPPORTED
    d.kh, d.kw, d.pad, d.in_pool = 1, 1, 0, 2
    assert call() == L.YCX_ERR_BAD_ARG


@pytest.mark.parametrize('dtype', [L.DT_BF16, L.DT_F32])
@pytest.mark.parametrize('scale,nchw', [(1, False), (2, False), (1, True)])
def test_copy_upsample(device, dtype, scale, nchw):
    tdt = torch.bfloat16 if dtype == L.DT_BF16 else torch.float32
    n, h, w, c = 2, 5, 6, 16
    x = torch.randn(n, h, w, c + 8).to(tdt)
    d = L.CopyDesc()
    d.n, d.h, d.w, d.c, d.in_c_off, d.in_c_stride, d.scale, d.dtype = n, h, w, c, 8, c + 8, scale, dtype
    ref = F.interpolate(x[..., 8:].permute(0, 3, 1, 2).float(), scale_factor=scale, mode='nearest')
    if nchw:
        y = torch.zeros(n, c, h, w, dtype=torch.float32)
        d.out_c_off, d.out_c_stride, d.out_layout = 0, c, L.OUT_NCHW_F32
    else:
        y = torch.zeros(n, h * scale, w * scale, c + 24, dtype=tdt)
        d.out_c_off, d.out_c_stride, d.out_layout = 24, c + 24, L.OUT_NHWC
    xd, yd = x.to(device), y.to(device)
    L.check(L.lib.ycx_copy_channels(ctypes.byref(d), xd.data_ptr(), yd.data_ptr(), L.stream_handle(device)))
    got = yd.cpu().float() if nchw else yd.cpu()[..., 24:].permute(0, 3, 1, 2).float()
    assert torch.equal(got, ref)


@pytest.mark.parametrize('cin,k,s', [(3, 3, 1), (3, 3, 2), (1, 3, 1)])
@pytest.mark.parametrize('dtype', [L.DT_BF16, L.DT_F32])
@pytest.mark.parametrize('h,w,cout', [(17, 19, 32), (18, 32, 32), (9, 64, 64)])  # wo % 16 == 0: MFMA stem
def test_stem(device, cin, k, s, dtype, h, w, cout):
    n = 2
    x = torch.rand(n, cin, h, w)
    wt = torch.randn(cout, cin, k, k) * 0.3
    b = torch.randn(cout) * 0.1
    p = k // 2
    ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
    tdt = torch.bfloat16 if dtype == L.DT_BF16 else torch.float32
    y = torch.zeros(n, ho, wo, cout, dtype=tdt)
    d = L.ConvDesc()
    d.n, d.h, d.w, d.cin, d.in_c_off, d.in_c_stride = n, h, w, cin, 0, cin
    d.ho, d.wo, d.cout, d.cout_pad, d.out_c_off, d.out_c_stride = ho, wo, cout, cout, 0, cout
    d.kh = d.kw = k
    d.stride, d.pad, d.act, d.leaky_slope, d.dtype, d.out_layout = s, p, L.ACT_SILU, 0.1, dtype, L.OUT_NHWC
    wd = wt.permute(2, 3, 1, 0).contiguous().to(device)
    xd, bd, yd = x.to(device), b.to(device), y.to(device)
    L.check(L.lib.ycx_stem_conv(ctypes.byref(d), xd.data_ptr(), wd.data_ptr(), bd.data_ptr(), yd.data_ptr(),
                                L.stream_handle(device)))
    ref = _ref_conv(x, wt, b, s, p, L.ACT_SILU)
    got = yd.cpu().permute(0, 3, 1, 2).double()
    tol = 1e-2 if dtype == L.DT_BF16 else 1e-5
    torch.testing.assert_close(got, ref, rtol=tol, atol=tol)


@pytest.mark.parametrize('stem_s,cout,act,nhw', [(1, 64, L.ACT_SILU, (2, 32, 64)), (2, 64, L.ACT_LEAKY, (2, 64, 128)),
                                                 (1, 48, L.ACT_SILU, (2, 32, 64)), (1, 64, L.ACT_NONE, (2, 32, 64)),
                                                 (2, 32, L.ACT_SILU, (2, 64, 128)),
                                                 (1, 64, L.ACT_SILU, (3, 256, 512)),    # 3 tiles per block
                                                 (1, 64, L.ACT_SILU, (5, 128, 256)),    # ragged: 1-2 per block
                                                 (2, 64, L.ACT_LEAKY, (3, 512, 512)),   # ragged, stem stride 2
                                                 (1, 64, L.ACT_SILU_PS, (3, 256, 512)),  # pre-scaled SiLU (r06)
                                                 (2, 48, L.ACT_SILU_PS, (2, 64, 128))])
def test_stem_conv2_fused(device, stem_s, cout, act, nhw):
    """ycx_stem_conv2 = stem (3x3, 3->32) then 3x3/s2 conv, stem map kept in LDS
    (rounded to bf16 there, as the unfused path stores it); the larger shapes give each
    persistent block several tiles, and ranges of unequal length."""
    g = torch.Generator().manual_seed(5)
    n, h, w = nhw
    x = torch.rand(n, 3, h, w, generator=g)
    ws = torch.randn(32, 3, 3, 3, generator=g) * 0.3
    bs = torch.randn(32, generator=g) * 0.1
    wc = (torch.randn(cout, 32, 3, 3, generator=g) / 17.0).to(torch.bfloat16)
    bc = torch.randn(cout, generator=g) * 0.1
    sh, sw = (h - 1) // stem_s + 1, (w - 1) // stem_s + 1
    ho, wo = (sh - 1) // 2 + 1, (sw - 1) // 2 + 1
    out_extra = 8
    y = torch.zeros(n, ho, wo, cout + out_extra, dtype=torch.bfloat16)
    ds, dc = L.ConvDesc(), L.ConvDesc()
    ds.n, ds.h, ds.w, ds.cin, ds.in_c_off, ds.in_c_stride = n, h, w, 3, 0, 3
    ds.ho, ds.wo, ds.cout, ds.cout_pad, ds.out_c_off, ds.out_c_stride = sh, sw, 32, 32, 0, 32
    ds.kh = ds.kw = 3
    ds.stride, ds.pad, ds.act, ds.leaky_slope, ds.dtype, ds.out_layout = stem_s, 1, act, 0.1, L.DT_BF16, L.OUT_NHWC
    dc.n, dc.h, dc.w, dc.cin, dc.in_c_off, dc.in_c_stride = n, sh, sw, 32, 0, 32
    dc.ho, dc.wo, dc.cout, dc.cout_pad, dc.out_c_off, dc.out_c_stride = ho, wo, cout, 64, out_extra, cout + out_extra
    dc.kh = dc.kw = 3
    dc.stride, dc.pad, dc.act, dc.leaky_slope, dc.dtype, dc.out_layout = 2, 1, act, 0.1, L.DT_BF16, L.OUT_NHWC
    ks = L.SILU_PS_K if act == L.ACT_SILU_PS else 1.0  # YCX_ACT_SILU_PS: both layers packed x -log2(e)
    wsp = (ws.double() * ks).float().permute(2, 3, 1, 0).contiguous()  # [kh][kw][cin][cout_pad] fp32
    wcp = torch.zeros(64, 3, 3, 32, dtype=torch.bfloat16)
    wcp[:cout] = (wc.double() * ks).to(torch.bfloat16).permute(0, 2, 3, 1)
    bcp = torch.zeros(64)
    bcp[:cout] = bc * ks
    t = [v.to(device) for v in (x, wsp, (bs.double() * ks).float(), wcp, bcp, y)]
    L.check(L.lib.ycx_stem_conv2(ctypes.byref(ds), ctypes.byref(dc), *[v.data_ptr() for v in t],
                                 L.stream_handle(device)))
    torch.cuda.synchronize()
    mid = _ref_conv(x, ws, bs, stem_s, 1, act).to(torch.bfloat16)    # the stem map as bf16
    ref = _ref_conv(mid.float(), wc.float(), bc, 2, 1, act)
    got = t[5].cpu()
    assert torch.all(got[..., :out_extra] == 0)
    torch.testing.assert_close(got[..., out_extra:].permute(0, 3, 1, 2).double(), ref, rtol=2e-2, atol=2e-2)


def _desc_1x1(n, h, w, cin, cout, cpad, in_off, in_stride, out_off, out_stride, act, dtype, tile=0):
    d = L.ConvDesc()
    d.n, d.h, d.w, d.cin, d.in_c_off, d.in_c_stride = n, h, w, cin, in_off, in_stride
    d.ho, d.wo, d.cout, d.cout_pad, d.out_c_off, d.out_c_stride = h, w, cout, cpad, out_off, out_stride
    d.kh = d.kw = 1
    d.stride, d.pad, d.act, d.leaky_slope, d.dtype, d.out_layout, d.tile = 1, 0, act, 0.1, dtype, L.OUT_NHWC, tile
    return d


@pytest.mark.parametrize('dtype', [L.DT_BF16, L.DT_F16])
@pytest.mark.parametrize('n,hw,cin,cout2,store1', [(2, (13, 11), 256, 128, True), (2, (13, 11), 64, 256, True),
                                                   (1, (9, 7), 128, 120, False), (4, (128, 128), 256, 128, True),
                                                   (3, (96, 80), 256, 256, False), (2, (64, 72), 128, 128, True)])
def test_conv2d_pair(device, dtype, n, hw, cin, cout2, store1):
    """ycx_conv2d_pair (tile 55): y1 = act(W1 x + b1) (cin -> 256) and y2 = act(W2 y1 + b2) in one
    launch, against the same two convs run unfused with the weight-resident 1x1 (tile 22):
    y1 and y2 bit-identical (same float operations in the same order), and against a float64
    torch reference of the chain. Ragged pixel tails, several tiles per persistent block,
    input / output channel slices, cout2 < cout_pad, y1 not stored."""
    h, w = hw
    tdt = torch.bfloat16 if dtype == L.DT_BF16 else torch.float16
    g = torch.Generator().manual_seed(n * 7 + cin)
    x = torch.randn(n, h, w, cin + 8, generator=g).to(tdt)
    w1 = (torch.randn(256, cin, generator=g) / cin ** 0.5).to(tdt)
    b1 = torch.randn(256, generator=g) * 0.1
    cpad2 = 128 if cout2 <= 128 else 256
    w2 = torch.zeros(cpad2, 256, dtype=tdt)
    w2[:cout2] = (torch.randn(cout2, 256, generator=g) / 16.0).to(tdt)
    b2 = torch.zeros(cpad2)
    b2[:cout2] = torch.randn(cout2, generator=g) * 0.1
    xd, w1d, b1d, w2d, b2d = [t.to(device) for t in (x, w1, b1, w2, b2)]
    ya = torch.zeros(n, h, w, 256 + 16, dtype=tdt, device=device)
    yb = torch.zeros(n, h, w, cout2 + 8, dtype=tdt, device=device)
    da = _desc_1x1(n, h, w, cin, 256, 256, 8, cin + 8, 16, 272, L.ACT_SILU, dtype)
    db = _desc_1x1(n, h, w, 256, cout2, cpad2, 16, 272, 8, cout2 + 8, L.ACT_LEAKY, dtype)
    st = L.stream_handle(device)
    L.check(L.lib.ycx_conv2d_pair(ctypes.byref(da), ctypes.byref(db), xd.data_ptr(), w1d.data_ptr(), b1d.data_ptr(),
                                  ya.data_ptr() if store1 else None, w2d.data_ptr(), b2d.data_ptr(), yb.data_ptr(), st))
    # unfused: the same two convs through ycx_conv2d, weight-resident 1x1 tiles
    ya2, yb2 = torch.zeros_like(ya), torch.zeros_like(yb)
    da.tile, db.tile = 22, 22
    L.check(L.lib.ycx_conv2d(ctypes.byref(da), xd.data_ptr(), w1d.data_ptr(), b1d.data_ptr(), ya2.data_ptr(), None, st))
    L.check(L.lib.ycx_conv2d(ctypes.byref(db), ya2.data_ptr(), w2d.data_ptr(), b2d.data_ptr(), yb2.data_ptr(), None, st))
    torch.cuda.synchronize()
    assert torch.equal(yb, yb2)
    if store1:
        assert torch.equal(ya, ya2)
    else:
        assert not ya.any()
    assert not yb[..., :8].any() and not ya[..., :16].any()
    mid = F.silu(x[..., 8:].double() @ w1.double().t() + b1.double())
    ref = F.leaky_relu(mid.to(tdt).double() @ w2[:cout2].double().t() + b2[:cout2].double(), 0.1)
    tol = 1e-2 if dtype == L.DT_BF16 else 2e-3
    torch.testing.assert_close(yb[..., 8:].cpu().double(), ref, rtol=tol, atol=tol)


def test_conv2d_pair_rejects(device):
    """Tile 55 needs 1x1 / s1 pairs with cout_a = 256 (pad 256), cin_b = 256, cout_pad_b 128 / 256,
    cin_a in {64, 128, 256} and 16-bit NHWC."""
    t = torch.zeros(1 << 16, device=device)
    ok = dict(a=(2, 8, 8, 128, 256, 256), b=(2, 8, 8, 256, 128, 128))
    for a, b, dt in [((2, 8, 8, 128, 192, 256), ok['b'], L.DT_BF16), ((2, 8, 8, 96, 256, 256), ok['b'], L.DT_BF16),
                     (ok['a'], (2, 8, 8, 256, 200, 256), L.DT_F32), (ok['a'], (2, 8, 8, 256, 384, 384), L.DT_BF16)]:
        da = _desc_1x1(*a, 0, a[3], 0, a[4], L.ACT_SILU, dt)
        db = _desc_1x1(*b, 0, b[3], 0, b[4], L.ACT_SILU, dt)
        with pytest.raises(L.YcxError, match='unsupported|bad argument'):
            L.check(L.lib.ycx_conv2d_pair(ctypes.byref(da), ctypes.byref(db), t.data_ptr(), t.data_ptr(),
                                          t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr(), t.data_ptr(),
                                          L.stream_handle(device)))
