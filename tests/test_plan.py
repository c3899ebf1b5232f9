"""Host-side (CPU) checks of the builder, the lowering passes and the weight folding."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import ANCHORS, make_model
from ycx.engine import Plan, fold_bn, fold_repconv
from ycx.nets.common import RepConv
from ycx.nets.yolo import Model, parse_model
from ycx.utils.helper_io import cvt_cfg


def test_parse_model_matches_reference_bookkeeping(manifest):
    m = Model(cvt_cfg('yolov7'), ANCHORS, 80)
    assert len(m.model) == 106 and len(m.save) == 62          # SURVEY.md §3.2 [measured]
    assert len(m.state_dict()) == 558
    assert sum(p.numel() for p in m.parameters()) == 37620125  # SURVEY.md §6 [measured]
    t = Model(cvt_cfg('yolov7-tiny'), ANCHORS, 1)
    assert len(t.model) == 78 and len(t.save) == 51
    assert sum(p.numel() for p in t.parameters()) == 6014038
    assert manifest['g2']['yolov7_160']['n_keys'] == 558 and manifest['g2']['tiny_640']['n_keys'] == 336


def test_safe_parser_rejects_out_of_scope_and_unknown():
    d = {'depth_multiple': 1.0, 'width_multiple': 1.0, 'backbone': [[-1, 1, 'GhostConv', [32, 3, 1]]], 'head': []}
    with pytest.raises(NotImplementedError, match='out of scope'):
        parse_model(d, [3], ANCHORS, 1)
    d['backbone'][0][2] = '__import__("os")'
    with pytest.raises(ValueError, match='unknown module'):
        parse_model(d, [3], ANCHORS, 1)


@pytest.mark.parametrize('net,nc,gflop', [('yolov7', 80, 104.5110784), ('yolov7-tiny', 1, 13.021184)])
def test_plan_flops_and_passes(net, nc, gflop):
    m = Model(cvt_cfg(net), ANCHORS, nc)
    plan = Plan(m, (1, 3, 640, 640))
    assert abs(plan.conv_flops / 1e9 - gflop) < 1e-6  # SURVEY.md §8(d) folded FLOP/img
    c = plan.counts()
    assert c.get('up', 0) == 0, "both nearest-x2 upsamples should be fused into their producer convs"
    assert c.get('copy', 0) == 0, "every concat input should alias its slice"
    assert len(plan.out_vals) == 3 and [v.h for v in plan.out_vals] == [20, 40, 80]


def test_plan_yolov7_layout():
    plan = Plan(Model(cvt_cfg('yolov7'), ANCHORS, 80), (2, 3, 640, 640))
    c = plan.counts()
    assert c['stem'] == 1 and c['conv'] + c['stem'] == 92  # 95 convs minus the 3 folded RepConv 1x1 branches
    assert c['merged'] == 8  # ELAN cv1/cv2 sibling 1x1 pairs stacked into one conv each
    assert c['pool'] == 8  # 5 MP (k2s2) + the SPPCSPC 5/9/13 set as a 3-deep k5 cascade
    assert all(nd.p['k'] in (2, 5) for nd in plan.graph.nodes if nd.kind == 'pool')


def test_pool_fusion_pass_finds_the_mp_blocks():
    """The engine's MP-pool fusion pass (host logic, no GPU): every yolov7 k2 s2 pool feeds
    exactly one 1x1 / s1 conv and is fused into it (bf16, and fp8 where cin % 128 == 0: all five);
    in yolov7-tiny only pools read by a lone 1x1 fuse; f32 plans and fuse_pool=False keep every pool."""
    from ycx import _lib as L
    from ycx.engine import Engine

    def pairs(net, nc, dt=L.DT_BF16, fuse=True):
        plan = Plan(Model(cvt_cfg(net), ANCHORS, nc), (2, 3, 640, 640))
        eng = Engine.__new__(Engine)  # the pass reads the plan graph and the plan dtype only
        eng.graph, eng.dt, eng.fuse_pool = plan.graph, dt, fuse
        return eng._pool_convs()

    got = pairs('yolov7', 80)
    assert len(got) == 5
    for pool in got.values():
        p = pool.p
        assert (p['k'], p['s'], p['p']) == (2, 2, 0) and pool.inputs[0].h == 2 * pool.out.h
        (conv,) = pool.out.consumers
        assert conv.kind == 'conv' and (conv.p['k'], conv.p['s'], conv.p['p']) == (1, 1, 0)
    f8 = pairs('yolov7', 80, dt=L.DT_FP8)
    assert len(f8) == 5 and all(int(pool.out.consumers[0].p['w'].shape[1]) % 128 == 0 for pool in f8.values())
    assert pairs('yolov7', 80, dt=L.DT_F32) == {}
    assert pairs('yolov7', 80, fuse=False) == {}
    for pool in pairs('yolov7-tiny', 1).values():
        assert pool.out.consumers[0].p['k'] == 1


def test_fold_bn_and_repconv_exact():
    torch.manual_seed(0)
    for c1, c2, s in ((16, 32, 1), (32, 32, 1), (16, 16, 2)):
        m = RepConv(c1, c2, 3, s).eval().double()
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.uniform_(-0.5, 0.5)
                mod.running_var.uniform_(0.5, 1.5)
                mod.weight.data.uniform_(0.5, 1.5)
                mod.bias.data.uniform_(-0.5, 0.5)
        x = torch.randn(2, c1, 9, 9, dtype=torch.float64)
        bn = lambda b, v: F.batch_norm(v, b.running_mean, b.running_var, b.weight, b.bias, False, 0.0, b.eps)
        ref = bn(m.rbr_dense[1], F.conv2d(x, m.rbr_dense[0].weight, None, s, 1)) + \
            bn(m.rbr_1x1[1], F.conv2d(x, m.rbr_1x1[0].weight, None, s, 0))
        if m.rbr_identity is not None:
            ref = ref + bn(m.rbr_identity, x)
        w, b = fold_repconv(m)
        torch.testing.assert_close(F.conv2d(x, w, b, s, 1), ref, rtol=1e-12, atol=1e-12)
    conv = torch.nn.Conv2d(8, 16, 3, 1, 1, bias=False).double()
    bnm = torch.nn.BatchNorm2d(16).double().eval()
    bnm.running_var.uniform_(0.5, 2.0)
    bnm.running_mean.uniform_(-1, 1)
    x = torch.randn(1, 8, 7, 7, dtype=torch.float64)
    w, b = fold_bn(conv.weight, bnm)
    torch.testing.assert_close(F.conv2d(x, w, b, 1, 1), bnm(conv(x)), rtol=1e-12, atol=1e-12)


def test_state_dict_roundtrip_and_invalidation():
    m, sd = make_model('yolov7-tiny', 1, 0)
    m._engines['sentinel'] = type('E', (), {'close': lambda self: None})()
    m.load_state_dict(sd)
    assert m._engines == {}, "load_state_dict must drop compiled plans (packed weights)"
    for k, v in m.state_dict().items():
        assert torch.equal(v, sd[k])


def test_fp8_weight_packing():
    """pack_fp8_weights: per-channel power-of-two scales, exact dequantisation of
    the e4m3 codes, rows in [kh][kw][cin] order zero-padded to 128-byte K steps."""
    from ycx.engine import pack_fp8_weights
    g = torch.Generator().manual_seed(0)
    w = torch.randn(64, 32, 3, 3, generator=g, dtype=torch.float64) * torch.logspace(-3, 1, 64,
                                                                                       dtype=torch.float64).reshape(
        -1, 1, 1, 1)
    w[5] = 0.0
    q, sw = pack_fp8_weights(w)
    assert q.dtype == torch.float8_e4m3fn and q.shape == (64, 384)  # 288 -> 3 x 128
    assert torch.all(q[:, 288:].float() == 0)
    assert torch.all(torch.log2(sw) == torch.round(torch.log2(sw))) and sw[5] == 1.0
    deq = q[:, :288].double() / sw.reshape(-1, 1)
    ref = w.permute(0, 2, 3, 1).reshape(64, -1)
    amax = q[:, :288].float().abs().amax(1)
    nz = torch.arange(64) != 5
    assert torch.all((amax[nz] >= 224) & (amax[nz] <= 448))
    # e4m3: 3 mantissa bits -> relative rounding error <= 2^-4 for normal values
    big = ref.abs() * sw.reshape(-1, 1) >= 2 ** -6
    assert torch.all(((deq - ref).abs() <= ref.abs() * 2 ** -4 + 1e-30)[big])


def test_prepack_file_format_checks(tmp_path):
    """ycx.prepack.load refuses files that are not ycx prepack files (CPU: format only)."""
    from safetensors.torch import save_file
    from ycx import prepack
    p = str(tmp_path / "plain.safetensors")
    save_file({"a": torch.zeros(2)}, p)
    with pytest.raises(ValueError, match="not a ycx prepack file"):
        prepack.load(p)
    save_file({"p0": torch.zeros(2)}, p, metadata={"ycx": '{"format": "other"}'})
    with pytest.raises(ValueError, match="format"):
        prepack.load(p)
    m, _ = make_model('yolov7-tiny', 1, 0)
    h = prepack.state_dict_sha256(m)
    assert h == prepack.state_dict_sha256(m) and len(h) == 64


def test_unfused_upsample_writes_its_concat_slice(manifest):
    """An upsample that cannot fuse (its producer is a pool) and lands in the
    middle of a concat buffer keeps that channel offset (the copy
    used offset 0 and overwrote the first concat input)."""
    e = manifest['g1']['upsample_offset']
    m = Model(e['cfg'], ANCHORS, e['nc'])
    plan = Plan(m, tuple(e['shape']))
    ups = [nd for nd in plan.graph.nodes if nd.kind == 'up']
    assert len(ups) == 1 and ups[0].out.coff == 32 and ups[0].out.buf.c == 160
    assert plan.counts().get('up') == 1


def test_iauxdetect_lowers_main_heads_only(manifest):
    """IAuxDetect eval (nets/iaux_detect.py:27-49): the plan's outputs are the
    three main heads; the aux convs m2 and the layers feeding only them are
    dead (their maps are discarded in eval) and never launched."""
    e = manifest['g1']['iauxdetect']
    m = Model(e['cfg'], ANCHORS, e['nc'])
    assert len(m.state_dict()) == e['n_keys']  # same schema as the reference (m, m2, ia, im, anchors)
    plan = Plan(m, tuple(e['shape']))
    convs = [nd for nd in plan.graph.nodes if nd.kind in ('conv', 'stem')]
    assert len(convs) == 4 + 3  # stem + 3 backbone convs + 3 main heads (aux layers 4-6 and m2 dropped)
    assert [v.c for v in plan.out_vals] == [3 * (e['nc'] + 5)] * 3
    assert [(v.h, v.w) for v in plan.out_vals] == [(12, 12), (6, 6), (3, 3)]


def test_cascade_fits_mirrors_the_kernel_limit():
    """ycx_maxpool levels > 1: two planes of a 16-byte-multiple channel slice in 64 KB."""
    from ycx.engine import cascade_fits
    assert cascade_fits(20, 20, 512, 2) and cascade_fits(40, 40, 256, 2)     # yolov7 at 640 / 1280
    assert cascade_fits(45, 45, 512, 2) and not cascade_fits(46, 46, 512, 2)  # 2025 / 2116 pixels, bf16
    assert not cascade_fits(40, 60, 512, 2)                                   # 1280x1920 input
    assert cascade_fits(45, 45, 512, 1) and not cascade_fits(46, 46, 512, 1)  # e4m3: a 16-channel slice
    assert not cascade_fits(8, 8, 4, 2)                                       # slice below 16 bytes
