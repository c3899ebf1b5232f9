"""Pin the oracle: CPU restatement vs golden vectors made by the reference itself.

The fixtures (tests/golden/make_golden.py) come from importing
xin-pu/yolo-continuous in the build container; these tests prove the oracle
reproduces them, so the GPU parity tests can use the oracle as the checker at
any size.
"""
import numpy as np
import pytest
import torch

from helpers import ANCHORS, MASK, arr_hash, g1_case, g3_heads, make_model, sd_hash
from oracle import ref_forward, ref_post
from ycx.utils.helper_io import cvt_cfg
from ycx.utils.synth import synthetic_images

G1_NAMES = ['conv_k3s1_cin32', 'conv_k3s2_cin32', 'conv_k1_cin64', 'conv_leaky', 'stem_s2_leaky', 'pools',
            'upsample_concat', 'upsample_shared', 'sppcspc', 'repconv', 'csp_blocks', 'detect', 'idetect',
            'upsample_offset', 'iauxdetect']


def _close(a, b):
    # Same ATen ops in the same order on the same CPU: identical up to oneDNN
    # thread/ISA-dependent reassociation (observed bit-exact in the build container).
    np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-6 * max(1.0, float(np.abs(b).max())))


@pytest.mark.parametrize('name', G1_NAMES)
def test_oracle_g1(manifest, g1, name):
    m, sd, x, e = g1_case(manifest, name)
    assert len(sd) == e['n_keys']
    assert sd_hash(sd) == e['sd_hash'], "synthetic weights / state_dict schema drifted from the fixture"
    fwd = ref_forward.build(e['cfg'], ANCHORS, e['nc'], sd)
    out = fwd(x)
    outs = out if isinstance(out, list) else [out]
    if name == 'iauxdetect':  # the fixture is the reference's eval output [z, x0, x1, x2], strides set
        z, xs = ref_post.idetect_eval(outs, ANCHORS, 3, e['nc'] + 5, e['strides'])
        outs = [z] + xs
    assert len(outs) == e['n_out']
    for j, o in enumerate(outs):
        gold = g1[f'{name}/{j}']
        if name == 'idetect':  # oracle returns NCHW maps; the fixture is the reference's (bs,na,ny,nx,no) view
            bs, _, ny, nx = o.shape
            o = o.view(bs, 3, -1, ny, nx).permute(0, 1, 3, 4, 2)
        _close(o.numpy(), gold)


@pytest.mark.parametrize('name', ['yolov7_160', 'tiny_640'])
def test_oracle_g2(manifest, g2, name):
    e = manifest['g2'][name]
    m, sd = make_model(e['net'], e['nc'], e['w_seed'])
    assert len(sd) == e['n_keys'] and sd_hash(sd) == e['sd_hash']
    x = synthetic_images(*e['shape'], seed=e['img_seed'])
    outs = ref_forward.build(cvt_cfg(e['net']), ANCHORS, e['nc'], sd)(x)
    for j, o in enumerate(outs):
        _close(o.numpy(), g2[f'{name}/{j}'])


@pytest.mark.parametrize('name', ['coco80_bs4', 'nc1_bs2', 'nc3_dense'])
def test_oracle_g3(manifest, g3, name):
    e = manifest['g3'][name]
    heads = g3_heads(e)
    assert arr_hash([h.numpy() for h in heads]) == e['heads_hash']
    anchors = np.asarray(ANCHORS).reshape(-1, 2)
    dec = torch.cat(ref_post.decode_box(heads, anchors, MASK, e['nc'], (e['size'], e['size'])), 1)
    assert arr_hash([dec.numpy()]) == e['decoded_hash'], "decode_box restatement is not bit-exact"
    for b in range(e['bs']):
        rows = g3[f'{name}/pass_rows/{b}']
        np.testing.assert_array_equal(dec[b, rows].numpy(), g3[f'{name}/pass_vals/{b}'])
    keep, _ = ref_post.nms_keep_rows(dec.clone(), e['nc'], e['conf'], e['iou'])
    final = ref_post.non_max_suppression(dec.clone(), e['nc'], (e['size'], e['size']),
                                         np.array(e['image_shape']), True, e['conf'], e['iou'])
    for b in range(e['bs']):
        np.testing.assert_array_equal(keep[b].numpy(), g3[f'{name}/keep_rows/{b}'])
        np.testing.assert_array_equal(final[b], g3[f'{name}/final/{b}'])


def test_nms_restatement_semantics():
    """torchvision.ops.nms contract: score-descending keep, stable ties, '>' threshold."""
    boxes = torch.tensor([[0, 0, 10, 10], [0, 0, 10, 10], [1, 1, 11, 11], [50, 50, 60, 60]], dtype=torch.float32)
    scores = torch.tensor([0.9, 0.9, 0.8, 0.95])
    assert ref_post.nms(boxes, scores, 0.5).tolist() == [3, 0]
    # IoU of boxes 0 and 2 is 81/119 = 0.68: equal-to-threshold is kept, strictly above is suppressed
    iou02 = float(np.float32(81) / (np.float32(100) + np.float32(100) - np.float32(81)))
    assert ref_post.nms(boxes[[0, 2]], scores[[0, 2]], iou02).tolist() == [0, 1]
    assert ref_post.nms(boxes[[0, 2]], scores[[0, 2]], iou02 - 1e-6).tolist() == [0]
    assert ref_post.nms(boxes[:0], scores[:0], 0.5).numel() == 0


def test_letterbox_geometry_restatement():
    """letter_box.py:27-60 geometry on the SURVEY §8(d) C1 image size (512 x 773 -> 640)."""
    from oracle import ref_letterbox
    rw, rh, top, left, oh, ow = ref_letterbox.letterbox_geometry(512, 773, (640, 640))
    assert (rw, rh, top, left, oh, ow) == (640, 424, 108, 0, 640, 640)
    img = np.full((512, 773, 3), 7, dtype=np.uint8)
    t = ref_letterbox.letterbox_tensor(img)
    assert t.shape == (3, 640, 640) and t.dtype == np.float32
    assert t[0, 0, 0] == np.float32(114) / np.float32(255) and t[0, 320, 320] == np.float32(7) / np.float32(255)


def test_oracle_idetect_eval(manifest):
    """IDetect eval (decoded z) vs the reference's own eval output, strides set
    on its module as the build does (make_golden.make_idetect_eval)."""
    import os
    e = manifest['g4']['idetect_eval']
    g4 = np.load(os.path.join(os.path.dirname(__file__), 'golden', 'g4_idetect.npz'))
    m, sd = make_model(e['cfg'], e['nc'], e['w_seed'], 'f32')
    assert sd_hash(sd) == e['sd_hash']
    x = synthetic_images(*e['shape'], seed=e['img_seed'])
    outs = ref_forward.build(e['cfg'], ANCHORS, e['nc'], sd)(x)
    z, xs = ref_post.idetect_eval(outs, ANCHORS, 3, e['nc'] + 5, e['strides'])
    _close(z.numpy(), g4['idetect_eval/z'])
    assert len(xs) == e['n_x']
    for j, t in enumerate(xs):
        _close(t.numpy(), g4[f'idetect_eval/x{j}'])


@pytest.mark.parametrize('seed', [0, 1, 2])
def test_oracle_c_nms_equals_numpy(seed):
    """oracle/nms_ref.c (the fast restatement bench.py's CPU baseline and the
    big-batch tests run) == the numpy restatement, on dense overlapping boxes
    with exact score ties, zero-area boxes and duplicates."""
    from oracle.ref_post import _clib, nms, nms_numpy
    assert _clib() is not None, "oracle C library not built (python -c 'import __graft_entry__ as g; g.build()')"
    g = torch.Generator().manual_seed(seed)
    n = 3000
    xy = torch.rand(n, 2, generator=g) * 50
    wh = torch.rand(n, 2, generator=g) * 20
    boxes = torch.cat([xy, xy + wh], 1)
    boxes[::97, 2:] = boxes[::97, :2]             # zero-area boxes
    boxes[1::53] = boxes[0::53][:boxes[1::53].shape[0]]  # exact duplicates
    scores = (torch.rand(n, generator=g) * 64).floor() / 64  # many exact ties
    if seed == 2:  # non-finite inputs: numpy's NaN propagation and NaN-last argsort
        boxes[5::211, 0] = float('nan')
        boxes[7::307, 3] = float('inf')
        boxes[11::401] = float('-inf')
        scores[13::97] = float('nan')
        scores[17::89] = float('inf')
    for thr in (0.3, 0.45, 0.7):
        a = nms(boxes, scores, thr)
        with np.errstate(invalid='ignore'):
            b = nms_numpy(boxes, scores, thr)
        assert torch.equal(a, b), (thr, len(a), len(b))
    assert len(nms(boxes[:0], scores[:0], 0.5)) == 0
