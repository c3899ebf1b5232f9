"""ycx.prepack: folded + packed weights (and the fp8 calibration)
round-trip through a safetensors file; a model that loads them reproduces the
packing model's outputs bit for bit without folding its own parameters."""
import pytest
import torch

from helpers import make_model
from ycx.utils.synth import synthetic_images

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('precision', ['bf16', 'fp8', 'f32'])
def test_prepack_roundtrip_bit_exact(device, tmp_path, precision):
    src, _ = make_model('yolov7-tiny', 1, 0, precision)
    src.to(device)
    x = synthetic_images(2, 3, 320, 320, seed=4).to(device)
    ref = [o.clone() for o in src(x)]
    path = str(tmp_path / f"tiny_{precision}.safetensors")
    meta = src.save_prepacked(path, (320, 320))
    assert meta['precision'] == precision and meta['hw'] == [320, 320]
    dst, _ = make_model('yolov7-tiny', 1, 7, 'bf16')  # other weights: the file must win
    with pytest.raises(ValueError, match='different state_dict'):
        dst.load_prepacked(path, strict=True)
    dst.load_prepacked(path)
    assert dst.precision == precision
    dst.to(device)
    out = dst(x)
    for a, b in zip(out, ref):
        assert torch.equal(a, b)


def test_prepack_rejects_other_plan(device, tmp_path):
    src, _ = make_model('yolov7-tiny', 1, 0, 'bf16')
    src.to(device)
    path = str(tmp_path / "tiny.safetensors")
    src.save_prepacked(path, (320, 320))
    other, _ = make_model('yolov7', 80, 0, 'bf16')
    other.load_prepacked(path)
    other.to(device)
    with pytest.raises(ValueError, match='do not match this plan'):
        other(torch.zeros(1, 3, 320, 320, device=device))


@pytest.mark.parametrize('precision', ['fp16', 'bf16'])
def test_prepack_yolov7_pair_batch_independent(device, tmp_path, precision):
    """the 1x1 pair (tile 55) forms only at bs >= 6 on a 640^2 yolov7, and
    prepack.save packs at bs 1. Tensors are named by conv node, so a file written at bs 1
    binds the right weights to both convs of the pair at bs 6: bit-identical outputs."""
    src, _ = make_model('yolov7', 80, 0, precision)
    src.to(device)
    x = synthetic_images(6, 3, 640, 640, seed=5).to(device)
    ref = [o.clone() for o in src(x)]
    assert any(i['kind'] == 'conv_pair' for i in src.engine_for(x.shape, device, slot=src.EAGER_SLOT).op_info)
    path = str(tmp_path / f"v7_{precision}.safetensors")
    src.save_prepacked(path, (640, 640))
    dst, _ = make_model('yolov7', 80, 7, 'bf16')
    dst.load_prepacked(path)
    dst.to(device)
    out = dst(x)
    for a, b in zip(out, ref):
        assert torch.equal(a, b)


def test_prepack_fp16_overflow_raises(device, tmp_path):
    """an fp16 plan bound to prepacked weights cannot re-plan itself in bf16 (that
    would fold the module's own parameters, not the file's), so a non-finite forward raises
    YcxRangeError instead of returning inf / NaN heads; an in-range prepacked fp16 forward
    returns the packing model's heads bit for bit."""
    from ycx import _lib as L
    src, sd = make_model('yolov7-tiny', 1, 0, 'fp16')
    src.to(device)
    x = synthetic_images(2, 3, 160, 160, seed=9).to(device)
    ref = [o.clone() for o in src(x)]
    ok_path = str(tmp_path / "tiny_fp16.safetensors")
    src.save_prepacked(ok_path, (160, 160))
    dst, _ = make_model('yolov7-tiny', 1, 0, 'bf16')
    dst.load_prepacked(ok_path)
    dst.to(device)
    for a, b in zip(dst(x), ref):
        assert torch.equal(a, b)
    bn = [k for k in sd if k.endswith('.bn.weight')][2]
    big = dict(sd)
    big[bn] = sd[bn] * 1e5  # that layer's activations pass 65504: inf in fp16
    src.load_state_dict(big)
    src.to(device)
    bad_path = str(tmp_path / "tiny_fp16_big.safetensors")
    src.save_prepacked(bad_path, (160, 160))
    bad, _ = make_model('yolov7-tiny', 1, 0, 'bf16')
    bad.load_prepacked(bad_path)
    bad.to(device)
    assert bad.precision == 'fp16'
    with pytest.raises(L.YcxRangeError, match='prepacked'):
        bad(x)
