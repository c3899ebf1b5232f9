"""Prepacked weights on disk.

A reference checkpoint is a 558-key ``state_dict`` (``train.py:116`` saves it,
``detect.py:175`` loads it). Lowering it for the HIP path folds BN, RepConv and
ImplicitA/M in float64 (``nets/common.py:488-529``) and packs every conv as
``[cout_pad][kh][kw][cin]`` bf16 / fp32, or per-channel-scaled e4m3 rows plus the
dequantisation vector for fp8 (``ycx/engine.py``). This module stores that
result, with the fp8 calibration record it depends on, in one safetensors file
so a serving process skips the host-side folding and calibration.

The file holds one plan (precision, input H x W): tensors ``p<2i>, p<2i+1>`` =
the packed weights and bias of the i-th conv / stem node of the lowered graph
(named by node, not by packing order, so the fusions that vary with the batch
size -- the 1x1 pair -- cannot permute them) and ``metadata['ycx']`` = JSON {format, precision, hw,
n_tensors, fp8_amax, state_dict_sha256}. The batch size is free: packed weights
do not depend on it. Loading checks every tensor's shape and dtype against the
plan it is bound to, and refuses a file written for another plan.

CLI (run where the GPU is; fp8 calibration runs a bf16 forward):

    python -m ycx.prepack --cfg yolov7 --nc 80 --weights best.pt --size 640 \\
        --precision fp8 --out yolov7_640_fp8.safetensors [--calib images.pt]
"""
from __future__ import annotations

import argparse
import hashlib
import json

import torch

FORMAT = "ycx-prepack-4"  # 3 (r05): tensors named by conv node (2i, 2i+1), independent of which convs fuse;
#                            4 (r06): SiLU convs of 16-bit / fp8 plans packed pre-scaled by -log2(e) (YCX_ACT_SILU_PS)


def state_dict_sha256(model):
    h = hashlib.sha256()
    for k, v in sorted(model.state_dict().items()):
        h.update(k.encode())
        h.update(v.detach().cpu().contiguous().reshape(-1).view(torch.uint8).numpy().tobytes())
    return h.hexdigest()


def save(model, path, hw, precision=None, device="cuda"):
    """Pack ``model`` for input size ``hw`` = (H, W) and write ``path``."""
    from safetensors.torch import save_file
    precision = precision or model.precision
    old = model.precision
    model.set_precision(precision)
    try:
        eng = model.engine_for((1, model.image_chan, int(hw[0]), int(hw[1])), device)
        tensors = {k: t.detach().cpu().contiguous() for k, t in eng.packed.items()}
        meta = dict(format=FORMAT, precision=precision, hw=[int(hw[0]), int(hw[1])], n_tensors=len(tensors),
                    fp8_amax=model._fp8_amax.get((int(hw[0]), int(hw[1]))) if precision == "fp8" else None,
                    state_dict_sha256=state_dict_sha256(model))
    finally:
        model.set_precision(old)
    save_file(tensors, path, metadata={"ycx": json.dumps(meta)})
    return meta


def load(path):
    """-> (meta dict, {name: CPU tensor}); raises on a file of another format."""
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        md = f.metadata() or {}
        if "ycx" not in md:
            raise ValueError(f"ycx: {path} is not a ycx prepack file")
        meta = json.loads(md["ycx"])
        if meta.get("format") != FORMAT:
            raise ValueError(f"ycx: {path} has format {meta.get('format')!r}, expected {FORMAT!r}")
        tensors = {k: f.get_tensor(k) for k in f.keys()}
    if len(tensors) != meta["n_tensors"]:
        raise ValueError(f"ycx: {path} holds {len(tensors)} tensors, metadata says {meta['n_tensors']}")
    return meta, tensors


def main(argv=None):
    from .nets.yolo import Model
    from .utils.helper_io import cvt_cfg
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--cfg", required=True, help="model YAML (path or name under ycx/cfg)")
    ap.add_argument("--nc", type=int, required=True)
    ap.add_argument("--anchors", default="12,16,19,36,40,28,36,75,76,55,72,146,142,110,192,243,459,401")
    ap.add_argument("--weights", help="state_dict file (torch.save of Model.state_dict(); loaded weights_only)")
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--precision", default="bf16", choices=["fp16", "bf16", "f32", "fp8"])
    ap.add_argument("--calib", help="fp8: a tensor file of calibration images [N, 3, H, W] fp32 in [0, 1]")
    ap.add_argument("--out", required=True)
    args = ap.parse_args(argv)
    a = [int(v) for v in args.anchors.split(",")]
    anchors = [a[0:6], a[6:12], a[12:18]]
    model = Model(cvt_cfg(args.cfg), anchors, args.nc).eval()
    if args.weights:
        model.load_state_dict(torch.load(args.weights, map_location="cpu", weights_only=True))
    model.to("cuda")
    if args.precision == "fp8":
        images = torch.load(args.calib, weights_only=True) if args.calib else None
        model.calibrate_fp8(images, device="cuda", hw=(args.size, args.size))
    meta = save(model, args.out, (args.size, args.size), args.precision)
    print(json.dumps({k: v for k, v in meta.items() if k != "fp8_amax"}))


if __name__ == "__main__":
    main()
