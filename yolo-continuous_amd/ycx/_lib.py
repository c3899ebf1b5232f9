"""ctypes binding of libycx_hip.so (the C ABI declared in include/ycx.h).

The library is the only compute path of this package: there is no CPU or
PyTorch-op fallback. If the shared object is missing or does not match the
header, importing this module raises immediately (fail loudly).

torch is imported first so that the HIP runtime (libamdhip64.so.7) already
loaded by PyTorch is the one libycx_hip.so binds to (same SONAME): device
pointers and hipStream_t handles from torch are then valid inside the library.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must be loaded before the HIP library, see above)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("YCX_LIB", os.path.join(_HERE, "libycx_hip.so"))

ABI_VERSION = 9

# ---- enums (ycx.h) ----
YCX_OK, YCX_ERR_BAD_ARG, YCX_ERR_UNSUPPORTED, YCX_ERR_LAUNCH, YCX_ERR_CAPACITY = 0, 1, 2, 3, 4
DT_BF16, DT_F32, DT_FP8, DT_F16 = 0, 1, 2, 3
ACT_NONE, ACT_SILU, ACT_LEAKY, ACT_SILU_PS = 0, 1, 2, 3
SILU_PS_K = -1.4426950408889634  # -log2(e): the pre-scale of YCX_ACT_SILU_PS weights and bias (ycx.h)
OUT_NHWC, OUT_NCHW_F32, OUT_NHWC_UP2 = 0, 1, 2
OP_CONV, OP_STEM, OP_POOL, OP_COPY, OP_STEM2, OP_HEAD, OP_CONV_PAIR = 1, 2, 3, 4, 5, 6, 7

_i32 = ctypes.c_int32


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, _i32) for n in (
        "n", "h", "w", "cin", "in_c_off", "in_c_stride",
        "ho", "wo", "cout", "cout_pad", "out_c_off", "out_c_stride",
        "kh", "kw", "stride", "pad", "act")] + [("leaky_slope", ctypes.c_float)] + [
        (n, _i32) for n in ("dtype", "out_layout", "res_c_off", "res_c_stride", "tile")] + [
        ("out_scale", ctypes.c_float), ("res_scale", ctypes.c_float), ("in_pool", _i32), ("k_split", _i32)]


class PoolDesc(ctypes.Structure):
    _fields_ = [(n, _i32) for n in (
        "n", "h", "w", "c", "in_c_off", "in_c_stride",
        "ho", "wo", "out_c_off", "out_c_stride", "k", "stride", "pad", "dtype", "levels")]


class CopyDesc(ctypes.Structure):
    _fields_ = [(n, _i32) for n in (
        "n", "h", "w", "c", "in_c_off", "in_c_stride",
        "out_c_off", "out_c_stride", "scale", "dtype", "out_layout")] + [("dequant", ctypes.c_float)]


class DecodeDesc(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("n", "h", "w", "na", "no", "rows_total", "row_off")] + [
        ("anchors_scaled", ctypes.c_float * 16)]


class Cand(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in ("x1", "y1", "x2", "y2", "obj", "cls_conf")] + [
        ("cls", _i32), ("row", _i32)]


class FilterDesc(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("n", "rows", "no", "nc")] + [
        ("conf_thres", ctypes.c_float), ("write_xyxy", _i32)]


class DecodeFilterDesc(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("n", "nl", "na", "no", "nc")] + [
        ("h", _i32 * 4), ("w", _i32 * 4), ("row_off", _i32 * 4), ("rows_total", _i32),
        ("anchors_scaled", (ctypes.c_float * 16) * 4), ("conf_thres", ctypes.c_float)]


class NmsDesc(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("n", "rows_total", "nc", "max_det")] + [
        ("iou_thres", ctypes.c_double)]


class HeadDesc(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("na", "no", "nc", "rows_total", "row_off")] + [
        ("conf_thres", ctypes.c_float), ("anchors_scaled", ctypes.c_float * 16)]


class _HeadOp(ctypes.Structure):
    _fields_ = [("conv", ConvDesc), ("head", HeadDesc)]


class _OpUnion(ctypes.Union):
    _fields_ = [("conv", ConvDesc), ("pool", PoolDesc), ("copy", CopyDesc), ("pair", ConvDesc * 2),
                ("head", _HeadOp)]


class Op(ctypes.Structure):
    _fields_ = [("kind", _i32), ("pad_", _i32), ("d", _OpUnion),
                ("in_", ctypes.c_void_p), ("weight", ctypes.c_void_p), ("bias", ctypes.c_void_p),
                ("out", ctypes.c_void_p), ("residual", ctypes.c_void_p),
                ("weight2", ctypes.c_void_p), ("bias2", ctypes.c_void_p),
                ("cand", ctypes.c_void_p), ("cand_rows", ctypes.c_void_p), ("cand_counts", ctypes.c_void_p),
                ("status", ctypes.c_void_p), ("out2", ctypes.c_void_p), ("workspace", ctypes.c_void_p)]


class LetterboxDesc(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("h0", "w0", "c", "src_row_stride", "out_h", "out_w", "new_h", "new_w", "top",
                                    "left", "pad")]


class CorrectDesc(ctypes.Structure):
    _fields_ = [(n, _i32) for n in ("n", "max_det", "input_h", "input_w", "letterbox")]


_STRUCTS = [ConvDesc, PoolDesc, CopyDesc, DecodeDesc, Cand, FilterDesc, DecodeFilterDesc, NmsDesc, Op, LetterboxDesc,
            CorrectDesc, HeadDesc]

# (name, restype, argtypes) — every symbol declared in include/ycx.h.
_VP = ctypes.c_void_p
_SIGS = [
    ("ycx_abi_version", ctypes.c_int, []),
    ("ycx_struct_size", ctypes.c_size_t, [_i32]),
    ("ycx_strerror", ctypes.c_char_p, [_i32]),
    ("ycx_conv_tile_name", ctypes.c_char_p, [_i32]),
    ("ycx_conv_pick_tile", _i32, [ctypes.POINTER(ConvDesc)]),
    ("ycx_conv_tile_of", _i32, [_i32, _i32, _i32, _i32]),
    ("ycx_conv2d", _i32, [ctypes.POINTER(ConvDesc), _VP, _VP, _VP, _VP, _VP, _VP]),
    ("ycx_conv_workspace_size", ctypes.c_size_t, [ctypes.POINTER(ConvDesc)]),
    ("ycx_conv2d_ws", _i32, [ctypes.POINTER(ConvDesc), _VP, _VP, _VP, _VP, _VP, _VP, ctypes.c_size_t, _VP]),
    ("ycx_conv_pick_ksplit", _i32, [ctypes.POINTER(ConvDesc)]),
    ("ycx_conv2d_head", _i32, [ctypes.POINTER(ConvDesc), ctypes.POINTER(HeadDesc), _VP, _VP, _VP, _VP, _VP, _VP,
                               _VP, _VP, _VP]),
    ("ycx_stem_conv", _i32, [ctypes.POINTER(ConvDesc), _VP, _VP, _VP, _VP, _VP]),
    ("ycx_idetect_decode", _i32, [ctypes.POINTER(DecodeDesc), ctypes.c_float, _VP, _VP, _VP, _VP]),
    ("ycx_letterbox", _i32, [ctypes.POINTER(LetterboxDesc), _VP, _VP, _VP]),
    ("ycx_letterbox_batch", _i32, [ctypes.POINTER(LetterboxDesc), _i32, ctypes.c_int64, _VP, _VP, _VP]),
    ("ycx_correct_boxes", _i32, [ctypes.POINTER(CorrectDesc), _VP, _VP, _VP, _VP]),
    ("ycx_stem_conv2", _i32, [ctypes.POINTER(ConvDesc), ctypes.POINTER(ConvDesc), _VP, _VP, _VP, _VP, _VP, _VP,
                              _VP]),
    ("ycx_conv2d_pair", _i32, [ctypes.POINTER(ConvDesc), ctypes.POINTER(ConvDesc), _VP, _VP, _VP, _VP, _VP, _VP,
                               _VP, _VP]),
    ("ycx_maxpool", _i32, [ctypes.POINTER(PoolDesc), _VP, _VP, _VP]),
    ("ycx_copy_channels", _i32, [ctypes.POINTER(CopyDesc), _VP, _VP, _VP]),
    ("ycx_quantize_fp8", _i32, [_VP, _VP, ctypes.c_int64, ctypes.c_float, _VP]),
    ("ycx_decode", _i32, [ctypes.POINTER(DecodeDesc), _VP, _VP, _VP]),
    ("ycx_filter_decoded", _i32, [ctypes.POINTER(FilterDesc), _VP, _VP, _VP, _VP, _VP]),
    ("ycx_decode_filter", _i32, [ctypes.POINTER(DecodeFilterDesc), ctypes.POINTER(_VP), _VP, _VP, _VP, _VP]),
    ("ycx_check_sigmoid_monotone", _i32, [_VP, _VP]),
    ("ycx_nms_workspace_size", ctypes.c_size_t, [ctypes.POINTER(NmsDesc)]),
    ("ycx_sort_nms", _i32, [ctypes.POINTER(NmsDesc), _VP, _VP, _VP, _VP, ctypes.c_size_t, _VP, _VP, _VP, _VP]),
    ("ycx_run_ops", _i32, [ctypes.POINTER(Op), _i32, _VP, ctypes.POINTER(_VP)]),
    ("ycx_set_trace", _i32, [_i32]),
    ("ycx_debug_bounds", _i32, [ctypes.POINTER(ctypes.c_uint32), _i32]),
    ("ycx_graph_capture", _i32, [ctypes.POINTER(Op), _i32, _VP, ctypes.POINTER(_VP)]),
    ("ycx_graph_launch", _i32, [_VP, _VP]),
    ("ycx_graph_destroy", _i32, [_VP]),
]
SYMBOLS = [s[0] for s in _SIGS]


class YcxError(RuntimeError):
    """Raised for a nonzero ycx_status (mirrors the reference's exception-based errors)."""

    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"{what}: {lib.ycx_strerror(status).decode()} (status {status})" if what
                         else lib.ycx_strerror(status).decode())


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"ycx: HIP library not found at {LIB_PATH}; build it with `python -c 'import __graft_entry__ as g; "
            f"g.build()'` (or `make -C yolo-continuous_amd/csrc`). There is no CPU fallback.")
    handle = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, res, args in _SIGS:
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    if handle.ycx_abi_version() != ABI_VERSION:
        raise ImportError(f"ycx: ABI version mismatch ({handle.ycx_abi_version()} != {ABI_VERSION})")
    for i, st in enumerate(_STRUCTS):
        got = handle.ycx_struct_size(i)
        if got != ctypes.sizeof(st):
            raise ImportError(f"ycx: struct {st.__name__} is {got} bytes in C, {ctypes.sizeof(st)} in ctypes")
    return handle


lib = _load()
# YCX_ROCTX=1: one roctx range per op of every eager ycx_run_ops (rocprofv3 --marker-trace);
# Detector then runs eagerly, since a HIP-graph replay has no host loop to mark
TRACE = bool(os.environ.get("YCX_ROCTX"))
if TRACE and lib.ycx_set_trace(1) != 0:
    import warnings
    warnings.warn("ycx: YCX_ROCTX set but librocprofiler-sdk-roctx could not be loaded; tracing is off")
    TRACE = False


HEAD_NONFINITE = 1  # ycx_conv2d_head status flag (include/ycx.h)


class YcxRangeError(FloatingPointError):
    """A 16-bit plan produced inf / NaN head logits: some activation left the
    element type's range (fp16: |a| > 65504). The reference computes in fp32
    (nets/yolo.py:143-153); rebuild the model with precision='bf16' or 'f32'."""


def check(status: int, what: str = "") -> None:
    if status != YCX_OK:
        raise YcxError(status, what)


def dedicated_stream(device, priority: int = 0, slot: int | None = None):
    """A non-blocking HIP stream of our own (hipStreamCreateWithPriority), wrapped
    as a torch ExternalStream: unlike torch.cuda.Stream() it is not one of the
    pool streams that every other component (the RCCL communicator included)
    is handed round-robin, so no other work can share it. Never destroyed, so
    ``slot`` streams are kept per (device, priority, slot) and handed out again:
    detectors built one after another (bench.py's legs) reuse the same few
    streams instead of piling up more streams than the GPU has hardware queues
    (GPU_MAX_HW_QUEUES, 4), which slowed every later leg (r06: the pipelined leg
    after the fp16 leg ran 8.7 instead of 5.2 ms per step)."""
    import torch
    dev = torch.device(device)
    key = (dev.index if dev.index is not None else torch.cuda.current_device(), priority, slot)
    if slot is not None and key in _SLOT_STREAMS:
        return torch.cuda.ExternalStream(_SLOT_STREAMS[key], device=device)
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch already loaded (same soname)
    s = ctypes.c_void_p()
    with torch.cuda.device(device):
        rc = hip.hipStreamCreateWithPriority(ctypes.byref(s), ctypes.c_uint(1), ctypes.c_int(priority))
    if rc != 0:
        raise RuntimeError(f"ycx: hipStreamCreateWithPriority failed ({rc})")
    _STREAMS.append(s.value)
    if slot is not None:
        _SLOT_STREAMS[key] = s.value
    return torch.cuda.ExternalStream(s.value, device=device)


_SLOT_STREAMS = {}
_STREAMS = []


def ptr(t) -> int | None:
    """Device pointer of a tensor (None passes a null pointer)."""
    return None if t is None else t.data_ptr()


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
