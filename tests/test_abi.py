"""The C-ABI library loads and exports every symbol include/ycx.h declares
(no compute calls: runs without a GPU)."""
import ctypes
import os
import re

import pytest

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "ycx.h")


def header_symbols():
    src = open(HDR).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(ycx_[a-z0-9_]+)\s*\(', src)))


def test_header_declares_the_boundary():
    syms = header_symbols()
    for s in ('ycx_conv2d', 'ycx_stem_conv', 'ycx_maxpool', 'ycx_copy_channels', 'ycx_decode', 'ycx_filter_decoded',
              'ycx_decode_filter', 'ycx_sort_nms', 'ycx_run_ops', 'ycx_strerror', 'ycx_abi_version', 'ycx_stem_conv2'):
        assert s in syms


def test_library_exports_every_header_symbol():
    from ycx import _lib
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for s in header_symbols():
        assert hasattr(raw, s), f"{s} declared in ycx.h but not exported"
        assert s in _lib.SYMBOLS, f"{s} not bound in ycx/_lib.py"


def test_abi_metadata_without_gpu():
    from ycx import _lib
    assert _lib.lib.ycx_abi_version() == _lib.ABI_VERSION == 9
    for i, st in enumerate(_lib._STRUCTS):
        assert _lib.lib.ycx_struct_size(i) == ctypes.sizeof(st)
    assert _lib.lib.ycx_struct_size(99) == 0
    assert b"bad argument" in _lib.lib.ycx_strerror(1)
    assert _lib.lib.ycx_conv_tile_name(1) == b"bf16_co128_px128_k64"
    # tile ids are positions in the library's table: retired ids keep placeholders
    assert _lib.lib.ycx_conv_tile_name(16) == b"glds_co128_px128_k64_s2"
    assert _lib.lib.ycx_conv_tile_name(50) == b"halo3x3s2_wsr_co128"
    assert _lib.lib.ycx_conv_tile_name(55) == b"wres1x1_pair"
    assert _lib.lib.ycx_conv_tile_name(56) == b"glds_co64_px128_k64_s3"
    assert _lib.lib.ycx_conv_tile_name(57) == b"retired_wsp_co128_px128_k64_ns4"
    assert _lib.lib.ycx_conv_tile_name(58) == b"invalid"
    # argument validation happens before any device call
    assert _lib.lib.ycx_conv2d(None, None, None, None, None, None, None) == _lib.YCX_ERR_BAD_ARG
    assert _lib.lib.ycx_sort_nms(None, None, None, None, None, 0, None, None, None, None) == _lib.YCX_ERR_BAD_ARG


def test_tile_picker():
    from ycx import _lib
    d = _lib.ConvDesc()
    d.n, d.ho, d.wo, d.cin, d.cout_pad, d.dtype = 32, 160, 160, 64, 64, _lib.DT_BF16
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 15   # 512-thread 2-stage LDS-DMA co64 x px256
    d.h, d.w, d.kh, d.kw, d.stride, d.pad = 160, 160, 3, 3, 1, 1
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 23   # 3x3 s1 64->64: weight-stationary halo
    d.res_c_stride = 64
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 19   # ... with a residual: LDS halo tile
    d.res_c_stride = 0
    d.cout_pad = 128
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 20
    d.cout_pad, d.kh, d.kw, d.pad = 64, 1, 1, 0
    d.cin = 32
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 17  # two taps per K step
    d.ho = d.wo = 20
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 6
    d.ho = d.wo = 160
    d.cout_pad = 32
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 5
    d.cin, d.cout_pad, d.ho, d.wo = 512, 512, 20, 20
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 16
    d.h = d.w = d.ho = d.wo = 160
    d.cin, d.cout_pad, d.kh, d.kw, d.stride, d.pad = 256, 256, 1, 1, 1, 0
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 22  # weight-resident pointwise
    d.res_c_stride = 256
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 16  # ... which stores no residual
    d.res_c_stride = 0
    d.cout_pad, d.h, d.w, d.ho, d.wo = 512, 40, 40, 40, 40
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 22  # >= 4 pixel tiles per persistent block (r06)
    d.h = d.w = d.ho = d.wo = 20
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 16  # too few tiles per persistent block
    d.h = d.w = d.ho = d.wo = 40
    d.kh, d.kw, d.pad = 3, 3, 1
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 48  # 40-wide 3x3, 1280 band workgroups
    d.cout_pad = 256
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 16  # 640: too few for the band tile
    d.h = d.w = d.ho = d.wo = 20
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 16  # 20^2 x bs 32: 200 workgroups (r06)
    d.n = 4
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 18  # 26: co64 x px128 below 64
    d.n = 32
    d.dtype = _lib.DT_F32
    assert _lib.lib.ycx_conv_pick_tile(ctypes.byref(d)) == 8


def test_missing_library_fails_loudly(tmp_path):
    import subprocess
    import sys
    env = dict(os.environ, YCX_LIB=str(tmp_path / "nope.so"))
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "yolo-continuous_amd")
    r = subprocess.run([sys.executable, "-c", "import ycx._lib"], cwd=pkg, env=env, capture_output=True, text=True)
    assert r.returncode != 0 and "no CPU fallback" in r.stderr


@pytest.mark.parametrize('gc', [0, 1, 2, 4, 8])
def test_conv_tile_map_is_a_bijection(gc):
    """The XCD region map of the LDS-DMA conv tiles (ycx_tile_of) visits every
    (channel tile, pixel tile) exactly once for any grid, including pixel-tile
    counts that do not split evenly over the XCD regions (host-side call, no GPU)."""
    from ycx import _lib as L
    for n_ct in (1, 2, 3, 4, 8, 16):
        for n_pt in (1, 3, 7, 25, 100, 101, 800):
            nwg = n_ct * n_pt
            seen = set()
            for b in range(nwg):
                v = int(L.lib.ycx_conv_tile_of(b, nwg, n_ct, gc))
                assert v >= 0
                ct, pt = divmod(v, 65536)
                assert 0 <= ct < n_ct and 0 <= pt < n_pt
                seen.add((ct, pt))
            assert len(seen) == nwg, (gc, n_ct, n_pt)
    assert L.lib.ycx_conv_tile_of(0, 10, 3, 2) == -1   # nwg not a multiple of n_ct
