"""Kernel-side bounds-check build (`YCX_DEBUG_BOUNDS`): the G1 nets and
yolov7 / yolov7-tiny in every precision, plus the fused Detector path, run on
libycx_hip_dbg.so, whose conv epilogues test every global store against the output
extent the descriptor implies. No store may fall outside it."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DBG = os.path.join(REPO, "yolo-continuous_amd", "ycx", "libycx_hip_dbg.so")


def test_no_out_of_bounds_stores():
    if not os.path.exists(DBG):
        pytest.skip("libycx_hip_dbg.so not built (opt-in: YCX_BUILD_DEBUG=1 build()): make -C yolo-continuous_amd/csrc debug")
    env = dict(os.environ, YCX_LIB=DBG)
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "probes", "bounds_run.py")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    print(res)
    assert res["runs"] > 40 and res["violations"] == 0, res
