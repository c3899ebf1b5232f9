"""Host-side AddressSanitizer + UBSan run of libycx_hip's host code: the
library's sources rebuilt with -fsanitize=address,undefined on the host side
(`make -C yolo-continuous_amd/csrc asan`) and driven by tests/native/abi_check.c through
every host path that runs before a launch (struct sizes, tile heuristic, XCD tile-map
bijection, NMS workspace sizing, descriptor validation of bad arguments). CPU only."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "yolo-continuous_amd", "csrc")


def test_host_code_under_asan_ubsan():
    subprocess.run(["make", "-j8", "-C", CSRC, "asan"], check=True, capture_output=True, timeout=900)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([os.path.join(CSRC, "build", "asan", "abi_check")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0 and "abi_check ok" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
