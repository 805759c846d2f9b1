"""the host C++ (MJCF loader + xml_lite, spline fitting, C-ABI model helpers) and the
oracle's C restatement (scene build, FK, every narrowphase, both scorers) run clean under
AddressSanitizer + UndefinedBehaviorSanitizer (tests/sanitize/, host code only)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_under_asan_ubsan():
    d = os.path.join(HERE, "sanitize")
    subprocess.check_call(["make", "-s", "-C", d], stdout=subprocess.DEVNULL)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", OMP_NUM_THREADS="2")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([os.path.join(d, "build", "san_main"), os.path.join(ROOT, "sspp_amd", "scenes")],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
    assert "sanitize driver done" in r.stdout
