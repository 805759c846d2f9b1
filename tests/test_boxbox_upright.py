"""k_tsp's upright box-box specialisation (sspd::box_box_deep_count_up and its contact-polygon
clip sspd::bb_clip_count_up, used by k_tsp<..., UP> when every box-box pair of a
TaskSpacePlanner job is upright for its yaw-only mover) returns the deep-contact count of the
generic sspd::box_box_deep_count bit for bit: it only drops products with the exact zeros of
upright rotations from the same fma chains (z-face and side-face reference faces).  Checked on the host build
of sspp_device.h over random upright pairs (stacked, side by side, anywhere within reach;
identity, yawed and z-flipped boxes, both argument orders), whose counts span 0..8."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="needs hipcc")
def test_upright_box_box_deep_count_identical(tmp_path):
    exe = str(tmp_path / "check_up")
    hipcc = HIPCC if os.path.exists(HIPCC) else "hipcc"
    subprocess.check_call([hipcc, "-std=c++17", "-O2", "-ffp-contract=off",
                           "-I" + os.path.join(ROOT, "sspp_amd", "csrc"),
                           os.path.join(HERE, "boxbox", "check_up.cpp"), "-o", exe])
    r = subprocess.run([exe, "1000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    counts = [int(x) for x in r.stdout.split("counts")[1].split()]
    assert "mismatches 0" in r.stdout
    assert all(c > 0 for c in counts[:9]), counts  # every count 0..8 occurs
