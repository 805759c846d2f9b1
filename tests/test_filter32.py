"""k_sspp_c2f's FP32-filtered scan (sspp_amd/csrc/sspp_filter.h): FP32 may only settle what the
FP64 narrowphase settles the same way.  The host build of the filter runs against the FP64
functions the kernel falls back to (pair_near, sat_box_box, col_plane_box) on random box-box
and plane-box configurations placed 1e-8..1e-1 m from touching, through the kernel's input
pipeline (a 4-term spline evaluation of position and quaternion from control points, doubles vs
their float copies; v_rsq_f32's 1-ulp error emulated): every certain FP32 decision must equal
FP64's in both argument orders, and FP32's SAT separations must stay far inside eps."""
import os
import re
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="needs hipcc")
def test_filter_never_contradicts_fp64(tmp_path):
    exe = str(tmp_path / "check_filter")
    hipcc = HIPCC if os.path.exists(HIPCC) else "hipcc"
    subprocess.check_call([hipcc, "-std=c++17", "-O2", "-ffp-contract=off",
                           "-I" + os.path.join(ROOT, "sspp_amd", "csrc"),
                           os.path.join(HERE, "filter32", "check_filter.cpp"), "-o", exe])
    r = subprocess.run([exe, "300000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
    m = re.search(r"tested (\d+) certain-hit (\d+) certain-no (\d+)", r.stdout)
    tested, hit, no = (int(x) for x in m.groups())
    assert tested > 250000 and hit > 20000 and no > 20000  # both certificates exercised
    err = float(re.search(r"per metre of scale ([0-9.e+-]+)", r.stdout).group(1))
    assert err < 2e-4 / 50, r.stdout  # FP32's error is far inside the certified margin
