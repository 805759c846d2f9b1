"""CPU tests of the product's host side: C ABI exports, MJCF loader, host spline utilities.

No GPU needed: model loading, interpolation, spline evaluation and the host reducer are pure
host code in libsspp_hip.so; the library itself must load (it links the HIP runtime).
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from oracle import mjcf_ref
from oracle import oracle as O
from tests.conftest import REFERENCE, ROOT, SCENES

import sspp_amd as S
from sspp_amd import _lib

SCENE_FILES = ["robocrane.xml", "stacking.xml", "planner.xml"]
ORIGINALS = {"robocrane.xml": "mjcf/robocrane/robocrane.xml", "stacking.xml": "mjcf/stacking.xml",
             "planner.xml": "mjcf/planner.xml"}


def test_library_exports_every_declared_symbol():
    declared = _lib.declared_symbols()
    assert len(declared) >= 25
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    lib = _lib.lib()  # binds every signature in _lib.SIGNATURES
    assert set(_lib.SIGNATURES) == set(declared)
    assert lib.sspp_version() >= 10000


def test_library_matches_its_sources():
    """The product library carries the hash of the sources it was built from (sspp_build_id,
    sspp_amd/_stamp.py); a library not rebuilt after an edit would fail here."""
    from sspp_amd import _stamp
    lib = _lib.lib()
    assert lib.sspp_build_id().decode() == _stamp.source_hash()
    assert _lib.build_warning is None


@pytest.mark.parametrize("stamp", ["0123456789abcdef", None])
def test_stale_variant_library_is_refused(tmp_path, stamp):
    """A profiling variant (SSPP_LIB_PATH) built from other sources — or from before the stamp
    existed — is refused at load time with a message naming both revisions, not left to fail
    later on a missing export (a stale libsspp_wgt.so broke a profiling run)."""
    src = tmp_path / "stub.c"
    body = 'int sspp_version(void) { return 10000; }\n'
    if stamp:
        body += 'const char* sspp_build_id(void) { return "%s"; }\n' % stamp
    src.write_text(body)
    so = tmp_path / "libsspp_stub.so"
    subprocess.check_call(["gcc", "-shared", "-fPIC", str(src), "-o", str(so)])
    L = C.CDLL(str(so))
    with pytest.raises(_lib.SsppError, match="stale variant library") as e:
        _lib.check_revision(L, str(so), variant=True)
    assert ("built from sources " + stamp if stamp else "no source stamp") in str(e.value)
    with pytest.warns(RuntimeWarning, match="does not match its sources"):
        assert _lib.check_revision(L, str(so), variant=False)


def test_pybind_module_links_hip_library():
    import glob
    mods = glob.glob(os.path.join(ROOT, "sspp", "_sspp*.so"))
    assert mods, "sspp/_sspp extension not built"
    out = subprocess.check_output(["ldd", mods[0]], text=True)
    assert "libsspp_hip.so" in out and "not found" not in out.split("libsspp_hip.so")[1].split("\n")[0]


@pytest.mark.parametrize("name", SCENE_FILES)
def test_loader_matches_independent_reader(name):
    path = os.path.join(SCENES, name)
    a = S.Model(path).arrays()
    r = mjcf_ref.load(path)
    for k, v in a.items():
        np.testing.assert_array_equal(np.asarray(v), np.asarray(r[k]).reshape(np.asarray(v).shape), err_msg=k)


@pytest.mark.skipif(not os.path.isdir(REFERENCE), reason="reference checkout not present")
@pytest.mark.parametrize("name", SCENE_FILES)
def test_derived_scene_equals_original(name):
    """The committed collision-only scenes carry exactly the original collidable geometry."""
    d = mjcf_ref.load(os.path.join(SCENES, name))
    o = mjcf_ref.load(os.path.join(REFERENCE, ORIGINALS[name]))
    for k in ("body_parent", "body_jnt_type", "body_qpos_adr", "body_pos", "body_quat", "qpos0",
              "exclude"):
        np.testing.assert_array_equal(d[k], o[k], err_msg=k)
    keep = (o["geom_contype"] != 0) | (o["geom_conaffinity"] != 0)
    for k in ("geom_type", "geom_body", "geom_contype", "geom_conaffinity", "geom_size",
              "geom_pos", "geom_quat", "geom_margin"):
        np.testing.assert_array_equal(d[k], np.asarray(o[k])[keep], err_msg=k)
    # product loader on the original file gives the same arrays as the Python reader
    a = S.Model(os.path.join(REFERENCE, ORIGINALS[name])).arrays()
    for k, v in a.items():
        np.testing.assert_array_equal(np.asarray(v), np.asarray(o[k]).reshape(np.asarray(v).shape), err_msg=k)


def test_loader_errors(tmp_path):
    with pytest.raises(S.SsppError, match="cannot open"):
        S.Model(str(tmp_path / "missing.xml"))
    p = tmp_path / "hinge.xml"
    p.write_text('<mujoco><worldbody><body><joint type="hinge"/><geom type="box" size="1 1 1"/>'
                 '</body></worldbody></mujoco>')
    with pytest.raises(S.SsppError, match="unsupported joint"):
        S.Model(str(p))
    p.write_text("<mujoco><worldbody><body></worldbody></mujoco>")
    with pytest.raises(S.SsppError, match="xml"):
        S.Model(str(p))


def test_defaults_and_childclass(tmp_path):
    p = tmp_path / "d.xml"
    p.write_text("""<mujoco><compiler angle="degree"/>
      <default><geom margin="0.5"/>
        <default class="a"><geom type="box" size="1 2 3" contype="3"/>
          <default class="b"><geom pos="0 0 1"/></default></default></default>
      <worldbody>
        <body name="k" childclass="b" euler="0 0 90"><freejoint/>
          <geom name="g1"/><geom name="g2" class="a" pos="1 0 0" margin="0.25"/></body>
        <geom name="w" type="plane" size="0 0 1"/>
      </worldbody></mujoco>""")
    m = S.Model(str(p))
    a = m.arrays()
    r = mjcf_ref.load(str(p))
    for k, v in a.items():
        np.testing.assert_array_equal(np.asarray(v), np.asarray(r[k]).reshape(np.asarray(v).shape), err_msg=k)
    assert list(a["geom_type"]) == [0, 6, 6]   # world geom first, then body geoms
    np.testing.assert_array_equal(a["geom_size"][1], [1, 2, 3])
    np.testing.assert_array_equal(a["geom_pos"][1], [0, 0, 1])   # from class b
    np.testing.assert_array_equal(a["geom_pos"][2], [1, 0, 0])   # explicit
    np.testing.assert_array_equal(a["geom_margin"], [0.5, 0.5, 0.25])
    assert a["geom_contype"][1] == 3
    np.testing.assert_allclose(a["qpos0"][3:], [np.cos(np.pi / 4), 0, 0, np.sin(np.pi / 4)], atol=1e-15)
    np.testing.assert_allclose(m.body_point("k"), [0, 0, 0, np.pi / 2], atol=1e-15)


def test_body_point_matches_reference_scenario():
    m = S.Model(os.path.join(SCENES, "robocrane.xml"))
    np.testing.assert_allclose(m.body_point("block_green/"), [0.5, 0.15, 0.116, np.pi / 2], atol=1e-12)
    m = S.Model(os.path.join(SCENES, "stacking.xml"))
    np.testing.assert_array_equal(m.body_point("block1"), [0.205, 0, 0.1, 0])
    with pytest.raises(S.SsppError, match="not found"):
        m.body_point("nope")


@pytest.mark.parametrize("n,p,D", [(10, 3, 7), (7, 3, 9), (3, 2, 4), (6, 2, 3)])
def test_host_interpolation_matches_oracle(n, p, D):
    rng = np.random.default_rng(n + 100 * p)
    u = np.array([i / (n - 1) for i in range(n)])
    pts = rng.normal(size=(n, D))
    kp, cp = S.interpolate(pts, p, u)
    ko, co = O.interpolate(pts, p, u)
    np.testing.assert_array_equal(kp, ko)
    assert np.abs(cp - co).max() <= 1e-12
    for x in np.linspace(0, 1, 17):
        np.testing.assert_array_equal(S.spline_eval(kp, p, cp, x), O.spline_eval(kp, p, cp, x))


def test_host_best_reduce():
    inf = float("inf")
    assert S.reduce_best([(inf, -1, 0), (2.0, 7, 3), (2.0, 5, 1), (3.0, 1, 9)]) == (2.0, 5, 13)
    assert S.reduce_best([(inf, -1, 0), (inf, -1, 0)]) == (inf, -1, 0)


def test_records_reporting_lost_work_are_refused():
    """A step record whose `reserved` field is non-zero (a split launch's lost-work check found
    survivors it could not finish) is refused by every host consumer: sspp_best_check /
    sspp_best_reduce (SSPP_E_INCOMPLETE) and the Python layer (decode_best, check_records,
    reduce_best).  A clean record passes."""
    ok = np.zeros(4, np.int64)
    ok[:1] = np.array([1.5]).view(np.int64)
    ok[1], ok[2] = 17, 3
    assert S.decode_best(ok) == (1.5, 17, 3)
    bad = ok.copy()
    bad[3] = 2
    with pytest.raises(S.SsppError, match="lost candidates"):
        S.decode_best(bad)
    with pytest.raises(S.SsppError, match="lost candidates"):
        S.check_records(np.stack([ok, bad]))
    S.check_records(np.stack([ok, ok]))
    with pytest.raises(S.SsppError, match="lost candidates"):
        S.reduce_best([(1.5, 17, 3, 0), (2.0, 4, 1, 1)])
    arr = (_lib.Best * 2)()
    arr[1].reserved = 5
    assert _lib.lib().sspp_best_check(arr, 2) == _lib.SSPP_E_INCOMPLETE
    out = _lib.Best()
    assert _lib.lib().sspp_best_reduce(arr, 2, C.byref(out)) == _lib.SSPP_E_INCOMPLETE
    assert "5 lost candidates" in _lib.last_error()
    arr[1].reserved = 0
    assert _lib.lib().sspp_best_check(arr, 2) == 0
