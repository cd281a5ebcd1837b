"""Oracle pinning against the reference's own code.

The reference's header-only QMC / fast-math layer is compiled in the build
container straight from /root/reference/include with the survey build's flags
(oracle/ref.mk -> oracle/_ref/ref_check; g++ -O3 -ffast-math -DFAST_MATH
-DFAST_TRIG, CMakeLists.txt:239,336-342). No generated header, no stand-ins.
Pinned functions (reference file:line -> oracle/yk_oracle.c, device yk_math.h):

* Halton::setStart / getNext      utilities/mcqmc.h:29-94   hal_setstart / hal_next
* RI_vdC / RI_S / RI_LP           mcqmc.h:100-122           RI_vdC / RI_S / RI_LP
* fnv_32a_buf                     mcqmc.h:155-168           fnv_32a_buf
* fSin / fCos (FAST_TRIG)         mathOptimizations.h:249-280  fSin / fCos
* fExp2                           mathOptimizations.h:100-114  fExp2 (Gauss filter)
* Round2Int / Floor2Int           math_utils.h:60-86        Round2Int / Floor2Int

Three checks:
1. (CPU, build container only) ref_check runs the reference's functions and
   the oracle's side by side over dense / random ranges and reports zero
   mismatches; the exhaustive run (all 2^32 RI_vdC / fnv inputs, every float
   |x| <= 2^16 for fSin / fCos, every float in [-200, 0] for fExp2, every
   float in [-8, 8] for the rounding) is recorded in profiles/r05_ref_check_full.txt.
2. (CPU, everywhere) the oracle against the committed fixtures
   tests/golden/ref_qmc.npz (the reference's outputs, made by
   tests/golden/gen/make_ref_qmc.py), and libyk's host-side fExp2 / fSin
   (film filter tables) through yk_debug_qmc_probe.
3. (GPU) libyk's device functions against the same fixtures through
   yk_debug_qmc_probe.

FP environment. The reference's process computes with MXCSR FTZ+DAZ set:
every object GCC 11 links with -ffast-math (its core library and plugins)
carries crtfastmath's constructor. The oracle and the GPU keep IEEE
denormals. A difference is accepted only when the oracle's own call, repeated
in the reference's environment (orc_set_ftz), gives the reference's bits --
the same operations, differing only in denormal handling. Measured domains
of such differences (profiles/r05_ref_check_full.txt): fSin / fCos inputs
|x| <= 4.1e-38 (the path's arguments are 0 or >= 2*pi*2^-32), fExp2 results
below 2^-126 (x in [-126.5, -126]; the Gauss filter clamps them to 0),
Round2Int / Floor2Int of denormal doubles (never formed by the film's index
math). Every other input is bit-exact.

scrHalton and the Faure tables (yafraycore/scr_halton.h, faure_tables.cc)
include the generated yafray_config.h and are not built here: they stay
pinned only through the survey-build render fixtures.
"""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest

from core_amd import _abi as A
from tests.conftest import ROOT

GOLD = os.path.join(ROOT, "tests", "golden", "ref_qmc.npz")
REF = "/root/reference"
EXE = os.path.join(ROOT, "oracle", "_ref", "ref_check")


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD))


@pytest.fixture(scope="module")
def orc():
    from oracle.oracle import lib
    L = lib()
    for n in ("orc_fcos", "orc_fexp2"):
        getattr(L, n).restype = C.c_float
        getattr(L, n).argtypes = [C.c_float]
    for n in ("orc_round2int", "orc_floor2int"):
        getattr(L, n).restype = C.c_int
        getattr(L, n).argtypes = [C.c_double]
    L.orc_set_ftz.restype = C.c_int
    L.orc_set_ftz.argtypes = [C.c_int]
    return L


def _agree(orc, fn, xs, got_bits, ref_bits, to_bits):
    """got == ref bit for bit, except entries where the oracle's fn, rerun in
    the reference's FTZ+DAZ environment, gives the reference's bits (the
    denormal-flush class). Returns the number of such entries."""
    got_bits, ref_bits = np.asarray(got_bits), np.asarray(ref_bits)
    diff = np.nonzero(got_bits != ref_bits)[0]
    if len(diff) == 0:
        return 0
    prev = orc.orc_set_ftz(1)
    try:
        ftz = to_bits([fn(xs[i]) for i in diff])
    finally:
        orc.orc_set_ftz(prev)
    bad = diff[ftz != ref_bits[diff]]
    assert len(bad) == 0, (len(bad), [xs[i] for i in bad[:4]])
    return len(diff)


def _u32(x):
    return np.asarray(x, np.float32).view(np.uint32)


@pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "include", "utilities")),
                    reason="reference sources absent (GPU box): fixtures only")
def test_oracle_equals_reference_built_here():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "-f", "ref.mk"], check=True)
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    out = subprocess.run([EXE, "check", os.path.join(ROOT, "oracle", "liboracle.so"), "quick"], check=True,
                         capture_output=True, text=True, timeout=300).stdout
    rows = [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    names = {r["fn"] for r in rows}
    assert {"RI_vdC", "RI_S", "RI_LP", "fnv_32a_buf", "fSin", "fCos", "fExp2", "Round2Int", "Floor2Int",
            "Halton(2)", "Halton(3)", "Halton(5)"} <= names
    for r in rows:
        assert r["checked"] > 1000000 and r["mismatches"] == 0, r


def test_oracle_equals_reference_fixtures(gold, orc):
    g = gold
    n = len(g["u_in"])
    ui, ur = g["u_in"].tolist(), g["u_r"].tolist()
    for fn, key in ((orc.orc_ri_vdc, "ri_vdc"), (orc.orc_ri_s, "ri_s"), (orc.orc_ri_lp, "ri_lp")):
        got = np.array([fn(a, b) for a, b in zip(ui, ur)], np.float32)
        assert (_u32(got) == g[key]).all(), key
    assert (np.array([orc.orc_fnv(a) for a in ui], np.uint32) == g["fnv"]).all()
    fx = g["f_in"].tolist()
    for fn, key in ((orc.orc_fsin, "fsin"), (orc.orc_fcos, "fcos")):
        assert _agree(orc, fn, fx, _u32([fn(x) for x in fx]), g[key], _u32) == 0, key
    ex = g["e_in"].tolist()
    nflush = _agree(orc, orc.orc_fexp2, ex, _u32([orc.orc_fexp2(x) for x in ex]), g["fexp2"], _u32)
    # the only flush class in these inputs: fExp2 results below 2^-126
    assert 0 < nflush < 0.01 * len(ex)
    dv = g["d_in"].tolist()
    assert (np.array([orc.orc_round2int(v) for v in dv]) == g["round2int"]).all()
    assert (np.array([orc.orc_floor2int(v) for v in dv]) == g["floor2int"]).all()
    out = np.empty(8, np.float32)
    for base in (2, 3, 5):
        ref = g["hal%d" % base]
        for k, s in enumerate(g["hal_start"].tolist()):
            orc.orc_halton_seq(base, s, 8, out.ctypes.data)
            assert (out.view(np.uint32) == ref[k].view(np.uint32)).all(), (base, s)
    assert n == 65536


def _probe(dev, fn, x, x2=None, out_dtype=np.float32, per=1):
    x = np.ascontiguousarray(x)
    out = np.empty(len(x) * per, out_dtype)
    x2 = None if x2 is None else np.ascontiguousarray(x2, np.uint32)  # kept alive across the call
    in2 = None if x2 is None else x2.ctypes.data
    A.check(A.lib().yk_debug_qmc_probe(dev, fn, x.ctypes.data, in2, len(x), out.ctypes.data))
    return out


def test_host_filter_math_equals_reference(gold, orc, monkeypatch):
    """libyk's host-side fExp2 (Gauss filter table) and fSin (Lanczos table,
    camera bokeh polygon) against the reference's outputs; no GPU needed."""
    monkeypatch.setenv("YK_DEBUG_HOOKS", "1")
    ex = gold["e_in"].tolist()
    got = _probe(None, 11, gold["e_in"])
    assert 0 < _agree(orc, orc.orc_fexp2, ex, got.view(np.uint32), gold["fexp2"], _u32) < 0.01 * len(ex)
    got = _probe(None, 12, gold["f_in"])
    assert (got.view(np.uint32) == gold["fsin"]).all()


def test_probe_refused_without_hooks(gold, monkeypatch):
    monkeypatch.delenv("YK_DEBUG_HOOKS", raising=False)
    x = np.zeros(4, np.float32)
    rc = A.lib().yk_debug_qmc_probe(None, 11, x.ctypes.data, None, 4, x.ctypes.data)
    assert rc == A.YK_ERR_UNSUPPORTED


@pytest.mark.gpu
def test_device_qmc_equals_reference(gold, gpu_device, orc, monkeypatch):
    """The device's QMC, FAST_TRIG and film rounding functions (the ones every
    camera sample, BSDF direction and film splat goes through) against the
    reference's own outputs, bit for bit."""
    monkeypatch.setenv("YK_DEBUG_HOOKS", "1")
    g = gold
    d = gpu_device._p
    for fn, key in ((0, "ri_vdc"), (1, "ri_s"), (2, "ri_lp")):
        got = _probe(d, fn, g["u_in"], g["u_r"])
        assert (got.view(np.uint32) == g[key]).all(), key
    assert (_probe(d, 3, g["u_in"], out_dtype=np.uint32) == g["fnv"]).all()
    fx = g["f_in"].tolist()
    assert _agree(orc, orc.orc_fsin, fx, _probe(d, 4, g["f_in"]).view(np.uint32), g["fsin"], _u32) == 0
    assert _agree(orc, orc.orc_fcos, fx, _probe(d, 5, g["f_in"]).view(np.uint32), g["fcos"], _u32) == 0
    for fn, base in ((6, 2), (7, 3), (8, 5)):
        got = _probe(d, fn, g["hal_start"], per=8).reshape(-1, 8)
        assert (got.view(np.uint32) == g["hal%d" % base].view(np.uint32)).all(), base
    assert (_probe(d, 9, g["d_in"], out_dtype=np.int32) == g["round2int"]).all()
    assert (_probe(d, 10, g["d_in"], out_dtype=np.int32) == g["floor2int"]).all()
