"""GPU-native compressed arrays (include/zfp/hip/array.hpp) against the reference's.

The reference's zfp::array3 (include/zfp/array3.hpp, its fixed-rate block store
internal/array/store3.hpp:96-118 and block cache cache3.hpp) is compiled here
from its own headers over the reference library (oracle/Makefile `ref`:
oracle/_ref/array_check_ref); tests/arrays/array_check.cpp runs the same
sequence on it and on zfp::hip::array3 (oracle/build/array_check: set() and
get() as one GPU call each, element access through a cache of decoded block
lines, write-back of modified blocks in runs).  Bar: identical compressed
bytes after construction and after scattered and row-wise element writes,
identical get() arrays, identical sums of every element read through the cache.
"""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OURS = os.path.join(REPO, "oracle", "build", "array_check")
REF = os.path.join(REPO, "oracle", "_ref", "array_check_ref")
DROPIN = os.path.join(REPO, "oracle", "_ref", "array_check_dropin")


def _field(shape, dtype):
    i = np.indices(shape).astype(np.float64)
    n = shape[0]
    return (np.sin(0.05 * i[2]) * np.cos(0.03 * i[1]) + 0.5 * np.sin(0.02 * i[0] + 0.01 * i[2] * i[1] / n)).astype(dtype)


@pytest.mark.parametrize("dtype,shape,rate", [(np.float32, (129, 129, 129), 8), (np.float32, (129, 129, 129), 16),
                                              (np.float64, (37, 41, 43), 12), (np.float32, (5, 1030, 9), 4)])
def test_array3_matches_reference_array3(tmp_path, dtype, shape, rate):
    if not (os.path.exists(OURS) and os.path.exists(REF)):
        pytest.skip("array checkers not built (make -C oracle ref arrays)")
    a = _field(shape, dtype)
    src = str(tmp_path / "in.raw")
    a.tofile(src)
    nz, ny, nx = shape
    t = "d" if dtype == np.float64 else "f"
    outs = {}
    for name, exe in (("ours", OURS), ("ref", REF)):
        pre = str(tmp_path / name)
        r = subprocess.run([exe, t, str(nx), str(ny), str(nz), str(rate), src, pre], capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        outs[name] = (pre, r.stdout.strip())
    assert outs["ours"][1] == outs["ref"][1]  # element sums read through the caches, store size
    for part in ("set.z", "set.raw", "elem.z", "elem.raw"):
        mine = open(outs["ours"][0] + "." + part, "rb").read()
        theirs = open(outs["ref"][0] + "." + part, "rb").read()
        assert len(mine) == len(theirs) and mine == theirs, part


def _run(exe, t, shape, rate, src, pre):
    nz, ny, nx = shape
    r = subprocess.run([exe, t, str(nx), str(ny), str(nz), str(rate), src, pre], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout.strip()


@pytest.mark.parametrize("dtype,shape,rate", [(np.float32, (33, 34, 35), 8), (np.float64, (37, 41, 43), 12)])
def test_reference_array3_runs_unchanged_on_this_library(tmp_path, dtype, shape, rate):
    """code built on the per-block C API links and runs
    unchanged.  The reference's own zfp::array3 (its headers, compiled here)
    linked against this libzfp.so -- every block through zfp_encode_block_* /
    zfp_decode_block_* on the GPU, one round trip each -- gives the same
    compressed bytes, decoded values and element reads as the same program on
    the reference library (include/zfp/array3.hpp, internal/array/store3.hpp:96-118)."""
    if not (os.path.exists(DROPIN) and os.path.exists(REF)):
        pytest.skip("array checkers not built (make -C oracle ref)")
    a = _field(shape, dtype)
    src = str(tmp_path / "in.raw")
    a.tofile(src)
    t = "d" if dtype == np.float64 else "f"
    got = _run(DROPIN, t, shape, rate, src, str(tmp_path / "dropin"))
    want = _run(REF, t, shape, rate, src, str(tmp_path / "ref"))
    assert got == want
    for part in ("set.z", "set.raw", "elem.z", "elem.raw"):
        assert open(str(tmp_path / "dropin") + "." + part, "rb").read() == \
            open(str(tmp_path / "ref") + "." + part, "rb").read(), part


CFP_REF = os.path.join(REPO, "oracle", "_ref", "cfp_check_ref")
CFP_DROPIN = os.path.join(REPO, "oracle", "_ref", "cfp_check_dropin")


@pytest.mark.parametrize("shape,rate", [((33, 34, 35), 8), ((20, 9, 41), 16)])
def test_reference_cfp_runs_unchanged_on_this_library(tmp_path, shape, rate):
    """The reference's cfp (the C bindings of its compressed arrays,
    cfp/cfp.cpp compiled unchanged) driven from C over this libzfp.so writes the
    same compressed bytes and values as over the reference library: array3f
    construction, get_array, element get/set through the cache, flush
    (cfp/cfparray3f.cpp, include/zfp/internal/cfp/array3f.h)."""
    if not (os.path.exists(CFP_DROPIN) and os.path.exists(CFP_REF)):
        pytest.skip("cfp checkers not built (make -C oracle ref)")
    a = _field(shape, np.float32)
    src = str(tmp_path / "in.raw")
    a.tofile(src)
    outs = {}
    for name, exe in (("dropin", CFP_DROPIN), ("ref", CFP_REF)):
        nz, ny, nx = shape
        r = subprocess.run([exe, str(nx), str(ny), str(nz), str(rate), src, str(tmp_path / name)],
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
        outs[name] = r.stdout.strip()
    assert outs["dropin"] == outs["ref"]
    for part in ("set.z", "set.raw", "elem.z", "elem.raw"):
        assert open(str(tmp_path / "dropin") + "." + part, "rb").read() == \
            open(str(tmp_path / "ref") + "." + part, "rb").read(), part
