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
