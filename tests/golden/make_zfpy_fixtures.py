"""Generate tests/golden/zfpy_chunks.json from the REFERENCE's own Python zfpy.

Run only in the build container (needs /root/reference and oracle/_ref built by
`make -C oracle ref`); the GPU box never sees the reference.  The reference's
Cython module python/zfpy_c.pyx is translated with Cython and compiled with gcc
into a temporary directory outside the repository (not with the reference's
build system), linked against oracle/_ref/libzfp_ref.so (the reference library
compiled from its own sources), and imported together with the reference's
zfpy/__init__.py and zfpy/_zfp_par.py.  For each case the script records, per
chunk stream of zfp_parallel.compress(): byte length, SHA-256 and the first 16
bytes (the 96-bit whole-field header and the first block bits); and the SHA-256
of the array after zfp_parallel.decompress().  Inputs are regenerated from
`case_field` (seeded, exact in binary floating point) by the tests.

usage: python tests/golden/make_zfpy_fixtures.py
"""
import hashlib
import json
import os
import shutil
import subprocess
import sys
import sysconfig
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
REF_LIB_DIR = os.path.join(REPO, "oracle", "_ref")

# (name, shape, dtype, nparts, mode, param)
CASES = [
    ("64^3 f32 rate 8 nparts 4", (64, 64, 64), "float32", 4, "rate", 8),
    ("64^3 f32 rate 8 nparts 8", (64, 64, 64), "float32", 8, "rate", 8),
    ("64^3 f32 precision 16 nparts 8", (64, 64, 64), "float32", 8, "precision", 16),
    ("64^3 f32 tolerance 1e-3 nparts 8", (64, 64, 64), "float32", 8, "tolerance", 1e-3),
    ("64^3 f64 precision 32 nparts 4", (64, 64, 64), "float64", 4, "precision", 32),
    ("129^3 f32 rate 8 nparts 8", (129, 129, 129), "float32", 8, "rate", 8),
    ("16^4 f32 reversible nparts 4", (16, 16, 16, 16), "float32", 4, "reversible", None),
    # 1D/2D and integer fields
    ("96x128 i32 rate 12 nparts 4", (96, 128), "int32", 4, "rate", 12),
    ("40x72 f64 reversible nparts 2", (40, 72), "float64", 2, "reversible", None),
    ("4000 f32 precision 14 nparts 2", (4000,), "float32", 2, "precision", 14),
    ("24^3 i64 precision 40 nparts 2", (24, 24, 24), "int64", 2, "precision", 40),
    ("12^4 i32 reversible nparts 2", (12, 12, 12, 12), "int32", 2, "reversible", None),
]


def case_field(shape, dtype, seed=2024):
    """Deterministic input: a smooth part on a 1/64 grid plus seeded integer noise / 256."""
    rng = np.random.default_rng(seed)
    g = np.indices(shape, dtype=np.int64)
    y = g[-2] if len(shape) > 1 else 0
    smooth = (g[-1] * 3 + y * 5 - g[0] * 2) % 97 - 48  # integers
    noise = rng.integers(-128, 128, size=shape)
    if np.dtype(dtype).kind == "i":  # integer fields: the same pattern, scaled
        return (smooth * 4096 + noise).astype(dtype)
    return (smooth.astype(np.float64) / 64.0 + noise.astype(np.float64) / 256.0).astype(dtype)


def mode_kwargs(mode, param):
    if mode == "rate":
        return {"rate": param}
    if mode == "precision":
        return {"precision": param}
    if mode == "tolerance":
        return {"tolerance": param}
    return {}


def build_reference_zfpy(tmp):
    pkg = os.path.join(tmp, "pkg")
    os.makedirs(os.path.join(pkg, "zfpy"))
    csrc = os.path.join(tmp, "zfpy_c.c")
    subprocess.check_call([sys.executable, "-m", "cython", "-3", "-I", os.path.join(REF, "python"),
                           os.path.join(REF, "python", "zfpy_c.pyx"), "-o", csrc])
    ext = sysconfig.get_config_var("EXT_SUFFIX")
    so = os.path.join(tmp, "zfpy_c" + ext)
    # compress_numpy_portion sizes its buffer with zfp_stream_maximum_size_chunk,
    # which leaves no room for the 96 header bits it then writes:
    # the heap overflow aborts the process at free().  Pad the module's mallocs
    # so the run completes; the bytes the reference writes are unchanged.
    pad = os.path.join(tmp, "pad_malloc.h")
    with open(pad, "w") as f:
        f.write("#include <stdlib.h>\nstatic inline void* zfpyref_malloc(size_t n) { return malloc(n + 256); }\n"
                "#define malloc zfpyref_malloc\n")
    subprocess.check_call(["gcc", "-O2", "-shared", "-fPIC", "-w", "-include", pad, "-I" + os.path.join(REF, "include"),
                           "-I" + np.get_include(), "-I" + sysconfig.get_paths()["include"], csrc, "-o", so,
                           "-L" + REF_LIB_DIR, "-l:libzfp_ref.so", "-Wl,-rpath," + REF_LIB_DIR])
    shutil.copy(so, os.path.join(pkg, "zfpy_c" + ext))           # `from zfpy_c import` (_zfp_par.py:5)
    shutil.copy(so, os.path.join(pkg, "zfpy", "zfpy_c" + ext))   # `from .zfpy_c import` (__init__.py:1)
    for f in ("__init__.py", "_zfp_par.py"):
        shutil.copy(os.path.join(REF, "zfpy", f), os.path.join(pkg, "zfpy", f))
    return pkg


def main():
    if not os.path.exists(os.path.join(REF_LIB_DIR, "libzfp_ref.so")):
        sys.exit("build the reference library first: make -C oracle ref")
    tmp = tempfile.mkdtemp(prefix="zfpyref_")
    try:
        sys.path.insert(0, build_reference_zfpy(tmp))
        import zfpy
        out = []
        for name, shape, dtype, nparts, mode, param in CASES:
            zp = zfpy.zfp_parallel(shape, dtype, nparts=nparts)  # the reference keys dtype by name
            zp.get_numpy_array()[...] = case_field(shape, dtype)
            zp.compress(nthreads=4, **mode_kwargs(mode, param))
            streams = [bytes(s) for s in zp._compress_data]
            zp.get_numpy_array()[...] = 0
            zp.decompress(nthreads=4)
            back = np.ascontiguousarray(zp.get_numpy_array())
            note = None
            if len(shape) == 1:
                # The reference's contiguous 1D decompress ignores the chunk box
                # (src/template/decompress.c:3-15): every chunk decodes its stream
                # from element 0 over the whole field, so zfp_parallel.decompress()
                # of a 1D field races and its result changes from run to run.  The
                # chunk boxes are block aligned and blocks are independent, so the
                # expected array is the reference's whole-field round trip.
                back = np.ascontiguousarray(zfpy.decompress_numpy(
                    zfpy.compress_numpy(case_field(shape, dtype), **mode_kwargs(mode, param))))
                note = "whole-field zfpy round trip (reference 1D chunk decompress is racy)"
            out.append({
                "name": name, "shape": list(shape), "dtype": dtype, "nparts": nparts, "mode": mode, "param": param,
                "nchunks": len(streams),
                "chunks": [{"len": len(s), "sha256": hashlib.sha256(s).hexdigest(), "head": s[:16].hex()}
                           for s in streams],
                "decompressed_sha256": hashlib.sha256(back.tobytes()).hexdigest(),
                "decompressed_note": note,
                "input_sha256": hashlib.sha256(case_field(shape, dtype).tobytes()).hexdigest(),
            })
            print("%-36s %d chunks" % (name, len(streams)))
        with open(os.path.join(HERE, "zfpy_chunks.json"), "w") as f:
            json.dump({"generator": "tests/golden/make_zfpy_fixtures.py (reference zfpy, SEP-software/zfp-par)",
                       "cases": out}, f, indent=1)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
