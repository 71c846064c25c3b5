"""Index-scan timing: compress a smooth field on the GPU (variable rate), then
decompress it with and without the encoder's block index.

  python tools/scan_bench.py [--n 512] [--dtype f64] [--mode precision --param 32] [--reps 3]

Prints one line per run: scan ms, passes, decode ms (kernel), stream bytes.
ZFP_HIP_SCAN_SEG_BITS overrides the segment length.
"""
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "zfp-par_amd")]

import torch  # noqa: E402,F401  (one HIP runtime)
from capi import ZfpCAPI  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--dims", type=int, default=3)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--mode", default="precision")
    ap.add_argument("--param", type=float, default=32)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lib", default=os.path.join(REPO, "zfp-par_amd", "lib", "libzfp.so"))
    a = ap.parse_args()
    dtype = np.float64 if a.dtype == "f64" else np.float32
    api = ZfpCAPI(a.lib)
    api.enable_index()
    n = a.n
    shape = (n,) * a.dims
    g = np.meshgrid(*[np.arange(n, dtype=np.float64)] * a.dims, indexing="ij", sparse=True)
    v = np.sin(0.05 * g[-1]) * np.cos(0.03 * g[-2]) + 0.5 * np.sin(0.02 * g[-3] + 0.01 * g[-1] * g[-2] / n)
    if a.dims == 4:
        v = v + 0.25 * np.cos(0.04 * g[0])
    arr = np.ascontiguousarray(v.astype(dtype))
    param = None if a.mode == "reversible" else (int(a.param) if a.mode == "precision" else a.param)
    data = api.compress(arr, a.mode, param)
    idx = api.last_index
    out = np.empty_like(arr)
    for r in range(a.reps):
        t0 = time.perf_counter()
        _, n1 = api.decompress(data, shape, dtype, a.mode, param, out=out, index=idx)
        t1 = time.perf_counter()
        k = np.zeros(2)
        import ctypes
        km, tm = ctypes.c_double(), ctypes.c_double()
        api.lib.zfp_hip_last_timing(ctypes.byref(km), ctypes.byref(tm))
        ref = out.copy() if r == 0 else ref
        t2 = time.perf_counter()
        _, n2 = api.decompress(data, shape, dtype, a.mode, param, out=out)
        t3 = time.perf_counter()
        scan = api.last_scan()
        same = out.tobytes() == ref.tobytes()
        if a.mode == "reversible":  # lossless: both decodes must give the field back
            same = "%s (index decode lossless %s, scan decode lossless %s)" % (
                same, ref.tobytes() == arr.tobytes(), out.tobytes() == arr.tobytes())
        print("rep %d: stream %d B, with index %.1f ms (kernel %.3f ms), without %.1f ms: scan %.3f ms in %d passes, "
              "identical %s" % (r, len(data), 1e3 * (t1 - t0), km.value, 1e3 * (t3 - t2), scan[0], scan[1], same),
              flush=True)
    api.lib.zfp_hip_index_free(idx)


if __name__ == "__main__":
    main()
