#!/usr/bin/env python3
"""Host-resident zfp_parallel throughput (SURVEY 8 f2 / BASELINE C4 host case):
zfp_p over a shared host array, nparts chunks, a thread per chunk, every chunk
call on the GPU (host->device copy, kernel, device->host copy).

usage: python tools/zfp_par_bench.py [--shape 512 1024 1024] [--rate 8] [--nparts 8] [--threads 8] [--reps 3]
Prints compress / decompress GB/s of uncompressed data, host to host.
"""
import argparse
import os
import sys
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "zfp-par_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, nargs="+", default=[512, 1024, 1024])
    ap.add_argument("--rate", type=float, default=8)
    ap.add_argument("--nparts", type=int, default=8)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from zfpy._zfp_par import zfp_p
    zp = zfp_p(tuple(a.shape), "float32", nparts=a.nparts)
    arr = zp.get_numpy_array()
    nz, ny, nx = a.shape
    x = np.arange(nx, dtype=np.float64)
    y = np.arange(ny, dtype=np.float64)
    base = np.sin(0.05 * x)[None, :] * np.cos(0.03 * y)[:, None]
    xy = 0.01 * x[None, :] * y[:, None] / nx
    for k in range(nz):
        arr[k] = (base + 0.5 * np.sin(0.02 * k + xy)).astype(np.float32)
    ref = arr.copy()
    gb = arr.nbytes / 1e9
    tc, td = [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        data = zp.compress(nthreads=a.threads, rate=a.rate)
        tc.append(time.perf_counter() - t0)
        arr[:] = 0
        t0 = time.perf_counter()
        zp.decompress(nthreads=a.threads)
        td.append(time.perf_counter() - t0)
    err = float(np.abs(arr - ref).max())
    nbytes = sum(len(d) for d in data)
    print("zfp_parallel shape %s rate %g nparts %d threads %d chunks %d: stream %d B, compress %.2f GB/s (best %.3f s), "
          "decompress %.2f GB/s (best %.3f s), max abs err %.3g"
          % (a.shape, a.rate, a.nparts, a.threads, len(data), nbytes, gb / min(tc), min(tc), gb / min(td), min(td), err))


if __name__ == "__main__":
    main()
