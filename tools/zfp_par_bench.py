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


def mode(a):
    return {"precision": a.precision} if a.precision >= 0 else {"rate": a.rate}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", type=int, nargs="+", default=[512, 1024, 1024])
    ap.add_argument("--rate", type=float, default=8)
    ap.add_argument("--precision", type=int, default=-1, help="fixed precision instead of the rate (variable-rate chunks)")
    ap.add_argument("--nparts", type=int, default=8)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--profile", action="store_true", help="per-chunk time split of the last compress")
    ap.add_argument("--loop", type=int, default=0,
                    help="also time N back-to-back compress calls as a caller writes them (data = zp.compress()), "
                         "with the release of the previous streams timed apart")
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
    data = None
    for _ in range(a.reps):
        data = None  # the previous streams are freed before, not inside, the timed call
        t0 = time.perf_counter()
        data = zp.compress(nthreads=a.threads, **mode(a))
        tc.append(time.perf_counter() - t0)
        arr[:] = 0
        t0 = time.perf_counter()
        zp.decompress(nthreads=a.threads)
        td.append(time.perf_counter() - t0)
    if a.loop:
        loop_compress(zp, a)
    if a.profile:
        profile_compress(zp, a)
    err = float(np.abs(arr - ref).max())
    nbytes = sum(len(d) for d in data)
    import resource
    rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 1024.0
    print("zfp_parallel shape %s %s nparts %d threads %d chunks %d: stream %d B, compress %.2f GB/s (best %.3f s), "
          "decompress %.2f GB/s (best %.3f s), max abs err %.3g, peak RSS %.0f MB (field %.0f MB)"
          % (a.shape, mode(a), a.nparts, a.threads, len(data), nbytes, gb / min(tc), min(tc), gb / min(td), min(td),
             err, rss, arr.nbytes / 2**20))


def loop_compress(zp, a):
    """Back-to-back compress calls: each call's wall time, and (separately) the
    time to free the previous call's streams, which the caller's next
    assignment would otherwise do inside the next call."""
    try:
        thp = open("/sys/kernel/mm/transparent_hugepage/enabled").read().strip()
        thp += " | defrag " + open("/sys/kernel/mm/transparent_hugepage/defrag").read().strip()
    except OSError:
        thp = "unknown"
    print("transparent huge pages: %s" % thp)
    gb = zp.get_numpy_array().nbytes / 1e9
    calls, frees = [], []
    data = zp.compress(nthreads=a.threads, **mode(a))
    for _ in range(a.loop):
        t0 = time.perf_counter()
        data = None
        zp._compress_data, zp._index_of = [], []
        t1 = time.perf_counter()
        data = zp.compress(nthreads=a.threads, **mode(a))
        t2 = time.perf_counter()
        frees.append(t1 - t0)
        calls.append(t2 - t1)
    print("loop of %d compress calls: %s ms (median %.1f ms = %.1f GB/s); freeing the previous streams: %s ms"
          % (a.loop, " ".join("%.1f" % (1e3 * x) for x in calls), 1e3 * np.median(calls), gb / np.median(calls),
             " ".join("%.1f" % (1e3 * x) for x in frees)))


def profile_compress(zp, a):
    """Wall time of each compress_numpy_portion split into its native call, the
    stream copy into bytes and the index export (zfpy_c, timing wrappers)."""
    import threading
    from zfpy import zfpy_c
    lock = threading.Lock()
    rec = {}

    def timed(name, fn):
        def w(*x, **k):
            t0 = time.perf_counter()
            try:
                return fn(*x, **k)
            finally:
                with lock:
                    rec.setdefault(name, []).append((t0, time.perf_counter()))
        return w

    class Lib:
        def __init__(self, lib):
            self._l = lib

        def __getattr__(self, nm):
            f = getattr(self._l, nm)
            return timed(nm, f) if nm in ("zfp_compress_chunk", "zfp_write_header", "stream_open") else f

    saved = (zfpy_c._lib, zfpy_c._bytes_from, zfpy_c._export_index, zfpy_c._bytes_target, zfpy_c._make_resident)
    zfpy_c._lib = Lib(saved[0])
    zfpy_c._bytes_from = timed("bytes_from", saved[1])
    zfpy_c._export_index = timed("export_index", saved[2])
    zfpy_c._bytes_target = timed("bytes_target", saved[3])
    zfpy_c._make_resident = timed("make_resident", saved[4])
    import zfpy._zfp_par as zpar
    saved_p = zpar._compress_portion
    zpar._compress_portion = timed("portion", saved_p)
    try:
        t0 = time.perf_counter()
        zp.compress(nthreads=a.threads, **mode(a))
        t1 = time.perf_counter()
    finally:
        zfpy_c._lib, zfpy_c._bytes_from, zfpy_c._export_index, zfpy_c._bytes_target, zfpy_c._make_resident = saved
        zpar._compress_portion = saved_p
    print("profile: compress wall %.1f ms" % (1e3 * (t1 - t0)))
    for nm, v in sorted(rec.items()):
        d = [1e3 * (b - x) for x, b in v]
        print("  %-20s n=%d  sum %.1f ms  max %.1f ms  first start +%.1f ms  last end +%.1f ms"
              % (nm, len(v), sum(d), max(d), 1e3 * (min(x for x, _ in v) - t0), 1e3 * (max(b for _, b in v) - t0)))


if __name__ == "__main__":
    main()
