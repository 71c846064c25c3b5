#!/usr/bin/env python3
"""Light driver for profiling: device-resident zfp_compress / zfp_decompress loops.

usage: python tools/kprof.py [--mode rate|precision|reversible] [--param P] [--dtype f32|f64]
                             [--n 1024] [--iters 5] [--decode]
Prints per-call kernel ms from the library's HIP events.
"""
import argparse
import ctypes
import os
import sys
import time

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, R + "/tests", R + "/oracle"]


def field(torch, n, dtype, dev, nz=0):
    nz = nz or n
    x = torch.arange(n, device=dev, dtype=torch.float64)
    out = torch.empty((nz, n, n), device=dev, dtype=dtype)
    base = torch.sin(0.05 * x)[None, :] * torch.cos(0.03 * x)[:, None]
    xy = 0.01 * x[None, :] * x[:, None] / n
    for z0 in range(0, nz, 64):
        z = torch.arange(z0, min(nz, z0 + 64), device=dev, dtype=torch.float64)[:, None, None]
        out[z0:z0 + 64] = (base[None] + 0.5 * torch.sin(0.02 * z + xy[None])).to(dtype)
    return out


def field4(torch, n, dtype, dev):
    """F1 with the C5 w term: + .25 cos(.04 w)."""
    import math
    x = torch.arange(n, device=dev, dtype=torch.float64)
    base = torch.sin(0.05 * x)[None, :] * torch.cos(0.03 * x)[:, None]
    xy = 0.01 * x[None, :] * x[:, None] / n
    z = x[:, None, None]
    out = torch.empty((n, n, n, n), device=dev, dtype=dtype)
    for w in range(n):
        out[w] = (base[None] + 0.5 * torch.sin(0.02 * z + xy[None]) + 0.25 * math.cos(0.04 * w)).to(dtype)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="rate")
    ap.add_argument("--param", type=float, default=16)
    ap.add_argument("--dtype", default="f32")
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--decode", action="store_true")
    ap.add_argument("--dims", type=int, default=3)
    ap.add_argument("--sha", action="store_true", help="print a hash of the last stream (variant exactness)")
    ap.add_argument("--host", action="store_true", help="field and stream in host memory (PCIe-inclusive)")
    ap.add_argument("--nz", type=int, default=0, help="3D field n x n x nz (default cubic)")
    ap.add_argument("--header", action="store_true", help="write the 96-bit zfpy header first (C4 stream offset)")
    ap.add_argument("--lib", default=R + "/zfp-par_amd/lib/libzfp.so", help="libzfp.so to load (variant builds)")
    a = ap.parse_args()
    import torch
    from capi import ZfpCAPI
    api = ZfpCAPI(a.lib)
    api.enable_index()
    lib = api.lib
    dev = torch.device("cuda", 0)
    dt = torch.float32 if a.dtype == "f32" else torch.float64
    zt = 3 if a.dtype == "f32" else 4
    if a.dims == 4:
        f = field4(torch, a.n, dt, dev)
        zf = lib.zfp_field_4d(ctypes.c_void_p(f.data_ptr()), zt, a.n, a.n, a.n, a.n)
    else:
        f = field(torch, a.n, dt, dev, a.nz)
        zf = lib.zfp_field_3d(ctypes.c_void_p(f.data_ptr()), zt, a.n, a.n, a.nz or a.n)
    if a.host:  # pinned? no: plain pageable numpy arrays, as a zfpy caller hands them over
        f = f.cpu().numpy()
        shape = [a.n] * a.dims
        fn = lib.zfp_field_4d if a.dims == 4 else lib.zfp_field_3d
        zf = fn(ctypes.c_void_p(f.ctypes.data), zt, *shape)
    zs = lib.zfp_stream_open(None)
    api.set_mode(zs, a.mode, a.param if a.mode != "reversible" else None, zt, a.dims)
    cap = lib.zfp_stream_maximum_size(zs, zf)
    if a.host:
        import numpy as np
        out_np = np.zeros(cap, dtype=np.uint8)
        bs = lib.stream_open(ctypes.c_void_p(out_np.ctypes.data), cap)
    else:
        out = torch.zeros(cap, dtype=torch.uint8, device=dev)
        bs = lib.stream_open(ctypes.c_void_p(out.data_ptr()), cap)
    lib.zfp_stream_set_bit_stream(zs, bs)
    ks = []
    for i in range(a.iters):
        lib.zfp_stream_rewind(zs)
        if a.header:
            assert lib.zfp_write_header(zs, zf, 7) == 96
        nb = lib.zfp_compress(zs, zf)
        assert nb, lib.zfp_hip_last_error()
        k, t = ctypes.c_double(), ctypes.c_double()
        lib.zfp_hip_last_timing(ctypes.byref(k), ctypes.byref(t))
        ks.append(t.value if a.host else k.value)
    gb = (f.nbytes if a.host else f.numel() * f.element_size()) / 1e9
    print(("host->host call " if a.host else "") + "encode %dD %s %s %s: bytes=%d kernel_ms=%s  GB/s=%.1f" % (a.dims, a.dtype, a.mode, a.param, nb,
          " ".join("%.3f" % x for x in ks), gb / (min(ks) * 1e-3)))
    if a.sha:
        import hashlib
        raw = out_np[:nb].tobytes() if a.host else out[:nb].cpu().numpy().tobytes()
        print("stream sha256 %s" % hashlib.sha256(raw).hexdigest()[:16])
    if a.decode:
        if a.host:
            import numpy as np
            back = np.empty_like(f)
            lib.zfp_field_set_pointer(zf, ctypes.c_void_p(back.ctypes.data))
        else:
            back = torch.empty_like(f)
            lib.zfp_field_set_pointer(zf, ctypes.c_void_p(back.data_ptr()))
        ks = []
        for i in range(a.iters):
            lib.stream_rewind(bs)
            assert lib.zfp_decompress(zs, zf), lib.zfp_hip_last_error()
            k, t = ctypes.c_double(), ctypes.c_double()
            lib.zfp_hip_last_timing(ctypes.byref(k), ctypes.byref(t))
            ks.append(t.value if a.host else k.value)
        sm, sp = ctypes.c_double(), ctypes.c_int()
        scanned = lib.zfp_hip_last_scan(ctypes.byref(sm), ctypes.byref(sp))
        print(("host->host call " if a.host else "") + "decode kernel_ms=%s  GB/s=%.1f  stale_index=%d scan=%d"
              % (" ".join("%.3f" % x for x in ks), gb / (min(ks) * 1e-3), lib.zfp_hip_last_stale_index() if hasattr(lib, 'zfp_hip_last_stale_index') else -1, scanned))


if __name__ == "__main__":
    main()
