#!/usr/bin/env python3
"""Per-call latency of the low-level block API (zfp_encode_block_float_3 /
zfp_decode_block_float_3) on this library, where each call is one GPU round
trip, and of the bulk paths the GPU arrays use instead (one zfp_compress of a
line of 256 blocks, one of a whole 129^3 array).

usage: python tools/block_api_latency.py [--calls 2000]
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(R, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    a = ap.parse_args()
    from capi import ZfpCAPI
    api = ZfpCAPI(os.path.join(R, "zfp-par_amd", "lib", "libzfp.so"))
    lib = api.lib
    for fn in ("zfp_encode_block_float_3", "zfp_decode_block_float_3"):
        getattr(lib, fn).restype = ctypes.c_size_t
        getattr(lib, fn).argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    zs = lib.zfp_stream_open(None)
    lib.zfp_stream_set_rate(zs, 8.0, 3, 3, 1)
    buf = np.zeros(a.calls * 64 + 64, dtype=np.uint8)
    bs = lib.stream_open(ctypes.c_void_p(buf.ctypes.data), buf.nbytes)
    lib.zfp_stream_set_bit_stream(zs, bs)
    blk = np.sin(np.arange(64, dtype=np.float32) * 0.1)
    for _ in range(50):  # warm: contexts, code objects
        lib.zfp_stream_rewind(zs)
        lib.zfp_encode_block_float_3(zs, ctypes.c_void_p(blk.ctypes.data))
    lib.zfp_stream_rewind(zs)
    t0 = time.perf_counter()
    for _ in range(a.calls):
        lib.zfp_encode_block_float_3(zs, ctypes.c_void_p(blk.ctypes.data))
    enc = (time.perf_counter() - t0) / a.calls * 1e6
    lib.stream_flush(bs)
    lib.zfp_stream_rewind(zs)
    out = np.empty(64, dtype=np.float32)
    t0 = time.perf_counter()
    for _ in range(a.calls):
        lib.zfp_decode_block_float_3(zs, ctypes.c_void_p(out.ctypes.data))
    dec = (time.perf_counter() - t0) / a.calls * 1e6
    # bulk: a line of 256 blocks (1024 x 4 x 4) and a whole 129^3 array, one zfp_compress each
    res = {}
    for name, shape in (("line of 256 blocks", (4, 4, 1024)), ("129^3 array", (129, 129, 129))):
        f = np.sin(np.arange(int(np.prod(shape)), dtype=np.float32) * 1e-3).reshape(shape)
        zf = lib.zfp_field_3d(ctypes.c_void_p(f.ctypes.data), 3, shape[2], shape[1], shape[0])
        cap = lib.zfp_stream_maximum_size(zs, zf)
        ob = np.zeros(cap, dtype=np.uint8)
        b2 = lib.stream_open(ctypes.c_void_p(ob.ctypes.data), cap)
        lib.zfp_stream_set_bit_stream(zs, b2)
        ts = []
        for i in range(30):
            lib.zfp_stream_rewind(zs)
            t0 = time.perf_counter()
            assert lib.zfp_compress(zs, zf)
            ts.append(time.perf_counter() - t0)
        nb = -(-shape[0] // 4) * -(-shape[1] // 4) * -(-shape[2] // 4)
        res[name] = (np.median(ts[5:]) * 1e6, nb)
        lib.stream_close(b2)
        lib.zfp_field_free(zf)
    print("block API, one GPU round trip per call: encode %.1f us/block, decode %.1f us/block (%d calls, rate 8)"
          % (enc, dec, a.calls))
    for name, (us, nb) in res.items():
        print("zfp_compress of a %s: %.1f us per call, %.3f us per block (%d blocks)" % (name, us, us / nb, nb))


if __name__ == "__main__":
    main()
