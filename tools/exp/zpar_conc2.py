"""zfp_parallel chunk compress costs (experiment), 8 chunks of a
512x1024x1024 f32 zfp_p at rate 8 on 8 threads:
  bytes   the product path (each stream written into a new bytes object)
  reuse   streams written into per-thread buffers allocated once (no page faults)
  +pin    the same with the shared source array page-locked (hipHostRegister)
Prints wall ms per variant (best of 3)."""
import ctypes
import os
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "zfp-par_amd")]

from zfpy import zfpy_c  # noqa: E402
from zfpy._zfp_par import zfp_p  # noqa: E402


def main():
    zp = zfp_p((512, 1024, 1024), "float32", nparts=8)
    arr = zp.get_numpy_array()
    for k in range(arr.shape[0]):
        arr[k] = np.sin(np.arange(1024 * 1024, dtype=np.float32).reshape(1024, 1024) * 1e-3 + k)
    ck = zp.get_chunkit()
    raw = zp.get_raw_array()
    gb = arr.nbytes / 1e9
    tls = threading.local()
    real_target, real_take = zfpy_c._bytes_target, zfpy_c._bytes_take

    def reuse_target(size):
        b = getattr(tls, "b", None)
        if b is None or b.size < size:
            b = tls.b = np.ones(size, dtype=np.uint8)
        return 0, b.ctypes.data

    def one(i):
        return zfpy_c._compress_portion(raw, ck, i, -1, 8, -1, True, -1, True)

    def run(name):
        t = []
        with ThreadPoolExecutor(8) as ex:
            for _ in range(3):
                t0 = time.perf_counter()
                out = list(ex.map(one, range(8)))
                t.append(time.perf_counter() - t0)
                del out
        print("%-14s %7.1f ms  %5.1f GB/s" % (name, 1e3 * min(t), gb / min(t)), flush=True)

    run("bytes")
    zfpy_c._bytes_target, zfpy_c._bytes_take = reuse_target, (lambda h, n: b"")
    run("reuse")
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    t0 = time.perf_counter()
    rc = hip.hipHostRegister(arr.ctypes.data, arr.nbytes, 0)
    print("hipHostRegister rc %d in %.1f ms" % (rc, 1e3 * (time.perf_counter() - t0)), flush=True)
    run("reuse+pin")
    zfpy_c._bytes_target, zfpy_c._bytes_take = real_target, real_take
    run("bytes+pin")


if __name__ == "__main__":
    main()
