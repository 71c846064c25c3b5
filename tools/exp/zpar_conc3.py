"""zfp_parallel compress with the new bytes objects' pages made resident
before the GPU call (experiment; see zpar_conc2.py: page faults of fresh
stream memory inside the device-to-host copies cost about half the time):
  none      the product path
  memset    ctypes.memset of the object (GIL released) in the calling thread
  populate  madvise(MADV_POPULATE_WRITE) of its whole pages
  huge      madvise(MADV_HUGEPAGE) then MADV_POPULATE_WRITE
Prints wall ms per variant (best of 3)."""
import ctypes
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "zfp-par_amd")]

from zfpy import zfpy_c  # noqa: E402
from zfpy._zfp_par import zfp_p  # noqa: E402

libc = ctypes.CDLL(None, use_errno=True)
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
MADV_HUGEPAGE, MADV_POPULATE_WRITE = 14, 23
PAGE = 4096


def main():
    zp = zfp_p((512, 1024, 1024), "float32", nparts=8)
    arr = zp.get_numpy_array()
    for k in range(arr.shape[0]):
        arr[k] = np.sin(np.arange(1024 * 1024, dtype=np.float32).reshape(1024, 1024) * 1e-3 + k)
    ck = zp.get_chunkit()
    raw = zp.get_raw_array()
    gb = arr.nbytes / 1e9
    real = zfpy_c._bytes_target

    def make(how):
        def target(size):
            h, a = real(size)
            if how == "memset":
                ctypes.memset(a, 0, size)
            elif how in ("populate", "huge"):
                lo = (a + PAGE - 1) & ~(PAGE - 1)
                n = (a + size - lo) & ~(PAGE - 1)
                if how == "huge":
                    libc.madvise(lo, n, MADV_HUGEPAGE)
                if libc.madvise(lo, n, MADV_POPULATE_WRITE) != 0:
                    print("madvise errno", ctypes.get_errno(), flush=True)
            return h, a
        return target

    def one(i):
        return zfpy_c._compress_portion(raw, ck, i, -1, 8, -1, True, -1, True)

    for how in ("none", "memset", "populate", "huge", "none"):
        zfpy_c._bytes_target = make(how)
        t = []
        with ThreadPoolExecutor(8) as ex:
            for _ in range(3):
                t0 = time.perf_counter()
                out = list(ex.map(one, range(8)))
                t.append(time.perf_counter() - t0)
                del out
        print("%-10s %7.1f ms  %5.1f GB/s" % (how, 1e3 * min(t), gb / min(t)), flush=True)


if __name__ == "__main__":
    main()
