"""zfp_parallel chunk compress under different concurrency (experiment): the
eight 1024x1024x64 f32 chunks of a 512x1024x1024 zfp_p at rate 8, run
(a) one after another in one thread, (b) on 8 threads at once, (c) on 8
threads with the native call serialised by a lock, (d) on 8 threads with at
most 2 native calls at once.  Prints wall ms per variant (best of 3)."""
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
    n = 8
    gb = arr.nbytes / 1e9

    def one(i, gate=None):
        if gate is None:
            return zfpy_c._compress_portion(raw, ck, i, -1, 8, -1, True, -1, True)
        with gate:
            return zfpy_c._compress_portion(raw, ck, i, -1, 8, -1, True, -1, True)

    def run(name, fn):
        t = []
        for _ in range(3):
            t0 = time.perf_counter()
            out = fn()
            t.append(time.perf_counter() - t0)
            del out
        print("%-22s %7.1f ms  %5.1f GB/s" % (name, 1e3 * min(t), gb / min(t)), flush=True)

    run("serial 1 thread", lambda: [one(i) for i in range(n)])
    for th in (8, 4, 2):
        with ThreadPoolExecutor(th) as ex:
            run("%d threads" % th, lambda: list(ex.map(one, range(n))))
    for lim in (1, 2, 3):
        sem = threading.Semaphore(lim)
        with ThreadPoolExecutor(8) as ex:
            run("8 threads, %d at once" % lim, lambda: list(ex.map(lambda i: one(i, sem), range(n))))


if __name__ == "__main__":
    main()
