"""One zfp_parallel chunk compress (1024x1024x64 f32 z-slab, rate 8) timed by
source memory: the zfp_p RawArray (multiprocessing shared memory) against a
private numpy array of the same bytes, with and without the slab pipeline
(ZFP_HIP_NO_PIPE is read per call)."""
import ctypes
import os
import sys
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "zfp-par_amd")]

from zfpy import zfpy_c  # noqa: E402
from zfpy._zfp_par import zfp_p  # noqa: E402


def best(fn, reps=4):
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return 1e3 * min(t)


def main():
    zp = zfp_p((512, 1024, 1024), "float32", nparts=8)
    arr = zp.get_numpy_array()
    arr[:] = np.sin(np.arange(arr.size, dtype=np.float32) * 1e-3).reshape(arr.shape)
    ck = zp.get_chunkit()
    priv = np.ascontiguousarray(arr[:64]).copy()
    km, tm = ctypes.c_double(), ctypes.c_double()
    for pipe in ("1", None):
        if pipe:
            os.environ["ZFP_HIP_NO_PIPE"] = pipe
        else:
            os.environ.pop("ZFP_HIP_NO_PIPE", None)
        a = best(lambda: zfpy_c.compress_numpy_portion(zp.get_raw_array(), ck, 0, rate=8))
        zfpy_c._lib.zfp_hip_last_timing(ctypes.byref(km), ctypes.byref(tm))
        b = best(lambda: zfpy_c.compress_numpy(priv, rate=8))
        print("no_pipe=%s: RawArray chunk %.1f ms (last call: kernel %.2f ms, native %.1f ms), private numpy slab "
              "%.1f ms" % (pipe, a, km.value, tm.value, b), flush=True)


if __name__ == "__main__":
    main()
