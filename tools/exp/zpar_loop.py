"""zfp_parallel compress timed in two loops (experiment): alternating with
decompress (as tools/zfp_par_bench.py) and back to back."""
import os
import sys
import time

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(R, "zfp-par_amd")]
from zfpy._zfp_par import zfp_p  # noqa: E402

zp = zfp_p((512, 1024, 1024), "float32", nparts=8)
arr = zp.get_numpy_array()
for k in range(arr.shape[0]):
    arr[k] = np.sin(np.arange(1024 * 1024, dtype=np.float32).reshape(1024, 1024) * 1e-3 + k)
gb = arr.nbytes / 1e9
for name, dec in (("alternating", True), ("back-to-back", False), ("alternating", True)):
    t = []
    for _ in range(4):
        t0 = time.perf_counter()
        zp.compress(nthreads=8, rate=8)
        t.append(time.perf_counter() - t0)
        if dec:
            zp.decompress(nthreads=8)
    print("%-13s compress %s ms" % (name, " ".join("%.1f" % (1e3 * x) for x in t)), flush=True)
