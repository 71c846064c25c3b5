"""Debug helper: decode on the GPU vs the oracle, report mismatching blocks and
which lanes (block index % 64) they sit in."""
import os, sys, zlib
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (R, R + "/oracle", R + "/tests"):
    sys.path.insert(0, p)
import torch  # noqa: F401  (one HIP runtime)
from capi import ZfpCAPI
from pyoracle import Oracle, params_rate, params_reversible, params_precision
api = ZfpCAPI(R + "/zfp-par_amd/lib/libzfp.so"); api.enable_index()
o = Oracle()
shape = (16, 16, 16)
for mode, param, params in [("rate", 16, params_rate(16, 3, 3)), ("precision", 12, params_precision(12)),
                            ("reversible", None, params_reversible())]:
    rng = np.random.default_rng(3)
    a = (np.sin(np.arange(np.prod(shape)) * 0.01).reshape(shape) + 0.1 * rng.standard_normal(shape)).astype(np.float32)
    w, end = o.compress_words(a, params)
    got = api.compress(a, mode, param, ztype=3)
    print(mode, "stream equal:", got == w.tobytes())
    ref, _ = o.decompress_words(w, shape, np.float32, params)
    out, n = api.decompress(got, shape, np.float32, mode, param, ztype=3, index=api.last_index)
    bad = []
    for bz in range(4):
        for by in range(4):
            for bx in range(4):
                b = bx + 4 * by + 16 * bz
                s = (slice(4*bz, 4*bz+4), slice(4*by, 4*by+4), slice(4*bx, 4*bx+4))
                if not np.array_equal(out[s].view(np.uint32), ref[s].view(np.uint32)):
                    bad.append(b)
    print(mode, "bad blocks:", bad)
    if bad:
        b = bad[0]; bz, by, bx = b // 16, (b // 4) % 4, b % 4
        s = (slice(4*bz, 4*bz+4), slice(4*by, 4*by+4), slice(4*bx, 4*bx+4))
        print(" got ", out[s].ravel()[:8]); print(" want", ref[s].ravel()[:8])
    if api.last_index:
        api.lib.zfp_hip_index_free(api.last_index); api.last_index = None
