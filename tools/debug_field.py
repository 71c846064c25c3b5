"""Debug helper: compress a field on the GPU (fixed rate 16 by default), compare
with the oracle block by block, dump the first mismatching block's values."""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (R, R + "/oracle", R + "/tests"):
    sys.path.insert(0, p)
from capi import ZfpCAPI
from pyoracle import Oracle, params_rate

api = ZfpCAPI(R + "/zfp-par_amd/lib/libzfp.so"); api.enable_index()
o = Oracle()
shape = (20, 33, 40)
a = o.smooth_field(3, np.float32, min_total=int(np.prod(shape))).ravel()[: int(np.prod(shape))].reshape(shape)
rate = 16
bits = 64 * rate
w, end = o.compress_words(a, params_rate(rate, 3, 3))
want = w.view(np.uint8).tobytes()[:(end + 63) // 64 * 8]
got = api.compress(a, "rate", rate, ztype=3)
print("equal:", got == want, len(got), len(want))
gw = np.frombuffer(got, np.uint64)
ww = np.frombuffer(want, np.uint64)
nbx, nby, nbz = (shape[2] + 3) // 4, (shape[1] + 3) // 4, (shape[0] + 3) // 4
nbad = 0
for b in range(len(ww) * 64 // bits):
    sw = bits // 64
    g = gw[b * sw:(b + 1) * sw]
    x = ww[b * sw:(b + 1) * sw]
    if not np.array_equal(g, x):
        nbad += 1
        if nbad <= 3:
            bx, by, bz = b % nbx, (b // nbx) % nby, b // (nbx * nby)
            blk = a[4 * bz:4 * bz + 4, 4 * by:4 * by + 4, 4 * bx:4 * bx + 4]
            diff = [(i, int(g[i]) ^ int(x[i])) for i in range(sw) if g[i] != x[i]]
            print("block", b, (bx, by, bz), "shape", blk.shape, "diff words", [(i, hex(d)) for i, d in diff])
            np.save(os.path.join(R, "gpurun_out", "badblock_%d.npy" % b), np.ascontiguousarray(blk))
print("bad blocks", nbad)
