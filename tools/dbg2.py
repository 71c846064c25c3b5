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
# blocks of the first z-slab as a list of 4x4x4 blocks in raster order
blocks = [a[0:4, 4 * by:4 * by + 4, 4 * bx:4 * bx + 4] for by in range(8) for bx in range(10)]
def run(bl, tag):
    f = np.ascontiguousarray(np.concatenate(bl, axis=2))
    w, end = o.compress_words(f, params_rate(16, 3, 3))
    want = np.frombuffer(w.view(np.uint8).tobytes()[:(end + 63) // 64 * 8], np.uint64)
    got = np.frombuffer(api.compress(f, "rate", 16, ztype=3), np.uint64)
    bad = [i for i in range(len(bl)) if not np.array_equal(got[16 * i:16 * i + 16], want[16 * i:16 * i + 16])]
    print(tag, "bad lanes", bad)
    return bad
run(blocks[:64], "first64")
run(blocks[:2], "first2")
run(blocks[:8], "first8")
run(blocks[1:2] * 4, "b1x4")
run([blocks[0], blocks[1]] * 4, "b0b1x4")
for i in range(0, 10):
    run([blocks[i]], "single%d" % i)
print("---")
b8 = blocks[:8]
run(b8[::-1], "rev8")
run([b8[0], b8[2]], "b0b2")
run([b8[2], b8[0]], "b2b0")
run([b8[2], b8[3]], "b2b3")
run([b8[3], b8[2]], "b3b2")
run([b8[2], b8[2]], "b2b2")
run([b8[1], b8[2]], "b1b2")
f = np.ascontiguousarray(np.concatenate([b8[2], b8[3]], axis=2))
w, end = o.compress_words(f, params_rate(16, 3, 3))
want = np.frombuffer(w.view(np.uint8).tobytes()[:(end + 63) // 64 * 8], np.uint64)
got = np.frombuffer(api.compress(f, "rate", 16, ztype=3), np.uint64)
for i in range(32):
    print(i, "%016x %016x %s" % (got[i], want[i], "" if got[i] == want[i] else "DIFF %016x" % (got[i] ^ want[i])))
np.save(R + "/gpurun_out/b2b3.npy", f)
