"""Debug helper: compare product vs oracle block by block on crafted fields."""
import os, sys, zlib
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (R, R + "/oracle", R + "/tests"):
    sys.path.insert(0, p)
from capi import ZfpCAPI
from pyoracle import Oracle, params_rate
api = ZfpCAPI(R + "/zfp-par_amd/lib/libzfp.so"); api.enable_index()
o = Oracle()
info = np.finfo(np.float32)
cases = {
  "ones": np.ones((4,4,4), np.float32),
  "max": np.full((4,4,4), 0.5, np.float32),
  "nan": np.full((4,4,4), 0.5, np.float32),
  "inf": np.full((4,4,4), 0.5, np.float32),
  "sub": np.full((4,4,4), info.tiny/16, np.float32),
  "neg": -np.arange(64, dtype=np.float32).reshape(4,4,4),
  "rand": np.random.default_rng(1).standard_normal((4,4,4)).astype(np.float32),
  "rand2": np.random.default_rng(2).standard_normal((4,4,8)).astype(np.float32),
}
cases["max"][1,2,3] = info.max
cases["nan"][0,0,1] = np.nan
cases["inf"][3,3,3] = np.inf
for name, a in cases.items():
    w, end = o.compress_words(a, params_rate(16, 3, 3))
    want = w.view(np.uint8).tobytes()[:(end+63)//64*8]
    got = api.compress(a, "rate", 16, ztype=3)
    if got == want:
        print(name, "OK")
    else:
        gw = np.frombuffer(got, np.uint64); 
        print(name, "MISMATCH", [hex(x) for x in gw[:4]], [hex(x) for x in w[:4]])
