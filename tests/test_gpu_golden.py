"""The reference's own golden checksum tables on the GPU, every table.

tests/golden/checksums.json holds the end-to-end rows of the reference's
tests/constants/checksums/{1,2,3,4}d{Float,Double,Int32,Int64}.h (made by
tests/golden/make_checksums.py): for each dimensionality and scalar type, the
hash of the smooth test field, of the compressed stream and of the decompressed
array in every mode the reference tests.  The field generator and the key
reading are pinned on the CPU (test_oracle.py); here the product's streams and
decompressed arrays must hash to the same values.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GROUPS = [(d, t) for d in (1, 2, 3, 4) for t in ("float", "double", "int32", "int64")]
DTYPES = {"float": np.float32, "double": np.float64, "int32": np.int32, "int64": np.int64}
ZTYPES = {"float": 3, "double": 4, "int32": 1, "int64": 2}


@pytest.mark.parametrize("dims,tname", GROUPS)
def test_golden_checksums_every_table(product, oracle, golden, dims, tname):
    dtype = DTYPES[tname]
    inp = [e for e in golden if e["dims"] == dims and e["type"] == tname and e["subject"] == "input"][0]
    field = oracle.smooth_field(dims, dtype, min_total=int(np.prod(inp["n"])))
    assert oracle.hash_array(field) == int(inp["checksum"], 16)
    cases = {}
    for e in golden:
        if e["dims"] == dims and e["type"] == tname and e["subject"] != "input":
            cases.setdefault((e["mode"], e["param"]), {})[e["subject"]] = int(e["checksum"], 16)
    assert cases
    for (mode, param), want in sorted(cases.items(), key=str):
        data = product.compress(field, mode, param, ztype=ZTYPES[tname])
        if "stream" in want:
            assert oracle.hash_words(np.frombuffer(data, dtype=np.uint64)) == want["stream"], (mode, param)
        # with the block index the compress call made, then (variable rate) through the stream scan
        for index in ((product.last_index, None) if product.last_index else (None,)):
            out, n = product.decompress(data, field.shape, dtype, mode, param, ztype=ZTYPES[tname], index=index)
            assert n == len(data), (mode, param)
            if "decompressed" in want:
                assert oracle.hash_array(out) == want["decompressed"], (mode, param, index is None)
        if product.last_index:
            product.lib.zfp_hip_index_free(product.last_index)
            product.last_index = None
