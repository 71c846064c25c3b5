"""Pin the CPU oracle before trusting it (CPU-only tests).

(1) Golden checksums of the reference's own end-to-end tests
    (tests/constants/checksums, keys per tests/utils/zfpChecksums.c:75-136),
    on the reference's smooth-random generator fields (129^3, 33^4, ...).
(2) Byte-for-byte agreement with the reference itself (oracle/_ref, compiled
    from /root/reference) on seeded fields with partial blocks, special values,
    strides and chunk boxes, in every mode.
"""
import numpy as np
import pytest

from pyoracle import (TYPE_DOUBLE, TYPE_FLOAT, params_accuracy, params_precision, params_rate,
                      params_reversible)

GROUPS = [(d, t) for d in (1, 2, 3, 4) for t in ("float", "double")]


def _params(mode, param, ztype, dims):
    if mode == "rate":
        return params_rate(param, ztype, dims)
    if mode == "precision":
        return params_precision(param)
    if mode == "accuracy":
        return params_accuracy(param)
    return params_reversible()


@pytest.mark.parametrize("dims,tname", GROUPS)
def test_oracle_matches_golden_checksums(oracle, golden, dims, tname):
    dtype = np.float32 if tname == "float" else np.float64
    ztype = TYPE_FLOAT if tname == "float" else TYPE_DOUBLE
    entries = [e for e in golden if e["dims"] == dims and e["type"] == tname]
    field = oracle.smooth_field(dims, dtype)
    inp = [e for e in entries if e["subject"] == "input"][0]
    assert list(reversed(field.shape)) == inp["n"]
    assert oracle.hash_array(field) == int(inp["checksum"], 16)
    cases = {}
    for e in entries:
        if e["subject"] != "input":
            cases.setdefault((e["mode"], e["param"]), {})[e["subject"]] = int(e["checksum"], 16)
    assert len(cases) == 10
    for (mode, param), want in sorted(cases.items(), key=str):
        params = _params(mode, param, ztype, dims)
        words, end = oracle.compress_words(field, params)
        if "stream" in want:
            assert oracle.hash_words(words) == want["stream"], (mode, param)
        if "decompressed" in want:
            out, end2 = oracle.decompress_words(words, field.shape, dtype, params)
            assert end2 == end
            assert oracle.hash_array(out) == want["decompressed"], (mode, param)


def _special_field(shape, dtype, rng):
    a = (rng.standard_normal(shape) * rng.choice([1e-3, 1.0, 1e6], size=shape)).astype(dtype)
    flat = a.reshape(-1)
    info = np.finfo(dtype)
    specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, info.tiny, info.tiny / 4, -info.tiny / 8,
                         info.max, -info.max], dtype=dtype)
    idx = rng.choice(flat.size, size=max(1, flat.size // 50), replace=False)
    flat[idx] = rng.choice(specials, size=idx.size)
    # a few whole blocks of subnormals / zeros / negative zeros
    if a.ndim == 3 and min(shape) >= 8:
        a[:4, :4, :4] = info.tiny / 16
        a[4:8, :4, :4] = -0.0
        a[:4, 4:8, :4] = 0.0
    return a


MODES = [("rate", 8), ("rate", 16), ("rate", 1.5), ("precision", 12), ("precision", 32),
         ("accuracy", 1e-3), ("reversible", None), ("expert", (100, 1500, 20, -20))]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("shape", [(7, 9, 10), (16, 16, 16), (5, 6, 7, 9)])
@pytest.mark.parametrize("mode,param", MODES)
def test_oracle_matches_reference_library(oracle, ref_capi, dtype, shape, mode, param):
    rng = np.random.default_rng(hash((shape, mode)) & 0xffff)
    a = _special_field(shape, dtype, rng)
    ztype = TYPE_FLOAT if dtype == np.float32 else TYPE_DOUBLE
    if mode == "expert":
        params = param
    else:
        params = _params(mode, param, ztype, a.ndim)
    ref = ref_capi.compress(a, mode, param)
    words, end = oracle.compress_words(a, params)
    mine = words.view(np.uint8)[: len(ref)].tobytes()
    assert (end + 63) // 64 * 8 == len(ref)
    assert mine == ref
    ref_out, _ = ref_capi.decompress(ref, a.shape, dtype, mode, param)
    out, _ = oracle.decompress_words(words, a.shape, dtype, params)
    assert out.tobytes() == ref_out.tobytes()


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_oracle_chunk_boxes_and_strides_match_reference(oracle, ref_capi, dtype):
    rng = np.random.default_rng(7)
    a = rng.standard_normal((14, 13, 21)).astype(dtype)
    ztype = TYPE_FLOAT if dtype == np.float32 else TYPE_DOUBLE
    box = [(4, 21), (0, 8), (8, 14)]  # x, y, z (exclusive ends); z runs to the field edge
    ref = ref_capi.compress(a, "rate", 12, chunk=box, strided=True)
    params = params_rate(12, ztype, 3)
    words, end = oracle.compress_words(a, params, box=box + [(0, 0)])
    assert words.view(np.uint8)[: len(ref)].tobytes() == ref
    # a strided (transposed) view with a non-unit x stride
    t = np.ascontiguousarray(rng.standard_normal((11, 10, 9)).astype(dtype)).transpose(2, 1, 0)
    ref = ref_capi.compress(t, "precision", 20, strided=True)
    st = [s // t.itemsize for s in reversed(t.strides)] + [0]
    words, end = oracle.compress_words(t, params_precision(20), strides=st, base=t.ctypes.data)
    assert words.view(np.uint8)[: len(ref)].tobytes() == ref


# ---------------- integer golden tables ----------------
INT_GROUPS = [(d, t) for d in (1, 2, 3, 4) for t in ("int32", "int64")]


@pytest.mark.parametrize("dims,tname", INT_GROUPS)
def test_int_fields_and_reference_match_golden_checksums(oracle, ref_capi, golden, dims, tname):
    """The reference's Int32/Int64 end-to-end tables: the restated generator reproduces the
    input hashes, and the reference library compiled here reproduces stream and decompressed
    hashes under this module's reading of the table keys (the GPU test relies on both)."""
    dtype = np.int32 if tname == "int32" else np.int64
    entries = [e for e in golden if e["dims"] == dims and e["type"] == tname]
    inp = [e for e in entries if e["subject"] == "input"][0]
    # the integer tests use smaller fields: the generator refines until it holds inp["n"]
    field = oracle.smooth_field(dims, dtype, min_total=int(np.prod(inp["n"])))
    assert list(reversed(field.shape)) == inp["n"]
    assert oracle.hash_array(field) == int(inp["checksum"], 16)
    cases = {}
    for e in entries:
        if e["subject"] != "input":
            cases.setdefault((e["mode"], e["param"]), {})[e["subject"]] = int(e["checksum"], 16)
    assert len(cases) == 7
    for (mode, param), want in sorted(cases.items(), key=str):
        data = ref_capi.compress(field, mode, param)
        if "stream" in want:
            assert oracle.hash_words(np.frombuffer(data, dtype=np.uint64)) == want["stream"], (mode, param)
        out, _ = ref_capi.decompress(data, field.shape, dtype, mode, param)
        if "decompressed" in want:
            assert oracle.hash_array(out) == want["decompressed"], (mode, param)
