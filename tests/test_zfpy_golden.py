"""zfpy chunk streams against the reference's OWN Python zfpy.

tests/golden/zfpy_chunks.json holds, per case, the per-chunk stream lengths,
SHA-256 and first 16 bytes produced by the reference's zfpy.zfp_parallel
(zfpy/_zfp_par.py:103-157 over python/zfpy_c.pyx:330-376) and the SHA-256 of
its decompressed array, made by tests/golden/make_zfpy_fixtures.py in the build
container.  CPU tests pin the oracle + header writer to those streams (chunk
boxes from this library's partitioner); GPU tests check this framework's
zfp_parallel byte for byte, header bits included, and its decompression.
"""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np
import pytest

from pyoracle import TYPE_DOUBLE, TYPE_FLOAT, params_accuracy, params_precision, params_rate, params_reversible

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
from make_zfpy_fixtures import case_field  # noqa: E402  (input generator only; no reference import)

FIX = json.load(open(os.path.join(HERE, "golden", "zfpy_chunks.json")))["cases"]
IDS = [c["name"] for c in FIX]


def _params(c):
    ztype = TYPE_FLOAT if c["dtype"] == "float32" else TYPE_DOUBLE
    if c["mode"] == "rate":
        return params_rate(c["param"], 0, len(c["shape"]))  # zfpy passes zfp_type_none (pyx:300-302)
    if c["mode"] == "precision":
        return params_precision(c["param"])
    if c["mode"] == "tolerance":
        return params_accuracy(c["param"])
    return params_reversible()


def _kw(c):
    return {} if c["mode"] == "reversible" else {c["mode"]: c["param"]}


@pytest.mark.parametrize("case", FIX, ids=IDS)
def test_fixture_inputs_regenerate(case):
    a = case_field(tuple(case["shape"]), case["dtype"])
    assert hashlib.sha256(a.tobytes()).hexdigest() == case["input_sha256"]


@pytest.mark.parametrize("case", FIX, ids=IDS)
def test_oracle_and_header_writer_reproduce_reference_chunks(case, oracle):
    """CPU: header (this library's zfp_write_header, host buffer) + the oracle's
    blocks of each chunk box at bit 96 == the reference zfpy's chunk stream."""
    import zfpy
    from zfpy import zfpy_c
    shape, dtype = tuple(case["shape"]), np.dtype(case["dtype"])
    if len(shape) < 3 or dtype.kind == "i":
        pytest.skip("the oracle restates the 3D/4D float codec; 1D/2D/integer parity is checked against "
                    "oracle/_ref in test_gpu_types.py and against these fixtures on the GPU")
    arr = case_field(shape, dtype)
    ck = zfpy_c.zfp_chunkit(arr, np.prod([(n + 3) // 4 for n in shape]) / case["nparts"])
    assert ck.get_nchunks() == case["nchunks"]
    lib = zfpy_c._lib
    params = _params(case)
    for i, want in enumerate(case["chunks"]):
        # header of the whole field, mode from the zfpy mode setter
        field = zfpy_c._init_field_raw(arr, ck)
        zs = lib.zfp_stream_open(None)
        zfpy_c._set_compression_mode(zs, 0, len(shape), **_kw(case))
        hbuf = ctypes.create_string_buffer(64)
        bs = lib.stream_open(hbuf, 64)
        lib.zfp_stream_set_bit_stream(zs, bs)
        assert lib.zfp_write_header(zs, field, zfpy_c.HEADER_FULL) == 96
        lib.stream_flush.restype = ctypes.c_uint64
        lib.stream_flush.argtypes = [ctypes.c_void_p]
        lib.stream_flush(bs)  # the last 32 header bits are still in the bit buffer
        lib.stream_close(bs)
        lib.zfp_stream_close(zs)
        lib.zfp_field_free(field)
        head = np.frombuffer(hbuf.raw[:16], dtype=np.uint64).copy()
        box = [ck.boxes[i][a] for a in range(4)]
        words, end = oracle.compress_words(arr, params, box=box, bit_offset=96)
        words = np.concatenate([words, np.zeros(2, np.uint64)]) if len(words) < 2 else words
        words[0] |= head[0]
        words[1] |= head[1] & np.uint64((1 << 32) - 1)
        stream = words.view(np.uint8).tobytes()[: (end + 63) // 64 * 8]
        assert len(stream) == want["len"], (i, len(stream), want["len"])
        assert stream[:16].hex() == want["head"]
        assert hashlib.sha256(stream).hexdigest() == want["sha256"], i


@pytest.mark.gpu
@pytest.mark.parametrize("case", FIX, ids=IDS)
def test_zfp_parallel_matches_reference_zfpy(product, case):
    import zfpy
    shape, dtype = tuple(case["shape"]), case["dtype"]
    zp = zfpy.zfp_parallel(shape, dtype, nparts=case["nparts"])
    zp.get_numpy_array()[...] = case_field(shape, dtype)
    streams = zp.compress(nthreads=4, **_kw(case))
    assert len(streams) == case["nchunks"]
    for i, (s, want) in enumerate(zip(streams, case["chunks"])):
        s = bytes(s)
        assert len(s) == want["len"], i
        assert s[:16].hex() == want["head"], i  # the 96 header bits + first block bits
        assert hashlib.sha256(s).hexdigest() == want["sha256"], i
    zp.get_numpy_array()[...] = 0
    # plain bytes (no GPU block index attached): variable-rate chunks are scanned
    zp._compress_data = [bytes(s) for s in streams]
    zp.decompress(nthreads=4)
    back = np.ascontiguousarray(zp.get_numpy_array())
    assert hashlib.sha256(back.tobytes()).hexdigest() == case["decompressed_sha256"]
