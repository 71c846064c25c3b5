"""Host slab pipeline (zfp_hip.hip compress_slabs / decompress_slabs).

A host-resident field and stream go through the GPU in slabs of whole block
layers, with uploads, kernels and downloads overlapped on three streams.  The
environment knobs ZFP_HIP_PIPE_MIN_MB / ZFP_HIP_PIPE_SLAB_MB shrink the slabs so
that small fields exercise many slabs (partial last slab, unaligned slab
offsets, variable-rate offsets chained slab to slab, the chunk's block index
assembled from per-slab parts).  Bar: streams and decompressed arrays are
bit-identical to the oracle, exactly as for the one-shot path.
"""
import ctypes
import zlib

import numpy as np
import pytest

from pyoracle import TYPE_DOUBLE, TYPE_FLOAT, params_accuracy, params_precision, params_rate, params_reversible

pytestmark = pytest.mark.gpu


def _params(mode, param, ztype, dims):
    return {"rate": lambda: params_rate(param, ztype, dims), "precision": lambda: params_precision(param),
            "accuracy": lambda: params_accuracy(param), "reversible": params_reversible}[mode]()


@pytest.fixture
def slabs(monkeypatch):
    monkeypatch.setenv("ZFP_HIP_PIPE_MIN_MB", "1")
    monkeypatch.setenv("ZFP_HIP_PIPE_SLAB_MB", "1")


def _pipelined(product):
    k, t = ctypes.c_double(), ctypes.c_double()
    product.lib.zfp_hip_last_timing.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    product.lib.zfp_hip_last_timing(ctypes.byref(k), ctypes.byref(t))
    return k.value == 0.0 and t.value > 0.0  # the pipeline reports wall time only


def _field(shape, dtype, seed):
    rng = np.random.default_rng(seed)
    idx = np.indices(shape, dtype=np.float64)
    smooth = np.sin(0.05 * idx[-1]) * np.cos(0.03 * idx[-2]) + 0.5 * np.sin(0.02 * idx[0])
    return (smooth + 1e-3 * rng.standard_normal(shape)).astype(dtype)


MODES = [("rate", 16), ("rate", 12), ("rate", 3.5), ("precision", 16), ("accuracy", 1e-4), ("reversible", None)]


@pytest.mark.parametrize("shape", [(72, 64, 128), (70, 64, 128), (64, 24, 20, 32)])
@pytest.mark.parametrize("mode,param", MODES)
def test_pipelined_stream_and_roundtrip_match_oracle(product, oracle, slabs, shape, mode, param):
    dtype = np.float32
    a = _field(shape, dtype, zlib.crc32(repr((shape, mode)).encode()))
    ztype = TYPE_FLOAT
    params = _params(mode, param, ztype, a.ndim)
    ow, end = oracle.compress_words(a, params)
    want = ow.view(np.uint8).tobytes()[: (end + 63) // 64 * 8]
    product.keep_index = True
    try:
        got = product.compress(a, mode, param, ztype=ztype)
        assert _pipelined(product), "the slab pipeline did not run"
        assert got == want
        ref, _ = oracle.decompress_words(ow, a.shape, dtype, params)
        # with the index the slabs assembled, then without any index (scan)
        for index in (product.last_index, None):
            out, n = product.decompress(got, a.shape, dtype, mode, param, ztype=ztype, index=index)
            assert n == len(got)
            assert out.tobytes() == ref.tobytes()
            # fixed rate, or variable rate with its index: slab boundaries known up front, pipelined
            assert _pipelined(product) == (mode == "rate" or index is not None)
    finally:
        if product.last_index:
            product.lib.zfp_hip_index_free(product.last_index)
            product.last_index = None
        product.keep_index = True  # the fixture's setting (enable_index)


@pytest.mark.parametrize("mode,param", [("rate", 8), ("rate", 12), ("precision", 20), ("reversible", None)])
def test_pipelined_header_offset(product, oracle, slabs, mode, param):
    """zfpy layout: a 96-bit header first, so every slab starts at an unaligned bit."""
    a = _field((68, 64, 96), np.float32, 3)
    got = product.compress(a, mode, param, ztype=0, header=True)
    assert _pipelined(product)
    words = np.frombuffer(got + bytes((-len(got)) % 8), dtype=np.uint64).copy()
    params = _params(mode, param, 0, 3)
    ow, end = oracle.compress_words(a, params, bit_offset=96)
    words[0] = 0
    words[1] &= ~np.uint64((1 << 32) - 1)
    assert words[: len(ow)].tobytes() == ow.tobytes()
    out, _ = product.decompress(got, a.shape, np.float32, mode, param, ztype=0, header=True)
    ref, _ = oracle.decompress_words(ow, a.shape, np.float32, params, bit_offset=96)
    assert out.tobytes() == ref.tobytes()


def test_pipelined_double_and_one_shot_agree(product, slabs, monkeypatch):
    a = _field((72, 48, 64), np.float64, 9)
    for mode, param in (("rate", 24), ("precision", 32)):
        got = product.compress(a, mode, param, ztype=TYPE_DOUBLE)
        assert _pipelined(product)
        monkeypatch.setenv("ZFP_HIP_NO_PIPE", "1")
        one = product.compress(a, mode, param, ztype=TYPE_DOUBLE)
        assert not _pipelined(product)
        monkeypatch.delenv("ZFP_HIP_NO_PIPE")
        assert got == one, mode
