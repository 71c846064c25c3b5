"""Parity of the MI355X codec (libzfp.so -> libzfp_hip.so) with the oracle.

Every test calls the product through the C API exactly as the reference's own
end-to-end tests do (tests/src/endtoend/zfpEndtoendBase.c): field + stream +
mode, zfp_compress / zfp_decompress.  Bar: compressed streams and decompressed
arrays are bit-identical to the CPU oracle (which is itself pinned to the
reference's golden checksums and to the reference library in test_oracle.py).
"""
import ctypes
import zlib

import numpy as np
import pytest

from pyoracle import (TYPE_DOUBLE, TYPE_FLOAT, params_accuracy, params_precision, params_rate,
                      params_reversible)

pytestmark = pytest.mark.gpu


def _params(mode, param, ztype, dims):
    if mode == "rate":
        return params_rate(param, ztype, dims)
    if mode == "precision":
        return params_precision(param)
    if mode == "accuracy":
        return params_accuracy(param)
    if mode == "expert":
        return param
    return params_reversible()


def _oracle_bytes(oracle, arr, mode, param, ztype=None, box=None, bit_offset=0):
    zt = ztype if ztype is not None else (TYPE_FLOAT if arr.dtype == np.float32 else TYPE_DOUBLE)
    params = _params(mode, param, zt, arr.ndim)
    words, end = oracle.compress_words(arr, params, box=box, bit_offset=bit_offset)
    return words.view(np.uint8).tobytes()[: (end + 63) // 64 * 8], end


def _special_field(shape, dtype, rng):
    a = (rng.standard_normal(shape) * rng.choice([1e-3, 1.0, 1e5], size=shape)).astype(dtype)
    flat = a.reshape(-1)
    info = np.finfo(dtype)
    specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, info.tiny, info.tiny / 4, -info.tiny / 8,
                         info.max, -info.max], dtype=dtype)
    idx = rng.choice(flat.size, size=max(1, flat.size // 40), replace=False)
    flat[idx] = rng.choice(specials, size=idx.size)
    if min(shape) >= 8:
        a[:4, :4, :4] = info.tiny / 16
        a[4:8, :4, :4] = -0.0
        a[:4, 4:8, :4] = 0.0
        a[4:8, 4:8, :4] = np.nan
    return a


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("tname", ["float", "double"])
def test_golden_checksums_3d(product, oracle, golden, tname):
    """The reference's own golden stream + decompressed-array hashes (129^3)."""
    dtype = np.float32 if tname == "float" else np.float64
    field = oracle.smooth_field(3, dtype)
    cases = {}
    for e in golden:
        if e["dims"] == 3 and e["type"] == tname and e["subject"] != "input":
            cases.setdefault((e["mode"], e["param"]), {})[e["subject"]] = int(e["checksum"], 16)
    for (mode, param), want in sorted(cases.items(), key=str):
        ztype = 3 if tname == "float" else 4
        data = product.compress(field, mode, param, ztype=ztype)
        words = np.frombuffer(data, dtype=np.uint64)
        assert oracle.hash_words(words) == want["stream"], (mode, param)
        out, n = product.decompress(data, field.shape, dtype, mode, param, ztype=ztype, index=product.last_index)
        assert n == len(data), (mode, param)
        if "decompressed" in want:
            assert oracle.hash_array(out) == want["decompressed"], (mode, param)
        if product.last_index:
            product.lib.zfp_hip_index_free(product.last_index)
            product.last_index = None


MODES = [("rate", 16), ("rate", 8), ("rate", 1.5), ("rate", 5), ("precision", 12), ("precision", 32),
         ("accuracy", 1e-3), ("reversible", None), ("expert", (700, 900, 40, -60))]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("shape", [(7, 9, 10), (16, 16, 16), (12, 21, 70)])
@pytest.mark.parametrize("mode,param", MODES)
def test_stream_and_roundtrip_match_oracle(product, oracle, dtype, shape, mode, param):
    rng = np.random.default_rng(zlib.crc32(repr((shape, mode, param, np.dtype(dtype).name)).encode()))
    a = _special_field(shape, dtype, rng)
    ztype = TYPE_FLOAT if dtype == np.float32 else TYPE_DOUBLE
    want, end = _oracle_bytes(oracle, a, mode, param)
    got = product.compress(a, mode, param, ztype=ztype)
    assert got == want
    params = _params(mode, param, ztype, a.ndim)
    ref_out, _ = oracle.decompress_words(np.frombuffer(want, dtype=np.uint64), a.shape, dtype, params)
    out, n = product.decompress(got, a.shape, dtype, mode, param, ztype=ztype, index=product.last_index)
    assert n == len(got)
    assert out.tobytes() == ref_out.tobytes()
    if product.last_index:
        product.lib.zfp_hip_index_free(product.last_index)
        product.last_index = None


@pytest.mark.parametrize("mode,param", [("rate", 8), ("rate", 16), ("rate", 3.25), ("precision", 20),
                                        ("reversible", None)])
def test_header_offset_stream_matches_oracle(product, oracle, mode, param):
    """zfpy writes a 96-bit header first, so blocks start at bit 96 (unaligned)."""
    rng = np.random.default_rng(11)
    a = rng.standard_normal((20, 24, 36)).astype(np.float32)
    got = product.compress(a, mode, param, ztype=0, header=True)  # zfpy passes zfp_type_none
    words = np.frombuffer(got + bytes((-len(got)) % 8), dtype=np.uint64).copy()
    params = _params(mode, param, 0, 3)
    ow, end = oracle.compress_words(a, params, bit_offset=96)
    payload = words.copy()
    payload[0] = 0
    payload[1] &= ~np.uint64((1 << 32) - 1)
    assert payload[: len(ow)].tobytes() == ow.tobytes()
    assert len(got) == (end + 63) // 64 * 8
    out, _ = product.decompress(got, a.shape, np.float32, mode, param, ztype=0, header=True,
                                index=product.last_index)
    ref, _ = oracle.decompress_words(ow, a.shape, np.float32, params, bit_offset=96)
    assert out.tobytes() == ref.tobytes()


@pytest.mark.parametrize("pad", [1, 32, 64, 96, 100, 160, 255])
@pytest.mark.parametrize("dtype,mode,param", [(np.float32, "rate", 8), (np.float32, "rate", 16),
                                              (np.float64, "rate", 16), (np.float32, "rate", 12)])
def test_bit_offset_stream_matches_oracle(product, oracle, pad, dtype, mode, param):
    """Fixed-rate streams that start at any bit (the aligned encoder's copy-out
    funnel-shifts its run; 16-byte stores pair the out words by their address)."""
    rng = np.random.default_rng(pad)
    a = rng.standard_normal((21, 26, 72)).astype(dtype)
    got = product.compress(a, mode, param, pad_bits=pad)
    params = _params(mode, param, TYPE_FLOAT if dtype == np.float32 else TYPE_DOUBLE, 3)
    ow, end = oracle.compress_words(a, params, bit_offset=pad)
    words = np.frombuffer(got + bytes((-len(got)) % 8), dtype=np.uint64)
    assert words[: len(ow)].tobytes() == ow.tobytes()
    assert len(got) == (end + 63) // 64 * 8


@pytest.mark.parametrize("box", [[(0, 24), (0, 20), (8, 16)], [(8, 24), (4, 12), (0, 18)], [(4, 21), (0, 20), (16, 18)]])
@pytest.mark.parametrize("mode,param", [("rate", 8), ("precision", 16)])
def test_chunk_boxes_match_oracle(product, oracle, box, mode, param):
    """zfp_compress_chunk over a sub-box (fork chunk API), strided field as zfpy builds it."""
    rng = np.random.default_rng(5)
    a = rng.standard_normal((18, 20, 21)).astype(np.float32) if box[0][1] == 21 else \
        rng.standard_normal((18, 20, 24)).astype(np.float32)
    got = product.compress(a, mode, param, ztype=3, chunk=box, strided=True)
    want, end = _oracle_bytes(oracle, a, mode, param, ztype=3, box=box + [(0, 0)])
    assert got == want


def test_device_resident_buffers_match_host_path(product, oracle):
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(3)
    a = rng.standard_normal((64, 64, 64)).astype(np.float32)
    host = product.compress(a, "rate", 16, ztype=3)
    d_in = torch.from_numpy(a).cuda()
    cap = len(host) + 4096
    d_out = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    lib = product.lib
    field = lib.zfp_field_3d(ctypes.c_void_p(d_in.data_ptr()), 3, 64, 64, 64)
    zs = lib.zfp_stream_open(None)
    lib.zfp_stream_set_rate(zs, 16.0, 3, 3, 0)
    bs = lib.stream_open(ctypes.c_void_p(d_out.data_ptr()), cap)
    lib.zfp_stream_set_bit_stream(zs, bs)
    n = lib.zfp_compress(zs, field)
    assert n == len(host)
    assert d_out[:n].cpu().numpy().tobytes() == host
    # device decode into a device field
    d_back = torch.zeros_like(d_in)
    lib.zfp_field_set_pointer(field, ctypes.c_void_p(d_back.data_ptr()))
    lib.stream_rewind(bs)
    assert lib.zfp_decompress(zs, field) == n
    out, _ = product.decompress(host, a.shape, np.float32, "rate", 16)
    assert d_back.cpu().numpy().tobytes() == out.tobytes()
    lib.stream_close(bs)
    lib.zfp_stream_close(zs)
    lib.zfp_field_free(field)


def test_fixed_rate_large_field_bit_exact(product, oracle):
    """A field past the Infinity Cache size: 256^3 f32 rate 16 against the oracle."""
    x = np.arange(256, dtype=np.float32)
    a = (np.sin(0.05 * x)[None, None, :] * np.cos(0.03 * x)[None, :, None] +
         0.5 * np.sin(0.02 * x[:, None, None] + 0.01 * x[None, :, None] * x[None, None, :] / 256)).astype(np.float32)
    got = product.compress(a, "rate", 16, ztype=3)
    want, end = _oracle_bytes(oracle, a, "rate", 16)
    assert got == want


@pytest.mark.parametrize("slot_words,pool", [(3, None), (5, None), (9, None), (5, "7")])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("mode,param", [("precision", 32), ("precision", 12), ("accuracy", 1e-3),
                                        ("reversible", None)])
def test_short_slots_and_overflow_pool_match_oracle(product, oracle, monkeypatch, slot_words, pool, dtype, mode,
                                                   param):
    """Variable-rate 3D encoders with short LDS slots: blocks longer than their
    slot are coded again into the overflow pool (forced here with tiny slots);
    a pool that runs out makes the library redo the launch with full slots."""
    monkeypatch.setenv("ZFP_HIP_SLOT_WORDS", str(slot_words))
    if pool:
        monkeypatch.setenv("ZFP_HIP_OVF_POOL", pool)
    rng = np.random.default_rng(zlib.crc32(repr((slot_words, mode, param, np.dtype(dtype).name)).encode()))
    a = _special_field((40, 36, 33), dtype, rng)
    a[20:, :, :] = np.sin(np.arange(20 * 36 * 33, dtype=dtype) * 1e-3).reshape(20, 36, 33)  # short blocks too
    ztype = TYPE_FLOAT if dtype == np.float32 else TYPE_DOUBLE
    want, end = _oracle_bytes(oracle, a, mode, param)
    got = product.compress(a, mode, param, ztype=ztype)
    assert got == want
    params = _params(mode, param, ztype, a.ndim)
    ref_out, _ = oracle.decompress_words(np.frombuffer(want, dtype=np.uint64), a.shape, dtype, params)
    out, n = product.decompress(got, a.shape, dtype, mode, param, ztype=ztype, index=product.last_index)
    assert n == len(got)
    assert out.tobytes() == ref_out.tobytes()
    if product.last_index:
        product.lib.zfp_hip_index_free(product.last_index)
        product.last_index = None
