"""4D parity of the MI355X codec with the oracle (one 4^4 block per quad of lanes).

Same call sequence and bar as test_gpu_codec.py (the reference's end-to-end
tests, tests/src/endtoend/zfpEndtoendBase.c): zfp_compress / zfp_decompress
through the C API; streams and decompressed arrays bit-identical to the CPU
oracle, which test_oracle.py pins to the reference's 4dFloat golden checksums.
BASELINE C5 (512^4 f32 reversible) runs this path at scale.
"""
import zlib

import numpy as np
import pytest

from pyoracle import TYPE_DOUBLE, TYPE_FLOAT
from test_gpu_codec import MODES, _oracle_bytes, _params

pytestmark = pytest.mark.gpu


def _field4(shape, dtype, rng):
    a = (rng.standard_normal(shape) * rng.choice([1e-3, 1.0, 1e5], size=shape)).astype(dtype)
    flat = a.reshape(-1)
    info = np.finfo(dtype)
    specials = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, info.tiny, info.tiny / 4, -info.tiny / 8,
                         info.max, -info.max], dtype=dtype)
    idx = rng.choice(flat.size, size=max(1, flat.size // 50), replace=False)
    flat[idx] = rng.choice(specials, size=idx.size)
    if min(shape) >= 8:
        a[:4, :4, :4, :4] = info.tiny / 16
        a[4:8, :4, :4, :4] = -0.0
        a[:4, 4:8, :4, :4] = 0.0
        a[4:8, 4:8, :4, :4] = np.nan
    return a


def _free_index(product):
    if product.last_index:
        product.lib.zfp_hip_index_free(product.last_index)
        product.last_index = None


def test_golden_checksums_4d_float(product, oracle, golden):
    """The reference's own 4dFloat golden stream + decompressed-array hashes."""
    field = oracle.smooth_field(4, np.float32)
    cases = {}
    for e in golden:
        if e["dims"] == 4 and e["type"] == "float" and e["subject"] != "input":
            cases.setdefault((e["mode"], e["param"]), {})[e["subject"]] = int(e["checksum"], 16)
    assert cases
    for (mode, param), want in sorted(cases.items(), key=str):
        data = product.compress(field, mode, param, ztype=3)
        words = np.frombuffer(data, dtype=np.uint64)
        assert oracle.hash_words(words) == want["stream"], (mode, param)
        out, n = product.decompress(data, field.shape, np.float32, mode, param, ztype=3, index=product.last_index)
        assert n == len(data), (mode, param)
        if "decompressed" in want:
            assert oracle.hash_array(out) == want["decompressed"], (mode, param)
        _free_index(product)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("shape", [(4, 4, 4, 4), (5, 6, 7, 9), (9, 3, 4, 21), (8, 8, 8, 12)])
@pytest.mark.parametrize("mode,param", MODES)
def test_stream_and_roundtrip_match_oracle_4d(product, oracle, dtype, shape, mode, param):
    rng = np.random.default_rng(zlib.crc32(repr((shape, mode, param, np.dtype(dtype).name, 4)).encode()))
    a = _field4(shape, dtype, rng)
    ztype = TYPE_FLOAT if dtype == np.float32 else TYPE_DOUBLE
    want, end = _oracle_bytes(oracle, a, mode, param)
    got = product.compress(a, mode, param, ztype=ztype)
    assert got == want
    params = _params(mode, param, ztype, a.ndim)
    ref_out, _ = oracle.decompress_words(np.frombuffer(want, dtype=np.uint64), a.shape, dtype, params)
    out, n = product.decompress(got, a.shape, dtype, mode, param, ztype=ztype, index=product.last_index)
    assert n == len(got)
    assert out.tobytes() == ref_out.tobytes()
    _free_index(product)


@pytest.mark.parametrize("mode,param", [("rate", 8), ("rate", 3.25), ("reversible", None)])
def test_header_offset_stream_matches_oracle_4d(product, oracle, mode, param):
    """zfpy's 96-bit header first: 4D blocks start at bit 96."""
    rng = np.random.default_rng(13)
    a = rng.standard_normal((6, 8, 9, 10)).astype(np.float32)
    got = product.compress(a, mode, param, ztype=0, header=True)
    words = np.frombuffer(got + bytes((-len(got)) % 8), dtype=np.uint64).copy()
    params = _params(mode, param, 0, 4)
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
    _free_index(product)


@pytest.mark.parametrize("box", [[(0, 8), (4, 12), (0, 9), (4, 8)], [(4, 13), (0, 8), (4, 9), (0, 6)]])
@pytest.mark.parametrize("mode,param", [("rate", 8), ("precision", 16), ("reversible", None)])
def test_chunk_boxes_match_oracle_4d(product, oracle, box, mode, param):
    """zfp_compress_chunk over a 4D sub-box, strided field as zfpy builds it."""
    rng = np.random.default_rng(7)
    a = rng.standard_normal((8, 9, 12, 13)).astype(np.float32)
    got = product.compress(a, mode, param, ztype=3, chunk=box, strided=True)
    want, end = _oracle_bytes(oracle, a, mode, param, ztype=3, box=box)
    assert got == want
    _free_index(product)


def test_reversible_lossless_4d(product, oracle):
    """C5's mode on the reference's smooth 4D field: lossless and bit-exact."""
    a = oracle.smooth_field(4, np.float32)
    got = product.compress(a, "reversible", None, ztype=3)
    want, _ = _oracle_bytes(oracle, a, "reversible", None)
    assert got == want
    out, n = product.decompress(got, a.shape, np.float32, "reversible", None, ztype=3, index=product.last_index)
    assert n == len(got)
    assert out.tobytes() == a.tobytes()
    _free_index(product)


@pytest.mark.parametrize("slot_words,pool", [(9, None), (21, None), (9, "3")])
@pytest.mark.parametrize("mode,param", [("precision", 20), ("accuracy", 1e-3), ("reversible", None)])
def test_short_slots_and_patch_pass_match_oracle_4d(product, oracle, monkeypatch, slot_words, pool, mode, param):
    """Short-slot 4D encoder: blocks longer than their LDS slot are packed
    truncated, listed, and ORed in whole by encode4_patch (forced here with
    tiny slots); an exhausted list makes the library redo the launch with
    full-size slots.  The exchange areas are shared by quad pairs (HALF)."""
    monkeypatch.setenv("ZFP_HIP_SLOT_WORDS", str(slot_words))
    if pool:
        monkeypatch.setenv("ZFP_HIP_OVF_POOL", pool)
    rng = np.random.default_rng(zlib.crc32(repr((slot_words, mode, param, 4)).encode()))
    a = _field4((12, 9, 16, 20), np.float32, rng)
    a[8:] = np.cos(np.arange(4 * 9 * 16 * 20, dtype=np.float32) * 1e-3).reshape(4, 9, 16, 20)  # short blocks too
    want, end = _oracle_bytes(oracle, a, mode, param)
    got = product.compress(a, mode, param, ztype=TYPE_FLOAT)
    assert got == want
    params = _params(mode, param, TYPE_FLOAT, a.ndim)
    ref_out, _ = oracle.decompress_words(np.frombuffer(want, dtype=np.uint64), a.shape, np.float32, params)
    out, n = product.decompress(got, a.shape, np.float32, mode, param, ztype=TYPE_FLOAT, index=product.last_index)
    assert n == len(got)
    assert out.tobytes() == ref_out.tobytes()
    _free_index(product)


@pytest.mark.parametrize("pack_words", ["1666", "1100", "400", "full"])
@pytest.mark.parametrize("mode,param", [("precision", 20), ("accuracy", 1e-3), ("reversible", None)])
def test_packed_staging_decode_matches_oracle_4d(product, oracle, monkeypatch, pack_words, mode, param):
    """Variable-rate decode4 stages each wave's blocks back to back (the
    default, sized for 16 worst-case blocks).  With fewer staged words forced
    (ZFP_HIP_PACK_WORDS), waves whose segment exceeds them (the rough half of
    the field) make the library repeat the launch with padded slots for them;
    "full": padded slots only (ZFP_HIP_FULL_SLOTS).  (Decoding such a wave in
    two passes of eight blocks inside the first launch measured slower -- C5
    29.4 against 28.6 ms -- as its second decode body spills registers.)"""
    if pack_words == "full":
        monkeypatch.setenv("ZFP_HIP_FULL_SLOTS", "1")
    else:
        monkeypatch.setenv("ZFP_HIP_PACK_WORDS", pack_words)
    rng = np.random.default_rng(zlib.crc32(repr((pack_words, mode, param, 44)).encode()))
    a = _field4((12, 9, 16, 20), np.float32, rng)
    a[6:] = np.cos(np.arange(6 * 9 * 16 * 20, dtype=np.float32) * 1e-3).reshape(6, 9, 16, 20)
    want, end = _oracle_bytes(oracle, a, mode, param)
    params = _params(mode, param, TYPE_FLOAT, a.ndim)
    ref_out, _ = oracle.decompress_words(np.frombuffer(want, dtype=np.uint64), a.shape, np.float32, params)
    out, n = product.decompress(want, a.shape, np.float32, mode, param, ztype=TYPE_FLOAT)  # scan-built index
    assert n == len(want)
    assert out.tobytes() == ref_out.tobytes()


def _mixed_blocks4(pattern, rng):
    """A 4D f32 field in whole 4^4 blocks, raster block order (x fastest): block
    i is random normal data when pattern[i] (it fails the reversible cast: the
    bits-reinterpreting header, ~8,300 bits) and integer-valued smooth data
    otherwise (passes the cast, a few thousand bits at most)."""
    nbx, nby, nbz = 4, 4, 2
    nbw = -(-len(pattern) // (nbx * nby * nbz))
    shape = (4 * nbw, 4 * nbz, 4 * nby, 4 * nbx)
    i = np.indices(shape).astype(np.float32)
    a = np.round(900 * np.cos(0.07 * i[3] + 0.05 * i[2]) * np.sin(0.03 * i[1] + 0.02 * i[0]))
    a = a.astype(np.float32)
    pat = np.zeros(nbw * nbz * nby * nbx, dtype=bool)
    pat[:len(pattern)] = pattern
    blk = a.reshape(nbw, 4, nbz, 4, nby, 4, nbx, 4)
    for b in np.flatnonzero(pat):
        bx, by, bz, bw = b % nbx, b // nbx % nby, b // (nbx * nby) % nbz, b // (nbx * nby * nbz)
        blk[bw, :, bz, :, by, :, bx, :] = rng.standard_normal((4, 4, 4, 4))
    return a


@pytest.mark.parametrize("slot_words", [None, "75", "131"])
def test_big_and_small_slots_4d_reversible(product, oracle, monkeypatch, slot_words):
    """f32 reversible encode4 with short slots: the blocks of a wave that fail the
    reversible cast get full slots and the others share the rest of the region
    (kernels4.h place); waves with more such blocks than fit (here 7, 8, 16 of
    16 with the default 93-word slots) send the rest to the overflow list and
    encode4_patch.  Waves of 0, 1, 2, 5, 6, 7, 8 and 16 long blocks, stream and
    lossless round trip against the oracle; forced slot sizes move the limit."""
    if slot_words:
        monkeypatch.setenv("ZFP_HIP_SLOT_WORDS", slot_words)
    rng = np.random.default_rng(2024)
    pattern = []
    for k in (0, 1, 2, 5, 6, 7, 8, 16, 3):
        wave = np.zeros(16, dtype=bool)
        wave[rng.choice(16, size=k, replace=False)] = True
        pattern.extend(wave)
    a = _mixed_blocks4(pattern, rng)
    want, _ = _oracle_bytes(oracle, a, "reversible", None)
    got = product.compress(a, "reversible", None, ztype=TYPE_FLOAT)
    assert got == want
    out, n = product.decompress(got, a.shape, np.float32, "reversible", None, ztype=TYPE_FLOAT,
                                index=product.last_index)
    assert n == len(got)
    assert out.tobytes() == a.tobytes()
    _free_index(product)
