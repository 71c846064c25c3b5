"""Variable-rate streams decoded without a block index (scan.h).

The reference decodes any stream serially (src/template/decompress.c:66-140,
decode.c:69-246, revdecode.c:34-52), so a drop-in decoder must accept streams
it did not produce: from the reference library, from a file, from another
process.  Here no index is ever attached: the GPU finds the block starts by
its resynchronising parse, then decodes.  Bar: decompressed arrays bit-exact
against the oracle (pinned to the reference in test_oracle.py) -- and, for
streams made by the reference itself (oracle/_ref), through the C API, through
zfpy.decompress_numpy and through the CLI in a fresh process.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from pyoracle import (TYPE_DOUBLE, TYPE_FLOAT, params_accuracy, params_precision, params_reversible)

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(REPO, "zfp-par_amd", "bin", "zfp")


def _oracle_decode(oracle, data, shape, dtype, params, bit_offset=0, box=None):
    words = np.frombuffer(bytes(data) + bytes(-len(data) % 8), dtype=np.uint64)
    return oracle.decompress_words(words, shape, dtype, params, box=box, bit_offset=bit_offset)


def _ref_stream(ref_capi, arr, mode, param=None, header=False):
    return ref_capi.compress(arr, mode, param, header=header)


# ---- streams made by the reference itself (oracle/_ref) --------------------
REF_CASES = [
    # (name, dims, dtype, mode, param, oracle params)
    ("129^3 f64 precision 32", 3, np.float64, "precision", 32, params_precision(32)),
    ("33^4 f32 reversible", 4, np.float32, "reversible", None, params_reversible()),
]


@pytest.mark.parametrize("case", REF_CASES, ids=[c[0] for c in REF_CASES])
def test_reference_stream_decodes_through_c_api(product, oracle, ref_capi, case):
    name, dims, dtype, mode, param, params = case
    arr = oracle.smooth_field(dims, dtype)
    data = _ref_stream(ref_capi, arr, mode, param)
    want, end = _oracle_decode(oracle, data, arr.shape, dtype, params)
    got, n = product.decompress(data, arr.shape, dtype, mode, param)  # no index attached
    assert n == (end + 63) // 64 * 8
    assert got.tobytes() == want.tobytes()
    scan = product.last_scan()
    assert scan is not None, "decompress of a foreign stream must scan"
    print("%s: %d B stream, scan %.3f ms in %d passes" % (name, len(data), scan[0], scan[1]))


@pytest.mark.parametrize("case", REF_CASES, ids=[c[0] for c in REF_CASES])
def test_reference_stream_decodes_through_zfpy(product, oracle, ref_capi, case):
    import zfpy
    name, dims, dtype, mode, param, params = case
    arr = oracle.smooth_field(dims, dtype)
    data = _ref_stream(ref_capi, arr, mode, param, header=True)
    hdr_bits = 96 if mode != "expert" else 148
    want, _ = _oracle_decode(oracle, data, arr.shape, dtype, params, bit_offset=hdr_bits)
    got = zfpy.decompress_numpy(bytes(data))  # plain bytes: no index anywhere
    assert got.dtype == dtype and got.shape == arr.shape
    assert got.tobytes() == want.tobytes()


@pytest.mark.parametrize("case", REF_CASES, ids=[c[0] for c in REF_CASES])
def test_reference_stream_decodes_through_cli_fresh_process(product, oracle, ref_capi, case, tmp_path):
    name, dims, dtype, mode, param, params = case
    arr = oracle.smooth_field(dims, dtype)
    data = _ref_stream(ref_capi, arr, mode, param, header=True)
    want, _ = _oracle_decode(oracle, data, arr.shape, dtype, params, bit_offset=96)
    zpath, opath = tmp_path / "in.zfp", tmp_path / "out.raw"
    zpath.write_bytes(data)
    r = subprocess.run([CLI, "-z", str(zpath), "-h", "-o", str(opath)], capture_output=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert opath.read_bytes() == want.tobytes()


# ---- product streams, every variable-rate mode, no index -------------------
def _field(shape, dtype, rng, kind):
    if kind == "smooth":
        g = np.meshgrid(*[np.arange(n) for n in shape], indexing="ij")
        v = np.sin(0.07 * g[-1]) * np.cos(0.05 * g[-2]) + 0.5 * np.sin(0.03 * g[0] + 0.001 * g[-1] * g[-2])
        return v.astype(dtype)
    if kind == "rough":
        return rng.standard_normal(shape).astype(dtype)
    a = rng.standard_normal(shape).astype(dtype)  # sparse: zero slabs give runs of 1-bit blocks
    a[..., : shape[-1] // 2] = 0
    return a


MODES = [("precision", 16, params_precision(16)), ("precision", 32, params_precision(32)),
         ("accuracy", 1e-3, params_accuracy(1e-3)), ("reversible", None, params_reversible())]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("shape", [(37, 45, 52), (64, 64, 64), (9, 10, 11, 13), (16, 20, 24, 12)])
@pytest.mark.parametrize("mode,param,params", MODES)
@pytest.mark.parametrize("kind", ["smooth", "rough", "sparse"])
def test_product_stream_decodes_without_index(product, oracle, dtype, shape, mode, param, params, kind):
    rng = np.random.default_rng(hash((shape, kind)) & 0xffff)
    arr = _field(shape, dtype, rng, kind)
    data = product.compress(arr, mode, param)
    if product.last_index:
        product.lib.zfp_hip_index_free(product.last_index)
        product.last_index = None
    want, end = _oracle_decode(oracle, data, shape, dtype, params)
    got, n = product.decompress(data, shape, dtype, mode, param)
    assert n == (end + 63) // 64 * 8
    assert got.tobytes() == want.tobytes()


@pytest.mark.parametrize("seg_bits", ["64", "512", "4096"])
def test_small_segments_force_many_passes(product, oracle, seg_bits, monkeypatch):
    """Tiny segments: almost no speculative chain merges inside its segment, so
    exits move pass after pass (the serial worst case of the algorithm)."""
    monkeypatch.setenv("ZFP_HIP_SCAN_SEG_BITS", seg_bits)
    arr = oracle.smooth_field(3, np.float64, min_total=40000)
    data = product.compress(arr, "precision", 24)
    want, _ = _oracle_decode(oracle, data, arr.shape, np.float64, params_precision(24))
    got, _ = product.decompress(data, arr.shape, np.float64, "precision", 24)
    assert got.tobytes() == want.tobytes()
    assert product.last_scan()[1] >= 2


def test_stale_index_of_another_chunk_is_not_used(product, oracle):
    """Two chunks coded into one stream: the stream's index describes the last
    chunk only, so decoding the first chunk must not use it."""
    rng = np.random.default_rng(3)
    arr = rng.standard_normal((32, 32, 32)).astype(np.float32)
    import ctypes
    lib = product.lib
    field = product.field_for(arr)
    zs = lib.zfp_stream_open(None)
    lib.zfp_stream_set_precision(zs, 20)
    cap = lib.zfp_stream_maximum_size(zs, field) * 2 + 64
    buf = np.zeros(cap, dtype=np.uint8)
    bs = lib.stream_open(buf.ctypes.data, cap)
    lib.zfp_stream_set_bit_stream(zs, bs)
    lib.zfp_stream_rewind(zs)
    boxes = [[(0, 32), (0, 32), (0, 16)], [(0, 32), (0, 32), (16, 32)]]  # equal block counts
    for box in boxes:
        ck = product.make_chunk(3, box)
        assert lib.zfp_compress_chunk(zs, ck, field)
        lib.zfp_chunk_free(ck)
    n = lib.stream_size(bs)
    # decode the FIRST chunk with the stream's (second-chunk) index still attached
    out = np.zeros_like(arr)
    ofield = product.field_for(out)
    lib.zfp_stream_rewind(zs)
    ck = product.make_chunk(3, boxes[0])
    assert lib.zfp_decompress_chunk(zs, ck, ofield)
    lib.zfp_chunk_free(ck)
    words = np.frombuffer(bytes(buf[:n]), dtype=np.uint64)
    want = np.zeros_like(arr)
    oracle.decompress_words(words, arr.shape, np.float32, params_precision(20),
                            box=[(0, 32), (0, 32), (0, 16), (0, 0)], out=want)
    assert out[:16].tobytes() == want[:16].tobytes()
    lib.stream_close(bs)
    lib.zfp_stream_close(zs)
    lib.zfp_field_free(field)
    lib.zfp_field_free(ofield)


def test_truncated_stream_fails_cleanly(product, oracle):
    rng = np.random.default_rng(5)
    arr = rng.standard_normal((32, 32, 32)).astype(np.float64)
    data = product.compress(arr, "precision", 32)
    _, n = product.decompress(data[: len(data) // 3], arr.shape, np.float64, "precision", 32)
    assert n == 0


def test_scan_matches_encoder_index_at_scale(product, oracle):
    """256^3 f64 precision 32 (16 MiB of doubles): the decode without an index
    equals the decode with the encoder's index; prints the scan time."""
    g = np.meshgrid(*[np.arange(256)] * 3, indexing="ij")
    arr = (np.sin(0.05 * g[2]) * np.cos(0.03 * g[1]) + 0.5 * np.sin(0.02 * g[0] + 0.01 * g[2] * g[1] / 256))
    data = product.compress(arr, "precision", 32)
    idx = product.last_index
    with_idx, n1 = product.decompress(data, arr.shape, np.float64, "precision", 32, index=idx)
    product.lib.zfp_hip_index_free(idx)
    product.last_index = None
    no_idx, n2 = product.decompress(data, arr.shape, np.float64, "precision", 32)
    assert n1 == n2 == len(data)
    assert with_idx.tobytes() == no_idx.tobytes()
    ms, passes = product.last_scan()
    print("256^3 f64 precision 32: %d B, scan %.3f ms, %d passes" % (len(data), ms, passes))


def _field4(n, dtype):
    """The C5-mode 4D field at n^4 (tools/kprof.py field4): F1 + .25 cos(.04 w)."""
    x = np.arange(n, dtype=np.float64)
    base = np.sin(0.05 * x)[None, :] * np.cos(0.03 * x)[:, None]
    xy = 0.01 * x[None, :] * x[:, None] / n
    f3 = base[None] + 0.5 * np.sin(0.02 * x[:, None, None] + xy[None])
    return np.stack([(f3 + 0.25 * np.cos(0.04 * w)).astype(dtype) for w in range(n)])


@pytest.mark.parametrize("plausible", ["1", "0"])
@pytest.mark.parametrize("n,dtype,mode,param,params", [
    (64, np.float32, "reversible", None, params_reversible()),
    (48, np.float64, "precision", 32, params_precision(32)),
])
def test_scan_4d_at_scale_matches_index_and_oracle(product, oracle, n, dtype, mode, param, params, plausible,
                                                   monkeypatch):
    """Regression guard for the round-3 4D scan bug (a long group section's
    reference-loop fallback restarted behind the forward-only ring reader, so
    large 4D streams were indexed wrongly): a 4D stream of tens of megabytes is
    decoded once with the encoder's index and once with none (the scan); both
    equal the oracle's decode, and the second call really scanned
    (src/template/decompress.c:105-140 is the serial walk this replaces).  With
    pass 1's plausible chain starts and phase-A refusals (the default) and
    without them (ZFP_HIP_SCAN_PLAUSIBLE=0)."""
    monkeypatch.setenv("ZFP_HIP_SCAN_PLAUSIBLE", plausible)
    arr = _field4(n, dtype)
    data = product.compress(arr, mode, param)
    idx = product.last_index
    assert idx
    with_idx, n1 = product.decompress(data, arr.shape, dtype, mode, param, index=idx)
    product.lib.zfp_hip_index_free(idx)
    product.last_index = None
    assert product.last_scan() is None, "a matching encoder index must not be rescanned"
    no_idx, n2 = product.decompress(data, arr.shape, dtype, mode, param)
    scan = product.last_scan()
    assert scan is not None, "a stream without an index must be scanned"
    assert n1 == n2 == len(data)
    want, end = _oracle_decode(oracle, data, arr.shape, dtype, params)
    assert n1 == (end + 63) // 64 * 8
    assert with_idx.tobytes() == want.tobytes()
    assert no_idx.tobytes() == want.tobytes()
    if mode == "reversible":
        assert no_idx.tobytes() == arr.tobytes()
    print("%d^4 %s %s: %d B stream, scan %.3f ms in %d passes" % (n, np.dtype(dtype).name, mode, len(data),
                                                                 scan[0], scan[1]))


@pytest.mark.parametrize("shape,dtype,mode,param,params", [
    ((40, 44, 48), np.float64, "precision", 32, params_precision(32)),
    ((12, 16, 16, 20), np.float32, "reversible", None, params_reversible()),
])
def test_stale_index_with_matching_fingerprint_is_detected(product, oracle, shape, dtype, mode, param, params):
    """an index whose fingerprint (stream words sampled, total bits)
    matches but whose block lengths do not -- here two adjacent blocks of one
    wave, one 3 bits longer and the next 3 bits shorter, so every wave start and
    the total are unchanged -- must not decode wrong data.  The decode kernels
    compare every block's decoded length with its index entry; a difference
    makes the call decode again after a scan (zfp_hip_last_stale_index)."""
    import ctypes
    rng = np.random.default_rng(21)
    arr = _field(shape, dtype, rng, "smooth")
    data = product.compress(arr, mode, param)
    idx = product.last_index
    lib = product.lib
    n = lib.zfp_hip_index_export(idx, None, 0)
    blob = ctypes.create_string_buffer(n)
    assert lib.zfp_hip_index_export(idx, blob, n) == n
    lib.zfp_hip_index_free(idx)
    product.last_index = None
    want, _ = _oracle_decode(oracle, data, shape, dtype, params)
    # the exported index as is: decoded with it, no scan, not stale
    good = lib.zfp_hip_index_import(blob, n)
    got, _ = product.decompress(data, shape, dtype, mode, param, index=good)
    assert got.tobytes() == want.tobytes()
    assert product.last_scan() is None and lib.zfp_hip_last_stale_index() == 0
    lib.zfp_hip_index_free(good)
    # two adjacent lengths changed by +-3 (header: 10 words, then uint16 lengths)
    raw = bytearray(blob.raw)
    lens = np.frombuffer(raw, dtype=np.uint16, count=int(np.frombuffer(raw, np.uint64, 2)[1]), offset=80).copy()
    lens[5] += 3
    lens[6] -= 3
    raw[80:80 + lens.nbytes] = lens.tobytes()
    bad = lib.zfp_hip_index_import(bytes(raw), n)
    assert bad
    got, nb = product.decompress(data, shape, dtype, mode, param, index=bad)
    lib.zfp_hip_index_free(bad)
    assert nb == len(data)
    assert lib.zfp_hip_last_stale_index() == 1
    assert product.last_scan() is not None
    assert got.tobytes() == want.tobytes()


GOOD_INDEX_CASES = [(shape, dt, mode, param) for shape in [(8, 12, 8, 20)]
                    for dt in (np.float32, np.float64, np.int32, np.int64)
                    for mode, param in (("precision", 20), ("accuracy", 1e-3), ("reversible", None))
                    if not (np.issubdtype(dt, np.integer) and mode == "accuracy")]
GOOD_INDEX_CASES += [((1000,), np.float32, "precision", 16), ((40, 52), np.float64, "reversible", None),
                     ((30, 33, 35), np.float32, "reversible", None)]


@pytest.mark.parametrize("shape,dtype,mode,param", GOOD_INDEX_CASES,
                         ids=["%dD-%s-%s" % (len(c[0]), np.dtype(c[1]).name, c[2]) for c in GOOD_INDEX_CASES])
def test_encoder_index_is_never_flagged_stale(product, shape, dtype, mode, param):
    """every decoder checks each block's decoded length against the
    caller's index (a mismatch means a stale index: rescan, decode again).  An
    off-by-one in any decoder's `used` would flag every correct index and
    silently decode twice; so for each block kind -- 4D float/double/int32/int64
    in the variable-rate modes, and 1D/2D/3D -- the encoder's own index must
    decode without a scan and without the stale flag, to the same array as the
    scan-built index."""
    rng = np.random.default_rng(7)
    i = np.arange(int(np.prod(shape)), dtype=np.float64).reshape(shape)
    smooth = np.sin(0.011 * i) + 0.3 * np.cos(0.0007 * i)
    if np.issubdtype(dtype, np.integer):
        arr = (smooth * 1e5 + rng.integers(-50, 50, shape)).astype(dtype)
    else:
        arr = (smooth + 1e-3 * rng.standard_normal(shape)).astype(dtype)
    data = product.compress(arr, mode, param)
    idx = product.last_index
    assert idx
    lib = product.lib
    with_idx, n1 = product.decompress(data, shape, dtype, mode, param, index=idx)
    assert product.last_scan() is None
    assert lib.zfp_hip_last_stale_index() == 0
    lib.zfp_hip_index_free(idx)
    product.last_index = None
    no_idx, n2 = product.decompress(data, shape, dtype, mode, param)
    assert product.last_scan() is not None
    assert n1 == n2 == len(data)
    assert with_idx.tobytes() == no_idx.tobytes()
    if mode == "reversible":
        assert with_idx.tobytes() == arr.tobytes()
