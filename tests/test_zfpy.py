"""zfpy surface: chunk partitioner, zfp_parallel, whole-array
compress_numpy/decompress_numpy, header(), and the multi-rank shard + gather.

CPU tests: the partitioner against the reference library built from source
(oracle/_ref, when present) and against the partitions SURVEY a19 verified on
the reference; header parsing; the rank sharding and the stream gather over
gloo with world_size 2.  GPU tests: every chunk stream is the whole-field
header followed by exactly the oracle's blocks of that chunk; decompression
into the shared array equals the oracle's decode; for z-slab chunks the
payloads concatenate to the whole-field payload ([verified] on the
reference).
"""
import ctypes
import os
import types

import numpy as np
import pytest

import zfpy
from zfpy import distributed as zdist
from zfpy.zfpy_c import _Chunks
from pyoracle import REF_SO, params_precision, params_rate, params_reversible


def _boxes(lib, shape_np, chunks_per_block, method):
    nd = len(shape_np)
    nsize = (ctypes.c_int * nd)(*[int(shape_np[nd - 1 - i]) for i in range(nd)])
    lib.zfp_optimal_parts_from_size.restype = ctypes.c_void_p
    lib.zfp_optimal_parts_from_size.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_float, ctypes.c_int]
    lib.zfp_chunks_from_blocks.restype = ctypes.c_void_p
    lib.zfp_chunks_from_blocks.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    blocks = lib.zfp_optimal_parts_from_size(nd, nsize, ctypes.c_float(chunks_per_block), method)
    chunks = lib.zfp_chunks_from_blocks(nd, nsize, blocks)
    cs = ctypes.cast(chunks, ctypes.POINTER(_Chunks)).contents
    out = []
    for i in range(cs.nchunks):
        c = cs.chunks[i].contents
        out.append(((c.fx, c.ex), (c.fy, c.ey), (c.fz, c.ez), (c.fw, c.ew)))
    return out


def _chunkit(shape, nparts, dtype=np.float32, method="BEST_CACHE"):
    nblocks = int(np.prod([(n + 3) // 4 for n in shape]))
    return zfpy.zfp_chunkit(types.SimpleNamespace(shape=shape, dtype=np.dtype(dtype)), nblocks / nparts, method)


# ---------------- CPU: partitioner ----------------

@pytest.mark.parametrize("shape,nparts,planes", [
    ((512, 4096, 4096), 8, [64] * 8),            # C4: 8 z-slabs of 64 planes
    ((512, 512, 512, 512), 8, [64] * 8),          # C5: 8 w-slabs of 64 (numpy order w,z,y,x)
    ((1024, 1024, 1024), 8, [128] * 8),
    ((129, 129, 129), 8, [12, 12, 12, 16, 16, 16, 16, 16, 13]),
])
def test_chunk_partition_matches_reference_facts(shape, nparts, planes):
    ck = _chunkit(shape, nparts)
    assert ck.get_nchunks() == len(planes)
    slow = 3 if len(shape) == 4 else 2  # index of the slowest zfp axis in a box
    got = [b[slow][1] - b[slow][0] for b in ck.boxes]
    assert got == planes
    for b in ck.boxes:  # other axes whole
        for a in range(len(shape)):
            if a != slow:
                assert b[a] == (0, shape[len(shape) - 1 - a])


@pytest.mark.parametrize("shape", [(64, 64, 64), (33, 40, 129), (17, 5, 300), (20, 24, 28, 32)])
@pytest.mark.parametrize("nparts", [1, 2, 3, 4, 8, 16])
def test_chunk_partition_matches_reference_library(shape, nparts):
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref not built")
    ref = ctypes.CDLL(REF_SO)
    nblocks = int(np.prod([(n + 3) // 4 for n in shape]))
    ck = _chunkit(shape, nparts)
    assert ck.boxes == _boxes(ref, shape, nblocks / nparts, 1)


def test_zfp_parallel_partition_rules():
    # nparts: chunks_per_block = nblocks / nparts; block_size uses 2^ndim (reference _zfp_par.py:55)
    zp = zfpy.zfp_parallel((64, 64, 64), "float32", nparts=4)
    assert zp.get_chunkit().get_nchunks() == 4
    zb = zfpy.zfp_parallel((64, 64, 64), "float32", est_compression_rate=2, block_size=8192)
    # compress_block_size = 2^3 * 4 / 2 = 16 B -> chunks_per_block = 8192 / 16 = 512 -> 4096 / 512 = 8 parts
    assert zb.get_chunkit().get_nchunks() == 8
    with pytest.raises(ValueError):
        zfpy.zfp_parallel((4, 4), "float16", nparts=1)
    with pytest.raises(ValueError):
        zfpy.zfp_parallel((4, 4, 4, 4, 4), "float32", nparts=1)
    with pytest.raises(ValueError):
        zfpy.zfp_parallel((4, 4), "float32")
    assert zp.get_numpy_array().shape == (64, 64, 64)
    assert zp.get_numpy_array().dtype == np.float32


# ---------------- CPU: rank sharding and the gather (gloo, world 2) ----------------

def test_rank_chunks_cover_every_chunk_once():
    for n in (1, 7, 8, 9, 64):
        for world in (1, 2, 3, 8):
            owned = sorted(i for r in range(world) for i in zdist.rank_chunks(n, world, r))
            assert owned == list(range(n))


def _gather_worker(rank, world, port, nchunks, q, sub):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # sub: the gather runs on the subgroup of global ranks 1..world-1 (its
        # rank 0 is global rank 1): point-to-point peers must be global ranks
        group = dist.new_group(list(range(1, world))) if sub else None
        if sub and rank == 0:
            q.put(None)
            return
        grank, gworld = dist.get_rank(group), dist.get_world_size(group)
        local = {}
        for i in zdist.rank_chunks(nchunks, gworld, grank):
            local[i] = zfpy.zfpy_c.ZfpBytes(bytes([i % 251]) * (100 + 37 * i))
            if i % 2:  # variable-rate chunks carry their block index
                local[i].block_index = bytes([(7 * i) % 256]) * (50 + i)
        out = zdist.gather_streams(local, nchunks, dst=0, group=group)
        if grank == 0:
            q.put([(bytes(s), getattr(s, "block_index", None), type(s) is bytes) for s in out])
        else:
            q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,sub", [(2, False), (3, False), (3, True)])
def test_gather_streams_gloo(world, sub):
    import multiprocessing as mp
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    nchunks = 9
    ps = [ctx.Process(target=_gather_worker, args=(r, world, port, nchunks, q, sub)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    root = [r for r in res if r is not None]
    assert len(root) == 1 and res.count(None) == world - 1
    got = root[0]
    assert len(got) == nchunks
    for i, (s, blob, plain) in enumerate(got):
        assert s == bytes([i % 251]) * (100 + 37 * i)
        assert blob == (bytes([(7 * i) % 256]) * (50 + i) if i % 2 else None)
        assert plain == (i % 2 == 0)  # chunks without an index come back as plain bytes


# ---------------- CPU: header() ----------------

def test_header_of_header_only_stream():
    from capi import ZfpCAPI
    api = ZfpCAPI(os.path.join(os.path.dirname(zfpy.__file__), "..", "lib", "libzfp.so"))
    lib = api.lib
    f = lib.zfp_field_3d(None, 3, 40, 30, 20)
    zs = lib.zfp_stream_open(None)
    lib.zfp_stream_set_rate(zs, 8.0, 0, 3, 0)
    buf = np.zeros(64, dtype=np.uint8)
    bs = lib.stream_open(buf.ctypes.data, 64)
    lib.zfp_stream_set_bit_stream(zs, bs)
    assert lib.zfp_write_header(zs, f, 7) == 96
    lib.stream_flush(bs)
    h = zfpy.header(buf.tobytes()[:16])
    assert (h["nx"], h["ny"], h["nz"], h["nw"]) == (40, 30, 20, 0)
    assert h["type"] == np.float32 and h["mode"] == "rate"  # zfp_mode_map (pyx:91-98)
    assert h["config"]["rate"] == 8.0
    lib.stream_close(bs)
    lib.zfp_stream_close(zs)
    lib.zfp_field_free(f)


# ---------------- GPU: whole-array and chunked streams vs the oracle ----------------

def _field(oracle, shape, dtype):
    return oracle.smooth_field(len(shape), dtype, min_total=int(np.prod(shape))).ravel()[: int(np.prod(shape))] \
        .reshape(shape).copy()


ZMODES = [("rate", dict(rate=8), lambda t: params_rate(8, 0, 3)),
          ("precision", dict(precision=18), lambda t: params_precision(18)),
          ("reversible", dict(), lambda t: params_reversible())]


def _hdr_plus_blocks(stream, oracle, arr, params, box=None):
    """Expected stream: the first 96 bits of `stream` (the header) + the oracle's blocks at bit 96."""
    words, end = oracle.compress_words(arr, params, box=box, bit_offset=96)
    got = np.frombuffer(stream, dtype=np.uint64)
    hdr = got[:2].copy()
    hdr[1] &= np.uint64(0xffffffff)
    want = words.copy()
    want[0] |= hdr[0]
    want[1] |= hdr[1]
    return want.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,params", ZMODES, ids=[m[0] for m in ZMODES])
@pytest.mark.parametrize("dtype", [np.float32, np.float64], ids=["f32", "f64"])
def test_compress_numpy_matches_oracle(product, oracle, name, kw, params, dtype):
    a = _field(oracle, (24, 36, 52), dtype)
    s = zfpy.compress_numpy(a, **kw)
    assert s[:4] == b"zfp\x05"
    assert bytes(s) == _hdr_plus_blocks(s, oracle, a, params(0))
    back = zfpy.decompress_numpy(s)
    words, _ = oracle.compress_words(a, params(0))
    want, _ = oracle.decompress_words(words, a.shape, dtype, params(0))
    assert back.tobytes() == want.tobytes()
    if name == "reversible":
        assert back.tobytes() == a.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw,params", ZMODES, ids=[m[0] for m in ZMODES])
@pytest.mark.parametrize("shape,nparts", [((64, 64, 64), 4), ((64, 64, 64), 8), ((33, 40, 45), 8)])
def test_zfp_parallel_chunks_match_oracle(product, oracle, name, kw, params, shape, nparts):
    zp = zfpy.zfp_parallel(shape, "float32", nparts=nparts)
    a = _field(oracle, shape, np.float32)
    zp.get_numpy_array()[...] = a
    streams = zp.compress(nthreads=4, **{k: v for k, v in kw.items()})
    ck = zp.get_chunkit()
    assert len(streams) == ck.get_nchunks()
    for i, s in enumerate(streams):
        assert bytes(s) == _hdr_plus_blocks(s, oracle, a, params(0), box=ck.boxes[i]), i
    zp.get_numpy_array()[...] = 0
    zp.decompress(nthreads=4)
    words, _ = oracle.compress_words(a, params(0))
    want, _ = oracle.decompress_words(words, a.shape, np.float32, params(0))
    assert zp.get_numpy_array().tobytes() == want.tobytes()


@pytest.mark.gpu
def test_zslab_chunk_payloads_concatenate_to_whole_stream(product, oracle):
    shape = (64, 48, 40)
    zp = zfpy.zfp_parallel(shape, "float32", nparts=4)
    a = _field(oracle, shape, np.float32)
    zp.get_numpy_array()[...] = a
    streams = zp.compress(rate=16)
    whole = zfpy.compress_numpy(a, rate=16, write_header=False)
    # each chunk stream is the 96-bit header + a payload of P whole words, word flushed
    bits = b""
    for s in streams:
        w = np.frombuffer(bytes(s), dtype=np.uint64)
        p = (len(w) * 64 - 96) // 64
        body = (w[1:1 + p] >> np.uint64(32)) | (w[2:2 + p] << np.uint64(32))
        bits += body.tobytes()
    assert bits == bytes(whole)


@pytest.mark.gpu
def test_large_calls_do_not_keep_their_stream_buffer(product, monkeypatch):
    """the per-thread staging buffer of compress_numpy is
    kept only up to zfpy_c._KEEP_OUT_MAX bytes; a call that needs more allocates
    its own and drops it, so one huge call does not pin memory for the thread's
    lifetime.  (Cap lowered here so a small field exceeds it.)"""
    zc = zfpy.zfpy_c
    monkeypatch.setattr(zc, "_KEEP_OUT_MAX", 1 << 20)
    if hasattr(zc._tls, "out"):
        monkeypatch.delattr(zc._tls, "out")
    rng = np.random.default_rng(5)
    small = rng.standard_normal((16, 16, 16)).astype(np.float32)
    # variable-rate calls stage through the per-thread buffer (fixed-rate ones
    # write straight into the returned bytes)
    zfpy.compress_numpy(small, precision=16)
    kept = getattr(zc._tls, "out", None)
    assert kept is not None and kept.size <= 1 << 20
    big = rng.standard_normal((64, 128, 128)).astype(np.float32)  # > 1 MB stream bound
    s = zfpy.compress_numpy(big, precision=24)
    assert getattr(zc._tls, "out", None) is kept, "a buffer above the cap must not replace the kept one"
    back = zfpy.decompress_numpy(s)
    assert back.shape == big.shape
