"""Host-side logic of the product library vs the reference build (CPU only).

Everything here runs without a GPU: mode/parameter rules, headers, size
bounds, field metadata, the fork's chunk partitioner, the bit stream, and the
C-ABI export list of include/*.h.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from capi import ZfpCAPI

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRODUCT_SO = os.path.join(REPO, "zfp-par_amd", "lib", "libzfp.so")
HIP_SO = os.path.join(REPO, "zfp-par_amd", "lib", "libzfp_hip.so")


def _declared(header):
    text = open(os.path.join(REPO, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b((?:zfp|stream)_[a-z0-9_]+)\s*\(", text))
    return names


def test_library_exports_every_declared_symbol():
    import subprocess
    exported = set()
    for so in (PRODUCT_SO, HIP_SO):
        out = subprocess.check_output(["nm", "-D", "--defined-only", so]).decode()
        exported |= {line.split()[-1] for line in out.splitlines() if " T " in line or " D " in line or " R " in line}
    for header in ("zfp.h", "zfp/bitstream.h", "zfp_hip.h"):
        missing = sorted(n for n in _declared(header) if n not in exported)
        assert not missing, (header, missing)
    for data in ("zfp_codec_version", "zfp_library_version", "zfp_version_string", "stream_word_bits"):
        assert data in exported


def _params(api, zs):
    mb, xb, mp, me = ctypes.c_uint(), ctypes.c_uint(), ctypes.c_uint(), ctypes.c_int()
    api.zfp_stream_params(zs, ctypes.byref(mb), ctypes.byref(xb), ctypes.byref(mp), ctypes.byref(me))
    return mb.value, xb.value, mp.value, me.value


SETTERS = [("rate", r, t, d) for r in (0.5, 1.5, 8, 16, 31.9) for t in (0, 3, 4) for d in (1, 2, 3, 4)] + \
          [("precision", p, 0, 3) for p in (0, 1, 17, 32, 64, 99)] + \
          [("accuracy", a, 0, 3) for a in (0.0, 1e-7, 0.25, 3.0, 1e300)] + [("reversible", None, 0, 3)]


@pytest.mark.parametrize("mode,param,ztype,dims", SETTERS)
def test_mode_setters_and_mode_word_match_reference(prod, ref_capi, mode, param, ztype, dims):
    got = []
    for api in (prod, ref_capi):
        zs = api.zfp_stream_open(None)
        if mode == "rate":
            ret = api.zfp_stream_set_rate(zs, param, ztype, dims, 0)
        elif mode == "precision":
            ret = api.zfp_stream_set_precision(zs, param)
        elif mode == "accuracy":
            ret = api.zfp_stream_set_accuracy(zs, param)
        else:
            ret = api.zfp_stream_set_reversible(zs)
        word = api.zfp_stream_mode(zs)
        got.append((ret, _params(api, zs), word, api.zfp_stream_compression_mode(zs),
                    api.zfp_stream_rate(zs, dims), api.zfp_stream_precision(zs), api.zfp_stream_accuracy(zs)))
        zs2 = api.zfp_stream_open(None)
        got.append((api.zfp_stream_set_mode(zs2, word), _params(api, zs2)))
        api.zfp_stream_close(zs)
        api.zfp_stream_close(zs2)
    assert got[0] == got[2] and got[1] == got[3]


@pytest.mark.parametrize("expert", [(1, 16658, 64, -1074), (64, 64, 64, -1074), (5, 400, 33, -100),
                                    (0, 0, 1, 16000), (2000, 40000, 128, -20000)])
def test_expert_params_long_mode_word(prod, ref_capi, expert):
    out = []
    for api in (prod, ref_capi):
        zs = api.zfp_stream_open(None)
        ok = api.zfp_stream_set_params(zs, *expert)
        out.append((ok, api.zfp_stream_mode(zs), api.zfp_stream_compression_mode(zs), _params(api, zs)))
        api.zfp_stream_close(zs)
    assert out[0] == out[1]


FIELDS = [((7,), 3), ((9, 11), 4), ((5, 6, 7), 3), ((1024, 1024, 1024), 3), ((4096, 4096, 512), 3),
          ((8, 9, 10, 11), 4), ((512, 512, 512, 512), 3), ((70000, 5, 5), 3), ((5000, 5, 5, 5), 3)]


@pytest.mark.parametrize("shape,ztype", FIELDS)
def test_field_metadata_and_bounds_match_reference(prod, ref_capi, shape, ztype):
    res = []
    for api in (prod, ref_capi):
        n = list(reversed(shape))
        ctor = [api.zfp_field_1d, api.zfp_field_2d, api.zfp_field_3d, api.zfp_field_4d][len(n) - 1]
        f = ctor(None, ztype, *n)
        meta = api.zfp_field_metadata(f)
        row = [meta, api.zfp_field_blocks(f), api.zfp_field_size(f, None)]
        for mode in (("rate", 16.0), ("rate", 8.0), ("precision", 32), ("accuracy", 1e-3), ("reversible", None)):
            zs = api.zfp_stream_open(None)
            api.set_mode(zs, mode[0], mode[1], ztype, len(n))
            row.append(api.zfp_stream_maximum_size(zs, f))
            api.zfp_stream_close(zs)
        g = api.zfp_field_alloc()
        if meta != (1 << 64) - 1:
            row.append(api.zfp_field_set_metadata(g, meta))
            ff = ctypes.cast(g, ctypes.POINTER(__import__("capi").ZfpField)).contents
            row.append((ff.type, ff.nx, ff.ny, ff.nz, ff.nw, ff.sx, ff.sy, ff.sz, ff.sw))
        api.zfp_field_free(g)
        api.zfp_field_free(f)
        res.append(row)
    assert res[0] == res[1]


def _header_bytes(api, shape, ztype, mode, param):
    n = list(reversed(shape))
    ctor = [api.zfp_field_1d, api.zfp_field_2d, api.zfp_field_3d, api.zfp_field_4d][len(n) - 1]
    f = ctor(None, ztype, *n)
    zs = api.zfp_stream_open(None)
    api.set_mode(zs, mode, param, 0, len(n))
    buf = np.zeros(64, dtype=np.uint8)
    bs = api.stream_open(buf.ctypes.data, 64)
    api.zfp_stream_set_bit_stream(zs, bs)
    bits = api.zfp_write_header(zs, f, 7)
    api.stream_flush(bs)
    api.stream_rewind(bs)
    g = api.zfp_field_alloc()
    zs2 = api.zfp_stream_open(bs)
    rbits = api.zfp_read_header(zs2, g, 7)
    back = (_params(api, zs2), api.zfp_field_metadata(g))
    for h in (bs,):
        api.stream_close(h)
    api.zfp_stream_close(zs)
    api.zfp_stream_close(zs2)
    api.zfp_field_free(f)
    api.zfp_field_free(g)
    return bits, rbits, buf.tobytes(), back


@pytest.mark.parametrize("shape", [(1024, 1024, 1024), (512, 4096, 4096), (7, 11, 13), (512, 512, 512, 512)])
@pytest.mark.parametrize("mode,param", [("rate", 16), ("rate", 8), ("precision", 32), ("accuracy", 0.01),
                                        ("reversible", None), ("expert", (3, 5000, 20, -30))])
def test_header_write_read_match_reference(prod, ref_capi, shape, mode, param):
    assert _header_bytes(prod, shape, 3, mode, param) == _header_bytes(ref_capi, shape, 3, mode, param)


def _partition(api, shape, cpb, method):
    nd = len(shape)
    n = (ctypes.c_int * nd)(*reversed(shape))
    blocks = api.zfp_optimal_parts_from_size(nd, n, ctypes.c_float(cpb), method)

    class Blocks(ctypes.Structure):
        _fields_ = [("bx", ctypes.c_size_t), ("by", ctypes.c_size_t), ("bz", ctypes.c_size_t),
                    ("bw", ctypes.c_size_t), ("nbeg", ctypes.c_int), ("begs", ctypes.c_void_p)]

    class Chunk(ctypes.Structure):
        _fields_ = [(k, ctypes.c_size_t) for k in ("fx", "fy", "fz", "fw", "ex", "ey", "ez", "ew")]

    class Chunks(ctypes.Structure):
        _fields_ = [("nchunks", ctypes.c_size_t), ("chunks", ctypes.POINTER(ctypes.POINTER(Chunk)))]

    b = ctypes.cast(blocks, ctypes.POINTER(Blocks)).contents
    counts = (b.bx, b.by if nd > 1 else 0, b.bz if nd > 2 else 0, b.bw if nd > 3 else 0, b.nbeg)
    chunks = api.zfp_chunks_from_blocks(nd, n, blocks)
    cs = ctypes.cast(chunks, ctypes.POINTER(Chunks)).contents
    boxes = []
    for i in range(cs.nchunks):
        c = cs.chunks[i].contents
        box = [(c.fx, c.ex), (c.fy, c.ey), (c.fz, c.ez), (c.fw, c.ew)][:nd]
        boxes.append(box)
    api.zfp_chunks_free(chunks)
    api.zfp_blocks_free(blocks)
    return counts, boxes


PARTS = [((4096, 4096, 512), 8), ((512, 512, 512, 512), 8), ((1024, 1024, 1024), 8), ((129, 129, 129), 8),
         ((64, 64, 64), 4), ((64, 64, 64), 8), ((100, 37, 53), 3), ((33, 33, 33, 33), 5), ((256, 256, 256), 1000)]


@pytest.mark.parametrize("shape,nparts", PARTS)
def test_best_cache_partition_matches_reference(prod, ref_capi, shape, nparts):
    """zfp_optimal_parts_from_size(BEST_CACHE) + zfp_chunks_from_blocks, as zfp_parallel calls them."""
    nblocks = int(np.prod([(s + 3) // 4 for s in shape]))
    cpb = nblocks / nparts
    assert _partition(prod, shape, cpb, 1) == _partition(ref_capi, shape, cpb, 1)


def test_survey_partition_facts(prod):
    """C4 -> 8 z-slabs of 64 planes, C5 -> 8 w-slabs, 129^3/8 -> 9 chunks."""
    counts, boxes = _partition(prod, (512, 4096, 4096), (1024 * 1024 * 128) / 8, 1)
    assert len(boxes) == 8 and all(b[2][1] - b[2][0] == 64 for b in boxes)
    counts, boxes = _partition(prod, (512, 512, 512, 512), 128 ** 4 / 8, 1)
    assert len(boxes) == 8 and all(b[3][1] - b[3][0] == 64 for b in boxes)
    counts, boxes = _partition(prod, (129, 129, 129), 33 ** 3 / 8, 1)
    assert [b[2][1] - b[2][0] for b in boxes] == [12, 12, 12, 16, 16, 16, 16, 16, 13]


@pytest.mark.parametrize("n,parts", [(129, 9), (4096, 8), (7, 3), (1024, 7), (16, 4)])
def test_break_axis_matches_reference(prod, ref_capi, n, parts):
    out = []
    for api in (prod, ref_capi):
        f = (ctypes.c_int * parts)()
        e = (ctypes.c_int * parts)()
        api.zfp_break_axis(n, parts, f, e)
        out.append((list(f), list(e)))
    assert out[0] == out[1]


def test_bitstream_ops_match_reference(prod, ref_capi):
    rng = np.random.default_rng(9)
    ops = [(int(rng.integers(0, 65)), int(rng.integers(0, 1 << 62))) for _ in range(400)]
    res = []
    for api in (prod, ref_capi):
        buf = np.zeros(8192, dtype=np.uint8)
        bs = api.stream_open(buf.ctypes.data, 8192)
        rets = []
        for n, v in ops:
            rets.append(api.stream_write_bits(bs, v, n))
            if n % 7 == 0:
                api.stream_pad(bs, n)
        rets.append(api.stream_wtell(bs))
        rets.append(api.stream_flush(bs))
        rets.append(api.stream_size(bs))
        api.stream_rewind(bs)
        for n, v in ops:
            rets.append(api.stream_read_bits(bs, n))
            if n % 7 == 0:
                api.stream_skip(bs, n)
        rets.append(api.stream_rtell(bs))
        rets.append(api.stream_align(bs))
        api.stream_rseek(bs, 777)
        rets.append(api.stream_read_bits(bs, 33))
        api.stream_wseek(bs, 1001)
        api.stream_write_bits(bs, 0x155, 9)
        api.stream_flush(bs)
        api.stream_close(bs)
        res.append((rets, buf.tobytes()))
    assert res[0] == res[1]


def test_execution_policies(prod):
    zs = prod.zfp_stream_open(None)
    assert prod.zfp_stream_execution(zs) == 0
    assert prod.zfp_stream_set_execution(zs, 1) == 1
    assert prod.zfp_stream_execution(zs) == 1
    assert prod.zfp_stream_set_execution(zs, 2) == 0  # no CUDA, as a reference build without it
    assert prod.zfp_stream_set_execution(zs, 3) == 1
    assert prod.zfp_stream_set_execution(zs, 0) == 1
    prod.zfp_stream_close(zs)
