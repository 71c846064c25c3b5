"""Repeated zfp_parallel compress/decompress at C4 chunk scale.

zfpy builds a new thread pool per call and every worker thread calls into the
library; device contexts (HIP stream + scratch) come from a bounded process-wide
pool, so device memory must stay flat across calls, and every chunk stream must
be byte-identical to the reference library's (oracle/_ref, compiled from the
reference sources) on every repetition; the decompressed array must equal the
reference decompression of the same chunks.
"""
import ctypes
from multiprocessing.pool import ThreadPool

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHAPE = (512, 1024, 1024)  # 2 GiB of float32, 8 z-slab chunks of 64 planes
RATE = 8


def _ref_chunk(ref, arr, box):
    """Reference zfpy layout: whole-field header + the chunk's blocks (pyx:330-376)."""
    lib = ref.lib
    field = ref.field_for(arr)
    zs = lib.zfp_stream_open(None)
    lib.zfp_stream_set_rate(zs, float(RATE), 0, 3, 0)
    ck = ref.make_chunk(3, box)
    cap = lib.zfp_stream_maximum_size_chunk(zs, field, ck) + 64
    buf = np.zeros(cap, dtype=np.uint8)
    bs = lib.stream_open(buf.ctypes.data, cap)
    lib.zfp_stream_set_bit_stream(zs, bs)
    lib.zfp_stream_rewind(zs)
    assert lib.zfp_write_header(zs, field, 7) == 96
    n = lib.zfp_compress_chunk(zs, ck, field)
    lib.zfp_chunk_free(ck)
    lib.stream_close(bs)
    lib.zfp_stream_close(zs)
    lib.zfp_field_free(field)
    return bytes(buf[:n])


def _ref_decode_chunk(ref, stream, out, box):
    lib = ref.lib
    field = lib.zfp_field_alloc()
    buf = np.frombuffer(stream + bytes(64), dtype=np.uint8)
    bs = lib.stream_open(buf.ctypes.data, len(stream))
    zs = lib.zfp_stream_open(bs)
    assert lib.zfp_read_header(zs, field, 7)
    lib.zfp_field_set_pointer(field, out.ctypes.data)
    ck = ref.make_chunk(3, box)
    assert lib.zfp_decompress_chunk(zs, ck, field)
    lib.zfp_chunk_free(ck)
    lib.zfp_stream_close(zs)
    lib.stream_close(bs)
    lib.zfp_field_free(field)


def test_repeated_zfp_parallel_is_exact_and_memory_flat(product, ref_capi):
    import torch
    import zfpy
    zp = zfpy.zfp_parallel(SHAPE, "float32", nparts=8)
    a = zp.get_numpy_array()
    x = torch.arange(SHAPE[2], device="cuda", dtype=torch.float64)
    base = torch.sin(0.05 * x)[None, :] * torch.cos(0.03 * x)[:, None]
    for z in range(SHAPE[0]):
        a[z] = (base + 0.5 * torch.sin(0.02 * z + 0.01 * x[None, :] * x[:, None] / SHAPE[2])).float().cpu().numpy()
    ck = zp.get_chunkit()
    boxes = [[ck.boxes[i][ax] for ax in range(3)] for i in range(ck.get_nchunks())]
    assert len(boxes) == 8
    with ThreadPool(8) as pool:
        want = pool.map(lambda b: _ref_chunk(ref_capi, a, b), boxes)
    ref_back = np.zeros(SHAPE, dtype=np.float32)
    with ThreadPool(8) as pool:
        pool.starmap(lambda s, b: _ref_decode_chunk(ref_capi, s, ref_back, b), zip(want, boxes))
    orig = a.copy()
    scratch_bytes = product.lib.zfp_hip_scratch_bytes
    scratch_bytes.restype = ctypes.c_size_t
    free, pooled = [], []
    for it in range(4):
        a[...] = orig  # the previous iteration left the decompressed (lossy) field here
        streams = zp.compress(nthreads=8, rate=RATE)
        assert [bytes(s) == w for s, w in zip(streams, want)] == [True] * 8, it
        a[...] = 0
        zp.decompress(nthreads=8)
        assert np.array_equal(a, ref_back), it
        torch.cuda.synchronize()
        free.append(torch.cuda.mem_get_info()[0])
        pooled.append(scratch_bytes())  # every context is idle between calls
    # The pool holds one context per concurrently running call: which calls
    # overlap depends on thread timing, so a later repetition may add a context
    # (up to the 8 worker threads).  Everything the library holds on the device
    # is in the idle pool between calls -- free + pooled stays constant (HIP
    # streams and allocator granularity aside) -- and the pool stays bounded by
    # 8 contexts of at most one chunk's staging each.
    held = [f + p for f, p in zip(free, pooled)]
    assert max(held) - min(held) < (160 << 20), (free, pooled)  # a leaked context: >= 384 MiB
    chunk = SHAPE[0] * SHAPE[1] * SHAPE[2] * 4 // 8
    assert max(pooled) <= 8 * 4 * chunk, pooled
