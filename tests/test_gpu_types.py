"""1D/2D fields of every scalar type and 3D/4D integer fields on the GPU.

The generic per-lane codec (blockn.h: encode_block_n / decode_block_n, the
closed-form coder with 4^d coefficients) and the integer branch of the 4D quad
codec (block4.h) against the reference library itself
(oracle/_ref, compiled from /root/reference): compressed bytes and
decompressed arrays identical, through the C API exactly as the reference's
end-to-end tests call it (tests/src/endtoend/zfpEndtoendBase.c).
"""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TYPES = {np.dtype(np.int32): 1, np.dtype(np.int64): 2, np.dtype(np.float32): 3, np.dtype(np.float64): 4}


def _field(shape, dtype, seed):
    rng = np.random.default_rng(seed)
    idx = np.indices(shape, dtype=np.float64)
    smooth = sum(np.sin(0.07 * (a + 1) * idx[a]) for a in range(len(shape)))
    if np.dtype(dtype).kind == "i":
        # integers well inside the range the reference transform is lossless for
        scale = 1 << (20 if np.dtype(dtype).itemsize == 4 else 40)
        a = (smooth * scale).astype(np.int64) + rng.integers(-999, 1000, size=shape)
        return a.astype(dtype)
    a = (smooth + 1e-2 * rng.standard_normal(shape)).astype(dtype)
    flat = a.reshape(-1)
    flat[rng.choice(flat.size, size=max(1, flat.size // 50), replace=False)] = 0  # zero runs, partial zero blocks
    if flat.size > 64:
        flat[:16] = 0  # an all-zero block
    return a


def _modes(dtype):
    if np.dtype(dtype).kind == "i":
        return [("rate", 8), ("rate", 20), ("rate", 32.5), ("precision", 12), ("precision", 30), ("reversible", None)]
    return [("rate", 8), ("rate", 16), ("precision", 18), ("accuracy", 1e-3), ("reversible", None)]


CASES = []
for dtype in (np.float32, np.float64, np.int32, np.int64):
    shapes = [(1000,), (37,), (45, 67), (64, 64)]
    if np.dtype(dtype).kind == "i":
        shapes += [(20, 24, 28), (9, 13, 7), (12, 9, 10, 11), (8, 16, 16, 16)]
    for shape in shapes:
        for mode, param in _modes(dtype):
            CASES.append((np.dtype(dtype).name, shape, mode, param))


@pytest.mark.parametrize("dtype,shape,mode,param", CASES)
def test_stream_and_roundtrip_match_reference(product, ref_capi, dtype, shape, mode, param):
    dtype = np.dtype(dtype)
    a = _field(shape, dtype, zlib.crc32(repr((dtype.name, shape, mode)).encode()))
    ztype = TYPES[dtype]
    want = ref_capi.compress(a, mode, param, ztype=ztype)
    product.keep_index = True
    try:
        got = product.compress(a, mode, param, ztype=ztype)
        assert got == want, (dtype.name, shape, mode, param)
        ref_out, _ = ref_capi.decompress(want, shape, dtype, mode, param, ztype=ztype)
        for index in (product.last_index, None):  # the encoder's index, then the scan
            out, n = product.decompress(got, shape, dtype, mode, param, ztype=ztype, index=index)
            assert n == len(got)
            assert out.tobytes() == ref_out.tobytes(), (dtype.name, shape, mode, param, index is None)
    finally:
        if product.last_index:
            product.lib.zfp_hip_index_free(product.last_index)
            product.last_index = None


@pytest.mark.parametrize("dtype", ["float32", "int32", "int64"])
def test_header_offset_2d(product, ref_capi, dtype):
    """zfpy layout (96-bit header first): unaligned block starts in 2D."""
    a = _field((33, 50), np.dtype(dtype), 5)
    ztype = 0 if dtype == "float32" else TYPES[np.dtype(dtype)]
    for mode, param in (("rate", 12), ("precision", 14), ("reversible", None)):
        want = ref_capi.compress(a, mode, param, ztype=ztype, header=True)
        got = product.compress(a, mode, param, ztype=ztype, header=True)
        assert got == want, (dtype, mode)
        ref_out, _ = ref_capi.decompress(want, a.shape, a.dtype, mode, param, ztype=ztype, header=True)
        out, _ = product.decompress(got, a.shape, a.dtype, mode, param, ztype=ztype, header=True)
        assert out.tobytes() == ref_out.tobytes(), (dtype, mode)


@pytest.mark.parametrize("shape,dtype", [((10000,), "float32"), ((90, 70), "float64"), ((50, 60), "int32")])
def test_threaded_chunks_sharing_pages(product, ref_capi, shape, dtype):
    """zfp_parallel decompresses the chunks of one array from a thread pool; chunk
    boundaries in 1D/2D fall inside memory pages, and every byte must still be
    the reference's (the library copies partial pages to the user array itself)."""
    import zfpy
    a = _field(shape, np.dtype(dtype), 9)
    zp = zfpy.zfp_parallel(shape, dtype, nparts=8)
    zp.get_numpy_array()[...] = a
    streams = zp.compress(nthreads=8, precision=20)
    whole = ref_capi.compress(a, "precision", 20, ztype=TYPES[np.dtype(dtype)])
    want, _ = ref_capi.decompress(whole, shape, dtype, "precision", 20, ztype=TYPES[np.dtype(dtype)])
    for _ in range(3):
        zp.get_numpy_array()[...] = 0
        zp._compress_data = [bytes(s) for s in streams]
        zp.decompress(nthreads=8)
        assert np.ascontiguousarray(zp.get_numpy_array()).tobytes() == want.tobytes()
