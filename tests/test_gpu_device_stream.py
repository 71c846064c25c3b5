"""Streams in HIP device memory through the plain C API, headers included.

zfp_write_header / zfp_read_header touch stream words from the host; with a
device-resident stream buffer (stream_open on hipMalloc memory) those words go
through hipMemcpy, the codec writes the rest on the device.  The bytes must be
those of the host-buffer path (itself checked against the oracle), for fixed
and variable rate, at the zfpy header offset (96 bits).
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode,param", [("rate", 8), ("rate", 12.5), ("precision", 20), ("reversible", None)])
def test_device_stream_with_header_matches_host_stream(product, mode, param):
    import torch
    lib = product.lib
    rng = np.random.default_rng(11)
    arr = rng.standard_normal((40, 36, 44)).astype(np.float32)
    want = product.compress(arr, mode, param, header=True)
    if product.last_index:
        lib.zfp_hip_index_free(product.last_index)
        product.last_index = None
    dev_in = torch.from_numpy(arr).cuda()
    field = lib.zfp_field_3d(ctypes.c_void_p(dev_in.data_ptr()), 3, 44, 36, 40)
    zs = lib.zfp_stream_open(None)
    product.set_mode(zs, mode, param, 3, 3)
    cap = lib.zfp_stream_maximum_size(zs, field) + 64
    dbuf = torch.zeros(cap, dtype=torch.uint8, device="cuda")
    bs = lib.stream_open(ctypes.c_void_p(dbuf.data_ptr()), cap)
    lib.zfp_stream_set_bit_stream(zs, bs)
    lib.zfp_stream_rewind(zs)
    assert lib.zfp_write_header(zs, field, 7) == 96
    n = lib.zfp_compress(zs, field)
    assert n == len(want)
    assert dbuf[:n].cpu().numpy().tobytes() == want
    # read it back from the device stream
    dev_out = torch.zeros_like(dev_in)
    ofield = lib.zfp_field_alloc()
    lib.zfp_stream_rewind(zs)
    assert lib.zfp_read_header(zs, ofield, 7) == 96
    lib.zfp_field_set_pointer(ofield, ctypes.c_void_p(dev_out.data_ptr()))
    assert lib.zfp_decompress(zs, ofield) == n
    host_out, _ = product.decompress(want, arr.shape, np.float32, mode, param, header=True)
    assert dev_out.cpu().numpy().tobytes() == host_out.tobytes()
    lib.stream_close(bs)
    lib.zfp_stream_close(zs)
    lib.zfp_field_free(field)
    lib.zfp_field_free(ofield)
