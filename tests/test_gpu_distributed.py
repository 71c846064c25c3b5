"""compress_distributed (zfpy/distributed.py) on the GPU box.

* gloo, world 2, both ranks on device 0, host bytes: the gathered chunk list on
  rank 0 equals the single-process zfp_parallel.compress() output byte for byte.
* nccl (RCCL), world 1: the device-resident path -- chunk streams compressed
  straight into HBM buffers and gathered device to device -- gives the same
  bytes.  (RCCL cannot put two ranks on one GPU; the 8-GPU gather is timed by
  bench.py --workload c4 under torch.distributed.run.)
"""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHAPE = (48, 40, 36)


def _field():
    rng = np.random.default_rng(12)
    g = np.indices(SHAPE).sum(axis=0)
    return (np.sin(0.2 * g) + 0.1 * rng.standard_normal(SHAPE)).astype(np.float32)


def _worker(rank, world, port, backend, kw, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch
    import torch.distributed as dist
    import zfpy
    from zfpy import distributed as zdist
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        zp = zfpy.zfp_parallel(SHAPE, "float32", nparts=8)
        zp.get_numpy_array()[...] = _field()
        out = zdist.compress_distributed(zp, **kw)
        q.put([(bytes(s), getattr(s, "block_index", None)) for s in out] if rank == 0 else None)
    finally:
        dist.destroy_process_group()


def _run(world, backend, kw):
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, backend, kw, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    return [r for r in res if r is not None][0]


@pytest.mark.parametrize("kw", [{"rate": 8}, {"precision": 20}, {}], ids=["rate8", "precision20", "reversible"])
@pytest.mark.parametrize("world,backend", [(2, "gloo"), (1, "nccl")])
def test_compress_distributed_matches_single_process(product, world, backend, kw):
    import zfpy
    zp = zfpy.zfp_parallel(SHAPE, "float32", nparts=8)
    zp.get_numpy_array()[...] = _field()
    want = [bytes(s) for s in zp.compress(nthreads=4, **kw)]
    res = _run(world, backend, kw)
    got = [g for g, _ in res]
    assert len(got) == len(want) == zp.get_chunkit().get_nchunks()
    assert got == want
    # variable-rate chunks arrive with their block index and decode without the stream scan
    import ctypes
    from zfpy import zfpy_c
    lib = zfpy_c._lib
    lib.zfp_hip_last_scan.restype = ctypes.c_int
    lib.zfp_hip_last_scan.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    zp3 = zfpy.zfp_parallel(SHAPE, "float32", nparts=8)
    ck = zp3.get_chunkit()
    for i, (g, blob) in enumerate(res):
        assert (blob is None) == ("rate" in kw)
        chunk = zfpy_c.ZfpBytes(g)
        chunk.block_index = blob
        zfpy_c.decompress_numpy_portion(chunk, zp3.get_raw_array(), ck, i, device=0)
        assert lib.zfp_hip_last_scan(None, None) == 0, "chunk %d was scanned despite its index" % i
        if blob is not None:  # the same bytes without the index are scanned
            zfpy_c.decompress_numpy_portion(zfpy_c.ZfpBytes(g), zp3.get_raw_array(), ck, i, device=0)
            assert lib.zfp_hip_last_scan(None, None) == 1
    # and the gathered plain bytes decompress to the single-process result
    zp2 = zfpy.zfp_parallel(SHAPE, "float32", nparts=8)
    zp2._compress_data = got
    zp2.decompress(nthreads=4)
    zp.decompress(nthreads=4)
    assert zp2.get_numpy_array().tobytes() == zp.get_numpy_array().tobytes()
