"""Multi-GPU chunked compression: one process per GPU, chunks sharded by rank.

SURVEY §8(e): zfp chunks are independent streams (whole-field header + the
chunk's blocks, `_zfp_par.py` / `pyx:330-376`), so the compression itself needs
no collective.  Chunk i is compressed by rank i % world on that rank's GPU.
The only exchange is handing every chunk stream to the root, in chunk order:
an all-reduce of the per-chunk sizes, then one gather of each rank's
concatenated payload (RCCL over xGMI with the "nccl" backend and device
tensors; gloo with host tensors in the CPU tests).  Variable-rate streams carry
their GPU block index (`ZfpBytes.block_index`), which travels the same way.
"""
import numpy as np

from .zfpy_c import ZfpBytes


def rank_chunks(nchunks, world, rank):
    """Chunk ids owned by `rank`: i % world == rank (chunk i -> GPU i on a full node)."""
    return list(range(rank, nchunks, world))


def _device_for(dist, group):
    import torch
    backend = dist.get_backend(group)
    if backend == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def gather_streams(local, nchunks, dst=0, group=None):
    """Gather {chunk id: bytes} from every rank to `dst`.

    Returns the list of all chunk streams in chunk order on `dst` (each a
    ZfpBytes with its block_index restored), None elsewhere.  Two collectives:
    all_reduce of the per-chunk (stream, index) sizes, gather of the payloads
    padded to the largest rank payload.
    """
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = _device_for(dist, group)

    sizes = torch.zeros(2 * nchunks, dtype=torch.int64, device=dev)
    for i, s in local.items():
        sizes[2 * i] = len(s)
        blob = getattr(s, "block_index", None)
        sizes[2 * i + 1] = len(blob) if blob else 0
    dist.all_reduce(sizes, op=dist.ReduceOp.SUM, group=group)
    sz = sizes.cpu().numpy().reshape(nchunks, 2)

    per_rank = [int(sz[rank_chunks(nchunks, world, r)].sum()) if nchunks else 0 for r in range(world)]
    mx = max(per_rank) if per_rank else 0
    payload = np.zeros(mx, dtype=np.uint8)
    off = 0
    for i in rank_chunks(nchunks, world, rank):
        s = bytes(local[i])
        payload[off:off + len(s)] = np.frombuffer(s, dtype=np.uint8)
        off += len(s)
        blob = getattr(local[i], "block_index", None) or b""
        if blob:
            payload[off:off + len(blob)] = np.frombuffer(blob, dtype=np.uint8)
        off += len(blob)
    send = torch.from_numpy(payload).to(dev)
    recv = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == dst else None
    dist.gather(send, gather_list=recv, dst=dst, group=group)
    if rank != dst:
        return None

    out = [None] * nchunks
    for r in range(world):
        buf = recv[r].cpu().numpy().tobytes()
        off = 0
        for i in rank_chunks(nchunks, world, r):
            n_s, n_b = int(sz[i, 0]), int(sz[i, 1])
            s = ZfpBytes(buf[off:off + n_s])
            off += n_s
            s.block_index = buf[off:off + n_b] if n_b else None
            off += n_b
            out[i] = s
    return out


def compress_distributed(zp, tolerance=-1, rate=-1, precision=-1, dst=0, group=None):
    """zfp_parallel.compress across ranks: this rank compresses its chunks of the
    shared array `zp` on its current GPU, then the streams are gathered on `dst`
    (stored in zp._compress_data there, as the single-process compress does)."""
    import torch
    import torch.distributed as dist

    from .zfpy_c import compress_numpy_portion
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    ck = zp.get_chunkit()
    n = ck.get_nchunks()
    device = torch.cuda.current_device() if torch.cuda.is_available() else -1
    local = {i: compress_numpy_portion(zp.get_raw_array(), ck, i, tolerance, rate, precision, device=device)
             for i in rank_chunks(n, world, rank)}
    streams = gather_streams(local, n, dst=dst, group=group)
    if streams is not None:
        zp._compress_data = streams
    return streams
