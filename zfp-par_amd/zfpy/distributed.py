"""Multi-GPU chunked compression: one process per GPU, chunks sharded by rank.

SURVEY §8(e): zfp chunks are independent streams (whole-field header + the
chunk's blocks, `_zfp_par.py` / `pyx:330-376`), so the compression itself needs
no collective.  Chunk i is compressed by rank i % world on that rank's GPU.
The only exchange is handing every chunk stream to the root, in chunk order:
an all-reduce of the per-chunk sizes, then one gather of each rank's
concatenated payload.

  nccl (RCCL over xGMI): each chunk is compressed straight into a device
        buffer (the stream's header words are written through hipMemcpy by the
        host library), the payloads are gathered device to device, and only
        the root copies the streams to host bytes -- the chunk never crosses
        PCIe on the compressing rank.
  gloo (CPU tests): host bytes, as the single-process zfp_parallel returns.

Variable-rate chunks carry their GPU block index (ZfpBytes.block_index)
through the gather, so the root decodes them without the stream scan; a stream
that arrives without one (or with one for another stream) is still decoded,
after the scan finds its block starts (zfp_hip_index_build).
"""
import ctypes

import numpy as np

from . import zfpy_c
from .zfpy_c import ZfpBytes


def rank_chunks(nchunks, world, rank):
    """Chunk ids owned by `rank`: i % world == rank (chunk i -> GPU i on a full node)."""
    return list(range(rank, nchunks, world))


def _device_for(dist, group):
    import torch
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _blob(s):
    """The block-index blob a chunk stream carries (ZfpBytes.block_index / tensor attribute), or b''."""
    b = getattr(s, "block_index", None)
    return bytes(b) if b else b""


def _peer(dist, group, r):
    """Global rank of rank r of `group` (point-to-point ops address global ranks)."""
    return r if group is None else dist.get_global_rank(group, r)


def gather_streams(local, nchunks, dst=0, group=None):
    """Gather {chunk id: stream} from every rank to `dst` (a rank of `group`);
    returns the list of all chunk streams in chunk order on `dst`, None
    elsewhere: plain bytes, or a ZfpBytes for a chunk that carries a block index.
    A local stream is host bytes, or a uint8 device tensor on the nccl path
    (gathered in HBM).

    Each chunk's GPU block index (variable-rate streams) travels with it, so the
    root decodes gathered chunks without scanning them.  One all-reduce carries
    the stream and index sizes of every chunk; then every rank sends its exact
    payload (its streams, then its index blobs) to `dst` point to point, no
    padding; on the root each payload is copied to the host once and every
    chunk's bytes object is cut from that copy."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = _device_for(dist, group)
    mine = rank_chunks(nchunks, world, rank)
    sizes = torch.zeros(2 * nchunks, dtype=torch.int64, device=dev)
    blobs = {i: _blob(local[i]) for i in mine}
    for i in mine:
        s = local[i]
        sizes[i] = s.numel() if hasattr(s, "numel") else len(s)
        sizes[nchunks + i] = len(blobs[i])
    dist.all_reduce(sizes, op=dist.ReduceOp.SUM, group=group)
    sz = sizes.cpu().numpy()
    per_rank = [int(sz[rank_chunks(nchunks, world, r)].sum() + sz[[nchunks + i for i in rank_chunks(nchunks, world, r)]].sum())
                for r in range(world)]
    pieces = []
    for i in mine:
        s = local[i]
        pieces.append(s.to(dev) if isinstance(s, torch.Tensor) else
                      torch.frombuffer(bytearray(s), dtype=torch.uint8).to(dev))
    for i in mine:
        if blobs[i]:
            pieces.append(torch.frombuffer(bytearray(blobs[i]), dtype=torch.uint8).to(dev))
    send = torch.cat(pieces) if pieces else torch.zeros(0, dtype=torch.uint8, device=dev)
    recv = None
    ops = []
    if rank == dst:
        recv = [send if r == rank else torch.empty(per_rank[r], dtype=torch.uint8, device=dev) for r in range(world)]
        ops = [dist.P2POp(dist.irecv, recv[r], _peer(dist, group, r), group)
               for r in range(world) if r != rank and per_rank[r]]
    elif per_rank[rank]:
        ops = [dist.P2POp(dist.isend, send, _peer(dist, group, dst), group)]
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    if rank != dst:
        return None
    out = [None] * nchunks
    for r in range(world):
        if recv[r].device.type == "cpu":
            host = recv[r].numpy()
        else:  # one device-to-host copy per rank payload
            host = np.empty(per_rank[r], dtype=np.uint8)
            torch.from_numpy(host).copy_(recv[r])
        view = memoryview(host)
        ids = rank_chunks(nchunks, world, r)
        boff = sum(int(sz[i]) for i in ids)  # the index blobs follow the streams
        off = 0
        for i in ids:
            n, nb = int(sz[i]), int(sz[nchunks + i])
            if nb:
                out[i] = ZfpBytes(view[off:off + n])
                out[i].block_index = bytes(view[boff:boff + nb])
            else:  # no index (fixed rate): plain bytes, copied outside the GIL
                out[i] = zfpy_c._bytes_from(host.ctypes.data + off, n)
            off += n
            boff += nb
    return out


def compress_chunk_to_device(zp, ichunk, tolerance=-1, rate=-1, precision=-1, device=None):
    """compress_numpy_portion with the stream in HBM: returns a uint8 device
    tensor holding the chunk stream (whole-field header + the chunk's blocks),
    byte-identical to compress_numpy_portion's bytes."""
    import torch
    lib = zfpy_c._lib
    ck = zp.get_chunkit()
    dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
    field = zfpy_c._init_field_raw(zp.get_raw_array(), ck)
    stream = lib.zfp_stream_open(None)
    bstream = None
    try:
        lib.zfp_stream_set_hip_device(stream, dev.index)
        zfpy_c._set_compression_mode(stream, zfpy_c.type_none, ck.ndim, tolerance, rate, precision)
        cp = ck.chunk_ptr(ichunk)
        cap = lib.zfp_stream_maximum_size_chunk(stream, field, cp) + (zfpy_c.HEADER_MAX_BITS + 63) // 64 * 8 + 8
        buf = torch.zeros(cap, dtype=torch.uint8, device=dev)
        bstream = lib.stream_open(ctypes.c_void_p(buf.data_ptr()), cap)
        lib.zfp_stream_set_bit_stream(stream, bstream)
        lib.zfp_stream_rewind(stream)
        if lib.zfp_write_header(stream, field, zfpy_c.HEADER_FULL) == 0:
            raise RuntimeError("Failed to write header to stream")
        n = lib.zfp_compress_chunk(stream, cp, field)
        if n == 0:
            raise RuntimeError("Failed to write to stream")
        out = buf[:n]
        out.block_index = zfpy_c._export_index(stream)  # variable rate: travels with the chunk
        return out
    finally:
        lib.zfp_field_free(field)
        lib.zfp_stream_close(stream)
        if bstream:
            lib.stream_close(bstream)


def compress_distributed(zp, tolerance=-1, rate=-1, precision=-1, dst=0, group=None):
    """zfp_parallel.compress across ranks: this rank compresses its chunks of the
    shared array `zp` on its current GPU, then the streams are gathered on `dst`
    (a rank of `group`; stored in zp._compress_data there, as the single-process
    compress does)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    ck = zp.get_chunkit()
    n = ck.get_nchunks()
    mine = rank_chunks(n, world, rank)
    if dist.get_backend(group) == "nccl":
        local = {i: compress_chunk_to_device(zp, i, tolerance, rate, precision) for i in mine}
    else:
        device = torch.cuda.current_device() if torch.cuda.is_available() else -1
        local = {i: zfpy_c.compress_numpy_portion(zp.get_raw_array(), ck, i, tolerance, rate, precision,
                                                  device=device) for i in mine}
    streams = gather_streams(local, n, dst=dst, group=group)
    if streams is not None:
        zp._compress_data = streams
    return streams
