#!/usr/bin/env python3
"""Benchmark: GB/s uncompressed, 3D float32 fixed-rate encode, device-resident.

One step = zfp_compress of one 1024^3 float32 field at rate 16 (BASELINE.json
configs[1]) through the drop-in C API, with the field and the stream buffer
already in HBM.  With N GPUs (one process per GPU, torchrun) each rank
compresses its own 1024^3 z-slab chunk of an N*1024-plane field: chunks are
independent zfp streams, so the timed region has no collective (weak scaling);
the RCCL gather that concatenates the chunk streams on rank 0 is timed
separately and reported as `gather_*`.

Printed JSON (rank 0): the contract keys plus
  roofline      dominant kernel (encode3_aligned) against HBM peak: achieved =
                algorithmic bytes per launch (4 B read + 2 B written per value)
                / mean kernel time from HIP events on the kernel's own stream;
                traffic = PMC HBM bytes per launch from profiles/*pmc*.json
                (rocprofv3 pass, gfx950 FETCH_SIZE x2 correction) or null
  cpu_baseline  the reference itself (oracle/_ref/libzfp_ref.so, compiled from
                /root/reference), OpenMP, on this host's cores, bounded sample
  decode_*      zfp_decompress of the same stream (same field, device-resident)
  bitexact      GPU stream bytes == reference CPU stream bytes on the sample
"""
import argparse
import ctypes
import glob
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "GB/s uncompressed, 3D float32 fixed-rate encode, device-resident"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
N = 1024
RATE = 16


def smooth_field_torch(torch, nx, ny, nz, z0, ntot_z, device):
    """F1: v = sin(.05x) cos(.03y) + .5 sin(.02z + .01 x y / n), x fastest."""
    x = torch.arange(nx, device=device, dtype=torch.float64)
    y = torch.arange(ny, device=device, dtype=torch.float64)
    out = torch.empty((nz, ny, nx), device=device, dtype=torch.float32)
    base = (torch.sin(0.05 * x)[None, :] * torch.cos(0.03 * y)[:, None])
    xy = 0.01 * x[None, :] * y[:, None] / nx
    for k in range(nz):
        z = float(z0 + k)
        out[k] = (base + 0.5 * torch.sin(0.02 * z + xy)).to(torch.float32)
    return out


def load_capi(path):
    from capi import ZfpCAPI
    api = ZfpCAPI(path)
    return api


def traffic_from_profiles():
    """Per-launch HBM bytes of encode3_aligned from a committed PMC summary, if any."""
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc*.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
            if "encode3_aligned" in d and d["encode3_aligned"].get("hbm_bytes_per_launch"):
                return d["encode3_aligned"]["hbm_bytes_per_launch"], os.path.basename(f)
        except Exception:
            continue
    return None, None


def cpu_baseline(field_np, threads):
    """The reference library (OpenMP policy) on a bounded slab; returns (GB/s, bytes)."""
    from pyoracle import REF_SO
    if not os.path.exists(REF_SO):
        return None
    ref = load_capi(REF_SO)
    ref.lib.zfp_stream_set_omp_threads.restype = ctypes.c_int
    ref.lib.zfp_stream_set_omp_threads.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    f = ref.field_for(field_np)
    zs = ref.lib.zfp_stream_open(None)
    ref.lib.zfp_stream_set_rate(zs, float(RATE), 3, 3, 0)
    ref.lib.zfp_stream_set_omp_threads(zs, threads)
    cap = ref.lib.zfp_stream_maximum_size(zs, f)
    buf = np.zeros(cap, dtype=np.uint8)
    bs = ref.lib.stream_open(buf.ctypes.data, cap)
    ref.lib.zfp_stream_set_bit_stream(zs, bs)
    best = None
    nbytes = 0
    for _ in range(3):
        ref.lib.zfp_stream_rewind(zs)
        t0 = time.perf_counter()
        nbytes = ref.lib.zfp_compress(zs, f)
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    ref.lib.stream_close(bs)
    ref.lib.zfp_stream_close(zs)
    ref.lib.zfp_field_free(f)
    return field_np.nbytes / best / 1e9, bytes(buf[:nbytes])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=N, help="edge of the per-GPU cube (default 1024)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if distributed:
        dist.init_process_group("nccl", device_id=dev)

    n = args.n
    api = load_capi(os.path.join(REPO, "zfp-par_amd", "lib", "libzfp.so"))
    api.enable_index()
    lib = api.lib
    lib.zfp_hip_last_timing.argtypes = [ctypes.c_void_p, ctypes.c_void_p]

    # this rank's chunk: z-slab [rank*n, rank*n + n) of an n x n x (world*n) field
    field_t = smooth_field_torch(torch, n, n, n, rank * n, world * n, dev)
    nvals = field_t.numel()
    zf = lib.zfp_field_3d(ctypes.c_void_p(field_t.data_ptr()), 3, n, n, n)
    zs = lib.zfp_stream_open(None)
    lib.zfp_stream_set_rate(zs, float(RATE), 3, 3, 0)
    cap = lib.zfp_stream_maximum_size(zs, zf)
    out_t = torch.zeros(cap, dtype=torch.uint8, device=dev)
    bs = lib.stream_open(ctypes.c_void_p(out_t.data_ptr()), cap)
    lib.zfp_stream_set_bit_stream(zs, bs)

    def step():
        lib.zfp_stream_rewind(zs)
        nb = lib.zfp_compress(zs, zf)
        if nb == 0:
            raise RuntimeError("zfp_compress failed: %s" % lib.zfp_hip_last_error())
        return nb

    for _ in range(args.warmup):
        nbytes = step()
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    kms, tms = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        nbytes = step()
        k, t = ctypes.c_double(), ctypes.c_double()
        lib.zfp_hip_last_timing(ctypes.byref(k), ctypes.byref(t))
        kms.append(k.value)
        tms.append(t.value)
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ms = elapsed / args.steps * 1e3
    if distributed:
        tt = torch.tensor([ms], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        ms = float(tt.item())

    # decode of the same stream into a device buffer (reported, not the metric)
    back_t = torch.empty_like(field_t)
    lib.zfp_field_set_pointer(zf, ctypes.c_void_p(back_t.data_ptr()))
    dms = []
    for i in range(max(3, args.steps // 2)):
        lib.stream_rewind(bs)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if lib.zfp_decompress(zs, zf) == 0:
            raise RuntimeError("zfp_decompress failed: %s" % lib.zfp_hip_last_error())
        torch.cuda.synchronize()
        if i:
            dms.append((time.perf_counter() - t1) * 1e3)
    lib.zfp_field_set_pointer(zf, ctypes.c_void_p(field_t.data_ptr()))

    # gather of the chunk streams to rank 0 over RCCL (timed separately)
    gather = None
    if distributed:
        sizes = torch.tensor([nbytes], device=dev, dtype=torch.int64)
        all_sizes = [torch.zeros_like(sizes) for _ in range(world)]
        dist.all_gather(all_sizes, sizes)
        mx = int(max(s.item() for s in all_sizes))
        send = out_t[:mx]
        recv = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(world)] if rank == 0 else None
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        dist.gather(send, gather_list=recv, dst=0)
        torch.cuda.synchronize()
        gms = (time.perf_counter() - g0) * 1e3
        gt = torch.tensor([gms], device=dev)
        dist.all_reduce(gt, op=dist.ReduceOp.MAX)
        total_bytes = sum(int(s.item()) for s in all_sizes)
        gather = {"ms": float(gt.item()), "bytes": total_bytes, "GBps": total_bytes / (float(gt.item()) * 1e6)}

    if rank == 0:
        kernel_ms = float(np.mean(kms))
        alg_bytes = nvals * 4 + nvals * RATE // 8
        achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
        traffic, tsrc = traffic_from_profiles()
        value = world * nvals * 4 / (ms * 1e-3) / 1e9
        result = {
            "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (F1 smooth field generated on device)",
            "config": {"workload": "%d^3 float32 fixed-rate %d zfp_compress per GPU (BASELINE configs[1])" % (n, RATE),
                       "field_per_gpu": [n, n, n], "rate": RATE, "stream_bytes_per_gpu": int(nbytes),
                       "parallelism": "%d independent z-slab chunks, one per GPU" % world},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "encode3_aligned<float>", "kernel_ms": round(kernel_ms, 4),
                         "algorithmic_bytes_per_launch": alg_bytes, "traffic_source": tsrc},
            "call_ms": round(float(np.mean(tms)), 4),
            "decode_ms": round(float(np.mean(dms)), 4) if dms else None,
            "decode_GBps": round(nvals * 4 / (np.mean(dms) * 1e-3) / 1e9, 2) if dms else None,
            "gather": gather,
        }
        if not args.no_cpu and world == 1:
            threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
            nz_s = min(n, 256)
            sample = field_t[:nz_s].cpu().numpy()
            cb = cpu_baseline(sample, threads)
            if cb is not None:
                gbs, ref_bytes = cb
                gpu_bytes = out_t[: len(ref_bytes)].cpu().numpy().tobytes()
                result["cpu_baseline"] = {"value": round(gbs, 3), "unit": "GB/s", "cores": threads,
                                          "kind": "reference",
                                          "sample": "%dx%dx%d z-slab of the same field, zfp_compress exec=omp, best of 3"
                                                    % (n, n, nz_s)}
                result["bitexact_vs_reference"] = gpu_bytes == ref_bytes
            else:
                result["cpu_baseline"] = None
        print(json.dumps(result), flush=True)

    lib.stream_close(bs)
    lib.zfp_stream_close(zs)
    lib.zfp_field_free(zf)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
