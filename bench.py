#!/usr/bin/env python3
"""Benchmark: GB/s uncompressed, 3D float32 fixed-rate encode, device-resident.

Workloads (--workload):
  c2 (default)  one step = zfp_compress of one 1024^3 float32 field at rate 16
                (BASELINE.json configs[1]) through the drop-in C API, field and
                stream already in HBM.  With N GPUs each rank compresses its own
                1024^3 z-slab chunk of an N*1024-plane field (weak scaling).
  c3            one step = zfp_compress of a 1024^3 float64 field at fixed
                precision 32 (configs[2]): variable-rate blocks, decoupled
                look-back, block index; per rank its own 1024^3 z-slab.
  c4            one step = the zfpy chunk stream of configs[3]: per rank one
                4096x4096x64 float32 z-slab of the 4096x4096x512 field, rate 8,
                written after the 96-bit whole-field header exactly as
                compress_numpy_portion lays it out (python/zfpy_c.pyx:330-376).
  c5            one step = zfp_compress in reversible (lossless) mode of one
                512x512x512x64 float32 w-slab of the 512^4 field of configs[4]
                (4D blocks); rank r owns slab r (8 ranks = the whole field).
                The lossless round trip is checked on the device.
Chunks are independent zfp streams, so the timed region has no collective; the
RCCL gather that concatenates the chunk streams on rank 0 is timed separately
and reported as `gather`, never inside `value`.

--gpus N without WORLD_SIZE in the environment re-launches this script under
torch.distributed.run with N ranks (before anything touches a GPU) and exits
with its status.  --dry-run runs the launcher, barriers and max-over-ranks
timing on CPU with gloo (a numpy copy stands in for the codec) -- for tests.

Printed JSON (rank 0): the contract keys plus
  roofline      dominant kernel (c2: encode3_aligned_full) against HBM peak: achieved =
                algorithmic bytes per launch (4 B read + R/8 B written per value)
                / mean kernel time from HIP events on the kernel's own stream;
                traffic = PMC HBM bytes per encode call (every dispatch of the call summed)
                from profiles/<round>_pmc_<workload>.json made by tools/pmc_bench.sh for
                the same workload and field (gfx950 FETCH_SIZE x2 correction), else null
                with traffic_null_reason
  cpu_baseline  the reference itself (oracle/_ref/libzfp_ref.so, compiled from
                /root/reference), OpenMP, every core this process may use, on
                the full per-GPU field (c2)
  decode_*      zfp_decompress of the same stream (same field, device-resident)
  bitexact      GPU stream bytes == reference CPU stream bytes (whole field)
"""
import argparse
import ctypes
import glob
import json
import os
import socket
import subprocess
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


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", choices=("c2", "c3", "c4", "c5"), default="c2")
    ap.add_argument("--n", type=int, default=N, help="c2: edge of the per-GPU cube (default 1024)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--clock-warm-ms", type=float, default=250.0,
                    help="untimed steps for at least this long before the W warmup steps: a cold MI355X needs "
                         "about 20 ms of work to reach its steady clock (DESIGN.md 3.4), more than W=5 C2 steps")
    ap.add_argument("--dry-run", action="store_true", help="CPU/gloo plumbing check, no GPU")
    return ap.parse_args(argv)


def relaunch(args):
    """Start N ranks under torch.distributed.run as a child process (this
    process has not initialised HIP) and return its exit status."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def smooth_slab_torch(torch, nx, ny, nz, z0, device, dtype=None):
    """F1: v = sin(.05x) cos(.03y) + .5 sin(.02z + .01 x y / nx), x fastest, planes z0.."""
    dtype = dtype or torch.float32
    x = torch.arange(nx, device=device, dtype=torch.float64)
    y = torch.arange(ny, device=device, dtype=torch.float64)
    out = torch.empty((nz, ny, nx), device=device, dtype=dtype)
    base = (torch.sin(0.05 * x)[None, :] * torch.cos(0.03 * y)[:, None])
    xy = 0.01 * x[None, :] * y[:, None] / nx
    for k in range(nz):
        z = float(z0 + k)
        out[k] = (base + 0.5 * torch.sin(0.02 * z + xy)).to(dtype)
    return out


def smooth_4d_torch(torch, n, nw, w0, device):
    """F1 with the C5 w term: F1(x, y, z) + .25 cos(.04 w) for w = w0 .. w0 + nw - 1,
    computed in float64 and rounded once (as tools/kprof.py field4)."""
    import math
    x = torch.arange(n, device=device, dtype=torch.float64)
    base = torch.sin(0.05 * x)[None, :] * torch.cos(0.03 * x)[:, None]
    xy = 0.01 * x[None, :] * x[:, None] / n
    z = x[:, None, None]
    f3 = base[None] + 0.5 * torch.sin(0.02 * z + xy[None])
    out = torch.empty((nw, n, n, n), device=device, dtype=torch.float32)
    for w in range(nw):
        out[w] = (f3 + 0.25 * math.cos(0.04 * (w0 + w))).to(torch.float32)
    del f3
    return out


def load_capi(path):
    from capi import ZfpCAPI
    return ZfpCAPI(path)


def traffic_from_profiles(workload, field_ext, alg_bytes):
    """(per-call HBM bytes, source file, reason) of this workload's encode call from the newest
    committed profiles/<round>_pmc_<workload>.json -- tools/pmc_bench.sh output: rocprofv3 --pmc
    passes over this bench command, FETCH_SIZE x2 + WRITE_SIZE summed over every dispatch of the
    call (the main kernel, its fix-ups, a patch or redo launch) and divided by the number of calls.
    Only a summary made for the same workload, field and algorithmic bytes is taken; otherwise the
    traffic is null and `reason` says why."""
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*pmc_%s.json" % workload)),
                   key=lambda f: os.path.basename(f).split("_")[0])
    reason = "no profiles/*pmc_%s.json" % workload
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        meta, call = d.get("meta") or {}, d.get("encode_call") or {}
        if meta.get("workload_key") != workload or list(meta.get("field_per_gpu") or []) != list(field_ext):
            reason = "%s: made for another workload or field" % os.path.basename(f)
            continue
        if meta.get("algorithmic_bytes_per_call") != alg_bytes:
            reason = "%s: algorithmic bytes differ (another stream)" % os.path.basename(f)
            continue
        if not call.get("hbm_bytes_per_call"):
            reason = "%s: no per-call FETCH_SIZE/WRITE_SIZE" % os.path.basename(f)
            continue
        return call["hbm_bytes_per_call"], os.path.basename(f), None
    return None, None, reason


def host_cores():
    """CPUs this process may run on: the affinity mask, capped by a cgroup CPU quota."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except Exception:
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return min(aff, quota) if quota else aff, aff, quota, model


def cpu_baseline(field_np, mode, param, threads):
    """The reference library (OpenMP policy) compressing `field_np` in `mode`; returns (GB/s, stream bytes, best s)."""
    from pyoracle import REF_SO
    if not os.path.exists(REF_SO):
        return None
    ref = load_capi(REF_SO)
    ref.lib.zfp_stream_set_omp_threads.restype = ctypes.c_int
    ref.lib.zfp_stream_set_omp_threads.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    f = ref.field_for(field_np)
    zs = ref.lib.zfp_stream_open(None)
    ref.set_mode(zs, mode, param, 3 if field_np.dtype == np.float32 else 4, field_np.ndim)
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
    return field_np.nbytes / best / 1e9, buf[:nbytes], best


# per workload: BASELINE config, dims, scalar, mode, dominant kernel, CPU-baseline sample (leading slab)
WORKLOADS = {
    "c2": dict(metric=METRIC, cfg="configs[1]", dtype="f32", mode="rate", param=16,
               kernel="encode3_aligned_full<float>", sample_planes=None),
    "c3": dict(metric="GB/s uncompressed, 3D float64 fixed-precision-32 encode, device-resident", cfg="configs[2]",
               dtype="f64", mode="precision", param=32, kernel="encode3_general<double, hi planes>",
               sample_planes=256),
    "c4": dict(metric=METRIC, cfg="configs[3]", dtype="f32", mode="rate", param=8, kernel="encode3_aligned<float>",
               sample_planes=None),
    "c5": dict(metric="GB/s uncompressed, 4D float32 reversible (lossless) encode, device-resident", cfg="configs[4]",
               dtype="f32", mode="reversible", param=None, kernel="encode4<float, reversible>", sample_planes=4),
}


def main():
    args = parse_args()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch(args))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    if args.dry_run:
        if distributed:
            dist.init_process_group("gloo")
        return dry_run(args, torch, dist, world, rank)

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if distributed:
        dist.init_process_group("nccl", device_id=dev)

    # ZFP_BENCH_LIB: a variant build for A/B timing (tools/exp); the product library otherwise
    api = load_capi(os.environ.get("ZFP_BENCH_LIB") or os.path.join(REPO, "zfp-par_amd", "lib", "libzfp.so"))
    api.enable_index()
    lib = api.lib
    lib.zfp_hip_last_timing.argtypes = [ctypes.c_void_p, ctypes.c_void_p]

    wl = WORKLOADS[args.workload]
    f64 = wl["dtype"] == "f64"
    tdtype = torch.float64 if f64 else torch.float32
    es = 8 if f64 else 4
    ztype = 4 if f64 else 3
    hdr_field = None
    if args.workload in ("c2", "c3"):
        n = args.n
        shape = (n, n, n)  # numpy order: z, y, x
        field_t = smooth_slab_torch(torch, n, n, n, rank * n, dev, tdtype)
        workload = "%d^3 %s %s zfp_compress per GPU (BASELINE %s)" % (
            n, "float64" if f64 else "float32",
            "fixed-rate %g" % wl["param"] if wl["mode"] == "rate" else "fixed-precision %d" % wl["param"], wl["cfg"])
        parallelism = "%d independent z-slab chunks, one per GPU" % world
    elif args.workload == "c4":
        shape = (64, 4096, 4096)
        field_t = smooth_slab_torch(torch, 4096, 4096, 64, rank * 64, dev)
        workload = ("4096x4096x64 float32 fixed-rate 8 z-slab per GPU = one zfpy chunk of 4096x4096x512 "
                    "(BASELINE configs[3]), stream after the 96-bit whole-field header")
        parallelism = "%d independent z-slab chunks, one per GPU" % world
    else:
        n4 = 512 if args.n == N else args.n
        nw = 64 if args.n == N else max(1, args.n // 8)
        shape = (nw, n4, n4, n4)
        field_t = smooth_4d_torch(torch, n4, nw, rank * nw, dev)
        workload = ("%dx%dx%dx%d float32 reversible w-slab per GPU = chunk %d of the %d^4 field of BASELINE "
                    "configs[4] (4D blocks)" % (n4, n4, n4, nw, rank, n4))
        parallelism = "%d independent w-slab chunks, one per GPU" % world
    nvals = field_t.numel()
    dims = len(shape)
    ext = list(reversed(shape))
    ptr = ctypes.c_void_p(field_t.data_ptr())
    zf = lib.zfp_field_3d(ptr, ztype, *ext) if dims == 3 else lib.zfp_field_4d(ptr, ztype, *ext)
    zs = lib.zfp_stream_open(None)
    if args.workload == "c4":
        # zfpy passes zfp_type_none to set_rate (pyx:300-302); the C API bench passes the scalar type
        lib.zfp_stream_set_rate(zs, 8.0, 0, 3, 0)
        hdr_field = lib.zfp_field_3d(None, 3, 4096, 4096, 512)  # header of the whole field, in the device stream
    else:
        api.set_mode(zs, wl["mode"], wl["param"], ztype, dims)
    cap = lib.zfp_stream_maximum_size(zs, zf) + 64
    out_t = torch.zeros(cap, dtype=torch.uint8, device=dev)
    bs = lib.stream_open(ctypes.c_void_p(out_t.data_ptr()), cap)
    lib.zfp_stream_set_bit_stream(zs, bs)

    def step():
        lib.zfp_stream_rewind(zs)
        if hdr_field is not None and lib.zfp_write_header(zs, hdr_field, 7) != 96:
            raise RuntimeError("zfp_write_header failed")
        nb = lib.zfp_compress(zs, zf)
        if nb == 0:
            raise RuntimeError("zfp_compress failed: %s" % lib.zfp_hip_last_error())
        return nb

    nbytes = 0
    # clock warm-up (untimed, like the warmup steps): steady-clock throughput
    warm_launches = 0
    tw = time.perf_counter()
    while (time.perf_counter() - tw) * 1e3 < args.clock_warm_ms:
        step()
        warm_launches += 1
        if warm_launches % 8 == 0:
            torch.cuda.synchronize()
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
    ms = elapsed / max(1, args.steps) * 1e3
    if distributed:
        tt = torch.tensor([ms], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        ms = float(tt.item())

    # decode of the same stream into a device buffer (reported, not the metric); variable-rate
    # streams decode with the block index the compress call left on the stream
    back_t = torch.empty_like(field_t)
    lib.zfp_field_set_pointer(zf, ctypes.c_void_p(back_t.data_ptr()))
    dms, dkms = [], []
    n_decode = max(3, args.steps // 2)
    for i in range(n_decode):
        lib.zfp_stream_rewind(zs)
        if hdr_field is not None:
            lib.stream_rseek(bs, 96)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        if lib.zfp_decompress(zs, zf) == 0:
            raise RuntimeError("zfp_decompress failed: %s" % lib.zfp_hip_last_error())
        torch.cuda.synchronize()
        if i:
            dms.append((time.perf_counter() - t1) * 1e3)
            k, t = ctypes.c_double(), ctypes.c_double()
            lib.zfp_hip_last_timing(ctypes.byref(k), ctypes.byref(t))
            dkms.append(k.value)
    lib.zfp_field_set_pointer(zf, ctypes.c_void_p(field_t.data_ptr()))
    roundtrip = {}
    if wl["mode"] == "reversible":
        roundtrip["lossless_roundtrip"] = bool(torch.equal(back_t, field_t))
    else:
        roundtrip["decode_max_abs_err"] = float((back_t - field_t).abs().max().item())
    del back_t

    # gather of the chunk streams to rank 0 over RCCL (timed separately): every rank
    # sends exactly its stream (point to point, no padding to the largest), as
    # zfpy.distributed.gather_streams does
    gather = None
    if distributed:
        sizes = torch.zeros(world, device=dev, dtype=torch.int64)
        sizes[rank] = nbytes
        dist.all_reduce(sizes, op=dist.ReduceOp.SUM)
        sz = [int(x) for x in sizes.cpu().tolist()]
        recv = [torch.empty(sz[r], dtype=torch.uint8, device=dev) for r in range(world)] if rank == 0 else None
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        if rank == 0:
            ops = [dist.P2POp(dist.irecv, recv[r], r) for r in range(1, world) if sz[r]]
            recv[0].copy_(out_t[:sz[0]])
        else:
            ops = [dist.P2POp(dist.isend, out_t[:sz[rank]], 0)] if sz[rank] else []
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        torch.cuda.synchronize()
        gms = (time.perf_counter() - g0) * 1e3
        gt = torch.tensor([gms], device=dev)
        dist.all_reduce(gt, op=dist.ReduceOp.MAX)
        total_bytes = sum(sz)
        gather = {"ms": round(float(gt.item()), 3), "bytes": total_bytes,
                  "GBps": round(total_bytes / (float(gt.item()) * 1e6), 2),
                  "collective": "RCCL point-to-point gather of exact-size chunk streams to rank 0"}
        del recv

    if rank == 0:
        kernel_ms = float(np.mean(kms))
        # algorithmic bytes of the dominant kernel: the field read once, the stream written once
        stream_bytes = nvals * wl["param"] // 8 if wl["mode"] == "rate" else int(nbytes)
        alg_bytes = nvals * es + stream_bytes
        achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9
        traffic, tsrc, treason = traffic_from_profiles(args.workload, ext, alg_bytes)
        value = world * nvals * es / (ms * 1e-3) / 1e9
        result = {
            "metric": wl["metric"], "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": wl["dtype"], "data": "synthetic (F1 smooth field generated on device)",
            "config": {"workload": workload, "field_per_gpu": ext, "mode": wl["mode"], "param": wl["param"],
                       "stream_bytes_per_gpu": int(nbytes), "parallelism": parallelism},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": wl["kernel"], "kernel_ms": round(kernel_ms, 4),
                         "algorithmic_bytes_per_launch": alg_bytes, "traffic_source": tsrc,
                         "traffic_per": "encode call (every dispatch of the call summed)",
                         **({"traffic_null_reason": treason} if traffic is None else {})},
            "call_ms": round(float(np.mean(tms)), 4),
            "decode_ms": round(float(np.mean(dms)), 4) if dms else None,
            "decode_kernel_ms": round(float(np.mean(dkms)), 4) if dkms else None,
            "decode_GBps": round(nvals * es / (np.mean(dms) * 1e-3) / 1e9, 2) if dms else None,
            "gather": gather,
            "clock_warmup": {"ms": args.clock_warm_ms, "launches": warm_launches},
            "workload_key": args.workload,
            "calls": {"encode": warm_launches + args.warmup + args.steps, "decode": n_decode},
        }
        result.update(roundtrip)
        if not args.no_cpu and world == 1 and args.workload != "c4":
            cores, aff, quota, model = host_cores()
            planes = wl["sample_planes"]
            sample_t = field_t if planes is None else field_t[:planes]
            sample = sample_t.cpu().numpy()
            cb = cpu_baseline(sample, wl["mode"], wl["param"], cores)
            if cb is not None:
                gbs, ref_bytes, best = cb
                what = ("the full %s field" % "x".join(map(str, ext)) if planes is None else
                        "the leading %s slab of the per-GPU field" % "x".join(map(str, list(reversed(sample.shape)))))
                result["cpu_baseline"] = {
                    "value": round(gbs, 3), "unit": "GB/s", "cores": cores, "kind": "reference",
                    "sample": "%s, reference zfp_compress exec=omp with %d threads, best of 3 (%.3f s)" % (
                        what, cores, best),
                    "cpu_model": model, "affinity_cpus": aff, "cgroup_cpu_quota": quota}
                # the sample is a leading slab: its stream is a prefix of the GPU stream (blocks in
                # raster order); the last word also holds the next blocks' bits on the GPU side
                nw_cmp = len(ref_bytes) // 8 - (0 if planes is None else 1)
                gpu_bytes = out_t[: nw_cmp * 8].cpu().numpy()
                result["bitexact_vs_reference"] = bool(np.array_equal(gpu_bytes, ref_bytes[: nw_cmp * 8]))
            else:
                result["cpu_baseline"] = None
        print(json.dumps(result), flush=True)

    lib.stream_close(bs)
    lib.zfp_stream_close(zs)
    lib.zfp_field_free(zf)
    if hdr_field is not None:
        lib.zfp_field_free(hdr_field)
    if distributed:
        dist.destroy_process_group()


def dry_run(args, torch, dist, world, rank):
    """Launcher/timing plumbing on CPU: a numpy copy of a small field stands in
    for the codec step; the JSON says so (`dry_run`)."""
    distributed = world > 1
    src = np.random.default_rng(rank).standard_normal(1 << 20).astype(np.float32)
    dst = np.empty_like(src)
    for _ in range(args.warmup):
        np.copyto(dst, src)
    if distributed:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        np.copyto(dst, src)
    if distributed:
        dist.barrier()
    ms = (time.perf_counter() - t0) / max(1, args.steps) * 1e3
    if distributed:
        t = torch.tensor([ms])
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": round(world * src.nbytes / (ms * 1e-3) / 1e9, 3), "unit": "GB/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
                          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
                          "data": "synthetic", "dry_run": True,
                          "config": {"workload": "dry run of --workload %s: numpy copy of 4 MiB per rank "
                                                 "(no codec, no GPU)" % args.workload}}),
              flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
