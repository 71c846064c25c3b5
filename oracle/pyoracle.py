"""TEST INFRASTRUCTURE ONLY -- ctypes bindings for the CPU oracle.

Loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only.
Never imported by the product (zfp-par_amd/).

  Oracle      oracle/build/liboracle.so    -- plain-C restatement of the codec
  RefLib      oracle/_ref/libzfp_ref.so    -- the reference itself (if built)
  RefTestLib  oracle/_ref/libzfptest_ref.so -- reference test generator (if built)
"""
import ctypes
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "build", "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libzfp_ref.so")
REFTEST_SO = os.path.join(HERE, "_ref", "libzfptest_ref.so")
REF_CLI = os.path.join(HERE, "_ref", "zfp_ref")

ZFP_MIN_BITS = 1
ZFP_MAX_BITS = 16658
ZFP_MAX_PREC = 64
ZFP_MIN_EXP = -1074

TYPE_FLOAT = 3
TYPE_DOUBLE = 4


class OzJob(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("minbits", ctypes.c_uint32), ("maxbits", ctypes.c_uint32),
                ("maxprec", ctypes.c_uint32), ("minexp", ctypes.c_int32),
                ("n", ctypes.c_uint64 * 4), ("s", ctypes.c_int64 * 4),
                ("f", ctypes.c_uint64 * 4), ("e", ctypes.c_uint64 * 4)]


# ---- mode parameter rules, restated from zfp.c:1157-1219 ----

def params_rate(rate, ztype, dims, align=False):
    """zfp_stream_set_rate (zfp.c:1166-1192); ztype 0 = zfp_type_none (zfpy)."""
    n = 1 << (2 * dims)
    bits = int(math.floor(n * rate + 0.5)) & 0xffffffff
    if ztype == TYPE_FLOAT:
        bits = max(bits, 9)
    elif ztype == TYPE_DOUBLE:
        bits = max(bits, 12)
    if align:
        bits = (bits + 63) & ~63
    return (bits, bits, ZFP_MAX_PREC, ZFP_MIN_EXP)


def params_precision(prec):
    """zfp_stream_set_precision (zfp.c:1194-1201)."""
    p = min(prec, ZFP_MAX_PREC) if prec else ZFP_MAX_PREC
    return (ZFP_MIN_BITS, ZFP_MAX_BITS, p, ZFP_MIN_EXP)


def params_accuracy(tol):
    """zfp_stream_set_accuracy (zfp.c:1204-1219)."""
    emin = ZFP_MIN_EXP
    if tol > 0:
        _, e = math.frexp(tol)
        emin = e - 1
    return (ZFP_MIN_BITS, ZFP_MAX_BITS, ZFP_MAX_PREC, emin)


def params_reversible():
    """zfp_stream_set_reversible (zfp.c:1157-1163)."""
    return (ZFP_MIN_BITS, ZFP_MAX_BITS, ZFP_MAX_PREC, ZFP_MIN_EXP - 1)


def ztype_of(arr):
    if arr.dtype == np.float32:
        return TYPE_FLOAT
    if arr.dtype == np.float64:
        return TYPE_DOUBLE
    raise TypeError(arr.dtype)


def max_block_bits(params, ztype, dims):
    """Per-block bound, as zfp_stream_maximum_size's inner term (zfp.c:1128-1148)."""
    minbits, maxbits, maxprec, minexp = params
    values = 1 << (2 * dims)
    rev = minexp < ZFP_MIN_EXP
    if ztype == TYPE_FLOAT:
        b = (1 + 1 + 8 + 5) if rev else (1 + 8)
        prec = 32
    else:
        b = (1 + 1 + 11 + 6) if rev else (1 + 11)
        prec = 64
    b += values - 1 + values * min(maxprec, prec)
    b = min(b, maxbits)
    return max(b, minbits)


class Oracle:
    def __init__(self, path=ORACLE_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path + " (run: make -C oracle)")
        lib = ctypes.CDLL(path)
        lib.oz_compress.restype = ctypes.c_uint64
        lib.oz_compress.argtypes = [ctypes.POINTER(OzJob), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        lib.oz_decompress.restype = ctypes.c_uint64
        lib.oz_decompress.argtypes = [ctypes.POINTER(OzJob), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64]
        lib.oz_block_bits.restype = ctypes.c_uint64
        lib.oz_block_bits.argtypes = [ctypes.POINTER(OzJob), ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_uint64]
        lib.oz_gen_smooth_floats.restype = ctypes.c_size_t
        lib.oz_gen_smooth_floats.argtypes = [ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
        lib.oz_gen_smooth_doubles.restype = ctypes.c_size_t
        lib.oz_gen_smooth_doubles.argtypes = [ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
        for fn in (lib.oz_gen_smooth_int32, lib.oz_gen_smooth_int64):
            fn.restype = ctypes.c_size_t
            fn.argtypes = [ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
        lib.oz_hash_words.restype = ctypes.c_uint64
        lib.oz_hash_words.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        lib.oz_hash_array32.restype = ctypes.c_uint32
        lib.oz_hash_array32.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        self.lib = lib

    # ---- generator and hashes (reference tests/utils restated) ----
    def smooth_field(self, dims, dtype, min_total=1000000):
        fn = {np.dtype(np.float32): self.lib.oz_gen_smooth_floats, np.dtype(np.float64): self.lib.oz_gen_smooth_doubles,
              np.dtype(np.int32): self.lib.oz_gen_smooth_int32, np.dtype(np.int64): self.lib.oz_gen_smooth_int64}[
            np.dtype(dtype)]
        side = fn(min_total, dims, None, 0)
        out = np.empty((side,) * dims, dtype=dtype)
        fn(min_total, dims, out.ctypes.data, out.size)
        return out

    def hash_words(self, words):
        words = np.ascontiguousarray(words, dtype=np.uint64)
        return int(self.lib.oz_hash_words(words.ctypes.data, words.size))

    def hash_array(self, arr):
        arr = np.ascontiguousarray(arr)
        if arr.dtype.itemsize == 4:
            return int(self.lib.oz_hash_array32(arr.ctypes.data, arr.size))
        return self.hash_words(arr.view(np.uint64))

    # ---- codec ----
    @staticmethod
    def make_job(arr_shape, ztype, params, strides=None, box=None):
        """arr_shape is numpy order (slowest first); zfp order is reversed."""
        j = OzJob()
        j.type = ztype
        j.minbits, j.maxbits, j.maxprec, j.minexp = params
        n = list(reversed(arr_shape)) + [0] * (4 - len(arr_shape))
        for a in range(4):
            j.n[a] = n[a]
            j.s[a] = 0 if strides is None else strides[a]
        dims = len(arr_shape)
        for a in range(4):
            if box is None:
                j.f[a], j.e[a] = 0, n[a]
            else:
                j.f[a], j.e[a] = box[a]
            if a >= dims:
                j.f[a], j.e[a] = 0, 0
        return j

    def compress_words(self, arr, params, box=None, bit_offset=0, strides=None, base=None):
        """Encode `arr` (or the chunk `box`) and return (words, end_bit)."""
        arr = np.ascontiguousarray(arr) if strides is None else arr
        ztype = ztype_of(arr)
        dims = arr.ndim
        j = self.make_job(arr.shape, ztype, params, strides, box)
        nblocks = 1
        for a in range(dims):
            nblocks *= (j.e[a] - j.f[a] + 3) // 4
        cap = (bit_offset + nblocks * max_block_bits(params, ztype, dims)) // 64 + 4
        words = np.zeros(cap, dtype=np.uint64)
        ptr = arr.ctypes.data if base is None else base
        end = self.lib.oz_compress(ctypes.byref(j), ptr, words.ctypes.data, bit_offset)
        nwords = (end + 63) // 64
        return words[:nwords].copy(), int(end)

    def decompress_words(self, words, shape, dtype, params, box=None, bit_offset=0, out=None):
        ztype = TYPE_FLOAT if dtype == np.float32 else TYPE_DOUBLE
        j = self.make_job(shape, ztype, params, None, box)
        if out is None:
            out = np.zeros(shape, dtype=dtype)
        w = np.zeros(len(words) + 4, dtype=np.uint64)
        w[:len(words)] = words
        end = self.lib.oz_decompress(ctypes.byref(j), out.ctypes.data, w.ctypes.data, bit_offset)
        return out, int(end)

    def block_bits(self, arr, params):
        arr = np.ascontiguousarray(arr)
        j = self.make_job(arr.shape, ztype_of(arr), params)
        nblocks = 1
        for a in range(arr.ndim):
            nblocks *= (j.e[a] - j.f[a] + 3) // 4
        lens = np.zeros(nblocks, dtype=np.uint32)
        scratch = np.zeros(600, dtype=np.uint64)
        self.lib.oz_block_bits(ctypes.byref(j), arr.ctypes.data, scratch.ctypes.data, lens.ctypes.data, nblocks)
        return lens


def have_ref():
    return os.path.exists(REF_SO)
