"""zfpy_c for MI355X: the reference's Cython module surface over ctypes.

Mirrors python/zfpy_c.pyx of SEP-software/zfp-par (function names, argument
meaning, return types, error behaviour) but drives this framework's libzfp.so,
whose zfp_compress / zfp_decompress run on the GPU.  ctypes releases the GIL
for every foreign call, like the reference's `with nogil:` blocks (pyx:317,
:364, :587), so a ThreadPool over chunks runs concurrently.

Additions (keyword-only, optional):
  * `device=` on the compress/decompress functions selects the HIP device;
  * arrays exposing __cuda_array_interface__ (e.g. torch CUDA tensors) are
    accepted by compress_numpy and compressed straight from device memory;
  * variable-rate streams carry their GPU block index as an attribute of the
    returned bytes object (`ZfpBytes.block_index`), an optional shortcut:
    decompress uses it when present and otherwise (plain bytes, a file, a
    stream from another library) finds the block starts on the GPU by a
    parallel parse of the stream (zfp_hip_index_build), so any valid stream
    decodes, as with the reference.
"""
import ctypes
import itertools
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIBPATH = os.path.join(os.path.dirname(_HERE), "lib", "libzfp.so")
if not os.path.exists(_LIBPATH):
    raise ImportError("zfpy: native library %s is missing (build: make -C zfp-par_amd)" % _LIBPATH)
if os.environ.get("ZFPY_NO_TORCH") != "1":
    # PyTorch-ROCm bundles a HIP runtime with the same SONAME as /opt/rocm's but
    # reaches it through an unversioned NEEDED entry; if libzfp loaded first the
    # process would map two runtimes.  Loading torch first makes both share one.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
_lib = ctypes.CDLL(_LIBPATH)

_vp, _sz, _u32, _i32, _dbl, _u64, _pd = (ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint, ctypes.c_int,
                                         ctypes.c_double, ctypes.c_uint64, ctypes.c_ssize_t)
for _name, _res, _args in [
    ("zfp_stream_open", _vp, [_vp]), ("zfp_stream_close", None, [_vp]),
    ("zfp_stream_set_bit_stream", None, [_vp, _vp]), ("zfp_stream_rewind", None, [_vp]),
    ("zfp_stream_set_rate", _dbl, [_vp, _dbl, _i32, _u32, _i32]),
    ("zfp_stream_set_precision", _u32, [_vp, _u32]), ("zfp_stream_set_accuracy", _dbl, [_vp, _dbl]),
    ("zfp_stream_set_reversible", None, [_vp]), ("zfp_stream_compression_mode", _i32, [_vp]),
    ("zfp_stream_params", None, [_vp, _vp, _vp, _vp, _vp]), ("zfp_stream_rate", _dbl, [_vp, _u32]),
    ("zfp_stream_precision", _u32, [_vp]), ("zfp_stream_accuracy", _dbl, [_vp]),
    ("zfp_stream_maximum_size", _sz, [_vp, _vp]), ("zfp_stream_maximum_size_chunk", _sz, [_vp, _vp, _vp]),
    ("zfp_stream_set_hip_device", _i32, [_vp, _i32]), ("zfp_stream_hip_index", _vp, [_vp]),
    ("zfp_stream_set_hip_index", _i32, [_vp, _vp]),
    ("zfp_field_alloc", _vp, []), ("zfp_field_1d", _vp, [_vp, _i32, _sz]),
    ("zfp_field_2d", _vp, [_vp, _i32, _sz, _sz]), ("zfp_field_3d", _vp, [_vp, _i32, _sz, _sz, _sz]),
    ("zfp_field_4d", _vp, [_vp, _i32, _sz, _sz, _sz, _sz]), ("zfp_field_free", None, [_vp]),
    ("zfp_field_set_pointer", None, [_vp, _vp]), ("zfp_field_set_type", _i32, [_vp, _i32]),
    ("zfp_field_set_stride_1d", None, [_vp, _pd]), ("zfp_field_set_stride_2d", None, [_vp, _pd, _pd]),
    ("zfp_field_set_stride_3d", None, [_vp, _pd, _pd, _pd]),
    ("zfp_field_set_stride_4d", None, [_vp, _pd, _pd, _pd, _pd]),
    ("zfp_compress", _sz, [_vp, _vp]), ("zfp_decompress", _sz, [_vp, _vp]),
    ("zfp_compress_chunk", _sz, [_vp, _vp, _vp]), ("zfp_decompress_chunk", _sz, [_vp, _vp, _vp]),
    ("zfp_write_header", _sz, [_vp, _vp, _u32]), ("zfp_read_header", _sz, [_vp, _vp, _u32]),
    ("zfp_optimal_parts_from_size", _vp, [_i32, _vp, ctypes.c_float, _i32]),
    ("zfp_chunks_from_blocks", _vp, [_i32, _vp, _vp]), ("zfp_blocks_free", None, [_vp]),
    ("zfp_chunks_free", None, [_vp]),
    ("stream_open", _vp, [_vp, _sz]), ("stream_close", None, [_vp]),
    ("zfp_hip_index_free", None, [_vp]), ("zfp_hip_index_export", _sz, [_vp, _vp, _sz]),
    ("zfp_hip_index_import", _vp, [_vp, _sz]), ("zfp_hip_device_count", _i32, []),
]:
    _fn = getattr(_lib, _name)
    _fn.restype = _res
    _fn.argtypes = _args


class _Field(ctypes.Structure):
    """zfp_field (include/zfp.h)."""
    _fields_ = [("type", _i32), ("nx", _sz), ("ny", _sz), ("nz", _sz), ("nw", _sz),
                ("sx", _pd), ("sy", _pd), ("sz", _pd), ("sw", _pd), ("data", _vp)]


class _Chunk(ctypes.Structure):
    _fields_ = [("fx", _sz), ("fy", _sz), ("fz", _sz), ("fw", _sz),
                ("ex", _sz), ("ey", _sz), ("ez", _sz), ("ew", _sz)]


class _Chunks(ctypes.Structure):
    _fields_ = [("nchunks", _sz), ("chunks", ctypes.POINTER(ctypes.POINTER(_Chunk)))]


# exported #defines and enums (pyx:35-50)
HEADER_MAGIC = 0x1
HEADER_META = 0x2
HEADER_MODE = 0x4
HEADER_FULL = 0x7
HEADER_MAX_BITS = 148

type_none = 0
type_int32 = 1
type_int64 = 2
type_float = 3
type_double = 4
mode_null = 0
mode_expert = 1
mode_fixed_rate = 2
mode_fixed_precision = 3
mode_fixed_accuracy = 4
mode_reversible = 5


def dtype_to_ztype(dtype):
    dtype = np.dtype(dtype)
    for dt, zt in ((np.int32, type_int32), (np.int64, type_int64), (np.float32, type_float),
                   (np.float64, type_double)):
        if dtype == dt:
            return zt
    raise TypeError("Unknown dtype: {}".format(dtype))


def dtype_to_format(dtype):
    dtype = np.dtype(dtype)
    for dt, fmt in ((np.int32, "i"), (np.int64, "q"), (np.float32, "f"), (np.float64, "d")):
        if dtype == dt:
            return fmt
    raise TypeError("Unknown dtype: {}".format(dtype))


_zfp_to_dtype = {type_int32: np.int32, type_int64: np.int64, type_float: np.float32, type_double: np.float64}


def ztype_to_dtype(ztype):
    try:
        return _zfp_to_dtype[ztype]
    except KeyError:
        raise ValueError("Unsupported zfp_type {}".format(ztype))


_mode_names = {mode_null: "null", mode_expert: "expert", mode_reversible: "reversible",
               mode_fixed_accuracy: "tolerance", mode_fixed_precision: "precision", mode_fixed_rate: "rate"}


def zmode_to_str(zmode):
    try:
        return _mode_names[zmode]
    except KeyError:
        raise ValueError("Unsupported zfp_mode {}".format(zmode))


class ZfpBytes(bytes):
    """Compressed stream (a bytes object) that may carry its GPU block index."""
    block_index = None


# Stream buffers.  Output: a per-thread scratch buffer reused across calls
# (fresh pages of a new buffer cost a page fault each while the device-to-host
# copy fills them; the header and stream writers store whole words, so its old
# contents never reach the result), kept only up to _KEEP_OUT_MAX bytes so one
# huge call does not pin its buffer for the thread's lifetime.  The result is a
# new bytes object filled by ctypes.memmove, which runs with the GIL released:
# zfp_parallel's worker threads copy their chunk streams concurrently instead
# of queueing on the GIL (bytes(memoryview) copies under it).
_tls = threading.local()
_KEEP_OUT_MAX = 256 << 20

# (indexing makes a function object of its own: attribute access returns one
# shared object, whose restype the second binding below would overwrite)
_bytes_uninit = ctypes.pythonapi["PyBytes_FromStringAndSize"]
_bytes_uninit.restype = ctypes.py_object
_bytes_uninit.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t]


def _out_buffer(size):
    a = getattr(_tls, "out", None)
    if a is not None and a.size >= size:
        return a, a.ctypes.data
    a = np.empty(max(size, 1 << 20), dtype=np.uint8)
    if a.size <= _KEEP_OUT_MAX:
        _tls.out = a
    return a, a.ctypes.data


# PyBytes_AsString: the storage of a bytes object.  The C API lets a caller fill
# that storage only for an object it has just made with
# PyBytes_FromStringAndSize(NULL, n) and not yet shared -- exactly how the
# stream targets below are used.  Public API only: no private resize, no
# assumption about the object layout.
_bytes_addr = ctypes.pythonapi["PyBytes_AsString"]
_bytes_addr.restype = ctypes.c_void_p
_bytes_addr.argtypes = [ctypes.py_object]


try:
    _madvise = ctypes.CDLL(None, use_errno=True).madvise
    _madvise.restype = ctypes.c_int
    _madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
except (OSError, AttributeError):  # not Linux/glibc: pages fault in as written
    _madvise = None
_MADV_HUGEPAGE, _MADV_POPULATE_WRITE = 14, 23
_RESIDENT_MIN = 8 << 20


def _make_resident(addr, size):
    """Back a large new buffer with huge pages and fault them in here, in the
    calling thread (outside the GIL: ctypes releases it).  Otherwise every 4 KB
    page of a fresh stream faults inside the library's device-to-host copy:
    zfp_parallel's eight 64 MB chunk streams took 74-83 ms to compress instead
    of 54 ms (tools/exp/zpar_conc3.py, profiles/r4_zfp_parallel.txt).  Best
    effort: kernels without MADV_POPULATE_WRITE (Linux < 5.14) or without
    transparent huge pages ignore it."""
    if _madvise is None or size < _RESIDENT_MIN:
        return
    lo = (addr + 4095) & ~4095
    n = (addr + size - lo) & ~4095
    _madvise(lo, n, _MADV_HUGEPAGE)
    _madvise(lo, n, _MADV_POPULATE_WRITE)


def _bytes_target(size):
    """(bytes object, address): a new bytes object of exactly `size` bytes (> 0)
    that the library writes a stream into directly -- no staging buffer and no
    copy afterwards.  Only for streams whose length is known before they are
    written (fixed rate, _fixed_rate_size)."""
    if size <= 0:
        raise ValueError("stream target of %d bytes" % size)
    out = _bytes_uninit(None, size)  # uninitialised storage, refcount 1, hash not yet cached
    addr = _bytes_addr(out)
    _make_resident(addr, size)
    return out, addr


def _bytes_from(addr, n):
    """A new bytes object holding n bytes from address addr, copied outside the GIL."""
    out = _bytes_uninit(None, n)
    if n:
        ctypes.memmove(_bytes_addr(out), addr, n)
    return out


def _header_bits(stream, field):
    """Bits zfp_write_header(HEADER_FULL) writes for this stream and field (into scratch)."""
    scratch = (ctypes.c_uint64 * 4)()
    bs = _lib.stream_open(ctypes.addressof(scratch), ctypes.sizeof(scratch))
    try:
        _lib.zfp_stream_set_bit_stream(stream, bs)
        _lib.zfp_stream_rewind(stream)
        return int(_lib.zfp_write_header(stream, field, HEADER_FULL))
    finally:
        _lib.zfp_stream_set_bit_stream(stream, None)
        _lib.stream_close(bs)


def _fixed_rate_size(stream, field, nblocks, write_header):
    """Exact byte length of a fixed-rate stream: the header, nblocks blocks of
    maxbits bits each, flushed to a whole 64-bit word (zfp_compress's result)."""
    hbits = 0
    if write_header:
        hbits = _header_bits(stream, field)
        if hbits == 0:
            raise RuntimeError("Failed to write header to stream")
    mb, xb, mp, me = _u32(), _u32(), _u32(), _i32()
    _lib.zfp_stream_params(stream, ctypes.byref(mb), ctypes.byref(xb), ctypes.byref(mp), ctypes.byref(me))
    return (hbits + nblocks * int(xb.value) + 63) // 64 * 8


def _nblocks(extents):
    n = 1
    for e in extents:
        n *= (int(e) + 3) // 4
    return n


def _stream_bytes(obuf, n, index=None):
    """The returned stream.  A fixed-rate stream (no block index) is plain bytes,
    as the reference's zfpy returns, made by one copy with the GIL released.  A
    variable-rate stream with a block index is a ZfpBytes carrying it; building
    that bytes subclass from a buffer copies the data twice under the GIL (a
    plain bytes object, then the subclass object), so zfp_parallel keeps its
    chunks' indexes beside plain bytes instead (_compress_portion)."""
    if index is None:
        return _bytes_from(obuf.ctypes.data, n)
    out = ZfpBytes(memoryview(obuf)[:n])
    out.block_index = index
    return out


def _in_buffer(compressed_data):
    """(array, address) of the stream for the C reader.  A stream of whole 64-bit
    words -- every stream zfp writes is flushed to a word -- is read in place
    (the library copies whole words only, and never writes to it); otherwise it
    is copied into a zeroed buffer padded to a whole word plus one spare word."""
    src = np.frombuffer(compressed_data, dtype=np.uint8)
    if src.size and src.size % 8 == 0:
        return src, src.ctypes.data
    a = np.zeros((src.size + 15) // 8 * 8, dtype=np.uint8)
    a[:src.size] = src
    return a, a.ctypes.data


def _fixed_rate(tolerance, rate):
    """The mode _set_compression_mode picks is fixed rate (tolerance first, then
    rate): its stream has no block index, so it is returned as plain bytes and
    can be written straight into the result object."""
    return tolerance < 0 and rate >= 0


def _check_native(ret, what):
    if ret == 0:
        raise RuntimeError(what)
    return ret


def _set_compression_mode(stream, ztype, ndim, tolerance=-1, rate=-1, precision=-1):
    """pyx:414-429: first non-negative of tolerance, rate, precision; else reversible."""
    if tolerance >= 0:
        _lib.zfp_stream_set_accuracy(stream, tolerance)
    elif rate >= 0:
        _lib.zfp_stream_set_rate(stream, rate, ztype, ndim, 0)
    elif precision >= 0:
        _lib.zfp_stream_set_precision(stream, precision)
    else:
        _lib.zfp_stream_set_reversible(stream)


def _one_mode(tolerance, rate, precision):
    if sum(1 for x in (tolerance, rate, precision) if x >= 0) > 1:
        raise ValueError("Only one of tolerance, rate, or precision can be set")


def _make_field(pointer, ztype, shape_xfirst, strides_xfirst=None):
    nd = len(shape_xfirst)
    ctor = (_lib.zfp_field_1d, _lib.zfp_field_2d, _lib.zfp_field_3d, _lib.zfp_field_4d)
    if nd < 1 or nd > 4:
        raise RuntimeError("Greater than 4 dimensions not supported")
    field = ctor[nd - 1](pointer, ztype, *shape_xfirst)
    if strides_xfirst is not None:
        setter = (_lib.zfp_field_set_stride_1d, _lib.zfp_field_set_stride_2d, _lib.zfp_field_set_stride_3d,
                  _lib.zfp_field_set_stride_4d)
        setter[nd - 1](field, *strides_xfirst)
    return field


def _export_index(stream):
    idx = _lib.zfp_stream_hip_index(stream)
    if not idx:
        return None
    need = _lib.zfp_hip_index_export(idx, None, 0)
    buf = ctypes.create_string_buffer(need)
    if _lib.zfp_hip_index_export(idx, buf, need) != need:
        return None
    return buf.raw


def _attach_index(stream, blob):
    if not blob:
        return None
    idx = _lib.zfp_hip_index_import(blob, len(blob))
    if idx:
        _lib.zfp_stream_set_hip_index(stream, idx)
    return idx


def _array_pointer(arr):
    """(pointer, shape, strides in elements, dtype) for numpy or CUDA-array objects."""
    cai = getattr(arr, "__cuda_array_interface__", None)
    if cai is not None:
        dtype = np.dtype(cai["typestr"])
        shape = tuple(cai["shape"])
        st = cai.get("strides")
        if st is None:
            st, acc = [], dtype.itemsize
            for n in reversed(shape):
                st.insert(0, acc)
                acc *= n
        return cai["data"][0], shape, [s // dtype.itemsize for s in st], dtype
    if not isinstance(arr, np.ndarray):
        raise TypeError("Input must be a numpy array or expose __cuda_array_interface__")
    return arr.ctypes.data, arr.shape, [s // arr.itemsize for s in arr.strides], arr.dtype


def compress_numpy(arr, tolerance=-1, rate=-1, precision=-1, write_header=True, *, device=-1):
    """Compress a whole array into one stream (pyx:281-328)."""
    if arr is None:
        raise TypeError("Input array cannot be None")
    _one_mode(tolerance, rate, precision)
    ptr, shape, strides, dtype = _array_pointer(arr)
    ndim = len(shape)
    field = _make_field(ptr, dtype_to_ztype(dtype), list(reversed(shape)), list(reversed(strides)))
    stream = _lib.zfp_stream_open(None)
    bstream = None
    try:
        if device >= 0:
            _lib.zfp_stream_set_hip_device(stream, device)
        _set_compression_mode(stream, type_none, ndim, tolerance, rate, precision)
        maxsize = _lib.zfp_stream_maximum_size(stream, field)
        fixed = _fixed_rate(tolerance, rate)
        if fixed:
            maxsize = _fixed_rate_size(stream, field, _nblocks(shape), write_header)
            target, buf = _bytes_target(maxsize)
        else:
            obuf, buf = _out_buffer(maxsize)
        bstream = _lib.stream_open(buf, maxsize)
        _lib.zfp_stream_set_bit_stream(stream, bstream)
        _lib.zfp_stream_rewind(stream)
        if write_header and _lib.zfp_write_header(stream, field, HEADER_FULL) == 0:
            raise RuntimeError("Failed to write header to stream")
        n = _lib.zfp_compress(stream, field)
        if n == 0:
            raise RuntimeError("Failed to write to stream")
        if fixed:
            if n != maxsize:
                raise RuntimeError("fixed-rate stream of %d bytes, %d expected" % (n, maxsize))
            return target
        return _stream_bytes(obuf, n, _export_index(stream))
    finally:
        _lib.zfp_field_free(field)
        _lib.zfp_stream_close(stream)
        if bstream:
            _lib.stream_close(bstream)


def _decompress_into(stream, field_ptr, out, blob):
    fld = ctypes.cast(field_ptr, ctypes.POINTER(_Field)).contents
    fld.data = out.ctypes.data
    idx = _attach_index(stream, blob)
    try:
        ret = _lib.zfp_decompress(stream, field_ptr)
    finally:
        if idx:
            _lib.zfp_stream_set_hip_index(stream, None)
            _lib.zfp_hip_index_free(idx)
    if ret == 0:
        raise RuntimeError("error during zfp decompression")
    return out


def decompress_numpy(compressed_data, *, device=-1):
    """Decompress a stream written with a full header (pyx:533-557)."""
    if compressed_data is None:
        raise TypeError("compressed_data cannot be None")
    ibuf, buf = _in_buffer(compressed_data)
    field = _lib.zfp_field_alloc()
    bstream = _lib.stream_open(buf, ibuf.size)
    stream = _lib.zfp_stream_open(bstream)
    try:
        if device >= 0:
            _lib.zfp_stream_set_hip_device(stream, device)
        if _lib.zfp_read_header(stream, field, HEADER_FULL) == 0:
            raise ValueError("Failed to read required zfp header")
        fld = ctypes.cast(field, ctypes.POINTER(_Field)).contents
        shape = tuple(n for n in (fld.nw, fld.nz, fld.ny, fld.nx) if n > 0)
        out = np.empty(shape, dtype=ztype_to_dtype(fld.type))
        return _decompress_into(stream, field, out, getattr(compressed_data, "block_index", None))
    finally:
        _lib.zfp_field_free(field)
        _lib.zfp_stream_close(stream)
        _lib.stream_close(bstream)


def _decompress(compressed_data, ztype, shape, out=None, tolerance=-1, rate=-1, precision=-1, *, device=-1):
    """Headerless decompression with caller-supplied type, shape and mode (pyx:450-531)."""
    if compressed_data is None:
        raise TypeError("compressed_data cannot be None")
    if compressed_data is out:
        raise ValueError("Cannot decompress in-place")
    if len(shape) > 4:
        raise ValueError("User-provided shape has too many dimensions (up to 4 supported)")
    if len(shape) <= 0:
        raise ValueError("User-provided shape needs at least one dimension")
    ibuf, buf = _in_buffer(compressed_data)
    bstream = _lib.stream_open(buf, ibuf.size)
    stream = _lib.zfp_stream_open(bstream)
    dtype = ztype_to_dtype(ztype)
    zshape = [int(x) for x in itertools.islice(itertools.chain(reversed(shape), itertools.repeat(0)), 4)]
    field = _lib.zfp_field_alloc()
    try:
        if device >= 0:
            _lib.zfp_stream_set_hip_device(stream, device)
        fld = ctypes.cast(field, ctypes.POINTER(_Field)).contents
        fld.nx, fld.ny, fld.nz, fld.nw = zshape
        _lib.zfp_field_set_type(field, ztype)
        ndim = sum(1 for x in zshape if x > 0)
        _set_compression_mode(stream, ztype, ndim, tolerance, rate, precision)
        if out is None:
            output = np.empty(tuple(x for x in shape if x > 0), dtype=dtype)
        elif isinstance(out, np.ndarray):
            if out.dtype != dtype:
                raise ValueError("Out ndarray has dtype {} but decompression is using {}. Use out=ndarray.data "
                                 "to avoid this check.".format(out.dtype, dtype))
            if list(out.shape) != [x for x in shape if x > 0]:
                raise ValueError("Out ndarray has shape {} but decompression is using {}.  Use out=ndarray.data "
                                 "to avoid this check.".format(out.shape, [x for x in shape if x > 0]))
            output = out
        else:
            output = np.frombuffer(out, dtype=dtype).reshape(shape)
        return _decompress_into(stream, field, output, getattr(compressed_data, "block_index", None))
    finally:
        _lib.zfp_field_free(field)
        _lib.zfp_stream_close(stream)
        _lib.stream_close(bstream)


def header(compressed_data):
    """Stream header as a dict (pyx:596-650; `expert.maxbits` reports minbits as the reference does)."""
    if compressed_data is None:
        raise TypeError("compressed_data cannot be None")
    ibuf, buf = _in_buffer(compressed_data)
    field = _lib.zfp_field_alloc()
    bstream = _lib.stream_open(buf, ibuf.size)
    stream = _lib.zfp_stream_open(bstream)
    try:
        if _lib.zfp_read_header(stream, field, HEADER_FULL) == 0:
            raise ValueError("Failed to read required zfp header")
        mode = _lib.zfp_stream_compression_mode(stream)
        fld = ctypes.cast(field, ctypes.POINTER(_Field)).contents
        ndim = sum(1 for n in (fld.nx, fld.ny, fld.nz, fld.nw) if n > 0)
        mb, xb, mp, me = _u32(), _u32(), _u32(), _i32()
        _lib.zfp_stream_params(stream, ctypes.byref(mb), ctypes.byref(xb), ctypes.byref(mp), ctypes.byref(me))
        return {
            "nx": int(fld.nx), "ny": int(fld.ny), "nz": int(fld.nz), "nw": int(fld.nw),
            "type": ztype_to_dtype(fld.type), "mode": zmode_to_str(mode),
            "config": {
                "mode": int(mode),
                "tolerance": float(_lib.zfp_stream_accuracy(stream)),
                "rate": float(_lib.zfp_stream_rate(stream, ndim)),
                "precision": int(_lib.zfp_stream_precision(stream)),
                "expert": {"minbits": int(mb.value), "maxbits": int(mb.value), "maxprec": int(mp.value),
                           "minexp": int(me.value)},
            },
        }
    finally:
        _lib.zfp_field_free(field)
        _lib.zfp_stream_close(stream)
        _lib.stream_close(bstream)


class zfp_chunkit:
    """Chunk partition of an array (pyx:137-193): zfp_optimal_parts_from_size +
    zfp_chunks_from_blocks with zfp axis order (x = last numpy axis)."""

    def __init__(self, arr, chunks_per_block, method="BEST_CACHE"):
        method_opts = {"BEST_CACHE": 1, "MAKE_EQUAL": 2}
        method_c = method_opts.get(method, -1)
        if method_c == -1:
            raise ValueError("Invalid method '{}'. Valid options are: {}".format(method, ", ".join(method_opts)))
        shape = tuple(getattr(arr, "shape"))
        self.ndim = len(shape)
        nsize = (ctypes.c_int * self.ndim)(*[int(shape[self.ndim - 1 - i]) for i in range(self.ndim)])
        blocks = _lib.zfp_optimal_parts_from_size(self.ndim, nsize, ctypes.c_float(chunks_per_block), method_c)
        if not blocks:
            raise MemoryError("Failed to allocate zfp_blocks")
        chunks = _lib.zfp_chunks_from_blocks(self.ndim, nsize, blocks)
        if not chunks:
            _lib.zfp_blocks_free(blocks)
            raise MemoryError("Failed to allocate zfp_chunks")
        cs = ctypes.cast(chunks, ctypes.POINTER(_Chunks)).contents
        self.boxes = []
        for i in range(cs.nchunks):
            c = cs.chunks[i].contents
            self.boxes.append(((c.fx, c.ex), (c.fy, c.ey), (c.fz, c.ez), (c.fw, c.ew)))
        self.nchunks = int(cs.nchunks)
        self._chunks = chunks
        self._blocks = blocks
        self.ns_python = list(shape)
        self.n123 = int(np.prod(shape)) if shape else 0
        self.dtype = np.dtype(getattr(arr, "dtype"))

    def __del__(self):
        try:
            _lib.zfp_chunks_free(self._chunks)
            _lib.zfp_blocks_free(self._blocks)
        except Exception:
            pass

    def chunk_ptr(self, ichunk):
        cs = ctypes.cast(self._chunks, ctypes.POINTER(_Chunks)).contents
        if not 0 <= ichunk < cs.nchunks:
            raise IndexError("chunk index out of range")
        return ctypes.cast(cs.chunks[ichunk], _vp)

    def get_nchunks(self):
        return self.nchunks

    def get_ndim(self):
        return self.ndim  # (the reference's version recurses forever)

    def get_dtype(self):
        return self.dtype

    def get_shape(self):
        return self.ns_python


def _raw_pointer(py_raw_array):
    cai = getattr(py_raw_array, "__cuda_array_interface__", None)
    if cai is not None:
        return cai["data"][0]
    if isinstance(py_raw_array, np.ndarray):
        return py_raw_array.ctypes.data
    return ctypes.addressof(ctypes.c_char.from_buffer(py_raw_array))


def _init_field_raw(py_raw_array, chunkit):
    """Field over a raw buffer: zfp order sizes, strides (1, nx, nx*ny, ...) set explicitly (pyx:196-250)."""
    nd = chunkit.ndim
    shape = [chunkit.ns_python[nd - 1 - i] for i in range(nd)]
    strides = [1]
    for i in range(nd - 1):
        strides.append(strides[i] * shape[i])
    return _make_field(_raw_pointer(py_raw_array), dtype_to_ztype(chunkit.dtype), shape, strides)


def _compress_portion(py_raw_array, chunkit, ichunk, tolerance, rate, precision, write_header, device, plain):
    """compress_numpy_portion's work.  plain=False: its return value (a ZfpBytes
    when the stream has a block index); plain=True: (plain bytes, index blob or
    None), one GIL-free copy at most whatever the mode (zfp_parallel keeps the
    blobs).  A fixed-rate stream, whose length is known in advance, is written
    straight into the returned bytes; a variable-rate one goes through the
    thread's reusable staging buffer (its worst-case size is about the chunk's
    uncompressed size, far more than the stream)."""
    if py_raw_array is None:
        raise TypeError("Input array cannot be None")
    _one_mode(tolerance, rate, precision)
    field = _init_field_raw(py_raw_array, chunkit)
    stream = _lib.zfp_stream_open(None)
    bstream = None
    try:
        if device >= 0:
            _lib.zfp_stream_set_hip_device(stream, device)
        _set_compression_mode(stream, type_none, chunkit.ndim, tolerance, rate, precision)
        ck = chunkit.chunk_ptr(ichunk)
        fixed = _fixed_rate(tolerance, rate)
        if fixed:
            box = chunkit.boxes[ichunk][:chunkit.ndim]
            maxsize = _fixed_rate_size(stream, field, _nblocks(e - f for f, e in box), write_header)
            target, buf = _bytes_target(maxsize)
        else:
            maxsize = _lib.zfp_stream_maximum_size_chunk(stream, field, ck) + (HEADER_MAX_BITS + 63) // 64 * 8 + 8
            obuf, buf = _out_buffer(maxsize)
        bstream = _lib.stream_open(buf, maxsize)
        _lib.zfp_stream_set_bit_stream(stream, bstream)
        _lib.zfp_stream_rewind(stream)
        if write_header and _lib.zfp_write_header(stream, field, HEADER_FULL) == 0:
            raise RuntimeError("Failed to write header to stream")
        n = _lib.zfp_compress_chunk(stream, ck, field)
        if n == 0:
            raise RuntimeError("Failed to write to stream")
        if fixed:
            if n != maxsize:
                raise RuntimeError("fixed-rate chunk stream of %d bytes, %d expected" % (n, maxsize))
            return (target, None) if plain else target  # no block index: the reference's plain bytes
        blob = _export_index(stream)
        if plain:
            return _bytes_from(obuf.ctypes.data, n), blob
        return _stream_bytes(obuf, n, blob)
    finally:
        _lib.zfp_field_free(field)
        _lib.zfp_stream_close(stream)
        if bstream:
            _lib.stream_close(bstream)


def compress_numpy_portion(py_raw_array, chunkit, ichunk, tolerance=-1, rate=-1, precision=-1, write_header=True,
                           *, device=-1):
    """Compress one chunk into a self-contained stream: full whole-field header + the chunk's blocks
    (pyx:330-376).  The buffer reserves header room (the reference under-allocates)."""
    return _compress_portion(py_raw_array, chunkit, ichunk, tolerance, rate, precision, write_header, device, False)


def decompress_numpy_portion(compressed_data, py_raw_array, chunkit, ichunk, *, device=-1):
    """Decompress one chunk stream into its box of the shared array (pyx:559-593).  Like the
    reference, zfp_read_header resets the field strides to contiguous and nothing is returned."""
    _decompress_portion(compressed_data, py_raw_array, chunkit, ichunk, device,
                        getattr(compressed_data, "block_index", None))


def _decompress_portion(compressed_data, py_raw_array, chunkit, ichunk, device, blob):
    if compressed_data is None:
        raise TypeError("compressed_data cannot be None")
    field = _init_field_raw(py_raw_array, chunkit)
    ibuf, buf = _in_buffer(compressed_data)
    bstream = _lib.stream_open(buf, ibuf.size)
    stream = _lib.zfp_stream_open(bstream)
    idx = None
    try:
        if device >= 0:
            _lib.zfp_stream_set_hip_device(stream, device)
        if _lib.zfp_read_header(stream, field, HEADER_FULL) == 0:
            raise ValueError("Failed to read required zfp header")
        idx = _attach_index(stream, blob)
        ret = _lib.zfp_decompress_chunk(stream, chunkit.chunk_ptr(ichunk), field)
        if ret == 0:
            raise RuntimeError("error during zfp decompression")
    finally:
        if idx:
            _lib.zfp_stream_set_hip_index(stream, None)
            _lib.zfp_hip_index_free(idx)
        _lib.zfp_field_free(field)
        _lib.zfp_stream_close(stream)
        _lib.stream_close(bstream)


def device_count():
    """Number of visible HIP devices."""
    return int(_lib.zfp_hip_device_count())
