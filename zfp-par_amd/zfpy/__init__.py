"""zfpy -- zfp compression for numpy arrays, running on AMD MI355X.

Drop-in for the reference package (zfpy/__init__.py of SEP-software/zfp-par):
compress_numpy / decompress_numpy, the mode constants, and zfp_parallel for
chunked compression of a shared array.  The codec runs in hand-written HIP
kernels (libzfp_hip.so) behind the zfp C API (libzfp.so).
"""
from .zfpy_c import (HEADER_FULL, HEADER_MAGIC, HEADER_META, HEADER_MODE, _decompress, compress_numpy,
                     compress_numpy_portion, decompress_numpy, decompress_numpy_portion, device_count, header,
                     mode_expert, mode_fixed_accuracy, mode_fixed_precision, mode_fixed_rate, mode_null,
                     mode_reversible, type_double, type_float, type_int32, type_int64, type_none, zfp_chunkit)
from ._zfp_par import zfp_p as zfp_parallel
from ._zfp_par import read_json_header, write_json_header

__all__ = ["compress_numpy", "decompress_numpy", "zfp_parallel", "header", "zfp_chunkit", "compress_numpy_portion",
           "decompress_numpy_portion", "mode_expert", "mode_fixed_accuracy", "mode_fixed_precision",
           "mode_fixed_rate", "mode_null", "mode_reversible", "type_none", "type_int32", "type_int64", "type_float",
           "type_double", "HEADER_FULL", "HEADER_MAGIC", "HEADER_META", "HEADER_MODE", "_decompress",
           "device_count", "read_json_header", "write_json_header"]
