/*
 * zfp C API -- MI355X-native framework, drop-in for SEP-software/zfp-par.
 *
 * Struct layouts, enum values and prototypes follow the reference header
 * include/zfp.h (types :60-169, prototypes :183-908) for everything on the
 * data-parallel path: fields, streams, compression modes, headers, chunk boxes
 * and the chunk partitioner.  Compression and decompression run on the GPU
 * (hand-written HIP kernels for gfx950 in zfp-par_amd/csrc/hip, reached through
 * the C-ABI in include/zfp_hip.h); the field and stream buffers may live in
 * host or device memory.
 *
 * Additions (all additive, numbering of existing enums unchanged):
 *   zfp_exec_hip = 3            MI355X execution policy (zfp.h:72-76 gains a row)
 *   zfp_exec_params_hip         device ordinal
 *   zfp_stream_set_hip_device / zfp_stream_hip_index / zfp_stream_set_hip_index
 *                               (block index of a variable-rate stream: the GPU
 *                               decoder needs per-block offsets that the zfp
 *                               stream format does not store; zfp_compress keeps
 *                               the index with the zfp_stream, zfp_decompress on
 *                               that zfp_stream uses it)
 *
 * Errors follow the reference: functions return 0 (or NULL) on failure or for
 * an unsupported combination, leaving the bit stream untouched.
 */
#ifndef ZFP_H
#define ZFP_H

#include <stddef.h>
#include <stdint.h>

#include "zfp/bitstream.h"
#include "zfp/types.h"

/* version (reference include/zfp/version.h:5-11) */
#define ZFP_VERSION_MAJOR 1
#define ZFP_VERSION_MINOR 0
#define ZFP_VERSION_PATCH 1
#define ZFP_VERSION_TWEAK 0
#define ZFP_CODEC 5
#define ZFP_VERSION ((ZFP_VERSION_MAJOR << 12) + (ZFP_VERSION_MINOR << 8) + (ZFP_VERSION_PATCH << 4) + ZFP_VERSION_TWEAK)
#define ZFP_VERSION_STRING "1.0.1"

/* default compression parameters (zfp.h:18-21) */
#define ZFP_MIN_BITS 1
#define ZFP_MAX_BITS 16658
#define ZFP_MAX_PREC 64
#define ZFP_MIN_EXP -1074

/* header masks (zfp.h:24-28) */
#define ZFP_HEADER_NONE 0x0u
#define ZFP_HEADER_MAGIC 0x1u
#define ZFP_HEADER_META 0x2u
#define ZFP_HEADER_MODE 0x4u
#define ZFP_HEADER_FULL 0x7u

#define ZFP_META_NULL (UINT64C(-1))

/* header field widths (zfp.h:43-51) */
#define ZFP_MAGIC_BITS 32
#define ZFP_META_BITS 52
#define ZFP_MODE_SHORT_BITS 12
#define ZFP_MODE_LONG_BITS 64
#define ZFP_HEADER_MAX_BITS 148
#define ZFP_HEADER_BLOCKS_MAX_BITS 448
#define ZFP_MODE_SHORT_MAX ((1u << ZFP_MODE_SHORT_BITS) - 2)

/* rounding modes (zfp.h:54-56); this build is ZFP_ROUND_NEVER like the reference default */
#define ZFP_ROUND_FIRST (-1)
#define ZFP_ROUND_NEVER 0
#define ZFP_ROUND_LAST 1

/* chunk partitioner methods (zfp.h:58-59) */
#define ZFP_BEST_CACHE 1
#define ZFP_MAKE_EQUAL 2

enum { zfp_false = 0, zfp_true = !zfp_false };
typedef int zfp_bool;

/* execution policy (zfp.h:72-76) + MI355X */
typedef enum {
  zfp_exec_serial = 0,
  zfp_exec_omp = 1,
  zfp_exec_cuda = 2,
  zfp_exec_hip = 3
} zfp_exec_policy;

typedef struct {
  uint threads;
  uint chunk_size;
} zfp_exec_params_omp;

typedef struct zfp_hip_index zfp_hip_index; /* opaque; see zfp_hip.h */

typedef struct {
  int device; /* HIP device ordinal (-1: current device) */
} zfp_exec_params_hip;

typedef struct {
  zfp_exec_policy policy;
  void* params;
} zfp_execution;

/* compressed stream (zfp.h:90-97) */
typedef struct {
  uint minbits;
  uint maxbits;
  uint maxprec;
  int minexp;
  bitstream* stream;
  zfp_execution exec;
} zfp_stream;

typedef enum {
  zfp_mode_null = 0,
  zfp_mode_expert = 1,
  zfp_mode_fixed_rate = 2,
  zfp_mode_fixed_precision = 3,
  zfp_mode_fixed_accuracy = 4,
  zfp_mode_reversible = 5
} zfp_mode;

typedef struct {
  zfp_mode mode;
  union {
    double rate;
    uint precision;
    double tolerance;
    struct {
      uint minbits;
      uint maxbits;
      uint maxprec;
      int minexp;
    } expert;
  } arg;
} zfp_config;

typedef enum {
  zfp_type_none = 0,
  zfp_type_int32 = 1,
  zfp_type_int64 = 2,
  zfp_type_float = 3,
  zfp_type_double = 4
} zfp_type;

/* uncompressed array (zfp.h:135-140) */
typedef struct {
  zfp_type type;
  size_t nx, ny, nz, nw;
  ptrdiff_t sx, sy, sz, sw;
  void* data;
} zfp_field;

/* element box [f, e) per axis; e is an exclusive END INDEX (zfp.h:146-149) */
typedef struct {
  size_t fx, fy, fz, fw;
  size_t ex, ey, ez, ew;
} zfp_chunk;

typedef struct {
  size_t nchunks;
  zfp_chunk** chunks;
} zfp_chunks;

/* chunk partition: chunks per axis + bit offsets table (zfp.h:158-162) */
typedef struct {
  size_t bx, by, bz, bw;
  int nbeg;
  size_t* begs;
} zfp_blocks;

typedef struct {
  zfp_stream** streams;
  int nstreams;
} zfp_streams;

#ifdef __cplusplus
extern "C" {
#endif

extern const uint zfp_codec_version;
extern const uint zfp_library_version;
extern const char* const zfp_version_string;

size_t zfp_type_size(zfp_type type);

/* ---- compressed stream ---- */
zfp_stream* zfp_stream_open(bitstream* stream);
void zfp_stream_close(zfp_stream* stream);
bitstream* zfp_stream_bit_stream(const zfp_stream* stream);
zfp_mode zfp_stream_compression_mode(const zfp_stream* stream);
double zfp_stream_rate(const zfp_stream* stream, uint dims);
uint zfp_stream_precision(const zfp_stream* stream);
double zfp_stream_accuracy(const zfp_stream* stream);
uint64 zfp_stream_mode(const zfp_stream* stream);
void zfp_stream_params(const zfp_stream* stream, uint* minbits, uint* maxbits, uint* maxprec, int* minexp);
size_t zfp_stream_compressed_size(const zfp_stream* stream);
size_t zfp_stream_maximum_size(const zfp_stream* stream, const zfp_field* field);
size_t zfp_stream_maximum_size_chunk(const zfp_stream* stream, const zfp_field* field, const zfp_chunk* chunk);
size_t zfp_stream_maximum_size_blocks(const zfp_stream* stream, const zfp_field* field, const zfp_blocks* blocks);
void zfp_stream_rewind(zfp_stream* stream);
void zfp_stream_set_bit_stream(zfp_stream* stream, bitstream* bs);
void zfp_stream_set_reversible(zfp_stream* stream);
double zfp_stream_set_rate(zfp_stream* stream, double rate, zfp_type type, uint dims, zfp_bool align);
uint zfp_stream_set_precision(zfp_stream* stream, uint precision);
double zfp_stream_set_accuracy(zfp_stream* stream, double tolerance);
zfp_mode zfp_stream_set_mode(zfp_stream* stream, uint64 mode);
zfp_bool zfp_stream_set_params(zfp_stream* stream, uint minbits, uint maxbits, uint maxprec, int minexp);
size_t zfp_stream_flush(zfp_stream* stream);
size_t zfp_stream_align(zfp_stream* stream);

/* ---- execution policy ---- */
zfp_exec_policy zfp_stream_execution(const zfp_stream* stream);
uint zfp_stream_omp_threads(const zfp_stream* stream);
uint zfp_stream_omp_chunk_size(const zfp_stream* stream);
zfp_bool zfp_stream_set_execution(zfp_stream* stream, zfp_exec_policy policy);
zfp_bool zfp_stream_set_omp_threads(zfp_stream* stream, uint threads);
zfp_bool zfp_stream_set_omp_chunk_size(zfp_stream* stream, uint chunk_size);
/* MI355X additions */
zfp_bool zfp_stream_set_hip_device(zfp_stream* stream, int device);
zfp_hip_index* zfp_stream_hip_index(const zfp_stream* stream);
zfp_bool zfp_stream_set_hip_index(zfp_stream* stream, zfp_hip_index* index);

/* ---- configurations ---- */
zfp_config zfp_config_none(void);
zfp_config zfp_config_rate(double rate, zfp_bool align);
zfp_config zfp_config_precision(uint precision);
zfp_config zfp_config_accuracy(double tolerance);
zfp_config zfp_config_reversible(void);
zfp_config zfp_config_expert(uint minbits, uint maxbits, uint maxprec, int minexp);

/* ---- fields ---- */
zfp_field* zfp_field_alloc(void);
zfp_field* zfp_field_1d(void* pointer, zfp_type type, size_t nx);
zfp_field* zfp_field_2d(void* pointer, zfp_type type, size_t nx, size_t ny);
zfp_field* zfp_field_3d(void* pointer, zfp_type type, size_t nx, size_t ny, size_t nz);
zfp_field* zfp_field_4d(void* pointer, zfp_type type, size_t nx, size_t ny, size_t nz, size_t nw);
void zfp_field_free(zfp_field* field);
void* zfp_field_pointer(const zfp_field* field);
void* zfp_field_begin(const zfp_field* field);
zfp_type zfp_field_type(const zfp_field* field);
uint zfp_field_precision(const zfp_field* field);
uint zfp_field_dimensionality(const zfp_field* field);
size_t zfp_field_size(const zfp_field* field, size_t* size);
size_t zfp_field_size_bytes(const zfp_field* field);
size_t zfp_field_blocks(const zfp_field* field);
zfp_bool zfp_field_stride(const zfp_field* field, ptrdiff_t* stride);
zfp_bool zfp_field_is_contiguous(const zfp_field* field);
uint64 zfp_field_metadata(const zfp_field* field);
void zfp_field_set_pointer(zfp_field* field, void* pointer);
zfp_type zfp_field_set_type(zfp_field* field, zfp_type type);
void zfp_field_set_size_1d(zfp_field* field, size_t nx);
void zfp_field_set_size_2d(zfp_field* field, size_t nx, size_t ny);
void zfp_field_set_size_3d(zfp_field* field, size_t nx, size_t ny, size_t nz);
void zfp_field_set_size_4d(zfp_field* field, size_t nx, size_t ny, size_t nz, size_t nw);
void zfp_field_set_stride_1d(zfp_field* field, ptrdiff_t sx);
void zfp_field_set_stride_2d(zfp_field* field, ptrdiff_t sx, ptrdiff_t sy);
void zfp_field_set_stride_3d(zfp_field* field, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
void zfp_field_set_stride_4d(zfp_field* field, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
zfp_bool zfp_field_set_metadata(zfp_field* field, uint64 meta);

/* ---- chunk boxes and partitioner (fork API, zfp.h:280-304, :455-536, :905-908) ---- */
zfp_chunk* zfp_chunk_alloc(void);
void zfp_chunk_free(zfp_chunk* chunk);
zfp_chunks* zfp_chunks_alloc(const int nchunks);
void zfp_chunks_free(zfp_chunks* chunks);
zfp_blocks* zfp_blocks_alloc(void);
void zfp_alloc_nblocks(zfp_blocks* blocks, const size_t nblocks);
void zfp_blocks_free(zfp_blocks* blocks);
zfp_blocks* zfp_blocks_alloc_beg(const size_t nchunks, const size_t* begs);
void zfp_set_chunk_1d(zfp_chunk* chunk, const int fx, const int ex);
void zfp_set_chunk_2d(zfp_chunk* chunk, const int fx, const int fy, const int ex, const int ey);
void zfp_set_chunk_3d(zfp_chunk* chunk, const int fx, const int fy, const int fz, const int ex, const int ey, const int ez);
void zfp_set_chunk_4d(zfp_chunk* chunk, const int fx, const int fy, const int fz, const int fw,
                      const int ex, const int ey, const int ez, const int ew);
int zfp_break_axis(const int n, const int nparts, int* fwind, int* ewind);
zfp_blocks* zfp_optimal_parts_from_size(const int ndim, const int* n, const float chunks_per_block, const int method);
zfp_chunks* zfp_chunks_from_blocks(const int ndim, const int* nsize, const zfp_blocks* blocks);
zfp_blocks* zfp_break_into_blocks(const int ndim, const int* nsize, const int storage_per_block, const int elem_size,
                                  const float est_compression_rate, const int method);
int zfp_total_chunks(const int ndim, const zfp_blocks* blocks, int* nchunk_blocks);
int zfp_field_to_n(const zfp_field* field, int* n);

/* ---- compression (zfp.h:705-835) ---- */
size_t zfp_compress(zfp_stream* stream, const zfp_field* field);
size_t zfp_compress_chunk(zfp_stream* stream, const zfp_chunk* chunk, const zfp_field* field);
size_t zfp_decompress(zfp_stream* stream, zfp_field* field);
size_t zfp_decompress_chunk(zfp_stream* stream, const zfp_chunk* chunk, zfp_field* field);
/* zfp.h:797-838: dispatch with an explicit execution policy, strided flag,
 * dimensionality and scalar type (zfp_compress_chunk derives them) */
size_t zfp_compress_call(zfp_stream* stream, const zfp_chunk* chunk, const zfp_field* field, const uint exec,
                         const uint strided, const uint dims, const uint type);
size_t zfp_decompress_call(zfp_stream* stream, const zfp_chunk* chunk, zfp_field* field, const uint exec,
                           const uint strided, const uint dims, const uint type);
size_t zfp_write_header(zfp_stream* stream, const zfp_field* field, uint mask);
size_t zfp_read_header(zfp_stream* stream, zfp_field* field, uint mask);

/* ---- the fork's "blocks" API: chunk streams + offset header (zfp.h:714-868) ---- */
zfp_streams* zfp_streams_alloc(const int nstreams);
void zfp_streams_free(zfp_streams* streams);
zfp_streams* zfp_create_streams(const zfp_stream* zfp_in, const int nblocks, const size_t* blocks_boundaries);
zfp_streams* zfp_blocks_portions(zfp_stream* stream, const zfp_field* field, const int nthreads, zfp_blocks* blocks,
                                 size_t initial_pos);
size_t zfp_write_blocks_header(zfp_stream* stream, const zfp_field* field, const zfp_blocks* blocks,
                               const int begs_after_header);
size_t zfp_read_blocks_header(zfp_stream* stream, zfp_field* field, zfp_blocks* blocks);
zfp_streams* zfp_blocks_compress(zfp_stream* stream, const zfp_field* field, const int nthreads,
                                 const float blocks_per_chunk, const int method, const int begs_after_header);
zfp_streams* zfp_blocks_compress_multi(zfp_stream* stream, const zfp_field* field, const int nthreads,
                                       const float blocks_per_chunk, const int method);
size_t zfp_blocks_compress_single_stream(zfp_stream* stream, const zfp_field* field, const int nthreads,
                                         const float blocks_per_chunk, const int method);
size_t zfp_blocks_compress_internal(zfp_stream* stream, const zfp_field* field, const int nthreads,
                                    zfp_blocks* blocks);
size_t zfp_blocks_decompress(zfp_stream* stream, zfp_field* field, const int nthreads, const zfp_blocks* blocks);
size_t zfp_blocks_decompress_multi_stream(zfp_stream* stream, zfp_field* field, zfp_streams* streams,
                                          const int nthreads);
size_t zfp_blocks_decompress_single_stream(zfp_stream* stream, zfp_field* field, const int nthreads);

/* ---- low-level block API (zfp.h:911-1061): one block per call, run on the GPU ---- */
/* Each call codes one block at the stream's current bit position and leaves the
 * stream positioned after it (not flushed), returning the bits written / read.
 * A block is a field of at most 4 values per axis; partial blocks are padded
 * as at a field's edge (encode.c:9-27).  Every call is a GPU call. */
size_t zfp_encode_block_int32_1(zfp_stream* stream, const int32* block);
size_t zfp_encode_block_int64_1(zfp_stream* stream, const int64* block);
size_t zfp_encode_block_float_1(zfp_stream* stream, const float* block);
size_t zfp_encode_block_double_1(zfp_stream* stream, const double* block);
size_t zfp_encode_block_strided_int32_1(zfp_stream* stream, const int32* p, ptrdiff_t sx);
size_t zfp_encode_block_strided_int64_1(zfp_stream* stream, const int64* p, ptrdiff_t sx);
size_t zfp_encode_block_strided_float_1(zfp_stream* stream, const float* p, ptrdiff_t sx);
size_t zfp_encode_block_strided_double_1(zfp_stream* stream, const double* p, ptrdiff_t sx);
size_t zfp_encode_partial_block_strided_int32_1(zfp_stream* stream, const int32* p, size_t nx,
                                              ptrdiff_t sx);
size_t zfp_encode_partial_block_strided_int64_1(zfp_stream* stream, const int64* p, size_t nx,
                                              ptrdiff_t sx);
size_t zfp_encode_partial_block_strided_float_1(zfp_stream* stream, const float* p, size_t nx,
                                              ptrdiff_t sx);
size_t zfp_encode_partial_block_strided_double_1(zfp_stream* stream, const double* p, size_t nx,
                                              ptrdiff_t sx);
size_t zfp_encode_block_int32_2(zfp_stream* stream, const int32* block);
size_t zfp_encode_block_int64_2(zfp_stream* stream, const int64* block);
size_t zfp_encode_block_float_2(zfp_stream* stream, const float* block);
size_t zfp_encode_block_double_2(zfp_stream* stream, const double* block);
size_t zfp_encode_block_strided_int32_2(zfp_stream* stream, const int32* p, ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_encode_block_strided_int64_2(zfp_stream* stream, const int64* p, ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_encode_block_strided_float_2(zfp_stream* stream, const float* p, ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_encode_block_strided_double_2(zfp_stream* stream, const double* p, ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_encode_partial_block_strided_int32_2(zfp_stream* stream, const int32* p, size_t nx, size_t ny,
                                              ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_encode_partial_block_strided_int64_2(zfp_stream* stream, const int64* p, size_t nx, size_t ny,
                                              ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_encode_partial_block_strided_float_2(zfp_stream* stream, const float* p, size_t nx, size_t ny,
                                              ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_encode_partial_block_strided_double_2(zfp_stream* stream, const double* p, size_t nx, size_t ny,
                                              ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_encode_block_int32_3(zfp_stream* stream, const int32* block);
size_t zfp_encode_block_int64_3(zfp_stream* stream, const int64* block);
size_t zfp_encode_block_float_3(zfp_stream* stream, const float* block);
size_t zfp_encode_block_double_3(zfp_stream* stream, const double* block);
size_t zfp_encode_block_strided_int32_3(zfp_stream* stream, const int32* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_encode_block_strided_int64_3(zfp_stream* stream, const int64* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_encode_block_strided_float_3(zfp_stream* stream, const float* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_encode_block_strided_double_3(zfp_stream* stream, const double* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_encode_partial_block_strided_int32_3(zfp_stream* stream, const int32* p, size_t nx, size_t ny, size_t nz,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_encode_partial_block_strided_int64_3(zfp_stream* stream, const int64* p, size_t nx, size_t ny, size_t nz,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_encode_partial_block_strided_float_3(zfp_stream* stream, const float* p, size_t nx, size_t ny, size_t nz,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_encode_partial_block_strided_double_3(zfp_stream* stream, const double* p, size_t nx, size_t ny, size_t nz,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_encode_block_int32_4(zfp_stream* stream, const int32* block);
size_t zfp_encode_block_int64_4(zfp_stream* stream, const int64* block);
size_t zfp_encode_block_float_4(zfp_stream* stream, const float* block);
size_t zfp_encode_block_double_4(zfp_stream* stream, const double* block);
size_t zfp_encode_block_strided_int32_4(zfp_stream* stream, const int32* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_encode_block_strided_int64_4(zfp_stream* stream, const int64* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_encode_block_strided_float_4(zfp_stream* stream, const float* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_encode_block_strided_double_4(zfp_stream* stream, const double* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_encode_partial_block_strided_int32_4(zfp_stream* stream, const int32* p, size_t nx, size_t ny, size_t nz, size_t nw,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_encode_partial_block_strided_int64_4(zfp_stream* stream, const int64* p, size_t nx, size_t ny, size_t nz, size_t nw,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_encode_partial_block_strided_float_4(zfp_stream* stream, const float* p, size_t nx, size_t ny, size_t nz, size_t nw,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_encode_partial_block_strided_double_4(zfp_stream* stream, const double* p, size_t nx, size_t ny, size_t nz, size_t nw,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_decode_block_int32_1(zfp_stream* stream, int32* block);
size_t zfp_decode_block_int64_1(zfp_stream* stream, int64* block);
size_t zfp_decode_block_float_1(zfp_stream* stream, float* block);
size_t zfp_decode_block_double_1(zfp_stream* stream, double* block);
size_t zfp_decode_block_strided_int32_1(zfp_stream* stream, int32* p, ptrdiff_t sx);
size_t zfp_decode_block_strided_int64_1(zfp_stream* stream, int64* p, ptrdiff_t sx);
size_t zfp_decode_block_strided_float_1(zfp_stream* stream, float* p, ptrdiff_t sx);
size_t zfp_decode_block_strided_double_1(zfp_stream* stream, double* p, ptrdiff_t sx);
size_t zfp_decode_partial_block_strided_int32_1(zfp_stream* stream, int32* p, size_t nx,
                                              ptrdiff_t sx);
size_t zfp_decode_partial_block_strided_int64_1(zfp_stream* stream, int64* p, size_t nx,
                                              ptrdiff_t sx);
size_t zfp_decode_partial_block_strided_float_1(zfp_stream* stream, float* p, size_t nx,
                                              ptrdiff_t sx);
size_t zfp_decode_partial_block_strided_double_1(zfp_stream* stream, double* p, size_t nx,
                                              ptrdiff_t sx);
size_t zfp_decode_block_int32_2(zfp_stream* stream, int32* block);
size_t zfp_decode_block_int64_2(zfp_stream* stream, int64* block);
size_t zfp_decode_block_float_2(zfp_stream* stream, float* block);
size_t zfp_decode_block_double_2(zfp_stream* stream, double* block);
size_t zfp_decode_block_strided_int32_2(zfp_stream* stream, int32* p, ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_decode_block_strided_int64_2(zfp_stream* stream, int64* p, ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_decode_block_strided_float_2(zfp_stream* stream, float* p, ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_decode_block_strided_double_2(zfp_stream* stream, double* p, ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_decode_partial_block_strided_int32_2(zfp_stream* stream, int32* p, size_t nx, size_t ny,
                                              ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_decode_partial_block_strided_int64_2(zfp_stream* stream, int64* p, size_t nx, size_t ny,
                                              ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_decode_partial_block_strided_float_2(zfp_stream* stream, float* p, size_t nx, size_t ny,
                                              ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_decode_partial_block_strided_double_2(zfp_stream* stream, double* p, size_t nx, size_t ny,
                                              ptrdiff_t sx, ptrdiff_t sy);
size_t zfp_decode_block_int32_3(zfp_stream* stream, int32* block);
size_t zfp_decode_block_int64_3(zfp_stream* stream, int64* block);
size_t zfp_decode_block_float_3(zfp_stream* stream, float* block);
size_t zfp_decode_block_double_3(zfp_stream* stream, double* block);
size_t zfp_decode_block_strided_int32_3(zfp_stream* stream, int32* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_decode_block_strided_int64_3(zfp_stream* stream, int64* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_decode_block_strided_float_3(zfp_stream* stream, float* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_decode_block_strided_double_3(zfp_stream* stream, double* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_decode_partial_block_strided_int32_3(zfp_stream* stream, int32* p, size_t nx, size_t ny, size_t nz,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_decode_partial_block_strided_int64_3(zfp_stream* stream, int64* p, size_t nx, size_t ny, size_t nz,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_decode_partial_block_strided_float_3(zfp_stream* stream, float* p, size_t nx, size_t ny, size_t nz,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_decode_partial_block_strided_double_3(zfp_stream* stream, double* p, size_t nx, size_t ny, size_t nz,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz);
size_t zfp_decode_block_int32_4(zfp_stream* stream, int32* block);
size_t zfp_decode_block_int64_4(zfp_stream* stream, int64* block);
size_t zfp_decode_block_float_4(zfp_stream* stream, float* block);
size_t zfp_decode_block_double_4(zfp_stream* stream, double* block);
size_t zfp_decode_block_strided_int32_4(zfp_stream* stream, int32* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_decode_block_strided_int64_4(zfp_stream* stream, int64* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_decode_block_strided_float_4(zfp_stream* stream, float* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_decode_block_strided_double_4(zfp_stream* stream, double* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_decode_partial_block_strided_int32_4(zfp_stream* stream, int32* p, size_t nx, size_t ny, size_t nz, size_t nw,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_decode_partial_block_strided_int64_4(zfp_stream* stream, int64* p, size_t nx, size_t ny, size_t nz, size_t nw,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_decode_partial_block_strided_float_4(zfp_stream* stream, float* p, size_t nx, size_t ny, size_t nz, size_t nw,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
size_t zfp_decode_partial_block_strided_double_4(zfp_stream* stream, double* p, size_t nx, size_t ny, size_t nz, size_t nw,
                                              ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw);
void zfp_promote_int8_to_int32(int32* oblock, const int8* iblock, uint dims);
void zfp_promote_uint8_to_int32(int32* oblock, const uint8* iblock, uint dims);
void zfp_promote_int16_to_int32(int32* oblock, const int16* iblock, uint dims);
void zfp_promote_uint16_to_int32(int32* oblock, const uint16* iblock, uint dims);
void zfp_demote_int32_to_int8(int8* oblock, const int32* iblock, uint dims);
void zfp_demote_int32_to_uint8(uint8* oblock, const int32* iblock, uint dims);
void zfp_demote_int32_to_int16(int16* oblock, const int32* iblock, uint dims);
void zfp_demote_int32_to_uint16(uint16* oblock, const int32* iblock, uint dims);

#ifdef __cplusplus
}
#endif

#endif
