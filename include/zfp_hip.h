/*
 * zfp_hip.h -- C-ABI of the MI355X (gfx950) codec library libzfp_hip.so.
 *
 * This is the seam the host C library (libzfp.so, include/zfp.h) calls for the
 * data-parallel hot path.  Plain pointers and sizes only: no HIP, torch or C++
 * types cross it, so any FFI (ctypes, cffi, Cython, cgo, JNI) can bind it.
 *
 * What each entry point replaces in the reference (SEP-software/zfp-par):
 *
 *   zfp_hip_compress    the execution-policy table slot of zfp_compress_call
 *                       (src/zfp.c:1510-1564) -> compress_strided_<T>_3/_4
 *                       (src/template/compress.c:67-153), i.e. the raster block
 *                       traversal plus the per-block codec of
 *                       src/template/{encodef,encode,encode3,encode4,revencode*}.c
 *   zfp_hip_decompress  the slot of zfp_decompress_call (src/zfp.c:1605-1649) ->
 *                       decompress_strided_<T>_3/_4 (src/template/decompress.c:66-140)
 *                       with the decoders of src/template/{decodef,decode,...}.c
 *   zfp_hip_index_*     no reference equivalent: variable-rate streams carry no
 *                       block offsets (docs execution.rst).  The GPU encoder can
 *                       emit a side-band block index; without one (a stream
 *                       from the reference, a file, another process) the
 *                       decoder first finds the block starts with a parallel
 *                       resynchronising parse of the stream (zfp_hip_index_build),
 *                       which replaces the serial block walk of
 *                       src/template/decompress.c:66-140.
 *
 * Memory: `field_base` and `words` may each be host or device (hipMalloc)
 * memory; the library stages host buffers through device memory itself.
 * Threading: distinct calls may run concurrently from different host threads
 * (each thread gets its own HIP stream and scratch); one call is not reentrant.
 * Errors: entry points return 0 on failure (unsupported type/dimensionality,
 * capacity too small, HIP error); zfp_hip_last_error() describes the failure.
 */
#ifndef ZFP_HIP_H
#define ZFP_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One (de)compression job: field geometry, chunk box, codec parameters. */
typedef struct zfp_hip_job {
  int32_t type;        /* zfp_type: 1 = int32, 2 = int64, 3 = float, 4 = double */
  int32_t dims;        /* 1 .. 4 */
  uint64_t n[4];       /* field extents, x first (zfp_field nx..nw) */
  int64_t s[4];        /* element strides, resolved (zfp_field_stride) */
  uint64_t f[4];       /* chunk box first element per axis (zfp_chunk fx..fw) */
  uint64_t e[4];       /* chunk box exclusive end per axis (zfp_chunk ex..ew) */
  uint32_t minbits;    /* zfp_stream parameters (zfp.h:90-97) */
  uint32_t maxbits;
  uint32_t maxprec;
  int32_t minexp;
} zfp_hip_job;

typedef struct zfp_hip_index zfp_hip_index;

/* Number of visible HIP devices (0 when no GPU or no driver). */
int zfp_hip_device_count(void);

/* Human-readable description of the last failure on this thread. */
const char* zfp_hip_last_error(void);

/* 1 if p points into HIP device memory (0 without a GPU).  The host bitstream
 * (stream_open) uses it to move the words it touches itself with hipMemcpy. */
int zfp_hip_is_device_ptr(const void* p);
/* Synchronous copy between any host/device pointers; 0 on failure. */
int zfp_hip_memcpy(void* dst, const void* src, size_t bytes);

/*
 * Encode the chunk box of `job` into the stream whose word array begins at
 * `words` (capacity `capacity_words` 64-bit words), starting at bit
 * `bit_offset`.  `head_word` holds the stream bits already written below
 * bit_offset in word bit_offset/64 (the bitstream's pending buffer).
 * On success the stream is written through the last partial word, which is
 * zero-padded (flushed); *end_bit receives the bit position after the last
 * block.  For variable-rate modes, `index` (optional) receives the block index.
 */
int zfp_hip_compress(const zfp_hip_job* job, const void* field_base, uint64_t* words,
                     uint64_t capacity_words, uint64_t bit_offset, uint64_t head_word,
                     int device, zfp_hip_index* index, uint64_t* end_bit);

/*
 * Decode the chunk box of `job` from the stream at `words` (readable capacity
 * `capacity_words`), starting at bit `bit_offset`; *end_bit receives the bit
 * position after the last block.  For variable-rate modes `index` is used when
 * it was made for this block count, layout and bit offset (zfp_hip_compress or
 * zfp_hip_index_build); otherwise (or when NULL) the stream is scanned first.
 */
int zfp_hip_decompress(const zfp_hip_job* job, void* field_base, const uint64_t* words,
                       uint64_t capacity_words, uint64_t bit_offset, int device,
                       const zfp_hip_index* index, uint64_t* end_bit);

/*
 * Build the block index of the variable-rate stream at `words` for the chunk
 * box of `job`, blocks starting at bit `bit_offset` (a parallel parse of the
 * stream on the GPU; see scan.h).  Returns 0 for fixed-rate jobs, truncated
 * streams or HIP errors.
 */
int zfp_hip_index_build(const zfp_hip_job* job, const uint64_t* words, uint64_t capacity_words,
                        uint64_t bit_offset, int device, zfp_hip_index* index);

/* Block index (variable-rate streams). */
zfp_hip_index* zfp_hip_index_create(void);
void zfp_hip_index_free(zfp_hip_index* index);
uint64_t zfp_hip_index_blocks(const zfp_hip_index* index);
/* serialise to / restore from host bytes (returns bytes written / NULL) */
size_t zfp_hip_index_export(const zfp_hip_index* index, void* buffer, size_t capacity);
zfp_hip_index* zfp_hip_index_import(const void* buffer, size_t bytes);

/*
 * Timing of the most recent zfp_hip_compress/zfp_hip_decompress on this
 * thread, from HIP events recorded on the stream the kernels ran on:
 * kernel_ms = the codec kernel alone, total_ms = everything enqueued by the
 * call (staging copies, fix-ups, kernel).  Returns 0 if no call has run.
 */
int zfp_hip_last_timing(double* kernel_ms, double* total_ms);

/* Index scan of the most recent call on this thread (decompress without a
 * matching index, or zfp_hip_index_build): its duration from HIP events and
 * the number of segment passes.  Returns 0 if that call did not scan. */
int zfp_hip_last_scan(double* scan_ms, int* passes);

/* 1 if the most recent zfp_hip_decompress on this thread was handed an index
 * that passed the stream fingerprint but whose block lengths disagreed with
 * the decoded blocks (an index made for another stream): that call decoded
 * the stream again after an index scan, so its output is still correct. */
int zfp_hip_last_stale_index(void);

/*
 * Device scratch: calls borrow a context (HIP stream + reusable buffers) from
 * a process-wide pool, so scratch is bounded by the peak number of concurrent
 * calls.  zfp_hip_scratch_bytes() reports what idle contexts hold;
 * zfp_hip_release_scratch() frees them (returns how many were freed).
 */
size_t zfp_hip_scratch_bytes(void);
int zfp_hip_release_scratch(void);

#ifdef __cplusplus
}
#endif

#endif
