/* Internal definitions shared by the host library's translation units. */
#ifndef ZFP_AMD_INTERNAL_H
#define ZFP_AMD_INTERNAL_H

#include "zfp.h"
#include "zfp/bitstream.h"

/* bit stream state (reference: include/zfp/bitstream.inl:133-143) */
struct bitstream {
  size_t bits;   /* number of buffered bits (0 <= bits < 64) */
  uint64 buffer; /* incoming/outgoing bits (partial word) */
  uint64* ptr;   /* next word to be read/written */
  uint64* begin; /* first word */
  uint64* end;   /* one past last word */
  int device;    /* the word array is HIP device memory: word I/O goes through hipMemcpy */
};

/* One block through the GPU codec at the stream's current position (the
 * low-level block API, zfp_block.c): a field of n[0..dims-1] <= 4 values with
 * strides st (in elements) at p.  Returns the bits written or read; the stream
 * is left just past the block, not flushed. */
size_t zfp_block_code(zfp_stream* zfp, zfp_type type, uint dims, void* p, const size_t* n, const ptrdiff_t* st,
                      int decode);

#endif
