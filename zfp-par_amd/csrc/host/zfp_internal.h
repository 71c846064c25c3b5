/* Internal definitions shared by the host library's translation units. */
#ifndef ZFP_AMD_INTERNAL_H
#define ZFP_AMD_INTERNAL_H

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

#endif
