/*
 * zfp bit stream API -- MI355X framework (drop-in for SEP-software/zfp-par).
 *
 * Same entry points and semantics as the reference's include/zfp/bitstream.h
 * (declarations :28-94, behaviour include/zfp/bitstream.inl:133-460): 64-bit
 * little-endian words, bits written and read least-significant first,
 * stream_flush zero-pads to a word, stream_size counts whole words.
 * The host owns the buffer (stream_open only wraps it).  The buffer may be
 * host or device memory: the codec entry points (zfp_compress/zfp_decompress)
 * accept both; the bit-level functions below touch memory on the host and
 * therefore need host-accessible buffers.
 */
#ifndef ZFP_BITSTREAM_H
#define ZFP_BITSTREAM_H

#include <stddef.h>
#include <stdint.h>

#include "zfp/types.h"

typedef struct bitstream bitstream;  /* opaque */
typedef uint64 bitstream_offset;     /* bit offset into a stream */
typedef bitstream_offset bitstream_size;
typedef size_t bitstream_count;

#ifdef __cplusplus
extern "C" {
#endif

extern const size_t stream_word_bits; /* = 64 */

bitstream* stream_open(void* buffer, size_t bytes);
void stream_close(bitstream* stream);
bitstream* stream_clone(const bitstream* stream);
bitstream_count stream_alignment(void);
void* stream_data(const bitstream* stream);
size_t stream_size(const bitstream* stream);
size_t stream_capacity(const bitstream* stream);
size_t stream_stride_block(const bitstream* stream);
ptrdiff_t stream_stride_delta(const bitstream* stream);
uint stream_read_bit(bitstream* stream);
uint stream_write_bit(bitstream* stream, uint bit);
uint64 stream_read_bits(bitstream* stream, bitstream_count n);
uint64 stream_write_bits(bitstream* stream, uint64 value, bitstream_count n);
bitstream_offset stream_rtell(const bitstream* stream);
bitstream_offset stream_wtell(const bitstream* stream);
void stream_rewind(bitstream* stream);
void stream_rseek(bitstream* stream, bitstream_offset offset);
void stream_wseek(bitstream* stream, bitstream_offset offset);
void stream_skip(bitstream* stream, bitstream_size n);
void stream_pad(bitstream* stream, bitstream_size n);
bitstream_count stream_align(bitstream* stream);
bitstream_count stream_flush(bitstream* stream);
void stream_copy(bitstream* dst, bitstream* src, bitstream_size n);

#ifdef __cplusplus
}
#endif

#endif
