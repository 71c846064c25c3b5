/*
 * Bit stream I/O for the zfp host library (semantics of the reference's
 * include/zfp/bitstream.inl:133-460; word size fixed at 64 bits, no strided
 * streams).  Bits are appended least significant first into 64-bit words; a
 * partially filled word is held in `buffer` until it fills or the stream is
 * flushed (zero padding).  Reading mirrors that with `buffer` holding the
 * unread high bits of the last fetched word.
 *
 * MI355X addition: a stream may live in HIP device memory (stream_open
 * detects it).  The codec writes such streams on the device; the few words the
 * host touches itself (headers, seeks) are moved with hipMemcpy, so
 * zfp_write_header / zfp_read_header work on device-resident streams too.
 */
#include <stdlib.h>

#include "zfp/bitstream.h"
#include "zfp_hip.h"
#include "zfp_internal.h"

const size_t stream_word_bits = 64;

static uint64 peek_word(const bitstream* s)
{
  uint64 w = 0;
  if (!s->device)
    return *s->ptr;
  (void)zfp_hip_memcpy(&w, s->ptr, sizeof w);
  return w;
}

static uint64 load_word(bitstream* s)
{
  uint64 w = peek_word(s);
  s->ptr++;
  return w;
}

static void store_word(bitstream* s, uint64 w)
{
  if (s->device)
    (void)zfp_hip_memcpy(s->ptr, &w, sizeof w);
  else
    *s->ptr = w;
  s->ptr++;
}

bitstream* stream_open(void* buffer, size_t bytes)
{
  bitstream* s = (bitstream*)malloc(sizeof(bitstream));
  if (s) {
    s->begin = (uint64*)buffer;
    s->end = s->begin + bytes / sizeof(uint64);
    s->device = zfp_hip_is_device_ptr(buffer);
    stream_rewind(s);
  }
  return s;
}

void stream_close(bitstream* s) { free(s); }

bitstream* stream_clone(const bitstream* s)
{
  bitstream* c = (bitstream*)malloc(sizeof(bitstream));
  if (c)
    *c = *s;
  return c;
}

bitstream_count stream_alignment(void) { return 64; }
void* stream_data(const bitstream* s) { return s->begin; }
size_t stream_size(const bitstream* s) { return (size_t)(s->ptr - s->begin) * sizeof(uint64); }
size_t stream_capacity(const bitstream* s) { return (size_t)(s->end - s->begin) * sizeof(uint64); }
size_t stream_stride_block(const bitstream* s) { (void)s; return 1; }
ptrdiff_t stream_stride_delta(const bitstream* s) { (void)s; return 0; }

uint stream_read_bit(bitstream* s)
{
  if (!s->bits) {
    s->buffer = load_word(s);
    s->bits = 64;
  }
  s->bits--;
  uint bit = (uint)(s->buffer & 1u);
  s->buffer >>= 1;
  return bit;
}

uint stream_write_bit(bitstream* s, uint bit)
{
  s->buffer += (uint64)bit << s->bits;
  if (++s->bits == 64) {
    store_word(s, s->buffer);
    s->buffer = 0;
    s->bits = 0;
  }
  return bit;
}

uint64 stream_read_bits(bitstream* s, bitstream_count n)
{
  uint64 value = s->buffer;
  if (s->bits < n) {
    /* need the next word: its low bits complete the value */
    uint64 w = load_word(s);
    value += w << s->bits; /* s->bits < n <= 64, and s->bits < 64 */
    size_t left = s->bits + 64 - n; /* bits of w not consumed, in [0, 63] */
    if (left) {
      s->buffer = w >> (64 - left);
      value &= ((uint64)2 << (n - 1)) - 1;
    } else {
      s->buffer = 0;
    }
    s->bits = left;
  } else {
    s->bits -= n;
    if (n < 64) {
      s->buffer >>= n;
      value &= ((uint64)1 << n) - 1;
    } else {
      s->buffer = 0;
    }
  }
  return value;
}

uint64 stream_write_bits(bitstream* s, uint64 value, bitstream_count n)
{
  if (n == 0)
    return value;
  s->buffer += value << s->bits;
  size_t total = s->bits + n;
  if (total >= 64) {
    store_word(s, s->buffer);
    total -= 64;
    /* the top `total` bits of the n-bit value did not fit */
    s->buffer = s->bits ? (value >> (64 - s->bits)) : 0;
  }
  s->bits = total;
  if (total < 64)
    s->buffer &= ((uint64)1 << total) - 1;
  return n >= 64 ? 0 : value >> n;
}

bitstream_offset stream_rtell(const bitstream* s) { return (bitstream_offset)(s->ptr - s->begin) * 64 - s->bits; }
bitstream_offset stream_wtell(const bitstream* s) { return (bitstream_offset)(s->ptr - s->begin) * 64 + s->bits; }

void stream_rewind(bitstream* s)
{
  s->ptr = s->begin;
  s->buffer = 0;
  s->bits = 0;
}

void stream_rseek(bitstream* s, bitstream_offset offset)
{
  size_t r = (size_t)(offset % 64);
  s->ptr = s->begin + (size_t)(offset / 64);
  if (r) {
    s->buffer = load_word(s) >> r;
    s->bits = 64 - r;
  } else {
    s->buffer = 0;
    s->bits = 0;
  }
}

void stream_wseek(bitstream* s, bitstream_offset offset)
{
  size_t r = (size_t)(offset % 64);
  s->ptr = s->begin + (size_t)(offset / 64);
  if (r) {
    s->buffer = peek_word(s) & (((uint64)1 << r) - 1);
    s->bits = r;
  } else {
    s->buffer = 0;
    s->bits = 0;
  }
}

void stream_skip(bitstream* s, bitstream_size n) { stream_rseek(s, stream_rtell(s) + n); }

void stream_pad(bitstream* s, bitstream_size n)
{
  bitstream_offset bits = s->bits + n;
  while (bits >= 64) {
    store_word(s, s->buffer);
    s->buffer = 0;
    bits -= 64;
  }
  s->bits = (size_t)bits;
}

bitstream_count stream_align(bitstream* s)
{
  bitstream_count bits = s->bits;
  if (bits)
    stream_skip(s, bits);
  return bits;
}

bitstream_count stream_flush(bitstream* s)
{
  bitstream_count bits = (64 - s->bits) % 64;
  if (bits)
    stream_pad(s, bits);
  return bits;
}

void stream_copy(bitstream* dst, bitstream* src, bitstream_size n)
{
  while (n > 64) {
    stream_write_bits(dst, stream_read_bits(src, 64), 64);
    n -= 64;
  }
  if (n)
    stream_write_bits(dst, stream_read_bits(src, (bitstream_count)n), (bitstream_count)n);
}
