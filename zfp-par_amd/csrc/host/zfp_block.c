/*
 * Low-level block API of include/zfp.h (reference declarations zfp.h:911-1061,
 * semantics src/template/encode.c / decode.c `zfp_encode_block_*`,
 * `zfp_encode_block_strided_*`, `zfp_encode_partial_block_strided_*` and the
 * decode twins; the C++ wrappers zfp.hpp:63-95 and the compressed-array caches
 * call them).  Every function is one block through the GPU codec
 * (zfp_block_code in zfp.c): the block is handed over as a field of at most
 * 4 values per axis, so full, strided and partial blocks share the kernels and
 * the padding rule of whole-field compression.  There is no CPU codec.
 *
 * The promote/demote helpers (zfp.c:1398-1476) are plain element conversions
 * of one block between 8/16-bit integers and the 32-bit integers the codec
 * takes.
 */
#include "zfp.h"
#include "zfp_internal.h"

/* contiguous 4^d block: strides 1, 4, 16, 64 */
static const size_t k4[4] = {4, 4, 4, 4};
static const ptrdiff_t kc[4] = {1, 4, 16, 64};

#define ZFP_BLOCK_FNS(T, CT, ZT)                                                                                   \
  size_t zfp_encode_block_##T##_1(zfp_stream* z, const CT* b) { return zfp_block_code(z, ZT, 1, (void*)b, k4, kc, 0); } \
  size_t zfp_encode_block_##T##_2(zfp_stream* z, const CT* b) { return zfp_block_code(z, ZT, 2, (void*)b, k4, kc, 0); } \
  size_t zfp_encode_block_##T##_3(zfp_stream* z, const CT* b) { return zfp_block_code(z, ZT, 3, (void*)b, k4, kc, 0); } \
  size_t zfp_encode_block_##T##_4(zfp_stream* z, const CT* b) { return zfp_block_code(z, ZT, 4, (void*)b, k4, kc, 0); } \
  size_t zfp_decode_block_##T##_1(zfp_stream* z, CT* b) { return zfp_block_code(z, ZT, 1, b, k4, kc, 1); }             \
  size_t zfp_decode_block_##T##_2(zfp_stream* z, CT* b) { return zfp_block_code(z, ZT, 2, b, k4, kc, 1); }             \
  size_t zfp_decode_block_##T##_3(zfp_stream* z, CT* b) { return zfp_block_code(z, ZT, 3, b, k4, kc, 1); }             \
  size_t zfp_decode_block_##T##_4(zfp_stream* z, CT* b) { return zfp_block_code(z, ZT, 4, b, k4, kc, 1); }             \
  size_t zfp_encode_block_strided_##T##_1(zfp_stream* z, const CT* p, ptrdiff_t sx)                                  \
  {                                                                                                                  \
    const ptrdiff_t s[1] = {sx};                                                                                     \
    return zfp_block_code(z, ZT, 1, (void*)p, k4, s, 0);                                                             \
  }                                                                                                                  \
  size_t zfp_encode_block_strided_##T##_2(zfp_stream* z, const CT* p, ptrdiff_t sx, ptrdiff_t sy)                    \
  {                                                                                                                  \
    const ptrdiff_t s[2] = {sx, sy};                                                                                 \
    return zfp_block_code(z, ZT, 2, (void*)p, k4, s, 0);                                                             \
  }                                                                                                                  \
  size_t zfp_encode_block_strided_##T##_3(zfp_stream* z, const CT* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz)      \
  {                                                                                                                  \
    const ptrdiff_t s[3] = {sx, sy, sz};                                                                             \
    return zfp_block_code(z, ZT, 3, (void*)p, k4, s, 0);                                                             \
  }                                                                                                                  \
  size_t zfp_encode_block_strided_##T##_4(zfp_stream* z, const CT* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz,      \
                                          ptrdiff_t sw)                                                              \
  {                                                                                                                  \
    const ptrdiff_t s[4] = {sx, sy, sz, sw};                                                                         \
    return zfp_block_code(z, ZT, 4, (void*)p, k4, s, 0);                                                             \
  }                                                                                                                  \
  size_t zfp_decode_block_strided_##T##_1(zfp_stream* z, CT* p, ptrdiff_t sx)                                        \
  {                                                                                                                  \
    const ptrdiff_t s[1] = {sx};                                                                                     \
    return zfp_block_code(z, ZT, 1, p, k4, s, 1);                                                                    \
  }                                                                                                                  \
  size_t zfp_decode_block_strided_##T##_2(zfp_stream* z, CT* p, ptrdiff_t sx, ptrdiff_t sy)                          \
  {                                                                                                                  \
    const ptrdiff_t s[2] = {sx, sy};                                                                                 \
    return zfp_block_code(z, ZT, 2, p, k4, s, 1);                                                                    \
  }                                                                                                                  \
  size_t zfp_decode_block_strided_##T##_3(zfp_stream* z, CT* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz)            \
  {                                                                                                                  \
    const ptrdiff_t s[3] = {sx, sy, sz};                                                                             \
    return zfp_block_code(z, ZT, 3, p, k4, s, 1);                                                                    \
  }                                                                                                                  \
  size_t zfp_decode_block_strided_##T##_4(zfp_stream* z, CT* p, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz,            \
                                          ptrdiff_t sw)                                                              \
  {                                                                                                                  \
    const ptrdiff_t s[4] = {sx, sy, sz, sw};                                                                         \
    return zfp_block_code(z, ZT, 4, p, k4, s, 1);                                                                    \
  }                                                                                                                  \
  size_t zfp_encode_partial_block_strided_##T##_1(zfp_stream* z, const CT* p, size_t nx, ptrdiff_t sx)               \
  {                                                                                                                  \
    const size_t n[1] = {nx};                                                                                        \
    const ptrdiff_t s[1] = {sx};                                                                                     \
    return zfp_block_code(z, ZT, 1, (void*)p, n, s, 0);                                                              \
  }                                                                                                                  \
  size_t zfp_encode_partial_block_strided_##T##_2(zfp_stream* z, const CT* p, size_t nx, size_t ny, ptrdiff_t sx,    \
                                                  ptrdiff_t sy)                                                      \
  {                                                                                                                  \
    const size_t n[2] = {nx, ny};                                                                                    \
    const ptrdiff_t s[2] = {sx, sy};                                                                                 \
    return zfp_block_code(z, ZT, 2, (void*)p, n, s, 0);                                                              \
  }                                                                                                                  \
  size_t zfp_encode_partial_block_strided_##T##_3(zfp_stream* z, const CT* p, size_t nx, size_t ny, size_t nz,       \
                                                  ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz)                          \
  {                                                                                                                  \
    const size_t n[3] = {nx, ny, nz};                                                                                \
    const ptrdiff_t s[3] = {sx, sy, sz};                                                                             \
    return zfp_block_code(z, ZT, 3, (void*)p, n, s, 0);                                                              \
  }                                                                                                                  \
  size_t zfp_encode_partial_block_strided_##T##_4(zfp_stream* z, const CT* p, size_t nx, size_t ny, size_t nz,       \
                                                  size_t nw, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw) \
  {                                                                                                                  \
    const size_t n[4] = {nx, ny, nz, nw};                                                                            \
    const ptrdiff_t s[4] = {sx, sy, sz, sw};                                                                         \
    return zfp_block_code(z, ZT, 4, (void*)p, n, s, 0);                                                              \
  }                                                                                                                  \
  size_t zfp_decode_partial_block_strided_##T##_1(zfp_stream* z, CT* p, size_t nx, ptrdiff_t sx)                     \
  {                                                                                                                  \
    const size_t n[1] = {nx};                                                                                        \
    const ptrdiff_t s[1] = {sx};                                                                                     \
    return zfp_block_code(z, ZT, 1, p, n, s, 1);                                                                     \
  }                                                                                                                  \
  size_t zfp_decode_partial_block_strided_##T##_2(zfp_stream* z, CT* p, size_t nx, size_t ny, ptrdiff_t sx,          \
                                                  ptrdiff_t sy)                                                      \
  {                                                                                                                  \
    const size_t n[2] = {nx, ny};                                                                                    \
    const ptrdiff_t s[2] = {sx, sy};                                                                                 \
    return zfp_block_code(z, ZT, 2, p, n, s, 1);                                                                     \
  }                                                                                                                  \
  size_t zfp_decode_partial_block_strided_##T##_3(zfp_stream* z, CT* p, size_t nx, size_t ny, size_t nz,             \
                                                  ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz)                          \
  {                                                                                                                  \
    const size_t n[3] = {nx, ny, nz};                                                                                \
    const ptrdiff_t s[3] = {sx, sy, sz};                                                                             \
    return zfp_block_code(z, ZT, 3, p, n, s, 1);                                                                     \
  }                                                                                                                  \
  size_t zfp_decode_partial_block_strided_##T##_4(zfp_stream* z, CT* p, size_t nx, size_t ny, size_t nz, size_t nw,  \
                                                  ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw)            \
  {                                                                                                                  \
    const size_t n[4] = {nx, ny, nz, nw};                                                                            \
    const ptrdiff_t s[4] = {sx, sy, sz, sw};                                                                         \
    return zfp_block_code(z, ZT, 4, p, n, s, 1);                                                                     \
  }

ZFP_BLOCK_FNS(int32, int32, zfp_type_int32)
ZFP_BLOCK_FNS(int64, int64, zfp_type_int64)
ZFP_BLOCK_FNS(float, float, zfp_type_float)
ZFP_BLOCK_FNS(double, double, zfp_type_double)

/* ------------------------------------------------------------------------ */
/* promote / demote (zfp.c:1398-1476): values scaled to the top of an int32 */

static uint block_count(uint dims) { return 1u << (2 * dims); }

static int32 clamp32(int32 x, int32 lo, int32 hi) { return x < lo ? lo : x > hi ? hi : x; }

void zfp_promote_int8_to_int32(int32* oblock, const int8* iblock, uint dims)
{
  for (uint i = 0, n = block_count(dims); i < n; i++)
    oblock[i] = (int32)((uint32)(int32)iblock[i] << 23);
}

void zfp_promote_uint8_to_int32(int32* oblock, const uint8* iblock, uint dims)
{
  for (uint i = 0, n = block_count(dims); i < n; i++)
    oblock[i] = (int32)((uint32)((int32)iblock[i] - 0x80) << 23);
}

void zfp_promote_int16_to_int32(int32* oblock, const int16* iblock, uint dims)
{
  for (uint i = 0, n = block_count(dims); i < n; i++)
    oblock[i] = (int32)((uint32)(int32)iblock[i] << 15);
}

void zfp_promote_uint16_to_int32(int32* oblock, const uint16* iblock, uint dims)
{
  for (uint i = 0, n = block_count(dims); i < n; i++)
    oblock[i] = (int32)((uint32)((int32)iblock[i] - 0x8000) << 15);
}

void zfp_demote_int32_to_int8(int8* oblock, const int32* iblock, uint dims)
{
  for (uint i = 0, n = block_count(dims); i < n; i++)
    oblock[i] = (int8)clamp32(iblock[i] >> 23, -0x80, 0x7f);
}

void zfp_demote_int32_to_uint8(uint8* oblock, const int32* iblock, uint dims)
{
  for (uint i = 0, n = block_count(dims); i < n; i++)
    oblock[i] = (uint8)clamp32((iblock[i] >> 23) + 0x80, 0x00, 0xff);
}

void zfp_demote_int32_to_int16(int16* oblock, const int32* iblock, uint dims)
{
  for (uint i = 0, n = block_count(dims); i < n; i++)
    oblock[i] = (int16)clamp32(iblock[i] >> 15, -0x8000, 0x7fff);
}

void zfp_demote_int32_to_uint16(uint16* oblock, const int32* iblock, uint dims)
{
  for (uint i = 0, n = block_count(dims); i < n; i++)
    oblock[i] = (uint16)clamp32((iblock[i] >> 15) + 0x8000, 0x0000, 0xffff);
}
