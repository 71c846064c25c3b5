/*
 * TEST INFRASTRUCTURE ONLY -- NOT PART OF THE PRODUCT.
 *
 * CPU oracle for the zfp block codec of SEP-software/zfp-par (zfp 1.0.1, codec
 * version 5, default build: 64-bit stream words, ZFP_ROUND_NEVER, no tight
 * error, no DAZ).  It restates the serial codec from the reference sources and
 * exists only to check the HIP product path.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product library never links it.
 *
 * Parity pin: tests/test_oracle.py checks this oracle against (a) the golden
 * checksum tables of the reference's own tests (tests/constants/checksums/{3d,4d}{Float,Double}.h,
 * reproduced in tests/golden/checksums.json) and (b) the reference itself,
 * compiled from its sources into oracle/_ref/ by oracle/Makefile, on seeded
 * random fields.
 *
 * Scope: 1-4D float/double, every mode (fixed rate / precision / accuracy /
 * reversible / expert), chunk boxes, arbitrary strides, partial blocks.
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "oz_perm.h"

#define OZ_MIN_EXP (-1074) /* zfp.h:21 */

/* compression parameters: zfp_stream fields, zfp.h:90-97 */
typedef struct {
  uint32_t minbits, maxbits, maxprec;
  int32_t minexp;
} oz_params;

/* one (de)compression job: field descriptor (zfp.h:135-140) + chunk box
 * (zfp.h:146-149, e[] is an exclusive end index) + parameters */
typedef struct {
  int32_t type; /* zfp_type numbering: 3 float, 4 double */
  int32_t pad_;
  oz_params p;
  uint64_t n[4];
  int64_t s[4];
  uint64_t f[4];
  uint64_t e[4];
} oz_job;

/* ---- bit stream: 64-bit little-endian words, bits appended LSB first
 *      (bitstream.inl:241-313); writer ORs into a zero-filled buffer ---- */
typedef struct {
  uint64_t* w;
  uint64_t pos;
} oz_bits;

static void oz_put(oz_bits* s, uint64_t v, uint32_t n)
{
  if (!n)
    return;
  if (n < 64)
    v &= ((uint64_t)1 << n) - 1;
  uint64_t i = s->pos >> 6;
  uint32_t r = (uint32_t)(s->pos & 63);
  s->w[i] |= v << r;
  if (r && r + n > 64)
    s->w[i + 1] |= v >> (64 - r);
  s->pos += n;
}

static uint64_t oz_get(oz_bits* s, uint32_t n)
{
  if (!n)
    return 0;
  uint64_t i = s->pos >> 6;
  uint32_t r = (uint32_t)(s->pos & 63);
  uint64_t v = s->w[i] >> r;
  if (r && r + n > 64)
    v |= s->w[i + 1] << (64 - r);
  if (n < 64)
    v &= ((uint64_t)1 << n) - 1;
  s->pos += n;
  return v;
}

static void oz_pad(oz_bits* s, uint64_t n) { s->pos += n; }
static void oz_skip(oz_bits* s, uint64_t n) { s->pos += n; }

static const unsigned char* oz_perm_table(uint32_t dims)
{
  switch (dims) {
    case 1: return oz_perm1;
    case 2: return oz_perm2;
    case 3: return oz_perm3;
    default: return oz_perm4;
  }
}

/* zfp_field_dimensionality: zfp.c:291-294 */
static uint32_t oz_dims(const oz_job* j)
{
  return j->n[0] ? j->n[1] ? j->n[2] ? j->n[3] ? 4 : 3 : 2 : 1 : 0;
}

/* default strides for zero entries: zfp.c:332-334, :370-373 */
static void oz_strides(const oz_job* j, ptrdiff_t st[4])
{
  st[0] = j->s[0] ? (ptrdiff_t)j->s[0] : 1;
  st[1] = j->s[1] ? (ptrdiff_t)j->s[1] : (ptrdiff_t)j->n[0];
  st[2] = j->s[2] ? (ptrdiff_t)j->s[2] : (ptrdiff_t)(j->n[0] * j->n[1]);
  st[3] = j->s[3] ? (ptrdiff_t)j->s[3] : (ptrdiff_t)(j->n[0] * j->n[1] * j->n[2]);
}

/* single precision instance (traitsf.h: EBITS 8, PBITS 5) */
#define OZ_SFX f
#define OZ_REAL float
#define OZ_INT int32_t
#define OZ_UINT uint32_t
#define OZ_EBITS 8
#define OZ_PBITS 5
#define OZ_NBMASK 0xaaaaaaaau
#define OZ_TCMASK 0x7fffffffu
#define OZ_FREXP frexpf
#define OZ_LDEXP ldexpf
#define OZ_FABS fabsf
#include "oz_codec_body.h"
#undef OZ_SFX
#undef OZ_REAL
#undef OZ_INT
#undef OZ_UINT
#undef OZ_EBITS
#undef OZ_PBITS
#undef OZ_NBMASK
#undef OZ_TCMASK
#undef OZ_FREXP
#undef OZ_LDEXP
#undef OZ_FABS

/* double precision instance (traitsd.h: EBITS 11, PBITS 6) */
#define OZ_SFX d
#define OZ_REAL double
#define OZ_INT int64_t
#define OZ_UINT uint64_t
#define OZ_EBITS 11
#define OZ_PBITS 6
#define OZ_NBMASK 0xaaaaaaaaaaaaaaaaull
#define OZ_TCMASK 0x7fffffffffffffffull
#define OZ_FREXP frexp
#define OZ_LDEXP ldexp
#define OZ_FABS fabs
#include "oz_codec_body.h"

/* ---- exported entry points (ctypes) ---- */

/* Encode the chunk box of j into `words` starting at bit `bitpos`.  The
 * caller zero-fills `words`.  Returns the end bit position (not flushed). */
uint64_t oz_compress(const oz_job* j, const void* data, uint64_t* words, uint64_t bitpos)
{
  oz_bits s = {words, bitpos};
  if (!oz_dims(j))
    return bitpos;
  if (j->type == 3)
    return oz_run_f(j, (void*)data, &s, 0);
  if (j->type == 4)
    return oz_run_d(j, (void*)data, &s, 0);
  return bitpos;
}

/* Decode the chunk box of j from `words` starting at bit `bitpos`; returns
 * the end bit position. */
uint64_t oz_decompress(const oz_job* j, void* data, const uint64_t* words, uint64_t bitpos)
{
  oz_bits s = {(uint64_t*)words, bitpos};
  if (!oz_dims(j))
    return bitpos;
  if (j->type == 3)
    return oz_run_f(j, data, &s, 1);
  if (j->type == 4)
    return oz_run_d(j, data, &s, 1);
  return bitpos;
}

/* Per-block bit lengths of a whole-box encode (variable-rate index check). */
uint64_t oz_block_bits(const oz_job* j, const void* data, uint64_t* scratch, uint32_t* lens, uint64_t maxblocks)
{
  uint32_t dims = oz_dims(j);
  ptrdiff_t st[4];
  size_t bcount[4] = {1, 1, 1, 1};
  uint64_t nb = 0;
  oz_strides(j, st);
  for (uint32_t a = 0; a < dims; a++)
    bcount[a] = (j->e[a] > j->f[a]) ? (j->e[a] - j->f[a] + 3) / 4 : 0;
  for (size_t bw = 0; bw < bcount[3]; bw++)
    for (size_t bz = 0; bz < bcount[2]; bz++)
      for (size_t by = 0; by < bcount[1]; by++)
        for (size_t bx = 0; bx < bcount[0] && nb < maxblocks; bx++) {
          size_t b[4] = {bx, by, bz, bw};
          size_t cnt[4] = {4, 4, 4, 4};
          ptrdiff_t off = 0;
          for (uint32_t a = 0; a < dims; a++) {
            size_t x = j->f[a] + 4 * b[a];
            size_t left = j->n[a] - x;
            cnt[a] = left < 4 ? left : 4;
            off += (ptrdiff_t)x * st[a];
          }
          oz_bits s = {scratch, 0};
          memset(scratch, 0, 600 * sizeof(uint64_t));
          if (j->type == 3) {
            float blk[256];
            oz_gather_f(blk, (const float*)data + off, dims, cnt, st);
            lens[nb++] = oz_encode_block_f(&s, &j->p, dims, blk);
          } else {
            double blk[256];
            oz_gather_d(blk, (const double*)data + off, dims, cnt, st);
            lens[nb++] = oz_encode_block_d(&s, &j->p, dims, blk);
          }
        }
  return nb;
}
