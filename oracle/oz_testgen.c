/*
 * TEST INFRASTRUCTURE ONLY -- NOT PART OF THE PRODUCT.
 *
 * Restatement of the reference test suite's deterministic input generator and
 * checksums, so the golden checksum tables of tests/constants/checksums/{3d,4d}{Float,Double}.h
 * can be used as oracle pins:
 *   - smooth random fields:  tests/utils/genSmoothRandNums.c:1-918
 *     (repeated 2x refinement of a +-amplitude seed tensor with fixed-point
 *      stencil weights plus noise, then ldexp(., -12) for float / -26 double)
 *   - 96-bit fixed point:     tests/utils/fixedpoint96.c (Q64.32; multiply
 *                             truncates toward -inf, round adds 1/2 up)
 *   - LCG:                    tests/utils/rand64.c:4-52 (seed 5)
 *   - Jenkins one-at-a-time:  tests/utils/zfpHash.c:1-126
 * The Q64.32 arithmetic is done exactly with 128-bit integers.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef __int128 q96; /* value * 2^32 */

static uint64_t lcg_state;

static void lcg_reset(void) { lcg_state = 5; }

static uint32_t lcg_next32(void)
{
  lcg_state = 2862933555777941757ull * lcg_state + 3037000493ull;
  return (uint32_t)((lcg_state & 0x7fffffffffffffffull) >> 31);
}

static q96 q_from_int(int64_t i) { return (q96)i * ((q96)1 << 32); }
static q96 q_frac(uint32_t f) { return (q96)f; }
/* floor((a*b) / 2^32): fixedpoint96.c multiply() drops the low 32 bits */
static q96 q_mul(q96 a, q96 b) { return (a * b) >> 32; }
/* roundFixedPt: integer part + (fraction >= 1/2) */
static int64_t q_round(q96 a)
{
  int64_t ip = (int64_t)(a >> 32);
  uint32_t fp = (uint32_t)(a & 0xffffffff);
  return ip + (fp >= 0x80000000u ? 1 : 0);
}

/* generateWeights: four stencil weights from the noise factor f */
static void gen_weights(q96 f, q96 w[4])
{
  q96 half = q_frac(0x80000000u), one = q_from_int(1), nine = q_from_int(9);
  q96 sixteenth = q_frac(0x10000000u);
  w[0] = q_mul(q_mul(q_frac(lcg_next32()) - half, f) - one, sixteenth);
  w[1] = q_mul(q_mul(q_frac(lcg_next32()) - half, f) + nine, sixteenth);
  w[2] = q_mul(q_mul(q_frac(lcg_next32()) - half, f) + nine, sixteenth);
  w[3] = one - w[0] - w[1] - w[2];
}

static int64_t knock_back(int64_t v, int64_t amp)
{
  if (v > amp) v -= 2 * (v - amp);
  else if (v < -amp) v += 2 * (-amp - v);
  return v;
}

static size_t ipow(size_t b, int e) { size_t r = 1; while (e--) r *= b; return r; }

/* weighted sum over a 4^k stencil along `k` axes with strides st[]; weights
 * are the tensor product of one fresh 4-vector (computeTensorProductDouble:
 * products taken in i, j, k, l order, each truncated) */
static int64_t stencil(const int64_t* a, int k, const size_t st[4], q96 f, int64_t amp)
{
  q96 w4[4], acc = 0;
  gen_weights(f, w4);
  size_t total = ipow(4, k);
  for (size_t idx = 0; idx < total; idx++) {
    size_t c[4] = {idx & 3, (idx >> 2) & 3, (idx >> 4) & 3, (idx >> 6) & 3};
    q96 wt = w4[c[0]];
    for (int d = 1; d < k; d++)
      wt = q_mul(wt, w4[c[d]]);
    size_t off = 0;
    for (int d = 0; d < k; d++)
      off += c[d] * st[d];
    acc += q_mul(q_from_int(a[off]), wt);
  }
  return knock_back(q_round(acc), amp);
}

/* produceLargerNoisedArray: side n -> 2n-1 */
static void refine(const int64_t* in, size_t n, int dims, int64_t amp, q96 f, int64_t* out)
{
  size_t pn = n + 2, on = 2 * n - 1;
  size_t ptot = ipow(pn, dims);
  int64_t* pad = (int64_t*)calloc(ptot, sizeof(int64_t));
  size_t pst[4] = {1, pn, pn * pn, pn * pn * pn};
  size_t ist[4] = {1, n, n * n, n * n * n};
  size_t ost[4] = {1, on, on * on, on * on * on};
  size_t itot = ipow(n, dims);
  for (size_t i = 0; i < itot; i++) {
    size_t r = i, off = 0;
    for (int d = 0; d < dims; d++) { off += (r % n + 1) * pst[d]; r /= n; }
    pad[off] = in[i];
  }
  size_t lim[4] = {1, 1, 1, 1};
  for (int d = 0; d < dims; d++) lim[d] = on;
  for (size_t ol = 0; ol < lim[3]; ol++)
    for (size_t ok = 0; ok < lim[2]; ok++)
      for (size_t oj = 0; oj < lim[1]; oj++)
        for (size_t oi = 0; oi < lim[0]; oi++) {
          size_t o[4] = {oi, oj, ok, ol};
          int odd[4] = {0, 0, 0, 0}, k = 0;
          size_t sst[4];
          size_t base = 0;
          for (int d = 0; d < dims; d++) {
            odd[d] = (int)(o[d] & 1);
            /* odd coordinate: stencil starts one cell before (padded index
             * in = o/2); even coordinate: the cell itself (padded in+1) */
            base += (o[d] / 2 + (odd[d] ? 0 : 1)) * pst[d];
          }
          int64_t v;
          for (int d = 0; d < dims; d++)
            if (odd[d]) sst[k++] = pst[d];
          if (!k) {
            size_t off = 0;
            for (int d = 0; d < dims; d++) off += (o[d] / 2) * ist[d];
            v = in[off];
          } else {
            v = stencil(pad + base, k, sst, f, amp);
          }
          size_t ooff = 0;
          for (int d = 0; d < dims; d++) ooff += o[d] * ost[d];
          out[ooff] = v;
        }
  free(pad);
}

/* generateSmoothRandInts64: returns malloc'ed array, side length in *side */
int64_t* oz_gen_smooth_ints(size_t min_total, int dims, int amp_exp, size_t* side)
{
  int64_t amp = (int64_t)(((uint64_t)1 << amp_exp) - 1);
  static const int64_t seed[5] = {0, 1, 0, -1, 0};
  size_t n = 5;
  size_t tot = ipow(n, dims);
  int64_t* cur = (int64_t*)malloc(tot * sizeof(int64_t));
  for (size_t i = 0; i < tot; i++) {
    size_t r = i;
    int64_t prod = 1;
    for (int d = 0; d < dims; d++) { prod *= seed[r % 5]; r /= 5; }
    cur[i] = prod > 0 ? amp : prod < 0 ? -amp : 0;
  }
  lcg_reset();
  q96 f = q_from_int(7);
  q96 shrink = q_frac(0xaaaaaaaau);
  while (tot < min_total) {
    size_t nn = 2 * n - 1;
    size_t nt = ipow(nn, dims);
    int64_t* nxt = (int64_t*)malloc(nt * sizeof(int64_t));
    refine(cur, n, dims, amp, f, nxt);
    free(cur);
    cur = nxt; n = nn; tot = nt;
    f = q_mul(f, shrink);
  }
  for (size_t i = 0; i < tot; i++) {
    if (cur[i] < -amp) cur[i] = -amp;
    else if (cur[i] > amp) cur[i] = amp;
  }
  *side = n;
  return cur;
}

/* generateSmoothRandFloats / Doubles into caller buffers sized side^dims */
size_t oz_gen_smooth_floats(size_t min_total, int dims, float* out, size_t cap)
{
  size_t side;
  int64_t* v = oz_gen_smooth_ints(min_total, dims, 23, &side);
  size_t tot = ipow(side, dims);
  if (out && tot <= cap)
    for (size_t i = 0; i < tot; i++) out[i] = ldexpf((float)v[i], -12);
  free(v);
  return side;
}

size_t oz_gen_smooth_doubles(size_t min_total, int dims, double* out, size_t cap)
{
  size_t side;
  int64_t* v = oz_gen_smooth_ints(min_total, dims, 52, &side);
  size_t tot = ipow(side, dims);
  if (out && tot <= cap)
    for (size_t i = 0; i < tot; i++) out[i] = ldexp((double)v[i], -26);
  free(v);
  return side;
}

/* ---- Jenkins one-at-a-time hashes, zfpHash.c ---- */
static void jh_step(uint32_t v, uint32_t* h) { *h += v; *h += *h << 10; *h ^= *h >> 6; }
static uint32_t jh_finish(uint32_t h) { h += h << 3; h ^= h >> 11; h += h << 15; return h; }

/* hashBitstream: two interleaved 32-bit hashes over 64-bit words */
uint64_t oz_hash_words(const uint64_t* w, size_t nwords)
{
  uint32_t h1 = 0, h2 = 0;
  for (size_t i = 0; i < nwords; i++) {
    jh_step((uint32_t)w[i], &h1);
    jh_step((uint32_t)(w[i] >> 32), &h2);
  }
  return (uint64_t)jh_finish(h1) + ((uint64_t)jh_finish(h2) << 32);
}

/* hashArray32 with unit stride */
uint32_t oz_hash_array32(const uint32_t* a, size_t n)
{
  uint32_t h = 0;
  for (size_t i = 0; i < n; i++) jh_step(a[i], &h);
  return jh_finish(h);
}

/* hashArray64 with unit stride (same as the word hash) */
uint64_t oz_hash_array64(const uint64_t* a, size_t n) { return oz_hash_words(a, n); }

/* generateSmoothRandInts32 / Ints64 as the reference's end-to-end tests call
 * them (tests/src/endtoend/zfpEndtoendBase.c:78-84: amplitude exponent
 * intprec - 2; genSmoothRandNums.c:885-893 cast64ArrayTo32) */
size_t oz_gen_smooth_int32(size_t min_total, int dims, int32_t* out, size_t cap)
{
  size_t side;
  int64_t* v = oz_gen_smooth_ints(min_total, dims, 32 - 2, &side);
  size_t tot = ipow(side, dims);
  if (out && tot <= cap)
    for (size_t i = 0; i < tot; i++) out[i] = (int32_t)v[i];
  free(v);
  return side;
}

size_t oz_gen_smooth_int64(size_t min_total, int dims, int64_t* out, size_t cap)
{
  size_t side;
  int64_t* v = oz_gen_smooth_ints(min_total, dims, 64 - 2, &side);
  size_t tot = ipow(side, dims);
  if (out && tot <= cap)
    for (size_t i = 0; i < tot; i++) out[i] = v[i];
  free(v);
  return side;
}
