// Device-side building blocks of the zfp block codec for gfx950 (CDNA4).
//
// One 4x4x4 block per lane: the block lives in VGPRs (64 scalars), the
// lifting transform runs on registers, bit planes come from in-register bit
// matrix transposes, and the embedded coder writes each lane's bits into a
// per-lane LDS slot that the wave later packs into the stream.
//
// Bit-exactness notes (reference behaviour being reproduced, x86 + glibc):
//  * block max ignores NaN (`max < |x|`), encodef.c:31-40;
//  * glibc frexp of +inf stores exponent 0 -> emax = 0;
//  * the cast scale 2^(intprec-2-emax) overflows to +inf for subnormal-max
//    blocks (ldexp), and C's float->int conversion yields INT_MIN for NaN and
//    for |y| >= 2^(intprec-1) (x86 cvtt "integer indefinite") -- the GPU
//    conversion saturates instead, so it is wrapped in an explicit select.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "zfp_perm_dev.h"

namespace zfp_amd {

constexpr int kMinExp = -1074;  // zfp.h:21

template <typename S>
struct Traits;

template <>
struct Traits<float> {
  using Int = int32_t;
  using UInt = uint32_t;
  static constexpr int kEbits = 8;
  static constexpr int kPbits = 5;
  static constexpr int kEbias = 127;
  static constexpr int kIntPrec = 32;
  static constexpr UInt kNbMask = 0xaaaaaaaau;
  static constexpr UInt kTcMask = 0x7fffffffu;
};

template <>
struct Traits<double> {
  using Int = int64_t;
  using UInt = uint64_t;
  static constexpr int kEbits = 11;
  static constexpr int kPbits = 6;
  static constexpr int kEbias = 1023;
  static constexpr int kIntPrec = 64;
  static constexpr UInt kNbMask = 0xaaaaaaaaaaaaaaaaull;
  static constexpr UInt kTcMask = 0x7fffffffffffffffull;
};

struct CodecParams {
  uint32_t minbits, maxbits, maxprec;
  int32_t minexp;
};

__device__ __forceinline__ uint64_t low_mask(uint32_t n)
{
  return n >= 64 ? ~0ull : ((1ull << n) - 1);
}

__device__ __forceinline__ uint32_t ctz64(uint64_t x)
{
  return x ? (uint32_t)__builtin_ctzll(x) : 64u;
}

// ---------------------------------------------------------------------------
// Encoder output: a per-lane slot of 64-bit words in LDS, zeroed before the
// block is coded.  Bits are ORed in at their absolute position (LSB first,
// bitstream.inl:289-313 word layout), so no write depends on an earlier one
// and the coder needs no serial accumulator.  Positions past the block's
// budget are garbage by construction: every word index is clamped to a trash
// word (`trash`) that is never read, and readers mask at the block length.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void lds_or(uint64_t* p, uint64_t v)
{
  __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

struct OrSlot {
  uint64_t* w;
  uint32_t trash;

  __device__ __forceinline__ void or_word(uint32_t i, uint64_t v) { lds_or(w + (i < trash ? i : trash), v); }
  // v < 2^len, len <= 64
  __device__ __forceinline__ void put(uint32_t p, uint64_t v, uint32_t len)
  {
    const uint32_t i = p >> 6, sh = p & 63;
    or_word(i, v << sh);
    if (__any(sh + len > 64))
      or_word(i + 1, (v >> 1) >> (63 - sh));
  }
  // (lo | hi << 64) < 2^len, len <= 128.  The spill words are written under
  // wave-uniform tests (a lane with nothing to spill ORs a zero).
  __device__ __forceinline__ void put128(uint32_t p, uint64_t lo, uint64_t hi, uint32_t len)
  {
    const uint32_t i = p >> 6, sh = p & 63;
    or_word(i, lo << sh);
    if (__any(sh + len > 64))
      or_word(i + 1, ((lo >> 1) >> (63 - sh)) | (hi << sh));
    if (__any(sh + len > 128))
      or_word(i + 2, (hi >> 1) >> (63 - sh));
  }
};

// Doubled-ones table: entry b holds the 8 bits of b LSB first with every one
// written twice ("1" -> "11", "0" -> "0"), 8 + popcount(b) bits.  The group
// tests of a bit plane are this expansion of the plane's remaining bits (see
// code_plane), so one table look-up replaces a loop over the ones.
__device__ __forceinline__ uint32_t dbl_entry(uint32_t b)
{
  uint32_t d = 0, p = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    if ((b >> i) & 1u) {
      d |= 3u << p;
      p += 2;
    } else {
      p += 1;
    }
  }
  return d;
}

// expansion of a 16-bit unit: 16 + popcount(u) bits
__device__ __forceinline__ uint32_t dbl16(const uint32_t* lut, uint32_t u)
{
  const uint32_t b0 = u & 0xffu, b1 = (u >> 8) & 0xffu;
  return lut[b0] | (lut[b1] << (8u + (uint32_t)__popc(b0)));
}

// Bit reader over a word array in LDS (or global memory).
struct WordReader {
  const uint64_t* w;
  uint64_t pos;

  __device__ __forceinline__ uint64_t peek64() const
  {
    uint64_t i = pos >> 6;
    uint32_t r = (uint32_t)(pos & 63);
    uint64_t v = w[i] >> r;
    if (r)
      v |= w[i + 1] << (64 - r);
    return v;
  }
  __device__ __forceinline__ uint64_t read(uint32_t n)
  {
    uint64_t v = n ? (peek64() & low_mask(n)) : 0ull;
    pos += n;
    return v;
  }
  __device__ __forceinline__ uint32_t read1()
  {
    uint64_t i = pos >> 6;
    uint32_t r = (uint32_t)(pos & 63);
    pos++;
    return (uint32_t)((w[i] >> r) & 1u);
  }
  __device__ __forceinline__ void skip(uint64_t n) { pos += n; }
};

// ---------------------------------------------------------------------------
// Exponents and casts (encodef.c:11-59, codecf.c:17-32)
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ float block_absmax(const float (&v)[N])
{
  float m = 0.0f;
#pragma unroll
  for (int i = 0; i < N; i++) {
    float a = fabsf(v[i]);
    m = (m < a) ? a : m;  // NaN never wins
  }
  return m;
}

template <int N>
__device__ __forceinline__ double block_absmax(const double (&v)[N])
{
  double m = 0.0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    double a = fabs(v[i]);
    m = (m < a) ? a : m;
  }
  return m;
}

// exponent(): frexp exponent of the max, clamped to 1-EBIAS; 0 -> -EBIAS.
// glibc's frexp stores 0 for +-inf at run time (checked against the reference
// build; a compile-time-folded frexp would leave it untouched instead), so an
// inf-max block gets emax = 0.
__device__ __forceinline__ int block_emax(float m)
{
  uint32_t b = __float_as_uint(m);
  if (b == 0)
    return -127;
  int be = (int)(b >> 23);
  if (be == 255)
    return 0;
  if (be == 0)
    return -126;
  return be - 126;
}

__device__ __forceinline__ int block_emax(double m)
{
  uint64_t b = (uint64_t)__double_as_longlong(m);
  if (b == 0)
    return -1023;
  int be = (int)(b >> 52);
  if (be == 2047)
    return 0;
  if (be == 0)
    return -1022;
  return be - 1022;
}

// exact ldexp(1, e) in the scalar type, with IEEE overflow to +inf and
// gradual underflow (subnormal powers of two) then zero
__device__ __forceinline__ float pow2f(int e)
{
  if (e > 127)
    return __uint_as_float(0x7f800000u);
  if (e >= -126)
    return __uint_as_float((uint32_t)(e + 127) << 23);
  if (e >= -149)
    return __uint_as_float(1u << (e + 149));
  return 0.0f;
}

__device__ __forceinline__ double pow2d(int e)
{
  if (e > 1023)
    return __longlong_as_double(0x7ff0000000000000ll);
  if (e >= -1022)
    return __longlong_as_double((long long)((uint64_t)(e + 1023) << 52));
  if (e >= -1074)
    return __longlong_as_double((long long)(1ull << (e + 1074)));
  return 0.0;
}

// (Int)(s * x) with x86 semantics: NaN / out of range -> INT_MIN
__device__ __forceinline__ int32_t cast_trunc(float y)
{
  return (fabsf(y) < 2147483648.0f) ? (int32_t)y : (int32_t)0x80000000u;
}

__device__ __forceinline__ int64_t cast_trunc(double y)
{
  return (fabs(y) < 9223372036854775808.0) ? (int64_t)y : (int64_t)0x8000000000000000ull;
}

template <int N>
__device__ __forceinline__ void fwd_cast(int32_t (&q)[N], const float (&v)[N], int emax)
{
  float s = pow2f(30 - emax);
#pragma unroll
  for (int i = 0; i < N; i++)
    q[i] = cast_trunc(s * v[i]);
}

template <int N>
__device__ __forceinline__ void fwd_cast(int64_t (&q)[N], const double (&v)[N], int emax)
{
  double s = pow2d(62 - emax);
#pragma unroll
  for (int i = 0; i < N; i++)
    q[i] = cast_trunc(s * v[i]);
}

template <int N>
__device__ __forceinline__ void inv_cast(float (&v)[N], const int32_t (&q)[N], int emax)
{
  float s = pow2f(emax - 30);
#pragma unroll
  for (int i = 0; i < N; i++)
    v[i] = s * (float)q[i];
}

template <int N>
__device__ __forceinline__ void inv_cast(double (&v)[N], const int64_t (&q)[N], int emax)
{
  double s = pow2d(emax - 62);
#pragma unroll
  for (int i = 0; i < N; i++)
    v[i] = s * (double)q[i];
}

__device__ __forceinline__ uint32_t bits_of(float x) { return __float_as_uint(x); }
__device__ __forceinline__ uint64_t bits_of(double x) { return (uint64_t)__double_as_longlong(x); }

// ---------------------------------------------------------------------------
// Lifting (encode.c:31-56, decode.c:9-34, revencode.c:7-30, revdecode.c:7-29)
// Arithmetic is done on the unsigned type to get the reference's wrap-around.
// ---------------------------------------------------------------------------
template <typename Int>
struct Lift {
  using U = typename std::make_unsigned<Int>::type;
  static __device__ __forceinline__ Int add(Int a, Int b) { return (Int)((U)a + (U)b); }
  static __device__ __forceinline__ Int sub(Int a, Int b) { return (Int)((U)a - (U)b); }
  static __device__ __forceinline__ Int shl1(Int a) { return (Int)((U)a << 1); }

  static __device__ __forceinline__ void fwd(Int& x, Int& y, Int& z, Int& w)
  {
    x = add(x, w); x >>= 1; w = sub(w, x);
    z = add(z, y); z >>= 1; y = sub(y, z);
    x = add(x, z); x >>= 1; z = sub(z, x);
    w = add(w, y); w >>= 1; y = sub(y, w);
    w = add(w, y >> 1); y = sub(y, w >> 1);
  }
  static __device__ __forceinline__ void inv(Int& x, Int& y, Int& z, Int& w)
  {
    y = add(y, w >> 1); w = sub(w, y >> 1);
    y = add(y, w); w = shl1(w); w = sub(w, y);
    z = add(z, x); x = shl1(x); x = sub(x, z);
    y = add(y, z); z = shl1(z); z = sub(z, y);
    w = add(w, x); x = shl1(x); x = sub(x, w);
  }
  static __device__ __forceinline__ void rfwd(Int& x, Int& y, Int& z, Int& w)
  {
    w = sub(w, z); z = sub(z, y); y = sub(y, x);
    w = sub(w, z); z = sub(z, y);
    w = sub(w, z);
  }
  static __device__ __forceinline__ void rinv(Int& x, Int& y, Int& z, Int& w)
  {
    w = add(w, z);
    z = add(z, y); w = add(w, z);
    y = add(y, x); z = add(z, y); w = add(w, z);
  }
};

// Separable transform of a 4^D block held in registers; axis order x,y,z(,w)
// forward and reversed for the inverse (encode3.c:35-49, decode3.c:27-42 and
// the 4D twins).  All indices are compile-time after unrolling.
template <int D, bool INV, bool REV, typename Int>
__device__ __forceinline__ void xform(Int (&p)[1 << (2 * D)])
{
  constexpr int N = 1 << (2 * D);
#pragma unroll
  for (int step = 0; step < D; step++) {
    const int axis = INV ? D - 1 - step : step;
    const int s = 1 << (2 * axis);
#pragma unroll
    for (int base = 0; base < N; base++) {
      if ((base >> (2 * axis)) & 3)
        continue;
      Int& x = p[base];
      Int& y = p[base + s];
      Int& z = p[base + 2 * s];
      Int& w = p[base + 3 * s];
      if (REV) {
        if (INV) Lift<Int>::rinv(x, y, z, w);
        else Lift<Int>::rfwd(x, y, z, w);
      } else {
        if (INV) Lift<Int>::inv(x, y, z, w);
        else Lift<Int>::fwd(x, y, z, w);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Bit-matrix transpose of 32x32 bits held in 32 registers: a[r] bit c <-> a[c] bit r.
// Used both ways: coefficients -> bit planes (encode) and back (decode).
// ---------------------------------------------------------------------------
// Byte-granular steps are one v_perm_b32 per output word, the rest one shift
// plus one v_bfi_b32.
template <int J>
__device__ __forceinline__ void transpose_step(uint32_t (&a)[32])
{
  constexpr uint32_t M = (J == 4) ? 0x0f0f0f0fu : (J == 2) ? 0x33333333u : 0x55555555u;
#pragma unroll
  for (int k = 0; k < 32; k++) {
    if (k & J)
      continue;
    const uint32_t x = a[k], y = a[k | J];
    if constexpr (J == 16) {
      a[k] = __builtin_amdgcn_perm(y, x, 0x05040100u);
      a[k | J] = __builtin_amdgcn_perm(y, x, 0x07060302u);
    } else if constexpr (J == 8) {
      a[k] = __builtin_amdgcn_perm(y, x, 0x06020400u);
      a[k | J] = __builtin_amdgcn_perm(y, x, 0x07030501u);
    } else {
      a[k] = (x & M) | ((y << J) & ~M);
      a[k | J] = ((x >> J) & M) | (y & ~M);
    }
  }
}

__device__ __forceinline__ void transpose32(uint32_t (&a)[32])
{
  transpose_step<16>(a);
  transpose_step<8>(a);
  transpose_step<4>(a);
  transpose_step<2>(a);
  transpose_step<1>(a);
}

// ---------------------------------------------------------------------------
// Embedded coder for a 64-coefficient block (encode.c:92-256).  Planes are
// visited MSB first in lock-step across the wave (compile-time plane index,
// so P[k] stays in registers); per-lane state: remaining budget and the
// significance count n.  A plane is: the first n bits verbatim, then group
// tests -- a run "1 0^t 1" per newly significant coefficient (the final
// coefficient's closing 1 implicit), "0" ends the plane.  The budget may cut a
// run anywhere: exactly the reference's bit-by-bit truncation.
// ---------------------------------------------------------------------------
//
// Closed form of one plane.  With n significant coefficients, x = plane >> n
// (the not-yet-significant bits), h its highest one and c its popcount, the
// reference's group tests emit "1", then for every bit of x up to h the bit
// itself plus, after a one, the next group test's "1" -- i.e. "1" followed by
// the doubled-ones expansion of x[0..h] with its final bit dropped -- then a
// "0" test if n + h + 1 < 64 (otherwise the last one is implicit).  Clearing
// the top one (x') makes the expansion garbage-free: "1" + dbl(x') is exact for
// h + c bits and the final "1 0" (or nothing) is added as a tail.  A plane is
// then one OR of (verbatim | group << n) into the slot plus, for lanes whose
// x reaches past bit 15, one OR per further 16-bit unit.  The budget is not
// checked inside a plane: bits beyond it fall past the block end.
//
// The significance count after a plane is known as soon as its top one is,
// so the loop is software-pipelined: plane k-1 is analysed and its table
// look-ups issued before plane k's slot writes, and the look-up latency (LDS
// ops complete in order, so a wait on a read also waits on earlier writes)
// stays off the critical path.
struct PlaneScan {
  uint64_t x, xp;  // remaining bits, and with the top one cleared
  uint32_t h, c;   // top one, popcount
  uint32_t e0, e1; // table entries of xp's low two bytes
  bool nz;
};

__device__ __forceinline__ PlaneScan scan_plane(const uint32_t* lut, uint64_t plane, uint32_t n)
{
  PlaneScan r;
  r.x = n < 64 ? plane >> (n & 63u) : 0ull;
  r.nz = r.x != 0;
  r.h = 63u - (uint32_t)__clzll((long long)(r.x | 1ull));
  r.c = (uint32_t)__popcll(r.x);
  r.xp = r.x & ~(1ull << r.h);
  r.e0 = lut[(uint32_t)r.xp & 0xffu];
  r.e1 = lut[((uint32_t)r.xp >> 8) & 0xffu];
  return r;
}

__device__ __forceinline__ uint32_t next_sig(const PlaneScan& r, uint32_t n)
{
  return r.nz ? ((n + r.h == 63u) ? 64u : n + r.h + 1u) : n;
}

__device__ __forceinline__ void emit_plane(OrSlot& s, const uint32_t* lut, const PlaneScan& r, uint64_t plane,
                                           uint32_t n, uint32_t& pos)
{
  const uint32_t nn = n & 63u;
  const uint64_t verb = plane ^ (r.x << nn);
  const bool impl = r.nz && (n + r.h == 63u);
  const bool normal = r.nz && !impl;
  const uint32_t lr = r.nz ? r.h + r.c : 0u;
  const uint32_t b0 = (uint32_t)r.xp & 0xffu;
  const uint32_t d16 = r.e0 | (r.e1 << (8u + (uint32_t)__popc(b0)));
  uint64_t grp = ((uint64_t)d16 << 1) | (r.nz ? 1ull : 0ull);
  if (normal && lr < 64)
    grp |= 1ull << lr;
  const uint32_t glen = r.nz ? (impl ? lr : lr + 2u) : (n < 64 ? 1u : 0u);
  const uint64_t lo = verb | (grp << nn);
  const uint64_t hi = nn ? (grp >> (64 - nn)) : 0ull;
  s.put128(pos, lo, hi, n + glen);
  if (__any(r.nz && r.h >= 16)) {
    const uint32_t ps = pos + n;
    uint32_t off = 17u + (uint32_t)__popc((uint32_t)r.xp & 0xffffu);
#pragma unroll
    for (int j = 1; j < 4; j++) {
      const uint32_t u = (uint32_t)(r.xp >> (16 * j)) & 0xffffu;
      if (__any(u != 0))
        s.put(ps + off, dbl16(lut, u), 32);  // u == 0 ORs zeros
      off += 16u + (uint32_t)__popc(u);
    }
    if (__any(normal && lr >= 64))
      s.put(ps + lr, (normal && lr >= 64) ? 1ull : 0ull, 1);
  }
  pos += n + glen;
}

// Codes planes PREC-1 .. PREC-maxprec starting at bit `pos` of the slot;
// returns the end position clamped to `lim` (the block's bit budget end).
// The plane index is wave-uniform, so Pl[k]/Ph[k] are register reads with a
// scalar index (no unrolling: one copy of the plane code).
template <int PREC>
__device__ __forceinline__ uint32_t code_planes(OrSlot& s, const uint32_t* lut, uint32_t pos, uint32_t lim,
                                                uint32_t maxprec, const uint32_t (&Pl)[PREC],
                                                const uint32_t (&Ph)[PREC])
{
  const uint32_t kmin = (uint32_t)PREC > maxprec ? (uint32_t)PREC - maxprec : 0u;
  uint32_t n = 0;
  uint64_t plane = ((uint64_t)Ph[PREC - 1] << 32) | Pl[PREC - 1];
  PlaneScan cur = scan_plane(lut, plane, 0);
  for (int k = PREC - 1; k >= 0; k--) {
    const bool act = pos < lim && (uint32_t)k >= kmin;
    if (!__any(act))
      break;
    const uint32_t nnext = next_sig(cur, n);
    const int kn = __builtin_amdgcn_readfirstlane(k > 0 ? k - 1 : 0);
    const uint64_t pnext = ((uint64_t)Ph[kn] << 32) | Pl[kn];
    const PlaneScan nxt = scan_plane(lut, pnext, nnext);
    if (act)
      emit_plane(s, lut, cur, plane, n, pos);
    n = nnext;
    plane = pnext;
    cur = nxt;
  }
  return pos < lim ? pos : lim;
}

// Decoder twin (decode.c:69-246), including the reference quirk that a
// positive group test sets the bit where the scan stopped even when the
// budget ran out first.
//
// Fast path (closed form).  After a "1" group test the section is a sequence
// of tokens, one per coefficient position: "0" (zero), "11" (one, next test
// positive), "10" (one, stop).  Every run of ones starts on a token boundary,
// so the section ends at the first run of ones of ODD length, found without a
// loop by the carry trick: adding 1 at the starts of runs that begin on even
// (odd) bits carries past each run, and the carry lands on an odd (even) bit
// exactly when the run is odd.  The ones of the plane are the first bits of the
// pairs; squeezing those bits (bit p_i + i -> p_i) is one table look-up per
// byte.  Lanes whose section does not end inside the next 63 bits, reaches the
// implicit last coefficient, or is cut by the budget run the reference loop.
constexpr uint64_t kEven = 0x5555555555555555ull;
constexpr uint64_t kOdd = 0xaaaaaaaaaaaaaaaaull;

// squeeze table: entry b has bit (l - r) set for the r-th one of b at bit l
__device__ __forceinline__ uint32_t squeeze_entry(uint32_t b)
{
  uint32_t o = 0, r = 0;
#pragma unroll
  for (int l = 0; l < 8; l++) {
    if ((b >> l) & 1u) {
      o |= 1u << (l - r);
      r++;
    }
  }
  return o;
}

__device__ __forceinline__ void decode_group_slow(WordReader& r, uint64_t& x, uint32_t& bits, uint32_t& n)
{
  while (bits && n < 64) {
    bits--;
    if (!r.read1())
      break;
    uint32_t lim = 63 - n;
    if (lim > bits)
      lim = bits;
    uint32_t z = ctz64(r.peek64());
    if (z < lim) {
      r.skip(z + 1);
      bits -= z + 1;
      n += z;
    } else {
      r.skip(lim);
      bits -= lim;
      n += lim;
    }
    x |= 1ull << n;
    n++;
  }
}

__device__ __forceinline__ uint64_t decode_plane64(WordReader& r, const uint32_t* sq, uint32_t& bits, uint32_t& n)
{
  uint32_t m = n < bits ? n : bits;
  uint64_t x = r.read(m);
  bits -= m;
  bool slow = false;
  if (n < 64 && bits) {
    const uint64_t w = r.peek64();
    if (!(w & 1)) {
      r.skip(1);
      bits--;
    } else {
      const uint64_t S = w >> 1;
      const uint64_t starts = S & ~(S << 1);
      const uint64_t se = S + (starts & kEven), so = S + (starts & kOdd);
      // S holds 63 stream bits; its bit 63 is not data, so a run reaching
      // bit 62 must not be taken as ended there
      const uint64_t ends = (((se & ~S) & kOdd) | ((so & ~S) & kEven)) & ~(1ull << 63);
      const uint32_t q = ctz64(ends);
      const uint64_t mq = low_mask(q);
      const uint32_t ones = (uint32_t)__popcll(S & mq);
      const uint32_t P = q - (ones - 1) / 2;
      if (ends != 0 && n + P <= 63 && q + 2 <= bits) {
        uint64_t F = S & mq & (((S & ~se) & kEven) | ((S & ~so) & kOdd));
        uint64_t xx = 0;
        uint32_t sh = 0;
        while (__any(F != 0)) {
          const uint32_t b = (uint32_t)F & 0xffu;
          xx |= (uint64_t)sq[b] << sh;
          sh += 8u - (uint32_t)__popc(b);
          F >>= 8;
        }
        x |= xx << n;
        n += P;
        r.skip(q + 2);
        bits -= q + 2;
      } else {
        slow = true;
      }
    }
  }
  if (slow)
    decode_group_slow(r, x, bits, n);
  return x;
}

template <int K, int PREC>
struct DecodePlanes {
  static __device__ __forceinline__ void run(WordReader& r, const uint32_t* sq, uint64_t (&P)[PREC], uint32_t kmin,
                                             uint32_t& bits, uint32_t& n)
  {
    bool act = bits != 0 && (uint32_t)K >= kmin;
    if (!__any(act))
      return;
    if (act)
      P[K] = decode_plane64(r, sq, bits, n);
    DecodePlanes<K - 1, PREC>::run(r, sq, P, kmin, bits, n);
  }
};

template <int PREC>
struct DecodePlanes<-1, PREC> {
  static __device__ __forceinline__ void run(WordReader&, const uint32_t*, uint64_t (&)[PREC], uint32_t, uint32_t&,
                                             uint32_t&)
  {
  }
};

template <int PREC>
__device__ __forceinline__ uint32_t decode_planes64(WordReader& r, const uint32_t* sq, uint32_t budget,
                                                    uint32_t maxprec, uint64_t (&P)[PREC])
{
  const uint32_t kmin = (uint32_t)PREC > maxprec ? (uint32_t)PREC - maxprec : 0u;
  uint32_t bits = budget;
  uint32_t n = 0;
#pragma unroll
  for (int k = 0; k < PREC; k++)
    P[k] = 0;
  DecodePlanes<PREC - 1, PREC>::run(r, sq, P, kmin, bits, n);
  return budget - bits;
}

}  // namespace zfp_amd
