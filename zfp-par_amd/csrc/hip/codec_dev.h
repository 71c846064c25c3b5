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

// integer fields (encodei.c / decodei.c, traitsi.h, traitsl.h): no exponent
template <>
struct Traits<int32_t> {
  using Int = int32_t;
  using UInt = uint32_t;
  static constexpr int kEbits = 0;
  static constexpr int kPbits = 5;
  static constexpr int kEbias = 0;
  static constexpr int kIntPrec = 32;
  static constexpr UInt kNbMask = 0xaaaaaaaau;
  static constexpr UInt kTcMask = 0;
};

template <>
struct Traits<int64_t> {
  using Int = int64_t;
  using UInt = uint64_t;
  static constexpr int kEbits = 0;
  static constexpr int kPbits = 6;
  static constexpr int kEbias = 0;
  static constexpr int kIntPrec = 64;
  static constexpr UInt kNbMask = 0xaaaaaaaaaaaaaaaaull;
  static constexpr UInt kTcMask = 0;
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
// and the coder needs no serial accumulator.  Bits past the block's budget
// land in spare words at the slot's end (sized by slot_words_for) that are
// never read; readers mask at the block length.
// ---------------------------------------------------------------------------
#define ZFP_LDS_OR(p, v) (void)__hip_atomic_fetch_or((p), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT)
__device__ __forceinline__ void lds_or32(uint32_t* p, uint32_t v)
{
  ZFP_LDS_OR(p, v);
}

// Writes are dword-granular funnel shifts (v_alignbit_b32: one full-rate op per
// output dword; a 64-bit shift costs about three).  A value placed at bit p
// (p >= 1) starts in dword j-1 with j = ceil(p / 32), at offset s = p - 32(j-1)
// in [1, 32]; dword j-1+i receives ((v << s) >> 32 i), which is
// alignbit(v_i, v_{i-1}, -p) since alignbit shifts by its operand mod 32.
struct OrSlot {
  uint64_t* w;    // slot base (bit 0 = bit 0 of w[0])
  uint32_t jmax;  // last dword index of the slot (clamp target of put*_clamped)

  __device__ __forceinline__ uint32_t* d() const { return reinterpret_cast<uint32_t*>(w); }
  // block header bits at bit 0 (v < 2^32)
  __device__ __forceinline__ void head(uint32_t v) { lds_or32(d(), v); }
  // v1:v0 at bit p >= 1: dwords j-1 .. j+1
  __device__ __forceinline__ void put64(uint32_t p, uint32_t v0, uint32_t v1)
  {
    uint32_t* q = d() + ((p + 31u) >> 5) - 1;
    const uint32_t t = 0u - p;
    lds_or32(q, __builtin_amdgcn_alignbit(v0, 0u, t));
    lds_or32(q + 1, __builtin_amdgcn_alignbit(v1, v0, t));
    lds_or32(q + 2, __builtin_amdgcn_alignbit(0u, v1, t));
  }
  // v (32 bits) at bit p >= 1: dwords j-1, j
  __device__ __forceinline__ void put32(uint32_t p, uint32_t v)
  {
    uint32_t* q = d() + ((p + 31u) >> 5) - 1;
    const uint32_t t = 0u - p;
    lds_or32(q, __builtin_amdgcn_alignbit(v, 0u, t));
    lds_or32(q + 1, __builtin_amdgcn_alignbit(0u, v, t));
  }
  // as put64, with the dwords clamped into the slot (bits past the budget)
  __device__ __forceinline__ void put64_clamped(uint32_t p, uint32_t v0, uint32_t v1)
  {
    uint32_t j = (p + 31u) >> 5;
    j = j < jmax - 1 ? j : jmax - 1;
    uint32_t* q = d() + j - 1;
    const uint32_t t = 0u - p;
    lds_or32(q, __builtin_amdgcn_alignbit(v0, 0u, t));
    lds_or32(q + 1, __builtin_amdgcn_alignbit(v1, v0, t));
    lds_or32(q + 2, __builtin_amdgcn_alignbit(0u, v1, t));
  }
  __device__ __forceinline__ void put32_clamped(uint32_t p, uint32_t v)
  {
    uint32_t j = (p + 31u) >> 5;
    j = j < jmax ? j : jmax;
    uint32_t* q = d() + j - 1;
    const uint32_t t = 0u - p;
    lds_or32(q, __builtin_amdgcn_alignbit(v, 0u, t));
    lds_or32(q + 1, __builtin_amdgcn_alignbit(0u, v, t));
  }
};

// Slot size (64-bit words) for a block budget of `lim` bits: a plane that starts
// at or before lim writes its verbatim bits through dword ceil(lim/32)+1 and its
// group bits through dword ceil((lim+64)/32); group extensions are clamped.
__host__ __device__ constexpr uint32_t slot_words_for(uint32_t lim) { return ((lim + 95u) / 32u) / 2u + 1u; }

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

// expansion of a 16-bit unit: 16 + popcount(u) <= 32 bits
__device__ __forceinline__ uint32_t dbl16(const uint32_t* lut, uint32_t u)
{
  const uint32_t b0 = u & 0xffu, b1 = (u >> 8) & 0xffu;
  return lut[b0] | (lut[b1] << (8u + (uint32_t)__popc(b0)));
}

// The coder tables as constants in device memory (a kernel copies them to LDS
// with one 16-byte load per lane instead of computing them):
//   dbl[b]  = dbl_entry(b)
//   lead[b] = (dbl(b) << 1 | 1) << 5 | (9 + popcount(b)): the first byte of a
//             plane's group bits with the leading "1" test, and in its low five
//             bits the shift that places the second byte's expansion after it
//             (code_planes_fr32).
struct CoderTables {
  uint32_t dbl[256];
  uint32_t lead[256];
  constexpr CoderTables() : dbl(), lead()
  {
    for (uint32_t b = 0; b < 256; b++) {
      uint32_t d = 0, p = 0, c = 0;
      for (int i = 0; i < 8; i++) {
        if ((b >> i) & 1u) {
          d |= 3u << p;
          p += 2;
          c++;
        } else {
          p += 1;
        }
      }
      dbl[b] = d;
      lead[b] = (((d << 1) | 1u) << 5) | (9u + c);
    }
  }
};
static __device__ const CoderTables kCoderTables{};

// ---------------------------------------------------------------------------
// LDS by byte address: the fixed-rate coder keeps each lane's stream position
// as a bit address in LDS, so the dword address and the funnel shift of every
// write come from one register.  (Host emulation: addresses are offsets from
// zfp_emu_lds_base.)
#ifdef __HIP_DEVICE_COMPILE__
typedef __attribute__((address_space(3))) uint32_t lds_dword;
__device__ __forceinline__ lds_dword* lds_at(uint32_t byte) { return (lds_dword*)(uintptr_t)byte; }
__device__ __forceinline__ uint32_t lds_off(const void* p) { return (uint32_t)(uintptr_t)p; }
// (byte k of x) * 4 in one SDWA instruction (the compiler spends a v_mov on the constant)
__device__ __forceinline__ uint32_t byte0_x4(uint32_t x)
{
  uint32_t r;
  asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0"
      : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ uint32_t byte1_x4(uint32_t x)
{
  uint32_t r;
  asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1"
      : "=v"(r) : "v"(x));
  return r;
}
__device__ __forceinline__ uint32_t ubfe(uint32_t x, uint32_t off, uint32_t w) { return __builtin_amdgcn_ubfe(x, off, w); }
#else
#ifdef __HIP__
// hipcc's host pass parses the device code but never runs it
#define ZFP_LDS_FN __device__ inline
static constexpr char* zfp_emu_lds_base = nullptr;
#else
#define ZFP_LDS_FN inline
inline char* zfp_emu_lds_base = nullptr;
#endif
typedef uint32_t lds_dword;
ZFP_LDS_FN lds_dword* lds_at(uint32_t byte) { return (lds_dword*)(zfp_emu_lds_base + byte); }
ZFP_LDS_FN uint32_t lds_off(const void* p) { return (uint32_t)((const char*)p - zfp_emu_lds_base); }
ZFP_LDS_FN uint32_t byte0_x4(uint32_t x) { return (x & 0xffu) << 2; }
ZFP_LDS_FN uint32_t byte1_x4(uint32_t x) { return ((x >> 8) & 0xffu) << 2; }
ZFP_LDS_FN uint32_t ubfe(uint32_t x, uint32_t off, uint32_t w)
{
  off &= 31;
  w &= 31;
  return w ? (uint32_t)((x >> off) & ((1ull << w) - 1)) : 0u;
}
#undef ZFP_LDS_FN
#endif

// Scheduling fence (no instruction moves across it).
#ifdef __HIP_DEVICE_COMPILE__
#define ZFP_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#else
#define ZFP_SCHED_FENCE() ((void)0)
#endif

template <typename U>
__device__ __forceinline__ void pin_value(U& x)
{
#ifdef __HIP_DEVICE_COMPILE__
  asm volatile("" : "+v"(x));
#endif
}

// Materialise every element at this point: the IR passes cannot sink the
// computation of these values into later (branchy) code, e.g. the last
// transpose steps into the plane coder, which would keep their inputs live.
template <typename U, int N>
__device__ __forceinline__ void pin_registers(U (&a)[N])
{
#ifdef __HIP_DEVICE_COMPILE__
#pragma unroll
  for (int i = 0; i < N; i++)
    asm volatile("" : "+v"(a[i]));
#endif
}

// Rare wave-uniform branches of the decoder (slow sections, sections past
// bit 32, the implicit last coefficient), laid out after the hot path: the f64
// short-slot decoder, at its register bound, 5.54 -> 4.84 ms on C3 (its
// per-block index check included); the f32 decoder's instruction-cache misses
// 5.8 -> 3.7 per wave at the same time (profiles/r4m_cold_ab.txt)
#define ZFP_RARE(x) __builtin_expect(!!(x), 0)

// Wave masks of a 32-bit unsigned compare (one v_cmp into an SGPR pair), for
// wave-level decisions: the same bits as __builtin_amdgcn_ballot_w64(a OP b),
// which the compiler tends to lower as a select, a compare and the ballot when
// the condition is combined with others.
__device__ __forceinline__ uint64_t lanes_ult(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 36); }
__device__ __forceinline__ uint64_t lanes_ule(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 37); }
__device__ __forceinline__ uint64_t lanes_ugt(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 34); }
__device__ __forceinline__ uint64_t lanes_ne(uint32_t a, uint32_t b) { return __builtin_amdgcn_uicmp(a, b, 33); }
// Bit reader over a word array in LDS (or global memory).
struct WordReader {
  const uint64_t* w;
  uint32_t pos;  // bit position within the lane's slot (slots are small)

  // Branch-free 64-bit window at bit p: the three dwords from dword p/32 on,
  // funnel-shifted by p % 32 (two v_alignbit_b32; a 64-bit shift costs about
  // three times a 32-bit op); they stay inside the slot, which has a spare
  // word past its last.
  __device__ __forceinline__ uint64_t peek_at(uint32_t p) const
  {
    const uint32_t* d = reinterpret_cast<const uint32_t*>(w) + (p >> 5);
    const uint32_t s = p & 31u;
    const uint32_t d0 = d[0], d1 = d[1], d2 = d[2];
    const uint32_t lo = __builtin_amdgcn_alignbit(d1, d0, s), hi = __builtin_amdgcn_alignbit(d2, d1, s);
    return ((uint64_t)hi << 32) | lo;
  }
  __device__ __forceinline__ uint64_t peek64() const { return peek_at(pos); }
  __device__ __forceinline__ uint64_t read(uint32_t n)
  {
    uint64_t v = n ? (peek64() & low_mask(n)) : 0ull;
    pos += n;
    return v;
  }
  __device__ __forceinline__ uint32_t read1()
  {
    const uint32_t i = pos >> 6, s = pos & 63u;
    pos++;
    return (uint32_t)((w[i] >> s) & 1u);
  }
  __device__ __forceinline__ void skip(uint32_t n) { pos += n; }
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
    // decode.c:9-34.  Each "a += b; b <<= 1; b -= a" is, in wrapping
    // arithmetic, b' = 2b - (a + b) = b - a and a' = a + b: two operations.
    y = add(y, w >> 1); w = sub(w, y >> 1);
    Int t = y; y = add(y, w); w = sub(w, t);
    t = z; z = add(z, x); x = sub(x, t);
    t = y; y = add(y, z); z = sub(z, t);
    t = w; w = add(w, x); x = sub(x, t);
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

// Negabinary is u = (x + K) ^ K with K = 0xaa..a (encode.c:67-71).  The XOR
// only inverts the odd bit planes, so the encoders transpose x + K and invert
// the odd planes in the transpose's last step, where the inversion is free
// (a three-input bit operation either way).
#ifndef ZFP_NB_FOLD
#define ZFP_NB_FOLD 1
#endif
template <typename U>
__device__ __forceinline__ U nb_planes(U x)
{
  return ZFP_NB_FOLD ? x : x ^ (U)0xaaaaaaaaaaaaaaaaull;
}

// ---------------------------------------------------------------------------
// Bit-matrix transpose of 32x32 bits held in 32 registers: a[r] bit c <-> a[c] bit r.
// Used both ways: coefficients -> bit planes (encode) and back (decode).
// ---------------------------------------------------------------------------
// Byte-granular steps are one v_perm_b32 per output word, the rest one shift
// plus one v_bfi_b32.
// INV_ODD: the encoders' last step also inverts the odd output words (odd
// planes); ODD_BITS: the decoders' last step inverts the odd bits of every
// output word (u ^ 0xaa..a of every coefficient, the first half of the
// negabinary decode), in the same single bit operation.
template <int J, bool INV_ODD = false, bool ODD_BITS = false>
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
    } else if constexpr (ODD_BITS) {  // M ? first : ~second, one v_bitop3 each
      a[k] = __builtin_amdgcn_bitop3_b32(x, y << J, M, 0xb1);
      a[k | J] = __builtin_amdgcn_bitop3_b32(x >> J, y, M, 0xb1);
    } else {
      a[k] = (x & M) | ((y << J) & ~M);
      if constexpr (INV_ODD)  // ~(x >> J ? M : y) as one v_bitop3 (the compiler would split it)
        a[k | J] = __builtin_amdgcn_bitop3_b32(x >> J, y, M, 0x1b);
      else
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

// decoder: bit planes -> coefficients u ^ K (negabinary decode: less K)
__device__ __forceinline__ void transpose32_dnb(uint32_t (&a)[32])
{
  transpose_step<16>(a);
  transpose_step<8>(a);
  transpose_step<4>(a);
  transpose_step<2>(a);
  transpose_step<1, false, true>(a);
}

// encoder: coefficients x + K -> negabinary bit planes (odd planes inverted)
__device__ __forceinline__ void transpose32_nb(uint32_t (&a)[32])
{
  transpose_step<16>(a);
  transpose_step<8>(a);
  transpose_step<4>(a);
  transpose_step<2>(a);
  transpose_step<1, ZFP_NB_FOLD != 0>(a);
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
// Closed form of one plane.  With n significant coefficients (mask S = the low
// n bits), N = plane & ~S holds the not-yet-significant ones; let h be the top
// one of xs = N >> n and c = popcount(N).  The reference's group tests
// (encode.c:92-132) emit "1", then every bit of xs up to h, each one followed by
// the next test's "1" -- the doubled-ones expansion dbl(xs) -- except that the
// top one's test is "0" (and both the top one and its test are implicit when
// it is coefficient 63); an empty N emits a single "0" (none when n == 64).
// So the group bits are g = [N != 0] | dbl(xs) << 1 minus the top pair's
// surplus: (2 + implicit) << (h + c).  The plane's length is
// n' + c + 1 - [n' == 64] - implicit with n' = bitlen(S | N).  One table look-up
// per byte gives dbl; lanes whose xs reaches past bit 15 (at most three planes
// per block) add the remaining 16-bit units in a wave-uniform branch.  The
// budget is not checked inside a plane: bits beyond it fall past the block end
// into the slot's spare words.
//
// Group units 1..3 of a plane whose top one lies past bit 15 of xs (h >= 16):
// at most three such planes per block (each makes >= 17 coefficients
// significant).  The 32-plane coder expands them where they occur, in a
// wave-uniform branch; the 64-plane coder records them and expands them after
// the plane loop.
struct ExtEvent {
  uint32_t gp;      // slot position of the plane's group bits
  uint32_t xl, xh;  // xs
  uint32_t hb;      // h | implicit << 6 | (bit 32 of g) << 7; h < 16: no event
};

__device__ __forceinline__ void expand_event(OrSlot& s, const uint32_t* lut, const ExtEvent& e)
{
  const uint32_t h = e.hb & 63u, impl = (e.hb >> 6) & 1u;
  const uint64_t xs = ((uint64_t)e.xh << 32) | e.xl;
  uint32_t D = 16u + (uint32_t)__popc(e.xl & 0xffffu);  // dbl length of unit 0
#pragma unroll
  for (int j = 1; j < 4; j++) {
    // the branch is entered for the wave: every per-lane effect is predicated
    const bool unit = h >= 16u * j;
    if (__any(unit)) {
      const uint32_t u = (uint32_t)(xs >> (16 * j)) & 0xffffu;
      const uint32_t cu = (uint32_t)__popc(u);
      uint32_t dj = dbl16(lut, u);
      if (h < 16u * (j + 1))  // the top one is in this unit
        dj -= (2u + impl) << ((h - 16u * j + cu - 1u) & 31u);
      if (unit) {
        if (j == 1)  // also carries bit 32 of g (unit 0 all ones)
          s.put64_clamped(e.gp + D, (dj << 1) | (e.hb >> 7), dj >> 31);
        else
          s.put32_clamped(e.gp + 1u + D, dj);
      }
      D += 16u + cu;
    }
  }
}

// Codes planes PREC-1 .. PREC-maxprec starting at bit `pos` (>= 1) of the slot;
// returns the end position clamped to `lim` (the block's bit budget end).
// Fully unrolled: plane k is a register, the coder state is renamed, not
// copied.  PLIM = false (fixed rate, maxprec >= PREC): lanes that reach the
// budget keep going with their position pinned at lim, so their bits land in
// the slot's spare words and no per-lane predication is needed.  PLIM = true:
// a lane stops at its precision limit, so its state is updated under `act`.
#ifndef ZFP_FR_EXIT_PLANES
#define ZFP_FR_EXIT_PLANES 16
#endif
// x >> 5 hidden from the optimizer, which would otherwise rewrite the dword
// address (x >> 5) * 4 + base as ((x >> 3) & ~3) + base: three operations
// instead of a shift and a v_lshl_add_u32
__device__ __forceinline__ uint32_t opaque_shr5(uint32_t x)
{
#ifdef __HIP_DEVICE_COMPILE__
  uint32_t r;
  asm("v_lshrrev_b32 %0, 5, %1" : "=v"(r) : "v"(x));
  return r;
#else
  return x >> 5;
#endif
}

// SIZE: coefficients per block (4^d; 64 for 3D).  Only the block's last
// coefficient (implicit one and test) and the all-significant plane depend on it.
// kstart, n0: start at plane kstart (wave-uniform) with n0 coefficients already
// significant (the fixed-rate f32 coder hands over to this one mid-block).
template <int PREC, bool PLIM, int SIZE = 64>
__device__ __forceinline__ uint32_t code_planes(OrSlot& s, const uint32_t* lut, uint32_t pos, uint32_t lim,
                                                uint32_t maxprec, const uint32_t (&Pl)[PREC],
                                                const uint32_t (&Ph)[PREC], int kstart = PREC - 1, uint32_t n0 = 0)
{
  const uint32_t kmin = (uint32_t)PREC > maxprec ? (uint32_t)PREC - maxprec : 0u;
  uint32_t* const dm1 = s.d() - 1;  // dword j-1 of a position with j = ceil(p / 32)
  const uint32_t lim31 = lim + 31u;
  uint32_t p31 = pos + 31u;  // position + 31: j = p31 >> 5, alignbit shift = 31 - p31
  uint32_t n = n0, nn = ~n0;
  uint32_t Sl = n0 >= 32u ? ~0u : (1u << n0) - 1u, Sh = n0 >= 64u ? ~0u : n0 > 32u ? (1u << (n0 - 32u)) - 1u : 0u;
  ExtEvent e0{0, 0, 0, 0}, e1{0, 0, 0, 0}, e2{0, 0, 0, 0};  // PREC > 32 only
#ifdef ZFP_PLANE_UNROLL
#pragma unroll ZFP_PLANE_UNROLL
#else
#pragma unroll
#endif
  for (int k = PREC - 1; k >= 0; k--) {
    if (k > kstart)
      continue;
    const bool act = p31 < lim31 && (!PLIM || (uint32_t)k >= kmin);
    // wave-level exit once every lane is done; without a precision limit
    // (fixed rate) only the low planes are checked: a block rarely spends
    // its budget in fewer planes, and each check is a VALU->SALU->branch
    // round trip
    if ((PLIM || k < ZFP_FR_EXIT_PLANES) && __builtin_amdgcn_ballot_w64(act) == 0)
      break;
    const uint32_t pl = Pl[k], ph = Ph[k];
    const uint32_t Nl = pl & ~Sl, Nh = ph & ~Sh;
    const uint64_t N = ((uint64_t)Nh << 32) | Nl;
    const bool nz = N != 0;
    const uint32_t clz = (uint32_t)__clzll((long long)(N | 1ull));  // of N when nz
    const uint32_t n1 = nz ? 64u - clz : n;
    const uint64_t S1 = nz ? (~0ull >> clz) : (((uint64_t)Sh << 32) | Sl);
    const uint32_t t2 = (uint32_t)__popc(Nh) + ((uint32_t)__popc(Nl) + n1);  // n' + c
    // top one is the last coefficient (SIZE - 1)
    const uint32_t impl = SIZE == 64 ? Nh >> 31 : (uint32_t)(N >> (SIZE - 1)) & 1u;
    const uint64_t xs = N >> (n & 63u);  // n == 64 only with N == 0
    const uint32_t x0 = (uint32_t)xs;
    const uint32_t b0 = x0 & 0xffu;
    const uint32_t sh1 = 8u + (uint32_t)__popc(b0);
    // the table reads fly while the verbatim bits and the rare branch below
    // are issued; the doubled-ones unit d16 is assembled where it is used
    const uint32_t l0 = lut[b0], l1 = lut[(x0 >> 8) & 0xffu];
    const uint32_t m = (2u | impl) << ((t2 + nn) & 31u);  // surplus of the top pair at h + c
    const uint32_t h = n1 + nn;  // top one of xs (when nz)
    const bool ext = SIZE > 16 && act && nz && h >= 16u;
    const int32_t dlen = SIZE == 64 ? (int32_t)t2 + 1 + ((int32_t)(uint32_t)(S1 >> 32) >> 31) + ((int32_t)Nh >> 31)
                                    : (int32_t)t2 + 1 - (int32_t)((S1 >> (SIZE - 1)) & 1u) - (int32_t)impl;
    if (!PLIM) {
      uint32_t* q = dm1 + opaque_shr5(p31);
      const uint32_t t = 31u - p31;
      const uint32_t v0 = pl ^ Nl, v1 = ph ^ Nh;  // the n verbatim bits
      lds_or32(q, __builtin_amdgcn_alignbit(v0, 0u, t));
      lds_or32(q + 1, __builtin_amdgcn_alignbit(v1, v0, t));
      lds_or32(q + 2, __builtin_amdgcn_alignbit(0u, v1, t));
    }
    if (__builtin_amdgcn_ballot_w64(ext) != 0) {
      const uint32_t g32 = (l1 << sh1) >> 31;  // bit 31 of d16: bit 32 of the plane's group bits
      const ExtEvent e{p31 - 31u + n, x0, (uint32_t)(xs >> 32), h | (impl << 6) | (g32 << 7)};
      if constexpr (PREC <= 32) {
        // rare (a few planes per wave): the lanes whose top one lies past
        // unit 0 write their remaining group units now, the others take no part
        expand_event(s, lut, ExtEvent{e.gp, e.xl, e.xh, ext ? e.hb : 0u});
      } else if (ext) {
        // 64 planes: the inline expansion would keep the plane loop from
        // being unrolled, so the (at most three) events are expanded after it
        e2 = e1;
        e1 = e0;
        e0 = e;
      }
    }
    const uint32_t d16 = l0 | (l1 << sh1);
    // the top pair's surplus is in unit 0 unless the top one lies past it
    const uint32_t g = ((d16 << 1) | (nz ? 1u : 0u)) - (ext ? 0u : m);
    if (PLIM) {
      if (act) {
        // clamped: a short slot (encode3_general) may be outrun by a block
        // that is coded again into an overflow slot
        s.put64_clamped(p31 - 31u, pl ^ Nl, ph ^ Nh);  // the n verbatim bits
        s.put32_clamped(p31 - 31u + n, g);
      }
      p31 = act ? p31 + (uint32_t)dlen : p31;
      n = act ? n1 : n;
      Sl = act ? (uint32_t)S1 : Sl;
      Sh = act ? (uint32_t)(S1 >> 32) : Sh;
    } else {
      const uint32_t pg = p31 + n;
      uint32_t* q = dm1 + opaque_shr5(pg);
      const uint32_t t = 31u - pg;
      lds_or32(q, __builtin_amdgcn_alignbit(g, 0u, t));
      lds_or32(q + 1, __builtin_amdgcn_alignbit(0u, g, t));
      p31 += (uint32_t)dlen;
      p31 = p31 < lim31 ? p31 : lim31;
      n = n1;
      Sl = (uint32_t)S1;
      Sh = (uint32_t)(S1 >> 32);
    }
    nn = ~n;
  }
  if constexpr (PREC > 32) {
    if (__any(e0.hb >= 16u)) {
      expand_event(s, lut, e0);
      if (__any(e1.hb >= 16u)) {
        expand_event(s, lut, e1);
        if (__any(e2.hb >= 16u))
          expand_event(s, lut, e2);
      }
    }
  }
  const uint32_t end = p31 - 31u;
  return end < lim ? end : lim;
}

// ---------------------------------------------------------------------------
// Fixed-rate coder of a 32-plane block (f32, encode3_aligned): the same planes
// and bits as code_planes<32, false>, with a 32-bit plane body for the planes
// in which no lane of the wave has anything in coefficients 32..63 and fewer
// than 32 significant coefficients -- on smooth data all but the last few
// planes (the C2 field: planes 31..8).  There the plane needs no 64-bit
// arithmetic:
//   xs = plane >> n (the not-yet-significant coefficients), bl = bitlen(xs),
//   c = popcount(xs); the plane is n verbatim bits then e1 + 1 group bits with
//   e1 = bl + c, g = (dbl(xs) << 1 | 1) - 2^e1 (code_planes' closed form: the
//   leading test, the doubled-ones expansion, the top pair's surplus; xs == 0
//   gives the single "0").  The first byte's expansion with the leading 1 and
//   the shift for the second byte come from one table entry (lead[]).
//   xs >= 0xffff (the top one past unit 0, or e1 == 32) takes the wave-uniform
//   extension branch of code_planes.
// The lane's position is kept as Q = -(bit address in LDS): the dword address
// of a write is ~((Q >> 3) | 3) and the funnel shift is Q itself (mod 32).  At
// the first plane where some lane leaves the 32-bit form (the condition only
// becomes true once: n never shrinks) the rest of the block goes to
// code_planes from that plane on.  `slot`: the lane's zeroed slot of `jmax`+1
// dwords; lut: dbl[256] then lead[256] (CoderTables layout, in LDS).
__device__ __forceinline__ void fr_write32(int32_t Q, uint32_t v)
{
  const uint32_t a = ~(((uint32_t)(Q >> 3)) | 3u);
  ZFP_LDS_OR(lds_at(a), __builtin_amdgcn_alignbit(v, 0u, (uint32_t)Q));
  ZFP_LDS_OR(lds_at(a + 4u), __builtin_amdgcn_alignbit(0u, v, (uint32_t)Q));
}

// v1:v0 at bit address -Q: three dwords
__device__ __forceinline__ void fr_write64(int32_t Q, uint32_t v0, uint32_t v1)
{
  const uint32_t a = ~(((uint32_t)(Q >> 3)) | 3u);
  ZFP_LDS_OR(lds_at(a), __builtin_amdgcn_alignbit(v0, 0u, (uint32_t)Q));
  ZFP_LDS_OR(lds_at(a + 4u), __builtin_amdgcn_alignbit(v1, v0, (uint32_t)Q));
  ZFP_LDS_OR(lds_at(a + 8u), __builtin_amdgcn_alignbit(0u, v1, (uint32_t)Q));
}

#ifndef ZFP_FR32
#define ZFP_FR32 1
#endif
#ifndef ZFP_FRU
#define ZFP_FRU 1
#endif

// Fixed-rate plane body for the planes after the 32-bit lo form (any lane
// with coefficients 32..63 in play): every lane codes from a 32-bit window
// x0 = bits 0..31 of xs = N >> n,
//   n < 32:  alignbit(Nh, pl, n)   (the plane's bits n..n+31)
//   n >= 32: Nh >> (n - 32)        (Nh = ph & ~Sh; n == 64 gives 0)
// and, while xs has its top one inside unit 0 (x0 < 0xffff, bits 32.. of xs
// zero), the group bits are the lead-table expansion cut to e1 - impl bits
// (e1 = bitlen(x0) + popcount(x0); impl: the top one is coefficient 63, whose
// test and value are implicit), the plane's length n + e1 - impl + [n' < 64].
// Lanes whose xs reaches past unit 0 (or is 0xffff: 33 group bits) are
// recomputed in a wave-uniform branch from the 64-bit xs, as code_planes does.
// No 64-bit arithmetic on the common path; the verbatim bits are pl cut to n
// bits (n < 32) or pl and ph & Sh (Sh: the significant high coefficients).
// Positions as in code_planes_fr32 (Q = -bit address).
__device__ __forceinline__ void code_planes_fru(OrSlot& os, const uint32_t* lut, uint32_t sb, int32_t Q,
                                                int32_t Qlim, uint32_t n, int kstart, const uint32_t (&Pl)[32],
                                                const uint32_t (&Ph)[32])
{
  const uint32_t tdbl = lds_off(lut), tlead = tdbl + 1024u;
  uint32_t Sh = n > 32u ? ~0u >> ((0u - n) & 31u) : 0u;
#pragma unroll
  for (int k = 31; k >= 0; k--) {
    if (k > kstart)
      continue;
    if (k < ZFP_FR_EXIT_PLANES && __builtin_amdgcn_ballot_w64(Q > Qlim) == 0)
      break;
    const uint32_t pl = Pl[k], ph = Ph[k];
    const bool hi = n >= 32u;
    const uint32_t Nh = ph & ~Sh;
    const uint32_t t = Nh >> (n & 31u);
    const uint32_t x0 = hi ? t : __builtin_amdgcn_alignbit(Nh, pl, n);
    const uint32_t x1 = hi ? 0u : t;  // bits 32..63 of xs
    const uint32_t l0 = *lds_at(tlead + byte0_x4(x0));
    const uint32_t l1 = *lds_at(tdbl + byte1_x4(x0));
    const uint32_t bl = 31u - (uint32_t)__clz((int)((x0 << 1) | 1u));  // bitlen(x0) for x0 < 2^31
    const uint32_t e1 = (uint32_t)__popc(x0) + bl;
    const uint32_t impl = Nh >> 31;  // top one at coefficient 63 (lanes without ext)
    uint32_t n1 = n + bl;
    const uint32_t d = (l1 << (l0 & 31u)) | (l0 >> 5);  // (dbl(x0 & 0xffff) << 1 | 1) mod 2^32
    uint32_t g = ubfe(d, 0u, e1 - impl);
    uint32_t L = e1 - impl + 1u - (n1 >> 6);  // group bits: none once all 64 are significant
    const bool ext = x0 > 0xfffeu || x1 != 0u;
    const int32_t Qg = Q - (int32_t)n;
    if (__builtin_amdgcn_ballot_w64(ext) != 0) {
      // rare: xs reaches past unit 0 (or x0 == 0xffff); the other lanes take no part
      uint32_t hb = 0;
      if (ext) {
        const uint32_t hx = x1 ? 63u - (uint32_t)__clz((int)x1) : 31u - (uint32_t)__clz((int)x0);  // top of xs
        const uint32_t c = (uint32_t)__popc(x0) + (uint32_t)__popc(x1);
        n1 = n + hx + 1u;
        const uint32_t im = n1 >> 6;
        L = hx + c + 2u - 2u * im;
        // top one in unit 0 (x0 == 0xffff): the 33-bit expansion less the
        // top pair's surplus (bit 32, and bit 31 when implicit); else unit 0
        // whole, the surplus in a later unit, and bit 32 of the group bits
        // the last of an all-ones unit 0's expansion
        g = hx < 16u ? d & ~(im << 31) : d;
        hb = hx | (im << 6) | ((x0 & 0xffffu) == 0xffffu ? 0x80u : 0u);
      }
      expand_event(os, lut, ExtEvent{(uint32_t)(-Qg) - sb, x0, x1, hb});
    }
    fr_write64(Q, hi ? pl : ubfe(pl, 0u, n), ph & Sh);  // the n verbatim bits
    fr_write32(Qg, g);
    const int32_t Qn = Qg - (int32_t)L;
    Q = Qn > Qlim ? Qn : Qlim;
    n = n1;
    Sh = n > 32u ? ~0u >> ((0u - n) & 31u) : 0u;
  }
}

__device__ __forceinline__ void code_planes_fr32(uint32_t* slot, uint32_t jmax, const uint32_t* lut, uint32_t pos,
                                                 uint32_t lim, const uint32_t (&Pl)[32], const uint32_t (&Ph)[32])
{
  OrSlot os{reinterpret_cast<uint64_t*>(slot), jmax};
#if ZFP_FR32
  const uint32_t sb = lds_off(slot) * 8u;  // slot bit address
  const uint32_t tdbl = lds_off(lut), tlead = tdbl + 1024u;
  int32_t Q = -(int32_t)(sb + pos);
  const int32_t Qlim = -(int32_t)(sb + lim);
  uint32_t n = 0;
  bool m32 = true;
  int ksw = 0;
#pragma unroll
  for (int k = 31; k >= 0; k--) {
    if (m32) {
      if (__builtin_amdgcn_ballot_w64(Ph[k] != 0u || n > 31u) != 0) {
        m32 = false;
        ksw = k;
      } else {
        const uint32_t pl = Pl[k];
        const uint32_t xs = pl >> n;
        const uint32_t l0 = *lds_at(tlead + byte0_x4(xs));
        const uint32_t l1 = *lds_at(tdbl + byte1_x4(xs));
        const uint32_t bl = 32u - (uint32_t)__clz((int)xs);
        const uint32_t e1 = (uint32_t)__popc(xs) + bl;
        fr_write32(Q, ubfe(pl, 0u, n));  // the n verbatim bits
        const int32_t Qg = Q - (int32_t)n;
        const uint32_t d = (l1 << (l0 & 31u)) | (l0 >> 5);  // (dbl(xs & 0xffff) << 1 | 1) mod 2^32
        uint32_t g = d - (1u << (e1 & 31u));
        const bool ext = xs > 0xfffeu;
        if (__builtin_amdgcn_ballot_w64(ext) != 0) {
          // rare: the lanes whose top one lies past unit 0 (or xs == 0xffff,
          // whose group bits are 33 long) have no surplus in unit 0; their
          // later units are written as in code_planes (bit 32 of the group
          // bits is the last bit of an all-ones unit 0's expansion)
          const uint32_t h = 31u - (uint32_t)__clz((int)xs);
          const uint32_t gp = (uint32_t)(-Qg) - sb;
          const uint32_t g32 = (xs & 0xffffu) == 0xffffu ? 1u : 0u;
          g = ext ? d : g;
          expand_event(os, lut, ExtEvent{gp, xs, 0u, ext ? h | (g32 << 7) : 0u});
        }
        fr_write32(Qg, g);
        const int32_t Qn = Qg - (int32_t)e1 - 1;
        Q = Qn > Qlim ? Qn : Qlim;
        n += bl;
      }
    }
  }
  if (!m32) {
#if ZFP_FRU
    code_planes_fru(os, lut, sb, Q, Qlim, n, ksw, Pl, Ph);
#else
    code_planes<32, false>(os, lut, (uint32_t)(-Q) - sb, lim, 32u, Pl, Ph, ksw, n);
#endif
  }
#else
  code_planes<32, false>(os, lut, pos, lim, 32u, Pl, Ph);
#endif
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

template <int SIZE = 64>
__device__ __forceinline__ void decode_group_slow(WordReader& r, uint64_t& x, uint32_t& bits, uint32_t& n)
{
  while (bits && n < (uint32_t)SIZE) {
    bits--;
    if (!r.read1())
      break;
    uint32_t lim = (uint32_t)SIZE - 1 - n;
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

// Squeeze of a mask F of pair-first bits (each one is followed by its pair's
// deleted second bit): the r-th one, at bit p, moves to bit p - r.  Eight byte
// look-ups merged pairwise in 32-bit halves -- no loop, no 64-bit shift per
// byte; the length of a squeezed piece is its bit width minus its ones.
__device__ __forceinline__ uint32_t squeeze32(const uint32_t* sq, uint32_t f)
{
  const uint32_t b0 = f & 0xffu, b1 = (f >> 8) & 0xffu, b2 = (f >> 16) & 0xffu, b3 = f >> 24;
  const uint32_t u0 = sq[b0] | (sq[b1] << (8u - (uint32_t)__popc(b0)));
  const uint32_t u1 = sq[b2] | (sq[b3] << (8u - (uint32_t)__popc(b2)));
  return u0 | (u1 << (16u - (uint32_t)__popc(f & 0xffffu)));
}

// One bit plane: n verbatim bits, then the group section.  Straight-line for
// every lane (the verbatim window and the section window are both read, the
// section is parsed in closed form and its consumption selected); only lanes
// whose section is not closed-form run the reference loop, in a wave-uniform
// branch.
template <bool IMP = true, int SIZE = 64>
__device__ __forceinline__ uint64_t decode_plane64(WordReader& r, const uint32_t* sq, uint32_t& bits, uint32_t& n)
{
  const uint32_t m = n < bits ? n : bits;
  uint32_t pos = r.pos;
  const uint64_t V = r.peek_at(pos);
  uint64_t x = m ? V & (~0ull >> ((64u - m) & 63u)) : 0ull;
  pos += m;
  uint32_t bl = bits - m;
  const bool grp = n < (uint32_t)SIZE && bl != 0;
  if (!__any(grp)) {  // every lane's plane is all verbatim (n == 64) or out of budget
    r.pos = pos;
    bits = bl;
    return x;
  }
  const uint64_t w = r.peek_at(pos);
  const bool one = (w & 1) != 0;
  const uint64_t S = w >> 1;
  const uint64_t starts = S & ~(S << 1);
  const uint64_t se = S + (starts & kEven), so = S + (starts & kOdd);
  // S holds 63 stream bits; its bit 63 is not data, so a run reaching
  // bit 62 must not be taken as ended there
  const uint64_t ends = (((se & ~S) & kOdd) | ((so & ~S) & kEven)) & ~(1ull << 63);
  const uint32_t q = ctz64(ends);
  const uint64_t mq = (ends - 1) & ~ends;  // bits below q (all when ends == 0)
  const uint32_t ones = (uint32_t)__popcll(S & mq);
  const uint32_t P = q - (ones - 1) / 2;
  const bool fast = grp && one && ends != 0 && n + P <= (uint32_t)SIZE - 1 && q + 2 <= bl;
  // The section reaches coefficient 63 before its stop (or runs past the
  // window): the reference parses the k63 = 63 - n tokens below it and sets
  // bit 63 without reading it (decode.c:69-120, n < size - 1).  In the
  // squeezed (token) domain a token costs 1 bit plus 1 if it is a one.
  const bool imp0 = IMP && grp && one && !fast && (ends == 0 || n + P > (uint32_t)SIZE - 1);
  const uint64_t F = (fast || imp0) ? S & mq & (((S & ~se) & kEven) | ((S & ~so) & kOdd)) : 0ull;
  const uint32_t Fl = (uint32_t)F, Fh = (uint32_t)(F >> 32);
  uint64_t xx = squeeze32(sq, Fl);
  if (ZFP_RARE(__any(Fh != 0)))  // some section reaches past stream bit 32
    xx |= (uint64_t)squeeze32(sq, Fh) << (32u - (uint32_t)__popc(Fl));
  uint32_t k63 = 0, si = 0;
  uint64_t xi = 0;
  bool imp = false;
  if (ZFP_RARE(__any(imp0))) {  // wave-uniform: most planes have no such lane
    k63 = ((uint32_t)SIZE - 1 - n) & 63u;  // tokens below the last coefficient
    xi = xx & ((1ull << k63) - 1);
    si = k63 + (uint32_t)__popcll(xi);  // section bits of those tokens
    imp = imp0 && si <= 63u && si + 1u <= bl;
  }
  x |= (fast ? xx : (imp ? xi | (1ull << k63) : 0ull)) << (n & 63u);
  const uint32_t used = fast ? q + 2u : (imp ? si + 1u : (grp && !one ? 1u : 0u));
  n = fast ? n + P : (imp ? (uint32_t)SIZE : n);
  r.pos = pos + used;
  bits = bl - used;
  const bool slow = grp && one && !fast && !imp;
  if (ZFP_RARE(__any(slow))) {
    if (slow)
      decode_group_slow<SIZE>(r, x, bits, n);
  }
  return x;
}

template <int K, int PREC, bool IMP, int SIZE = 64>
struct DecodePlanes {
  static __device__ __forceinline__ void run(WordReader& r, const uint32_t* sq, uint64_t (&P)[PREC], uint32_t kmin,
                                             uint32_t& bits, uint32_t& n)
  {
    const bool act = bits != 0 && (uint32_t)K >= kmin;
    if (!__any(act))
      return;
    // a lane past its precision limit decodes with no budget: no effect
    uint32_t b = act ? bits : 0u;
    P[K] = decode_plane64<IMP, SIZE>(r, sq, b, n);
    bits = act ? b : bits;
    DecodePlanes<K - 1, PREC, IMP, SIZE>::run(r, sq, P, kmin, bits, n);
  }
};

template <int PREC, bool IMP, int SIZE>
struct DecodePlanes<-1, PREC, IMP, SIZE> {
  static __device__ __forceinline__ void run(WordReader&, const uint32_t*, uint64_t (&)[PREC], uint32_t, uint32_t&,
                                             uint32_t&)
  {
  }
};

// IMP: closed form for sections reaching coefficient 63 (false for the f64
// maxprec <= 32 decoder, where it measured slower than the reference loop).
template <int PREC, bool IMP = true, int SIZE = 64>
__device__ __forceinline__ uint32_t decode_planes64(WordReader& r, const uint32_t* sq, uint32_t budget,
                                                    uint32_t maxprec, uint64_t (&P)[PREC])
{
  const uint32_t kmin = (uint32_t)PREC > maxprec ? (uint32_t)PREC - maxprec : 0u;
  uint32_t bits = budget;
  uint32_t n = 0;
#pragma unroll
  for (int k = 0; k < PREC; k++)
    P[k] = 0;
  DecodePlanes<PREC - 1, PREC, IMP, SIZE>::run(r, sq, P, kmin, bits, n);
  return budget - bits;
}

// ---------------------------------------------------------------------------
// 32-plane decoder (f32 blocks) with a 32-bit plane body, the twin of
// code_planes_fr32: while every lane of the wave has fewer than 32
// significant coefficients, a plane is parsed from ONE 64-bit window at its
// start (the n verbatim bits, the lead test and 31 section bits), with 32-bit
// arithmetic: the section's end by decode_plane64's carry trick on 31 bits,
// its ones squeezed out with the byte table.  A lane takes decode_plane64
// (the reference loop included) for the plane instead when its section does
// not end inside the window, makes coefficient 32 or later significant, or
// its budget could end inside the plane (bits < 64); past its precision limit
// a lane reads nothing.  Once some lane has 32 significant coefficients the
// remaining planes go to decode_plane64 for every lane.
// more lanes than this in a plane's slow path: the rest of the block without the
// 32-bit body (tests/test_emu.py sets it to 0 to run the switch on every slow plane)
#ifndef ZFP_DEC32_DENSE
#define ZFP_DEC32_DENSE 16
#endif
template <bool IMP = true>
__device__ __forceinline__ uint32_t decode_planes32(WordReader& r, const uint32_t* sq, uint32_t budget,
                                                    uint32_t maxprec, uint64_t (&P)[32])
{
  const uint32_t kmin = 32u > maxprec ? 32u - maxprec : 0u;
  uint32_t bits = budget, n = 0;
#pragma unroll
  for (int k = 0; k < 32; k++)
    P[k] = 0;
  bool m32 = true;
  int ksw = -1;
#pragma unroll
  for (int k = 31; k >= 0; k--) {
    if (!m32)
      continue;
    if (__builtin_amdgcn_ballot_w64(n > 31u) != 0) {
      m32 = false;
      ksw = k;
      continue;
    }
    const bool act = bits != 0 && (uint32_t)k >= kmin;
    if (__builtin_amdgcn_ballot_w64(act) == 0) {  // every lane done (budget or precision): so are later planes
      m32 = false;
      continue;
    }
    const uint64_t W = r.peek_at(r.pos);
    const uint32_t lo = (uint32_t)W, hi = (uint32_t)(W >> 32);
    const uint32_t g = __builtin_amdgcn_alignbit(hi, lo, n);  // stream bits n .. n+31 of the plane
    const uint32_t S = g >> 1;                                // 31 section bits after the lead test
    const uint32_t starts = S & ~(S << 1);
    const uint32_t se = S + (starts & 0x55555555u), so = S + (starts & 0xaaaaaaaau);
    // bit 31 of S is not data: a run reaching bit 30 has not ended there
    const uint32_t ends = ((se & ~S) & 0x2aaaaaaau) | ((so & ~S) & 0x55555555u);
    const uint32_t q = ends ? (uint32_t)__builtin_ctz(ends) : 32u;
    const uint32_t mq = (ends - 1u) & ~ends;
    const uint32_t ones = (uint32_t)__popc(S & mq);
    const uint32_t np = q - (ones - 1u) / 2u;  // coefficient positions the section covers
    const bool one = (g & 1u) != 0;
    const bool fast = act && bits >= 64u && (!one || (ends != 0u && n + np <= 32u));
    const uint32_t F = one ? S & mq & (((S & ~se) & 0x55555555u) | ((S & ~so) & 0xaaaaaaaau)) : 0u;
    const uint32_t xx = squeeze32(sq, F);
    const uint32_t x = ubfe(lo, 0u, n) | (xx << n);
    const uint32_t used = n + (one ? q + 2u : 1u);
    if (fast) {
      P[k] = x;
      r.pos += used;
      bits -= used;
      n += one ? np : 0u;
    }
    const bool slow = act && !fast;
    const uint64_t sm = __builtin_amdgcn_ballot_w64(slow);
    if (ZFP_RARE(sm != 0)) {
      if (slow) {
        uint32_t b = bits;
        P[k] = decode_plane64<IMP>(r, sq, b, n);
        bits = b;
      }
      // dense planes (long sections: reversible, high precision): from here on
      // decode_plane64 alone, without the 32-bit attempt first
      if (__popcll(sm) > ZFP_DEC32_DENSE) {
        m32 = false;
        ksw = k - 1;
      }
    }
  }
  if (!m32) {
#pragma unroll
    for (int k = 31; k >= 0; k--) {
      if (k > ksw)
        continue;
      const bool act = bits != 0 && (uint32_t)k >= kmin;
      if (__builtin_amdgcn_ballot_w64(act) == 0)
        break;
      uint32_t b = act ? bits : 0u;  // a lane past its precision limit decodes with no budget: no effect
      P[k] = decode_plane64<IMP>(r, sq, b, n);
      bits = act ? b : bits;
    }
  }
  return budget - bits;
}

}  // namespace zfp_amd
