// Per-lane codec of one 4x4x4 block (float or double) for every zfp mode.
//
// encode_block3: lossy (encodef.c:63-90 + encode.c:260-280) and reversible
//                (revencodef.c:45-80 + revencode.c:54-76) block encoders.
// decode_block3: decodef.c:7-36 + decode.c:271-287, revdecodef.c:22-59 +
//                revdecode.c:34-52.
// Block gather/scatter with partial-block padding: encode3.c:5-31 /
// decode3.c:5-23, pad rule encode.c:9-27.
#pragma once

#include "codec_dev.h"

namespace zfp_amd {

// pad a partial line of n valid values (n >= 1 here; n == 0 cannot occur
// for a block whose origin lies inside the field)
template <typename S>
__device__ __forceinline__ void pad_line(S* v, int b, int s, int n)
{
  if (n <= 1) v[b + s] = v[b];
  if (n <= 2) v[b + 2 * s] = v[b + s];
  if (n <= 3) v[b + 3 * s] = v[b];
}

// x / d for 32-bit x by an invariant d >= 1 (round-up method: 33-bit magic
// split into m and two shifts; exact for every x)
struct FastDiv {
  uint32_t m, s1, s2;
};

__host__ __device__ inline FastDiv make_fastdiv(uint32_t d)
{
  if (d == 0)
    d = 1;
  uint32_t l = 0;
  while (l < 32 && (1ull << l) < d)
    l++;  // ceil(log2 d)
  const uint64_t m = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
  return FastDiv{(uint32_t)m, l < 1 ? l : 1u, l > 1 ? l - 1 : 0u};
}

__device__ __forceinline__ uint32_t fastdiv(uint32_t x, const FastDiv& f)
{
  const uint32_t t = __umulhi(x, f.m);
  return (t + ((x - t) >> f.s1)) >> f.s2;
}

struct Geometry {
  uint64_t n[4];
  int64_t s[4];
  uint64_t f[4];
  uint32_t nb[4];  // blocks per axis in the chunk box
  FastDiv dv[3];   // division by nb[0..2] (block index -> coordinates)
  uint64_t nblocks;  // < 2^32 (checked by the host)
};

struct BlockPos {
  int64_t off;  // element offset of the block origin
  int cnt[4];   // valid extent per axis (<= 4)
  bool full;
};

__device__ __forceinline__ BlockPos block_pos(const Geometry& g, uint64_t b64, int dims)
{
  BlockPos p;
  p.off = 0;
  p.full = true;
  uint32_t b = (uint32_t)b64;
#pragma unroll
  for (int a = 0; a < 4; a++) {
    p.cnt[a] = 4;
    if (a < dims) {
      uint32_t bi = b;
      if (a < dims - 1) {
        const uint32_t q = fastdiv(b, g.dv[a]);
        bi = b - q * g.nb[a];
        b = q;
      }
      uint64_t x = g.f[a] + 4ull * bi;
      uint64_t left = g.n[a] - x;
      p.cnt[a] = left < 4 ? (int)left : 4;
      p.full = p.full && left >= 4;
      p.off += (int64_t)x * g.s[a];
    }
  }
  return p;
}

// 16 bytes of scalars, for one vector load/store
template <typename S, int N>
struct alignas(16) Vec16 {
  S v[N];
};

// Streaming field reads (each byte is read once): ZFP_NT_LOAD marks them
// non-temporal.
#ifndef ZFP_NT_LOAD
#define ZFP_NT_LOAD 1
#endif
#ifndef ZFP_NT_STORE
#define ZFP_NT_STORE 1
#endif
template <typename S, int N>
__device__ __forceinline__ Vec16<S, N> load16(const S* p)
{
#if ZFP_NT_LOAD && defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  const u4 x = __builtin_nontemporal_load(reinterpret_cast<const u4*>(p));
  Vec16<S, N> r;
  __builtin_memcpy(&r, &x, 16);
  return r;
#else
  return *reinterpret_cast<const Vec16<S, N>*>(p);
#endif
}

// streaming writes of decoded values / stream words (ZFP_NT_STORE: non-temporal)
template <typename S, int N>
__device__ __forceinline__ void store16(S* p, const Vec16<S, N>& q)
{
#if ZFP_NT_STORE && defined(__HIP_DEVICE_COMPILE__)
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  u4 x;
  __builtin_memcpy(&x, &q, 16);
  __builtin_nontemporal_store(x, reinterpret_cast<u4*>(p));
#else
  *reinterpret_cast<Vec16<S, N>*>(p) = q;
#endif
}

template <typename S, bool VEC>
__device__ __forceinline__ void gather3(S (&v)[64], const S* __restrict__ base, const Geometry& g, const BlockPos& p)
{
  const S* o = base + p.off;
  const int64_t sx = g.s[0], sy = g.s[1], sz = g.s[2];
  if (p.full) {
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const S* r = o + j * sy + k * sz;
        if (VEC) {
          // 16-byte loads of any scalar type (4 floats/int32 or 2 doubles/int64)
          if constexpr (sizeof(S) == 4) {
            const Vec16<S, 4> q = load16<S, 4>(r);
#pragma unroll
            for (int i = 0; i < 4; i++)
              v[16 * k + 4 * j + i] = q.v[i];
          } else {
            const Vec16<S, 2> q0 = load16<S, 2>(r);
            const Vec16<S, 2> q1 = load16<S, 2>(r + 2);
            v[16 * k + 4 * j + 0] = q0.v[0];
            v[16 * k + 4 * j + 1] = q0.v[1];
            v[16 * k + 4 * j + 2] = q1.v[0];
            v[16 * k + 4 * j + 3] = q1.v[1];
          }
        } else {
#pragma unroll
          for (int i = 0; i < 4; i++)
            v[16 * k + 4 * j + i] = r[i * sx];
        }
      }
  } else {
    const int cx = p.cnt[0], cy = p.cnt[1], cz = p.cnt[2];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int i = 0; i < 4; i++)
          v[16 * k + 4 * j + i] = (i < cx && j < cy && k < cz) ? o[i * sx + j * sy + k * sz] : (S)0;
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int j = 0; j < 4; j++)
        if (k < cz && j < cy) pad_line(v, 16 * k + 4 * j, 1, cx);
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int i = 0; i < 4; i++)
        if (k < cz) pad_line(v, 16 * k + i, 4, cy);
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
      for (int i = 0; i < 4; i++)
        pad_line(v, 4 * j + i, 16, cz);
  }
}

template <typename S, bool VEC>
__device__ __forceinline__ void scatter3(const S (&v)[64], S* __restrict__ base, const Geometry& g, const BlockPos& p)
{
  S* o = base + p.off;
  const int64_t sx = g.s[0], sy = g.s[1], sz = g.s[2];
  if (p.full) {
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        S* r = o + j * sy + k * sz;
        if (VEC) {
          if constexpr (sizeof(S) == 4) {
            Vec16<S, 4> q;
#pragma unroll
            for (int i = 0; i < 4; i++)
              q.v[i] = v[16 * k + 4 * j + i];
            store16<S, 4>(r, q);
          } else {
            Vec16<S, 2> q0, q1;
            q0.v[0] = v[16 * k + 4 * j + 0];
            q0.v[1] = v[16 * k + 4 * j + 1];
            q1.v[0] = v[16 * k + 4 * j + 2];
            q1.v[1] = v[16 * k + 4 * j + 3];
            store16<S, 2>(r, q0);
            store16<S, 2>(r + 2, q1);
          }
        } else {
#pragma unroll
          for (int i = 0; i < 4; i++)
            r[i * sx] = v[16 * k + 4 * j + i];
        }
      }
  } else {
    const int cx = p.cnt[0], cy = p.cnt[1], cz = p.cnt[2];
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int j = 0; j < 4; j++)
#pragma unroll
        for (int i = 0; i < 4; i++)
          if (i < cx && j < cy && k < cz) o[i * sx + j * sy + k * sz] = v[16 * k + 4 * j + i];
  }
}

// ---- coefficient order + negabinary, then bit planes ----
// Negabinary: nb_planes / transpose32_nb (codec_dev.h).
// Planes as two 32-bit halves: Pl[k] bit i = plane k of coefficient i (i < 32),
// Ph[k] bit i = plane k of coefficient 32 + i.  P3: q is in raster order and is
// read through kPerm3 (3D); false: q is already in coding order (a 4D lane's
// segment, block4.h).
template <bool P3 = true>
__device__ __forceinline__ void planes_from_coeffs(uint32_t (&Pl)[32], uint32_t (&Ph)[32], const int32_t (&q)[64])
{
#pragma unroll
  for (int i = 0; i < 32; i++) {
    Pl[i] = nb_planes((uint32_t)q[P3 ? kPerm3[i] : i] + 0xaaaaaaaau);
    Ph[i] = nb_planes((uint32_t)q[P3 ? kPerm3[i + 32] : i + 32] + 0xaaaaaaaau);
  }
  transpose32_nb(Pl);
  transpose32_nb(Ph);
}

// double: planes 32..63 from the high words; 0..31 only when `need_low`
template <bool P3 = true>
__device__ __forceinline__ void planes_from_coeffs(uint32_t (&Pl)[64], uint32_t (&Ph)[64], const int64_t (&q)[64],
                                                   bool need_low)
{
  uint32_t a[32], b[32];
#pragma unroll
  for (int i = 0; i < 32; i++) {
    uint64_t u0 = nb_planes((uint64_t)q[P3 ? kPerm3[i] : i] + 0xaaaaaaaaaaaaaaaaull);
    uint64_t u1 = nb_planes((uint64_t)q[P3 ? kPerm3[i + 32] : i + 32] + 0xaaaaaaaaaaaaaaaaull);
    a[i] = (uint32_t)(u0 >> 32);
    b[i] = (uint32_t)(u1 >> 32);
  }
  transpose32_nb(a);
  transpose32_nb(b);
#pragma unroll
  for (int k = 0; k < 32; k++) {
    Pl[32 + k] = a[k];
    Ph[32 + k] = b[k];
  }
  if (__any(need_low)) {
#pragma unroll
    for (int i = 0; i < 32; i++) {
      uint64_t u0 = nb_planes((uint64_t)q[P3 ? kPerm3[i] : i] + 0xaaaaaaaaaaaaaaaaull);
      uint64_t u1 = nb_planes((uint64_t)q[P3 ? kPerm3[i + 32] : i + 32] + 0xaaaaaaaaaaaaaaaaull);
      a[i] = (uint32_t)u0;
      b[i] = (uint32_t)u1;
    }
    transpose32_nb(a);
    transpose32_nb(b);
#pragma unroll
    for (int k = 0; k < 32; k++) {
      Pl[k] = a[k];
      Ph[k] = b[k];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 32; k++) {
      Pl[k] = 0;
      Ph[k] = 0;
    }
  }
}

template <bool P3 = true>
__device__ __forceinline__ void coeffs_from_planes(int32_t (&q)[64], const uint64_t (&P)[32])
{
  uint32_t lo[32], hi[32];
#pragma unroll
  for (int k = 0; k < 32; k++) {
    lo[k] = (uint32_t)P[k];
    hi[k] = (uint32_t)(P[k] >> 32);
  }
  transpose32_dnb(lo);
  transpose32_dnb(hi);
#pragma unroll
  for (int i = 0; i < 32; i++) {
    q[P3 ? kPerm3[i] : i] = (int32_t)(lo[i] - 0xaaaaaaaau);
    q[P3 ? kPerm3[i + 32] : i + 32] = (int32_t)(hi[i] - 0xaaaaaaaau);
  }
}

template <bool P3 = true>
__device__ __forceinline__ void coeffs_from_planes(int64_t (&q)[64], const uint64_t (&P)[64], bool need_low)
{
  uint32_t a[32], b[32], c[32], d[32];
#pragma unroll
  for (int k = 0; k < 32; k++) {
    a[k] = (uint32_t)P[32 + k];
    b[k] = (uint32_t)(P[32 + k] >> 32);
  }
  transpose32_dnb(a);
  transpose32_dnb(b);
  if (__any(need_low)) {
#pragma unroll
    for (int k = 0; k < 32; k++) {
      c[k] = (uint32_t)P[k];
      d[k] = (uint32_t)(P[k] >> 32);
    }
    transpose32_dnb(c);
    transpose32_dnb(d);
  } else {
#pragma unroll
    for (int k = 0; k < 32; k++) {
      c[k] = 0xaaaaaaaau;  // zero planes, odd bits inverted
      d[k] = 0xaaaaaaaau;
    }
  }
#pragma unroll
  for (int i = 0; i < 32; i++) {
    uint64_t u0 = ((uint64_t)a[i] << 32) | c[i];
    uint64_t u1 = ((uint64_t)b[i] << 32) | d[i];
    q[P3 ? kPerm3[i] : i] = (int64_t)(u0 - 0xaaaaaaaaaaaaaaaaull);
    q[P3 ? kPerm3[i + 32] : i + 32] = (int64_t)(u1 - 0xaaaaaaaaaaaaaaaaull);
  }
}

// double, planes 32..63 only (the HI coder): Pl[k] = plane 32 + k
template <bool P3 = true>
__device__ __forceinline__ void planes_hi(uint32_t (&Pl)[32], uint32_t (&Ph)[32], const int64_t (&q)[64])
{
#pragma unroll
  for (int i = 0; i < 32; i++) {
    uint64_t u0 = nb_planes((uint64_t)q[P3 ? kPerm3[i] : i] + 0xaaaaaaaaaaaaaaaaull);
    uint64_t u1 = nb_planes((uint64_t)q[P3 ? kPerm3[i + 32] : i + 32] + 0xaaaaaaaaaaaaaaaaull);
    Pl[i] = (uint32_t)(u0 >> 32);
    Ph[i] = (uint32_t)(u1 >> 32);
  }
  transpose32_nb(Pl);
  transpose32_nb(Ph);
}

// twin of planes_hi: coefficients from planes 32..63 (low planes zero)
template <bool P3 = true>
__device__ __forceinline__ void coeffs_from_planes_hi(int64_t (&q)[64], const uint64_t (&P)[32])
{
  uint32_t a[32], b[32];
#pragma unroll
  for (int k = 0; k < 32; k++) {
    a[k] = (uint32_t)P[k];
    b[k] = (uint32_t)(P[k] >> 32);
  }
  transpose32_dnb(a);
  transpose32_dnb(b);
#pragma unroll
  for (int i = 0; i < 32; i++) {
    // low planes zero: (u ^ K) - K has a zero low half and high half a' - K32 (a' = a ^ K32)
    q[P3 ? kPerm3[i] : i] = (int64_t)((uint64_t)(a[i] - 0xaaaaaaaau) << 32);
    q[P3 ? kPerm3[i + 32] : i + 32] = (int64_t)((uint64_t)(b[i] - 0xaaaaaaaau) << 32);
  }
}

__device__ __forceinline__ uint32_t precision3(int emax, const CodecParams& cp)
{
  int p = emax - cp.minexp + 2 * 3 + 2;
  if (p < 0) p = 0;
  return (uint32_t)p < cp.maxprec ? (uint32_t)p : cp.maxprec;
}

// integer part of the block: order, planes, coder (encode.c:260-280).
// Codes from bit `pos` of the slot; returns the end position (<= lim).
// HI (double with maxprec <= 32): only planes 32..63 can be coded (kmin >= 32),
// so the 32-plane coder runs on the high words -- its kmin = 32 - prec is the
// same cut -- and the low planes are never built: half the plane registers.
template <bool PLIM, bool HI = false, typename Int>
__device__ __forceinline__ uint32_t encode_ints3(OrSlot& w, const uint32_t* lut, Int (&q)[64], uint32_t pos,
                                                 uint32_t lim, uint32_t prec)
{
  using S = typename std::conditional<sizeof(Int) == 4, float, double>::type;
  constexpr int PREC = Traits<S>::kIntPrec;
  if constexpr (HI && PREC == 64) {
    uint32_t Pl[32], Ph[32];
    planes_hi(Pl, Ph, q);
    pin_registers(Pl);
    pin_registers(Ph);
    return code_planes<32, PLIM>(w, lut, pos, lim, prec, Pl, Ph);
  } else {
    uint32_t Pl[PREC], Ph[PREC];
    if constexpr (PREC == 32)
      planes_from_coeffs(Pl, Ph, q);
    else
      planes_from_coeffs(Pl, Ph, q, prec > 32);
    pin_registers(Pl);
    pin_registers(Ph);
    return code_planes<PREC, PLIM>(w, lut, pos, lim, prec, Pl, Ph);
  }
}

template <bool HI = false, typename Int>
__device__ __forceinline__ uint32_t decode_ints3(WordReader& r, const uint32_t* sq, Int (&q)[64], uint32_t budget,
                                                 uint32_t prec)
{
  using S = typename std::conditional<sizeof(Int) == 4, float, double>::type;
  constexpr int PREC = Traits<S>::kIntPrec;
  if constexpr (HI && PREC == 64) {
    uint64_t P[32];
    const uint32_t used = decode_planes32<false>(r, sq, budget, prec, P);
    pin_registers(P);
    coeffs_from_planes_hi(q, P);
    return used;
  } else {
    uint64_t P[PREC];
    uint32_t used;
    if constexpr (PREC == 32)
      used = decode_planes32(r, sq, budget, prec, P);
    else
      used = decode_planes64<PREC>(r, sq, budget, prec, P);
    pin_registers(P);
    if constexpr (PREC == 32)
      coeffs_from_planes(q, P);
    else
      coeffs_from_planes(q, P, prec > 32);
    return used;
  }
}

// Block exponent and block-floating-point cast for the lossy encoder.  Fast
// path: the max magnitude comes from integer maxima of the bit patterns (NaN
// sorts above inf, so one compare flags inf/NaN blocks), and for a finite
// block with a finite scale s*x < 2^30 always, so the hardware conversion
// matches C's.  Blocks holding inf/NaN or with a scale that overflows take the
// exact path (NaN-ignoring max, x86 INT_MIN conversions); that branch is
// wave-uniform, taken only if some lane needs it, and re-reads the block
// through `reload` so the inputs are dead after the fast cast (the cast is
// done in place, keeping the register footprint at one block).
template <typename Reload>
__device__ __forceinline__ int lossy_emax_cast(int32_t (&q)[64], float (&v)[64], const CodecParams& cp,
                                               uint32_t& mp, Reload&& reload)
{
  int32_t mi = 0;
  uint32_t mu = 0;
#pragma unroll
  for (int i = 0; i < 64; i++) {
    const uint32_t b = __float_as_uint(v[i]);
    mi = max(mi, (int32_t)b);
    mu = max(mu, b);
  }
  const uint32_t mb = max((uint32_t)mi, mu & 0x7fffffffu);
  int emax = mb == 0 ? -127 : ((mb >> 23) == 0 ? -126 : (int)(mb >> 23) - 126);
  const bool bad = mb >= 0x7f800000u;
  if (bad)
    emax = block_emax(block_absmax(v));
  mp = precision3(emax, cp);
  const bool cast = mp != 0 && emax != -127;
  const float s = __uint_as_float((uint32_t)(157 - emax) << 23);
#pragma unroll
  for (int i = 0; i < 64; i++)
    q[i] = (int32_t)(s * v[i]);
  if (__any(cast && (bad || emax < -97))) {
    float w[64];
    reload(w);
    fwd_cast(q, w, emax);
  }
  return emax;
}

template <typename Reload>
__device__ __forceinline__ int lossy_emax_cast(int64_t (&q)[64], double (&v)[64], const CodecParams& cp,
                                               uint32_t& mp, Reload&&)
{
  const int emax = block_emax(block_absmax(v));
  mp = precision3(emax, cp);
  fwd_cast(q, v, emax);
  return emax;
}

// Scheduling fence between the phases of a block (cast, lift, planes, coder):
// without it the scheduler interleaves neighbouring phases, which keeps both
// phases' registers live and costs occupancy.
#if defined(__HIP_DEVICE_COMPILE__)
#define ZFP_PHASE_BARRIER() __builtin_amdgcn_sched_barrier(0)
#else
#define ZFP_PHASE_BARRIER() ((void)0)
#endif

// Fixed-rate block (maxprec >= intprec, minbits == maxbits): encodef.c:63-90 +
// encode.c:260-280 with every lane on one control path.  An all-zero block
// (e == 0: the single bit "0", then padding) runs the transform and the coder
// like the others with its position pinned at the budget end, so its bits all
// land in the slot's spare words and its block stays "0" + zeros.  `mid` runs
// once the block's bit planes are built and the field values are dead: the
// pipelined kernel issues the next batch's loads there, so they fly during the
// coder.
template <typename S, typename Reload, typename Mid>
__device__ __forceinline__ void encode_block3_fixed(OrSlot& w, const uint32_t* lut, S (&v)[64], const CodecParams& cp,
                                                    Reload&& reload, Mid&& mid)
{
  using T = Traits<S>;
  using Int = typename T::Int;
  constexpr int PREC = T::kIntPrec;
  constexpr uint32_t kE = T::kEbits;
  Int q[64];
  uint32_t mp;
  const int emax = lossy_emax_cast(q, v, cp, mp, reload);
  const uint32_t e = mp ? (uint32_t)(emax + T::kEbias) : 0u;
  if (e)
    w.head(2 * e + 1);
  ZFP_PHASE_BARRIER();
  xform<3, false, false>(q);
  ZFP_PHASE_BARRIER();
  uint32_t Pl[PREC], Ph[PREC];
  if constexpr (PREC == 32)
    planes_from_coeffs(Pl, Ph, q);
  else
    planes_from_coeffs(Pl, Ph, q, true);
  ZFP_PHASE_BARRIER();
  pin_registers(Pl);
  pin_registers(Ph);
  mid();
  if constexpr (PREC == 32)  // lut: dbl[256] then lead[256] (CoderTables)
    code_planes_fr32(w.d(), w.jmax, lut, e ? 1 + kE : cp.maxbits, cp.maxbits, Pl, Ph);
  else
    code_planes<PREC, false>(w, lut, e ? 1 + kE : cp.maxbits, cp.maxbits, mp, Pl, Ph);
}

// Encode one block into a zeroed slot; returns its length in bits including
// minbits padding (padding bits are the slot's zeros).  FR: fixed rate with
// maxprec >= intprec (no per-block precision limit; see code_planes).
template <typename S, bool REV, bool FR = false, bool HI = false, typename Reload>
__device__ __forceinline__ uint32_t encode_block3(OrSlot& w, const uint32_t* lut, S (&v)[64], const CodecParams& cp,
                                                  Reload&& reload)
{
  using T = Traits<S>;
  using Int = typename T::Int;
  using UInt = typename T::UInt;
  constexpr uint32_t kE = T::kEbits;
  Int q[64];
  if constexpr (REV) {
    // reversible (revencodef.c:45-80)
    int emax = block_emax(block_absmax(v));
    // bitwise accumulation: a short-circuit && becomes 64 nested lane branches
    decltype(bits_of(v[0])) sdiff = 0;
    bool same;
    if (emax != -T::kEbias) {
      fwd_cast(q, v, emax);
      S s = (sizeof(S) == 4) ? (S)pow2f(emax - 30) : (S)pow2d(emax - 62);
#pragma unroll
      for (int i = 0; i < 64; i++) {
        sdiff |= bits_of((S)(s * (S)q[i])) ^ bits_of(v[i]);
        if ((i & 3) == 3)
          pin_value(sdiff);  // accumulated in order (not as a tree of 64 live terms)
      }
    } else {
#pragma unroll
      for (int i = 0; i < 64; i++) {
        q[i] = 0;
        sdiff |= bits_of(v[i]);
      }
    }
    same = sdiff == 0;
    uint32_t bits;
    if (same) {
      uint32_t e = (uint32_t)(emax + T::kEbias);
      if (!e) {
        // a single 0 bit (already zero in the slot)
        return 1u < cp.minbits ? cp.minbits : 1u;
      }
      w.head(1u | (e << 2));
      bits = 2 + kE;
    } else {
#pragma unroll
      for (int i = 0; i < 64; i++) {
        const Int x = (Int)bits_of(v[i]);
        q[i] = x < 0 ? (Int)((UInt)x ^ T::kTcMask) : x;
        if ((i & 3) == 3)
          ZFP_SCHED_FENCE();
      }
      w.head(3u);
      bits = 2;
    }
    // rev_encode_block_<Int> (revencode.c:54-76)
    const uint32_t minb = cp.minbits - (bits < cp.minbits ? bits : cp.minbits);
    xform<3, false, true>(q);
    UInt all = 0;
#pragma unroll
    for (int i = 0; i < 64; i++)
      all |= ((UInt)q[i] + T::kNbMask) ^ T::kNbMask;
    uint32_t prec = all ? (uint32_t)(T::kIntPrec - (sizeof(S) == 4 ? __builtin_ctz((uint32_t)all)
                                                                    : __builtin_ctzll((uint64_t)all)))
                        : 0u;
    if (prec > cp.maxprec) prec = cp.maxprec;
    if (prec < 1) prec = 1;
    w.put32(bits, prec - 1);
    const uint32_t end = encode_ints3<true, HI>(w, lut, q, bits + T::kPbits, cp.maxbits, prec);
    uint32_t ib = end - bits;
    if (ib < minb) ib = minb;
    return bits + ib;
  } else {
    // lossy (encodef.c:63-90)
    if constexpr (FR && !HI) {
      encode_block3_fixed(w, lut, v, cp, reload, [] {});
      return cp.maxbits;
    }
    uint32_t mp;
    const int emax = lossy_emax_cast(q, v, cp, mp, reload);
    const uint32_t e = mp ? (uint32_t)(emax + T::kEbias) : 0u;
    uint32_t bits = 1;
    if (e) {
      w.head(2 * e + 1);
      bits += kE;
      xform<3, false, false>(q);
      const uint32_t minb = cp.minbits - (bits < cp.minbits ? bits : cp.minbits);
      uint32_t ib = encode_ints3<!FR, HI>(w, lut, q, bits, cp.maxbits, mp) - bits;
      if (ib < minb) ib = minb;
      bits += ib;
    } else if (cp.minbits > bits) {
      bits = cp.minbits;
    }
    return bits;
  }
}

// Decode one block; returns the number of bits consumed (incl. padding).
template <typename S, bool REV, bool HI = false>
__device__ __forceinline__ uint32_t decode_block3(WordReader& r, const uint32_t* sq, S (&v)[64], const CodecParams& cp)
{
  using T = Traits<S>;
  using Int = typename T::Int;
  using UInt = typename T::UInt;
  constexpr uint32_t kE = T::kEbits;
  Int q[64];
  if constexpr (REV) {
    uint32_t bits = 1;
    if (!r.read1()) {
#pragma unroll
      for (int i = 0; i < 64; i++) v[i] = 0;
      if (cp.minbits > bits) {
        r.skip(cp.minbits - bits);
        bits = cp.minbits;
      }
      return bits;
    }
    bits++;
    bool reinterp = r.read1() != 0;
    int emax = 0;
    if (!reinterp) {
      bits += kE;
      emax = (int)r.read(kE) - T::kEbias;
    }
    uint32_t minb = cp.minbits - (bits < cp.minbits ? bits : cp.minbits);
    uint32_t maxb = cp.maxbits - bits;
    uint32_t prec = (uint32_t)r.read(T::kPbits) + 1;
    uint32_t ib = T::kPbits + decode_ints3<HI>(r, sq, q, maxb - T::kPbits, prec);
    if (ib < minb) {
      r.skip(minb - ib);
      ib = minb;
    }
    xform<3, true, true>(q);
    if (reinterp) {
#pragma unroll
      for (int i = 0; i < 64; i++) {
        Int x = q[i] < 0 ? (Int)((UInt)q[i] ^ T::kTcMask) : q[i];
        if constexpr (sizeof(S) == 4)
          v[i] = __uint_as_float((uint32_t)x);
        else
          v[i] = __longlong_as_double((long long)x);
      }
    } else if (emax != -T::kEbias) {
      inv_cast(v, q, emax);
    } else {
#pragma unroll
      for (int i = 0; i < 64; i++) v[i] = 0;
    }
    return bits + ib;
  } else {
  uint32_t bits = 1;
  if (r.read1()) {
    bits += kE;
    int emax = (int)r.read(kE) - T::kEbias;
    uint32_t mp = precision3(emax, cp);
    uint32_t minb = cp.minbits - (bits < cp.minbits ? bits : cp.minbits);
    uint32_t ib = decode_ints3<HI>(r, sq, q, cp.maxbits - bits, mp);
    if (ib < minb) {
      r.skip(minb - ib);
      ib = minb;
    }
    bits += ib;
    xform<3, true, false>(q);
    inv_cast(v, q, emax);
  } else {
#pragma unroll
    for (int i = 0; i < 64; i++) v[i] = 0;
    if (cp.minbits > bits) {
      r.skip(cp.minbits - bits);
      bits = cp.minbits;
    }
  }
  return bits;
  }
}

}  // namespace zfp_amd
