// Per-lane codec for the instantiations the 3D/4D float kernels do not cover
// (SURVEY §8 f3): 1D and 2D blocks of every scalar type and 3D integer blocks
// -- one 4^d-value block per lane, d = 1..3, float, double, int32, int64.
//
// encode_block_n: float lossy encodef.c:63-90, float reversible
//                 revencodef.c:45-80, integer lossy encode.c:260-280 (no
//                 header: the integers are coded as they are), integer
//                 reversible revencode.c:54-76 (precision header only).
// decode_block_n: decodef.c:7-36, revdecodef.c:22-59, decode.c:271-287,
//                 revdecode.c:34-52.
// gather_n / scatter_n: encode1.c / encode2.c / encode3.c gather with the pad
//                 rule of encode.c:9-27, decode{1,2,3}.c scatter.
//
// The stages are the 3D codec's (block3.h, codec_dev.h) with the block size
// as a parameter: lifting xform<D>, order tables kPerm1/kPerm2/kPerm3, bit
// planes by 32x32 transposes (coefficients past the block are zero), and the
// closed-form coder / decoder with SIZE = 4^d.  These kernels are not tuned:
// they exist so that every field type the reference accepts runs on the GPU.
#pragma once

#include <type_traits>

#include "block3.h"

namespace zfp_amd {

template <typename S>
constexpr bool kIntField = std::is_integral<S>::value;

template <int D>
__device__ __forceinline__ int perm_n(int i)
{
  return D == 1 ? kPerm1[i] : D == 2 ? kPerm2[i] : kPerm3[i];
}

// gather of a 4^D block (x fastest) with partial-block padding
template <typename S, int D>
__device__ __forceinline__ void gather_n(S (&v)[64], const S* __restrict__ base, const Geometry& g, const BlockPos& p)
{
  constexpr int N = 1 << (2 * D);
  const S* o = base + p.off;
  const int64_t sx = g.s[0], sy = D > 1 ? g.s[1] : 0, sz = D > 2 ? g.s[2] : 0;
  const int cx = p.cnt[0], cy = D > 1 ? p.cnt[1] : 1, cz = D > 2 ? p.cnt[2] : 1;
#pragma unroll
  for (int idx = 0; idx < N; idx++) {
    const int i = idx & 3, j = (idx >> 2) & 3, k = idx >> 4;
    v[idx] = (i < cx && j < cy && k < cz) ? o[i * sx + j * sy + k * sz] : (S)0;
  }
  if (p.full)
    return;
#pragma unroll
  for (int k = 0; k < (D > 2 ? 4 : 1); k++)
#pragma unroll
    for (int j = 0; j < (D > 1 ? 4 : 1); j++)
      if (k < cz && j < cy) pad_line(v, 16 * k + 4 * j, 1, cx);
  if constexpr (D > 1) {
#pragma unroll
    for (int k = 0; k < (D > 2 ? 4 : 1); k++)
#pragma unroll
      for (int i = 0; i < 4; i++)
        if (k < cz) pad_line(v, 16 * k + i, 4, cy);
  }
  if constexpr (D > 2) {
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
      for (int i = 0; i < 4; i++)
        pad_line(v, 4 * j + i, 16, cz);
  }
}

template <typename S, int D>
__device__ __forceinline__ void scatter_n(const S (&v)[64], S* __restrict__ base, const Geometry& g,
                                          const BlockPos& p)
{
  constexpr int N = 1 << (2 * D);
  S* o = base + p.off;
  const int64_t sx = g.s[0], sy = D > 1 ? g.s[1] : 0, sz = D > 2 ? g.s[2] : 0;
  const int cx = p.cnt[0], cy = D > 1 ? p.cnt[1] : 1, cz = D > 2 ? p.cnt[2] : 1;
#pragma unroll
  for (int idx = 0; idx < N; idx++) {
    const int i = idx & 3, j = (idx >> 2) & 3, k = idx >> 4;
    if (i < cx && j < cy && k < cz) o[i * sx + j * sy + k * sz] = v[idx];
  }
}

// the first N entries of a 64-entry register array as an N-entry array
template <int N, typename U>
__device__ __forceinline__ U (&head_n(U (&a)[64]))[N]
{
  return *reinterpret_cast<U(*)[N]>(&a[0]);
}

// bit planes of the N coefficients in coding order (negabinary; odd planes
// inverted in the transpose, see nb_planes): Pl/Ph[k] = plane k of
// coefficients 0..31 / 32..63 (zero past N)
template <int D, typename Int, int PREC>
__device__ __forceinline__ void planes_n(uint32_t (&Pl)[PREC], uint32_t (&Ph)[PREC], const Int (&q)[64])
{
  constexpr int N = 1 << (2 * D);
  using UInt = typename std::make_unsigned<Int>::type;
  constexpr UInt K = (UInt)0xaaaaaaaaaaaaaaaaull;
  if constexpr (PREC == 32) {
#pragma unroll
    for (int i = 0; i < 32; i++)
      Pl[i] = nb_planes((uint32_t)(i < N ? q[perm_n<D>(i < N ? i : 0)] : 0) + (uint32_t)K);
    transpose32_nb(Pl);
#pragma unroll
    for (int i = 0; i < 32; i++)
      Ph[i] = nb_planes((uint32_t)(i + 32 < N ? q[perm_n<D>(i + 32 < N ? i + 32 : 0)] : 0) + (uint32_t)K);
    transpose32_nb(Ph);
  } else {
    uint32_t a[32], b[32];
#pragma unroll
    for (int half = 0; half < 2; half++) {  // coefficients 0..31, then 32..63
#pragma unroll
      for (int i = 0; i < 32; i++) {
        const int c = 32 * half + i;
        const uint64_t u = nb_planes((uint64_t)(c < N ? q[perm_n<D>(c < N ? c : 0)] : 0) + (uint64_t)K);
        a[i] = (uint32_t)u;          // planes 0..31
        b[i] = (uint32_t)(u >> 32);  // planes 32..63
      }
      transpose32_nb(a);
      transpose32_nb(b);
#pragma unroll
      for (int k = 0; k < 32; k++) {
        if (half == 0) {
          Pl[k] = a[k];
          Pl[32 + k] = b[k];
        } else {
          Ph[k] = a[k];
          Ph[32 + k] = b[k];
        }
      }
    }
  }
}

// inverse: planes P[k] (bit i = plane k of coefficient i) -> coefficients
template <int D, typename Int, int PREC>
__device__ __forceinline__ void coeffs_n(Int (&q)[64], const uint64_t (&P)[PREC])
{
  constexpr int N = 1 << (2 * D);
  using UInt = typename std::make_unsigned<Int>::type;
  constexpr UInt K = (UInt)0xaaaaaaaaaaaaaaaaull;
#pragma unroll
  for (int half = 0; half < (N > 32 ? 2 : 1); half++) {
    uint32_t a[32], b[32];
#pragma unroll
    for (int k = 0; k < 32; k++) {
      a[k] = (uint32_t)(P[k] >> (32 * half));
      b[k] = PREC == 64 ? (uint32_t)(P[PREC == 64 ? 32 + k : k] >> (32 * half)) : 0u;
    }
    transpose32(a);
    if (PREC == 64)
      transpose32(b);
#pragma unroll
    for (int i = 0; i < 32; i++) {
      const int c = 32 * half + i;
      if (c < N) {
        const UInt u = PREC == 64 ? (UInt)(((uint64_t)b[i] << 32) | a[i]) : (UInt)a[i];
        q[perm_n<D>(c)] = (Int)((u ^ K) - K);
      }
    }
  }
}

__device__ __forceinline__ uint32_t precision_n(int emax, const CodecParams& cp, int d)
{
  int p = emax - cp.minexp + 2 * (d + 1);  // encodef.c:49-54
  if (p < 0) p = 0;
  return (uint32_t)p < cp.maxprec ? (uint32_t)p : cp.maxprec;
}

// integer part: order + planes + coder from slot bit `pos` (budget end `lim`)
template <int D, typename Int>
__device__ __forceinline__ uint32_t encode_ints_n(OrSlot& w, const uint32_t* lut, const Int (&q)[64], uint32_t pos,
                                                  uint32_t lim, uint32_t prec)
{
  constexpr int PREC = 8 * sizeof(Int);
  uint32_t Pl[PREC], Ph[PREC];
  planes_n<D, Int, PREC>(Pl, Ph, q);
  return code_planes<PREC, true, 1 << (2 * D)>(w, lut, pos, lim, prec, Pl, Ph);
}

template <int D, typename Int>
__device__ __forceinline__ uint32_t decode_ints_n(WordReader& r, const uint32_t* sq, Int (&q)[64], uint32_t budget,
                                                  uint32_t prec)
{
  constexpr int PREC = 8 * sizeof(Int);
  uint64_t P[PREC];
  const uint32_t used = decode_planes64<PREC, true, 1 << (2 * D)>(r, sq, budget, prec, P);
  coeffs_n<D, Int, PREC>(q, P);
  return used;
}

// Encode one block into a zeroed slot (the slot may be written at bit 0, so
// the dword before it must be writable: it only ever receives zero bits);
// returns its length in bits including minbits padding.
template <typename S, int D, bool REV>
__device__ __forceinline__ uint32_t encode_block_n(OrSlot& w, const uint32_t* lut, S (&v)[64], const CodecParams& cp)
{
  using T = Traits<S>;
  using Int = typename T::Int;
  using UInt = typename T::UInt;
  constexpr int N = 1 << (2 * D);
  constexpr uint32_t kE = T::kEbits;
  Int q[64];
  uint32_t bits = 0;  // header bits
  uint32_t prec;
  if constexpr (kIntField<S>) {
#pragma unroll
    for (int i = 0; i < N; i++)
      q[i] = (Int)v[i];
    if constexpr (!REV) {
      // encode.c:260-280: transform, order, coder, padding
      xform<D, false, false>(head_n<N>(q));
      uint32_t ib = encode_ints_n<D>(w, lut, q, 0, cp.maxbits, cp.maxprec);
      return ib < cp.minbits ? cp.minbits : ib;
    }
  } else if constexpr (!REV) {
    // encodef.c:63-90
    S m = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const S a = sizeof(S) == 4 ? (S)fabsf((float)v[i]) : (S)fabs((double)v[i]);
      m = (m < a) ? a : m;  // NaN never wins
    }
    const int emax = block_emax(m);
    const uint32_t mp = precision_n(emax, cp, D);
    const uint32_t e = mp ? (uint32_t)(emax + T::kEbias) : 0u;
    bits = 1;
    if (!e)
      return cp.minbits > bits ? cp.minbits : bits;  // a single 0 bit (the slot is zero)
    w.head(2 * e + 1);
    bits += kE;
    fwd_cast(head_n<N>(q), head_n<N>(v), emax);
    xform<D, false, false>(head_n<N>(q));
    const uint32_t minb = cp.minbits - (bits < cp.minbits ? bits : cp.minbits);
    uint32_t ib = encode_ints_n<D>(w, lut, q, bits, cp.maxbits, mp) - bits;
    if (ib < minb) ib = minb;
    return bits + ib;
  } else {
    // revencodef.c:45-80: lossless block-floating-point, else the bit patterns
    S m = 0;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const S a = sizeof(S) == 4 ? (S)fabsf((float)v[i]) : (S)fabs((double)v[i]);
      m = (m < a) ? a : m;
    }
    const int emax = block_emax(m);
    // bitwise accumulation: a short-circuit && becomes 64 nested lane branches
    decltype(bits_of(v[0])) sdiff = 0;
    bool same;
    if (emax != -T::kEbias) {
      fwd_cast(head_n<N>(q), head_n<N>(v), emax);
      const S s = (sizeof(S) == 4) ? (S)pow2f(emax - 30) : (S)pow2d(emax - 62);
#pragma unroll
      for (int i = 0; i < N; i++)
        sdiff |= bits_of((S)(s * (S)q[i])) ^ bits_of(v[i]);
    } else {
#pragma unroll
      for (int i = 0; i < N; i++) {
        q[i] = 0;
        sdiff |= bits_of(v[i]);
      }
    }
    same = sdiff == 0;
    if (same) {
      const uint32_t e = (uint32_t)(emax + T::kEbias);
      if (!e)
        return 1u < cp.minbits ? cp.minbits : 1u;  // a single 0 bit
      w.head(1u | (e << 2));
      bits = 2 + kE;
    } else {
#pragma unroll
      for (int i = 0; i < N; i++) {
        const Int x = (Int)bits_of(v[i]);
        q[i] = x < 0 ? (Int)((UInt)x ^ T::kTcMask) : x;
      }
      w.head(3u);
      bits = 2;
    }
  }
  // reversible integer part (revencode.c:54-76) after `bits` header bits
  xform<D, false, true>(head_n<N>(q));
  UInt all = 0;
#pragma unroll
  for (int i = 0; i < N; i++)
    all |= ((UInt)q[i] + T::kNbMask) ^ T::kNbMask;
  prec = all ? (uint32_t)(T::kIntPrec - (sizeof(Int) == 4 ? __builtin_ctz((uint32_t)all)
                                                            : __builtin_ctzll((uint64_t)all)))
             : 0u;
  if (prec > cp.maxprec) prec = cp.maxprec;
  if (prec < 1) prec = 1;
  if (bits)
    w.put32(bits, prec - 1);
  else
    w.head(prec - 1);
  const uint32_t minb = cp.minbits - (bits < cp.minbits ? bits : cp.minbits);
  uint32_t ib = encode_ints_n<D>(w, lut, q, bits + T::kPbits, cp.maxbits, prec) - bits;
  if (ib < minb) ib = minb;
  return bits + ib;
}

// Decode one block; returns the number of bits consumed (incl. padding).
template <typename S, int D, bool REV>
__device__ __forceinline__ uint32_t decode_block_n(WordReader& r, const uint32_t* sq, S (&v)[64],
                                                   const CodecParams& cp)
{
  using T = Traits<S>;
  using Int = typename T::Int;
  using UInt = typename T::UInt;
  constexpr int N = 1 << (2 * D);
  constexpr uint32_t kE = T::kEbits;
  Int q[64];
  if constexpr (kIntField<S> && !REV) {
    // decode.c:271-287
    uint32_t ib = decode_ints_n<D>(r, sq, q, cp.maxbits, cp.maxprec);
    if (ib < cp.minbits) {
      r.skip(cp.minbits - ib);
      ib = cp.minbits;
    }
    xform<D, true, false>(head_n<N>(q));
#pragma unroll
    for (int i = 0; i < N; i++)
      v[i] = (S)q[i];
    return ib;
  } else if constexpr (kIntField<S>) {
    // revdecode.c:34-52
    const uint32_t prec = (uint32_t)r.read(T::kPbits) + 1;
    uint32_t bits = T::kPbits + decode_ints_n<D>(r, sq, q, cp.maxbits - T::kPbits, prec);
    if (bits < cp.minbits) {
      r.skip(cp.minbits - bits);
      bits = cp.minbits;
    }
    xform<D, true, true>(head_n<N>(q));
#pragma unroll
    for (int i = 0; i < N; i++)
      v[i] = (S)q[i];
    return bits;
  } else if constexpr (!REV) {
    // decodef.c:7-36
    uint32_t bits = 1;
    if (!r.read1()) {
#pragma unroll
      for (int i = 0; i < N; i++) v[i] = 0;
      if (cp.minbits > bits) {
        r.skip(cp.minbits - bits);
        bits = cp.minbits;
      }
      return bits;
    }
    bits += kE;
    const int emax = (int)r.read(kE) - T::kEbias;
    const uint32_t mp = precision_n(emax, cp, D);
    const uint32_t minb = cp.minbits - (bits < cp.minbits ? bits : cp.minbits);
    uint32_t ib = decode_ints_n<D>(r, sq, q, cp.maxbits - bits, mp);
    if (ib < minb) {
      r.skip(minb - ib);
      ib = minb;
    }
    xform<D, true, false>(head_n<N>(q));
    inv_cast(head_n<N>(v), head_n<N>(q), emax);
    return bits + ib;
  } else {
    // revdecodef.c:22-59
    uint32_t bits = 1;
    if (!r.read1()) {
#pragma unroll
      for (int i = 0; i < N; i++) v[i] = 0;
      if (cp.minbits > bits) {
        r.skip(cp.minbits - bits);
        bits = cp.minbits;
      }
      return bits;
    }
    bits++;
    const bool reinterp = r.read1() != 0;
    int emax = 0;
    if (!reinterp) {
      bits += kE;
      emax = (int)r.read(kE) - T::kEbias;
    }
    const uint32_t minb = cp.minbits - (bits < cp.minbits ? bits : cp.minbits);
    const uint32_t maxb = cp.maxbits - bits;
    const uint32_t prec = (uint32_t)r.read(T::kPbits) + 1;
    uint32_t ib = T::kPbits + decode_ints_n<D>(r, sq, q, maxb - T::kPbits, prec);
    if (ib < minb) {
      r.skip(minb - ib);
      ib = minb;
    }
    xform<D, true, true>(head_n<N>(q));
    if (reinterp) {
#pragma unroll
      for (int i = 0; i < N; i++) {
        const Int x = q[i] < 0 ? (Int)((UInt)q[i] ^ T::kTcMask) : q[i];
        if constexpr (sizeof(S) == 4)
          v[i] = __uint_as_float((uint32_t)x);
        else
          v[i] = __longlong_as_double((long long)x);
      }
    } else if (emax != -T::kEbias) {
      inv_cast(head_n<N>(v), head_n<N>(q), emax);
    } else {
#pragma unroll
      for (int i = 0; i < N; i++) v[i] = 0;
    }
    return bits + ib;
  }
}

}  // namespace zfp_amd
