// Per-quad codec of one 4x4x4x4 block (float or double) for every zfp mode.
//
// The four lanes of a quad (lanes 4q .. 4q+3, 16 blocks per wave) share a
// block.  Lane r holds
//   * up to the w-lift: the 3D slice w = r (64 values, raster x + 4y + 16z),
//     so gather, block-floating-point cast and the x, y, z lifts are the 3D
//     per-lane code (block3.h);
//   * after the w-lift and the reordering: the coefficients of coding order
//     64r .. 64r+63 (codec4.c perm_4), i.e. bits [64r, 64r+64) of every
//     256-bit bit plane -- the 3D plane representation (Pl/Ph halves), per lane.
// The w-lift and the reordering go through a per-block LDS exchange area.
// Block-wide values (max, OR, prefix sums over the four plane segments) are
// quad reductions on DPP quad permutes, so every branch on them is
// quad-uniform.
//
// encode_block4: encodef.c:63-90, revencodef.c:45-80, encode.c:136-175 and
//                208-234 (encode_many_ints[_prec]), transform encode4.c:40-65,
//                gather/pad encode4.c:4-38.
// decode_block4: decodef.c:7-36, revdecodef.c:22-59, decode.c:122-173 and
//                212-246, inverse transform decode4.c:27-52.
#pragma once

#include <type_traits>

#include "block3.h"

namespace zfp_amd {

// ---------------------------------------------------------------------------
// quad permutes: DPP quad_perm, lane i of each quad reads lane sel_i
// (ctrl = sel_0 | sel_1 << 2 | sel_2 << 4 | sel_3 << 6).  Called only where the
// whole quad is active.  bound_ctrl (no source lane of a quad_perm is ever
// invalid, so it changes nothing) lets the compiler fold the permute into the
// instruction that consumes it (v_max_u32_dpp, v_add_u32_dpp).
template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t x)
{
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xf, 0xf, true);
}

template <int CTRL>
__device__ __forceinline__ uint64_t qperm(uint64_t x)
{
  return ((uint64_t)qperm<CTRL>((uint32_t)(x >> 32)) << 32) | qperm<CTRL>((uint32_t)x);
}

constexpr int kQSwap1 = 0xb1;  // [1,0,3,2]
constexpr int kQSwap2 = 0x4e;  // [2,3,0,1]

template <typename U>
__device__ __forceinline__ U quad_max(U x)
{
  U y = qperm<kQSwap1>(x);
  x = x > y ? x : y;
  y = qperm<kQSwap2>(x);
  return x > y ? x : y;
}

template <typename U>
__device__ __forceinline__ U quad_or(U x)
{
  x |= qperm<kQSwap1>(x);
  return x | qperm<kQSwap2>(x);
}

// exclusive prefix sum over the quad; `total` receives the quad's sum.  Pair
// sums s01 (lanes 0,1: x0 + x1; lanes 2,3: x2 + x3), the total from the two
// pair sums, and lane r's prefix as (odd r: x of lane r-1) + (r >= 2: s01 of
// lane 0), the lane selections as AND masks: five VALU, each permute folded
// into its instruction (v_add_u32_dpp, v_and_b32_dpp).
__device__ __forceinline__ uint32_t quad_excl(uint32_t x, uint32_t& total, uint32_t m_odd, uint32_t m_hi)
{
  const uint32_t s01 = x + qperm<0xb1>(x);  // [1,0,3,2]
  total = s01 + qperm<0x4e>(s01);           // [2,3,0,1]
  return (qperm<0xa0>(x) & m_odd) + (qperm<0x00>(s01) & m_hi);  // [0,0,2,2], [0,0,0,0]
}

// the lane masks of quad_excl: m_odd = ~0 on lanes 1 and 3, m_hi = ~0 on lanes
// 2 and 3 (opaque to the compiler, which would otherwise turn the ANDs into
// selects and keep the permutes apart)
__device__ __forceinline__ void quad_excl_masks(uint32_t& m_odd, uint32_t& m_hi)
{
  const uint32_t r = threadIdx.x & 3u;
  m_odd = 0u - (r & 1u);
  m_hi = 0u - (r >> 1);
  pin_value(m_odd);
  pin_value(m_hi);
}

__device__ __forceinline__ uint32_t quad_excl(uint32_t x, uint32_t& total)
{
  uint32_t m_odd, m_hi;
  quad_excl_masks(m_odd, m_hi);
  return quad_excl(x, total, m_odd, m_hi);
}

// block max |x| (NaN ignored) over the quad's four slices
template <typename S>
__device__ __forceinline__ S quad_absmax(const S (&v)[64])
{
  const S m = block_absmax(v);  // >= +0, never NaN: ordered like its bit pattern
  if constexpr (sizeof(S) == 4)
    return __uint_as_float(quad_max(__float_as_uint(m)));
  else
    return __longlong_as_double((long long)quad_max((uint64_t)__double_as_longlong(m)));
}

// ---------------------------------------------------------------------------
// Gather / scatter of lane r's slice.  A partial block is padded along w by
// reading the slice the pad rule copies (encode.c:9-27: nw = 1 -> all from
// w = 0; nw = 2 -> w2 = w1, w3 = w0; nw = 3 -> w3 = w0); x, y, z padding is the
// 3D gather's.
__device__ __forceinline__ int pad_src_w(int r, int nw)
{
  return r < nw ? r : ((r == 2 && nw == 2) ? 1 : 0);
}

__device__ __forceinline__ BlockPos slice_pos(const Geometry& g, const BlockPos& p, int w)
{
  BlockPos s = p;
  s.off = p.off + (int64_t)w * g.s[3];
  s.full = p.cnt[0] == 4 && p.cnt[1] == 4 && p.cnt[2] == 4;
  return s;
}

// ---------------------------------------------------------------------------
// Exchange area of a block: entry 4 pos + w holds value (pos, w), pos =
// x + 4y + 16z.  Blocks are kXStride entries apart: 260 = 4 (mod 64), so the 64
// lanes' slice writes of one pos hit 64 distinct banks (float).
constexpr uint32_t kXStride = 260;

// Order table: dword k packs the exchange entries of coding-order indices
// 4k .. 4k+3, one byte each (perm_4 of codec4.c via kPerm4).
struct OrderTab4 {
  uint32_t t[64];
};

constexpr OrderTab4 make_order_tab4()
{
  OrderTab4 o{};
  for (int k = 0; k < 64; k++) {
    uint32_t t = 0;
    for (int i = 0; i < 4; i++) {
      const uint32_t c = kPerm4[4 * k + i];
      t |= ((c & 63u) * 4u + (c >> 6)) << (8 * i);
    }
    o.t[k] = t;
  }
  return o;
}

__constant__ OrderTab4 kOrderTab4 = make_order_tab4();

// forward: slices (after the x, y, z lifts) -> w-lift (encode4.c:60-64) ->
// lane r gets the coefficients of coding order 64r .. 64r+63.  Called by the
// whole wave (one 64-thread workgroup).  HALF: the exchange areas of quads
// q and q + 8 coincide (X at (q & 7) * kXStride) and the two halves of the
// wave take turns, halving the LDS the exchange needs.
template <bool REV, bool HALF = false, typename Int>
__device__ __forceinline__ void exchange_fwd(Int (&q)[64], Int* X, const uint32_t* tab)
{
  const uint32_t r = threadIdx.x & 3u;
  const uint32_t mine_h = (threadIdx.x >> 5) & 1u;
#pragma unroll
  for (uint32_t h = 0; h < (HALF ? 2u : 1u); h++) {
    const bool mine = !HALF || mine_h == h;
    if (mine) {
#pragma unroll
      for (int i = 0; i < 64; i++)
        X[4 * i + r] = q[i];
    }
    __syncthreads();
    if (mine) {
#pragma unroll
      for (int j = 0; j < 16; j++) {
        Int* e = X + 4 * (16 * r + j);
        Int a = e[0], b = e[1], c = e[2], d = e[3];
        if (REV) Lift<Int>::rfwd(a, b, c, d);
        else Lift<Int>::fwd(a, b, c, d);
        e[0] = a;
        e[1] = b;
        e[2] = c;
        e[3] = d;
      }
    }
    __syncthreads();
    if (mine) {
#pragma unroll
      for (int m = 0; m < 16; m++) {
        const uint32_t t = tab[16 * r + m];
#pragma unroll
        for (int i = 0; i < 4; i++)
          q[4 * m + i] = X[(t >> (8 * i)) & 0xffu];
      }
    }
    __syncthreads();
  }
}

// inverse: coefficients in coding order -> inverse w-lift (decode4.c:31-36) ->
// lane r gets slice w = r.  HALF: as exchange_fwd.
template <bool REV, bool HALF = false, typename Int>
__device__ __forceinline__ void exchange_inv(Int (&q)[64], Int* X, const uint32_t* tab)
{
  const uint32_t r = threadIdx.x & 3u;
  const uint32_t mine_h = (threadIdx.x >> 5) & 1u;
  __syncthreads();
#pragma unroll
  for (uint32_t h = 0; h < (HALF ? 2u : 1u); h++) {
    const bool mine = !HALF || mine_h == h;
    if (mine) {
#pragma unroll
      for (int m = 0; m < 16; m++) {
        const uint32_t t = tab[16 * r + m];
#pragma unroll
        for (int i = 0; i < 4; i++)
          X[(t >> (8 * i)) & 0xffu] = q[4 * m + i];
      }
    }
    __syncthreads();
    if (mine) {
#pragma unroll
      for (int j = 0; j < 16; j++) {
        Int* e = X + 4 * (16 * r + j);
        Int a = e[0], b = e[1], c = e[2], d = e[3];
        if (REV) Lift<Int>::rinv(a, b, c, d);
        else Lift<Int>::inv(a, b, c, d);
        e[0] = a;
        e[1] = b;
        e[2] = c;
        e[3] = d;
      }
    }
    __syncthreads();
    if (mine) {
#pragma unroll
      for (int i = 0; i < 64; i++)
        q[i] = X[4 * i + r];
    }
    if (HALF)
      __syncthreads();
  }
}

// zero `words` 64-bit words at w (whole wave)
__device__ __forceinline__ void zero_region(uint64_t* w, uint32_t words)
{
  for (uint32_t i = threadIdx.x & 63u; i < words; i += 64)
    w[i] = 0;
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Embedded coder over 256-coefficient planes (encode.c:136-175, 208-234).
// Same closed form as code_planes (codec_dev.h) with the plane split into four
// 64-bit segments: lane r writes its segment's verbatim bits at pos + 64r and
// the doubled-ones expansion of its part of xs at the offset given by the
// quad's exclusive scan of the new ones below it; the lane holding the top
// one removes the top pair's surplus.
//
// Slot writes are funnel-shifted dwords ORed into LDS.  A write of v at bit p
// covers dwords j-1 .. j+1 (j = ceil(p / 32)); its first dword is clamped to
// jmax - 2 (one v_min for the three dwords, which then take immediate
// offsets).  A write clamped that way starts at bit >= 32 (jmax - 1), so it
// lands in the slot's last three dwords only, which hold no block bits: a slot
// keeps its first 32 (jmax - 2) bits intact (the host's cap_bits, slot_words4).
// p >= 1, or p == 0 with a zero first dword (the write at dword -1 ORs 0).
__device__ __forceinline__ void or64_at(uint32_t* dm, uint32_t jmax, uint32_t p, uint32_t v0, uint32_t v1)
{
  const uint32_t j = min((p + 31u) >> 5, jmax - 1u);
  const uint32_t t = 0u - p;
  uint32_t* q = dm + j;  // dm = slot - 1 dword: q = dword j - 1
  lds_or32(q, __builtin_amdgcn_alignbit(v0, 0u, t));
  lds_or32(q + 1, __builtin_amdgcn_alignbit(v1, v0, t));
  lds_or32(q + 2, __builtin_amdgcn_alignbit(0u, v1, t));
}

// or64_at of a segment write at bit p + 64 r, given jp = ceil(p / 32): the
// lane's offset of 2 r dwords is folded into its base pointer dmr = dm + 2 r and
// its clamp jlr = jmax - 1 - 2 r
__device__ __forceinline__ void or64_seg(uint32_t* dmr, uint32_t jlr, uint32_t jp, uint32_t t, uint32_t v0,
                                         uint32_t v1)
{
  uint32_t* q = dmr + min(jp, jlr);
  lds_or32(q, __builtin_amdgcn_alignbit(v0, 0u, t));
  lds_or32(q + 1, __builtin_amdgcn_alignbit(v1, v0, t));
  lds_or32(q + 2, __builtin_amdgcn_alignbit(0u, v1, t));
}

__device__ __forceinline__ void or32_at(uint32_t* dm, uint32_t jmax, uint32_t p, uint32_t v)
{
  const uint32_t j = min((p + 31u) >> 5, jmax - 1u);
  const uint32_t t = 0u - p;
  uint32_t* q = dm + j;
  lds_or32(q, __builtin_amdgcn_alignbit(v, 0u, t));
  lds_or32(q + 1, __builtin_amdgcn_alignbit(0u, v, t));
}

// doubled-ones expansion of 32 bits (32 + popcount bits <= 64)
__device__ __forceinline__ uint64_t dbl32(const uint32_t* lut, uint32_t x)
{
  const uint32_t lo = x & 0xffffu;
  return (uint64_t)dbl16(lut, lo) | ((uint64_t)dbl16(lut, x >> 16) << (16u + (uint32_t)__popc(lo)));
}

// Planes PREC-1 .. kmin of the quad's block from bit `pos` of its slot (d,
// last dword jmax); returns the end bit, at most lim.  Per plane, with n the
// coefficients already significant:
//   nr = clamp(n - 64r, 0, 64)     significant coefficients of the segment
//   xs = segment >> nr             its not-yet-significant bits
//   n1 = max(n, quad max of 1 + the top new one)
//   the plane's length n1 + (new ones) + 1 - [n1 == 256] - [new top one is coefficient 255].
// Once every active quad of the wave has all 256 coefficients significant, the
// remaining planes are 256 verbatim bits each (no group tests) and take a short
// loop of their own (a reversible C5 wave: about 6 of its 30 planes).
template <int PREC>
__device__ __forceinline__ uint32_t code_planes4(uint32_t* d, uint32_t jmax, const uint32_t* lut, uint32_t pos,
                                                 uint32_t lim, uint32_t maxprec, const uint32_t (&Pl)[PREC],
                                                 const uint32_t (&Ph)[PREC])
{
  const uint32_t r = threadIdx.x & 3u;
  const uint32_t base = 64u * r;  // first coefficient of this lane's segment
  const uint32_t kmin = (uint32_t)PREC > maxprec ? (uint32_t)PREC - maxprec : 0u;
  uint32_t* dm = d - 1;
  uint32_t* dmr = dm + 2u * r;
  const uint32_t jlr = jmax - 1u - 2u * r;
  uint32_t m_odd, m_hi;
  quad_excl_masks(m_odd, m_hi);
  uint32_t p = pos, n = 0;
  int kf = -1;  // wave-uniform: first plane of the all-significant tail (-1: none)
#pragma unroll
  for (int k = PREC - 1; k >= 0; k--) {
    if (kf >= 0)
      continue;
    const bool act = p < lim && (uint32_t)k >= kmin;  // quad-uniform
    const uint64_t am = lanes_ult(p, lim) & lanes_ule(kmin, (uint32_t)k);  // ballot(act)
    if (am == 0)
      break;
    if ((am & lanes_ne(n, 256u)) == 0) {
      kf = k;
      continue;
    }
    const uint64_t P = ((uint64_t)Ph[k] << 32) | Pl[k];
    const uint32_t nr = (uint32_t)min(max((int)(n - base), 0), 64);  // v_med3_i32
    // Straight-line for every lane: an inactive lane (or an empty part) ORs
    // zeros, so no per-lane branch (and no exec-mask bookkeeping) is needed.
    const uint64_t xs = (act && nr < 64u) ? P >> nr : 0ull;
    // V = P & low_mask(nv), inactive lanes nv = 0: M = ~0 << nv (0 for nv = 64), V = P & ~M
    const uint32_t nv = act ? nr : 0u;
    const uint64_t M = ~0ull << (nv & 63u);
    const uint32_t Ml = nv < 64u ? (uint32_t)M : 0u, Mh = nv < 64u ? (uint32_t)(M >> 32) : 0u;
    const uint32_t Vl = __builtin_amdgcn_bitop3_b32(Ml, Pl[k], 0u, 0x0c), Vh = __builtin_amdgcn_bitop3_b32(Mh, Ph[k], 0u, 0x0c);
    const uint32_t L = xs ? 64u - (uint32_t)__clzll((long long)xs) : 0u;  // xs's length
    const uint32_t tb = L ? base + nr + L : 0u;                            // 1 + the lane's top new one
    const uint32_t n1 = quad_max(max(tb, n));
    const uint32_t c = (uint32_t)__popcll(xs);
    uint32_t ctot;
    const uint32_t cex = quad_excl(c, ctot, m_odd, m_hi);
    const bool grow = n1 > n;
    const uint32_t all = n1 == 256u ? 1u : 0u;
    const uint32_t impl = grow ? all : 0u;  // coefficient 255: its one and test are implicit
    const uint32_t dlen = n1 + ctot + 1u - all - impl;
    or64_seg(dmr, jlr, (p + 31u) >> 5, 0u - p, Vl, Vh);
    const uint32_t gp = p + n;  // the plane's positive group test
    lds_or32(d + min(gp >> 5, jmax), (grow && r == 0u) ? 1u << (gp & 31u) : 0u);
    // Group bits: the expansion of xs unit 0 (bits 0..15) is written here; a
    // lane whose xs reaches past bit 15 (at most three planes per segment: each
    // moves the frontier by >= 17) writes its whole expansion again in a
    // wave-uniform branch (OR is idempotent on the unit-0 bits), as code_planes
    // does.  The top one at xs bit h: its pair starts at h + (c - 1).
    const uint32_t x0 = (uint32_t)xs;
    const bool top = L != 0u && tb == n1;
    const uint32_t h = L - 1u;
    const uint32_t t = h + c - 1u;
    const uint32_t co = p + 1u + base + nr + cex;
    const uint32_t m0 = (top && h < 16u) ? ((2u | impl) << (t & 31u)) : 0u;
    or32_at(dm, jmax, co, dbl16(lut, x0 & 0xffffu) & ~m0);
    const bool ext = (xs >> 16) != 0ull;
    if ((lanes_ne((uint32_t)(xs >> 32), 0u) | lanes_ugt((uint32_t)xs, 0xffffu)) != 0) {
      if (ext) {
        const uint32_t x1 = (uint32_t)(xs >> 32);
        uint64_t E0 = dbl32(lut, x0), E1 = dbl32(lut, x1);
        const uint32_t L0 = 32u + (uint32_t)__popc(x0);
        const uint64_t m = top ? (uint64_t)(2u | impl) : 0ull;
        E0 &= ~(h < 32u ? m << (t & 63u) : 0ull);
        E1 &= ~(h < 32u ? 0ull : m << ((t - L0) & 63u));
        or64_at(dm, jmax, co, (uint32_t)E0, (uint32_t)(E0 >> 32));
        or64_at(dm, jmax, co + L0, (uint32_t)E1, (uint32_t)(E1 >> 32));
      }
    }
    p = act ? p + dlen : p;
    n = act ? n1 : n;
  }
  if (kf >= 0) {
    // every active quad has n == 256: a plane is its 256 bits verbatim
#pragma unroll
    for (int k = PREC - 1; k >= 0; k--) {
      if (k > kf)
        continue;
      const bool act = p < lim && (uint32_t)k >= kmin;
      if ((lanes_ult(p, lim) & lanes_ule(kmin, (uint32_t)k)) == 0)
        break;
      or64_seg(dmr, jlr, (p + 31u) >> 5, 0u - p, act ? Pl[k] : 0u, act ? Ph[k] : 0u);
      p = act ? p + 256u : p;
    }
  }
  return p < lim ? p : lim;
}

// Decoder twin (decode.c:122-173, 212-246): the quad parses the group tests
// redundantly (same stream bits, same control flow), each lane keeping the
// ones of its segment; verbatim bits are read per segment.  One iteration per
// group test, i.e. per newly significant coefficient plus one per plane.
template <int PREC>
__device__ __forceinline__ uint32_t decode_planes4(WordReader& rd, uint32_t budget, uint32_t maxprec,
                                                   uint64_t (&P)[PREC])
{
  const uint32_t r = threadIdx.x & 3u;
  const uint32_t base = 64u * r;
  const uint32_t kmin = (uint32_t)PREC > maxprec ? (uint32_t)PREC - maxprec : 0u;
  uint32_t bits = budget, n = 0;
#pragma unroll
  for (int k = 0; k < PREC; k++)
    P[k] = 0;
#pragma unroll
  for (int k = PREC - 1; k >= 0; k--) {
    const bool act = bits != 0 && (uint32_t)k >= kmin;
    if (__builtin_amdgcn_ballot_w64(act) == 0)
      break;
    if (act) {
      const uint32_t m = n < bits ? n : bits;
      const uint32_t cnt = m > base ? min(m - base, 64u) : 0u;
      WordReader seg{rd.w, rd.pos + base};
      uint64_t x = seg.read(cnt);
      rd.skip(m);
      bits -= m;
      while (n < 256u && bits) {
        // one window per group test: bit 0 the test, then the zeros up to the
        // next one; a run of zeros past the window's 63 bits reads the next 64
        uint64_t W = rd.peek64();
        bits--;
        rd.skip(1);
        if (!(W & 1u))
          break;
        W >>= 1;
        uint32_t avail = 63;
        for (;;) {
          const uint32_t lim = min(255u - n, bits);  // at most to coefficient 255 / the budget
          const uint32_t z = ctz64(W);
          if (z < avail || lim <= avail) {
            const uint32_t t = min(z, lim);
            const uint32_t one = z < lim ? 1u : 0u;  // the one is read (not the implicit last / cut)
            rd.skip(t + one);
            bits -= t + one;
            n += t;
            break;
          }
          rd.skip(avail);
          bits -= avail;
          n += avail;
          W = rd.peek64();
          avail = 64;
        }
        if (n - base < 64u)
          x |= 1ull << (n - base);
        n++;
      }
      P[k] = x;
    }
  }
  return budget - bits;
}

__device__ __forceinline__ uint32_t precision4(int emax, const CodecParams& cp)
{
  int p = emax - cp.minexp + 2 * (4 + 1);
  if (p < 0) p = 0;
  return (uint32_t)p < cp.maxprec ? (uint32_t)p : cp.maxprec;
}

// lossy exponent + cast (the 3D fast path with quad-wide maxima)
template <typename Reload>
__device__ __forceinline__ int lossy_emax_cast4(int32_t (&q)[64], float (&v)[64], const CodecParams& cp,
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
  const uint32_t mb = quad_max(max((uint32_t)mi, mu & 0x7fffffffu));
  int emax = mb == 0 ? -127 : ((mb >> 23) == 0 ? -126 : (int)(mb >> 23) - 126);
  const bool bad = mb >= 0x7f800000u;  // inf/NaN in the block: NaN-ignoring max
  if (__any(bad)) {
    const float am = quad_absmax(v);
    if (bad)
      emax = block_emax(am);
  }
  mp = precision4(emax, cp);
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
__device__ __forceinline__ int lossy_emax_cast4(int64_t (&q)[64], double (&v)[64], const CodecParams& cp,
                                                uint32_t& mp, Reload&&)
{
  const int emax = block_emax(quad_absmax(v));
  mp = precision4(emax, cp);
  fwd_cast(q, v, emax);
  return emax;
}

// Encode the quad's block into its zeroed slot; returns the block length in
// bits including minbits padding.  Called by the whole wave: the exchange and
// the slot zeroing are wave-wide (`region`, `region_words`: the wave's slot
// area, which aliases the exchange areas).  The slot comes from
// place(big, d, jmax), called by the whole wave once the region is zeroed
// (d: the slot's dwords, jmax: its last dword); big: the block codes with the
// reversible reinterpreted-bits header (the long ones, about 8,300 bits on
// f32 data), so a kernel with short slots can give it a full one.
template <typename S, bool REV, bool HALF = false, typename Place, typename Reload>
__device__ __forceinline__ uint32_t encode_block4(Place&& place, const uint32_t* lut, const uint32_t* tab,
                                                  typename Traits<S>::Int* X, uint64_t* region, uint32_t region_words,
                                                  S (&v)[64], const CodecParams& cp, Reload&& reload)
{
  using T = Traits<S>;
  using Int = typename T::Int;
  using UInt = typename T::UInt;
  constexpr uint32_t kE = T::kEbits;
  constexpr int PREC = T::kIntPrec;
  const uint32_t r = threadIdx.x & 3u;
  uint32_t* d;
  uint32_t jmax;
  Int q[64];
  uint32_t Pl[PREC], Ph[PREC];
  if constexpr (std::is_integral<S>::value) {
    // integer blocks (encode.c:260-280, revencode.c:54-76): no exponent, and
    // only the reversible mode has a header (the precision)
#pragma unroll
    for (int i = 0; i < 64; i++)
      q[i] = (Int)v[i];
    xform<3, false, REV>(q);
    exchange_fwd<REV, HALF>(q, X, tab);
    zero_region(region, region_words);
    place(false, d, jmax);
    OrSlot os{reinterpret_cast<uint64_t*>(d), jmax};
    uint32_t prec = cp.maxprec, bits = 0;
    if constexpr (REV) {
      UInt all = 0;
#pragma unroll
      for (int i = 0; i < 64; i++)
        all |= ((UInt)q[i] + T::kNbMask) ^ T::kNbMask;
      all = quad_or(all);
      prec = all ? (uint32_t)(PREC - (sizeof(S) == 4 ? __builtin_ctz((uint32_t)all) : __builtin_ctzll((uint64_t)all)))
                 : 0u;
      if (prec > cp.maxprec) prec = cp.maxprec;
      if (prec < 1) prec = 1;
      if (r == 0u) os.head(prec - 1);
      bits = T::kPbits;
    }
    if constexpr (PREC == 32)
      planes_from_coeffs<false>(Pl, Ph, q);
    else
      planes_from_coeffs<false>(Pl, Ph, q, prec > 32);
    pin_registers(Pl);
    pin_registers(Ph);
    const uint32_t end = code_planes4<PREC>(d, jmax, lut, bits, cp.maxbits, prec, Pl, Ph);
    return end < cp.minbits ? cp.minbits : end;
  } else if constexpr (REV) {
    // reversible (revencodef.c:45-80)
    int emax = 0;
    bool fast = false;  // wave-uniform: no inf/NaN in any block of the wave (f32)
    if constexpr (sizeof(S) == 4) {
      // block maximum from integer maxima of the bit patterns (as
      // lossy_emax_cast4): a tree of v_max3 instead of a chain of 64 float
      // compares; NaN sorts above inf, so one compare flags the blocks that
      // need the exact NaN-ignoring maximum
      int32_t mi = 0;
      uint32_t mu = 0;
#pragma unroll
      for (int i = 0; i < 64; i++) {
        const uint32_t b = __float_as_uint(v[i]);
        mi = max(mi, (int32_t)b);
        mu = max(mu, b);
      }
      const uint32_t mb = quad_max(max((uint32_t)mi, mu & 0x7fffffffu));
      fast = !__any(mb >= 0x7f800000u);
      emax = mb == 0 ? -127 : ((mb >> 23) == 0 ? -126 : (int)(mb >> 23) - 126);
    }
    if (!fast)
      emax = block_emax(quad_absmax(v));
    // bitwise accumulation: a short-circuit && becomes 64 nested lane branches
    decltype(bits_of(v[0])) sdiff = 0;
    bool same;
    if (emax != -T::kEbias) {
      if constexpr (sizeof(S) == 4) {
        if (fast) {
          // finite block: |2^(30 - emax) x| < 2^30, the plain conversion is the
          // reference's (no x86 out-of-range emulation needed)
          const float sc = pow2f(30 - emax);
#pragma unroll
          for (int i = 0; i < 64; i++)
            q[i] = (int32_t)(sc * v[i]);
        } else {
          fwd_cast(q, v, emax);
        }
      } else {
        fwd_cast(q, v, emax);
      }
      const S s = (sizeof(S) == 4) ? (S)pow2f(emax - 30) : (S)pow2d(emax - 62);
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
    same = quad_or(sdiff != 0 ? 1u : 0u) == 0u;
    if (!same) {
#pragma unroll
      for (int i = 0; i < 64; i++) {
        const Int x = (Int)bits_of(v[i]);
        q[i] = x < 0 ? (Int)((UInt)x ^ T::kTcMask) : x;
        if ((i & 3) == 3)
          ZFP_SCHED_FENCE();
      }
    }
    xform<3, false, true>(q);
    exchange_fwd<true, HALF>(q, X, tab);
    zero_region(region, region_words);
    place(!same, d, jmax);
    OrSlot os{reinterpret_cast<uint64_t*>(d), jmax};
    const uint32_t e = (uint32_t)(emax + T::kEbias);
    if (same && !e)
      return 1u < cp.minbits ? cp.minbits : 1u;  // a single 0 bit
    uint32_t bits;
    if (same) {
      if (r == 0u) os.head(1u | (e << 2));
      bits = 2 + kE;
    } else {
      if (r == 0u) os.head(3u);
      bits = 2;
    }
    // rev_encode_block (revencode.c:54-76): precision from the OR of all 256
    const uint32_t minb = cp.minbits - (bits < cp.minbits ? bits : cp.minbits);
    UInt all = 0;
#pragma unroll
    for (int i = 0; i < 64; i++)
      all |= ((UInt)q[i] + T::kNbMask) ^ T::kNbMask;
    all = quad_or(all);
    uint32_t prec = all ? (uint32_t)(PREC - (sizeof(S) == 4 ? __builtin_ctz((uint32_t)all)
                                                            : __builtin_ctzll((uint64_t)all)))
                        : 0u;
    if (prec > cp.maxprec) prec = cp.maxprec;
    if (prec < 1) prec = 1;
    if (r == 0u) os.put32(bits, prec - 1);
    if constexpr (PREC == 32)
      planes_from_coeffs<false>(Pl, Ph, q);
    else
      planes_from_coeffs<false>(Pl, Ph, q, prec > 32);
    pin_registers(Pl);
    pin_registers(Ph);
    const uint32_t end = code_planes4<PREC>(d, jmax, lut, bits + T::kPbits, cp.maxbits, prec, Pl, Ph);
    uint32_t ib = end - bits;
    if (ib < minb) ib = minb;
    return bits + ib;
  } else {
    // lossy (encodef.c:63-90)
    uint32_t mp;
    const int emax = lossy_emax_cast4(q, v, cp, mp, reload);
    const uint32_t e = mp ? (uint32_t)(emax + T::kEbias) : 0u;
    xform<3, false, false>(q);
    exchange_fwd<false, HALF>(q, X, tab);
    zero_region(region, region_words);
    place(false, d, jmax);
    OrSlot os{reinterpret_cast<uint64_t*>(d), jmax};
    uint32_t bits = 1;
    if (e) {
      if (r == 0u) os.head(2 * e + 1);
      bits += kE;
      const uint32_t minb = cp.minbits - (bits < cp.minbits ? bits : cp.minbits);
      if constexpr (PREC == 32)
        planes_from_coeffs<false>(Pl, Ph, q);
      else
        planes_from_coeffs<false>(Pl, Ph, q, mp > 32);
      pin_registers(Pl);
      pin_registers(Ph);
      uint32_t ib = code_planes4<PREC>(d, jmax, lut, bits, cp.maxbits, mp, Pl, Ph) - bits;
      if (ib < minb) ib = minb;
      bits += ib;
    } else if (cp.minbits > bits) {
      bits = cp.minbits;
    }
    return bits;
  }
}

// Decode the quad's block (invalid quads decode nothing but take part in the
// wave-wide exchange); lane r receives slice w = r.  Returns the block's length
// in bits including minbits padding (0 for an invalid quad), the encoder's.
#ifdef ZFP_EXP4_TRACE
__shared__ uint64_t zfp_dmarks[4];  // experiment: phase clocks of decode_block4 (lane 0)
#define ZFP_DEC4_MARK(i) do { if (threadIdx.x == 0) zfp_dmarks[i] = wall_clock64(); } while (0)
#else
#define ZFP_DEC4_MARK(i) ((void)0)
#endif

template <typename S, bool REV, bool HALF = false>
__device__ __forceinline__ uint32_t decode_block4(WordReader& rd, S (&v)[64], const CodecParams& cp,
                                                  typename Traits<S>::Int* X, const uint32_t* tab, bool valid)
{
  using T = Traits<S>;
  using Int = typename T::Int;
  using UInt = typename T::UInt;
  constexpr uint32_t kE = T::kEbits;
  constexpr int PREC = T::kIntPrec;
  Int q[64];
#pragma unroll
  for (int i = 0; i < 64; i++)
    q[i] = 0;
  int emax = 0;
  uint32_t kind = 0;  // 0: zero block, 1: block-floating-point, 2: reinterpreted bits
  uint32_t used = 0;
  if constexpr (std::is_integral<S>::value) {
    // integer blocks (decode.c:271-287, revdecode.c:34-52)
    if (valid) {
      uint32_t prec = cp.maxprec, bits = 0;
      if constexpr (REV) {
        prec = (uint32_t)rd.read(T::kPbits) + 1;
        bits = T::kPbits;
      }
      uint64_t P[PREC];
      used = bits + decode_planes4<PREC>(rd, cp.maxbits - bits, prec, P);
      used = used < cp.minbits ? cp.minbits : used;
      pin_registers(P);
      if constexpr (PREC == 32)
        coeffs_from_planes<false>(q, P);
      else
        coeffs_from_planes<false>(q, P, prec > 32);
    }
    exchange_inv<REV, HALF>(q, X, tab);
    xform<3, true, REV>(q);
#pragma unroll
    for (int i = 0; i < 64; i++)
      v[i] = (S)q[i];
    return used;
  } else {
    if (valid)
      used = 1u < cp.minbits ? cp.minbits : 1u;  // a zero block: one bit and the padding
    if (valid && rd.read1()) {
      uint32_t bits = 1;
      uint32_t prec;
      if constexpr (REV) {
        bits++;
        const bool reinterp = rd.read1() != 0;
        if (!reinterp) {
          bits += kE;
          emax = (int)rd.read(kE) - T::kEbias;
        }
        prec = (uint32_t)rd.read(T::kPbits) + 1;
        bits += T::kPbits;
        kind = reinterp ? 2u : (emax != -T::kEbias ? 1u : 0u);
      } else {
        bits += kE;
        emax = (int)rd.read(kE) - T::kEbias;
        prec = precision4(emax, cp);
        kind = 1;
      }
      uint64_t P[PREC];
      used = bits + decode_planes4<PREC>(rd, cp.maxbits - bits, prec, P);
      used = used < cp.minbits ? cp.minbits : used;
      pin_registers(P);
      ZFP_DEC4_MARK(0);
      if constexpr (PREC == 32)
        coeffs_from_planes<false>(q, P);
      else
        coeffs_from_planes<false>(q, P, prec > 32);
    }
    ZFP_DEC4_MARK(1);
    exchange_inv<REV, HALF>(q, X, tab);
    ZFP_DEC4_MARK(2);
    xform<3, true, REV>(q);
    ZFP_DEC4_MARK(3);
    if (REV && kind == 2u) {
#pragma unroll
      for (int i = 0; i < 64; i++) {
        const Int x = q[i] < 0 ? (Int)((UInt)q[i] ^ T::kTcMask) : q[i];
        if constexpr (sizeof(S) == 4)
          v[i] = __uint_as_float((uint32_t)x);
        else
          v[i] = __longlong_as_double((long long)x);
      }
    } else if (kind == 1u) {
      inv_cast(v, q, emax);
    } else {
#pragma unroll
      for (int i = 0; i < 64; i++)
        v[i] = 0;
    }
    return used;
  }
}

}  // namespace zfp_amd
