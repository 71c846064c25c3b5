// 4D encode/decode kernels: one 4x4x4x4 block per quad of lanes (block4.h),
// 16 blocks per wave, one wave per 64-thread workgroup.  The per-block LDS
// exchange area of the w-lift is what limits occupancy, so workgroups are kept
// to one wave and the CU packs as many as its LDS holds.
//
//  encode4  every mode; blocks are packed at their bit offsets exactly as by
//           encode3_general (fixed rate: analytic offsets; variable rate:
//           decoupled look-back over per-wave bit totals + block index), the
//           words shared with neighbouring waves go to the fix-up kernels.
//  decode4  stages the wave's 16 blocks in LDS (fixed rate: analytic offsets;
//           variable rate: from the index), each quad decodes its block.
#pragma once

#include "block4.h"
#include "kernels3.h"

namespace zfp_amd {

constexpr uint32_t kBlocks4PerWave = 16;
// LDS words ahead of the slot / exchange region.  Encoder: doubled-ones table
// (256 dwords), order table (64), per-block bit offsets and written counts
// (16 + 16).  (f32 reversible: 176 + 16 x 93 words = 13,312 bytes, 12 waves
// per CU at the 512-byte LDS granule; 8 more bytes would cost a wave.)
constexpr uint32_t kEnc4HeadWords = (256 + 64 + 16 + 16) / 2;
// Short reversible slots (a.ovf set): a block that fails the reversible cast
// (the reinterpreted-bits header, about 8,300 bits on f32 data -- 7.5 % of the
// C5 blocks, in half of its waves) gets a full slot of a.ovf_swp words, the
// others share the rest of the wave's 16 a.swp words, at least kMinSlot4
// words each (4,192 bits: 99.9 % of the other C5 blocks code shorter).
// Blocks that still outrun their slot (a long cast block, more big blocks
// than fit) take the overflow list and encode4_patch.
constexpr uint32_t kMinSlot4 = 67;
// Decoder: order table (64 dwords), per-block stream bit offsets (16).
constexpr uint32_t kDec4HeadWords = (64 + 16) / 2;

// Slot of a 4D block with budget `lim` bits: its dwords plus three spare
// dwords (targets of the clamped writes past the budget, block4.h or64_at);
// odd, so the 16 slots of a wave start on different banks.
__host__ __device__ constexpr uint32_t slot_words4(uint32_t lim) { return ((((lim + 31u) >> 5) + 4u) / 2u) | 1u; }
// Bits of a slot of swp words that clamped writes never touch
__host__ __device__ constexpr uint32_t slot_cap_bits4(uint32_t swp) { return 32u * (2u * swp - 3u); }

// Overflow list of the short-slot 4D encoder: a block longer than its LDS slot
// is packed with its first cap_bits only (the rest zero) and listed with its
// stream bit position; encode4_patch codes it again with a full-size slot and
// ORs it in.  The list lives in GeneralArgs::ovf (two words per entry).
struct OvfEntry {
  uint64_t b;    // block
  uint64_t pos;  // bit position of its first bit relative to out[0]
};

// In-place compaction of a wave's 16 slots into one bit string in LDS (local
// bit 0 = the wave's first block), before its stream offset is known: block q
// (wrt[q] bits at bit 0 of slot_of(q)) moves to local bit off[q], one block
// after another, as funnel-shifted dwords.  Safe in place when every block fits
// its slot (the caller's `simple` test): block q's destination ends at
// off[q + 1] <= 64 x the words of slots 0..q, i.e. before slot q + 1, and within
// a block every lane reads its dwords before any lane writes.  The last dword
// is masked to the block's bits (a budget cut leaves the rest of the cut plane
// in the slot); the first dword ORs onto the end of the previous block.  NT: dwords per lane of the longest slot (f32: 272 dwords, f64: 526).
template <int NT, typename SlotOf>
__device__ __forceinline__ void compact_wave4(uint64_t* region, const uint32_t* off, const uint32_t* wrt,
                                              SlotOf&& slot_of)
{
  const uint32_t lane = threadIdx.x & 63u;
  uint32_t* dst0 = reinterpret_cast<uint32_t*>(region);
  for (uint32_t q = 0; q < kBlocks4PerWave; q++) {
    // wave-uniform block geometry in scalar registers
    const uint32_t L = (uint32_t)__builtin_amdgcn_readfirstlane((int)wrt[q]);
    const uint32_t D = (uint32_t)__builtin_amdgcn_readfirstlane((int)off[q]);
    const uint32_t d = D & 31u, nd = (d + L + 31u) >> 5;
    // dword k of the destination holds block bits [32 k - d, 32 k - d + 32):
    // alignbit(s[k], s[k - 1], 32 - d), read as the pair at src - 1 (d == 0:
    // the pair at src, shift 0)
    const uint32_t* src = reinterpret_cast<const uint32_t*>(slot_of(q)) - (d ? 1 : 0);
    const uint32_t sh = (32u - d) & 31u;
    // the last dword keeps the block's bits only: past a budget cut the slot
    // holds the rest of the cut plane
    const uint32_t valid = d + L - 32u * (nd - 1u);  // 1 .. 32
    const uint32_t last_mask = valid >= 32u ? ~0u : (1u << valid) - 1u;
    uint32_t* dst = dst0 + (D >> 5);
    uint32_t v[NT];
#pragma unroll
    for (int t = 0; t < NT; t++) {
      if (64u * t < nd) {
        const uint32_t k = lane + 64u * t;
        uint32_t lo = src[k], hi = src[k + 1];
        if (t == 0)
          lo = k == 0 && d ? 0u : lo;  // nothing below the block's first bit
        v[t] = __builtin_amdgcn_alignbit(hi, lo, sh) & (k == nd - 1u ? last_mask : ~0u);
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the block's reads have returned
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int t = 0; t < NT; t++) {
      if (64u * t < nd) {
        const uint32_t k = lane + 64u * t;
        if (t == 0 && k == 0 && d)
          dst[0] |= v[t];  // onto the end of the previous block (same wave: in order)
        else if (k < nd)
          dst[k] = v[t];
      }
    }
    // LDS operations of a wave complete in order: the next block reads after these writes
    __builtin_amdgcn_wave_barrier();
  }
}

// Copy-out of a compacted wave (local words loc[0 ..]) to its stream bits
// [G, G + total), G = g0 + start.  Output dword e holds local bits [32 e - r0,
// 32 e - r0 + 32) = alignbit(Ld[e - j + 1], Ld[e - j], 32 j - r0), j = ceil(r0 /
// 32) (as encode3_aligned's copy-out).  Each lane writes a pair of output words
// aligned to 16 bytes in memory; the first and last word (shared with the
// neighbouring waves) go to the partials for the fix-up kernels, as in
// pack_wave.
__device__ __forceinline__ void copy_out_wave(const GeneralArgs& a, const uint64_t* loc, uint64_t w, uint64_t start,
                                              uint32_t total)
{
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t G = a.g0 + start;
  const uint64_t W0 = G >> 6;
  const uint32_t r0 = (uint32_t)(G & 63);
  const uint64_t end = G + total;
  const uint32_t nw = (uint32_t)(((end - 1) >> 6) - W0 + 1);
  const uint32_t nld = (total + 31u) >> 5;  // local dwords that hold bits (the compaction wrote no others)
  const bool head_part = r0 != 0 || (nw == 1 && (end & 63));
  const bool tail_part = (end & 63) != 0;
  const uint32_t jj = (r0 + 31u) >> 5, sh = (32u * jj - r0) & 31u;
  const uint32_t* Ld = reinterpret_cast<const uint32_t*>(loc);
  auto ld = [&](int32_t i) -> uint32_t { return (i >= 0 && (uint32_t)i < nld) ? Ld[i] : 0u; };
  // output word o at memory word W0 + o: pairs (o, o + 1) with W0 + o even
  const uint32_t o0 = (uint32_t)((reinterpret_cast<uintptr_t>(a.out + W0) >> 3) & 1u);
  auto emit = [&](uint32_t o, uint64_t val) {
    const bool head = o == 0 && head_part;
    const bool tail = o == nw - 1 && tail_part;
    if (head || tail)
      a.partials[2 * w + (o == 0 ? 0 : 1)] = Partial{W0 + o, val};
    else
      a.out[W0 + o] = val;
  };
  for (uint32_t c = lane; o0 + 2 * c < nw; c += 64) {
    const uint32_t o = o0 + 2 * c;
    const int32_t e = (int32_t)(2 * o) - (int32_t)jj;  // first input dword of output dword 2 o
    const uint32_t x0 = ld(e), x1 = ld(e + 1), x2 = ld(e + 2), x3 = ld(e + 3), x4 = ld(e + 4);
    const uint32_t y0 = __builtin_amdgcn_alignbit(x1, x0, sh), y1 = __builtin_amdgcn_alignbit(x2, x1, sh);
    const uint32_t y2 = __builtin_amdgcn_alignbit(x3, x2, sh), y3 = __builtin_amdgcn_alignbit(x4, x3, sh);
    const uint64_t v0 = ((uint64_t)y1 << 32) | y0, v1 = ((uint64_t)y3 << 32) | y2;
    const bool whole = o + 1 < nw && !(o == 0 && head_part) && !(o + 1 == nw - 1 && tail_part);
    if (whole) {
      typedef uint32_t u4 __attribute__((ext_vector_type(4)));
      *reinterpret_cast<u4*>(a.out + W0 + o) = u4{y0, y1, y2, y3};
    } else {
      emit(o, v0);
      if (o + 1 < nw)
        emit(o + 1, v1);
    }
  }
  if (lane == 0) {
    if (o0 == 1) {  // word 0 alone (before the first aligned pair)
      const uint32_t y0 = __builtin_amdgcn_alignbit(ld(1 - (int32_t)jj), ld(-(int32_t)jj), sh);
      const uint32_t y1 = __builtin_amdgcn_alignbit(ld(2 - (int32_t)jj), ld(1 - (int32_t)jj), sh);
      emit(0, ((uint64_t)y1 << 32) | y0);
    }
    if (!head_part)
      a.partials[2 * w].idx = kNoWord;
    if (!tail_part || nw == 1)
      a.partials[2 * w + 1].idx = kNoWord;
  }
}

// bits of a block to copy from its slot: all of them, or the intact cap of an
// overflowed block, or the slot (past it a block holds minbits padding zeros)
__device__ __forceinline__ uint32_t wrt_of(uint32_t len, uint32_t sw, uint32_t cap, bool over)
{
  return over ? cap : (len < 64 * sw ? len : 64 * sw);
}

// HALF: exchange areas shared by quads q and q + 8 (block4.h exchange_fwd), so
// the LDS region is max(16 slots, 8 exchange areas); with a.ovf the slots are
// short (see OvfEntry).
// (Compiled for 4 waves per SIMD the f32 reversible encoder spills and ran
// 1.56 -> 1.92 ms on 128^4; it is left unbounded: 140 VGPRs, 3 waves.)
template <typename S, bool VEC, bool REV, bool HALF = false>
__global__ __launch_bounds__(64) void encode4(const S* __restrict__ data, Geometry g, CodecParams cp, GeneralArgs a)
{
  using Int = typename Traits<S>::Int;
  extern __shared__ uint64_t lds[];
  uint32_t* lut = reinterpret_cast<uint32_t*>(lds);
  uint32_t* tab = lut + 256;
  uint32_t* off = tab + 64;
  uint32_t* wrt = off + kBlocks4PerWave;
  uint64_t* region = lds + kEnc4HeadWords;
  const uint32_t lane = threadIdx.x;
  // the doubled-ones table from device memory (CoderTables.dbl), one 16-byte load per lane
  reinterpret_cast<uint4*>(lut)[lane] = reinterpret_cast<const uint4*>(kCoderTables.dbl)[lane];
  tab[lane] = kOrderTab4.t[lane];

#ifdef ZFP_EXP4_TRACE
  const uint64_t tr0 = wall_clock64();
#define ZFP_TR4(i) do { if (a.trace && (w & 63) == 0 && lane == 0) a.trace[(w >> 6) * 8 + (i)] = wall_clock64() - tr0; } while (0)
#else
#define ZFP_TR4(i) ((void)0)
#endif
  const uint64_t nwaves = (g.nblocks + kBlocks4PerWave - 1) / kBlocks4PerWave;
  uint64_t w;
  if (a.var) {
    uint32_t t = 0;
    if (lane == 0)
      t = atomicAdd(a.ticket, 1u);
    w = (uint64_t)__shfl(t, 0, 64);
  } else {
    w = blockIdx.x;
  }
  ZFP_TR4(0);
  const bool live = w < nwaves;
  const uint64_t first = w * kBlocks4PerWave;
  const uint32_t qd = lane >> 2, r = lane & 3u;
  const uint64_t b = first + qd;
  const bool valid = live && b < g.nblocks;
  BlockPos ps{};
  S v[64];
  if (valid) {
    const BlockPos p = block_pos(g, b, 4);
    ps = slice_pos(g, p, pad_src_w((int)r, p.cnt[3]));
    gather3<S, VEC>(v, data, g, ps);
  } else {
#pragma unroll
    for (int i = 0; i < 64; i++)
      v[i] = 0;
  }
  __syncthreads();
#ifdef ZFP_EXP4_TRACE
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the gather has landed
  ZFP_TR4(1);
#endif
  Int* X = reinterpret_cast<Int*>(region) + (size_t)(HALF ? (qd & 7u) : qd) * kXStride;
  // Slot layout of the wave's region (wave-uniform): block l's slot starts at
  // word gb * B + (l - gb) * small, gb = min(big blocks below l, m), and the
  // first m big blocks have B words; uniform a.swp words unless short
  // reversible slots meet a big block.
  uint64_t bm = 0;                         // bit 4l: block l is big
  uint32_t m = 0, small = a.swp, B = a.swp;
  auto slot_words_of = [&](uint32_t l) -> uint32_t {
    const uint32_t below = (uint32_t)__popcll(bm & ((1ull << (4u * l)) - 1ull));
    const uint32_t gb = min(below, m);
    return gb * B + (l - gb) * small;
  };
  uint32_t sw = a.swp;  // the quad's slot words
  auto place = [&](bool big, uint32_t*& d, uint32_t& jmax) {
    ZFP_TR4(2);
    if (REV && a.ovf) {
      bm = __builtin_amdgcn_ballot_w64(big && r == 0u) & 0x1111111111111111ull;
      if (bm) {
        const uint32_t R = kBlocks4PerWave * a.swp;
        B = a.ovf_swp;
        // big slots granted: as many as leave kMinSlot4 words for every other block
        const uint32_t fit = R > kBlocks4PerWave * kMinSlot4 ? (R - kBlocks4PerWave * kMinSlot4) / (B - kMinSlot4) : 0u;
        m = min((uint32_t)__popcll(bm), fit);  // < 16: R < 16 B
        small = (((R - m * B) / (kBlocks4PerWave - m)) - 1u) | 1u;  // odd
        const uint32_t below = (uint32_t)__popcll(bm & ((1ull << (4u * qd)) - 1ull));
        sw = (big && below < m) ? B : small;
      }
    }
    d = reinterpret_cast<uint32_t*>(region + slot_words_of(qd));
    jmax = 2 * sw - 1;
  };
  uint32_t len = encode_block4<S, REV, HALF>(place, lut, tab, X, region, kBlocks4PerWave * a.swp, v, cp,
                                             [&](S (&rr)[64]) {
                                               if (valid) {
                                                 gather3<S, VEC>(rr, data, g, ps);
                                               } else {
#pragma unroll
                                                 for (int i = 0; i < 64; i++)
                                                   rr[i] = 0;
                                               }
                                             });
  ZFP_TR4(3);
  len = valid ? len : 0u;
  const uint32_t cap = slot_cap_bits4(sw);
  const bool over = a.ovf && len > cap;  // quad-uniform
  const uint32_t lq = r == 0u ? len : 0u;  // the quad's lanes agree on len
  const uint32_t incl = wave_incl_scan(lq);
  const uint32_t total = __shfl(incl, 63, 64);
  if (r == 0u) {
    off[qd] = incl - lq;
    wrt[qd] = wrt_of(len, sw, cap, over);
  }
  // Every block fits its slot (wave-uniform; not so only when a block overflows
  // a short slot or minbits pads past it): the wave compacts its slots in LDS
  // while its predecessors finish, publishing its aggregate first, and writes
  // the stream words as whole funnel-shifted words once its offset is known.
  const bool simple = __builtin_amdgcn_ballot_w64(live && (over || (r == 0u && wrt_of(len, sw, cap, over) != len))) == 0;
  if (live && a.var)
    lookback_publish(a.status, w, total);
  __syncthreads();  // off / wrt
  if (live && simple)
    compact_wave4<sizeof(S) == 4 ? 5 : 9>(region, off, wrt, [&](uint32_t l) { return region + slot_words_of(l); });
  uint64_t start = 0;
  if (!live) {
  } else if (a.var) {
    start = lookback_walk(a.status, w, total, a.error);
    if (a.idx_len && valid && r == 0u)
      a.idx_len[b] = (uint16_t)len;
    if (lane == 0) {
      if (a.idx_base)
        a.idx_base[w] = start + a.idx_add;
      if (w == nwaves - 1)
        *a.total_bits = start + total;
    }
  } else {
    start = first * (uint64_t)a.maxbits;
  }
  ZFP_TR4(4);
  if (over && r == 0u) {
    const uint32_t k = take_overflow_slot(a);
    if (k != kNoSlot)
      reinterpret_cast<OvfEntry*>(a.ovf)[k] = OvfEntry{b, a.g0 + start + (incl - lq)};
  }
  __syncthreads();
  if (!live)
    return;
  if (simple)
    copy_out_wave(a, region, w, start, total);
  else
    pack_wave<kBlocks4PerWave, false>(a, region, off, wrt, nullptr, w, start, total,
                                      [&](uint32_t l) { return region + slot_words_of(l); });
#ifdef ZFP_EXP4_TRACE
  __builtin_amdgcn_s_waitcnt(0);
  ZFP_TR4(5);
  if (a.trace && (w & 63) == 0 && lane == 0) a.trace[(w >> 6) * 8 + 6] = tr0;
#endif
}

// Second pass of a short-slot encode4: the listed blocks (n entries, 16 per
// wave), each coded with a full-size slot and ORed into the stream at its
// recorded position (its first cap_bits are already there; OR is idempotent
// on them).
template <typename S, bool VEC, bool REV>
__global__ __launch_bounds__(64) void encode4_patch(const S* __restrict__ data, Geometry g, CodecParams cp,
                                                    uint64_t* __restrict__ out, const OvfEntry* __restrict__ list,
                                                    uint32_t n, uint32_t swp)
{
  using Int = typename Traits<S>::Int;
  extern __shared__ uint64_t lds[];
  uint32_t* lut = reinterpret_cast<uint32_t*>(lds);
  uint32_t* tab = lut + 256;
  uint64_t* region = lds + kEnc4HeadWords;
  const uint32_t lane = threadIdx.x;
#pragma unroll
  for (uint32_t i = 0; i < 4; i++)
    lut[lane + 64 * i] = kCoderTables.dbl[lane + 64 * i];
  tab[lane] = kOrderTab4.t[lane];
  const uint32_t qd = lane >> 2, r = lane & 3u;
  const uint64_t e = (uint64_t)blockIdx.x * kBlocks4PerWave + qd;
  const bool valid = e < n;
  const uint64_t b = valid ? list[e].b : 0ull;
  BlockPos ps{};
  S v[64];
  if (valid) {
    const BlockPos p = block_pos(g, b, 4);
    ps = slice_pos(g, p, pad_src_w((int)r, p.cnt[3]));
    gather3<S, VEC>(v, data, g, ps);
  } else {
#pragma unroll
    for (int i = 0; i < 64; i++)
      v[i] = 0;
  }
  __syncthreads();
  Int* X = reinterpret_cast<Int*>(region) + (size_t)qd * kXStride;
  auto place = [&](bool, uint32_t*& d, uint32_t& jmax) {
    d = reinterpret_cast<uint32_t*>(region + (size_t)qd * swp);
    jmax = 2 * swp - 1;
  };
  const uint32_t len = encode_block4<S, REV>(place, lut, tab, X, region, kBlocks4PerWave * swp, v, cp,
                                             [&](S (&rr)[64]) {
                                               if (valid) {
                                                 gather3<S, VEC>(rr, data, g, ps);
                                               } else {
#pragma unroll
                                                 for (int i = 0; i < 64; i++)
                                                   rr[i] = 0;
                                               }
                                             });
  __syncthreads();
  if (!valid)
    return;
  const uint64_t pos = list[e].pos;
  const uint32_t r0 = (uint32_t)(pos & 63);
  const uint32_t bits = len < 64 * swp ? len : 64 * swp;  // beyond the slot: minbits padding zeros
  const uint32_t nw = (r0 + bits + 63) >> 6;
  const uint64_t* slot = region + (size_t)qd * swp;
  for (uint32_t k = r; k < nw; k += 4) {
    const int64_t lo = (int64_t)k * 64 - r0;  // block bit at the word's bit 0
    const int64_t x0 = lo > 0 ? lo : 0;
    const int64_t x1 = lo + 64 < (int64_t)bits ? lo + 64 : (int64_t)bits;
    if (x0 < x1) {
      const uint64_t val = slot_bits(slot, (uint32_t)x0, (uint32_t)(x1 - x0)) << (x0 - lo);
      atomicOr((unsigned long long*)&out[(pos >> 6) + k], (unsigned long long)val);
    }
  }
}

// Waves per SIMD the decoder is compiled for: float blocks at 4 (<= 128 VGPRs,
// 20-32 bytes of spills; unbounded they take 131-135, i.e. 3 waves) with the
// packed staging sized to match (kDec4WavesPerCu): 128^4 f32 reversible
// decode 1.37 -> 1.09 ms; double blocks spill 750+ bytes at 128, so they are
// left unbounded.
template <typename S>
constexpr int kDec4Waves = (sizeof(S) == 4 && !kIntField<S>) ? 4 : 1;
template <typename S>
constexpr uint32_t kDec4WavesPerCu = sizeof(S) == 4 ? (kIntField<S> ? 12u : 16u) : 8u;
template <typename S, bool VEC, bool REV, bool HALF = false>
__global__ __launch_bounds__(64, kDec4Waves<S>) void decode4(S* __restrict__ data, Geometry g, CodecParams cp, DecodeArgs a)
{
  using Int = typename Traits<S>::Int;
  extern __shared__ uint64_t lds[];
  uint32_t* tab = reinterpret_cast<uint32_t*>(lds);
  uint32_t* sbit = tab + 64;
  uint64_t* region = lds + kDec4HeadWords;
  const uint32_t lane = threadIdx.x;
  tab[lane] = kOrderTab4.t[lane];
  const uint64_t w = a.wave_list ? a.wave_list[blockIdx.x] : blockIdx.x;
#ifdef ZFP_EXP4_TRACE
  const uint64_t dt0 = wall_clock64();
#define ZFP_DTR4(i) do { if (a.trace && !a.wave_list && (w & 63) == 0 && lane == 0) a.trace[(w >> 6) * 8 + (i)] = wall_clock64() - dt0; } while (0)
#else
#define ZFP_DTR4(i) ((void)0)
#endif
  const uint64_t first = w * kBlocks4PerWave;
  const uint32_t qd = lane >> 2, r = lane & 3u;
  const uint64_t b = first + qd;
  const bool valid = b < g.nblocks;
  uint64_t start;
  uint32_t pos;
  uint32_t len = 0;  // the block's index length (lane r == 0 of the quad)
  if (a.var) {
    len = (valid && r == 0u) ? a.idx_len[b] : 0u;
    pos = wave_incl_scan(len) - len;
    start = a.idx_base[w];
  } else {
    pos = qd * a.maxbits;
    start = first * (uint64_t)a.maxbits;
  }
  const uint64_t G = a.g0 + start;
  const uint64_t W0 = G >> 6;
  if (r == 0u)
    sbit[qd] = (uint32_t)(G & 63) + pos;
  __syncthreads();
  const uint64_t left = g.nblocks - first;
  const uint32_t nb = left < kBlocks4PerWave ? (uint32_t)left : kBlocks4PerWave;
  const uint32_t pairs = nb * a.W;
  uint32_t rpos = 0;  // the quad's first bit in its staged words
  const uint64_t* rbase = region + (size_t)qd * a.swp;
  if (a.packw) {
    // Packed (variable rate): the wave's blocks are contiguous in the stream,
    // so its segment is staged as is, one word per lane and step, and each
    // quad reads its block at its bit offset -- no slot sized for the worst
    // block.  A segment longer than the LDS holds (runs of long blocks) puts
    // the wave on the overflow list, decoded by the host's second launch with
    // padded slots.
    const uint32_t total = __shfl(pos + (r == 0u && valid ? (uint32_t)a.idx_len[b] : 0u), 4 * (nb - 1), 64);
    const uint32_t nwords = ((uint32_t)(G & 63) + total + 63) / 64 + 1;  // + 1: the window reads past the end
    if (nwords > a.packw) {
      if (lane == 0) {
        const uint32_t k = atomicAdd(a.ovf_count, 1u);
        if (k < a.ovf_cap)
          a.wave_ovf[k] = (uint32_t)w;
        else
          atomicOr(a.error, 2u);
      }
      return;  // wave-uniform: a one-wave workgroup
    }
    stage_batched(
        nwords,
        [&](uint32_t t) {
          const uint64_t gw = W0 + t;
          return gw < a.in_words ? a.in[gw] : 0ull;
        },
        [&](uint32_t t, uint64_t v) { region[t] = v; });
    rpos = sbit[qd];
    rbase = region;
  } else if (!a.var && (G & 63) == 0 && (a.maxbits & 63) == 0) {
    // word-aligned fixed rate (wave-uniform): block l starts at word l * bw
    const uint32_t bw = a.maxbits >> 6;
    stage_batched(
        pairs,
        [&](uint32_t t) {
          const uint32_t l = __umulhi(t, a.wmagic);
          const uint64_t gw = W0 + l * bw + (t - l * a.W);
          return gw < a.in_words ? a.in[gw] : 0ull;
        },
        [&](uint32_t t, uint64_t v) {
          const uint32_t l = __umulhi(t, a.wmagic);
          region[l * a.swp + (t - l * a.W)] = v;
        });
  } else {
    stage_batched(
        pairs,
        [&](uint32_t t) {
          const uint32_t l = __umulhi(t, a.wmagic);
          const uint32_t sb = sbit[l];
          const uint64_t gw = W0 + (sb >> 6) + (t - l * a.W);
          const uint32_t sh = sb & 63;
          const uint64_t lo = gw < a.in_words ? a.in[gw] : 0ull;
          const uint64_t hi = gw + 1 < a.in_words ? a.in[gw + 1] : 0ull;
          return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
        },
        [&](uint32_t t, uint64_t v) {
          const uint32_t l = __umulhi(t, a.wmagic);
          region[(size_t)l * a.swp + (t - l * a.W)] = v;
        });
  }
  __syncthreads();
  ZFP_DTR4(0);
  WordReader rd;
  rd.w = rbase;
  rd.pos = rpos;
  S v[64];
  Int* X = reinterpret_cast<Int*>(region) + (size_t)(HALF ? (qd & 7u) : qd) * kXStride;
  const uint32_t used = decode_block4<S, REV, HALF>(rd, v, cp, X, tab, valid);
  ZFP_DTR4(1);
#ifdef ZFP_EXP4_TRACE
  if (a.trace && !a.wave_list && (w & 63) == 0 && lane == 0)
    for (int i = 0; i < 4; i++) a.trace[(w >> 6) * 8 + 2 + i] = zfp_dmarks[i] - dt0;
#endif
  if (a.idx_bad && valid && r == 0u && used != len)
    atomicOr(a.idx_bad, 1u);
  if (!valid)
    return;
  const BlockPos p = block_pos(g, b, 4);
  if ((int)r < p.cnt[3])
    scatter3<S, VEC>(v, data, g, slice_pos(g, p, (int)r));
#ifdef ZFP_EXP4_TRACE
  __builtin_amdgcn_s_waitcnt(0);
  if (a.trace && !a.wave_list && (w & 63) == 0 && lane == 0) {
    a.trace[(w >> 6) * 8 + 6] = dt0;
    a.trace[(w >> 6) * 8 + 7] = wall_clock64() - dt0;
  }
#endif
}

}  // namespace zfp_amd
