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
// (256 dwords), order table (64), per-block offsets and written counts (16+16).
constexpr uint32_t kEnc4HeadWords = (256 + 64 + 16 + 16) / 2;
// Decoder: order table (64 dwords), per-block stream bit offsets (16).
constexpr uint32_t kDec4HeadWords = (64 + 16) / 2;

// Slot of a 4D block with budget `lim` bits: its dwords plus two spare dwords
// (targets of the clamped writes past the budget); odd, so the 16 slots of a
// wave start on different banks.
__host__ __device__ constexpr uint32_t slot_words4(uint32_t lim) { return ((((lim + 31u) >> 5) + 3u) / 2u) | 1u; }

// Overflow list of the short-slot 4D encoder: a block longer than its LDS slot
// is packed with its first cap_bits only (the rest zero) and listed with its
// stream bit position; encode4_patch codes it again with a full-size slot and
// ORs it in.  The list lives in GeneralArgs::ovf (two words per entry).
struct OvfEntry {
  uint64_t b;    // block
  uint64_t pos;  // bit position of its first bit relative to out[0]
};

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
  uint32_t* d = reinterpret_cast<uint32_t*>(region + (size_t)qd * a.swp);
  Int* X = reinterpret_cast<Int*>(region) + (size_t)(HALF ? (qd & 7u) : qd) * kXStride;
  uint32_t len = encode_block4<S, REV, HALF>(d, 2 * a.swp - 1, lut, tab, X, region, kBlocks4PerWave * a.swp, v, cp,
                                             [&](S (&rr)[64]) {
                                               if (valid) {
                                                 gather3<S, VEC>(rr, data, g, ps);
                                               } else {
#pragma unroll
                                                 for (int i = 0; i < 64; i++)
                                                   rr[i] = 0;
                                               }
                                             });
  len = valid ? len : 0u;
  const bool over = a.ovf && len > a.cap_bits;  // quad-uniform
  const uint32_t lq = r == 0u ? len : 0u;  // the quad's lanes agree on len
  const uint32_t incl = wave_incl_scan(lq);
  const uint32_t total = __shfl(incl, 63, 64);
  if (r == 0u) {
    off[qd] = incl - lq;
    wrt[qd] = over ? a.cap_bits : (len < 64 * a.swp ? len : 64 * a.swp);
  }
  uint64_t start = 0;
  if (!live) {
  } else if (a.var) {
    start = lookback_wave(a.status, w, total, a.error);
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
  if (over && r == 0u) {
    const uint32_t k = take_overflow_slot(a);
    if (k != kNoSlot)
      reinterpret_cast<OvfEntry*>(a.ovf)[k] = OvfEntry{b, a.g0 + start + (incl - lq)};
  }
  __syncthreads();
  if (!live)
    return;
  pack_wave<kBlocks4PerWave, false>(a, region, off, wrt, nullptr, w, start, total);
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
  uint32_t* d = reinterpret_cast<uint32_t*>(region + (size_t)qd * swp);
  Int* X = reinterpret_cast<Int*>(region) + (size_t)qd * kXStride;
  const uint32_t len = encode_block4<S, REV>(d, 2 * swp - 1, lut, tab, X, region, kBlocks4PerWave * swp, v, cp,
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
  WordReader rd;
  rd.w = rbase;
  rd.pos = rpos;
  S v[64];
  Int* X = reinterpret_cast<Int*>(region) + (size_t)(HALF ? (qd & 7u) : qd) * kXStride;
  const uint32_t used = decode_block4<S, REV, HALF>(rd, v, cp, X, tab, valid);
  if (a.idx_bad && valid && r == 0u && used != len)
    atomicOr(a.idx_bad, 1u);
  if (!valid)
    return;
  const BlockPos p = block_pos(g, b, 4);
  if ((int)r < p.cnt[3])
    scatter3<S, VEC>(v, data, g, slice_pos(g, p, (int)r));
}

}  // namespace zfp_amd
