// 3D encode/decode kernels: one block per lane, 4 independent waves per
// 256-thread workgroup, each wave owning 64 consecutive blocks (raster order of
// the chunk box, compress.c:86-94) and a private LDS region of per-lane slots
// (slot_words_for(budget) words each, odd stride).
//
//  encode3_aligned  fixed rate with every block starting on a 64-bit word:
//                   lane slots in LDS are copied out as one contiguous run.
//  encode3_general  any mode/alignment: blocks are packed at their bit
//                   offsets (fixed rate: analytic; variable rate: decoupled
//                   look-back over per-wave bit totals), interior words are
//                   plain stores, words shared with a neighbouring wave are
//                   handed to the fix-up kernels.
//  decode3          stages the wave's segment of the stream in LDS, then each
//                   lane decodes its block from its bit offset.
#pragma once

#include "block3.h"
#include "blockn.h"

namespace zfp_amd {

constexpr int kWavesPerGroup = 4;
constexpr size_t kLutBytes = 256 * sizeof(uint32_t);  // static LDS of the encoders
constexpr uint64_t kNoWord = ~0ull;

struct Partial {
  uint64_t idx;  // stream word index relative to the kernel's `out`
  uint64_t val;
};

// inclusive prefix sum across the 64 lanes of a wave
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x)
{
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  return x;
}

// Kernel prologue shared by the encoders: the doubled-ones table (one entry
// per thread of the 256-thread group) and the wave's zeroed slot region.
__device__ __forceinline__ void encode_prologue(uint32_t* lut, uint64_t* wslot, uint32_t words)
{
  lut[threadIdx.x] = kCoderTables.dbl[threadIdx.x];
  const int lane = threadIdx.x & 63;
  uint4* z = reinterpret_cast<uint4*>(wslot);
  for (uint32_t i = lane; i < words / 2; i += 64)
    z[i] = make_uint4(0, 0, 0, 0);
  if ((words & 1) && lane == 0)
    wslot[words - 1] = 0;
  __syncthreads();
}

// floor(i / d) for i < 2^20, d < 2^12 with m = ceil(2^32 / d) (m = 0 for d = 1)
__device__ __forceinline__ uint32_t div_magic(uint32_t i, uint32_t m) { return m ? __umulhi(i, m) : i; }

// ---------------------------------------------------------------------------
// Fixed rate, block size a multiple of 64 bits (sw words).  The wave's 64
// blocks form one contiguous run of words; with a stream offset r0 = g0
// (mod 64) != 0 every output word is a funnel shift of two run words, and the
// run's first and last words (shared with neighbouring waves) go to the
// fix-up kernels.  Lane slots are sdw dwords apart (odd: the 32 lanes of a
// ds_or_b32 half-wave at the same slot offset hit 32 different banks),
// sdw >= slot_dwords_for(64 sw); dwords from 2 sw on are spare (bits past the
// budget) and never copied.  magic_w / magic_c: ceil(2^32 / d) for d = sw and
// d = sw / 2 (0 for d = 1).
__host__ __device__ constexpr uint32_t slot_dwords_for(uint32_t lim) { return (lim + 95u) / 32u + 1u; }

// (ZFP_NT_STORE, block3.h: the stream is written once and not read back)

template <typename S, bool VEC, bool REV, int WPG = kWavesPerGroup>
__global__ __launch_bounds__(64 * WPG, 3) void encode3_aligned(const S* __restrict__ data, Geometry g, CodecParams cp,
                                                       uint64_t* __restrict__ out, uint32_t sw, uint32_t sdw,
                                                       uint32_t magic_w, uint32_t magic_c, uint32_t r0,
                                                       Partial* __restrict__ partials)
{
  __shared__ uint32_t lut[512];  // CoderTables: dbl[256], lead[256]
  extern __shared__ uint32_t ldsw[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint32_t* wslot = ldsw + (size_t)wv * 64 * sdw;
  const uint64_t w = (uint64_t)blockIdx.x * WPG + wv;
  const uint64_t first = w * 64;
  const uint64_t b = first + lane;
  // the block loads are in flight while the wave copies the coder tables from
  // device memory and zeroes its slots: every wave writes the whole (identical)
  // tables, so no workgroup barrier is needed
  S v[64];
  BlockPos p{};
  // the block loads go out at wave priority 1, ahead of the coding waves
  // (C4 chunk 1.25-1.27 -> 1.20-1.22 ms, profiles/r4s_prio_ab.txt)
  __builtin_amdgcn_s_setprio(1);
  if (b < g.nblocks) {
    p = block_pos(g, b, 3);
    gather3<S, VEC>(v, data, g, p);
  }
  __builtin_amdgcn_s_setprio(0);
  {
    const uint4* src = reinterpret_cast<const uint4*>(&kCoderTables);
    uint4* dst = reinterpret_cast<uint4*>(lut);
    dst[lane] = src[lane];
    dst[lane + 64] = src[lane + 64];
    uint4* z = reinterpret_cast<uint4*>(wslot);
    for (uint32_t i = lane; i < 16 * sdw; i += 64)
      z[i] = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) only (vmcnt/expcnt at max)
    __builtin_amdgcn_wave_barrier();
  }
  if (b < g.nblocks) {
    OrSlot os{reinterpret_cast<uint64_t*>(wslot + (size_t)lane * sdw), sdw - 1};
    encode_block3<S, REV, true>(os, lut, v, cp, [&](S (&r)[64]) { gather3<S, VEC>(r, data, g, p); });
  }
  if (first >= g.nblocks)
    return;
  // slots are read across lanes of this wave only: LDS ops of a wave complete in order
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const uint64_t nb = (g.nblocks - first) < 64 ? (g.nblocks - first) : 64;
  const uint32_t total = (uint32_t)nb * sw;  // run length in words
  uint64_t* dst = out + first * sw;
  // word i of the wave's run
  auto run_word = [&](uint32_t i) -> uint64_t {
    const uint32_t l = div_magic(i, magic_w);
    const uint32_t* s = wslot + (size_t)l * sdw + 2 * (i - l * sw);
    return (uint64_t)s[0] | ((uint64_t)s[1] << 32);
  };
  if (r0 == 0) {
    if ((sw & 1) == 0) {
      // 16-byte stores: dword quads never straddle two slots
      const uint32_t hw = sw >> 1, chunks = (uint32_t)nb * hw;
      for (uint32_t c = lane; c < chunks; c += 64) {
        const uint32_t l = div_magic(c, magic_c);
        const uint32_t* s = wslot + (size_t)l * sdw + 4 * (c - l * hw);
#if ZFP_NT_STORE && defined(__HIP_DEVICE_COMPILE__)
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(u4{s[0], s[1], s[2], s[3]}, reinterpret_cast<u4*>(dst + 2 * c));
#else
        *reinterpret_cast<uint4*>(dst + 2 * c) = make_uint4(s[0], s[1], s[2], s[3]);
#endif
      }
    } else {
      for (uint32_t i = lane; i < total; i += 64)
        dst[i] = run_word(i);
    }
    return;
  }
  // run words j = 0..total-1 land at bit r0 + 64 j of out[first*sw ...]: out
  // word o (o = 0..total) holds bits of run words o-1 and o; words 0 and total
  // are shared with the neighbouring waves (partials).
  if ((sw & 1) == 0) {
    // 16-byte stores of out-word pairs aligned in memory: (o0 + 2c, o0 + 2c + 1)
    // with o0 = 1 when dst is 8 (mod 16).  In dwords, with D the run's dwords
    // and j = ceil(r0 / 32), out dword k = alignbit(D[k-j+1], D[k-j], 32j - r0).
    // A pair reads its chunk's four run dwords (one slot) and the neighbouring
    // run word: the previous one (o0 = 0) or the next one (o0 = 1).
    const uint32_t hw = sw >> 1, chunks = (uint32_t)nb * hw;
    const uint32_t jj = (r0 + 31u) >> 5, sh = 32u * jj - r0;
    const uint32_t o0 = (uint32_t)(reinterpret_cast<uintptr_t>(dst) >> 3) & 1u;
    for (uint32_t c = lane; c < chunks; c += 64) {
      const uint32_t l = div_magic(c, magic_c), cs = c - l * hw;
      const uint32_t* s = wslot + (size_t)l * sdw + 4 * cs;
      uint32_t X[6];
      if (o0 == 0) {
        // run word 2c - 1: the previous chunk's, or the last word of slot l - 1
        const uint32_t* q = cs ? s - 2 : wslot + (size_t)(l ? l - 1 : 0) * sdw + 2 * sw - 2;
        X[0] = c ? q[0] : 0u;
        X[1] = c ? q[1] : 0u;
        X[2] = s[0], X[3] = s[1], X[4] = s[2], X[5] = s[3];
      } else {
        // run word 2c + 2: the next chunk's, or the first word of slot l + 1
        const bool in_run = 2 * c + 2 < total;
        const uint32_t* q = cs + 1 < hw ? s + 4 : wslot + (size_t)(in_run ? l + 1 : l) * sdw;
        X[0] = s[0], X[1] = s[1], X[2] = s[2], X[3] = s[3];
        X[4] = in_run ? q[0] : 0u;
        X[5] = in_run ? q[1] : 0u;
      }
      // out dwords 2 o0 + 4c + i, i = 0..3 (X[0] is run dword 2 o0 + 4c - 2)
      uint32_t y[4];
#pragma unroll
      for (int i = 0; i < 4; i++)
        y[i] = jj == 1 ? __builtin_amdgcn_alignbit(X[i + 2], X[i + 1], sh) : __builtin_amdgcn_alignbit(X[i + 1], X[i], sh);
      const uint32_t o = o0 + 2 * c;  // first out word of the pair
      const uint64_t v0 = ((uint64_t)y[1] << 32) | y[0], v1 = ((uint64_t)y[3] << 32) | y[2];
      if (o == 0) {
        partials[2 * w] = Partial{first * sw, v0};
        dst[1] = v1;
      } else if (o + 1 == total) {
        dst[o] = v0;
        partials[2 * w + 1] = Partial{first * sw + total, v1};
      } else {
#if ZFP_NT_STORE && defined(__HIP_DEVICE_COMPILE__)
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(u4{y[0], y[1], y[2], y[3]}, reinterpret_cast<u4*>(dst + o));
#else
        *reinterpret_cast<uint4*>(dst + o) = make_uint4(y[0], y[1], y[2], y[3]);
#endif
      }
    }
    if (lane == 0) {
      // the word no pair covers: the tail (o0 = 0) or the head (o0 = 1)
      if (o0 == 0)
        partials[2 * w + 1] = Partial{first * sw + total, run_word(total - 1) >> (64 - r0)};
      else
        partials[2 * w] = Partial{first * sw, run_word(0) << r0};
    }
    return;
  }
  for (uint32_t j = lane; j <= total; j += 64) {
    const uint64_t cur = j < total ? run_word(j) : 0ull;
    const uint64_t prev = j > 0 ? run_word(j - 1) : 0ull;
    const uint64_t val = (cur << r0) | (prev >> (64 - r0));
    if (j == 0) {
      partials[2 * w] = Partial{first * sw, val};
    } else if (j == total) {
      partials[2 * w + 1] = Partial{first * sw + total, val};
    } else {
      dst[j] = val;
    }
  }
}

// The common case of encode3_aligned on its own: whole workgroups of full
// waves (nblocks a multiple of 256), a word-aligned stream start and an even
// number of words per block (C2: 1024^3 at rate 16).  Same blocks and bits; the
// block loads are issued at wave priority 1 (so a wave that starts while others
// code gets its 16 loads out first) and the copy-out has no edge cases.
// Measured 3-5 % faster than encode3_aligned on the same launch (round 4,
// tools/exp/c2var.hip `pf0 p1`); the launcher picks it when it applies.
template <typename S, bool VEC>
__global__ __launch_bounds__(256, 3) void encode3_aligned_full(const S* __restrict__ data, Geometry g, CodecParams cp,
                                                            uint64_t* __restrict__ out, uint32_t sw, uint32_t sdw,
                                                            uint32_t magic_c)
{
  __shared__ uint32_t lut[512];  // CoderTables: dbl[256], lead[256]
  extern __shared__ uint32_t ldsw[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint32_t* wslot = ldsw + (size_t)wv * 64 * sdw;
  const uint64_t w = (uint64_t)blockIdx.x * kWavesPerGroup + wv;
  const uint64_t first = w * 64;
  const uint64_t b = first + lane;
  S v[64];
  __builtin_amdgcn_s_setprio(1);
  const BlockPos p = block_pos(g, b, 3);
  gather3<S, VEC>(v, data, g, p);
  __builtin_amdgcn_s_setprio(0);
  {
    const uint4* src = reinterpret_cast<const uint4*>(&kCoderTables);
    uint4* dst = reinterpret_cast<uint4*>(lut);
    dst[lane] = src[lane];
    dst[lane + 64] = src[lane + 64];
    uint4* z = reinterpret_cast<uint4*>(wslot);
    for (uint32_t i = lane; i < 16 * sdw; i += 64)
      z[i] = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) only
    __builtin_amdgcn_wave_barrier();
  }
  OrSlot os{reinterpret_cast<uint64_t*>(wslot + (size_t)lane * sdw), sdw - 1};
  encode_block3<S, false, true>(os, lut, v, cp, [&](S (&r)[64]) { gather3<S, VEC>(r, data, g, p); });
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const uint32_t hw = sw >> 1, chunks = 64 * hw;
  uint64_t* dst = out + first * sw;
  for (uint32_t c = lane; c < chunks; c += 64) {
    const uint32_t l = div_magic(c, magic_c);
    const uint32_t* s = wslot + (size_t)l * sdw + 4 * (c - l * hw);
#if ZFP_NT_STORE && defined(__HIP_DEVICE_COMPILE__)
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(u4{s[0], s[1], s[2], s[3]}, reinterpret_cast<u4*>(dst + 2 * c));
#else
    *reinterpret_cast<uint4*>(dst + 2 * c) = make_uint4(s[0], s[1], s[2], s[3]);
#endif
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
}

// ---------------------------------------------------------------------------
// Extract `cnt` (<= 64) bits starting at bit `pos` of a lane slot.
__device__ __forceinline__ uint64_t slot_bits(const uint64_t* slot, uint32_t pos, uint32_t cnt)
{
  uint32_t i = pos >> 6, r = pos & 63;
  uint64_t v = slot[i] >> r;
  if (r && r + cnt > 64)
    v |= slot[i + 1] << (64 - r);
  return v & low_mask(cnt);
}

// slot_bits from an overflow slot: L2 reads (its words were written by other
// lanes' atomics)
__device__ __forceinline__ uint64_t slot_bits_l2(uint64_t* slot, uint32_t pos, uint32_t cnt)
{
  uint32_t i = pos >> 6, r = pos & 63;
  uint64_t v = __hip_atomic_load(slot + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> r;
  if (r && r + cnt > 64)
    v |= __hip_atomic_load(slot + i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) << (64 - r);
  return v & low_mask(cnt);
}

struct GeneralArgs {
  uint64_t* out;          // stream words, index 0 = word containing bit g0
  uint32_t g0;            // start bit within out[0]
  uint32_t swp;           // slot stride (words) per lane
  uint32_t var;           // 1: variable rate (look-back), 0: fixed rate
  uint32_t maxbits;       // fixed rate block size
  uint64_t* status;       // per-wave look-back words (zeroed per launch)
  uint32_t* ticket;       // wave ticket counter (zeroed per launch)
  Partial* partials;      // 2 per wave
  uint16_t* idx_len;      // per-block bit lengths (variable rate; optional)
  uint64_t* idx_base;     // per-wave start offsets relative to g0 (optional)
  uint64_t* total_bits;   // written by the last wave (variable rate)
  uint32_t* error;        // bit 0: look-back timeout; bit 1: overflow pool exhausted
  uint64_t idx_add;       // added to the index bases (offset of this launch in its chunk)
  // Short LDS slots (variable rate): a slot of swp words holds cap_bits intact
  // bits; a block that codes longer is coded again into a full-size slot
  // (ovf_swp words) of the overflow pool in global memory.  ovf == nullptr:
  // the LDS slots are full size.
  uint64_t* ovf;
  uint32_t* ovf_count;    // pool slots handed out (zeroed per launch)
  uint32_t ovf_cap;       // pool slots
  uint32_t ovf_swp;       // words per pool slot
  uint32_t cap_bits;      // intact bits of an LDS slot
#ifdef ZFP_EXP4_TRACE
  uint64_t* trace;        // experiment: per-phase clocks of every 64th wave (encode4)
#endif
};

// Overflow slot of a lane whose block did not fit its LDS slot: ~0u when none
// (or when the pool is exhausted: the error flag makes the host redo the
// launch with full-size slots).
constexpr uint32_t kNoSlot = ~0u;

__device__ __forceinline__ uint32_t take_overflow_slot(const GeneralArgs& a)
{
  uint32_t oi = atomicAdd(a.ovf_count, 1u);
  if (oi >= a.ovf_cap) {
    atomicOr(a.error, 2u);
    oi = kNoSlot;
  }
  return oi;
}

__device__ __forceinline__ void zero_words(uint64_t* p, uint32_t n)
{
  for (uint32_t i = 0; i < n; i++)
    p[i] = 0;
}

constexpr uint64_t kStAgg = 1ull << 62;
constexpr uint64_t kStIncl = 2ull << 62;
constexpr uint64_t kStMask = (1ull << 62) - 1;

// Decoupled look-back (single-pass chained scan, lookback_wave below): each
// wave publishes its aggregate, walks back over predecessors' status words
// until an inclusive prefix, publishes its own inclusive prefix.  Status words
// are the data (one 8-byte agent-scope atomic store/load each), so no separate
// flag or fence is needed; waves take tickets in launch order so every awaited
// wave is already running.  Spins are bounded (error flag on timeout).

// One lane walks back (lane 0 returns the prefix).  The f64 encoders keep this
// form: their waves are few and slow, a predecessor has nearly always published
// its inclusive prefix, and the wave-wide window measured slower there (C3).
__device__ __forceinline__ uint64_t lookback_lane(uint64_t* status, uint64_t w, uint32_t agg, uint32_t* error)
{
  uint64_t excl = 0;
  if (w == 0) {
    __hip_atomic_store(&status[0], kStIncl | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  __hip_atomic_store(&status[w], kStAgg | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t j = w - 1;
  uint32_t spins = 0;
  for (;;) {
    const uint64_t st = __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t tag = st & ~kStMask;
    if (tag == 0) {
      if (++spins > (1u << 26)) {
        atomicOr(error, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    excl += st & kStMask;
    if (tag == kStIncl || j == 0)
      break;
    j--;
  }
  __hip_atomic_store(&status[w], kStIncl | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

// wave-wide sum of a 64-bit value
__device__ __forceinline__ uint64_t wave_sum64(uint64_t x)
{
#pragma unroll
  for (int d = 1; d < 64; d <<= 1)
    x += __shfl_xor(x, d, 64);
  return x;
}

// The look-back runs on the whole wave: lane l inspects predecessor
// top - l, so one round trip to L2 covers 64 predecessors.  With thousands of
// waves resident, the predecessors of a wave have mostly published only their
// aggregates when it looks back (their own look-backs are still walking), and
// a one-lane walk pays one round trip per predecessor, holding the wave's slots
// meanwhile; the window makes that chain 64 times shorter.  Called by every
// lane of the wave with the same arguments.
// First half of lookback_wave: publish the wave's aggregate (wave 0: its
// inclusive prefix), so successors can look past it while it does other work.
__device__ __forceinline__ void lookback_publish(uint64_t* status, uint64_t w, uint32_t agg)
{
  if ((threadIdx.x & 63u) == 0)
    __hip_atomic_store(&status[w], (w == 0 ? kStIncl : kStAgg) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Second half: walk back to an inclusive prefix, publish the wave's own.
__device__ __forceinline__ uint64_t lookback_walk(uint64_t* status, uint64_t w, uint32_t agg, uint32_t* error)
{
  const uint32_t lane = threadIdx.x & 63u;
  if (w == 0)
    return 0;
  uint64_t excl = 0;
  int64_t top = (int64_t)w - 1;
  uint32_t spins = 0;
  for (;;) {
    const int64_t j = top - (int64_t)lane;
    // before wave 0: an inclusive zero
    const uint64_t st = j >= 0 ? __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kStIncl;
    const uint64_t tag = st & ~kStMask;
    const uint64_t incl = __builtin_amdgcn_ballot_w64(tag == kStIncl);
    const uint32_t m = incl ? (uint32_t)__builtin_ctzll(incl) : 64u;  // nearest inclusive prefix
    const uint64_t need = m < 63u ? ((2ull << m) - 1ull) : ~0ull;     // lanes 0 .. m
    if (__builtin_amdgcn_ballot_w64(tag == 0) & need) {  // a predecessor has not published yet
      if (++spins > (1u << 24)) {
        if (lane == 0)
          atomicOr(error, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    excl += wave_sum64(lane <= m ? (st & kStMask) : 0ull);
    if (m < 64u)
      break;
    top -= 64;
  }
  if (lane == 0)
    __hip_atomic_store(&status[w], kStIncl | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

__device__ __forceinline__ uint64_t lookback_wave(uint64_t* status, uint64_t w, uint32_t agg, uint32_t* error)
{
  lookback_publish(status, w, agg);
  return lookback_walk(status, w, agg, error);
}

template <int NB, bool OVF, typename SlotOf>
__device__ __forceinline__ void pack_wave(const GeneralArgs& a, const uint64_t* wbase, const uint32_t* off,
                                          const uint32_t* wrt, const uint32_t* ovi, uint64_t w, uint64_t start,
                                          uint32_t total, SlotOf&& slot_of);

// Waves per SIMD the general encoder is compiled for: the f64 kernels that code
// planes 32..63 fit three (<= 168 VGPRs, 48 bytes of spills) when their LDS
// slots are short (launch_encode) -- C3 4.44 ms, against 5.44 ms at two waves
// without spills (profiles/r4u_gw2_ab.txt); the others are not bounded.
template <typename S, bool REV, bool HI>
constexpr int kGenWaves = (sizeof(S) == 8 && HI) ? 3 : 1;

// Per-wave LDS of encode3_general: 64 slots of swp words, then 64 offsets, 64
// written counts and 64 overflow slot numbers (uint32).
__host__ __device__ constexpr uint32_t gen_wave_words(uint32_t swp) { return 64 * swp + 96; }

// HI: double with maxprec <= 32 (planes 32..63 only, block3.h encode_ints3).
// D: block dimensionality; 1D/2D blocks and integer fields take the generic
// per-lane codec (blockn.h).
template <typename S, bool VEC, bool REV, bool HI = false, int D = 3>
__global__ __launch_bounds__(256, (kGenWaves<S, REV, HI>)) void encode3_general(const S* __restrict__ data,
                                                                               Geometry g, CodecParams cp,
                                                                               GeneralArgs a)
{
  __shared__ uint32_t lut[256];
  extern __shared__ uint64_t lds[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint64_t* wbase = lds + (size_t)wv * gen_wave_words(a.swp);
  uint32_t* off = reinterpret_cast<uint32_t*>(wbase + 64 * a.swp);
  uint32_t* wrt = off + 64;
  uint32_t* ovi = wrt + 64;
  encode_prologue(lut, wbase, 64 * a.swp);

  const uint64_t nwaves = (g.nblocks + 63) / 64;
  uint64_t w;
  if (a.var) {
    uint32_t t = 0;
    if (lane == 0)
      t = atomicAdd(a.ticket, 1u);
    w = (uint64_t)__shfl(t, 0, 64);
  } else {
    w = (uint64_t)blockIdx.x * kWavesPerGroup + wv;
  }
  const bool live = w < nwaves;
  const uint64_t first = w * 64;
  const uint64_t b = first + lane;
  const bool act = live && b < g.nblocks;

  // code the lane's block into `os`: the LDS slot, or an overflow slot
  // (inlined at both sites: the LDS copy must keep its ds_or writes)
  auto code = [&](OrSlot& os) __attribute__((always_inline)) -> uint32_t {
    S v[64];
    BlockPos p = block_pos(g, b, D);
    if constexpr (D == 3 && !kIntField<S>) {
      gather3<S, VEC>(v, data, g, p);
      return encode_block3<S, REV, false, HI>(os, lut, v, cp, [&](S (&r)[64]) { gather3<S, VEC>(r, data, g, p); });
    } else {
      gather_n<S, D>(v, data, g, p);
      return encode_block_n<S, D, REV>(os, lut, v, cp);
    }
  };
  uint32_t len = 0;
  if (act) {
    OrSlot os{wbase + (size_t)lane * a.swp, 2 * a.swp - 1};
    len = code(os);
  }
  const uint32_t incl = wave_incl_scan(len);
  const uint32_t excl_l = incl - len;
  const uint32_t total = __shfl(incl, 63, 64);
  off[lane] = excl_l;
  // bits below the budget are exact (past it the slot holds spill); beyond the
  // slot a block can only hold minbits padding zeros
  wrt[lane] = len < 64 * a.swp ? len : 64 * a.swp;

  uint64_t start = 0;  // bit offset of the wave's first block relative to g0
  if (!live) {
  } else if (a.var) {
    if constexpr (sizeof(S) == 8) {
      uint64_t e = 0;
      if (lane == 0)
        e = lookback_lane(a.status, w, total, a.error);
      start = __shfl(e, 0, 64);
    } else {
      start = lookback_wave(a.status, w, total, a.error);
    }
    if (a.idx_len && b < g.nblocks)
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
  if (!live)
    return;
  // Blocks longer than their short LDS slot (wave-uniform, rare on smooth
  // data): coded again into full-size overflow slots, after the look-back so
  // that no successor waits for it.
  const bool over = a.ovf && act && len > a.cap_bits;
  const bool spill = __any(over);
  if (spill) {
    uint32_t oi = kNoSlot;
    if (over) {
      oi = take_overflow_slot(a);
      if (oi != kNoSlot) {
        uint64_t* gs = a.ovf + (size_t)oi * a.ovf_swp;
        zero_words(gs, a.ovf_swp);
        OrSlot os{gs, 2 * a.ovf_swp - 1};
        code(os);
        wrt[lane] = len < 64 * a.ovf_swp ? len : 64 * a.ovf_swp;
      }
    }
    ovi[lane] = oi;
  }
  // off/wrt and the slots are this wave's own: LDS ops of a wave complete in order
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (spill) {
    __threadfence();  // the overflow slots' atomics have landed before they are read
    pack_wave<64, true>(a, wbase, off, wrt, ovi, w, start, total,
                        [&](uint32_t l) { return wbase + (size_t)l * a.swp; });
  } else {
    pack_wave<64, false>(a, wbase, off, wrt, ovi, w, start, total,
                         [&](uint32_t l) { return wbase + (size_t)l * a.swp; });
  }
}

// Pack the NB block slots of one wave (bit lengths wrt[], bit offsets off[]
// relative to the wave's first bit) into the stream words of [G, G + total),
// G = g0 + start: interior words are plain stores, the first and last word
// (shared with the neighbouring waves) go to the partials for the fix-up
// kernels.  Shared by encode3_general (NB = 64) and encode4 (NB = 16).
// OVF: some blocks of the wave sit in overflow slots (ovi[l] != kNoSlot).
// slot_of(l): the first word of block l's slot.
template <int NB, bool OVF, typename SlotOf>
__device__ __forceinline__ void pack_wave(const GeneralArgs& a, const uint64_t* wbase, const uint32_t* off,
                                          const uint32_t* wrt, const uint32_t* ovi, uint64_t w, uint64_t start,
                                          uint32_t total, SlotOf&& slot_of)
{
  const int lane = threadIdx.x & 63;
  const uint64_t G = a.g0 + start;
  const uint64_t W0 = G >> 6;
  const uint32_t r0 = (uint32_t)(G & 63);
  const uint64_t end = G + total;
  const uint64_t W1 = (end - 1) >> 6;
  const uint32_t nw = (uint32_t)(W1 - W0 + 1);
  for (uint32_t o = lane; o < nw; o += 64) {
    // local bit range of this word relative to the wave's first bit
    int64_t lo = (int64_t)o * 64 - r0;
    int64_t hi = lo + 64;
    // first block that ends after lo
    int l = 0;
    {
      int lo_i = 0, hi_i = NB - 1;
      int64_t key = lo < 0 ? 0 : lo;
      while (lo_i < hi_i) {
        int mid = (lo_i + hi_i + 1) >> 1;
        if ((int64_t)off[mid] <= key) lo_i = mid;
        else hi_i = mid - 1;
      }
      l = lo_i;
    }
    uint64_t val = 0;
    for (; l < NB && (int64_t)off[l] < hi; l++) {
      int64_t s0 = off[l];
      int64_t s1 = s0 + wrt[l];
      int64_t x0 = s0 > lo ? s0 : lo;
      int64_t x1 = s1 < hi ? s1 : hi;
      if (x0 < x1) {
        const uint32_t sp = (uint32_t)(x0 - s0), cnt = (uint32_t)(x1 - x0);
        uint64_t bits;
        if (OVF && ovi[l] != kNoSlot)
          bits = slot_bits_l2(a.ovf + (size_t)ovi[l] * a.ovf_swp, sp, cnt);
        else
          bits = slot_bits(slot_of((uint32_t)l), sp, cnt);
        val |= bits << (x0 - lo);
      }
    }
    bool head = (o == 0) && (r0 != 0 || (nw == 1 && (end & 63)));
    bool tail = (o == nw - 1) && (end & 63);
    if (head || tail) {
      Partial pr;
      pr.idx = W0 + o;
      pr.val = val;
      a.partials[2 * w + (o == 0 ? 0 : 1)] = pr;
    } else {
      a.out[W0 + o] = val;
    }
  }
  if (lane == 0) {
    bool head = r0 != 0 || (nw == 1 && (end & 63));
    bool tail = (end & 63) != 0;
    if (!head)
      a.partials[2 * w].idx = kNoWord;
    if (!tail || nw == 1)
      a.partials[2 * w + 1].idx = kNoWord;
  }
}

// Zero every word that receives partial contributions (the word holding the
// stream's pending bits below g0 gets those bits instead), then OR them in.
// `head_keep` selects bits of the head word's current device value to keep
// (a host slab pipeline: the bits the previous slab wrote below g0).
static __global__ void fixup_zero(const Partial* __restrict__ partials, uint64_t n, uint64_t* out, uint64_t head_idx,
                           uint64_t head_val, uint64_t head_keep)
{
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  uint64_t idx = partials[i].idx;
  if (idx != kNoWord)
    out[idx] = (idx == head_idx) ? ((out[idx] & head_keep) | head_val) : 0ull;
}

static __global__ void fixup_or(const Partial* __restrict__ partials, uint64_t n, uint64_t* out)
{
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n)
    return;
  Partial p = partials[i];
  if (p.idx != kNoWord)
    atomicOr((unsigned long long*)&out[p.idx], (unsigned long long)p.val);
}

// ---------------------------------------------------------------------------
struct DecodeArgs {
  const uint64_t* in;      // stream words, index 0 = word containing bit g0
  uint64_t in_words;       // readable words from `in`
  uint32_t g0;
  uint32_t var;
  uint32_t maxbits;
  uint32_t W;              // words staged per block (block bound + 1)
  uint32_t swp;            // LDS slot stride (odd, >= W)
  uint32_t wmagic;         // ceil(2^32 / W)
  const uint16_t* idx_len;
  const uint64_t* idx_base;
  // Short LDS slots (variable rate): a block longer than cap_bits is staged
  // into an overflow slot of ovf_W words in global memory instead.
  uint64_t* ovf;
  uint32_t* ovf_count;
  uint32_t* error;       // bit 1: overflow pool exhausted (the host redoes the launch)
  uint32_t ovf_cap;
  uint32_t ovf_W;
  uint32_t cap_bits;
  // decode4, variable rate: the wave's blocks staged back to back (packw words
  // of LDS at most; 0: one padded slot per block).  A wave whose segment is
  // longer appends its number to wave_ovf (count in ovf_count, capacity
  // ovf_cap; bit 1 of *error when full) and is decoded by a second launch
  // with padded slots over that list (wave_list: the waves of this launch,
  // nullptr = 0 .. grid - 1).
  uint32_t packw;
  uint32_t* wave_ovf;
  const uint32_t* wave_list;
  // Variable rate with a caller-supplied index: every block's decoded length
  // is compared with its index entry and *idx_bad set on a difference (the
  // index was made for another stream; the host decodes again after a scan).
  // Equal lengths for every block prove the index right: block 0 starts at the
  // stream start, and each next start is the previous start plus its length.
  uint32_t* idx_bad;
#ifdef ZFP_EXP4_TRACE
  uint64_t* trace;  // experiment: per-phase clocks of every 64th wave (decode4)
#endif
};

// Copy n 64-bit items to LDS, item t = lane + 64 i per lane: U loads are issued
// before their stores, so U memory round trips overlap (a loop with a store
// after every load waits out one full round trip per item).
#ifndef ZFP_STAGE_BATCH
#define ZFP_STAGE_BATCH 8
#endif
template <int U = ZFP_STAGE_BATCH, typename Load, typename Store>
__device__ __forceinline__ void stage_batched(uint32_t n, Load&& load, Store&& store)
{
  const uint32_t lane = threadIdx.x & 63u;
  for (uint32_t base = 0; base < n; base += 64u * U) {
    uint64_t v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t t = base + lane + 64u * u;
      v[u] = t < n ? load(t) : 0ull;
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t t = base + lane + 64u * u;
      if (t < n)
        store(t, v[u]);
    }
  }
}

// Each lane's block is staged into its own LDS slot (odd stride: lanes reading
// the same offset of their blocks hit different banks), funnel-shifted so the
// block starts at bit 0.  Staging is cooperative: thread t copies word j of
// block l for t = l*W + j, so consecutive threads read consecutive stream words.
// SHORT: short staging slots with the global overflow path (instantiated for
// the f64 planes-32..63 decoder only, which then fits three waves per SIMD; a
// second inlined decoder costs the others registers).
template <typename S, bool VEC, bool REV, bool HI = false, int D = 3, bool SHORT = false>
__global__ __launch_bounds__(256, SHORT ? 3 : 1) void decode3(S* __restrict__ data, Geometry g, CodecParams cp,
                                                             DecodeArgs a)
{
  __shared__ uint32_t sq[256];
  __shared__ uint32_t sbit[kWavesPerGroup * 64];
  extern __shared__ uint64_t lds[];
  const int lane = threadIdx.x & 63;
  // every wave writes the whole (identical) table: no workgroup barrier below
#pragma unroll
  for (int k = 0; k < 4; k++)
    sq[lane + 64 * k] = squeeze_entry(lane + 64 * k);
  const int wv = threadIdx.x >> 6;
  uint64_t* wslot = lds + (size_t)wv * 64 * a.swp;
  const uint64_t w = (uint64_t)blockIdx.x * kWavesPerGroup + wv;
  const uint64_t first = w * 64;
  const bool live = first < g.nblocks;
  const uint64_t b = first + lane;
  const bool act = b < g.nblocks;

  uint64_t start = 0;
  uint32_t pos = 0, len = 0;
  if (!live) {
  } else if (a.var) {
    len = act ? a.idx_len[b] : 0u;
    uint32_t incl = wave_incl_scan(len);
    pos = incl - len;
    start = a.idx_base[w];
  } else {
    pos = lane * a.maxbits;
    start = first * (uint64_t)a.maxbits;
  }
  const uint64_t G = a.g0 + start;
  const uint64_t W0 = G >> 6;
  sbit[threadIdx.x] = (uint32_t)(G & 63) + pos;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const uint64_t nb = live ? ((g.nblocks - first) < 64 ? (g.nblocks - first) : 64) : 0;
  const uint32_t pairs = (uint32_t)nb * a.W;
  auto slot_of = [&](uint32_t t) -> uint64_t* {
    const uint32_t l = __umulhi(t, a.wmagic);
    return wslot + (size_t)l * a.swp + (t - l * a.W);
  };
  if (!a.var && (G & 63) == 0 && (a.maxbits & 63) == 0) {
    // word-aligned fixed rate (wave-uniform): block l starts at word l * bw
    const uint32_t bw = a.maxbits >> 6;
    stage_batched(
        pairs,
        [&](uint32_t t) {
          const uint32_t l = __umulhi(t, a.wmagic);
          const uint64_t gw = W0 + l * bw + (t - l * a.W);
          return gw < a.in_words ? a.in[gw] : 0ull;
        },
        [&](uint32_t t, uint64_t v) { *slot_of(t) = v; });
  } else {
    stage_batched(
        pairs,
        [&](uint32_t t) {
          const uint32_t l = __umulhi(t, a.wmagic);
          const uint32_t sb = sbit[wv * 64 + l];
          const uint64_t gw = W0 + (sb >> 6) + (t - l * a.W);
          const uint32_t sh = sb & 63;
          const uint64_t lo = gw < a.in_words ? a.in[gw] : 0ull;
          const uint64_t hi = gw + 1 < a.in_words ? a.in[gw + 1] : 0ull;
          return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
        },
        [&](uint32_t t, uint64_t v) { *slot_of(t) = v; });
  }
  // Blocks longer than a short slot (wave-uniform, rare on smooth data): the
  // lane stages its whole block into an overflow slot in global memory.
  const bool over = SHORT && act && len > a.cap_bits;
  uint64_t* gs = nullptr;
  if (__any(over) && over) {
    const uint32_t oi = atomicAdd(a.ovf_count, 1u);
    if (oi < a.ovf_cap) {
      gs = a.ovf + (size_t)oi * a.ovf_W;
      const uint32_t sb = sbit[threadIdx.x];
      const uint32_t sh = sb & 63;
      for (uint32_t j = 0; j < a.ovf_W; j++) {
        const uint64_t gw = W0 + (sb >> 6) + j;
        const uint64_t lo = gw < a.in_words ? a.in[gw] : 0ull;
        const uint64_t hi = gw + 1 < a.in_words ? a.in[gw + 1] : 0ull;
        gs[j] = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
      }
    } else {
      atomicOr(a.error, 2u);
    }
  }
  // the staged slots and the table are this wave's own writes
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  if (!act)
    return;
  // (inlined at both sites: the LDS copy must keep its ds_read accesses; the
  // block's position is computed after the decode, not held across it)
  auto dec = [&](WordReader& r) __attribute__((always_inline)) {
    S v[64];
    uint32_t used;
    if constexpr (D == 3 && !kIntField<S>) {
      used = decode_block3<S, REV, HI>(r, sq, v, cp);
      scatter3<S, VEC>(v, data, g, block_pos(g, b, D));
    } else {
      used = decode_block_n<S, D, REV>(r, sq, v, cp);
      scatter_n<S, D>(v, data, g, block_pos(g, b, D));
    }
    // (every decoder, the short-slot f64 one included: at its register bound
    // the check moved its spills into the plane loop, C3 decode 4.94 -> 5.54
    // ms, until the rare branches were laid out cold: 4.84 ms, ZFP_RARE)
    if (a.idx_bad && used != len)
      atomicOr(a.idx_bad, 1u);
  };
  if (SHORT && __any(over)) {
    if (over) {
      if (gs) {
        WordReader r;
        r.w = gs;
        r.pos = 0;
        dec(r);
      }
      return;
    }
  }
  WordReader r;
  r.w = wslot + (size_t)lane * a.swp;
  r.pos = 0;
  dec(r);
}

}  // namespace zfp_amd
