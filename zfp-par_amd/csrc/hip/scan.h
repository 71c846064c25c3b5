// Block index of a variable-rate stream that carries none (any zfp stream in
// precision, accuracy, reversible or expert mode -- the reference's serial
// decoder finds block i only by decoding blocks 0..i-1: decompress.c:66-140,
// decode.c:69-246, revdecode.c:34-52).
//
// Parallel resynchronising parse.  The stream is cut into segments of L bits,
// one lane per segment:
//
//   pass 1  lane s parses blocks from `lead` bits before the segment's first
//           bit as if a block started there (speculatively: only bit 0 starts
//           a real block), follows that chain into the segment and on until
//           it leaves it, marking every block start inside the segment in a
//           bitmap (1 bit per stream bit) and recording where it left, X[s].
//           The lead-in lets the chain resynchronise with the true one before
//           the segment starts, so that pass 2 usually confirms it at once.
//   pass k  lane s re-parses from X[s-1], the exit of the chain of segment
//           s-1.  Parsing is deterministic, so the moment this chain lands on
//           a start already marked in segment s it coincides with segment s's
//           chain from there on: the lane rewrites the bits before that point
//           and stops ("merged"; X[s] unchanged).  A chain that crosses the
//           whole segment without merging replaces it and moves X[s], so
//           segment s+1 is redone in the next pass.  Passes repeat until no
//           exit moves; then segment 0's true chain runs through every
//           segment, so the first nblocks+1 set bits are the block starts and
//           the end of the last block.
//
// Invariant after every pass: each segment's bitmap holds exactly one parse
// chain restricted to the segment, and X[s] is that chain's exit.
//
// The per-block parse is the decoder's bit consumption without the values:
// header (decodef.c:7-36, revdecodef.c:22-59), minbits/maxbits (decode.c:
// 271-287), and per plane the n verbatim bits plus the group-test section,
// in closed form when the section ends inside a 64-bit window (the decoder's
// carry trick, codec_dev.h) and by the reference loop otherwise.  A lane's
// stream bits come through a per-lane LDS ring refilled from prefetched
// registers, so global latency is paid once per 512 bits.
#pragma once

#include <type_traits>

#include "codec_dev.h"

namespace zfp_amd {

// ---------------------------------------------------------------------------
// per-lane stream reader: ring of kRing words in LDS + kHalf prefetched words
#ifndef ZFP_SCAN_RING_WORDS
#define ZFP_SCAN_RING_WORDS 16
#endif
constexpr uint32_t kRing = ZFP_SCAN_RING_WORDS;
constexpr uint32_t kHalf = kRing / 2;

struct RingReader {
  const uint64_t* in;   // stream words (word 0 holds relative bit -g0 .. )
  uint64_t in_words;
  uint32_t g0;          // relative position r is absolute bit g0 + r of in[]
  uint64_t* ring;       // kRing words (this lane's)
  uint64_t base;        // absolute word index held in ring slot base % kRing
  uint64_t nxt[kHalf];  // words [base + kRing, base + kRing + kHalf)

  __device__ __forceinline__ uint64_t word(uint64_t i) const { return i < in_words ? in[i] : 0ull; }

  __device__ __forceinline__ void fetch_next()
  {
#pragma unroll
    for (uint32_t j = 0; j < kHalf; j++)
      nxt[j] = word(base + kRing + j);
  }
  // fill the ring with the words from the one holding absolute word i
  __device__ __forceinline__ void start_word(uint64_t i)
  {
    base = i & ~(uint64_t)(kHalf - 1);
#pragma unroll
    for (uint32_t j = 0; j < kRing; j++)
      ring[(base + j) % kRing] = word(base + j);
    fetch_next();
  }
  __device__ __forceinline__ void start(uint64_t rel) { start_word((g0 + rel) >> 6); }
  // make words i and i+1 resident (i >= base: positions only move forward)
  __device__ __forceinline__ void ensure(uint64_t i)
  {
#ifdef EMU_KERNEL_BUILTINS
    if (i < base) {  // host emulation: a read behind the ring (positions must only move forward)
      fprintf(stderr, "RingReader: word %llu behind the ring base %llu\n", (unsigned long long)i,
              (unsigned long long)base);
      abort();
    }
#endif
    if (i + 1 < base + kRing)
      return;
    if (i + 1 >= base + kRing + kHalf) {  // jumped past the prefetched half
      start_word(i);
      return;
    }
#pragma unroll
    for (uint32_t j = 0; j < kHalf; j++)
      ring[(base + kRing + j) % kRing] = nxt[j];
    base += kHalf;
    fetch_next();
  }
  // 64 stream bits starting at relative bit r (LSB = bit r)
  __device__ __forceinline__ uint64_t peek(uint64_t r)
  {
    const uint64_t a = g0 + r;
    const uint64_t i = a >> 6;
    const uint32_t s = (uint32_t)(a & 63);
    ensure(i);
    const uint64_t lo = ring[i % kRing], hi = ring[(i + 1) % kRing];
    return s ? (lo >> s) | (hi << (64 - s)) : lo;
  }
};

// ---------------------------------------------------------------------------
// bit consumption of one block

struct ScanParams {
  uint32_t minbits, maxbits, maxprec;
  int32_t minexp;
};

// Group-test section of one plane (decode.c:69-246 group loop) at bit p with
// n < SIZE coefficients significant and bits > 0 budget.
template <int SIZE, typename R>
__device__ __forceinline__ void scan_section(R& rd, uint64_t& p, uint32_t& bits, uint32_t& n)
{
  const uint64_t w = rd.peek(p);
  if (!(w & 1)) {  // "0": no one left in this plane
    p++;
    bits--;
    return;
  }
  uint64_t q0 = p + 1;        // stream bit of the current window's token bit 0
  uint32_t used = 1, nn = n;  // bits (the "1" test) and coefficients before it
  {
    // closed form: after the "1" test the section is tokens "0", "11", "10"
    // and ends at the first run of ones of odd length (codec_dev.h), taken
    // one 64-bit window at a time: a window without an end holds only "0"
    // and "11" tokens (every run of ones even) except a last run of ones
    // reaching its top, whose odd "1" starts a token that the next window
    // continues.  4D sections are often longer than one window; one window
    // costs a peek, where the reference loop costs one per coefficient.
    uint64_t S = w >> 1;   // token bits from stream bit q0
    uint32_t avail = 63;   // of which the low `avail` are stream bits
    for (;;) {
      const uint64_t real = low_mask(avail);
      S &= real;
      const uint64_t starts = S & ~(S << 1);
      const uint64_t se = S + (starts & kEven), so = S + (starts & kOdd);
      const uint64_t ends = (((se & ~S) & kOdd) | ((so & ~S) & kEven)) & real;
      if (ends) {
        const uint32_t q = ctz64(ends);
        const uint64_t mq = (ends - 1) & ~ends;
        const uint32_t ones = (uint32_t)__popcll(S & mq);
        const uint32_t P = q - (ones - 1) / 2;
        if (nn + P <= (uint32_t)SIZE - 1 && used + q + 1 <= bits) {
          p = q0 + q + 1;
          bits -= used + q + 1;
          n = nn + P;
          return;
        }
        break;
      }
      // the run of ones at the window's top: an odd one leaves its last "1"
      const uint64_t top = S << (64 - avail);  // avail >= 63
      const uint32_t run = ~top ? (uint32_t)__builtin_clzll(~top) : 64u;
      const uint32_t c = avail - (run & 1u);
      const uint32_t ones = (uint32_t)__popcll(S & low_mask(c));  // even
      const uint32_t cnt = c - ones / 2;  // "0" tokens + "11" tokens
      if (nn + cnt > (uint32_t)SIZE - 1 || used + c > bits)
        break;
      nn += cnt;
      used += c;
      q0 += c;
      S = rd.peek(q0);
      avail = 64;
    }
  }
  // reference loop (the implicit last coefficient, budget cuts), entered where
  // the windows stopped -- at a token boundary, past a "1" test (the ring
  // reader only moves forward)
  p = q0;
  bits -= used;
  n = nn;
  for (bool inner = true;; inner = false) {
    if (!inner) {
      if (!(bits && n < (uint32_t)SIZE))
        break;
      bits--;
      const uint32_t t = (uint32_t)(rd.peek(p) & 1);
      p++;
      if (!t)
        break;
    }
    uint32_t rem = (uint32_t)SIZE - 1 - n;
    rem = rem < bits ? rem : bits;
    for (;;) {
      const uint32_t z = ctz64(rd.peek(p));
      if (z < 64 && z < rem) {  // a one: the coefficient at n + z
        p += z + 1;
        bits -= z + 1;
        n += z;
        break;
      }
      if (rem <= 64) {  // all zeros up to the implicit coefficient or the budget
        p += rem;
        bits -= rem;
        n += rem;
        break;
      }
      p += 64;
      bits -= 64;
      n += 64;
      rem -= 64;
    }
    n++;
  }
}

// planes intprec-1 .. intprec-maxprec with `budget` bits: decode_ints
template <int SIZE, int INTPREC, typename R>
__device__ __forceinline__ uint32_t scan_planes(R& rd, uint64_t p, uint32_t budget, uint32_t maxprec)
{
  const uint32_t np = maxprec < (uint32_t)INTPREC ? maxprec : (uint32_t)INTPREC;
  uint32_t bits = budget, n = 0;
  for (uint32_t k = 0; k < np && bits; k++) {
    const uint32_t m = n < bits ? n : bits;
    p += m;
    bits -= m;
    if (n < (uint32_t)SIZE && bits)
      scan_section<SIZE>(rd, p, bits, n);
  }
  return budget - bits;
}

// Length in bits of the block starting at p (decodef.c:7-36 / revdecodef.c:22-59)
template <typename S, int DIMS, bool REV, typename R>
__device__ __forceinline__ uint32_t scan_block(R& rd, uint64_t p, const ScanParams& sp)
{
  using T = Traits<S>;
  constexpr int SIZE = 1 << (2 * DIMS);
  constexpr uint32_t kE = T::kEbits, kP = T::kPbits;
  if constexpr (std::is_integral<S>::value) {
    // integer blocks: no header (encode.c:260-280), or the reversible
    // precision (revencode.c:54-76)
    uint32_t bits;
    if constexpr (REV) {
      const uint32_t prec = (uint32_t)(rd.peek(p) & ((1u << kP) - 1)) + 1;
      bits = kP + scan_planes<SIZE, T::kIntPrec>(rd, p + kP, sp.maxbits - kP, prec);
    } else {
      bits = scan_planes<SIZE, T::kIntPrec>(rd, p, sp.maxbits, sp.maxprec);
    }
    return bits < sp.minbits ? sp.minbits : bits;
  }
  const uint64_t h = rd.peek(p);
  const uint32_t zero_len = sp.minbits > 1 ? sp.minbits : 1u;
  if (!(h & 1))
    return zero_len;
  if constexpr (REV) {
    const bool reinterp = (h >> 1) & 1;
    const uint32_t bits = reinterp ? 2u : 2u + kE;
    const uint32_t minb = sp.minbits - (bits < sp.minbits ? bits : sp.minbits);
    const uint32_t maxb = sp.maxbits - bits;
    const uint32_t prec = (uint32_t)((h >> bits) & ((1u << kP) - 1)) + 1;
    uint32_t ib = kP + scan_planes<SIZE, T::kIntPrec>(rd, p + bits + kP, maxb - kP, prec);
    if (ib < minb)
      ib = minb;
    return bits + ib;
  } else {
    const int emax = (int)((h >> 1) & ((1u << kE) - 1)) - T::kEbias;
    int pr = emax - sp.minexp + 2 * DIMS + 2;
    if (pr < 0)
      pr = 0;
    const uint32_t mp = (uint32_t)pr < sp.maxprec ? (uint32_t)pr : sp.maxprec;
    const uint32_t bits = 1 + kE;
    const uint32_t minb = sp.minbits - (bits < sp.minbits ? bits : sp.minbits);
    uint32_t ib = scan_planes<SIZE, T::kIntPrec>(rd, p + bits, sp.maxbits - bits, mp);
    if (ib < minb)
      ib = minb;
    return bits + ib;
  }
}

// ---------------------------------------------------------------------------
// segment pass

struct ScanArgs {
  const uint64_t* in;
  uint64_t in_words;
  uint32_t g0;
  uint32_t first;        // 1: pass 1 (bitmap is all zero; speculative starts)
  uint64_t seg_bits;     // L, a multiple of 64
  uint64_t lead;         // pass 1: a segment's chain starts this many bits early
  uint64_t nseg;
  uint64_t limit;        // bits [0, limit) are scanned (limit = extent + 1)
  uint64_t* bm;          // boundary bitmap, ceil(limit / 64) words
  uint64_t* entry_used;  // per segment: the entry the current chain started at
  const uint64_t* xsnap; // per segment: exits before this pass
  uint64_t* x;           // per segment: exits after this pass
  uint32_t* moved;       // count of exits that moved in this pass
  ScanParams sp;
  const int32_t* win;    // pass 1, float blocks: plausible block starts' exponent window, min precision (null: off)
  uint64_t* plaus;       // per segment: its pass-1 plausible start (~0: none); null: off
  uint32_t refuse;       // phase A: refuse implausible chains at segments that keep their plausible chain
  uint32_t* refused;     // count of refusals in this pass
};

// ---------------------------------------------------------------------------
// Plausible chain starts (pass 1).  A chain started at an arbitrary bit parses
// garbage -- mostly one-bit "zero blocks" and long blocks of random planes --
// and on a 4D reversible stream runs for about 0.5 Mbit on average before it
// lands on a true block start, at about ten times the window reads per bit of
// the true chain (tools/exp/scanstats.cpp).  So pass 1 starts each segment's
// chain at the first bit whose next kPlausibleBlocks blocks look like real
// ones instead: a nonzero flag, and an exponent inside the window of the
// stream's first blocks (+-16) or, for reinterpreted reversible blocks, full
// precision.  On the C5 field that start is a true block start 97-99.7 % of
// the time, found within about 1-2 Kbit.  It only decides where the
// speculative chain begins: the passes and their merge rule are unchanged, so
// a wrong guess costs time, never correctness.
constexpr int kPlausibleBlocks = 4;

template <typename S, bool REV>
__device__ __forceinline__ bool head_plausible(uint64_t h, int32_t elo, int32_t ehi, int32_t pmin)
{
  using T = Traits<S>;
  if (!(h & 1))
    return false;
  if constexpr (REV) {
    if ((h >> 1) & 1)  // reinterpreted bits: precision in the next kPbits
      return (uint32_t)((h >> 2) & ((1u << T::kPbits) - 1)) + 1 == (uint32_t)T::kIntPrec;
    const int32_t e = (int32_t)((h >> 2) & ((1u << T::kEbits) - 1));
    const int32_t pr = (int32_t)((h >> (2 + T::kEbits)) & ((1u << T::kPbits) - 1)) + 1;
    return e >= elo && e <= ehi && pr >= pmin;
  } else {
    const int32_t e = (int32_t)((h >> 1) & ((1u << T::kEbits) - 1));
    return e >= elo && e <= ehi;
  }
}

// header bits a plausibility test reads (a 64-bit window tests 64 - this many starts)
template <typename S, bool REV>
constexpr uint32_t kHeadBits = 2 + Traits<S>::kEbits + (REV ? Traits<S>::kPbits : 0);

// first plausible chain start in [lo, hi) (found = true), else lo; leaves the ring at it
template <typename S, int DIMS, bool REV>
__device__ __forceinline__ uint64_t plausible_start(RingReader& rd, uint64_t lo, uint64_t hi, const ScanParams& sp,
                                                    int32_t elo, int32_t ehi, int32_t pmin, bool& found)
{
  found = true;
  constexpr uint32_t kStep = 64 - kHeadBits<S, REV>;
  for (uint64_t q = lo; q < hi; q += kStep) {
    const uint64_t W = rd.peek(q);
    uint64_t ones = W & ((1ull << kStep) - 1);
    if (q + kStep > hi)
      ones &= (1ull << (hi - q)) - 1;
    while (ones) {
      const uint32_t i = ctz64(ones);
      ones &= ones - 1;
      if (!head_plausible<S, REV>(W >> i, elo, ehi, pmin))
        continue;
      uint64_t c = q + i;
      bool ok = true;
      for (int k = 0; k < kPlausibleBlocks && ok; k++) {
        if (k && !head_plausible<S, REV>(rd.peek(c), elo, ehi, pmin))
          ok = false;
        else
          c += scan_block<S, DIMS, REV>(rd, c, sp);
      }
      rd.start(ok ? q + i : q);  // the check read ahead of the window: back to it
      if (ok)
        return q + i;
    }
  }
  rd.start(lo);
  found = false;
  return lo;
}

// the window of plausible starts from the stream's first 32 blocks: their
// exponents' range widened by 16 (empty when none carries one) and, for
// reversible blocks with an exponent, their lowest precision less 2
template <typename S, int DIMS, bool REV>
__device__ __forceinline__ void exp_window(const ScanArgs& a, uint64_t* ring, int32_t* win)
{
  using T = Traits<S>;
  RingReader rd;
  rd.in = a.in;
  rd.in_words = a.in_words;
  rd.g0 = a.g0;
  rd.ring = ring;
  rd.start(0);
  int32_t lo = 1 << 30, hi = -(1 << 30), pm = 1 << 30;
  uint64_t p = 0;
  for (int b = 0; b < 32 && p < a.limit; b++) {
    const uint64_t h = rd.peek(p);
    if ((h & 1) && !(REV && ((h >> 1) & 1))) {
      const int32_t e = (int32_t)((h >> (REV ? 2 : 1)) & ((1u << T::kEbits) - 1));
      lo = e < lo ? e : lo;
      hi = e > hi ? e : hi;
      if (REV) {
        const int32_t pr = (int32_t)((h >> (2 + T::kEbits)) & ((1u << T::kPbits) - 1)) + 1;
        pm = pr < pm ? pr : pm;
      }
    }
    p += scan_block<S, DIMS, REV>(rd, p, a.sp);
  }
  win[0] = lo <= hi ? lo - 16 : 1;
  win[1] = lo <= hi ? hi + 16 : 0;
  win[2] = REV && lo <= hi ? pm - 2 : 0;
}

// One segment of a pass (one lane).
template <typename S, int DIMS, bool REV>
__device__ __forceinline__ void scan_segment(const ScanArgs& a, uint64_t s, uint64_t* ring)
{
  const uint64_t lo = s * a.seg_bits;
  if (lo >= a.limit)
    return;
  const uint64_t hi = lo + a.seg_bits < a.limit ? lo + a.seg_bits : a.limit;
  uint64_t e;
  if (s == 0)
    e = 0;
  else if (a.first && !std::is_integral<S>::value && a.win)
    e = ~0ull;  // a plausible start in the segment, found below
  else if (a.first)
    e = lo > a.lead ? lo - a.lead : 0;  // lead-in start (0: the true chain)
  else
    e = a.xsnap[s - 1];
  uint64_t es = ~0ull;  // phase A: the plausible start this segment's chain still begins at
  if (!a.first) {
    const uint64_t cur = a.entry_used[s];
    if (e == cur)
      return;  // this segment's chain already starts where the previous one exits
    if (a.refuse && a.plaus && a.plaus[s] == cur && e < cur)
      es = cur;
  }
  RingReader rd;
  rd.in = a.in;
  rd.in_words = a.in_words;
  rd.g0 = a.g0;
  rd.ring = ring;
  if (e == ~0ull) {
    rd.start(lo);
    bool found;
    e = plausible_start<S, DIMS, REV>(rd, lo, hi, a.sp, a.win[0], a.win[1], a.win[2], found);
    if (a.plaus)
      a.plaus[s] = found ? e : ~0ull;
  } else {
    rd.start(e);
  }
  const bool check = !a.first;
  // a zero float block is the single bit "0" (integer blocks have no flag)
  const bool runs = !std::is_integral<S>::value && a.sp.minbits <= 1;
  uint64_t p = e;
  // pass 1: the speculative chain starts `lead` bits before the segment and
  // is only followed (nothing marked) until it enters it, so that it has
  // usually met the true chain by then
  while (p < lo) {
    const uint64_t h = rd.peek(p);
    if (runs && !(h & 1)) {
      const uint64_t c = ctz64(h);
      p += c < lo - p ? c : lo - p;
      continue;
    }
    p += scan_block<S, DIMS, REV>(rd, p, a.sp);
  }
  a.entry_used[s] = p;
  uint64_t wi = lo >> 6;     // bitmap word being assembled
  uint64_t acc = 0;          // this chain's starts in word wi
  bool merged = false;
  uint32_t odd = 0;          // blocks of this chain that do not look real (phase A)
  while (p < hi) {
    if (es != ~0ull && p > es) {
      // Phase A: the incoming chain passed this segment's plausible start
      // without landing on it, so one of the two is false.  A chain that has
      // already produced blocks that do not look real is taken to be the false
      // one: the segment keeps its chain (the words this parse flushed lie
      // below the plausible start, where that chain has no starts) and its
      // exit.  Phase B (normal passes) settles any refusal that was wrong.
      if (odd) {
        for (uint64_t j = lo >> 6; j < wi; j++)
          a.bm[j] = 0;
        a.entry_used[s] = es;
        atomicAdd(a.refused, 1u);
        return;
      }
      es = ~0ull;
    }
    const uint64_t pw = p >> 6;
    while (wi < pw) {
      a.bm[wi] = acc;
      acc = 0;
      wi++;
    }
    const uint32_t sh = (uint32_t)(p & 63);
    const uint64_t old = check ? a.bm[wi] : 0ull;  // consumed after the parse below
    const uint64_t h = rd.peek(p);
    if constexpr (!std::is_integral<S>::value) {
      if (es != ~0ull && !head_plausible<S, REV>(h, a.win[0], a.win[1], a.win[2]))
        odd++;
    }
    if (runs && !(h & 1)) {
      // a run of zero blocks, one bit each, within this bitmap word
      uint32_t c = ctz64(h);
      const uint32_t room = 64 - sh;
      c = c < room ? c : room;
      if ((uint64_t)c > hi - p)
        c = (uint32_t)(hi - p);
      const uint64_t m = (c >= 64 ? ~0ull : ((1ull << c) - 1)) << sh;
      const uint64_t hit = old & m;
      if (hit) {
        const uint64_t below = (1ull << ctz64(hit)) - 1;  // this chain's starts before the merge
        a.bm[wi] = acc | (m & below) | (old & ~below);
        merged = true;
        break;
      }
      acc |= m;
      p += c;
      continue;
    }
    const uint32_t len = scan_block<S, DIMS, REV>(rd, p, a.sp);
    if ((old >> sh) & 1) {
      // the chain of this segment already has a block at p: from here on the
      // two chains are the same
      a.bm[wi] = acc | (old & ~((1ull << sh) - 1));
      merged = true;
      break;
    }
    acc |= 1ull << sh;
    p += len;
  }
  if (merged)
    return;
  a.bm[wi] = acc;
  const uint64_t wend = (hi + 63) >> 6;
  for (uint64_t j = wi + 1; j < wend; j++)
    a.bm[j] = 0;
  if (!a.first && a.x[s] != p)
    atomicAdd(a.moved, 1u);
  a.x[s] = p;
}

template <typename S, int DIMS, bool REV>
__global__ __launch_bounds__(64) void scan_window(ScanArgs a, int32_t* win)
{
  __shared__ uint64_t ring[kRing];
  if (threadIdx.x == 0)
    exp_window<S, DIMS, REV>(a, ring, win);
}

template <typename S, int DIMS, bool REV>
__global__ __launch_bounds__(256) void scan_pass(ScanArgs a)
{
  __shared__ uint64_t rings[256 * (kRing + 1)];  // odd stride: fewer bank collisions
  const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (s >= a.nseg)
    return;
  scan_segment<S, DIMS, REV>(a, s, rings + threadIdx.x * (kRing + 1));
}

// ---------------------------------------------------------------------------
// bitmap -> block index.  Tiles of kTileWords bitmap words per 256-thread group.
constexpr uint32_t kTileWords = 2048;

static __global__ __launch_bounds__(256) void bm_tile_count(const uint64_t* __restrict__ bm, uint64_t nwords,
                                                     uint64_t* __restrict__ tile_cnt)
{
  __shared__ uint32_t red[256];
  const uint64_t t0 = (uint64_t)blockIdx.x * kTileWords;
  uint32_t c = 0;
  for (uint32_t j = threadIdx.x; j < kTileWords; j += 256) {
    const uint64_t i = t0 + j;
    if (i < nwords)
      c += (uint32_t)__popcll(bm[i]);
  }
  red[threadIdx.x] = c;
  __syncthreads();
  for (uint32_t d = 128; d > 0; d >>= 1) {
    if (threadIdx.x < d)
      red[threadIdx.x] += red[threadIdx.x + d];
    __syncthreads();
  }
  if (threadIdx.x == 0)
    tile_cnt[blockIdx.x] = red[0];
}

// exclusive scan of n tile counts in place (one 1024-thread group); total -> *sum
static __global__ __launch_bounds__(1024) void tile_scan(uint64_t* __restrict__ v, uint64_t n, uint64_t* __restrict__ sum)
{
  __shared__ uint64_t part[1024];
  const uint64_t per = (n + 1023) / 1024;
  const uint64_t b = threadIdx.x * per;
  uint64_t s = 0;
  for (uint64_t i = b; i < b + per && i < n; i++)
    s += v[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    uint64_t y = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += y;
    __syncthreads();
  }
  uint64_t run = part[threadIdx.x] - s;
  for (uint64_t i = b; i < b + per && i < n; i++) {
    const uint64_t c = v[i];
    v[i] = run;
    run += c;
  }
  if (threadIdx.x == 1023)
    *sum = part[1023];
}

// Set bit r of the bitmap with rank k (0-based) gives pos[k] = r, for k <= nb.
static __global__ __launch_bounds__(256) void bm_tile_emit(const uint64_t* __restrict__ bm, uint64_t nwords,
                                                    const uint64_t* __restrict__ tile_off, uint64_t nb,
                                                    uint64_t* __restrict__ pos)
{
  __shared__ uint32_t part[256];
  constexpr uint32_t kPer = kTileWords / 256;  // consecutive words per thread
  const uint64_t t0 = (uint64_t)blockIdx.x * kTileWords + (uint64_t)threadIdx.x * kPer;
  uint64_t w[kPer];
  uint32_t c = 0;
#pragma unroll
  for (uint32_t j = 0; j < kPer; j++) {
    w[j] = t0 + j < nwords ? bm[t0 + j] : 0ull;
    c += (uint32_t)__popcll(w[j]);
  }
  part[threadIdx.x] = c;
  __syncthreads();
  for (uint32_t d = 1; d < 256; d <<= 1) {
    uint32_t y = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += y;
    __syncthreads();
  }
  uint64_t k = tile_off[blockIdx.x] + part[threadIdx.x] - c;
  if (k > nb)
    return;
#pragma unroll
  for (uint32_t j = 0; j < kPer; j++) {
    uint64_t x = w[j];
    while (x) {
      if (k > nb)
        return;
      const uint32_t b = (uint32_t)__builtin_ctzll(x);
      pos[k++] = (t0 + j) * 64 + b;
      x &= x - 1;
    }
  }
}

// decoder index: per-block lengths and per-wave (nbw blocks) start offsets
static __global__ __launch_bounds__(256) void index_from_pos(const uint64_t* __restrict__ pos, uint64_t nb, uint32_t nbw,
                                                      uint16_t* __restrict__ len, uint64_t* __restrict__ base)
{
  const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= nb)
    return;
  len[b] = (uint16_t)(pos[b + 1] - pos[b]);
  if (b % nbw == 0)
    base[b / nbw] = pos[b];
}

}  // namespace zfp_amd
