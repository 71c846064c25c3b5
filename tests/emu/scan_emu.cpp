// Host run of the index scan (scan.h) against the C oracle: per-block lengths
// from scan_block, and the whole resynchronising segment algorithm (passes run
// lane after lane with the GPU's snapshot semantics), for every variable-rate
// mode, 3D and 4D, float and double, at several segment sizes and stream bit
// offsets.  Prints "<case> ok" or the first mismatch.
//
// Reversible mode with minbits > 1 is not exercised on zero blocks: the
// reference encoder writes an all-zero block as the single bit "0"
// (revencodef.c:62-66) while its decoder skips to minbits (revdecodef.c:
// 55-61), so such streams do not decode in the reference either; the scan
// follows the decoder.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
#define EMU_KERNEL_BUILTINS
#include "scan.h"
using namespace zfp_amd;

extern "C" {
typedef struct { uint32_t minbits, maxbits, maxprec; int32_t minexp; } oz_params;
typedef struct { int32_t type, pad_; oz_params p; uint64_t n[4]; int64_t s[4]; uint64_t f[4]; uint64_t e[4]; } oz_job;
uint64_t oz_compress(const oz_job* j, const void* data, uint64_t* words, uint64_t bitpos);
uint64_t oz_block_bits(const oz_job* j, const void* data, uint64_t* scratch, uint32_t* lens, uint64_t maxblocks);
}

static uint64_t g_refusals = 0;  // phase-A refusals over the run (printed at the end)

struct Case {
  const char* name;
  int type, dims;
  oz_params p;
  int field;  // 0 smooth, 1 rough, 2 sparse (many zero blocks), 3 specials
};

template <typename S, int DIMS, bool REV>
static bool run_scan(const Case& c, const std::vector<uint64_t>& words, uint64_t g0, uint64_t nb,
                     const std::vector<uint64_t>& truth, uint64_t seg_bits, uint64_t lead, uint32_t max_len,
                     int* passes, bool plausible = false)
{
  ScanArgs a{};
  a.in = words.data();
  a.in_words = words.size();
  a.g0 = (uint32_t)g0;
  a.seg_bits = seg_bits;
  a.lead = lead;
  const uint64_t avail = words.size() * 64 - g0;
  uint64_t extent = nb * (uint64_t)max_len;
  extent = extent < avail ? extent : avail;
  a.limit = extent + 1;
  a.nseg = (a.limit + seg_bits - 1) / seg_bits;
  std::vector<uint64_t> bm((a.limit + 63) / 64, 0), used(a.nseg, ~0ull), x(a.nseg, 0), xs(a.nseg, 0);
  uint32_t moved = 0;
  a.bm = bm.data();
  a.entry_used = used.data();
  a.x = x.data();
  a.xsnap = xs.data();
  a.moved = &moved;
  a.sp = ScanParams{c.p.minbits, c.p.maxbits, c.p.maxprec, c.p.minexp};
  uint64_t ring[kRing];
  int32_t win[3];
  std::vector<uint64_t> plaus(a.nseg, ~0ull);
  uint32_t refused = 0;
  if (plausible) {  // pass 1 starts its chains at plausible block starts (float blocks)
    exp_window<S, DIMS, REV>(a, ring, win);
    a.win = win;
    a.plaus = plaus.data();
    a.refused = &refused;
  }
  a.first = 1;
  for (uint64_t s = 0; s < a.nseg; s++)
    scan_segment<S, DIMS, REV>(a, s, ring);
  a.first = 0;
  a.refuse = a.plaus ? 1u : 0u;  // phase A, then ordinary passes (zfp_hip.hip scan_index)
  *passes = 1;
  for (;;) {
    xs = x;
    a.xsnap = xs.data();
    moved = 0;
    refused = 0;
    for (uint64_t s = 0; s < a.nseg; s++)
      scan_segment<S, DIMS, REV>(a, s, ring);
    ++*passes;
    g_refusals += refused;
    if (!moved) {
      if (!a.refuse || !refused)
        break;
      a.refuse = 0;
      continue;
    }
    if (*passes > 2 * (int)a.nseg + 5) {
      printf("%s: no convergence\n", c.name);
      return false;
    }
  }
  // first nb+1 set bits
  uint64_t k = 0;
  for (uint64_t i = 0; i < bm.size() && k <= nb; i++) {
    uint64_t w = bm[i];
    while (w && k <= nb) {
      uint64_t r = i * 64 + __builtin_ctzll(w);
      if (r != truth[k]) {
        printf("%s: seg %llu g0 %llu: start %llu is %llu, want %llu\n", c.name, (unsigned long long)seg_bits,
               (unsigned long long)g0, (unsigned long long)k, (unsigned long long)r, (unsigned long long)truth[k]);
        return false;
      }
      k++;
      w &= w - 1;
    }
  }
  if (k != nb + 1) {
    printf("%s: only %llu starts found\n", c.name, (unsigned long long)k);
    return false;
  }
  return true;
}

template <typename S, int DIMS, bool REV>
static int run_case(const Case& c, std::mt19937_64& rng)
{
  const uint64_t n = DIMS == 3 ? 23 : 10;  // partial blocks on every axis
  const uint64_t N = DIMS == 3 ? n * n * n : n * n * n * n;
  std::vector<S> f(N);
  std::normal_distribution<double> nd(0, 1);
  for (uint64_t i = 0; i < N; i++) {
    uint64_t x = i % n, y = (i / n) % n, z = (i / n / n) % n;
    double v;
    switch (c.field) {
      case 0: v = std::sin(0.3 * x) * std::cos(0.2 * y) + 0.5 * std::sin(0.1 * z + 0.01 * x * y); break;
      case 1: v = nd(rng); break;
      case 2: v = (z % 8 < 5) ? 0.0 : nd(rng); break;
      default: {
        const double sp[] = {0.0, -0.0, 1e-40, INFINITY, -INFINITY, NAN, 1e30, 1.0};
        v = (rng() % 3 == 0) ? sp[rng() % 8] : nd(rng);
      }
    }
    f[i] = (S)v;
  }
  oz_job j{};
  j.type = sizeof(S) == 4 ? 3 : 4;
  j.p = c.p;
  for (int a = 0; a < DIMS; a++) j.n[a] = n, j.f[a] = 0, j.e[a] = n;
  j.s[0] = 1, j.s[1] = n, j.s[2] = n * n, j.s[3] = DIMS == 4 ? n * n * n : 0;
  const uint64_t nbx = (n + 3) / 4;
  const uint64_t nb = DIMS == 3 ? nbx * nbx * nbx : nbx * nbx * nbx * nbx;
  std::vector<uint32_t> lens(nb);
  std::vector<uint64_t> scratch(4096);
  oz_block_bits(&j, f.data(), scratch.data(), lens.data(), nb);
  uint32_t max_len = 0;
  {
    const uint32_t ebits = sizeof(S) == 4 ? 8 : 11, pbits = sizeof(S) == 4 ? 5 : 6, ip = sizeof(S) * 8;
    const uint32_t hdr = REV ? 2 + ebits + pbits : 1 + ebits;
    const uint32_t size = DIMS == 3 ? 64 : 256;
    uint64_t body = hdr + (size - 1) + (uint64_t)size * (c.p.maxprec < ip ? c.p.maxprec : ip);
    if (c.p.maxbits >= hdr && c.p.maxbits < body) body = c.p.maxbits;
    max_len = (uint32_t)(body > c.p.minbits ? body : c.p.minbits);
  }
  int fails = 0;
  for (uint64_t g0 : {96ull, 37ull}) {
    std::vector<uint64_t> words((g0 + (uint64_t)nb * max_len) / 64 + 8, 0);
    // garbage below g0 and past the end, as a real buffer might hold
    for (uint64_t i = 0; i < words.size(); i++) words[i] = rng();
    const uint64_t end = 0;
    (void)end;
    // clear the stream range and encode
    for (uint64_t b = g0; b < g0 + (uint64_t)nb * max_len + 64 && b / 64 < words.size(); b++)
      words[b / 64] &= ~(1ull << (b % 64));
    uint64_t e = oz_compress(&j, f.data(), words.data(), g0);
    std::vector<uint64_t> truth(nb + 1);
    truth[0] = 0;
    for (uint64_t b = 0; b < nb; b++) truth[b + 1] = truth[b] + lens[b];
    if (truth[nb] != e - g0) {
      printf("%s: oracle lengths disagree with its stream\n", c.name);
      return 1;
    }
    // per-block lengths
    {
      RingReader rd;
      uint64_t ring[kRing];
      rd.in = words.data(), rd.in_words = words.size(), rd.g0 = (uint32_t)g0, rd.ring = ring;
      rd.start(0);
      ScanParams sp{c.p.minbits, c.p.maxbits, c.p.maxprec, c.p.minexp};
      for (uint64_t b = 0; b < nb; b++) {
        uint32_t l = scan_block<S, DIMS, REV>(rd, truth[b], sp);
        if (l != lens[b]) {
          printf("%s: block %llu length %u, want %u\n", c.name, (unsigned long long)b, l, lens[b]);
          return 1;
        }
      }
    }
    // lead-ins: none, shorter than a block, several segments
    for (uint64_t seg : {128ull, 2048ull, 1ull << 20})
      for (uint64_t lead : {(uint64_t)0, (uint64_t)300, 4 * seg + 77}) {
        int passes = 0;
        if (!run_scan<S, DIMS, REV>(c, words, g0, nb, truth, seg, lead, max_len, &passes))
          fails++;
      }
    // plausible chain starts in pass 1
    for (uint64_t seg : {128ull, 2048ull, 1ull << 20}) {
      int passes = 0;
      if (!run_scan<S, DIMS, REV>(c, words, g0, nb, truth, seg, 0, max_len, &passes, true))
        fails++;
    }
  }
  printf("%s %s\n", c.name, fails ? "FAIL" : "ok");
  return fails;
}

int main()
{
  std::mt19937_64 rng(7);
  const oz_params prec32d{1, 16658 + 4096, 32, -1074}, prec16{1, 16658 + 4096, 16, -1074},
      acc{1, 16658 + 4096, 64, -6}, rev{1, 16658 + 4096, 64, -1075}, expert{300, 900, 20, -1074},
      exprev{1, 1500, 64, -1075}, tight{1, 200, 64, -1074};
  int bad = 0;
  for (int fld = 0; fld < 4; fld++) {
    char nm[64];
#define RUN(S, D, R, P, label)                                                   \
    snprintf(nm, sizeof nm, "%s field%d", label, fld);                           \
    bad += run_case<S, D, R>(Case{nm, sizeof(S) == 4 ? 3 : 4, D, P, fld}, rng);
    RUN(double, 3, false, prec32d, "3d f64 precision32");
    RUN(float, 3, false, prec16, "3d f32 precision16");
    RUN(float, 3, false, acc, "3d f32 accuracy");
    RUN(double, 3, false, acc, "3d f64 accuracy");
    RUN(float, 3, true, rev, "3d f32 reversible");
    RUN(double, 3, true, rev, "3d f64 reversible");
    RUN(float, 3, false, expert, "3d f32 expert");
    RUN(float, 3, false, tight, "3d f32 maxbits200");
    RUN(float, 3, true, exprev, "3d f32 reversible expert");
    RUN(float, 4, true, rev, "4d f32 reversible");
    RUN(double, 4, true, rev, "4d f64 reversible");
    RUN(float, 4, false, prec16, "4d f32 precision16");
    RUN(double, 4, false, acc, "4d f64 accuracy");
    RUN(float, 4, false, expert, "4d f32 expert");
  }
  printf("scan mismatches %d (phase-A refusals %llu)\n", bad, (unsigned long long)g_refusals);
  return bad != 0;
}
