// Experiment (not product, not test): cost of the index scan's serial parse
// (scan.h scan_block) on a 4D f32 reversible stream of the C5 field, counted
// on the CPU with a reader that records every window read: reads per block,
// reads per 1,000 stream bits, and how often a read jumps past the 16-word
// ring (a ring restart on the GPU), for the true chain and for chains started
// at random bits.
// build: g++ -O2 -std=c++17 -I../emu/stub -I../../zfp-par_amd/csrc/hip ... (see tools/exp/Makefile)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define EMU_KERNEL_BUILTINS
#include "scan.h"
using namespace zfp_amd;

extern "C" {
typedef struct { uint32_t minbits, maxbits, maxprec; int32_t minexp; } oz_params;
typedef struct { int32_t type, pad_; oz_params p; uint64_t n[4]; int64_t s[4]; uint64_t f[4]; uint64_t e[4]; } oz_job;
uint64_t oz_compress(const oz_job* j, const void* data, uint64_t* words, uint64_t bitpos);
}

struct CountReader {
  const uint64_t* w;
  uint64_t nw;
  uint64_t reads = 0, jumps = 0, last = 0;
  uint64_t peek(uint64_t r)
  {
    reads++;
    if (r > last + 1024 || r + 64 < last) jumps++;
    last = r;
    const uint64_t i = r >> 6, s = r & 63;
    const uint64_t lo = i < nw ? w[i] : 0, hi = i + 1 < nw ? w[i + 1] : 0;
    return s ? (lo >> s) | (hi << (64 - s)) : lo;
  }
};

int main(int argc, char** argv)
{
  const int n = argc > 1 ? atoi(argv[1]) : 32, n4 = n * n * n * n;
  const int x0 = argc > 2 ? atoi(argv[2]) : 0, y0 = argc > 3 ? atoi(argv[3]) : 0, z0 = argc > 4 ? atoi(argv[4]) : 0;
  std::vector<float> f(n4);
  const int N = 512;  // the C5 field's x, y, z, w coordinates as in a 512^4 chunk
  for (int w = 0; w < n; w++)
    for (int z = 0; z < n; z++)
      for (int y = 0; y < n; y++)
        for (int x = 0; x < n; x++)
          f[((size_t)(w * n + z) * n + y) * n + x] =
              (float)(sin(0.05 * (x + x0)) * cos(0.03 * (y + y0)) + 0.5 * sin(0.02 * (z + z0) + 0.01 * (x + x0) * (y + y0) / N) +
                      0.25 * cos(0.04 * w));
  oz_job j{};
  j.type = 3;
  j.p = {1, 16658, 64, -1075};
  for (int a = 0; a < 4; a++) j.n[a] = n, j.f[a] = 0, j.e[a] = n;
  j.s[0] = 1, j.s[1] = n, j.s[2] = (int64_t)n * n, j.s[3] = (int64_t)n * n * n;
  std::vector<uint64_t> words((size_t)n4 / 2 + 4096, 0);
  const uint64_t bits = oz_compress(&j, f.data(), words.data(), 0);
  const uint64_t nb = (uint64_t)n4 / 256;
  ScanParams sp{1, 16658, 64, -1075};
  CountReader rd{words.data(), words.size()};
  uint64_t p = 0, blocks = 0, big = 0, big_reads = 0, big_bits = 0;
  while (blocks < nb) {
    const uint64_t r0 = rd.reads;
    const uint32_t len = scan_block<float, 4, true>(rd, p, sp);
    if (len > 6000) { big++; big_reads += rd.reads - r0; big_bits += len; }
    p += len;
    blocks++;
  }
  printf("true blocks over 6000 bits: %llu, %.1f reads per block (%.1f bits per block)\n", (unsigned long long)big,
         big ? (double)big_reads / big : 0.0, big ? (double)big_bits / big : 0.0);
  printf("true chain: %llu blocks, %llu bits (stream %llu): %.1f reads per block, %.2f reads per 1000 bits, %.3f ring jumps per block\n",
         (unsigned long long)blocks, (unsigned long long)p, (unsigned long long)bits, (double)rd.reads / blocks,
         1000.0 * rd.reads / p, (double)rd.jumps / blocks);
  // true block starts (for merge distances)
  std::vector<uint64_t> starts;
  {
    CountReader r3{words.data(), words.size()};
    uint64_t q = 0;
    for (uint64_t b = 0; b < nb; b++) { starts.push_back(q); q += scan_block<float, 4, true>(r3, q, sp); }
  }
  // chains from random bits until they land on a true start: distance and parse cost
  {
    srand(7);
    double dsum = 0, rsum = 0; uint64_t dmax = 0, nfail = 0;
    for (int t = 0; t < 200; t++) {
      CountReader r4{words.data(), words.size()};
      uint64_t q = (uint64_t)rand() % (bits - 200000), q0 = q;
      while (q < bits) {
        if (std::binary_search(starts.begin(), starts.end(), q)) break;
        q += scan_block<float, 4, true>(r4, q, sp);
      }
      if (q >= bits) { nfail++; continue; }
      dsum += q - q0; rsum += r4.reads; if (q - q0 > dmax) dmax = q - q0;
    }
    printf("random chains to their merge with the true chain: mean %.0f bits (max %llu, %llu ran off the end), %.1f reads per 1000 bits\n",
           dsum / (200 - nfail), (unsigned long long)dmax, (unsigned long long)nfail, 1000.0 * rsum / dsum);
  }
  // candidate starts: the first bit from a random position whose next K blocks
  // are nonzero and (if they carry an exponent) within +-D of the first one's
  for (int K : {2, 3, 4}) {
    const int D = 3;
    srand(11);
    uint64_t hits = 0, tries = 300, dist = 0, reads = 0;
    for (uint64_t t = 0; t < tries; t++) {
      CountReader r5{words.data(), words.size()};
      uint64_t q = (uint64_t)rand() % (bits - 300000), q0 = q;
      for (;; q++) {
        uint64_t c = q;
        int e0 = -1, ok = 1;
        for (int k = 0; k < K && ok; k++) {
          const uint64_t h = r5.peek(c);
          if (!(h & 1)) { ok = 0; break; }
          if (!((h >> 1) & 1)) {  // an exponent
            const int e = (int)((h >> 2) & 0xff);
            if (e0 < 0) e0 = e;
            else if (abs(e - e0) > D) ok = 0;
          } else if ((((h >> 2) & 31) + 1) != 32) {
            ok = 0;  // reinterpreted bits: full precision
          }
          if (ok) c += scan_block<float, 4, true>(r5, c, sp);
        }
        if (ok) break;
      }
      dist += q - q0;
      reads += r5.reads;
      hits += std::binary_search(starts.begin(), starts.end(), q);
    }
    printf("K=%d: first plausible start %.0f bits on, true %.1f%%, %.2f reads per searched bit\n", K,
           (double)dist / tries, 100.0 * hits / tries, (double)reads / dist);
  }
  // the same with a one-peek header test first, against the exponent window of
  // the stream's first 64 blocks (+-16)
  int emin = 255, emax = 0;
  {
    CountReader r6{words.data(), words.size()};
    for (int b = 0; b < 64; b++) {
      const uint64_t h = r6.peek(starts[b]);
      if ((h & 1) && !((h >> 1) & 1)) { const int e = (int)((h >> 2) & 0xff); emin = std::min(emin, e); emax = std::max(emax, e); }
    }
  }
  auto head_ok = [&](uint64_t h) {
    if (!(h & 1)) return false;
    if (!((h >> 1) & 1)) { const int e = (int)((h >> 2) & 0xff); return e >= emin - 16 && e <= emax + 16; }
    return (((h >> 2) & 31) + 1) == 32;
  };
  for (int K : {3, 4}) {
    srand(11);
    uint64_t hits = 0, tries = 300, dist = 0, reads = 0, parses = 0;
    for (uint64_t t = 0; t < tries; t++) {
      CountReader r5{words.data(), words.size()};
      uint64_t q = (uint64_t)rand() % (bits - 300000), q0 = q;
      for (;; q++) {
        if (!head_ok(r5.peek(q))) continue;
        uint64_t c = q;
        int ok = 1;
        for (int k = 0; k < K && ok; k++) {
          if (k && !head_ok(r5.peek(c))) { ok = 0; break; }
          c += scan_block<float, 4, true>(r5, c, sp);
          parses++;
        }
        if (ok) break;
      }
      dist += q - q0;
      reads += r5.reads;
      hits += std::binary_search(starts.begin(), starts.end(), q);
    }
    printf("window [%d, %d] K=%d: first plausible start %.0f bits on, true %.1f%%, %.2f reads and %.3f block parses per searched bit\n",
           emin - 16, emax + 16, K, (double)dist / tries, 100.0 * hits / tries, (double)reads / dist, (double)parses / dist);
  }
  // with a precision window too (reversible: the first 32 blocks' precisions -2),
  // and the bits the deep checks parse
  int pmin = 99;
  {
    CountReader r7{words.data(), words.size()};
    for (int b = 0; b < 32; b++) {
      const uint64_t h = r7.peek(starts[b]);
      if (h & 1) { const int pr = (int)(((h >> 1) & 1) ? ((h >> 2) & 31) : ((h >> 10) & 31)) + 1; pmin = std::min(pmin, pr); }
    }
  }
  auto head_ok2 = [&](uint64_t h) {
    if (!(h & 1)) return false;
    if (!((h >> 1) & 1)) {
      const int e = (int)((h >> 2) & 0xff);
      const int pr = (int)((h >> 10) & 31) + 1;
      return e >= emin - 16 && e <= emax + 16 && pr >= pmin - 2;
    }
    return (((h >> 2) & 31) + 1) == 32;
  };
  std::vector<uint64_t> lane_bits;
  for (int K : {4}) {
    srand(11);
    uint64_t hits = 0, tries = 1000, dist = 0, pbits = 0, parses = 0;
    for (uint64_t t = 0; t < tries; t++) {
      CountReader r5{words.data(), words.size()};
      uint64_t q = (uint64_t)rand() % (bits - 300000), q0 = q;
      const uint64_t pb0 = pbits;
      for (;; q++) {
        if (!head_ok2(r5.peek(q))) continue;
        uint64_t c = q;
        int ok = 1;
        for (int k = 0; k < K && ok; k++) {
          if (k && !head_ok2(r5.peek(c))) { ok = 0; break; }
          const uint32_t l = scan_block<float, 4, true>(r5, c, sp);
          c += l; pbits += l; parses++;
        }
        if (ok) break;
      }
      dist += q - q0;
      lane_bits.push_back(pbits - pb0);
      hits += std::binary_search(starts.begin(), starts.end(), q);
    }
    printf("e and prec (>= %d) windows, K=%d: start %.0f bits on, true %.1f%%, deep checks parse %.1f bits per searched bit (%.3f blocks)\n",
           pmin - 2, K, (double)dist / tries, 100.0 * hits / tries, (double)pbits / dist, (double)parses / dist);
    std::sort(lane_bits.begin(), lane_bits.end());
    if (!lane_bits.empty())
      printf("   bits parsed per search: median %llu, p90 %llu, p99 %llu, max %llu\n",
             (unsigned long long)lane_bits[lane_bits.size() / 2], (unsigned long long)lane_bits[lane_bits.size() * 9 / 10],
             (unsigned long long)lane_bits[lane_bits.size() * 99 / 100], (unsigned long long)lane_bits.back());
    lane_bits.clear();
  }
  // false chains from random starts, each followed for 64 Kbit
  srand(5);
  uint64_t fr = 0, fb = 0, fbits = 0, fj = 0;
  for (int t = 0; t < 200; t++) {
    CountReader r2{words.data(), words.size()};
    uint64_t q = (uint64_t)rand() % (bits / 2), q0 = q;
    while (q < q0 + 65536 && q < bits) {
      q += scan_block<float, 4, true>(r2, q, sp);
      fb++;
    }
    fr += r2.reads;
    fj += r2.jumps;
    fbits += q - q0;
  }
  printf("chains from random bits: %.1f bits per block, %.1f reads per block, %.2f reads per 1000 bits, %.3f ring jumps per block\n",
         (double)fbits / fb, (double)fr / fb, 1000.0 * fr / fbits, (double)fj / fb);
  return 0;
}
