// How far a speculative parse chain (scan.h) runs before it lands on a true
// block start, from random start bits, on an oracle stream of the smooth
// field used by tools/scan_bench.py (4D f32 reversible, or 3D f64 precision 32).
//   g++ -O2 -std=c++17 -I../../tests/emu/stub -I../../zfp-par_amd/csrc/hip resync.cpp ../../oracle/zfp_oracle.c -o resync
//   ./resync [dims] [n] [trials]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
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

template <typename S, int DIMS, bool REV>
static void run(uint64_t n, int trials, const oz_params& p)
{
  const uint64_t N = DIMS == 3 ? n * n * n : n * n * n * n;
  std::vector<S> f(N);
  for (uint64_t i = 0; i < N; i++) {
    const double x = i % n, y = (i / n) % n, z = (i / n / n) % n, w = DIMS == 4 ? (double)(i / n / n / n) : 0.0;
    // tools/scan_bench.py: axes reversed (x fastest = last numpy axis)
    double v = std::sin(0.05 * x) * std::cos(0.03 * y) + 0.5 * std::sin(0.02 * z + 0.01 * x * y / n);
    if (DIMS == 4) v += 0.25 * std::cos(0.04 * w);
    f[i] = (S)v;
  }
  oz_job j{};
  j.type = sizeof(S) == 4 ? 3 : 4;
  j.p = p;
  for (int a = 0; a < DIMS; a++) j.n[a] = n, j.f[a] = 0, j.e[a] = n;
  j.s[0] = 1, j.s[1] = n, j.s[2] = n * n, j.s[3] = DIMS == 4 ? n * n * n : 0;
  const uint64_t nbx = n / 4, nb = DIMS == 3 ? nbx * nbx * nbx : nbx * nbx * nbx * nbx;
  std::vector<uint32_t> lens(nb);
  std::vector<uint64_t> scratch(8192);
  oz_block_bits(&j, f.data(), scratch.data(), lens.data(), nb);
  std::vector<uint64_t> truth(nb + 1, 0);
  for (uint64_t b = 0; b < nb; b++) truth[b + 1] = truth[b] + lens[b];
  std::vector<uint64_t> words(truth[nb] / 64 + 64, 0);
  oz_compress(&j, f.data(), words.data(), 0);
  printf("%dD %s: %llu blocks, %.1f Mbit, %.0f bits/block\n", DIMS, REV ? "reversible" : "lossy",
         (unsigned long long)nb, truth[nb] / 1e6, (double)truth[nb] / nb);
  ScanParams sp{p.minbits, p.maxbits, p.maxprec, p.minexp};
  std::mt19937_64 rng(1);
  std::vector<double> d;
  uint64_t ring[kRing];
  for (int t = 0; t < trials; t++) {
    const uint64_t b0 = rng() % (truth[nb] / 2);
    RingReader rd;
    rd.in = words.data(), rd.in_words = words.size(), rd.g0 = 0, rd.ring = ring;
    rd.start(b0);
    uint64_t q = b0;
    while (q < truth[nb] && !std::binary_search(truth.begin(), truth.end(), q))
      q += scan_block<S, DIMS, REV>(rd, q, sp);
    d.push_back((double)(q - b0));
  }
  // K chains from consecutive-block-ish offsets after each random start: the
  // first of them to reach a true start
  std::vector<double> dk;
  const int K = getenv("K") ? atoi(getenv("K")) : 16;
  for (int t = 0; t < trials; t++) {
    const uint64_t b0 = rng() % (truth[nb] / 2);
    double best = 1e18;
    for (int k = 0; k < K; k++) {
      const uint64_t s0 = b0 + (uint64_t)k * 97;
      RingReader rd;
      rd.in = words.data(), rd.in_words = words.size(), rd.g0 = 0, rd.ring = ring;
      rd.start(s0);
      uint64_t q = s0;
      while (q < truth[nb] && !std::binary_search(truth.begin(), truth.end(), q))
        q += scan_block<S, DIMS, REV>(rd, q, sp);
      best = std::min(best, (double)(q - b0));
    }
    dk.push_back(best);
  }
  std::sort(dk.begin(), dk.end());
  printf("best of %d chains (starts 97 bits apart): median %.0f, p90 %.0f, max %.0f\n", K, dk[dk.size() / 2],
         dk[dk.size() * 9 / 10], dk.back());
  std::sort(d.begin(), d.end());
  double mean = 0;
  for (double x : d) mean += x;
  mean /= d.size();
  printf("resync bits over %d random starts: mean %.0f, median %.0f, p90 %.0f, p99 %.0f, max %.0f\n", trials, mean,
         d[d.size() / 2], d[d.size() * 9 / 10], d[d.size() * 99 / 100], d.back());
}

int main(int argc, char** argv)
{
  const int dims = argc > 1 ? atoi(argv[1]) : 4;
  const uint64_t n = argc > 2 ? strtoull(argv[2], nullptr, 10) : 48;
  const int trials = argc > 3 ? atoi(argv[3]) : 200;
  if (dims == 4)
    run<float, 4, true>(n, trials, oz_params{1, 16658 + 4096, 64, -1075});
  else
    run<double, 3, false>(n, trials, oz_params{1, 16658 + 4096, 32, -1074});
  return 0;
}
