// Four-lane host run of the 4D device block codec (block4.h) against the C
// oracle.  The lanes of one quad are four threads; DPP quad permutes and
// workgroup barriers are a four-thread rendezvous and the LDS is a shared
// array (slot ORs atomic), so the quad reductions, the LDS exchange of the
// w-lift and the segment-parallel plane coder run as they do on the GPU.
// Every mode, float and double, random and special blocks.
#include <hip/hip_runtime.h>

#include <atomic>
#include <thread>

struct EmuTid {
  uint32_t x;
};
inline thread_local EmuTid threadIdx{0};

// generation barrier for the four lane threads
struct QuadBarrier {
  std::atomic<int> n{0};
  std::atomic<unsigned> gen{0};
  void wait()
  {
    const unsigned g = gen.load(std::memory_order_acquire);
    if (n.fetch_add(1, std::memory_order_acq_rel) == 3) {
      n.store(0, std::memory_order_relaxed);
      gen.fetch_add(1, std::memory_order_release);
    } else {
      while (gen.load(std::memory_order_acquire) == g)
        std::this_thread::yield();
    }
  }
};
inline QuadBarrier g_bar;
inline uint32_t g_xchg[4];

inline int __builtin_amdgcn_mov_dpp(int x, int ctrl, int, int, bool)
{
  const uint32_t r = threadIdx.x & 3u;
  g_xchg[r] = (uint32_t)x;
  g_bar.wait();
  const int v = (int)g_xchg[(ctrl >> (2 * r)) & 3];
  g_bar.wait();
  return v;
}
inline int __builtin_amdgcn_update_dpp(int, int x, int ctrl, int, int, bool)
{
  return __builtin_amdgcn_mov_dpp(x, ctrl, 0, 0, false);
}
inline void __syncthreads() { g_bar.wait(); }

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <random>
#include <vector>

#include "block4.h"
using namespace zfp_amd;

extern "C" {
typedef struct { uint32_t minbits, maxbits, maxprec; int32_t minexp; } oz_params;
typedef struct { int32_t type, pad_; oz_params p; uint64_t n[4]; int64_t s[4]; uint64_t f[4]; uint64_t e[4]; } oz_job;
uint64_t oz_compress(const oz_job* j, const void* data, uint64_t* words, uint64_t bitpos);
uint64_t oz_decompress(const oz_job* j, void* data, const uint64_t* words, uint64_t bitpos);
}

template <typename F>
static void quad(F&& f)
{
  std::thread th[4];
  for (uint32_t r = 0; r < 4; r++)
    th[r] = std::thread([&f, r] { f(r); });
  for (auto& t : th)
    t.join();
}

template <typename S>
static int run(const CodecParams& cp, int type, std::mt19937_64& rng, int trials, const char* name)
{
  using Int = typename Traits<S>::Int;
  const bool rev = cp.minexp < kMinExp;
  uint32_t lut[256];
  for (int b = 0; b < 256; b++)
    lut[b] = dbl_entry(b);
  const uint32_t* tab = kOrderTab4.t;
  const uint32_t words = 1200;  // slot / exchange region: > 16658 bits and > 260 Ints
  int bad = 0;
  for (int t = 0; t < trials; t++) {
    std::vector<S> orig(256);
    const int kind = t % 8;
    std::normal_distribution<double> nd(0, 1);
    for (int i = 0; i < 256; i++) {
      double x = kind == 0 ? nd(rng) : kind == 1 ? std::sin(0.05 * i + t) : kind == 2 ? nd(rng) * 1e-30
               : kind == 3 ? (double)(rng() % 7) - 3 : kind == 4 ? nd(rng) * 1e20 : kind == 5 ? 0.0
               : kind == 6 ? (i % 37 == 3 ? INFINITY : i % 41 == 5 ? NAN : nd(rng))
               : nd(rng) * (double)std::numeric_limits<S>::denorm_min() * 64;
      orig[i] = (S)x;
    }
    oz_job j{};
    j.type = type;
    j.p = {cp.minbits, cp.maxbits, cp.maxprec, cp.minexp};
    for (int a = 0; a < 4; a++)
      j.n[a] = 4, j.f[a] = 0, j.e[a] = 4;
    j.s[0] = 1, j.s[1] = 4, j.s[2] = 16, j.s[3] = 64;
    std::vector<uint64_t> ow(words, 0);
    const uint64_t oend = oz_compress(&j, orig.data(), ow.data(), 0);

    // four lanes cannot zero a 64-lane region (zero_region): the exchange area
    // gets its own buffer and the slot starts out zeroed
    std::vector<uint64_t> region(words + 1, 0), xarea(words + 1, 0);
    uint32_t len[4];
    quad([&](uint32_t r) {
      threadIdx.x = r;
      S v[64];
      for (int i = 0; i < 64; i++)
        v[i] = orig[64 * r + i];
      auto reload = [&](S (&rr)[64]) {
        for (int i = 0; i < 64; i++)
          rr[i] = orig[64 * r + i];
      };
      uint32_t* d = reinterpret_cast<uint32_t*>(region.data());
      Int* X = reinterpret_cast<Int*>(xarea.data());
      auto place = [&](bool, uint32_t*& dd, uint32_t& jm) {
        dd = d;
        jm = 2 * words - 1;
      };
      len[r] = rev ? encode_block4<S, true>(place, lut, tab, X, region.data(), words, v, cp, reload)
                   : encode_block4<S, false>(place, lut, tab, X, region.data(), words, v, cp, reload);
    });
    bool ok = len[0] == oend && len[1] == len[0] && len[2] == len[0] && len[3] == len[0];
    for (uint32_t i = 0; ok && i < (len[0] + 63) / 64; i++) {
      const uint64_t m = (i == len[0] / 64 && (len[0] & 63)) ? ((1ull << (len[0] & 63)) - 1) : ~0ull;
      ok = (region[i] & m) == (ow[i] & m);
    }

    // decode the oracle's words (the staged stream aliases the exchange area, as on the GPU)
    std::vector<uint64_t> staged(words + 1, 0);
    std::copy(ow.begin(), ow.end(), staged.begin());
    std::vector<S> dec(256), od(256);
    quad([&](uint32_t r) {
      threadIdx.x = r;
      WordReader rd{staged.data(), 0};
      S v[64];
      Int* X = reinterpret_cast<Int*>(staged.data());
      if (rev)
        decode_block4<S, true>(rd, v, cp, X, tab, true);
      else
        decode_block4<S, false>(rd, v, cp, X, tab, true);
      for (int i = 0; i < 64; i++)
        dec[64 * r + i] = v[i];
    });
    oz_decompress(&j, od.data(), ow.data(), 0);
    const bool dok = std::memcmp(dec.data(), od.data(), 256 * sizeof(S)) == 0;
    if (!ok && getenv("QE_DEBUG") && bad == 0) {
      for (uint32_t b = 0; b < len[0]; b++)
        if (((region[b / 64] ^ ow[b / 64]) >> (b % 64)) & 1) {
          printf("first differing bit %u (got %d want %d)\n", b, (int)((region[b / 64] >> (b % 64)) & 1),
                 (int)((ow[b / 64] >> (b % 64)) & 1));
          break;
        }
    }
    if (!ok || !dok) {
      if (bad++ < 3)
        printf("%s trial %d kind %d: enc %s (len %u vs %llu) dec %s\n", name, t, kind, ok ? "ok" : "BAD", len[0],
               (unsigned long long)oend, dok ? "ok" : "BAD");
    }
  }
  printf("%-24s %d/%d bad\n", name, bad, trials);
  fflush(stdout);
  return bad;
}

int main()
{
  std::mt19937_64 rng(17);
  int bad = 0;
  struct M { const char* n; CodecParams c; } modes[] = {
    {"rate16", {4096, 4096, 64, -1074}},
    {"rate8", {2048, 2048, 64, -1074}},
    {"rate1.5", {384, 384, 64, -1074}},
    {"precision12", {1, 16658, 12, -1074}},
    {"precision32", {1, 16658, 32, -1074}},
    {"accuracy1e-3", {1, 16658, 64, -10}},
    {"reversible", {1, 16658, 64, -1075}},
    {"expert", {700, 900, 40, -60}},
  };
  for (int all : {0, 1}) {  // 1: every wave-level branch entered
    emu_any_all = all;
    for (auto& m : modes) {
      char nm[64];
      snprintf(nm, sizeof nm, "f32 %s%s", m.n, all ? " any" : "");
      bad += run<float>(m.c, 3, rng, 200, nm);
      snprintf(nm, sizeof nm, "f64 %s%s", m.n, all ? " any" : "");
      bad += run<double>(m.c, 4, rng, 200, nm);
    }
  }
  return bad != 0;
}
