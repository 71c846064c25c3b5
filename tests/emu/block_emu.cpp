// Single-lane host run of the device block codec (block3.h) against the C
// oracle: every mode, float and double, random and special blocks.  Catches
// per-lane logic errors without a GPU; wave-level behaviour is not modelled.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
#include "block3.h"
using namespace zfp_amd;

extern "C" {
typedef struct { uint32_t minbits, maxbits, maxprec; int32_t minexp; } oz_params;
typedef struct { int32_t type, pad_; oz_params p; uint64_t n[4]; int64_t s[4]; uint64_t f[4]; uint64_t e[4]; } oz_job;
uint64_t oz_compress(const oz_job* j, const void* data, uint64_t* words, uint64_t bitpos);
uint64_t oz_decompress(const oz_job* j, void* data, const uint64_t* words, uint64_t bitpos);
}

template <typename S>
static int run(const CodecParams& cp, int type, std::mt19937_64& rng, int trials, const char* name)
{
  // "LDS" arena: the fixed-rate f32 coder addresses its tables and slot by LDS
  // byte address (offsets from zfp_emu_lds_base)
  static std::vector<uint64_t> arena(4096, 0);
  zfp_emu_lds_base = reinterpret_cast<char*>(arena.data());
  uint32_t* lut = reinterpret_cast<uint32_t*>(arena.data()) + 64;  // dbl[256], lead[256]
  uint32_t sq[256];
  for (int b = 0; b < 256; b++) lut[b] = kCoderTables.dbl[b], lut[256 + b] = kCoderTables.lead[b], sq[b] = squeeze_entry(b);
  for (int b = 0; b < 256; b++)
    if (lut[b] != dbl_entry(b)) { printf("CoderTables.dbl[%d] differs from dbl_entry\n", b); return 1; }
  int bad = 0;
  for (int t = 0; t < trials; t++) {
    S v[64], orig[64];
    int kind = t % 6;
    std::normal_distribution<double> nd(0, 1);
    for (int i = 0; i < 64; i++) {
      double x = kind == 0 ? nd(rng) : kind == 1 ? std::sin(0.1 * i + t) : kind == 2 ? nd(rng) * 1e-30
               : kind == 3 ? (double)(rng() % 7) - 3 : kind == 4 ? nd(rng) * 1e20 : (i == 5 ? 0 : 0.0);
      orig[i] = v[i] = (S)x;
    }
    oz_job j{};
    j.type = type;
    j.p = {cp.minbits, cp.maxbits, cp.maxprec, cp.minexp};
    for (int a = 0; a < 3; a++) j.n[a] = 4, j.f[a] = 0, j.e[a] = 4;
    j.s[0] = 1, j.s[1] = 4, j.s[2] = 16;
    std::vector<uint64_t> ow(600, 0), slot(600, 0);
    uint64_t oend = oz_compress(&j, orig, ow.data(), 0);
    OrSlot os{slot.data(), 1199};
    uint32_t len = encode_block3<S, false>(os, lut, v, cp, [&](S (&r)[64]) { for (int i = 0; i < 64; i++) r[i] = orig[i]; });
    if (cp.minexp < kMinExp) {
      S v2[64];
      for (int i = 0; i < 64; i++) v2[i] = orig[i];
      std::fill(slot.begin(), slot.end(), 0);
      OrSlot os2{slot.data(), 1199};
      len = encode_block3<S, true>(os2, lut, v2, cp, [&](S (&r)[64]) { for (int i = 0; i < 64; i++) r[i] = orig[i]; });
    } else if (cp.minbits == cp.maxbits && cp.maxprec >= 64) {
      // fixed-rate specialisation (the aligned kernel's coder)
      S v2[64];
      for (int i = 0; i < 64; i++) v2[i] = orig[i];
      uint64_t* slot2 = arena.data() + 1024;  // inside the arena (see above)
      std::fill(slot2, slot2 + 600, 0ull);
      OrSlot os2{slot2, 1199};
      uint32_t len2 = encode_block3<S, false, true>(os2, lut, v2, cp, [&](S (&r)[64]) { for (int i = 0; i < 64; i++) r[i] = orig[i]; });
      bool same = len2 == len;
      for (uint32_t i = 0; same && i < (len + 63) / 64; i++) {
        uint64_t m = (i == len / 64 && (len & 63)) ? ((1ull << (len & 63)) - 1) : ~0ull;
        same = (slot2[i] & m) == (slot[i] & m);
      }
      if (!same)
        len = 0xffffffffu;  // reported as an encode mismatch below
    }
    if (sizeof(S) == 8 && cp.maxprec <= 32 && cp.minexp >= kMinExp) {
      // double with maxprec <= 32: the high-planes-only coder/decoder (HI)
      S v2[64];
      for (int i = 0; i < 64; i++) v2[i] = orig[i];
      std::vector<uint64_t> slot2(600, 0);
      OrSlot os2{slot2.data(), 1199};
      uint32_t len2 = encode_block3<S, false, false, true>(os2, lut, v2, cp, [&](S (&r)[64]) { for (int i = 0; i < 64; i++) r[i] = orig[i]; });
      bool same = len2 == len;
      for (uint32_t i = 0; same && i < (len + 63) / 64; i++) {
        uint64_t m = (i == len / 64 && (len & 63)) ? ((1ull << (len & 63)) - 1) : ~0ull;
        same = (slot2[i] & m) == (slot[i] & m);
      }
      S dh[64];
      const bool any_all = emu_any_all;
      emu_any_all = false;
      WordReader rh{slot2.data(), 0};
      uint32_t usedh = decode_block3<S, false, true>(rh, sq, dh, cp);
      emu_any_all = any_all;
      S dref[64];
      WordReader rr{slot.data(), 0};
      emu_any_all = false;
      decode_block3<S, false>(rr, sq, dref, cp);
      emu_any_all = any_all;
      if (!same || usedh != len || std::memcmp(dh, dref, sizeof dh) != 0)
        len = 0xfffffffeu;  // reported as an encode mismatch below
    }
    bool ok = len == oend;
    for (uint32_t i = 0; ok && i < (len + 63) / 64; i++) {
      uint64_t m = (i == len / 64 && (len & 63)) ? ((1ull << (len & 63)) - 1) : ~0ull;
      ok = (slot[i] & m) == (ow[i] & m);
    }
    // decode the oracle's words
    S d[64], od[64];
    const bool any_all = emu_any_all;
    emu_any_all = false;  // decoder loops gate on __any; run them as a lone lane
    WordReader r{ow.data(), 0};
    uint32_t used = (cp.minexp < kMinExp) ? decode_block3<S, true>(r, sq, d, cp) : decode_block3<S, false>(r, sq, d, cp);
    oz_decompress(&j, od, ow.data(), 0);
    emu_any_all = any_all;
    bool dok = used == oend && std::memcmp(d, od, sizeof d) == 0;
    if (!ok || !dok) {
      if (bad++ < 3)
        printf("%s trial %d kind %d: enc %s (len %u vs %llu) dec %s (used %u)\n", name, t, kind, ok ? "ok" : "BAD", len,
               (unsigned long long)oend, dok ? "ok" : "BAD", used);
    }
  }
  printf("%-24s %d/%d bad\n", name, bad, trials);
  return bad;
}

int main()
{
  std::mt19937_64 rng(11);
  int bad = 0;
  struct M { const char* n; CodecParams f, d; } modes[] = {
    {"rate16", {1024, 1024, 64, -1074}, {1024, 1024, 64, -1074}},
    {"rate8", {512, 512, 64, -1074}, {512, 512, 64, -1074}},
    {"rate1.5", {96, 96, 64, -1074}, {96, 96, 64, -1074}},
    {"precision12", {1, 16658, 12, -1074}, {1, 16658, 12, -1074}},
    {"precision32", {1, 16658, 32, -1074}, {1, 16658, 32, -1074}},
    {"accuracy1e-3", {1, 16658, 64, -10}, {1, 16658, 64, -10}},
    {"reversible", {1, 16658, 64, -1075}, {1, 16658, 64, -1075}},
    {"expert", {700, 900, 40, -60}, {700, 900, 40, -60}},
  };
  for (int all : {0, 1}) {  // 1: every wave-level branch of the encoder entered
    emu_any_all = all;
    for (auto& m : modes) {
      char nm[64];
      snprintf(nm, sizeof nm, "f32 %s%s", m.n, all ? " any" : "");
      bad += run<float>(m.f, 3, rng, 3000, nm);
      snprintf(nm, sizeof nm, "f64 %s%s", m.n, all ? " any" : "");
      bad += run<double>(m.d, 4, rng, 3000, nm);
    }
  }
  return bad != 0;
}
