// Plane coder (codec_dev.h code_planes) against a literal restatement of the
// reference's embedded coder (src/template/encode.c:92-132, encode_few_ints):
// adversarial plane patterns -- all-ones 16-bit units, tops at bit 63, long
// jumps of significance, budgets cut at every offset -- for 32 and 64 planes.
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>
#include "codec_dev.h"
using namespace zfp_amd;

// reference: encode.c:92-132 with a 64-bit LSB-first writer
static uint32_t ref_code(std::vector<uint64_t>& w, uint32_t pos0, uint32_t maxbits, uint32_t maxprec,
                         const uint64_t* planes, int prec, uint32_t size = 64)
{
  uint32_t kmin = (uint32_t)prec > maxprec ? prec - maxprec : 0;
  uint32_t bits = maxbits, n = 0, pos = pos0;
  auto put = [&](uint32_t b) { if (b) w[pos >> 6] |= 1ull << (pos & 63); pos++; return b; };
  for (uint32_t k = prec; bits && k-- > kmin;) {
    uint64_t x = planes[k];
    uint32_t m = n < bits ? n : bits;
    bits -= m;
    for (uint32_t i = 0; i < m; i++) put((x >> i) & 1);
    x = m < 64 ? x >> m : 0;
    for (; bits && n < size; x >>= 1, n++) {
      bits--;
      if (put(x != 0)) {
        for (; bits && n < size - 1; x >>= 1, n++) {
          bits--;
          if (put(x & 1u)) break;
        }
      } else
        break;
    }
  }
  return pos - pos0;
}

template <int PREC, bool PLIM, int SIZE = 64>
static int run(std::mt19937_64& rng, int trials)
{
  uint32_t lut[256];
  for (int b = 0; b < 256; b++) lut[b] = dbl_entry(b);
  int bad = 0;
  for (int t = 0; t < trials; t++) {
    uint64_t P[PREC];
    int kind = t % 7;
    for (int k = 0; k < PREC; k++) {
      uint64_t r = rng();
      switch (kind) {
        case 0: P[k] = r; break;                                      // dense
        case 1: P[k] = (rng() % 4 == 0) ? r & rng() & rng() : 0; break;  // sparse
        case 2: P[k] = (k == PREC - 1 - (int)(t % 5)) ? 0xffffull << (16 * (rng() % 4)) : r & 0xffff0000ffffull; break;
        case 3: P[k] = (rng() % 3 == 0) ? (1ull << 63) | (r & 0xffff) : (r & 0x00ff00ff00ff00ffull); break;
        case 4: P[k] = (k % 9 == 0) ? ~0ull : 0; break;
        case 5: P[k] = (k == PREC - 2) ? (r | (1ull << (rng() % 64))) >> (rng() % 40) : r >> (rng() % 64); break;
        default: P[k] = (k > PREC - 4) ? (1ull << (rng() % 64)) : r & (r >> 3); break;
      }
    }
    for (int k = 0; k < PREC; k++)
      P[k] &= SIZE == 64 ? ~0ull : (1ull << SIZE) - 1;  // 1D/2D blocks: 4 or 16 coefficients
    uint32_t Pl[PREC], Ph[PREC];
    for (int k = 0; k < PREC; k++) Pl[k] = (uint32_t)P[k], Ph[k] = (uint32_t)(P[k] >> 32);
    const uint32_t pos0 = 1 + (uint32_t)(rng() % 40);
    const uint32_t budgets[3] = {4096 * 2, 64 + (uint32_t)(rng() % 2000), 1 + (uint32_t)(rng() % 300)};
    for (uint32_t lim_bits : budgets) {
      uint32_t maxprec = (PLIM && t % 3 == 0) ? 1 + (uint32_t)(rng() % PREC) : 64;
      std::vector<uint64_t> rw(200, 0), slot(200, 0);
      uint32_t rlen = ref_code(rw, pos0, lim_bits, maxprec, P, PREC, SIZE);
      OrSlot os{slot.data(), 399};
      uint32_t end = code_planes<PREC, PLIM, SIZE>(os, lut, pos0, pos0 + lim_bits, maxprec, Pl, Ph);
      bool ok = end - pos0 == rlen;
      uint32_t e = pos0 + rlen;
      for (uint32_t i = 0; ok && i < (e + 63) / 64; i++) {
        uint64_t m = (i == e / 64 && (e & 63)) ? ((1ull << (e & 63)) - 1) : ~0ull;
        ok = (slot[i] & m) == (rw[i] & m);
      }
      if (!ok && bad++ < 5)
        printf("SIZE %d PREC %d PLIM %d trial %d kind %d lim %u maxprec %u: len %u vs ref %u\n", SIZE, PREC, PLIM, t, kind, lim_bits, maxprec,
               end - pos0, rlen);
    }
  }
  printf("size%d planes%d plim%d mismatches %d\n", SIZE, PREC, PLIM, bad);
  return bad;
}

// The fixed-rate f32 coder (code_planes_fr32): its 32-bit plane body runs while
// the wave's planes have nothing in coefficients 32..63 and n < 32, then it
// hands over to code_planes.  Patterns keep the high half empty for a varying
// number of top planes and hit the 32-bit body's edges: xs == 0xffff (33 group
// bits), tops past bit 15, n reaching 32, empty planes, budgets cut anywhere.
static int run_fr32(std::mt19937_64& rng, int trials)
{
  static std::vector<uint64_t> arena(8192, 0);
  zfp_emu_lds_base = reinterpret_cast<char*>(arena.data());
  uint32_t* lut = reinterpret_cast<uint32_t*>(arena.data()) + 64;
  for (int b = 0; b < 256; b++) lut[b] = kCoderTables.dbl[b], lut[256 + b] = kCoderTables.lead[b];
  uint64_t* slot = arena.data() + 1024;
  int bad = 0;
  for (int t = 0; t < trials; t++) {
    uint64_t P[32];
    const int kind = t % 8;
    const int khi = (int)(rng() % 33);  // planes >= khi: low half only
    for (int k = 0; k < 32; k++) {
      uint64_t r = rng();
      uint64_t lo;
      switch (kind) {
        case 0: lo = r & 0xffffffffull; break;
        case 1: lo = (rng() % 3 == 0) ? r & rng() & 0xffffffffull : 0; break;
        case 2: lo = (rng() % 4 == 0) ? 0xffffull << (rng() % 17) : (r & 0xffff); break;  // 0xffff units
        case 3: lo = (rng() % 5 == 0) ? (1ull << 31) : (r & 0xff); break;                  // n jumps to 32
        case 4: lo = (k % 7 == 0) ? 0xffffffffull : 0; break;
        case 5: lo = (r & 0xffffffffull) >> (rng() % 32); break;
        case 6: lo = (k > 24) ? (1ull << (rng() % 32)) : (r & (r >> 5) & 0xffffffffull); break;
        default: lo = (rng() % 2) ? 0xffff0000ull | (r & 0xffff) : ((r & 0xffff) << 16); break;  // tops past bit 15
      }
      const uint64_t hi = (t & 8) ? ((rng() % 3 == 0) ? (1ull << (32 + rng() % 3)) : 0ull) : (r & 0xffffffff00000000ull);
      P[k] = k >= khi ? lo : (lo | hi);
    }
    uint32_t Pl[32], Ph[32];
    for (int k = 0; k < 32; k++) Pl[k] = (uint32_t)P[k], Ph[k] = (uint32_t)(P[k] >> 32);
    const uint32_t pos0 = 1 + (uint32_t)(rng() % 40);
    const uint32_t budgets[3] = {4096, 64 + (uint32_t)(rng() % 1500), 1 + (uint32_t)(rng() % 300)};
    for (uint32_t lim_bits : budgets) {
      std::vector<uint64_t> rw(200, 0);
      std::fill(slot, slot + 200, 0ull);
      const uint32_t rlen = ref_code(rw, pos0, lim_bits, 64, P, 32);
      code_planes_fr32(reinterpret_cast<uint32_t*>(slot), 399, lut, pos0, pos0 + lim_bits, Pl, Ph);
      const uint32_t e = pos0 + rlen;
      bool ok = true;
      for (uint32_t i = 0; ok && i < (e + 63) / 64; i++) {
        uint64_t m = (i == e / 64 && (e & 63)) ? ((1ull << (e & 63)) - 1) : ~0ull;
        ok = (slot[i] & m) == (rw[i] & m);
      }
      if (!ok && bad++ < 5)
        printf("fr32 trial %d kind %d khi %d lim %u: stream differs\n", t, kind, khi, lim_bits);
    }
  }
  printf("fr32 mismatches %d\n", bad);
  return bad;
}

// The 32-plane decoder (decode_planes32) on streams written by the reference
// coder loop: the same plane patterns as run_fr32, budgets cut anywhere and
// precision limits; planes and consumed bits must match.
static int run_dec32(std::mt19937_64& rng, int trials)
{
  uint32_t sq[256];
  for (int b = 0; b < 256; b++) sq[b] = squeeze_entry(b);
  int bad = 0;
  for (int t = 0; t < trials; t++) {
    uint64_t P[32];
    const int kind = t % 8;
    const int khi = (int)(rng() % 33);
    for (int k = 0; k < 32; k++) {
      uint64_t r = rng();
      uint64_t lo;
      switch (kind) {
        case 0: lo = r & 0xffffffffull; break;
        case 1: lo = (rng() % 3 == 0) ? r & rng() & 0xffffffffull : 0; break;
        case 2: lo = (rng() % 4 == 0) ? 0xffffull << (rng() % 17) : (r & 0xffff); break;
        case 3: lo = (rng() % 5 == 0) ? (1ull << 31) : (r & 0xff); break;
        case 4: lo = (k % 7 == 0) ? 0xffffffffull : 0; break;
        case 5: lo = (r & 0xffffffffull) >> (rng() % 32); break;
        case 6: lo = (k > 24) ? (1ull << (rng() % 32)) : (r & (r >> 5) & 0xffffffffull); break;
        default: lo = (rng() % 2) ? 0xffff0000ull | (r & 0xffff) : ((r & 0xffff) << 16); break;
      }
      // high half: dense, or only coefficients 32..34 (sections ending right at the 32-bit edge)
      const uint64_t hi = (t & 8) ? ((rng() % 3 == 0) ? (1ull << (32 + rng() % 3)) : 0ull) : (r & 0xffffffff00000000ull);
      if (t & 16)
        lo &= (1ull << (rng() % 33)) - 1 | (1ull << 31);
      P[k] = k >= khi ? lo : (lo | hi);
    }
    const uint32_t budgets[3] = {4096, 64 + (uint32_t)(rng() % 1500), 1 + (uint32_t)(rng() % 300)};
    for (uint32_t budget : budgets) {
      const uint32_t maxprec = (t % 3 == 0) ? 1 + (uint32_t)(rng() % 32) : 64;
      std::vector<uint64_t> w(200, 0);
      const uint32_t len = ref_code(w, 0, budget, maxprec, P, 32);
      // what the reference decoder reconstructs: the coded planes, bits past the cut zero
      uint64_t want[32];
      {
        std::vector<uint64_t> w2(200, 0);
        for (int k = 0; k < 32; k++) want[k] = 0;
        // decode with the literal loop (decode_planes64 is itself checked against it in dec_emu)
        WordReader r0{w.data(), 0};
        decode_planes64<32>(r0, sq, budget, maxprec, want);
      }
      uint64_t got[32];
      WordReader r{w.data(), 0};
      const uint32_t used = decode_planes32(r, sq, budget, maxprec, got);
      bool ok = used == len && r.pos == len;
      for (int k = 0; ok && k < 32; k++) ok = got[k] == want[k];
      if (!ok && bad++ < 5)
        printf("dec32 trial %d kind %d khi %d budget %u maxprec %u: used %u vs %u\n", t, kind, khi, budget, maxprec, used,
               len);
    }
  }
  printf("dec32 mismatches %d\n", bad);
  return bad;
}

int main()
{
  std::mt19937_64 rng(12345);
  int bad = 0;
  for (int all : {0, 1}) {
    emu_any_all = all;
    bad += run_fr32(rng, 40000);
    bad += run_dec32(rng, 20000);
  }
  for (int all : {0, 1}) {  // 1: every wave-level branch entered (other lanes need it)
    emu_any_all = all;
    bad += run<32, true>(rng, 20000) + run<64, true>(rng, 10000) + run<32, false>(rng, 20000) + run<64, false>(rng, 10000);
    bad += run<32, true, 16>(rng, 10000) + run<64, true, 16>(rng, 5000) + run<32, false, 16>(rng, 10000);
    bad += run<32, true, 4>(rng, 10000) + run<64, true, 4>(rng, 5000) + run<64, false, 4>(rng, 5000);
  }
  printf("mismatches %d\n", bad);
  return bad != 0;
}
