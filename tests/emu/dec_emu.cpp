// Single-lane host check of the plane decoder fast path against the
// reference loop (decode.c:69-120) on random group sections.
#include <cstdio>
#include <cstdlib>
#include <random>
#include "codec_dev.h"
using namespace zfp_amd;

static void ref_plane(WordReader& r, uint64_t& x, uint32_t& bits, uint32_t& n) { decode_group_slow(r, x, bits, n); }

int main()
{
  uint32_t sq[256];
  for (int b = 0; b < 256; b++) sq[b] = squeeze_entry(b);
  std::mt19937_64 rng(7);
  long bad = 0, total = 0;
  for (int it = 0; it < 2000000; it++) {
    uint64_t w[8];
    for (auto& v : w) v = rng();
    // bias toward sparse sections
    int dens = it % 4;
    if (dens) for (int k = 0; k < dens; k++) w[0] &= rng(), w[1] &= rng();
    uint32_t n0 = (uint32_t)(rng() % 65), bits0 = (uint32_t)(rng() % 300) + 1;
    uint32_t pos0 = (uint32_t)(rng() % 64);
    WordReader a{w, pos0}, b{w, pos0};
    uint32_t na = n0, nb = n0, ba = bits0, bb = bits0;
    uint64_t xa = decode_plane64(a, sq, ba, na);
    // reference: verbatim then loop
    uint32_t m = nb < bb ? nb : bb;
    uint64_t xb = b.read(m);
    bb -= m;
    ref_plane(b, xb, bb, nb);
    total++;
    if (xa != xb || na != nb || ba != bb || a.pos != b.pos) {
      if (bad++ < 5)
        printf("mismatch n0=%u bits0=%u pos0=%llu: x %llx/%llx n %u/%u bits %u/%u pos %llu/%llu\n", n0, bits0,
               (unsigned long long)pos0, (unsigned long long)xa, (unsigned long long)xb, na, nb, ba, bb,
               (unsigned long long)a.pos, (unsigned long long)b.pos);
    }
  }
  printf("checked %ld, mismatches %ld\n", total, bad);
  return bad != 0;
}
