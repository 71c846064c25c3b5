// Single-lane host check of the plane decoder fast path against the
// reference loop (decode.c:69-120) on random group sections.
#include <cstdio>
#include <cstdlib>
#include <random>
#include "codec_dev.h"
using namespace zfp_amd;

// SIZE: coefficients per block (64: 3D; 16, 4: 2D, 1D)
template <int SIZE>
static long check(std::mt19937_64& rng, const uint32_t* sq, int iters, long& total)
{
  long bad = 0;
  for (int it = 0; it < iters; it++) {
    uint64_t w[8];
    for (auto& v : w) v = rng();
    // bias toward sparse sections
    int dens = it % 4;
    if (dens) for (int k = 0; k < dens; k++) w[0] &= rng(), w[1] &= rng();
    uint32_t n0 = (uint32_t)(rng() % (SIZE + 1)), bits0 = (uint32_t)(rng() % 300) + 1;
    uint32_t pos0 = (uint32_t)(rng() % 64);
    WordReader a{w, pos0}, b{w, pos0};
    uint32_t na = n0, nb = n0, ba = bits0, bb = bits0;
    uint64_t xa = decode_plane64<true, SIZE>(a, sq, ba, na);
    // reference: verbatim then loop
    uint32_t m = nb < bb ? nb : bb;
    uint64_t xb = b.read(m);
    bb -= m;
    decode_group_slow<SIZE>(b, xb, bb, nb);
    total++;
    if (xa != xb || na != nb || ba != bb || a.pos != b.pos) {
      if (bad++ < 5)
        printf("SIZE %d mismatch n0=%u bits0=%u pos0=%llu: x %llx/%llx n %u/%u bits %u/%u pos %llu/%llu\n", SIZE, n0, bits0,
               (unsigned long long)pos0, (unsigned long long)xa, (unsigned long long)xb, na, nb, ba, bb,
               (unsigned long long)a.pos, (unsigned long long)b.pos);
    }
  }
  return bad;
}

int main()
{
  uint32_t sq[256];
  for (int b = 0; b < 256; b++) sq[b] = squeeze_entry(b);
  std::mt19937_64 rng(7);
  long total = 0;
  const long bad = check<64>(rng, sq, 2000000, total) + check<16>(rng, sq, 500000, total) + check<4>(rng, sq, 500000, total);
  printf("checked %ld, mismatches %ld\n", total, bad);
  return bad != 0;
}
