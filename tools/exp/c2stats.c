/* Experiment (not product, not test): how the C2 field's blocks (1024^3 f32
 * F1, rate 16: 1024 bits per block) are decoded by decode_planes32 -- planes
 * per block, and per wave of 64 blocks along x how many planes run in the
 * 32-bit body before some lane has more than 31 significant coefficients (the
 * switch to decode_plane64 for the rest of the block), and how often a
 * section reaches past the 31-bit window.  Oracle restatement of the cast,
 * transform and order.
 * build: gcc -O2 -I../../oracle c2stats.c -lm -o /tmp/c2stats */
#include <stdio.h>
#include <stdlib.h>
#include "../../oracle/zfp_oracle.c"

static double F(int x, int y, int z, int n)
{
  return sin(0.05 * x) * cos(0.03 * y) + 0.5 * sin(0.02 * z + 0.01 * x * y / n);
}

int main(int argc, char** argv)
{
  const int n = 1024, waves = argc > 1 ? atoi(argv[1]) : 400;
  srand(3);
  double planes_sum = 0, p32_sum = 0, wmax_planes = 0, long_sec = 0, slow32 = 0;
  long hist_switch[40] = {0};
  for (int wv = 0; wv < waves; wv++) {
    int by = rand() % (n / 4), bz = rand() % (n / 4), bx0 = (rand() % (n / 4 / 64)) * 64;
    uint32_t nk[64] = {0}, bits[64], prec[64];
    uint32_t u[64][64];
    for (int l = 0; l < 64; l++) {
      float v[64];
      for (int i = 0; i < 64; i++)
        v[i] = (float)F(4 * (bx0 + l) + (i & 3), 4 * by + ((i >> 2) & 3), 4 * bz + (i >> 4), n);
      int emax = oz_emax_f(v, 64);
      int32_t q[64];
      oz_cast_fwd_f(q, v, 64, emax);
      oz_xform_f(q, 3, 0, 0);
      for (int i = 0; i < 64; i++) u[l][i] = oz_to_nb_f(q[oz_perm3[i]]);
      bits[l] = 1024 - 9;
      int p = emax - (-1074) + 2 * 3 + 2;
      prec[l] = p < 0 ? 0 : (p > 32 ? 32 : p);
    }
    /* planes in lockstep, as decode_planes32 runs them */
    int kswitch = -1, planes_w = 0;
    for (int k = 31; k >= 0; k--) {
      int any = 0, any_big = 0;
      for (int l = 0; l < 64; l++) if (nk[l] > 31) any_big = 1;
      if (any_big && kswitch < 0) kswitch = 31 - k;
      for (int l = 0; l < 64; l++) {
        if (!bits[l] || (uint32_t)k < 32 - prec[l]) continue;
        any = 1;
        uint32_t m = nk[l] < bits[l] ? nk[l] : bits[l];
        bits[l] -= m;
        uint32_t nn = nk[l], used = 0;
        /* group section: simulate the reference loop */
        for (; bits[l] && nn < 64; nn++) {
          int more = 0;
          for (uint32_t i = nn; i < 64; i++) if ((u[l][i] >> k) & 1u) { more = 1; break; }
          bits[l]--; used++;
          if (!more) break;
          for (; bits[l] && nn < 63; nn++) { uint32_t b = (u[l][nn] >> k) & 1u; bits[l]--; used++; if (b) break; }
        }
        if (used > 32) long_sec++;
        if (kswitch < 0 && (used > 32 || bits[l] < 64)) slow32++;
        nk[l] = nn;
        planes_sum++;
      }
      if (any) planes_w++;
    }
    if (kswitch < 0) kswitch = planes_w;
    hist_switch[kswitch < 39 ? kswitch : 39]++;
    p32_sum += kswitch;
    wmax_planes += planes_w;
  }
  printf("C2 blocks: planes per block %.2f; per wave: planes %.2f, of them in the 32-bit body %.2f\n",
         planes_sum / (64.0 * waves), wmax_planes / waves, p32_sum / waves);
  printf("block-planes with a section past 32 bits %.2f per block; lanes taking decode_plane64 inside the 32-bit phase %.2f per wave\n",
         long_sec / (64.0 * waves), slow32 / waves);
  printf("32-bit planes per wave (hist):");
  for (int i = 0; i < 40; i++) if (hist_switch[i]) printf(" %d:%ld", i, hist_switch[i]);
  printf("\n");
  return 0;
}
