/* Experiment (not product, not test): statistics of the C5 field's 4D f32
 * reversible blocks from the oracle restatement -- how many blocks fail the
 * reversible cast, their precision and length, and how many of their planes
 * are coded with every coefficient already significant (pure verbatim planes).
 * build: gcc -O2 -I../../oracle c5stats.c -lm -o /tmp/c5stats */
#include <stdio.h>
#include <stdlib.h>
#include "../../oracle/zfp_oracle.c"

static double F(int x, int y, int z, int w, int n)
{
  return sin(0.05 * x) * cos(0.03 * y) + 0.5 * sin(0.02 * z + 0.01 * x * y / n) + 0.25 * cos(0.04 * w);
}

int main(int argc, char** argv)
{
  int n = 512, samples = argc > 1 ? atoi(argv[1]) : 20000;
  srand(1);
  long same = 0, hist_full[40] = {0}, hist_prec[40] = {0};
  double bits_same = 0, bits_not = 0, full_planes = 0, planes = 0;
  long over93 = 0; static uint32_t wu[16][256]; static int wprec[16]; static long cls[3], sec_hist[10], sec_wmax_hist[10], sec_fine[8]; double ext16 = 0, ext32 = 0, dec_it = 0, dec_win = 0, dec_seg = 0, gplanes = 0; static long lenhist_same[40], lenhist_not[40]; long wave_ns = 0, wave_cnt = 0; int wns = 0;
  uint64_t scratch[700];
  double wmaxprec = 0, wminfull = 0, wmaxnf = 0; int wmax = 0, wminf = 99, wnf = 0;
  for (int s = 0; s < samples; s++) {
    if (s % 16 == 0 && s) { wmaxprec += wmax; wminfull += wminf; wmaxnf += wnf; wmax = 0; wminf = 99; wnf = 0; }
    static int bx0, by0, bz0, bw0;
    if (s % 16 == 0) { bx0 = rand() % (n / 4 / 16) * 16; by0 = rand() % (n / 4); bz0 = rand() % (n / 4); bw0 = rand() % 16; }
    int bx = bx0 + s % 16, by = by0, bz = bz0, bw = bw0;
    (void)by;
    float v[256];
    for (int i = 0; i < 256; i++)
      v[i] = (float)F(4 * bx + (i & 3), 4 * by + ((i >> 2) & 3), 4 * bz + ((i >> 4) & 3), 4 * bw + (i >> 6), n);
    oz_params p = {0, 8 * 256 * 4 + 600, 32, -1075};
    memset(scratch, 0, sizeof scratch);
    oz_bits st = {scratch, 0};
    uint32_t len = oz_encode_block_f(&st, &p, 4, v);
    if (len > 5952) over93++;
    /* replicate the transform to count planes */
    int emax = oz_emax_f(v, 256);
    int32_t q[256];
    float back[256];
    oz_cast_fwd_f(q, v, 256, emax);
    oz_cast_inv_f(q, back, 256, emax);
    int ok = !memcmp(back, v, sizeof back);
    if (!ok) {
      memcpy(q, v, sizeof q);
      for (int i = 0; i < 256; i++) if (q[i] < 0) q[i] = (int32_t)((uint32_t)q[i] ^ 0x7fffffffu);
    }
    oz_xform_f(q, 4, 0, 1);
    uint32_t u[256], all = 0;
    for (int i = 0; i < 256; i++) { u[i] = oz_to_nb_f(q[oz_perm4[i]]); all |= u[i]; }
    int prec = all ? 32 - __builtin_ctz(all) : 1;
    hist_prec[prec]++;
    memcpy(wu[s % 16], u, sizeof u); wprec[s % 16] = prec;
    if (s % 16 == 15) {
      /* per plane of the wave: does some lane (block q, segment r) have xs >= 2^16 / 2^32 */
      uint32_t nn[16] = {0}, nk[16] = {0};
      for (int k = 31; k >= 0; k--) {
        int any = 0, e16 = 0, e32 = 0;
        for (int q = 0; q < 16; q++) {
          if (k < 32 - wprec[q]) continue;
          any = 1;
          for (int r = 0; r < 4; r++) {
            int base = 64 * r, nr = (int)nn[q] - base; nr = nr < 0 ? 0 : nr > 64 ? 64 : nr;
            uint64_t P = 0;
            for (int j = 0; j < 64; j++) P |= (uint64_t)((wu[q][base + j] >> k) & 1) << j;
            uint64_t xs = nr < 64 ? P >> nr : 0;
            if (xs >> 16) e16 = 1;
            if (xs >> 32) e32 = 1;
          }
          for (int i = 255; i >= (int)nn[q]; i--) if ((wu[q][i] >> k) & 1) { nn[q] = i + 1; break; }
        }
        if (any) { gplanes++; ext16 += e16; ext32 += e32; }
        /* decode cost of this plane: serial group-test iterations (max over quads) and, for a
           windowed parse, new ones per 128-bit window of the group bits (max over lanes) */
        int it_max = 0, win_max = 0, seg_max = 0, sec_wmax = 0, anyone = 0, anylong = 0;
        for (int q = 0; q < 16; q++) {
          if (k < 32 - wprec[q] || nk[q] >= 256) continue;
          uint32_t n0 = nk[q], tpos = 0, it = 1, cnt[5] = {0}, segc[4] = {0};
          for (uint32_t i = n0; i < 256; i++) {
            int b = (wu[q][i] >> k) & 1;
            int rest = 0;
            for (uint32_t j = i; j < 256; j++) rest |= (wu[q][j] >> k) & 1;
            if (!rest) break;
            if (b) { cnt[tpos / 128 < 4 ? tpos / 128 : 4]++; segc[i / 64]++; it++; tpos += 2; nk[q] = i + 1; } else tpos++;
          }
          if (it > it_max) it_max = it;
          if (it > 1) { anyone = 1; if (tpos + 1 > 62 || nk[q] == 256) anylong = 1; }
          /* section bits after the lead test: tokens up to the stop + the stop test */
          if (it > 1) { uint32_t sl = tpos + 1; sec_hist[sl / 64 < 9 ? sl / 64 : 9]++; if ((int)sl > sec_wmax) sec_wmax = sl; }
          for (int w = 0; w < 5; w++) if ((int)cnt[w] > win_max) win_max = cnt[w];
          for (int w = 0; w < 4; w++) if ((int)segc[w] > seg_max) seg_max = segc[w];
        }
        if (any) { cls[anyone + anylong]++; sec_wmax_hist[sec_wmax / 64 < 9 ? sec_wmax / 64 : 9]++; if (sec_wmax < 64) sec_fine[sec_wmax / 8]++; dec_it += it_max; dec_win += win_max; dec_seg += seg_max; }
      }
    }
    /* n after each plane: the top one's index + 1 */
    uint32_t nn = 0; int full = 0;
    for (int k = 31; k >= 32 - prec; k--) {
      if (nn == 256) full++;
      for (int i = 255; i >= (int)nn; i--) if ((u[i] >> k) & 1) { nn = i + 1; break; }
    }
    hist_full[full]++;
    if (prec > wmax) wmax = prec;
    if (full < wminf) wminf = full;
    if (prec - full > wnf) wnf = prec - full;
    full_planes += full; planes += prec;
    if (ok) { same++; bits_same += len; lenhist_same[len / 256]++; } else { bits_not += len; lenhist_not[len / 256]++; wns++; }
    if (s % 16 == 15) { wave_cnt++; if (wns) wave_ns++; wns = 0; }
  }
  printf("samples %d same %ld (%.1f%%) mean bits same %.0f not-same %.0f  >5952 bits: %.2f%%\n", samples, same,
         100.0 * same / samples, bits_same / (same ? same : 1), bits_not / (samples - same ? samples - same : 1),
         100.0 * over93 / samples);
  printf("planes coded %.2f, of them with all 256 significant %.2f\n", planes / samples, full_planes / samples);
  printf("per wave of 16: mean max prec %.2f, mean min full planes %.2f, mean max non-full planes %.2f\n",
         wmaxprec / (samples / 16 - 1), wminfull / (samples / 16 - 1), wmaxnf / (samples / 16 - 1));
  printf("waves with a not-same block: %.1f%%\n", 100.0 * wave_ns / wave_cnt);
  printf("same len hist (256-bit bins):"); for (int i = 0; i < 40; i++) if (lenhist_same[i]) printf(" %d:%ld", i, lenhist_same[i]);
  printf("\nnot-same len hist:"); for (int i = 0; i < 40; i++) if (lenhist_not[i]) printf(" %d:%ld", i, lenhist_not[i]);
  printf("\n");
  printf("per wave: planes %.2f, planes taking ext (xs >= 2^16) %.2f, (xs >= 2^32) %.2f\n", gplanes / (samples / 16), ext16 / (samples / 16), ext32 / (samples / 16));
  printf("per wave: serial group-test iterations %.1f (sum over planes of the max over quads), max new ones per 128-bit window %.1f, per 64-coefficient segment %.1f\n",
         dec_it / (samples / 16), dec_win / (samples / 16), dec_seg / (samples / 16));
  printf("section bits per block-plane (64-bit bins):"); for (int i = 0; i < 10; i++) printf(" %d:%ld", i, sec_hist[i]);
  printf("\nper wave: planes with no new one %.2f, all sections in one 63-bit window %.2f, longer %.2f", cls[0] / (samples / 16.), cls[1] / (samples / 16.), cls[2] / (samples / 16.));
  printf("\nwave max section bits < 64 (8-bit bins):"); for (int i = 0; i < 8; i++) printf(" %d:%ld", i, sec_fine[i]);
  printf("\nwave max section bits per plane (64-bit bins):"); for (int i = 0; i < 10; i++) printf(" %d:%ld", i, sec_wmax_hist[i]);
  printf("\n");
  printf("prec hist:");
  for (int i = 0; i < 33; i++) if (hist_prec[i]) printf(" %d:%ld", i, hist_prec[i]);
  printf("\nfull-plane hist:");
  for (int i = 0; i < 33; i++) if (hist_full[i]) printf(" %d:%ld", i, hist_full[i]);
  printf("\n");
  return 0;
}
