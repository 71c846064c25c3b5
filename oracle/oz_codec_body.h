/*
 * TEST INFRASTRUCTURE ONLY -- CPU oracle for the zfp block codec.
 * Included twice by oracle/zfp_oracle.c (single and double precision).
 *
 * Parameter macros:  OZ_SFX  OZ_REAL  OZ_INT  OZ_UINT  OZ_EBITS  OZ_PBITS
 *                    OZ_NBMASK  OZ_TCMASK  OZ_FREXP  OZ_LDEXP  OZ_FABS
 *
 * Every function names the reference file:line whose behaviour it restates
 * (paths relative to the SEP-software/zfp-par root).
 */

#define OZ_CAT2(a, b) a##b
#define OZ_CAT(a, b) OZ_CAT2(a, b)
#define OZ_FN(name) OZ_CAT(name, OZ_SFX)
#define OZ_INTPREC ((uint32_t)(8 * sizeof(OZ_INT)))
#define OZ_EBIAS ((1 << (OZ_EBITS - 1)) - 1)

/* Largest block exponent: encodef.c:11-40.  |x| maxed with `<` so NaN never
 * wins; frexp of the max with the subnormal clamp MAX(e, 1-EBIAS).  frexp is
 * glibc's (it leaves e untouched for +inf, which the clamp then lifts). */
static int OZ_FN(oz_emax_)(const OZ_REAL* v, uint32_t n)
{
  OZ_REAL top = 0;
  for (uint32_t i = 0; i < n; i++) {
    OZ_REAL a = OZ_FABS(v[i]);
    if (top < a)
      top = a;
  }
  int e = -OZ_EBIAS;
  if (top > 0) {
    OZ_FREXP(top, &e);
    if (e < 1 - OZ_EBIAS)
      e = 1 - OZ_EBIAS;
  }
  return e;
}

/* Block-floating-point cast: encodef.c:44-59 -- scale by 2^(intprec-2-emax)
 * in the scalar type, then C truncating conversion. */
static void OZ_FN(oz_cast_fwd_)(OZ_INT* q, const OZ_REAL* v, uint32_t n, int emax)
{
  OZ_REAL scale = OZ_LDEXP((OZ_REAL)1, (int)OZ_INTPREC - 2 - emax);
  for (uint32_t i = 0; i < n; i++)
    q[i] = (OZ_INT)(scale * v[i]);
}

/* Inverse cast: codecf.c:17-32 -- (Scalar)int times 2^(emax-intprec+2). */
static void OZ_FN(oz_cast_inv_)(const OZ_INT* q, OZ_REAL* v, uint32_t n, int emax)
{
  OZ_REAL scale = OZ_LDEXP((OZ_REAL)1, emax - ((int)OZ_INTPREC - 2));
  for (uint32_t i = 0; i < n; i++)
    v[i] = (OZ_REAL)(scale * (OZ_REAL)q[i]);
}

/* wrap-around helpers: the reference relies on two's complement wrap */
#define OZ_ADD(a, b) ((OZ_INT)((OZ_UINT)(a) + (OZ_UINT)(b)))
#define OZ_SUB(a, b) ((OZ_INT)((OZ_UINT)(a) - (OZ_UINT)(b)))
#define OZ_SHL1(a) ((OZ_INT)((OZ_UINT)(a) << 1))

/* Forward decorrelating lift of one 4-vector at stride s: encode.c:31-56. */
static void OZ_FN(oz_lift_fwd_)(OZ_INT* p, ptrdiff_t s)
{
  OZ_INT x = p[0], y = p[s], z = p[2 * s], w = p[3 * s];
  x = OZ_ADD(x, w); x >>= 1; w = OZ_SUB(w, x);
  z = OZ_ADD(z, y); z >>= 1; y = OZ_SUB(y, z);
  x = OZ_ADD(x, z); x >>= 1; z = OZ_SUB(z, x);
  w = OZ_ADD(w, y); w >>= 1; y = OZ_SUB(y, w);
  w = OZ_ADD(w, y >> 1); y = OZ_SUB(y, w >> 1);
  p[0] = x; p[s] = y; p[2 * s] = z; p[3 * s] = w;
}

/* Inverse lift: decode.c:9-34. */
static void OZ_FN(oz_lift_inv_)(OZ_INT* p, ptrdiff_t s)
{
  OZ_INT x = p[0], y = p[s], z = p[2 * s], w = p[3 * s];
  y = OZ_ADD(y, w >> 1); w = OZ_SUB(w, y >> 1);
  y = OZ_ADD(y, w); w = OZ_SHL1(w); w = OZ_SUB(w, y);
  z = OZ_ADD(z, x); x = OZ_SHL1(x); x = OZ_SUB(x, z);
  y = OZ_ADD(y, z); z = OZ_SHL1(z); z = OZ_SUB(z, y);
  w = OZ_ADD(w, x); x = OZ_SHL1(x); x = OZ_SUB(x, w);
  p[0] = x; p[s] = y; p[2 * s] = z; p[3 * s] = w;
}

/* Reversible (Lorenzo) lifts: revencode.c:7-30, revdecode.c:7-29. */
static void OZ_FN(oz_rlift_fwd_)(OZ_INT* p, ptrdiff_t s)
{
  OZ_INT x = p[0], y = p[s], z = p[2 * s], w = p[3 * s];
  w = OZ_SUB(w, z); z = OZ_SUB(z, y); y = OZ_SUB(y, x);
  w = OZ_SUB(w, z); z = OZ_SUB(z, y);
  w = OZ_SUB(w, z);
  p[0] = x; p[s] = y; p[2 * s] = z; p[3 * s] = w;
}

static void OZ_FN(oz_rlift_inv_)(OZ_INT* p, ptrdiff_t s)
{
  OZ_INT x = p[0], y = p[s], z = p[2 * s], w = p[3 * s];
  w = OZ_ADD(w, z);
  z = OZ_ADD(z, y); w = OZ_ADD(w, z);
  y = OZ_ADD(y, x); z = OZ_ADD(z, y); w = OZ_ADD(w, z);
  p[0] = x; p[s] = y; p[2 * s] = z; p[3 * s] = w;
}

/* Separable d-dimensional transform: one lift per line, axis by axis
 * (x, y, z, w forward: encode{1..4}.c fwd_xform; reverse order inverse:
 * decode{1..4}.c inv_xform).  Lines along one axis are independent, so the
 * visiting order inside an axis pass does not matter. */
static void OZ_FN(oz_xform_)(OZ_INT* p, uint32_t dims, int inverse, int reversible)
{
  uint32_t size = 1u << (2 * dims);
  for (uint32_t step = 0; step < dims; step++) {
    uint32_t axis = inverse ? dims - 1 - step : step;
    ptrdiff_t stride = (ptrdiff_t)1 << (2 * axis);
    for (uint32_t base = 0; base < size; base++) {
      if ((base >> (2 * axis)) & 3u)
        continue; /* not the first element of a line along `axis` */
      if (reversible) {
        if (inverse) OZ_FN(oz_rlift_inv_)(p + base, stride);
        else         OZ_FN(oz_rlift_fwd_)(p + base, stride);
      } else {
        if (inverse) OZ_FN(oz_lift_inv_)(p + base, stride);
        else         OZ_FN(oz_lift_fwd_)(p + base, stride);
      }
    }
  }
}

/* Embedded bit-plane coder: encode.c:92-256.  One routine covers the four
 * reference variants -- few/many differ only in how a plane is held (64-bit
 * word vs. recount), and the *_prec variants equal the budgeted ones with a
 * budget that never binds (with_maxbits, codec.c:3-7).
 * Plane k, MSB first:  (1) the first n coefficients' bits verbatim;
 * (2) group tests: '1' if a one remains at index >= n, then scan bits up to
 * and including that one (the final coefficient's one is implicit);
 * '0' ends the plane.  Every emitted bit costs one unit of budget. */
static uint32_t OZ_FN(oz_code_planes_)(oz_bits* s, uint32_t maxbits, uint32_t maxprec,
                                       const OZ_UINT* u, uint32_t size)
{
  uint32_t kmin = OZ_INTPREC > maxprec ? OZ_INTPREC - maxprec : 0;
  uint32_t bits = maxbits;
  uint32_t n = 0;
  uint32_t k = OZ_INTPREC;
  while (bits && k-- > kmin) {
    uint32_t m = n < bits ? n : bits;
    bits -= m;
    for (uint32_t i = 0; i < m; i++)
      oz_put(s, (uint64_t)((u[i] >> k) & 1u), 1);
    for (; bits && n < size; n++) {
      int more = 0;
      for (uint32_t i = n; i < size; i++)
        if ((u[i] >> k) & 1u) { more = 1; break; }
      bits--;
      oz_put(s, (uint64_t)more, 1);
      if (!more)
        break;
      for (; bits && n < size - 1; n++) {
        uint32_t b = (uint32_t)((u[n] >> k) & 1u);
        bits--;
        oz_put(s, b, 1);
        if (b)
          break;
      }
    }
  }
  return maxbits - bits;
}

/* Decoder twin: decode.c:69-246.  Note the reference quirk kept here: after a
 * positive group test the bit at the scan's stopping index is set even when
 * the budget ran out before a one was read (decode.c:100, :156). */
static uint32_t OZ_FN(oz_decode_planes_)(oz_bits* s, uint32_t maxbits, uint32_t maxprec,
                                         OZ_UINT* u, uint32_t size)
{
  uint32_t kmin = OZ_INTPREC > maxprec ? OZ_INTPREC - maxprec : 0;
  uint32_t bits = maxbits;
  uint32_t n = 0;
  uint32_t k = OZ_INTPREC;
  for (uint32_t i = 0; i < size; i++)
    u[i] = 0;
  while (bits && k-- > kmin) {
    uint32_t m = n < bits ? n : bits;
    bits -= m;
    for (uint32_t i = 0; i < m; i++)
      if (oz_get(s, 1))
        u[i] += (OZ_UINT)1 << k;
    for (; bits && n < size; n++) {
      bits--;
      if (!oz_get(s, 1))
        break;
      for (; bits && n < size - 1; n++) {
        bits--;
        if (oz_get(s, 1))
          break;
      }
      u[n] += (OZ_UINT)1 << k;
    }
  }
  return maxbits - bits;
}

/* negabinary maps: encode.c:76-79, decode.c:52-56 */
static OZ_UINT OZ_FN(oz_to_nb_)(OZ_INT x) { return ((OZ_UINT)x + OZ_NBMASK) ^ OZ_NBMASK; }
static OZ_INT OZ_FN(oz_from_nb_)(OZ_UINT x) { return (OZ_INT)((x ^ OZ_NBMASK) - OZ_NBMASK); }

/* Integer block: encode.c:260-280 (lossy) and revencode.c:54-76 (reversible). */
static uint32_t OZ_FN(oz_encode_iblock_)(oz_bits* s, uint32_t dims, uint32_t minbits, uint32_t maxbits,
                                         uint32_t maxprec, OZ_INT* q, int reversible)
{
  uint32_t size = 1u << (2 * dims);
  const unsigned char* perm = oz_perm_table(dims);
  OZ_UINT u[256];
  uint32_t bits = 0;
  OZ_FN(oz_xform_)(q, dims, 0, reversible);
  for (uint32_t i = 0; i < size; i++)
    u[i] = OZ_FN(oz_to_nb_)(q[perm[i]]);
  if (reversible) {
    /* precision = intprec - ctz(OR of all coefficients), in [1, maxprec]
     * (revencode.c:34-50, :64-67) */
    OZ_UINT all = 0;
    uint32_t prec = 0;
    for (uint32_t i = 0; i < size; i++)
      all |= u[i];
    if (all) {
      uint32_t tz = 0;
      while (!((all >> tz) & 1u))
        tz++;
      prec = OZ_INTPREC - tz;
    }
    if (prec > maxprec) prec = maxprec;
    if (prec < 1) prec = 1;
    oz_put(s, prec - 1, OZ_PBITS);
    bits = OZ_PBITS;
    maxprec = prec;
  }
  bits += OZ_FN(oz_code_planes_)(s, maxbits - bits, maxprec, u, size);
  if (bits < minbits) {
    oz_pad(s, minbits - bits);
    bits = minbits;
  }
  return bits;
}

static uint32_t OZ_FN(oz_decode_iblock_)(oz_bits* s, uint32_t dims, uint32_t minbits, uint32_t maxbits,
                                         uint32_t maxprec, OZ_INT* q, int reversible)
{
  uint32_t size = 1u << (2 * dims);
  const unsigned char* perm = oz_perm_table(dims);
  OZ_UINT u[256];
  uint32_t bits = 0;
  if (reversible) {
    maxprec = (uint32_t)oz_get(s, OZ_PBITS) + 1; /* revdecode.c:36-40 */
    bits = OZ_PBITS;
  }
  bits += OZ_FN(oz_decode_planes_)(s, maxbits - bits, maxprec, u, size);
  if (bits < minbits) {
    oz_skip(s, minbits - bits);
    bits = minbits;
  }
  for (uint32_t i = 0; i < size; i++)
    q[perm[i]] = OZ_FN(oz_from_nb_)(u[i]);
  OZ_FN(oz_xform_)(q, dims, 1, reversible);
  return bits;
}

/* precision(): codecf.c:6-14 (default build: no tight error) */
static uint32_t OZ_FN(oz_precision_)(int emax, uint32_t maxprec, int minexp, uint32_t dims)
{
  int p = emax - minexp + 2 * (int)dims + 2;
  if (p < 0) p = 0;
  return (uint32_t)p < maxprec ? (uint32_t)p : maxprec;
}

/* Lossy float block: encodef.c:63-90. */
static uint32_t OZ_FN(oz_encode_block_)(oz_bits* s, const oz_params* zp, uint32_t dims, const OZ_REAL* v)
{
  uint32_t size = 1u << (2 * dims);
  OZ_INT q[256];
  if (zp->minexp < OZ_MIN_EXP) {
    /* reversible float block: revencodef.c:45-80 */
    uint32_t bits = 0;
    int emax = OZ_FN(oz_emax_)(v, size);
    OZ_REAL back[256];
    if (emax != -OZ_EBIAS) {
      OZ_FN(oz_cast_fwd_)(q, v, size, emax);
      OZ_FN(oz_cast_inv_)(q, back, size, emax);
    } else {
      for (uint32_t i = 0; i < size; i++) { q[i] = 0; back[i] = 0; }
    }
    if (!memcmp(back, v, size * sizeof(OZ_REAL))) {
      uint32_t e = (uint32_t)(emax + OZ_EBIAS);
      if (!e) {
        oz_put(s, 0, 1);
        return 1;
      }
      oz_put(s, 1, 2);
      oz_put(s, e, OZ_EBITS);
      bits = 2 + OZ_EBITS;
    } else {
      /* sign-magnitude bit patterns as two's complement: revencodef.c:30-41 */
      memcpy(q, v, size * sizeof(OZ_INT));
      for (uint32_t i = 0; i < size; i++)
        if (q[i] < 0)
          q[i] = (OZ_INT)((OZ_UINT)q[i] ^ OZ_TCMASK);
      oz_put(s, 3, 2);
      bits = 2;
    }
    return bits + OZ_FN(oz_encode_iblock_)(s, dims, zp->minbits - (bits < zp->minbits ? bits : zp->minbits),
                                           zp->maxbits - bits, zp->maxprec, q, 1);
  }
  else {
    uint32_t bits = 1;
    int emax = OZ_FN(oz_emax_)(v, size);
    uint32_t maxprec = OZ_FN(oz_precision_)(emax, zp->maxprec, zp->minexp, dims);
    uint32_t e = maxprec ? (uint32_t)(emax + OZ_EBIAS) : 0;
    if (e) {
      bits += OZ_EBITS;
      oz_put(s, 2 * (uint64_t)e + 1, bits);
      OZ_FN(oz_cast_fwd_)(q, v, size, emax);
      bits += OZ_FN(oz_encode_iblock_)(s, dims, zp->minbits - (bits < zp->minbits ? bits : zp->minbits),
                                       zp->maxbits - bits, maxprec, q, 0);
    } else {
      oz_put(s, 0, 1);
      if (zp->minbits > bits) {
        oz_pad(s, zp->minbits - bits);
        bits = zp->minbits;
      }
    }
    return bits;
  }
}

/* Float block decode: decodef.c:7-36 and revdecodef.c:22-59. */
static uint32_t OZ_FN(oz_decode_block_)(oz_bits* s, const oz_params* zp, uint32_t dims, OZ_REAL* v)
{
  uint32_t size = 1u << (2 * dims);
  OZ_INT q[256];
  if (zp->minexp < OZ_MIN_EXP) {
    uint32_t bits = 1;
    if (!oz_get(s, 1)) {
      for (uint32_t i = 0; i < size; i++) v[i] = 0;
      if (zp->minbits > bits) { oz_skip(s, zp->minbits - bits); bits = zp->minbits; }
      return bits;
    }
    bits++;
    if (oz_get(s, 1)) {
      bits += OZ_FN(oz_decode_iblock_)(s, dims, zp->minbits - (bits < zp->minbits ? bits : zp->minbits),
                                       zp->maxbits - bits, zp->maxprec, q, 1);
      for (uint32_t i = 0; i < size; i++)
        if (q[i] < 0)
          q[i] = (OZ_INT)((OZ_UINT)q[i] ^ OZ_TCMASK);
      memcpy(v, q, size * sizeof(OZ_REAL));
    } else {
      int emax;
      bits += OZ_EBITS;
      emax = (int)oz_get(s, OZ_EBITS) - OZ_EBIAS;
      bits += OZ_FN(oz_decode_iblock_)(s, dims, zp->minbits - (bits < zp->minbits ? bits : zp->minbits),
                                       zp->maxbits - bits, zp->maxprec, q, 1);
      if (emax != -OZ_EBIAS)
        OZ_FN(oz_cast_inv_)(q, v, size, emax);
      else
        for (uint32_t i = 0; i < size; i++) v[i] = 0;
    }
    return bits;
  }
  else {
    uint32_t bits = 1;
    if (oz_get(s, 1)) {
      int emax;
      uint32_t maxprec;
      bits += OZ_EBITS;
      emax = (int)oz_get(s, OZ_EBITS) - OZ_EBIAS;
      maxprec = OZ_FN(oz_precision_)(emax, zp->maxprec, zp->minexp, dims);
      bits += OZ_FN(oz_decode_iblock_)(s, dims, zp->minbits - (bits < zp->minbits ? bits : zp->minbits),
                                       zp->maxbits - bits, maxprec, q, 0);
      OZ_FN(oz_cast_inv_)(q, v, size, emax);
    } else {
      for (uint32_t i = 0; i < size; i++) v[i] = 0;
      if (zp->minbits > bits) { oz_skip(s, zp->minbits - bits); bits = zp->minbits; }
    }
    return bits;
  }
}

/* Pad a partial line of n <= 4 valid values: encode.c:9-27. */
static void OZ_FN(oz_pad_line_)(OZ_REAL* p, size_t n, ptrdiff_t s)
{
  switch (n) {
    case 0: p[0 * s] = 0;        /* fall through */
    case 1: p[1 * s] = p[0 * s]; /* fall through */
    case 2: p[2 * s] = p[1 * s]; /* fall through */
    case 3: p[3 * s] = p[0 * s]; /* fall through */
    default: break;
  }
}

/* Gather a (possibly partial) block at origin `o` with extents cnt[] <= 4:
 * encode3.c:5-31, encode4.c:5-34 (and 1D/2D twins).  Partial blocks are padded
 * axis by axis: x for every loaded line, then y, then z, then w. */
static void OZ_FN(oz_gather_)(OZ_REAL* blk, const OZ_REAL* o, uint32_t dims,
                              const size_t cnt[4], const ptrdiff_t st[4])
{
  uint32_t size = 1u << (2 * dims);
  for (uint32_t i = 0; i < size; i++) {
    size_t c[4] = {i & 3u, (i >> 2) & 3u, (i >> 4) & 3u, (i >> 6) & 3u};
    int inside = 1;
    ptrdiff_t off = 0;
    for (uint32_t a = 0; a < dims; a++) {
      if (c[a] >= cnt[a]) inside = 0;
      off += (ptrdiff_t)c[a] * st[a];
    }
    if (inside)
      blk[i] = o[off];
  }
  for (uint32_t a = 0; a < dims; a++) {
    if (cnt[a] >= 4)
      continue;
    ptrdiff_t stride = (ptrdiff_t)1 << (2 * a);
    for (uint32_t base = 0; base < size; base++) {
      if ((base >> (2 * a)) & 3u)
        continue;
      /* pad only lines whose higher-axis coordinates are inside the data;
       * lower axes are already complete after their own pass */
      int ok = 1;
      for (uint32_t b = a + 1; b < dims; b++)
        if (((base >> (2 * b)) & 3u) >= cnt[b]) ok = 0;
      if (ok)
        OZ_FN(oz_pad_line_)(blk + base, cnt[a], stride);
    }
  }
}

/* Scatter the valid part of a decoded block: decode3.c:5-23, decode4.c:5-25. */
static void OZ_FN(oz_scatter_)(const OZ_REAL* blk, OZ_REAL* o, uint32_t dims,
                               const size_t cnt[4], const ptrdiff_t st[4])
{
  uint32_t size = 1u << (2 * dims);
  for (uint32_t i = 0; i < size; i++) {
    size_t c[4] = {i & 3u, (i >> 2) & 3u, (i >> 4) & 3u, (i >> 6) & 3u};
    int inside = 1;
    ptrdiff_t off = 0;
    for (uint32_t a = 0; a < dims; a++) {
      if (c[a] >= cnt[a]) inside = 0;
      off += (ptrdiff_t)c[a] * st[a];
    }
    if (inside)
      o[off] = blk[i];
  }
}

/* Raster traversal of the blocks of a chunk box, x fastest:
 * compress.c:67-153 / decompress.c:66-140.  A block is partial when the FIELD
 * (not the chunk) ends less than 4 values past its origin. */
static uint64_t OZ_FN(oz_run_)(const oz_job* j, void* data, oz_bits* s, int decode)
{
  uint32_t dims = oz_dims(j);
  ptrdiff_t st[4];
  size_t bcount[4] = {1, 1, 1, 1};
  OZ_REAL blk[256];
  oz_strides(j, st);
  for (uint32_t a = 0; a < dims; a++)
    bcount[a] = (j->e[a] > j->f[a]) ? (j->e[a] - j->f[a] + 3) / 4 : 0;
  for (size_t bw = 0; bw < bcount[3]; bw++)
    for (size_t bz = 0; bz < bcount[2]; bz++)
      for (size_t by = 0; by < bcount[1]; by++)
        for (size_t bx = 0; bx < bcount[0]; bx++) {
          size_t b[4] = {bx, by, bz, bw};
          size_t cnt[4] = {4, 4, 4, 4};
          ptrdiff_t off = 0;
          for (uint32_t a = 0; a < dims; a++) {
            size_t x = j->f[a] + 4 * b[a];
            size_t left = j->n[a] - x;
            cnt[a] = left < 4 ? left : 4;
            off += (ptrdiff_t)x * st[a];
          }
          if (decode) {
            OZ_FN(oz_decode_block_)(s, &j->p, dims, blk);
            OZ_FN(oz_scatter_)(blk, (OZ_REAL*)data + off, dims, cnt, st);
          } else {
            OZ_FN(oz_gather_)(blk, (const OZ_REAL*)data + off, dims, cnt, st);
            OZ_FN(oz_encode_block_)(s, &j->p, dims, blk);
          }
        }
  return s->pos;
}

#undef OZ_ADD
#undef OZ_SUB
#undef OZ_SHL1
#undef OZ_INTPREC
#undef OZ_EBIAS
#undef OZ_FN
