/*
 * zfp host library (libzfp.so) for the MI355X framework.
 *
 * Implements the zfp C API of SEP-software/zfp-par (reference src/zfp.c) on
 * the host: fields, streams, mode parameters, size bounds, headers, chunk
 * boxes and the chunk partitioner.  zfp_compress/zfp_decompress (and their
 * _chunk forms) hand the block traversal and codec to the GPU through the
 * C-ABI of include/zfp_hip.h; there is no CPU codec in this library.
 * Each function names the reference lines whose behaviour it reproduces.
 */
#include <limits.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "zfp.h"
#include "zfp_hip.h"
#include "zfp_internal.h"

#define ZMIN(a, b) ((a) < (b) ? (a) : (b))
#define ZMAX(a, b) ((a) > (b) ? (a) : (b))

/* public data (zfp.c:13-15) */
const uint zfp_codec_version = ZFP_CODEC;
const uint zfp_library_version = ZFP_VERSION;
const char* const zfp_version_string = "zfp version " ZFP_VERSION_STRING " (December 15, 2023)";

/* ------------------------------------------------------------------------ */
/* fields (zfp.c:160-569)                                                   */

size_t zfp_type_size(zfp_type type)
{
  switch (type) {
    case zfp_type_int32: return sizeof(int32);
    case zfp_type_int64: return sizeof(int64);
    case zfp_type_float: return sizeof(float);
    case zfp_type_double: return sizeof(double);
    default: return 0;
  }
}

zfp_field* zfp_field_alloc(void)
{
  zfp_field* f = (zfp_field*)calloc(1, sizeof(zfp_field));
  if (f)
    f->type = zfp_type_none;
  return f;
}

static zfp_field* field_make(void* p, zfp_type t, size_t nx, size_t ny, size_t nz, size_t nw)
{
  zfp_field* f = zfp_field_alloc();
  if (f) {
    f->type = t;
    f->nx = nx;
    f->ny = ny;
    f->nz = nz;
    f->nw = nw;
    f->data = p;
  }
  return f;
}

zfp_field* zfp_field_1d(void* p, zfp_type t, size_t nx) { return field_make(p, t, nx, 0, 0, 0); }
zfp_field* zfp_field_2d(void* p, zfp_type t, size_t nx, size_t ny) { return field_make(p, t, nx, ny, 0, 0); }
zfp_field* zfp_field_3d(void* p, zfp_type t, size_t nx, size_t ny, size_t nz) { return field_make(p, t, nx, ny, nz, 0); }
zfp_field* zfp_field_4d(void* p, zfp_type t, size_t nx, size_t ny, size_t nz, size_t nw)
{
  return field_make(p, t, nx, ny, nz, nw);
}

void zfp_field_free(zfp_field* field) { free(field); }
void* zfp_field_pointer(const zfp_field* field) { return field->data; }
zfp_type zfp_field_type(const zfp_field* field) { return field->type; }
uint zfp_field_precision(const zfp_field* field) { return (uint)(CHAR_BIT * zfp_type_size(field->type)); }

uint zfp_field_dimensionality(const zfp_field* field)
{
  if (!field->nx) return 0;
  if (!field->ny) return 1;
  if (!field->nz) return 2;
  if (!field->nw) return 3;
  return 4;
}

/* strides with zero entries resolved to the contiguous layout (zfp.c:347-366) */
static void field_strides(const zfp_field* f, ptrdiff_t s[4])
{
  s[0] = f->sx ? f->sx : 1;
  s[1] = f->sy ? f->sy : (ptrdiff_t)f->nx;
  s[2] = f->sz ? f->sz : (ptrdiff_t)(f->nx * f->ny);
  s[3] = f->sw ? f->sw : (ptrdiff_t)(f->nx * f->ny * f->nz);
}

/* lowest/highest element offsets of the field (zfp.c:19-40) */
static size_t field_span(const zfp_field* f, ptrdiff_t* lo, ptrdiff_t* hi)
{
  ptrdiff_t s[4];
  size_t n[4] = {f->nx, f->ny, f->nz, f->nw};
  ptrdiff_t a = 0, b = 0;
  field_strides(f, s);
  for (int i = 0; i < 4; i++) {
    ptrdiff_t d = n[i] ? s[i] * (ptrdiff_t)(n[i] - 1) : 0;
    a += ZMIN(d, 0);
    b += ZMAX(d, 0);
  }
  if (lo) *lo = a;
  if (hi) *hi = b;
  return (size_t)(b - a + 1);
}

void* zfp_field_begin(const zfp_field* field)
{
  ptrdiff_t lo;
  if (!field->data)
    return NULL;
  field_span(field, &lo, NULL);
  return (uchar*)field->data + lo * (ptrdiff_t)zfp_type_size(field->type);
}

size_t zfp_field_size(const zfp_field* field, size_t* size)
{
  uint d = zfp_field_dimensionality(field);
  if (size) {
    if (d >= 4) size[3] = field->nw;
    if (d >= 3) size[2] = field->nz;
    if (d >= 2) size[1] = field->ny;
    if (d >= 1) size[0] = field->nx;
  }
  return ZMAX(field->nx, 1u) * ZMAX(field->ny, 1u) * ZMAX(field->nz, 1u) * ZMAX(field->nw, 1u);
}

size_t zfp_field_size_bytes(const zfp_field* field) { return field_span(field, NULL, NULL) * zfp_type_size(field->type); }

size_t zfp_field_blocks(const zfp_field* field)
{
  size_t b[4] = {(field->nx + 3) / 4, (field->ny + 3) / 4, (field->nz + 3) / 4, (field->nw + 3) / 4};
  uint d = zfp_field_dimensionality(field);
  size_t n = d ? 1 : 0;
  for (uint i = 0; i < d; i++)
    n *= b[i];
  return n;
}

zfp_bool zfp_field_stride(const zfp_field* field, ptrdiff_t* stride)
{
  if (stride) {
    ptrdiff_t s[4];
    uint d = zfp_field_dimensionality(field);
    field_strides(field, s);
    for (uint i = 0; i < d; i++)
      stride[i] = s[i];
  }
  return field->sx || field->sy || field->sz || field->sw;
}

zfp_bool zfp_field_is_contiguous(const zfp_field* field)
{
  return field_span(field, NULL, NULL) == zfp_field_size(field, NULL);
}

/* 52-bit metadata: type-1 (2 bits), dims-1 (2 bits), then sizes-1 packed with
 * 48/24/16/12 bits per axis, x in the low field (zfp.c:374-431) */
uint64 zfp_field_metadata(const zfp_field* field)
{
  uint d = zfp_field_dimensionality(field);
  size_t n[4] = {field->nx, field->ny, field->nz, field->nw};
  uint64 meta = 0;
  if (d >= 1 && d <= 4) {
    uint width = 48 / d;
    for (int i = (int)d - 1; i >= 0; i--) {
      uint64 v = (uint64)(n[i] - 1);
      if (v >> width)
        return ZFP_META_NULL;
      meta = (meta << width) + v;
    }
  }
  meta = (meta << 2) + (d - 1);
  meta = (meta << 2) + (uint64)(field->type - 1);
  return meta;
}

void zfp_field_set_pointer(zfp_field* field, void* p) { field->data = p; }

zfp_type zfp_field_set_type(zfp_field* field, zfp_type type)
{
  switch (type) {
    case zfp_type_int32:
    case zfp_type_int64:
    case zfp_type_float:
    case zfp_type_double:
      field->type = type;
      return type;
    default:
      return zfp_type_none;
  }
}

void zfp_field_set_size_1d(zfp_field* f, size_t nx) { f->nx = nx; f->ny = f->nz = f->nw = 0; }
void zfp_field_set_size_2d(zfp_field* f, size_t nx, size_t ny) { f->nx = nx; f->ny = ny; f->nz = f->nw = 0; }
void zfp_field_set_size_3d(zfp_field* f, size_t nx, size_t ny, size_t nz) { f->nx = nx; f->ny = ny; f->nz = nz; f->nw = 0; }
void zfp_field_set_size_4d(zfp_field* f, size_t nx, size_t ny, size_t nz, size_t nw)
{
  f->nx = nx; f->ny = ny; f->nz = nz; f->nw = nw;
}
void zfp_field_set_stride_1d(zfp_field* f, ptrdiff_t sx) { f->sx = sx; f->sy = f->sz = f->sw = 0; }
void zfp_field_set_stride_2d(zfp_field* f, ptrdiff_t sx, ptrdiff_t sy) { f->sx = sx; f->sy = sy; f->sz = f->sw = 0; }
void zfp_field_set_stride_3d(zfp_field* f, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz)
{
  f->sx = sx; f->sy = sy; f->sz = sz; f->sw = 0;
}
void zfp_field_set_stride_4d(zfp_field* f, ptrdiff_t sx, ptrdiff_t sy, ptrdiff_t sz, ptrdiff_t sw)
{
  f->sx = sx; f->sy = sy; f->sz = sz; f->sw = sw;
}

/* inverse of zfp_field_metadata; resets strides to contiguous (zfp.c:518-569);
 * 1D sizes are limited to 32 bits like the reference */
zfp_bool zfp_field_set_metadata(zfp_field* field, uint64 meta)
{
  if (meta >> ZFP_META_BITS)
    return zfp_false;
  field->type = (zfp_type)((meta & 3u) + 1);
  meta >>= 2;
  uint d = (uint)(meta & 3u) + 1;
  meta >>= 2;
  size_t n[4] = {0, 0, 0, 0};
  if (d == 1) {
    n[0] = (size_t)(meta & UINT64C(0xffffffff)) + 1;
  } else {
    uint width = 48 / d;
    uint64 mask = ((uint64)1 << width) - 1;
    for (uint i = 0; i < d; i++) {
      n[i] = (size_t)(meta & mask) + 1;
      meta >>= width;
    }
  }
  field->nx = n[0];
  field->ny = n[1];
  field->nz = n[2];
  field->nw = n[3];
  field->sx = field->sy = field->sz = field->sw = 0;
  return zfp_true;
}

/* ------------------------------------------------------------------------ */
/* compressed stream parameters (zfp.c:881-1309)                            */

/* per-zfp_stream side state: HIP device and the block index of the last
 * variable-rate stream compressed with it (see zfp.h additions) */
typedef struct ext_entry {
  const zfp_stream* key;
  zfp_hip_index* index;
  int owns;
  struct ext_entry* next;
} ext_entry;

static ext_entry* ext_head = NULL;
static pthread_mutex_t ext_lock = PTHREAD_MUTEX_INITIALIZER;

static ext_entry* ext_find(const zfp_stream* zfp, int create)
{
  ext_entry* e;
  pthread_mutex_lock(&ext_lock);
  for (e = ext_head; e; e = e->next)
    if (e->key == zfp)
      break;
  if (!e && create) {
    e = (ext_entry*)calloc(1, sizeof(ext_entry));
    if (e) {
      e->key = zfp;
      e->next = ext_head;
      ext_head = e;
    }
  }
  pthread_mutex_unlock(&ext_lock);
  return e;
}

static void ext_drop(const zfp_stream* zfp)
{
  ext_entry** pp;
  ext_entry* e = NULL;
  pthread_mutex_lock(&ext_lock);
  for (pp = &ext_head; *pp; pp = &(*pp)->next)
    if ((*pp)->key == zfp) {
      e = *pp;
      *pp = e->next;
      break;
    }
  pthread_mutex_unlock(&ext_lock);
  if (e) {
    if (e->owns && e->index)
      zfp_hip_index_free(e->index);
    free(e);
  }
}

zfp_stream* zfp_stream_open(bitstream* stream)
{
  zfp_stream* zfp = (zfp_stream*)malloc(sizeof(zfp_stream));
  if (zfp) {
    zfp->stream = stream;
    zfp->minbits = ZFP_MIN_BITS;
    zfp->maxbits = ZFP_MAX_BITS;
    zfp->maxprec = ZFP_MAX_PREC;
    zfp->minexp = ZFP_MIN_EXP;
    zfp->exec.policy = zfp_exec_serial;
    zfp->exec.params = NULL;
  }
  return zfp;
}

void zfp_stream_close(zfp_stream* zfp)
{
  ext_drop(zfp);
  free(zfp->exec.params);
  free(zfp);
}

bitstream* zfp_stream_bit_stream(const zfp_stream* zfp) { return zfp->stream; }
void zfp_stream_set_bit_stream(zfp_stream* zfp, bitstream* bs) { zfp->stream = bs; }

/* mode classification (zfp.c:916-958) */
zfp_mode zfp_stream_compression_mode(const zfp_stream* zfp)
{
  if (zfp->minbits > zfp->maxbits || !(0 < zfp->maxprec && zfp->maxprec <= 64))
    return zfp_mode_null;
  if (zfp->minbits == ZFP_MIN_BITS && zfp->maxbits == ZFP_MAX_BITS && zfp->maxprec == ZFP_MAX_PREC &&
      zfp->minexp == ZFP_MIN_EXP)
    return zfp_mode_expert;
  if (zfp->minbits == zfp->maxbits && 1 <= zfp->maxbits && zfp->maxbits <= ZFP_MAX_BITS &&
      zfp->maxprec >= ZFP_MAX_PREC && zfp->minexp == ZFP_MIN_EXP)
    return zfp_mode_fixed_rate;
  if (zfp->minbits <= ZFP_MIN_BITS && zfp->maxbits >= ZFP_MAX_BITS && zfp->maxprec >= 1 &&
      zfp->minexp == ZFP_MIN_EXP)
    return zfp_mode_fixed_precision;
  if (zfp->minbits <= ZFP_MIN_BITS && zfp->maxbits >= ZFP_MAX_BITS && zfp->maxprec >= ZFP_MAX_PREC &&
      zfp->minexp >= ZFP_MIN_EXP)
    return zfp_mode_fixed_accuracy;
  if (zfp->minbits <= ZFP_MIN_BITS && zfp->maxbits >= ZFP_MAX_BITS && zfp->maxprec >= ZFP_MAX_PREC &&
      zfp->minexp < ZFP_MIN_EXP)
    return zfp_mode_reversible;
  return zfp_mode_expert;
}

double zfp_stream_rate(const zfp_stream* zfp, uint dims)
{
  return zfp_stream_compression_mode(zfp) == zfp_mode_fixed_rate ? (double)zfp->maxbits / (1u << (2 * dims)) : 0.0;
}

uint zfp_stream_precision(const zfp_stream* zfp)
{
  return zfp_stream_compression_mode(zfp) == zfp_mode_fixed_precision ? zfp->maxprec : 0;
}

double zfp_stream_accuracy(const zfp_stream* zfp)
{
  return zfp_stream_compression_mode(zfp) == zfp_mode_fixed_accuracy ? ldexp(1.0, zfp->minexp) : 0.0;
}

/* 12-bit short codes for the common modes, else a 64-bit long code with the
 * four parameters (zfp.c:983-1045) */
uint64 zfp_stream_mode(const zfp_stream* zfp)
{
  switch (zfp_stream_compression_mode(zfp)) {
    case zfp_mode_fixed_rate:
      if (zfp->maxbits <= 2048)
        return zfp->maxbits - 1;
      break;
    case zfp_mode_fixed_precision:
      if (zfp->maxprec <= 128)
        return (zfp->maxprec - 1) + 2048;
      break;
    case zfp_mode_fixed_accuracy:
      if (zfp->minexp <= 843)
        return (uint64)(zfp->minexp - ZFP_MIN_EXP) + 2048 + 128 + 1;
      break;
    case zfp_mode_reversible:
      return 2048 + 128;
    default:
      break;
  }
  {
    uint64 minbits = ZMAX(1, ZMIN(zfp->minbits, 0x8000u)) - 1;
    uint64 maxbits = ZMAX(1, ZMIN(zfp->maxbits, 0x8000u)) - 1;
    uint64 maxprec = ZMAX(1, ZMIN(zfp->maxprec, 0x0080u)) - 1;
    uint64 minexp = (uint64)ZMAX(0, ZMIN(zfp->minexp + 16495, 0x7fff));
    uint64 mode = minexp;
    mode = (mode << 7) + maxprec;
    mode = (mode << 15) + maxbits;
    mode = (mode << 15) + minbits;
    mode = (mode << 12) + 0xfffu;
    return mode;
  }
}

void zfp_stream_params(const zfp_stream* zfp, uint* minbits, uint* maxbits, uint* maxprec, int* minexp)
{
  if (minbits) *minbits = zfp->minbits;
  if (maxbits) *maxbits = zfp->maxbits;
  if (maxprec) *maxprec = zfp->maxprec;
  if (minexp) *minexp = zfp->minexp;
}

size_t zfp_stream_compressed_size(const zfp_stream* zfp) { return stream_size(zfp->stream); }

/* per-block bit bound used by the size estimates (zfp.c:1091-1110) */
static uint block_bound_bits(const zfp_stream* zfp, const zfp_field* field, uint dims)
{
  int rev = zfp->minexp < ZFP_MIN_EXP;
  uint values = 1u << (2 * dims);
  uint bits;
  switch (field->type) {
    case zfp_type_int32: bits = rev ? 5 : 0; break;
    case zfp_type_int64: bits = rev ? 6 : 0; break;
    case zfp_type_float: bits = rev ? 1 + 1 + 8 + 5 : 1 + 8; break;
    case zfp_type_double: bits = rev ? 1 + 1 + 11 + 6 : 1 + 11; break;
    default: return 0;
  }
  bits += values - 1 + values * ZMIN(zfp->maxprec, zfp_field_precision(field));
  bits = ZMIN(bits, zfp->maxbits);
  bits = ZMAX(bits, zfp->minbits);
  return bits;
}

/* bound for the blocks of a chunk box; like the reference (zfp.c:1065-1112)
 * it reserves no header bits -- callers that write a header must add
 * ZFP_HEADER_MAX_BITS (the zfpy layer here does) */
size_t zfp_stream_maximum_size_chunk(const zfp_stream* zfp, const zfp_field* field, const zfp_chunk* chunk)
{
  uint dims = zfp_field_dimensionality(field);
  size_t f[4] = {chunk->fx, chunk->fy, chunk->fz, chunk->fw};
  size_t e[4] = {chunk->ex, chunk->ey, chunk->ez, chunk->ew};
  size_t blocks = 1;
  uint bits;
  if (!dims)
    return 0;
  for (uint a = 0; a < dims; a++)
    blocks *= (e[a] - f[a] + 3) / 4;
  bits = block_bound_bits(zfp, field, dims);
  if (!bits)
    return 0;
  return ((blocks * bits + 63) & ~(size_t)63) / CHAR_BIT;
}

/* whole-field bound including the fork's extra slack for the blocks header
 * and OpenMP stream seams (zfp.c:1117-1150) */
size_t zfp_stream_maximum_size(const zfp_stream* zfp, const zfp_field* field)
{
  uint dims = zfp_field_dimensionality(field);
  uint bits;
  const size_t slack = ZFP_HEADER_BLOCKS_MAX_BITS + 5 * 32 + 2 * 64;
  if (!dims)
    return 0;
  bits = block_bound_bits(zfp, field, dims);
  if (!bits)
    return 0;
  return ((slack + zfp_field_blocks(field) * bits + 63) & ~(size_t)63) / CHAR_BIT;
}

size_t zfp_stream_maximum_size_blocks(const zfp_stream* zfp, const zfp_field* field, const zfp_blocks* blocks)
{
  return 64 * (size_t)blocks->nbeg + zfp_stream_maximum_size(zfp, field);
}

void zfp_stream_rewind(zfp_stream* zfp) { stream_rewind(zfp->stream); }
size_t zfp_stream_flush(zfp_stream* zfp) { return stream_flush(zfp->stream); }
size_t zfp_stream_align(zfp_stream* zfp) { return stream_align(zfp->stream); }

/* mode setters (zfp.c:1157-1292) */
void zfp_stream_set_reversible(zfp_stream* zfp)
{
  zfp->minbits = ZFP_MIN_BITS;
  zfp->maxbits = ZFP_MAX_BITS;
  zfp->maxprec = ZFP_MAX_PREC;
  zfp->minexp = ZFP_MIN_EXP - 1;
}

double zfp_stream_set_rate(zfp_stream* zfp, double rate, zfp_type type, uint dims, zfp_bool align)
{
  uint n = 1u << (2 * dims);
  uint bits = (uint)floor(n * rate + 0.5);
  if (type == zfp_type_float)
    bits = ZMAX(bits, 1 + 8u);
  else if (type == zfp_type_double)
    bits = ZMAX(bits, 1 + 11u);
  if (align)
    bits = (bits + 63u) & ~63u;
  zfp->minbits = bits;
  zfp->maxbits = bits;
  zfp->maxprec = ZFP_MAX_PREC;
  zfp->minexp = ZFP_MIN_EXP;
  return (double)bits / n;
}

uint zfp_stream_set_precision(zfp_stream* zfp, uint precision)
{
  zfp->minbits = ZFP_MIN_BITS;
  zfp->maxbits = ZFP_MAX_BITS;
  zfp->maxprec = precision ? ZMIN(precision, ZFP_MAX_PREC) : ZFP_MAX_PREC;
  zfp->minexp = ZFP_MIN_EXP;
  return zfp->maxprec;
}

double zfp_stream_set_accuracy(zfp_stream* zfp, double tolerance)
{
  int emin = ZFP_MIN_EXP;
  if (tolerance > 0) {
    frexp(tolerance, &emin); /* tolerance = x 2^emin, 0.5 <= x < 1 */
    emin--;
  }
  zfp->minbits = ZFP_MIN_BITS;
  zfp->maxbits = ZFP_MAX_BITS;
  zfp->maxprec = ZFP_MAX_PREC;
  zfp->minexp = emin;
  return tolerance > 0 ? ldexp(1.0, emin) : 0;
}

zfp_bool zfp_stream_set_params(zfp_stream* zfp, uint minbits, uint maxbits, uint maxprec, int minexp)
{
  if (minbits > maxbits || !(0 < maxprec && maxprec <= 64))
    return zfp_false;
  zfp->minbits = minbits;
  zfp->maxbits = maxbits;
  zfp->maxprec = maxprec;
  zfp->minexp = minexp;
  return zfp_true;
}

/* decode the 12- or 64-bit mode word (zfp.c:1221-1280) */
zfp_mode zfp_stream_set_mode(zfp_stream* zfp, uint64 mode)
{
  uint minbits, maxbits, maxprec;
  int minexp;
  if (mode <= ZFP_MODE_SHORT_MAX) {
    if (mode < 2048) {
      minbits = maxbits = (uint)mode + 1;
      maxprec = ZFP_MAX_PREC;
      minexp = ZFP_MIN_EXP;
    } else if (mode < 2048 + 128) {
      minbits = ZFP_MIN_BITS;
      maxbits = ZFP_MAX_BITS;
      maxprec = (uint)mode + 1 - 2048;
      minexp = ZFP_MIN_EXP;
    } else if (mode == 2048 + 128) {
      minbits = ZFP_MIN_BITS;
      maxbits = ZFP_MAX_BITS;
      maxprec = ZFP_MAX_PREC;
      minexp = ZFP_MIN_EXP - 1;
    } else {
      minbits = ZFP_MIN_BITS;
      maxbits = ZFP_MAX_BITS;
      maxprec = ZFP_MAX_PREC;
      minexp = (int)mode + ZFP_MIN_EXP - (2048 + 128 + 1);
    }
  } else {
    mode >>= 12;
    minbits = (uint)(mode & 0x7fffu) + 1;
    mode >>= 15;
    maxbits = (uint)(mode & 0x7fffu) + 1;
    mode >>= 15;
    maxprec = (uint)(mode & 0x007fu) + 1;
    mode >>= 7;
    minexp = (int)(mode & 0x7fffu) - 16495;
  }
  if (!zfp_stream_set_params(zfp, minbits, maxbits, maxprec, minexp))
    return zfp_mode_null;
  return zfp_stream_compression_mode(zfp);
}

/* ------------------------------------------------------------------------ */
/* execution policy (zfp.c:1311-1394) + MI355X                              */

zfp_exec_policy zfp_stream_execution(const zfp_stream* zfp) { return zfp->exec.policy; }

uint zfp_stream_omp_threads(const zfp_stream* zfp)
{
  return zfp->exec.policy == zfp_exec_omp ? ((zfp_exec_params_omp*)zfp->exec.params)->threads : 0u;
}

uint zfp_stream_omp_chunk_size(const zfp_stream* zfp)
{
  return zfp->exec.policy == zfp_exec_omp ? ((zfp_exec_params_omp*)zfp->exec.params)->chunk_size : 0u;
}

/* serial and omp are accepted for compatibility and run on the GPU like
 * zfp_exec_hip; cuda is not available (as in a reference build without it) */
zfp_bool zfp_stream_set_execution(zfp_stream* zfp, zfp_exec_policy policy)
{
  if (policy == zfp->exec.policy)
    return zfp_true;
  switch (policy) {
    case zfp_exec_serial:
      free(zfp->exec.params);
      zfp->exec.params = NULL;
      break;
    case zfp_exec_omp: {
      zfp_exec_params_omp* p = (zfp_exec_params_omp*)calloc(1, sizeof(zfp_exec_params_omp));
      if (!p)
        return zfp_false;
      free(zfp->exec.params);
      zfp->exec.params = p;
      break;
    }
    case zfp_exec_hip: {
      zfp_exec_params_hip* p = (zfp_exec_params_hip*)calloc(1, sizeof(zfp_exec_params_hip));
      if (!p)
        return zfp_false;
      p->device = -1;
      free(zfp->exec.params);
      zfp->exec.params = p;
      break;
    }
    default:
      return zfp_false;
  }
  zfp->exec.policy = policy;
  return zfp_true;
}

zfp_bool zfp_stream_set_omp_threads(zfp_stream* zfp, uint threads)
{
  if (!zfp_stream_set_execution(zfp, zfp_exec_omp))
    return zfp_false;
  ((zfp_exec_params_omp*)zfp->exec.params)->threads = threads;
  return zfp_true;
}

zfp_bool zfp_stream_set_omp_chunk_size(zfp_stream* zfp, uint chunk_size)
{
  if (!zfp_stream_set_execution(zfp, zfp_exec_omp))
    return zfp_false;
  ((zfp_exec_params_omp*)zfp->exec.params)->chunk_size = chunk_size;
  return zfp_true;
}

zfp_bool zfp_stream_set_hip_device(zfp_stream* zfp, int device)
{
  if (!zfp_stream_set_execution(zfp, zfp_exec_hip))
    return zfp_false;
  ((zfp_exec_params_hip*)zfp->exec.params)->device = device;
  return zfp_true;
}

zfp_hip_index* zfp_stream_hip_index(const zfp_stream* zfp)
{
  ext_entry* e = ext_find(zfp, 0);
  return e ? e->index : NULL;
}

/* attach a caller-owned index (NULL detaches) */
zfp_bool zfp_stream_set_hip_index(zfp_stream* zfp, zfp_hip_index* index)
{
  ext_entry* e = ext_find(zfp, 1);
  if (!e)
    return zfp_false;
  if (e->owns && e->index && e->index != index)
    zfp_hip_index_free(e->index);
  e->index = index;
  e->owns = 0;
  return zfp_true;
}

static int stream_device(const zfp_stream* zfp)
{
  if (zfp->exec.policy == zfp_exec_hip && zfp->exec.params)
    return ((const zfp_exec_params_hip*)zfp->exec.params)->device;
  return -1;
}

/* ------------------------------------------------------------------------ */
/* configurations (zfp.c:816-879)                                           */

zfp_config zfp_config_none(void)
{
  zfp_config c;
  memset(&c, 0, sizeof c);
  c.mode = zfp_mode_null;
  return c;
}

zfp_config zfp_config_rate(double rate, zfp_bool align)
{
  zfp_config c = zfp_config_none();
  c.mode = zfp_mode_fixed_rate;
  c.arg.rate = align ? -rate : rate;
  return c;
}

zfp_config zfp_config_precision(uint precision)
{
  zfp_config c = zfp_config_none();
  c.mode = zfp_mode_fixed_precision;
  c.arg.precision = precision;
  return c;
}

zfp_config zfp_config_accuracy(double tolerance)
{
  zfp_config c = zfp_config_none();
  c.mode = zfp_mode_fixed_accuracy;
  c.arg.tolerance = tolerance;
  return c;
}

zfp_config zfp_config_reversible(void)
{
  zfp_config c = zfp_config_none();
  c.mode = zfp_mode_reversible;
  return c;
}

zfp_config zfp_config_expert(uint minbits, uint maxbits, uint maxprec, int minexp)
{
  zfp_config c = zfp_config_none();
  c.mode = zfp_mode_expert;
  c.arg.expert.minbits = minbits;
  c.arg.expert.maxbits = maxbits;
  c.arg.expert.maxprec = maxprec;
  c.arg.expert.minexp = minexp;
  return c;
}

/* ------------------------------------------------------------------------ */
/* chunk boxes and partitioner (fork API, zfp.c:107-259, :570-814)          */

zfp_chunk* zfp_chunk_alloc(void) { return (zfp_chunk*)calloc(1, sizeof(zfp_chunk)); }
void zfp_chunk_free(zfp_chunk* chunk) { free(chunk); }

zfp_chunks* zfp_chunks_alloc(const int nchunks)
{
  zfp_chunks* c = (zfp_chunks*)malloc(sizeof(zfp_chunks));
  if (!c)
    return NULL;
  c->nchunks = (size_t)(nchunks > 0 ? nchunks : 0);
  c->chunks = (zfp_chunk**)malloc((c->nchunks ? c->nchunks : 1) * sizeof(zfp_chunk*));
  for (size_t i = 0; i < c->nchunks; i++)
    c->chunks[i] = zfp_chunk_alloc();
  return c;
}

void zfp_chunks_free(zfp_chunks* chunks)
{
  if (!chunks)
    return;
  for (size_t i = 0; i < chunks->nchunks; i++)
    free(chunks->chunks[i]);
  free(chunks->chunks);
  free(chunks);
}

zfp_blocks* zfp_blocks_alloc(void) { return (zfp_blocks*)calloc(1, sizeof(zfp_blocks)); }

void zfp_alloc_nblocks(zfp_blocks* blocks, const size_t nblocks)
{
  blocks->nbeg = (int)nblocks;
  blocks->begs = (size_t*)calloc(nblocks + 1, sizeof(size_t));
}

/* zfp.c:141-147 (exported, not declared in the reference header): a
 * partition record holding nchunks + 1 given chunk offsets */
zfp_blocks* zfp_blocks_alloc_beg(const size_t nchunks, const size_t* begs)
{
  zfp_blocks* blocks = zfp_blocks_alloc();
  if (!blocks)
    return NULL;
  zfp_alloc_nblocks(blocks, nchunks);
  if (blocks->begs && begs)
    memcpy(blocks->begs, begs, sizeof(size_t) * (nchunks + 1));
  return blocks;
}

void zfp_blocks_free(zfp_blocks* blocks)
{
  if (!blocks)
    return;
  free(blocks->begs);
  free(blocks);
}

void zfp_set_chunk_1d(zfp_chunk* c, const int fx, const int ex)
{
  c->fx = (size_t)fx;
  c->ex = (size_t)ex;
}

void zfp_set_chunk_2d(zfp_chunk* c, const int fx, const int fy, const int ex, const int ey)
{
  zfp_set_chunk_1d(c, fx, ex);
  c->fy = (size_t)fy;
  c->ey = (size_t)ey;
}

void zfp_set_chunk_3d(zfp_chunk* c, const int fx, const int fy, const int fz, const int ex, const int ey, const int ez)
{
  zfp_set_chunk_2d(c, fx, fy, ex, ey);
  c->fz = (size_t)fz;
  c->ez = (size_t)ez;
}

void zfp_set_chunk_4d(zfp_chunk* c, const int fx, const int fy, const int fz, const int fw, const int ex, const int ey,
                      const int ez, const int ew)
{
  zfp_set_chunk_3d(c, fx, fy, fz, ex, ey, ez);
  c->fw = (size_t)fw;
  c->ew = (size_t)ew;
}

/* split the ceil(n/4) blocks of an axis into nparts runs; part i takes
 * floor(left / (nparts - i)) blocks (float division, as zfp.c:796-814);
 * boundaries in elements, the last part ends at n */
int zfp_break_axis(const int n, const int nparts, int* fwind, int* ewind)
{
  int nblk = (n + 3) / 4;
  int done = 0, left = nblk;
  if (nparts <= 0)
    return 0;
  for (int i = 0; i < nparts; i++) {
    int mine = (int)((float)left / (float)(nparts - i));
    fwind[i] = done * 4;
    ewind[i] = fwind[i] + mine * 4;
    done += mine;
    left -= mine;
  }
  ewind[nparts - 1] = n;
  return 0;
}

int zfp_total_chunks(const int ndim, const zfp_blocks* blocks, int* per_axis)
{
  size_t b[4] = {blocks->bx, blocks->by, blocks->bz, blocks->bw};
  int total = 1;
  if (ndim < 1 || ndim > 4)
    return 0;
  for (int a = ndim - 1; a >= 0; a--) {
    per_axis[a] = (int)b[a];
    total *= per_axis[a];
  }
  return total;
}

/* Chunk counts per axis for `chunks_per_block` zfp blocks per chunk
 * (zfp.c:669-794).  BEST_CACHE: absorb whole axes from x upward while the
 * product stays within the budget, cut the first axis that would exceed it;
 * the chunk count along an axis is ceil(blocks / blocks-per-chunk) in float.
 * MAKE_EQUAL is ill-defined in the reference (unsorted uninitialised entries,
 * a loop that never advances); here it is the evident intent: fill the
 * smallest axes first, then split the rest as evenly as the d-th root allows.
 * chunks_per_block < 1 (a zero chunk size, UB in the reference) is clamped. */
zfp_blocks* zfp_optimal_parts_from_size(const int ndim, const int* n, const float chunks_per_block, const int method)
{
  int nblk[4] = {1, 1, 1, 1};
  int csize[4] = {1, 1, 1, 1};
  size_t ntot = 1;
  zfp_blocks* zb = zfp_blocks_alloc();
  if (!zb || ndim < 1 || ndim > 4)
    return zb;
  for (int i = 0; i < ndim; i++) {
    nblk[i] = (n[i] + 3) / 4;
    ntot *= (size_t)nblk[i];
  }
  if ((float)ntot < chunks_per_block) {
    zb->bx = 1;
    if (ndim >= 2) zb->by = 1;
    if (ndim >= 3) zb->bz = 1;
    if (ndim >= 4) zb->bw = 1;
    zfp_alloc_nblocks(zb, 1);
    return zb;
  }
  if (method == ZFP_BEST_CACHE) {
    int acc = 1;
    for (int d = 0; d < 4; d++) {
      csize[d] = nblk[d];
      if ((float)(csize[d] * acc) > chunks_per_block) {
        csize[d] = (int)(chunks_per_block / (float)acc);
        break;
      }
      acc *= csize[d];
    }
  } else if (method == ZFP_MAKE_EQUAL) {
    int order[4] = {0, 1, 2, 3};
    float left = chunks_per_block;
    int i = 0;
    for (int a = 0; a < ndim; a++)
      for (int b = a + 1; b < ndim; b++)
        if (nblk[order[b]] < nblk[order[a]]) {
          int t = order[a];
          order[a] = order[b];
          order[b] = t;
        }
    for (; i < ndim; i++) {
      float root = powf(left, 1.0f / (float)(ndim - i));
      if (root > (float)nblk[order[i]]) {
        csize[order[i]] = nblk[order[i]];
        left /= (float)nblk[order[i]];
      } else {
        break;
      }
    }
    for (int j = i; j < ndim; j++) {
      int s = (int)powf(left, 1.0f / (float)(ndim - j));
      csize[order[j]] = s < 1 ? 1 : s;
      left /= (float)csize[order[j]];
    }
  } else {
    return zb;
  }
  {
    size_t out[4] = {1, 1, 1, 1};
    int nc = 1;
    for (int d = 0; d < ndim; d++) {
      int cs = csize[d] < 1 ? 1 : csize[d];
      out[d] = (size_t)ceil((float)nblk[d] / (float)cs);
      nc *= (int)out[d];
    }
    zb->bx = out[0];
    if (ndim >= 2) zb->by = out[1];
    if (ndim >= 3) zb->bz = out[2];
    if (ndim >= 4) zb->bw = out[3];
    zfp_alloc_nblocks(zb, (size_t)nc);
  }
  return zb;
}

/* chunk boxes of a partition, x-fastest chunk order (zfp.c:604-667) */
zfp_chunks* zfp_chunks_from_blocks(const int ndim, const int* nsize, const zfp_blocks* blocks)
{
  int per[4] = {1, 1, 1, 1};
  int total = zfp_total_chunks(ndim, blocks, per);
  int* f[4] = {NULL, NULL, NULL, NULL};
  int* e[4] = {NULL, NULL, NULL, NULL};
  zfp_chunks* chunks;
  if (total <= 0)
    return zfp_chunks_alloc(0);
  for (int a = 0; a < ndim; a++) {
    f[a] = (int*)malloc(sizeof(int) * (size_t)per[a]);
    e[a] = (int*)malloc(sizeof(int) * (size_t)per[a]);
    zfp_break_axis(nsize[a], per[a], f[a], e[a]);
  }
  chunks = zfp_chunks_alloc(total);
  for (int i = 0; i < total; i++) {
    int r = i, c[4] = {0, 0, 0, 0};
    for (int a = 0; a < ndim; a++) {
      c[a] = r % per[a];
      r /= per[a];
    }
    zfp_chunk* ck = chunks->chunks[i];
    ck->fx = (size_t)f[0][c[0]];
    ck->ex = (size_t)e[0][c[0]];
    if (ndim >= 2) { ck->fy = (size_t)f[1][c[1]]; ck->ey = (size_t)e[1][c[1]]; }
    if (ndim >= 3) { ck->fz = (size_t)f[2][c[2]]; ck->ez = (size_t)e[2][c[2]]; }
    if (ndim >= 4) { ck->fw = (size_t)f[3][c[3]]; ck->ew = (size_t)e[3][c[3]]; }
  }
  for (int a = 0; a < ndim; a++) {
    free(f[a]);
    free(e[a]);
  }
  return chunks;
}

/* chunking from a storage budget (zfp.c:571-576; 2^ndim as in the reference) */
zfp_blocks* zfp_break_into_blocks(const int ndim, const int* nsize, const int storage_per_block, const int elem_size,
                                  const float est_compression_rate, const int method)
{
  float approx = storage_per_block / (powf(2.f, (float)ndim) / est_compression_rate * elem_size);
  return zfp_optimal_parts_from_size(ndim, nsize, approx, method);
}

int zfp_field_to_n(const zfp_field* field, int* n)
{
  uint d = zfp_field_dimensionality(field);
  size_t sz[4] = {field->nx, field->ny, field->nz, field->nw};
  for (uint i = 0; i < d; i++)
    n[i] = (int)sz[i];
  return d ? (int)d : 1;
}

/* ------------------------------------------------------------------------ */
/* compression and decompression (zfp.c:1466-1649)                          */

static int job_from(zfp_hip_job* j, const zfp_stream* zfp, const zfp_chunk* chunk, const zfp_field* field)
{
  ptrdiff_t s[4];
  size_t n[4] = {field->nx, field->ny, field->nz, field->nw};
  size_t f[4] = {chunk->fx, chunk->fy, chunk->fz, chunk->fw};
  size_t e[4] = {chunk->ex, chunk->ey, chunk->ez, chunk->ew};
  uint d = zfp_field_dimensionality(field);
  memset(j, 0, sizeof *j);
  j->type = (int32_t)field->type;
  j->dims = (int32_t)d;
  field_strides(field, s);
  for (uint a = 0; a < 4; a++) {
    j->n[a] = a < d ? n[a] : 0;
    j->s[a] = a < d ? (int64_t)s[a] : 0;
    j->f[a] = a < d ? f[a] : 0;
    j->e[a] = a < d ? e[a] : 0;
  }
  j->minbits = zfp->minbits;
  j->maxbits = zfp->maxbits;
  j->maxprec = zfp->maxprec;
  j->minexp = zfp->minexp;
  return 1;
}

static void report(const char* what)
{
  const char* msg = zfp_hip_last_error();
  fprintf(stderr, "zfp (MI355X): %s failed: %s\n", what, msg && *msg ? msg : "unknown error");
}

static int variable_rate(const zfp_stream* zfp, const zfp_field* field)
{
  /* integer blocks carry no header in the lossy modes */
  uint hdr = field->type == zfp_type_double ? 12 : field->type == zfp_type_float ? 9 : 1;
  return !(zfp->minexp >= ZFP_MIN_EXP && zfp->minbits == zfp->maxbits && zfp->maxbits >= hdr);
}

size_t zfp_compress(zfp_stream* zfp, const zfp_field* field)
{
  zfp_chunk whole;
  whole.fx = whole.fy = whole.fz = whole.fw = 0;
  whole.ex = field->nx;
  whole.ey = field->ny;
  whole.ez = field->nz;
  whole.ew = field->nw;
  return zfp_compress_chunk(zfp, &whole, field);
}

static size_t compress_exec(zfp_stream* zfp, const zfp_chunk* chunk, const zfp_field* field, uint exec);
static size_t decompress_exec(zfp_stream* zfp, const zfp_chunk* chunk, zfp_field* field, uint exec);

size_t zfp_compress_chunk(zfp_stream* zfp, const zfp_chunk* chunk, const zfp_field* field)
{
  return compress_exec(zfp, chunk, field, (uint)zfp->exec.policy);
}

/* zfp.c:1510-1564: the reference's function-table dispatch with the execution
 * policy, strided flag, dimensionality and scalar type given by the caller
 * (zfp_compress_chunk derives them from the stream and field).  Here every
 * serial/OpenMP entry is the GPU path; `strided` selects nothing (the kernels
 * take strides either way); a type or dimensionality that disagrees with the
 * field has no table entry in this library and returns 0. */
size_t zfp_compress_call(zfp_stream* zfp, const zfp_chunk* chunk, const zfp_field* field, const uint exec,
                         const uint strided, const uint dims, const uint type)
{
  (void)strided;
  if (exec > (uint)zfp_exec_hip || dims != zfp_field_dimensionality(field) || type != (uint)field->type)
    return 0;
  return compress_exec(zfp, chunk, field, exec);
}

size_t zfp_decompress_call(zfp_stream* zfp, const zfp_chunk* chunk, zfp_field* field, const uint exec,
                           const uint strided, const uint dims, const uint type)
{
  (void)strided;
  if (exec > (uint)zfp_exec_hip || dims != zfp_field_dimensionality(field) || type != (uint)field->type)
    return 0;
  return decompress_exec(zfp, chunk, field, exec);
}

static size_t compress_exec(zfp_stream* zfp, const zfp_chunk* chunk, const zfp_field* field, uint exec)
{
  bitstream* s = zfp->stream;
  zfp_hip_job job;
  zfp_chunk whole;
  uint64 end = 0;
  zfp_hip_index* index = NULL;
  switch (field->type) {
    case zfp_type_int32:
    case zfp_type_int64:
    case zfp_type_float:
    case zfp_type_double:
      break;
    default:
      return 0;
  }
  if (exec == zfp_exec_cuda)
    return 0;
  if (exec == zfp_exec_omp) {
    /* the reference's OpenMP compressor ignores the chunk (ompcompress.c:155-210) */
    whole.fx = whole.fy = whole.fz = whole.fw = 0;
    whole.ex = field->nx;
    whole.ey = field->ny;
    whole.ez = field->nz;
    whole.ew = field->nw;
    chunk = &whole;
  }
  job_from(&job, zfp, chunk, field);
  if (variable_rate(zfp, field)) {
    ext_entry* e = ext_find(zfp, 1);
    if (e) {
      if (!e->index) {
        e->index = zfp_hip_index_create();
        e->owns = 1;
      }
      index = e->index;
    }
  }
  if (!zfp_hip_compress(&job, field->data, s->begin, (uint64)(s->end - s->begin), stream_wtell(s), s->buffer,
                        stream_device(zfp), index, &end)) {
    report("zfp_compress");
    return 0;
  }
  /* the device wrote everything through the zero-padded last word: leave the
   * stream flushed at that word boundary (what stream_flush would produce) */
  s->ptr = s->begin + (size_t)((end + 63) / 64);
  s->bits = 0;
  s->buffer = 0;
  return stream_size(s);
}

size_t zfp_decompress(zfp_stream* zfp, zfp_field* field)
{
  zfp_chunk whole;
  whole.fx = whole.fy = whole.fz = whole.fw = 0;
  whole.ex = field->nx;
  whole.ey = field->ny;
  whole.ez = field->nz;
  whole.ew = field->nw;
  return zfp_decompress_chunk(zfp, &whole, field);
}

size_t zfp_decompress_chunk(zfp_stream* zfp, const zfp_chunk* chunk, zfp_field* field)
{
  return decompress_exec(zfp, chunk, field, (uint)zfp->exec.policy);
}

static size_t decompress_exec(zfp_stream* zfp, const zfp_chunk* chunk, zfp_field* field, uint exec)
{
  bitstream* s = zfp->stream;
  zfp_hip_job job;
  uint64 end = 0;
  zfp_hip_index* index = NULL;
  switch (field->type) {
    case zfp_type_int32:
    case zfp_type_int64:
    case zfp_type_float:
    case zfp_type_double:
      break;
    default:
      return 0;
  }
  /* no OpenMP or CUDA decompressor in the reference table (zfp.c:1623-1637) */
  if (exec == zfp_exec_omp || exec == zfp_exec_cuda)
    return 0;
  job_from(&job, zfp, chunk, field);
  if (variable_rate(zfp, field)) {
    ext_entry* e = ext_find(zfp, 0);
    index = e ? e->index : NULL;
  }
  if (!zfp_hip_decompress(&job, field->data, s->begin, (uint64)(s->end - s->begin), stream_rtell(s),
                          stream_device(zfp), index, &end)) {
    report("zfp_decompress");
    return 0;
  }
  /* stream_align after the last block (zfp.c:1647) */
  s->ptr = s->begin + (size_t)((end + 63) / 64);
  s->bits = 0;
  s->buffer = 0;
  return stream_size(s);
}

/* One block of the low-level API (encode.c / decode.c templates: zfp_encode_
 * block_*, zfp_decode_block_*): the same GPU call as a chunk, on a field that
 * is the block, at the stream's bit position -- pending bits of a partly
 * written word included -- and with no flush, so consecutive blocks are packed
 * bit after bit as by the reference's serial coder.  Variable-rate blocks are
 * decoded with the index scan of that one block. */
size_t zfp_block_code(zfp_stream* zfp, zfp_type type, uint dims, void* p, const size_t* n, const ptrdiff_t* st,
                      int decode)
{
  bitstream* s = zfp->stream;
  zfp_field f;
  zfp_chunk box;
  zfp_hip_job job;
  uint64 start, end = 0;
  size_t* nn[4] = {&f.nx, &f.ny, &f.nz, &f.nw};
  ptrdiff_t* ss[4] = {&f.sx, &f.sy, &f.sz, &f.sw};
  size_t* bf[4] = {&box.fx, &box.fy, &box.fz, &box.fw};
  size_t* be[4] = {&box.ex, &box.ey, &box.ez, &box.ew};
  memset(&f, 0, sizeof f);
  f.type = type;
  f.data = p;
  for (uint a = 0; a < 4; a++) {
    *nn[a] = a < dims ? n[a] : 0;
    *ss[a] = a < dims ? st[a] : 0;
    *bf[a] = 0;
    *be[a] = a < dims ? n[a] : 0;
  }
  for (uint a = 0; a < dims; a++)
    if (n[a] < 1 || n[a] > 4)
      return 0;
  job_from(&job, zfp, &box, &f);
  if (!decode) {
    start = stream_wtell(s);
    if (!zfp_hip_compress(&job, p, s->begin, (uint64)(s->end - s->begin), start, s->buffer, stream_device(zfp), NULL,
                          &end)) {
      report("zfp_encode_block");
      return 0;
    }
    stream_wseek(s, end);
  } else if (zfp_hip_is_device_ptr(p)) {
    start = stream_rtell(s);
    if (!zfp_hip_decompress(&job, p, s->begin, (uint64)(s->end - s->begin), start, stream_device(zfp), NULL, &end)) {
      report("zfp_decode_block");
      return 0;
    }
    stream_rseek(s, end);
  } else {
    /* decoded into a contiguous block here, then copied out with the caller's
     * strides (a host field with any strides, as the reference's scatter) */
    unsigned char tmp[256 * sizeof(double)];
    const size_t es = zfp_type_size(type);
    size_t m[4] = {1, 1, 1, 1};
    ptrdiff_t cs[4] = {1, 0, 0, 0};
    for (uint a = 0; a < dims; a++)
      m[a] = n[a];
    for (uint a = 1; a < dims; a++)
      cs[a] = cs[a - 1] * (ptrdiff_t)n[a - 1];
    f.data = tmp;
    for (uint a = 0; a < 4; a++)
      *ss[a] = a < dims ? cs[a] : 0;
    job_from(&job, zfp, &box, &f);
    start = stream_rtell(s);
    if (!zfp_hip_decompress(&job, tmp, s->begin, (uint64)(s->end - s->begin), start, stream_device(zfp), NULL, &end)) {
      report("zfp_decode_block");
      return 0;
    }
    stream_rseek(s, end);
    for (size_t l = 0; l < m[3]; l++)
      for (size_t k = 0; k < m[2]; k++)
        for (size_t j = 0; j < m[1]; j++)
          for (size_t i = 0; i < m[0]; i++) {
            const ptrdiff_t o = (ptrdiff_t)i * st[0] + (dims > 1 ? (ptrdiff_t)j * st[1] : 0) +
                                (dims > 2 ? (ptrdiff_t)k * st[2] : 0) + (dims > 3 ? (ptrdiff_t)l * st[3] : 0);
            memcpy((unsigned char*)p + o * (ptrdiff_t)es, tmp + (i + m[0] * (j + m[1] * (k + m[2] * l))) * es, es);
          }
  }
  return (size_t)(end - start);
}

/* ------------------------------------------------------------------------ */
/* headers (zfp.c:1702-1840)                                                */

size_t zfp_write_header(zfp_stream* zfp, const zfp_field* field, uint mask)
{
  size_t bits = 0;
  uint64 meta = 0;
  if (mask & ZFP_HEADER_META) {
    meta = zfp_field_metadata(field);
    if (meta == ZFP_META_NULL)
      return 0;
  }
  if (mask & ZFP_HEADER_MAGIC) {
    stream_write_bits(zfp->stream, 'z', 8);
    stream_write_bits(zfp->stream, 'f', 8);
    stream_write_bits(zfp->stream, 'p', 8);
    stream_write_bits(zfp->stream, zfp_codec_version, 8);
    bits += ZFP_MAGIC_BITS;
  }
  if (mask & ZFP_HEADER_META) {
    stream_write_bits(zfp->stream, meta, ZFP_META_BITS);
    bits += ZFP_META_BITS;
  }
  if (mask & ZFP_HEADER_MODE) {
    uint64 mode = zfp_stream_mode(zfp);
    uint size = mode > ZFP_MODE_SHORT_MAX ? ZFP_MODE_LONG_BITS : ZFP_MODE_SHORT_BITS;
    stream_write_bits(zfp->stream, mode, size);
    bits += size;
  }
  return bits;
}

size_t zfp_read_header(zfp_stream* zfp, zfp_field* field, uint mask)
{
  size_t bits = 0;
  if (mask & ZFP_HEADER_MAGIC) {
    if (stream_read_bits(zfp->stream, 8) != 'z' || stream_read_bits(zfp->stream, 8) != 'f' ||
        stream_read_bits(zfp->stream, 8) != 'p' || stream_read_bits(zfp->stream, 8) != zfp_codec_version)
      return 0;
    bits += ZFP_MAGIC_BITS;
  }
  if (mask & ZFP_HEADER_META) {
    uint64 meta = stream_read_bits(zfp->stream, ZFP_META_BITS);
    if (!zfp_field_set_metadata(field, meta))
      return 0;
    bits += ZFP_META_BITS;
  }
  if (mask & ZFP_HEADER_MODE) {
    uint64 mode = stream_read_bits(zfp->stream, ZFP_MODE_SHORT_BITS);
    bits += ZFP_MODE_SHORT_BITS;
    if (mode > ZFP_MODE_SHORT_MAX) {
      uint size = ZFP_MODE_LONG_BITS - ZFP_MODE_SHORT_BITS;
      mode += stream_read_bits(zfp->stream, size) << ZFP_MODE_SHORT_BITS;
      bits += size;
    }
    if (zfp_stream_set_mode(zfp, mode) == zfp_mode_null)
      return 0;
  }
  return bits;
}

/* ------------------------------------------------------------------------ */
/* the fork's "blocks" API: chunk streams at offsets recorded in a header    */
/* (zfp.c:1651-1701 write, :1747-1797 read, :1880-2177 compress/decompress). */
/* In the reference these run one OpenMP thread per chunk; here every chunk  */
/* is one zfp_compress_chunk / zfp_decompress_chunk call on the GPU (a       */
/* variable-rate chunk without an index is found by the GPU stream scan), so */
/* `nthreads` is accepted and unused.                                        */

zfp_streams* zfp_streams_alloc(const int nstreams)
{
  zfp_streams* z = (zfp_streams*)malloc(sizeof(zfp_streams));
  if (!z)
    return NULL;
  z->nstreams = nstreams > 0 ? nstreams : 0;
  z->streams = (zfp_stream**)calloc(z->nstreams ? (size_t)z->nstreams : 1, sizeof(zfp_stream*));
  return z;
}

/* closes each sub-stream's bitstream and zfp_stream (not the shared buffer) */
void zfp_streams_free(zfp_streams* z)
{
  if (!z)
    return;
  for (int i = 0; i < z->nstreams; i++)
    if (z->streams[i]) {
      stream_close(z->streams[i]->stream);
      zfp_stream_close(z->streams[i]);
    }
  free(z->streams);
  free(z);
}

/* sub-stream i over bits [b[i], b[i+1]) of zfp_in's buffer, byte-addressed as
 * the reference does (b[i] / 8), with zfp_in's codec parameters */
zfp_streams* zfp_create_streams(const zfp_stream* zfp_in, const int nblocks, const size_t* b)
{
  zfp_streams* z = zfp_streams_alloc(nblocks);
  if (!z)
    return NULL;
  stream_rewind(zfp_in->stream);
  for (int i = 0; i < nblocks; i++) {
    bitstream* s = stream_open((uchar*)stream_data(zfp_in->stream) + b[i] / 8, b[i + 1] / 8 - b[i] / 8);
    z->streams[i] = zfp_stream_open(s);
    zfp_stream_set_params(z->streams[i], zfp_in->minbits, zfp_in->maxbits, zfp_in->maxprec, zfp_in->minexp);
    if (zfp_in->exec.policy == zfp_exec_hip)
      zfp_stream_set_hip_device(z->streams[i], stream_device(zfp_in));
  }
  return z;
}

/* Compress every chunk of `blocks` into its own sub-stream; chunk i is given
 * zfp_stream_maximum_size_chunk bytes starting at bit begs[i] (begs[0] =
 * initial_pos), flushed.  zfp.c:1914-1938. */
zfp_streams* zfp_blocks_portions(zfp_stream* stream, const zfp_field* field, const int nthreads, zfp_blocks* blocks,
                                 size_t initial_pos)
{
  int nsize[4];
  int ndims = zfp_field_to_n(field, nsize);
  zfp_chunks* chunks = zfp_chunks_from_blocks(ndims, nsize, blocks);
  zfp_streams* z;
  (void)nthreads;
  if (!chunks)
    return NULL;
  blocks->begs[0] = initial_pos;
  for (size_t i = 0; i < chunks->nchunks; i++)
    blocks->begs[i + 1] = blocks->begs[i] + CHAR_BIT * zfp_stream_maximum_size_chunk(stream, field, chunks->chunks[i]);
  z = zfp_create_streams(stream, (int)chunks->nchunks, blocks->begs);
  for (size_t i = 0; z && i < chunks->nchunks; i++) {
    zfp_compress_chunk(z->streams[i], chunks->chunks[i], field);
    stream_flush(z->streams[i]->stream);
  }
  zfp_chunks_free(chunks);
  return z;
}

/* Blocks header: magic, type (8 bits), nx..nw (32 bits each), the 64-bit mode
 * word, nbeg and bx..bw (32 bits each), nbeg+1 offsets of 64 bits; begs are
 * stored plus the header's size when begs_after_header == 1; flushed to a
 * word (the reference's 56-bit pad).  zfp.c:1651-1701. */
size_t zfp_write_blocks_header(zfp_stream* zfp, const zfp_field* field, const zfp_blocks* blocks,
                               const int begs_after_header)
{
  size_t bits = 0, use_offset = 0;
  stream_write_bits(zfp->stream, 'z', 8);
  stream_write_bits(zfp->stream, 'f', 8);
  stream_write_bits(zfp->stream, 'p', 8);
  stream_write_bits(zfp->stream, zfp_codec_version, 8);
  bits += ZFP_MAGIC_BITS;
  stream_write_bits(zfp->stream, (uint64)field->type, 8);
  stream_write_bits(zfp->stream, (uint64)field->nx, 32);
  stream_write_bits(zfp->stream, (uint64)field->ny, 32);
  stream_write_bits(zfp->stream, (uint64)field->nz, 32);
  stream_write_bits(zfp->stream, (uint64)field->nw, 32);
  bits += 136;
  stream_write_bits(zfp->stream, zfp_stream_mode(zfp), 64); /* always the long form */
  bits += 64;
  stream_write_bits(zfp->stream, (uint64)blocks->nbeg, 32);
  stream_write_bits(zfp->stream, (uint64)blocks->bx, 32);
  stream_write_bits(zfp->stream, (uint64)blocks->by, 32);
  stream_write_bits(zfp->stream, (uint64)blocks->bz, 32);
  stream_write_bits(zfp->stream, (uint64)blocks->bw, 32);
  bits += 160;
  bits += 64 * (size_t)(blocks->nbeg + 1) + 56;
  if (begs_after_header == 1)
    use_offset = bits;
  for (int i = 0; i < blocks->nbeg + 1; i++)
    stream_write_bits(zfp->stream, (uint64)(use_offset + blocks->begs[i]), 64);
  stream_flush(zfp->stream);
  return bits;
}

/* zfp.c:1747-1797: fills field type/extents and the partition (begs is
 * allocated here), leaves the stream after the 56-bit pad */
size_t zfp_read_blocks_header(zfp_stream* zfp, zfp_field* field, zfp_blocks* blocks)
{
  size_t bits = 0;
  uint64 mode;
  if (stream_read_bits(zfp->stream, 8) != 'z' || stream_read_bits(zfp->stream, 8) != 'f' ||
      stream_read_bits(zfp->stream, 8) != 'p' || stream_read_bits(zfp->stream, 8) != zfp_codec_version)
    return 0;
  bits += ZFP_MAGIC_BITS;
  field->type = (zfp_type)stream_read_bits(zfp->stream, 8);
  field->nx = (size_t)stream_read_bits(zfp->stream, 32);
  field->ny = (size_t)stream_read_bits(zfp->stream, 32);
  field->nz = (size_t)stream_read_bits(zfp->stream, 32);
  field->nw = (size_t)stream_read_bits(zfp->stream, 32);
  bits += 136;
  mode = stream_read_bits(zfp->stream, 64);
  bits += 64;
  if (zfp_stream_set_mode(zfp, mode) == zfp_mode_null)
    return 0;
  blocks->nbeg = (int)stream_read_bits(zfp->stream, 32);
  blocks->bx = (size_t)stream_read_bits(zfp->stream, 32);
  blocks->by = (size_t)stream_read_bits(zfp->stream, 32);
  blocks->bz = (size_t)stream_read_bits(zfp->stream, 32);
  blocks->bw = (size_t)stream_read_bits(zfp->stream, 32);
  bits += 160;
  free(blocks->begs);
  blocks->begs = (size_t*)malloc(sizeof(size_t) * (size_t)(blocks->nbeg + 1));
  if (!blocks->begs)
    return 0;
  for (int i = 0; i < blocks->nbeg + 1; i++)
    blocks->begs[i] = (size_t)stream_read_bits(zfp->stream, 64);
  bits += 64 * (size_t)(blocks->nbeg + 1);
  stream_rseek(zfp->stream, bits + 56);
  return bits;
}

/* zfp.c:2079-2114: partition the field, compress every chunk into a fresh
 * buffer (it replaces the stream's bit stream, as in the reference; the caller
 * owns it: stream_data(zfp_stream_bit_stream(stream))), then write the blocks
 * header at its start.  Returns the chunk sub-streams. */
zfp_streams* zfp_blocks_compress(zfp_stream* stream, const zfp_field* field, const int nthreads,
                                 const float blocks_per_chunk, const int method, const int begs_after_header)
{
  int n[4] = {0, 0, 0, 0}, per[4] = {1, 1, 1, 1};
  int ndims = zfp_field_to_n(field, n);
  zfp_blocks* zb = zfp_optimal_parts_from_size(ndims, n, blocks_per_chunk, method);
  int nchunks;
  size_t bufsize;
  void* buffer;
  bitstream* dst;
  zfp_streams* z;
  if (!zb)
    return NULL;
  nchunks = zfp_total_chunks(ndims, zb, per);
  bufsize = zfp_stream_maximum_size_blocks(stream, field, zb);
  buffer = malloc(bufsize);
  if (!buffer) {
    zfp_blocks_free(zb);
    return NULL;
  }
  dst = stream_open(buffer, bufsize);
  zfp_stream_set_bit_stream(stream, dst);
  z = zfp_blocks_portions(stream, field, nthreads, zb, ZFP_HEADER_BLOCKS_MAX_BITS + (size_t)(nchunks + 1) * 64);
  zb->begs[0] = 0;
  for (int i = 0; z && i < zb->nbeg; i++) {
    stream_flush(z->streams[i]->stream);
    zb->begs[i + 1] = zb->begs[i] + stream_wtell(z->streams[i]->stream);
  }
  zfp_write_blocks_header(stream, field, zb, begs_after_header);
  zfp_blocks_free(zb);
  return z;
}

zfp_streams* zfp_blocks_compress_multi(zfp_stream* stream, const zfp_field* field, const int nthreads,
                                       const float blocks_per_chunk, const int method)
{
  return zfp_blocks_compress(stream, field, nthreads, blocks_per_chunk, method, 0);
}

/* zfp.c:2037-2065: one stream = blocks header + the chunk streams packed after
 * it in chunk order (each chunk word-flushed); returns its size in bytes */
size_t zfp_blocks_compress_single_stream(zfp_stream* stream, const zfp_field* field, const int nthreads,
                                         const float blocks_per_chunk, const int method)
{
  zfp_streams* z = zfp_blocks_compress(stream, field, nthreads, blocks_per_chunk, method, 1);
  bitstream* dst;
  size_t offset;
  if (!z)
    return 0;
  dst = stream->stream;
  offset = stream_wtell(dst);
  for (int i = 0; i < z->nstreams; i++) {
    size_t bits = stream_wtell(z->streams[i]->stream);
    stream_rewind(z->streams[i]->stream);
    stream_copy(dst, z->streams[i]->stream, bits);
    offset += bits;
  }
  stream_wseek(dst, offset);
  zfp_streams_free(z);
  return offset / 8;
}

/* zfp.c:1942-1981, without the reference's misuse of stream_data() as a bit
 * stream (undefined behaviour there): chunks are compressed at their reserved
 * offsets from the stream's current byte, then packed after it; begs[] gets
 * the packed chunk offsets.  Returns the stream size in bytes. */
size_t zfp_blocks_compress_internal(zfp_stream* stream, const zfp_field* field, const int nthreads, zfp_blocks* blocks)
{
  size_t offset, start = stream_wtell(stream->stream);
  zfp_streams* z = zfp_blocks_portions(stream, field, nthreads, blocks, start);
  bitstream* dst = zfp_stream_bit_stream(stream);
  if (!z)
    return 0;
  stream_wseek(dst, start);
  offset = start;
  for (int i = 0; i < blocks->nbeg; i++) {
    size_t bits = stream_wtell(z->streams[i]->stream);
    blocks->begs[i + 1] = blocks->begs[i] + bits;
    stream_rewind(z->streams[i]->stream);
    stream_copy(dst, z->streams[i]->stream, bits);
    offset += bits;
  }
  zfp_streams_free(z);
  return offset / 8;
}

/* zfp.c:1984-2008: every chunk of `blocks` from sub-streams at begs[] */
size_t zfp_blocks_decompress(zfp_stream* stream, zfp_field* field, const int nthreads, const zfp_blocks* blocks)
{
  int nsize[4];
  int ndims = zfp_field_to_n(field, nsize);
  zfp_chunks* chunks = zfp_chunks_from_blocks(ndims, nsize, blocks);
  zfp_streams* z;
  size_t val;
  (void)nthreads;
  if (!chunks)
    return 0;
  z = zfp_create_streams(stream, (int)chunks->nchunks, blocks->begs);
  for (size_t i = 0; z && i < chunks->nchunks; i++)
    zfp_decompress_chunk(z->streams[i], chunks->chunks[i], field);
  zfp_streams_free(z);
  val = blocks->begs[chunks->nchunks];
  zfp_chunks_free(chunks);
  return val / 8;
}

/* zfp.c:2147-2177: re-reads the header from the start of `stream`, then every
 * chunk from its sub-stream */
size_t zfp_blocks_decompress_multi_stream(zfp_stream* stream, zfp_field* field, zfp_streams* zstreams,
                                          const int nthreads)
{
  int nsize[4];
  zfp_blocks* zb = zfp_blocks_alloc();
  zfp_chunks* chunks;
  size_t val;
  int ndims;
  (void)nthreads;
  if (!zb)
    return 0;
  stream_rewind(stream->stream);
  if (!zfp_read_blocks_header(stream, field, zb)) {
    zfp_blocks_free(zb);
    return 0;
  }
  ndims = zfp_field_to_n(field, nsize);
  chunks = zfp_chunks_from_blocks(ndims, nsize, zb);
  for (size_t i = 0; chunks && i < chunks->nchunks && (int)i < zstreams->nstreams; i++) {
    stream_rewind(zstreams->streams[i]->stream);
    zfp_decompress_chunk(zstreams->streams[i], chunks->chunks[i], field);
  }
  val = zb->begs[zb->nbeg];
  zfp_chunks_free(chunks);
  zfp_blocks_free(zb);
  return val / 8;
}

/* zfp.c:2116-2145 */
size_t zfp_blocks_decompress_single_stream(zfp_stream* stream, zfp_field* field, const int nthreads)
{
  int nsize[4];
  zfp_blocks* zb = zfp_blocks_alloc();
  zfp_chunks* chunks;
  zfp_streams* z;
  size_t loc;
  int ndims;
  if (!zb)
    return 0;
  if (!zfp_read_blocks_header(stream, field, zb)) {
    zfp_blocks_free(zb);
    return 0;
  }
  ndims = zfp_field_to_n(field, nsize);
  chunks = zfp_chunks_from_blocks(ndims, nsize, zb);
  z = zfp_create_streams(stream, (int)(chunks ? chunks->nchunks : 0), zb->begs);
  loc = z ? zfp_blocks_decompress_multi_stream(stream, field, z, nthreads) : 0;
  zfp_chunks_free(chunks);
  zfp_blocks_free(zb);
  zfp_streams_free(z);
  return loc;
}
