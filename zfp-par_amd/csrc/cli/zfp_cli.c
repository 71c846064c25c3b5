/*
 * zfp -- command-line front end over libzfp.so (MI355X), option-compatible
 * with the reference's utils/zfp.c (usage :82-136, driver :139-629):
 *
 *   -i <raw in>  -z <zfp file>  -o <raw out>  -h (header)  -q  -s (stats)
 *   -f | -d | -t <i32|i64|f32|f64>   -1 nx | -2 nx ny | -3 nx ny nz | -4 nx ny nz nw
 *   -r rate | -p precision | -a tolerance | -R | -c minbits maxbits maxprec minexp
 *   -x serial | omp[=threads[,chunk]] | cuda | hip[=device]
 *
 * Compression and decompression run on the GPU through the zfp C API; the
 * execution policy only selects the device ("serial" and "omp" are accepted
 * for script compatibility and run on the default device, as this library has
 * no CPU codec).  Output files are byte-identical to the reference's for the
 * same options (bit-exact codec, same header and word flushing).
 */
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "zfp.h"

typedef struct {
  zfp_type type;
  uint dims;
  size_t n[4];
  char mode; /* 'r' 'p' 'a' 'R' 'c' or 0 */
  double rate, tolerance;
  uint precision;
  uint minbits, maxbits, maxprec;
  int minexp;
  int header, quiet, stats;
  const char *in, *zfp, *out;
  int device; /* -1: default */
} options;

static void usage(void)
{
  static const char* text[] = {
    "Usage: zfp <options>",
    "General options:",
    "  -h : read/write array and compression parameters from/to compressed header",
    "  -q : quiet mode; suppress output",
    "  -s : print error statistics",
    "Input and output:",
    "  -i <path> : uncompressed binary input file (\"-\" for stdin)",
    "  -o <path> : decompressed binary output file (\"-\" for stdout)",
    "  -z <path> : compressed input (w/o -i) or output file (\"-\" for stdin/stdout)",
    "Array type and dimensions (needed with -i):",
    "  -f : single precision (float type)",
    "  -d : double precision (double type)",
    "  -t <i32|i64|f32|f64> : integer or floating scalar type",
    "  -1 <nx> | -2 <nx> <ny> | -3 <nx> <ny> <nz> | -4 <nx> <ny> <nz> <nw> : dimensions (x fastest)",
    "Compression parameters (needed with -i):",
    "  -R : reversible (lossless) compression",
    "  -r <rate> : fixed rate (# compressed bits per value)",
    "  -p <precision> : fixed precision (# uncompressed bits per value)",
    "  -a <tolerance> : fixed accuracy (absolute error tolerance)",
    "  -c <minbits> <maxbits> <maxprec> <minexp> : advanced usage",
    "Execution parameters:",
    "  -x hip[=device] : MI355X kernels (default)",
    "  -x serial | omp[=threads[,chunk]] | cuda : accepted for compatibility; run on the GPU",
    "Examples:",
    "  -f -3 256 256 256 -r 16 -i in.raw -z out.zfp : fixed-rate compression of 256^3 floats",
    "  -z out.zfp -f -3 256 256 256 -r 16 -o back.raw : decompression",
    NULL,
  };
  fprintf(stderr, "%s\n", zfp_version_string);
  for (int i = 0; text[i]; i++)
    fprintf(stderr, "%s\n", text[i]);
  exit(EXIT_FAILURE);
}

static void die(const char* msg)
{
  fprintf(stderr, "%s\n", msg);
  exit(EXIT_FAILURE);
}

/* consume `count` numeric arguments after option argv[*i] */
static const char* next_arg(int argc, char** argv, int* i)
{
  if (++*i >= argc)
    usage();
  return argv[*i];
}

static size_t arg_size(int argc, char** argv, int* i)
{
  size_t v;
  if (sscanf(next_arg(argc, argv, i), "%zu", &v) != 1)
    usage();
  return v;
}

static void parse(options* o, int argc, char** argv)
{
  memset(o, 0, sizeof *o);
  o->type = zfp_type_none;
  o->minbits = ZFP_MIN_BITS;
  o->maxbits = ZFP_MAX_BITS;
  o->maxprec = ZFP_MAX_PREC;
  o->minexp = ZFP_MIN_EXP;
  o->device = -1;
  if (argc == 1)
    usage();
  for (int i = 1; i < argc; i++) {
    const char* a = argv[i];
    if (a[0] != '-' || !a[1] || a[2])
      usage();
    char c = a[1];
    if (c >= '1' && c <= '4') {
      o->dims = (uint)(c - '0');
      for (uint d = 0; d < 4; d++)
        o->n[d] = d < o->dims ? arg_size(argc, argv, &i) : 1;
      continue;
    }
    switch (c) {
      case 'a':
        if (sscanf(next_arg(argc, argv, &i), "%lf", &o->tolerance) != 1) usage();
        o->mode = 'a';
        break;
      case 'c':
        if (sscanf(next_arg(argc, argv, &i), "%u", &o->minbits) != 1 ||
            sscanf(next_arg(argc, argv, &i), "%u", &o->maxbits) != 1 ||
            sscanf(next_arg(argc, argv, &i), "%u", &o->maxprec) != 1 ||
            sscanf(next_arg(argc, argv, &i), "%d", &o->minexp) != 1)
          usage();
        o->mode = 'c';
        break;
      case 'd': o->type = zfp_type_double; break;
      case 'f': o->type = zfp_type_float; break;
      case 'h': o->header = 1; break;
      case 'i': o->in = next_arg(argc, argv, &i); break;
      case 'o': o->out = next_arg(argc, argv, &i); break;
      case 'z': o->zfp = next_arg(argc, argv, &i); break;
      case 'p':
        if (sscanf(next_arg(argc, argv, &i), "%u", &o->precision) != 1) usage();
        o->mode = 'p';
        break;
      case 'q': o->quiet = 1; break;
      case 'r':
        if (sscanf(next_arg(argc, argv, &i), "%lf", &o->rate) != 1) usage();
        o->mode = 'r';
        break;
      case 'R': o->mode = 'R'; break;
      case 's': o->stats = 1; break;
      case 't': {
        static const struct { const char* name; zfp_type t; } types[] = {
          {"i32", zfp_type_int32}, {"i64", zfp_type_int64}, {"f32", zfp_type_float}, {"f64", zfp_type_double}};
        const char* t = next_arg(argc, argv, &i);
        uint k;
        for (k = 0; k < 4 && strcmp(t, types[k].name); k++)
          ;
        if (k == 4) usage();
        o->type = types[k].t;
        break;
      }
      case 'x': {
        const char* x = next_arg(argc, argv, &i);
        int dev;
        if (!strcmp(x, "hip") || !strcmp(x, "serial") || !strcmp(x, "cuda") || !strncmp(x, "omp", 3))
          o->device = -1;
        else if (sscanf(x, "hip=%d", &dev) == 1)
          o->device = dev;
        else
          usage();
        break;
      }
      default:
        usage();
    }
  }
}

static void* read_all(const char* path, size_t* bytes)
{
  FILE* f = strcmp(path, "-") ? fopen(path, "rb") : stdin;
  size_t cap = 1 << 16, len = 0;
  unsigned char* buf = NULL;
  if (!f)
    return NULL;
  for (;;) {
    unsigned char* nb = realloc(buf, cap);
    if (!nb) die("cannot allocate memory");
    buf = nb;
    len += fread(buf + len, 1, cap - len, f);
    if (len < cap)
      break;
    cap *= 2;
  }
  if (ferror(f)) die("cannot read file");
  if (f != stdin)
    fclose(f);
  *bytes = len;
  return buf;
}

static void write_all(const char* path, const void* data, size_t bytes, const char* what)
{
  FILE* f = strcmp(path, "-") ? fopen(path, "wb") : stdout;
  if (!f || fwrite(data, 1, bytes, f) != bytes) {
    fprintf(stderr, "cannot write %s\n", what);
    exit(EXIT_FAILURE);
  }
  if (f != stdout)
    fclose(f);
}

static double value_at(const void* p, zfp_type t, size_t i)
{
  switch (t) {
    case zfp_type_int32: return (double)((const int32*)p)[i];
    case zfp_type_int64: return (double)((const int64*)p)[i];
    case zfp_type_float: return (double)((const float*)p)[i];
    default: return ((const double*)p)[i];
  }
}

/* rmse, range-normalised rmse, max error, psnr (the reference's -s line) */
static void print_stats(const void* a, const void* b, zfp_type t, size_t count)
{
  double sum = 0, emax = 0, lo = 0, hi = 0;
  for (size_t i = 0; i < count; i++) {
    double x = value_at(a, t, i), y = value_at(b, t, i), e = y - x;
    sum += e * e;
    if (fabs(e) > emax) emax = fabs(e);
    if (!i || x < lo) lo = x;
    if (!i || x > hi) hi = x;
  }
  double rmse = count ? sqrt(sum / count) : 0, range = hi - lo;
  double nrmse = range > 0 ? rmse / range : 0;
  double psnr = (rmse > 0 && range > 0) ? 20 * log10(range / (2 * rmse)) : INFINITY;
  fprintf(stderr, " rmse=%.4g nrmse=%.4g maxe=%.4g psnr=%.2f", rmse, nrmse, emax, psnr);
}

static void configure(zfp_stream* zs, zfp_field* field, const options* o)
{
  zfp_field_set_type(field, o->type);
  switch (o->dims) {
    case 1: zfp_field_set_size_1d(field, o->n[0]); break;
    case 2: zfp_field_set_size_2d(field, o->n[0], o->n[1]); break;
    case 3: zfp_field_set_size_3d(field, o->n[0], o->n[1], o->n[2]); break;
    case 4: zfp_field_set_size_4d(field, o->n[0], o->n[1], o->n[2], o->n[3]); break;
  }
  switch (o->mode) {
    case 'R': zfp_stream_set_reversible(zs); break;
    case 'a': zfp_stream_set_accuracy(zs, o->tolerance); break;
    case 'p': zfp_stream_set_precision(zs, o->precision); break;
    case 'r': zfp_stream_set_rate(zs, o->rate, o->type, o->dims, zfp_false); break;
    case 'c':
      if (!zfp_stream_set_params(zs, o->minbits, o->maxbits ? o->maxbits : ZFP_MAX_BITS,
                                 o->maxprec ? o->maxprec : (uint)(CHAR_BIT * zfp_type_size(o->type)), o->minexp))
        die("invalid compression parameters");
      break;
  }
}

int main(int argc, char** argv)
{
  options o;
  parse(&o, argc, argv);
  size_t tsize = zfp_type_size(o.type);
  size_t count = o.n[0] * o.n[1] * o.n[2] * o.n[3];
  const int known_meta = tsize && o.dims;

  if (o.dims && !count) die("array size must be nonzero");
  if (!o.in && !o.zfp) die("must specify uncompressed or compressed input file via -i or -z");
  if (o.in && !tsize) die("must specify scalar type via -f, -d, or -t to compress");
  if (o.in && !o.dims) die("must specify array dimensions via -1, -2, -3, or -4 to compress");
  if (o.in && !o.mode) die("must specify compression parameters via -a, -c, -p, or -r to compress");
  if (!o.in && !o.header && !(known_meta && o.mode))
    die("must specify type, dimensions and compression parameters or header via -h to decompress");
  if (o.stats && !o.in) die("must specify input file via -i to compute stats");
  if (!o.in && o.header && (tsize || o.dims)) die("cannot specify both field type/size and header");

  zfp_stream* zs = zfp_stream_open(NULL);
  zfp_field* field = zfp_field_alloc();
  zfp_stream_set_execution(zs, zfp_exec_hip);
  if (o.device >= 0)
    zfp_stream_set_hip_device(zs, o.device);

  void *raw = NULL, *buf = NULL, *back = NULL;
  size_t rawsize = 0, zsize = 0, bufsize = 0;
  bitstream* bs = NULL;

  if (o.in) {
    raw = read_all(o.in, &rawsize);
    if (!raw) die("cannot open input file");
    if (rawsize < tsize * count) die("cannot read input file");
    rawsize = tsize * count;
    configure(zs, field, &o);
    zfp_field_set_pointer(field, raw);
    bufsize = zfp_stream_maximum_size(zs, field);
    if (!bufsize) die("invalid compression parameters");
    buf = malloc(bufsize);
    if (!buf) die("cannot allocate memory");
    bs = stream_open(buf, bufsize);
    zfp_stream_set_bit_stream(zs, bs);
    if (o.header && !zfp_write_header(zs, field, ZFP_HEADER_FULL)) die("cannot write header");
    zsize = zfp_compress(zs, field);
    if (!zsize) die("compression failed");
    if (o.zfp)
      write_all(o.zfp, buf, zsize, "compressed file");
  } else {
    buf = read_all(o.zfp, &zsize);
    if (!buf) die("cannot open compressed file");
    bufsize = zsize;
    bs = stream_open(buf, bufsize);
    zfp_stream_set_bit_stream(zs, bs);
    if (!o.header)
      configure(zs, field, &o);
  }

  if ((!o.in && o.zfp) || o.out || o.stats) {
    zfp_stream_rewind(zs);
    if (o.header) {
      if (!zfp_read_header(zs, field, ZFP_HEADER_FULL)) die("incorrect or missing header");
      o.type = field->type;
      tsize = zfp_type_size(o.type);
      if (!tsize) die("unsupported type");
      size_t sz[4] = {field->nx, field->ny, field->nz, field->nw};
      count = 1;
      for (int d = 0; d < 4; d++) {
        o.n[d] = sz[d] ? sz[d] : 1;
        count *= o.n[d];
      }
    }
    rawsize = tsize * count;
    back = malloc(rawsize);
    if (!back) die("cannot allocate memory");
    zfp_field_set_pointer(field, back);
    if (!zfp_decompress(zs, field)) die("decompression failed");
    if (o.out)
      write_all(o.out, back, rawsize, "output file");
  }

  if (!o.quiet) {
    static const char* names[] = {"int32", "int64", "float", "double"};
    fprintf(stderr, "type=%s nx=%zu ny=%zu nz=%zu nw=%zu", names[o.type - zfp_type_int32], o.n[0], o.n[1], o.n[2],
            o.n[3]);
    fprintf(stderr, " raw=%lu zfp=%lu ratio=%.3g rate=%.4g", (unsigned long)rawsize, (unsigned long)zsize,
            (double)rawsize / zsize, CHAR_BIT * (double)zsize / count);
    if (o.stats)
      print_stats(raw, back, o.type, count);
    fprintf(stderr, "\n");
  }
  zfp_field_free(field);
  zfp_stream_close(zs);
  stream_close(bs);
  free(buf);
  free(raw);
  free(back);
  return EXIT_SUCCESS;
}
