/* TEST INFRASTRUCTURE: the reference's cfp (C bindings of its compressed
 * arrays, cfp/cfp.cpp, compiled unchanged) driven from C, built twice by
 * oracle/Makefile: over the reference library (oracle/_ref/cfp_check_ref) and
 * over this libzfp.so (oracle/_ref/cfp_check_dropin).  tests/test_gpu_arrays.py
 * compares what both write:
 *   PREFIX.set.z / .set.raw    compressed bytes / get_array after construction
 *   PREFIX.elem.z / .elem.raw  the same after element writes through cfp set()
 * and the sum of the elements read through cfp get() (cache fills), printed.
 * usage: cfp_check NX NY NZ RATE INPUT.raw PREFIX   (float arrays, array3f) */
#include <stdio.h>
#include <stdlib.h>
#include "zfp/array.h"

static void put(const char* path, const void* p, size_t n)
{
  FILE* f = fopen(path, "wb");
  if (!f || fwrite(p, 1, n, f) != n) {
    perror(path);
    exit(1);
  }
  fclose(f);
}

int main(int argc, char** argv)
{
  if (argc != 7) {
    fprintf(stderr, "usage: cfp_check NX NY NZ RATE INPUT.raw PREFIX\n");
    return 2;
  }
  const size_t nx = (size_t)atol(argv[1]), ny = (size_t)atol(argv[2]), nz = (size_t)atol(argv[3]), n = nx * ny * nz;
  const double rate = atof(argv[4]);
  float* v = (float*)malloc(n * sizeof(float));
  float* out = (float*)malloc(n * sizeof(float));
  FILE* f = fopen(argv[5], "rb");
  if (!f || fread(v, sizeof(float), n, f) != n) {
    perror(argv[5]);
    return 1;
  }
  fclose(f);
  char path[4096];
  cfp_array3f a = cfp.array3f.ctor(nx, ny, nz, rate, v, 0);
  snprintf(path, sizeof path, "%s.set.z", argv[6]);
  put(path, cfp.array3f.compressed_data(a), cfp.array3f.compressed_size(a));
  cfp.array3f.get_array(a, out);
  snprintf(path, sizeof path, "%s.set.raw", argv[6]);
  put(path, out, n * sizeof(float));
  /* element reads and writes through the array's cache */
  double sum = 0;
  for (size_t t = 0; t < 400; t++) {
    const size_t i = (t * 7919) % nx, j = (t * 104729) % ny, k = (t * 1299709) % nz;
    const float x = cfp.array3f.get(a, i, j, k);
    sum += x;
    cfp.array3f.set(a, i, j, k, 0.5f * x + 1.0f);
  }
  cfp.array3f.flush_cache(a);
  snprintf(path, sizeof path, "%s.elem.z", argv[6]);
  put(path, cfp.array3f.compressed_data(a), cfp.array3f.compressed_size(a));
  cfp.array3f.get_array(a, out);
  snprintf(path, sizeof path, "%s.elem.raw", argv[6]);
  put(path, out, n * sizeof(float));
  printf("%.9g %zu\n", sum, cfp.array3f.compressed_size(a));
  cfp.array3f.dtor(a);
  free(v);
  free(out);
  return 0;
}
