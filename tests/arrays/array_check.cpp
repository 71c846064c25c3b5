// TEST INFRASTRUCTURE: one program, built twice (oracle/Makefile `arrays`):
//   oracle/build/array_check      zfp::hip::array3 (include/zfp/hip/array.hpp) over libzfp.so (GPU)
//   oracle/_ref/array_check_ref   the reference's zfp::array3 (its own headers, include/zfp/array3.hpp)
//                                 over the reference library compiled here
// Both run the same sequence on the same input and write what tests/test_gpu_arrays.py compares:
//   PREFIX.set.z     compressed bytes after construction from the input (array3.hpp:62-72, set)
//   PREFIX.set.raw   get() after that
//   PREFIX.elem.z    compressed bytes after element writes (cache write-back, array3.hpp:164-168)
//   PREFIX.elem.raw  get() after those
// and prints the sum of every element read through operator() (cache fills).
// usage: array_check f|d NX NY NZ RATE INPUT.raw PREFIX
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#ifdef USE_REF
#include "zfp/array3.hpp"
template <typename T> using Array3 = zfp::array3<T>;
#else
#include "zfp/hip/array.hpp"
template <typename T> using Array3 = zfp::hip::array3<T>;
#endif

static void put(const char* path, const void* p, size_t n)
{
  FILE* f = std::fopen(path, "wb");
  if (!f || std::fwrite(p, 1, n, f) != n) {
    std::perror(path);
    std::exit(1);
  }
  std::fclose(f);
}

template <typename T>
static int run(size_t nx, size_t ny, size_t nz, double rate, const char* in, const char* prefix)
{
  const size_t n = nx * ny * nz;
  std::vector<T> v(n), out(n);
  FILE* f = std::fopen(in, "rb");
  if (!f || std::fread(v.data(), sizeof(T), n, f) != n) {
    std::perror(in);
    return 1;
  }
  std::fclose(f);
  std::string pre(prefix);
  Array3<T> a(nx, ny, nz, rate, v.data());
  put((pre + ".set.z").c_str(), a.compressed_data(), a.compressed_size());
  a.get(out.data());
  put((pre + ".set.raw").c_str(), out.data(), n * sizeof(T));
  // reads through the cache
  double sum = 0;
  for (size_t k = 0; k < nz; k++)
    for (size_t j = 0; j < ny; j++)
      for (size_t i = 0; i < nx; i++)
        sum += (double)(T)a(i, j, k);
  // element writes: read-modify-writes of one element in each of 500 distinct
  // random blocks, then whole blocks one after another -- every block's
  // writes fall in one cache residency, in the reference's direct-mapped block
  // cache (cache.hpp) and in the line cache of zfp::hip alike (a block evicted
  // between two writes takes two lossy round trips, and the two caches evict
  // differently)
  const size_t bx = (nx + 3) / 4, by = (ny + 3) / 4, bz = (nz + 3) / 4;
  std::vector<char> hit(bx * by * bz, 0);
  uint64_t s = 88172645463325252ull;
  for (int t = 0; t < 500;) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    const size_t i = s % nx, j = (s >> 20) % ny, k = (s >> 40) % nz;
    const size_t b = i / 4 + bx * (j / 4 + by * (k / 4));
    if (hit[b])
      continue;
    hit[b] = 1;
    t++;
    a(i, j, k) = (T)(0.5 * (double)(T)a(i, j, k) + (double)(i + j + k));
  }
  // the last two z layers of blocks, block after block (each block's 64 writes in a row)
  for (size_t b = (bz > 2 ? bz - 2 : 0) * bx * by; b < bx * by * bz; b++)
    if (!hit[b])
      for (size_t k = 4 * (b / (bx * by)); k < nz && k < 4 * (b / (bx * by)) + 4; k++)
        for (size_t j = 4 * (b / bx % by); j < ny && j < 4 * (b / bx % by) + 4; j++)
          for (size_t i = 4 * (b % bx); i < nx && i < 4 * (b % bx) + 4; i++)
            a(i, j, k) += (T)1;
  put((pre + ".elem.z").c_str(), a.compressed_data(), a.compressed_size());
  a.get(out.data());
  put((pre + ".elem.raw").c_str(), out.data(), n * sizeof(T));
  std::printf("sum %.17g bytes %zu\n", sum, (size_t)a.compressed_size());
  return 0;
}

int main(int argc, char** argv)
{
  if (argc != 8) {
    std::fprintf(stderr, "usage: %s f|d NX NY NZ RATE INPUT PREFIX\n", argv[0]);
    return 2;
  }
  const size_t nx = std::strtoull(argv[2], 0, 10), ny = std::strtoull(argv[3], 0, 10), nz = std::strtoull(argv[4], 0, 10);
  const double rate = std::atof(argv[5]);
  try {
    return argv[1][0] == 'd' ? run<double>(nx, ny, nz, rate, argv[6], argv[7])
                             : run<float>(nx, ny, nz, rate, argv[6], argv[7]);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "error: %s\n", e.what());
    return 1;
  }
}
