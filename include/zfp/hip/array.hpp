// GPU-native fixed-rate compressed arrays (zfp::hip::array1 .. array4).
//
// The reference's C++ compressed arrays (include/zfp/array{1,2,3,4}.hpp of
// SEP-software/zfp-par, zfp 1.0.1) keep a fixed-rate block store -- block i of
// the raster block order at bit i * maxbits (internal/array/store{1..4}.hpp:
// 96-118, index implicit) -- and a cache of decompressed blocks, and code
// every block through the per-block C API (codec/zfpcodec.hpp), one block per
// call.  On this library a per-block call is a GPU round trip, so these arrays
// keep the same store, bit for bit, but move blocks through the codec in bulk:
//
//   set(p) / get(p)      one zfp_compress / zfp_decompress of the whole array
//                        (array3.hpp:187-225 loops over every block instead);
//   element access       a cache of decoded lines -- up to kLineBlocks blocks
//                        along x of one block row -- filled by one
//                        zfp_decompress of the line at its stream offset;
//   write-back           modified blocks are re-encoded, each run of
//                        consecutive modified blocks of a line by one
//                        zfp_compress at its offset (fixed-rate blocks are
//                        word-aligned: maxbits is a multiple of 64, so a run
//                        owns whole stream words).  Unmodified blocks keep
//                        their bits, as in the reference (cache3.hpp:40-50
//                        re-encodes dirty blocks only).
//
// The compressed bytes (compressed_data(), compressed_size()) equal the
// reference array's after set(), and after element writes whenever each
// block's writes fall in one cache residency in both arrays: a block evicted
// between two of its writes goes through two lossy encode/decode round trips,
// and the reference's direct-mapped block cache (cache.hpp) evicts at other
// times than this line cache (tests/test_gpu_arrays.py checks both against
// the reference's array3 built from its own headers).  Covered: construction, set/get, (i, j, k) and flat
// element access (read, assign, += -= *= /=), rate, resize, cache control.
// Not covered: views, iterators, pointers, serialization headers and the
// variable-rate (const) arrays of the reference.
#ifndef ZFP_HIP_ARRAY_HPP
#define ZFP_HIP_ARRAY_HPP

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <list>
#include <stdexcept>
#include <unordered_map>
#include <vector>

#include "zfp.h"

namespace zfp {
namespace hip {

template <typename Scalar> struct scalar_type;
template <> struct scalar_type<int32> { static const zfp_type type = zfp_type_int32; };
template <> struct scalar_type<int64> { static const zfp_type type = zfp_type_int64; };
template <> struct scalar_type<float> { static const zfp_type type = zfp_type_float; };
template <> struct scalar_type<double> { static const zfp_type type = zfp_type_double; };

// D-dimensional fixed-rate array; extents n[0] (x, fastest) .. n[D-1]
template <typename Scalar, unsigned D>
class array {
public:
  static const size_t kLineBlocks = 256;  // blocks per cache line (along x)

  array() : zs(0), bs(0), maxbits(0), nblocks(0), line_cap(0) { std::memset(n, 0, sizeof(n)); std::memset(nb, 0, sizeof(nb)); }

  // n: D extents (x first); rate in bits per value (word-aligned, as
  // zfp_config_rate(rate, true) in array3.hpp:62-72); optional initial data;
  // cache_size: bytes of decoded lines to keep (0: 16 lines)
  array(const size_t* extents, double rate, const Scalar* p = 0, size_t cache_size = 0) : array()
  {
    zs = zfp_stream_open(0);
    resize(extents, false);
    set_rate(rate);
    set_cache_size(cache_size);
    if (p)
      set(p);
  }

  ~array()
  {
    if (bs)
      stream_close(bs);
    if (zs)
      zfp_stream_close(zs);
  }

  array(const array&) = delete;
  array& operator=(const array&) = delete;

  size_t size() const
  {
    size_t s = 1;
    for (unsigned a = 0; a < D; a++)
      s *= n[a];
    return s;
  }
  size_t size_x() const { return n[0]; }
  size_t size_y() const { return D > 1 ? n[1] : 0; }
  size_t size_z() const { return D > 2 ? n[2] : 0; }
  size_t size_w() const { return D > 3 ? n[3] : 0; }

  double rate() const { return (double)maxbits / (double)(size_t(1) << (2 * D)); }

  // set rate (the array's contents are lost, as array3.hpp:143-147)
  double set_rate(double r)
  {
    lines.clear();
    order.clear();
    const double got = zfp_stream_set_rate(zs, r, scalar_type<Scalar>::type, D, 1);
    maxbits = zs->maxbits;
    alloc();
    return got;
  }

  // resize (contents lost unless clear == false and the size is unchanged)
  void resize(const size_t* extents, bool clear = true)
  {
    lines.clear();
    order.clear();
    nblocks = 1;
    for (unsigned a = 0; a < D; a++) {
      n[a] = extents[a];
      nb[a] = (n[a] + 3) / 4;
      nblocks *= nb[a];
    }
    if (maxbits)
      alloc();
    (void)clear;
  }

  size_t compressed_size() const { return store.size() * sizeof(uint64_t); }
  void* compressed_data() const
  {
    flush_cache();
    return (void*)store.data();
  }

  size_t cache_size() const { return line_cap * line_values() * sizeof(Scalar); }
  void set_cache_size(size_t bytes)
  {
    flush_cache();
    lines.clear();
    order.clear();
    const size_t per = line_values() * sizeof(Scalar);
    line_cap = bytes ? (bytes + per - 1) / per : 16;
    if (line_cap < 1)
      line_cap = 1;
  }
  void clear_cache() const
  {
    lines.clear();
    order.clear();
  }
  void flush_cache() const
  {
    for (auto& kv : lines)
      write_back(kv.first, kv.second);
  }

  // decompress the whole array to p (contiguous, x fastest): one GPU call
  void get(Scalar* p) const
  {
    flush_cache();
    zfp_field* f = field_over(p, n, nullptr);
    stream_rewind(bs);
    zfp_stream_rewind(zs);
    const size_t ok = zfp_decompress(zs, f);
    zfp_field_free(f);
    if (!ok)
      throw std::runtime_error("zfp::hip::array: decompression failed");
  }

  // compress the whole array from p (contiguous, x fastest), or zero it: one GPU call
  void set(const Scalar* p)
  {
    lines.clear();
    order.clear();
    if (!p) {
      std::fill(store.begin(), store.end(), uint64_t(0));  // every zero block codes as zero bits
      return;
    }
    zfp_field* f = field_over(const_cast<Scalar*>(p), n, nullptr);
    zfp_stream_rewind(zs);
    const size_t ok = zfp_compress(zs, f);
    zfp_field_free(f);
    if (!ok)
      throw std::runtime_error("zfp::hip::array: compression failed");
  }

  // element access (x index first)
  class reference {
  public:
    reference(array* a, const size_t* ix) : a(a) { std::memcpy(i, ix, sizeof(i)); }
    operator Scalar() const { return a->get_element(i); }
    reference& operator=(Scalar v) { a->ref_element(i) = v; return *this; }
    reference& operator=(const reference& r) { return *this = Scalar(r); }
    reference& operator+=(Scalar v) { a->ref_element(i) += v; return *this; }
    reference& operator-=(Scalar v) { a->ref_element(i) -= v; return *this; }
    reference& operator*=(Scalar v) { a->ref_element(i) *= v; return *this; }
    reference& operator/=(Scalar v) { a->ref_element(i) /= v; return *this; }
  private:
    array* a;
    size_t i[D];
  };

  Scalar get_element(const size_t* i) const { return *element(i, false); }
  Scalar& ref_element(const size_t* i) { return *element(i, true); }

  // flat index (x fastest) to indices
  void indices(size_t index, size_t* i) const
  {
    for (unsigned a = 0; a < D; a++) {
      i[a] = index % n[a];
      index /= n[a];
    }
  }

protected:
  struct Line {
    std::vector<Scalar> v;      // line values, layout [w][z][y][4 * blocks] (x fastest)
    std::vector<uint8_t> dirty; // per block of the line
  };

  size_t line_blocks() const { return nb[0] < kLineBlocks ? nb[0] : kLineBlocks; }
  size_t line_values() const { return 4 * line_blocks() * (size_t(1) << (2 * (D - 1))); }

  void alloc()
  {
    const size_t words = (nblocks * (size_t)maxbits + 63) / 64;
    store.assign(words ? words : 1, 0);
    if (bs)
      stream_close(bs);
    bs = stream_open(store.data(), store.size() * sizeof(uint64_t));
    zfp_stream_set_bit_stream(zs, bs);
  }

  // field over p with extents e (D of them) and strides st (nullptr: contiguous)
  zfp_field* field_over(Scalar* p, const size_t* e, const ptrdiff_t* st) const
  {
    const zfp_type t = scalar_type<Scalar>::type;
    zfp_field* f = D == 1 ? zfp_field_1d(p, t, e[0])
                 : D == 2 ? zfp_field_2d(p, t, e[0], e[1])
                 : D == 3 ? zfp_field_3d(p, t, e[0], e[1], e[2])
                          : zfp_field_4d(p, t, e[0], e[1], e[2], e[3]);
    if (st) {
      if (D == 1) zfp_field_set_stride_1d(f, st[0]);
      if (D == 2) zfp_field_set_stride_2d(f, st[0], st[1]);
      if (D == 3) zfp_field_set_stride_3d(f, st[0], st[1], st[2]);
      if (D == 4) zfp_field_set_stride_4d(f, st[0], st[1], st[2], st[3]);
    }
    return f;
  }

  // line key: (x segment, block row); first block index of the line; its extents
  size_t line_key(const size_t* i) const
  {
    size_t row = 0;
    for (unsigned a = D; a-- > 1;)
      row = row * nb[a] + i[a] / 4;
    const size_t segs = (nb[0] + line_blocks() - 1) / line_blocks();
    return row * segs + (i[0] / 4) / line_blocks();
  }
  void line_geometry(size_t key, size_t& first_block, size_t& nbl, size_t* e) const
  {
    const size_t L = line_blocks(), segs = (nb[0] + L - 1) / L;
    const size_t seg = key % segs;
    size_t row = key / segs;
    const size_t bx0 = seg * L;
    nbl = (nb[0] - bx0) < L ? nb[0] - bx0 : L;
    first_block = row * nb[0] + bx0;
    e[0] = (n[0] - 4 * bx0) < 4 * nbl ? n[0] - 4 * bx0 : 4 * nbl;
    for (unsigned a = 1; a < D; a++) {
      const size_t b = row % nb[a];
      row /= nb[a];
      e[a] = (n[a] - 4 * b) < 4 ? n[a] - 4 * b : 4;
    }
  }
  void line_strides(ptrdiff_t* st) const
  {
    st[0] = 1;
    for (unsigned a = 1; a < D; a++)
      st[a] = st[a - 1] * (a == 1 ? ptrdiff_t(4 * line_blocks()) : 4);
  }

  // one GPU call: decode the line's blocks from their stream offset
  void fetch(size_t key, Line& ln) const
  {
    size_t first, nbl, e[4];
    ptrdiff_t st[4];
    line_geometry(key, first, nbl, e);
    line_strides(st);
    ln.v.assign(line_values(), Scalar(0));
    ln.dirty.assign(nbl, 0);
    zfp_field* f = field_over(ln.v.data(), e, st);
    stream_rseek(bs, (bitstream_offset)(first * (size_t)maxbits));
    const size_t ok = zfp_decompress(zs, f);
    zfp_field_free(f);
    if (!ok)
      throw std::runtime_error("zfp::hip::array: line decompression failed");
  }

  // re-encode the modified blocks of a line: one GPU call per run of them
  void write_back(size_t key, Line& ln) const
  {
    size_t first, nbl, e[4];
    ptrdiff_t st[4];
    line_geometry(key, first, nbl, e);
    line_strides(st);
    for (size_t b = 0; b < nbl;) {
      if (!ln.dirty[b]) {
        b++;
        continue;
      }
      size_t c = b;
      while (c < nbl && ln.dirty[c])
        c++;
      size_t re[4];
      std::memcpy(re, e, sizeof(re));
      re[0] = (e[0] - 4 * b) < 4 * (c - b) ? e[0] - 4 * b : 4 * (c - b);
      zfp_field* f = field_over(ln.v.data() + 4 * b, re, st);
      stream_wseek(bs, (bitstream_offset)((first + b) * (size_t)maxbits));
      const size_t ok = zfp_compress(zs, f);
      zfp_field_free(f);
      if (!ok)
        throw std::runtime_error("zfp::hip::array: block write-back failed");
      for (size_t k = b; k < c; k++)
        ln.dirty[k] = 0;
      b = c;
    }
  }

  Scalar* element(const size_t* i, bool write) const
  {
    const size_t key = line_key(i);
    auto it = lines.find(key);
    if (it == lines.end()) {
      if (lines.size() >= line_cap) {  // evict the least recently fetched line
        const size_t old = order.front();
        order.pop_front();
        auto o = lines.find(old);
        write_back(old, o->second);
        lines.erase(o);
      }
      it = lines.emplace(key, Line()).first;
      order.push_back(key);
      fetch(key, it->second);
    }
    Line& ln = it->second;
    const size_t bx0 = ((i[0] / 4) / line_blocks()) * line_blocks();
    size_t off = i[0] - 4 * bx0;
    const size_t sx = 4 * line_blocks();
    size_t st = sx;
    for (unsigned a = 1; a < D; a++) {
      off += (i[a] % 4) * st;
      st *= 4;
    }
    if (write)
      ln.dirty[i[0] / 4 - bx0] = 1;
    return &ln.v[off];
  }

  zfp_stream* zs;
  bitstream* bs;
  uint maxbits;
  size_t n[4], nb[4], nblocks;
  std::vector<uint64_t> store;                   // the fixed-rate block store
  size_t line_cap;                               // decoded lines kept
  mutable std::unordered_map<size_t, Line> lines;
  mutable std::list<size_t> order;
};

// the reference's constructors and accessors per dimensionality (array1.hpp .. array4.hpp)
template <typename Scalar>
class array1 : public array<Scalar, 1> {
public:
  typedef array<Scalar, 1> base;
  array1(size_t nx, double rate, const Scalar* p = 0, size_t cache_size = 0) : base(ext(nx), rate, p, cache_size) {}
  typename base::reference operator()(size_t i) { size_t x[1] = {i}; return typename base::reference(this, x); }
  Scalar operator()(size_t i) const { size_t x[1] = {i}; return this->get_element(x); }
  typename base::reference operator[](size_t i) { return (*this)(i); }
  void resize(size_t nx, bool clear = true) { base::resize(ext(nx), clear); }
private:
  static const size_t* ext(size_t nx) { thread_local size_t e[1]; e[0] = nx; return e; }
};

template <typename Scalar>
class array2 : public array<Scalar, 2> {
public:
  typedef array<Scalar, 2> base;
  array2(size_t nx, size_t ny, double rate, const Scalar* p = 0, size_t cache_size = 0)
      : base(ext(nx, ny), rate, p, cache_size) {}
  typename base::reference operator()(size_t i, size_t j) { size_t x[2] = {i, j}; return typename base::reference(this, x); }
  Scalar operator()(size_t i, size_t j) const { size_t x[2] = {i, j}; return this->get_element(x); }
  typename base::reference operator[](size_t index) { size_t x[2]; this->indices(index, x); return typename base::reference(this, x); }
  void resize(size_t nx, size_t ny, bool clear = true) { base::resize(ext(nx, ny), clear); }
private:
  static const size_t* ext(size_t nx, size_t ny) { thread_local size_t e[2]; e[0] = nx; e[1] = ny; return e; }
};

template <typename Scalar>
class array3 : public array<Scalar, 3> {
public:
  typedef array<Scalar, 3> base;
  array3(size_t nx, size_t ny, size_t nz, double rate, const Scalar* p = 0, size_t cache_size = 0)
      : base(ext(nx, ny, nz), rate, p, cache_size) {}
  typename base::reference operator()(size_t i, size_t j, size_t k)
  {
    size_t x[3] = {i, j, k};
    return typename base::reference(this, x);
  }
  Scalar operator()(size_t i, size_t j, size_t k) const { size_t x[3] = {i, j, k}; return this->get_element(x); }
  typename base::reference operator[](size_t index) { size_t x[3]; this->indices(index, x); return typename base::reference(this, x); }
  void resize(size_t nx, size_t ny, size_t nz, bool clear = true) { base::resize(ext(nx, ny, nz), clear); }
private:
  static const size_t* ext(size_t nx, size_t ny, size_t nz)
  {
    thread_local size_t e[3];
    e[0] = nx, e[1] = ny, e[2] = nz;
    return e;
  }
};

template <typename Scalar>
class array4 : public array<Scalar, 4> {
public:
  typedef array<Scalar, 4> base;
  array4(size_t nx, size_t ny, size_t nz, size_t nw, double rate, const Scalar* p = 0, size_t cache_size = 0)
      : base(ext(nx, ny, nz, nw), rate, p, cache_size) {}
  typename base::reference operator()(size_t i, size_t j, size_t k, size_t l)
  {
    size_t x[4] = {i, j, k, l};
    return typename base::reference(this, x);
  }
  Scalar operator()(size_t i, size_t j, size_t k, size_t l) const
  {
    size_t x[4] = {i, j, k, l};
    return this->get_element(x);
  }
  typename base::reference operator[](size_t index) { size_t x[4]; this->indices(index, x); return typename base::reference(this, x); }
  void resize(size_t nx, size_t ny, size_t nz, size_t nw, bool clear = true) { base::resize(ext(nx, ny, nz, nw), clear); }
private:
  static const size_t* ext(size_t nx, size_t ny, size_t nz, size_t nw)
  {
    thread_local size_t e[4];
    e[0] = nx, e[1] = ny, e[2] = nz, e[3] = nw;
    return e;
  }
};

typedef array1<float> array1f;
typedef array1<double> array1d;
typedef array2<float> array2f;
typedef array2<double> array2d;
typedef array3<float> array3f;
typedef array3<double> array3d;
typedef array4<float> array4f;
typedef array4<double> array4d;

}  // namespace hip
}  // namespace zfp

#endif
