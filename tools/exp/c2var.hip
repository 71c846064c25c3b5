// Experiment harness (not product code): the product fixed-rate 3D f32 encoder
// (encode3_aligned, kernels3.h) and stage-removal variants of it, timed with
// HIP events on a device-resident 1024^3 F1 field at rate 16.  Build variants
// with -D switches (tools/exp/build_c2var.sh); every binary prints the kernel
// time and a checksum of the stream, so variants can be checked for identical
// output.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <string>
#include "kernels3.h"
#include "ilv.h"
using namespace zfp_amd;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void fill_f1(float* d, uint32_t n)
{
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)n * n * n) return;
  const uint32_t x = (uint32_t)(i % n), y = (uint32_t)((i / n) % n), z = (uint32_t)(i / ((uint64_t)n * n));
  d[i] = (float)(sin(0.05 * x) * cos(0.03 * y) + 0.5 * sin(0.02 * z + 0.01 * (double)x * y / n));
}

__global__ void checksum(const uint64_t* w, uint64_t n, unsigned long long* out)
{
  uint64_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    acc += w[i] * (2 * i + 1);
  atomicAdd(out, (unsigned long long)acc);
}

// stage variants: 1 = loads + tables + slot zeroing + copy-out only;
// 2 = + cast, lift, planes (no coder); 3 = + coder on zero planes
template <int MODE>
__global__ __launch_bounds__(256, 3) void enc_stage(const float* __restrict__ data, Geometry g, CodecParams cp,
                                                   uint64_t* __restrict__ out, uint32_t sw, uint32_t sdw, uint32_t magic_c)
{
  __shared__ uint32_t lut[512];
  extern __shared__ uint32_t ldsw[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint32_t* wslot = ldsw + (size_t)wv * 64 * sdw;
  const uint64_t w = (uint64_t)blockIdx.x * kWavesPerGroup + wv;
  const uint64_t first = w * 64;
  const uint64_t b = first + lane;
  float v[64];
  BlockPos p = block_pos(g, b, 3);
  gather3<float, true>(v, data, g, p);
  {
    const uint4* src = reinterpret_cast<const uint4*>(&kCoderTables);
    uint4* dst = reinterpret_cast<uint4*>(lut);
    dst[lane] = src[lane];
    dst[lane + 64] = src[lane + 64];
    uint4* z = reinterpret_cast<uint4*>(wslot);
    for (uint32_t i = lane; i < 16 * sdw; i += 64)
      z[i] = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  }
  uint32_t* slot = wslot + (size_t)lane * sdw;
  if (MODE == 1) {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 64; i++) acc ^= __float_as_uint(v[i]);
    slot[0] = acc;
  } else {
    int32_t q[64];
    uint32_t mp;
    lossy_emax_cast(q, v, cp, mp, [&](float (&r)[64]) { gather3<float, true>(r, data, g, p); });
    xform<3, false, false>(q);
    uint32_t Pl[32], Ph[32];
    planes_from_coeffs(Pl, Ph, q);
    pin_registers(Pl);
    pin_registers(Ph);
    if (MODE == 2) {
      uint32_t acc = 0;
#pragma unroll
      for (int k = 0; k < 32; k++) acc ^= Pl[k] + 3u * Ph[k] + k;
      slot[0] = acc;
    } else {
#pragma unroll
      for (int k = 0; k < 32; k++) { Pl[k] &= 0xffu; Ph[k] = 0; }
      code_planes_fr32(slot, sdw - 1, lut, 9, cp.maxbits, Pl, Ph);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const uint32_t hw = sw >> 1, chunks = 64 * hw;
  uint64_t* dst = out + first * sw;
  for (uint32_t c = lane; c < chunks; c += 64) {
    const uint32_t l = div_magic(c, magic_c);
    const uint32_t* s = wslot + (size_t)l * sdw + 4 * (c - l * hw);
    *reinterpret_cast<uint4*>(dst + 2 * c) = make_uint4(s[0], s[1], s[2], s[3]);
  }
}

// round 4: the product kernel with the block loads of a workgroup's waves
// staggered -- wave wv issues its loads once waves < wv/G*G have theirs in
// registers (G waves load together); fewer bytes in flight per CU and the
// waves' coder phases spread apart.
template <int G, bool SYNC = true, bool WAIT0 = true>
__global__ __launch_bounds__(256, 3) void enc_gate(const float* __restrict__ data, Geometry g, CodecParams cp,
                                                 uint64_t* __restrict__ out, uint32_t sw, uint32_t sdw, uint32_t magic_c)
{
  constexpr int MORPH = 0;
  __shared__ uint32_t lut[512];
  __shared__ uint32_t gate;
  extern __shared__ uint32_t ldsw[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint32_t* wslot = ldsw + (size_t)wv * 64 * sdw;
  const uint64_t w = (uint64_t)blockIdx.x * kWavesPerGroup + wv;
  const uint64_t first = w * 64;
  const uint64_t b = first + lane;
  if (threadIdx.x == 0) gate = 0;
  if (SYNC) __syncthreads();
  float v[64];
  BlockPos p = block_pos(g, b, 3);
  const uint32_t need = (uint32_t)(wv / G) * G;
  if (need) {
    while (__hip_atomic_load(&gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need)
      __builtin_amdgcn_s_sleep(2);
  }
  gather3<float, true>(v, data, g, p);
  {
    const uint4* src = reinterpret_cast<const uint4*>(&kCoderTables);
    uint4* dst = reinterpret_cast<uint4*>(lut);
    dst[lane] = src[lane];
    dst[lane + 64] = src[lane + 64];
    uint4* z = reinterpret_cast<uint4*>(wslot);
    for (uint32_t i = lane; i < 16 * sdw; i += 64)
      z[i] = make_uint4(0, 0, 0, 0);
  }
  if (WAIT0) {
    __builtin_amdgcn_s_waitcnt(0);  // the block is in registers
    if (lane == 0) __hip_atomic_fetch_add(&gate, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
    __builtin_amdgcn_s_waitcnt(0xc07f);
  }
  __builtin_amdgcn_wave_barrier();
  if (!(MORPH & 4) || b < g.nblocks) {
    OrSlot os{reinterpret_cast<uint64_t*>(wslot + (size_t)lane * sdw), sdw - 1};
    encode_block3<float, false, true>(os, lut, v, cp, [&](float (&r)[64]) { gather3<float, true>(r, data, g, p); });
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (MORPH & 1) {
    if (first >= g.nblocks)
      return;
    const uint64_t nb = (g.nblocks - first) < 64 ? (g.nblocks - first) : 64;
    const uint32_t hw = sw >> 1, chunks = (uint32_t)nb * hw;
    uint64_t* dst = out + first * sw;
    if ((sw & 1) == 0) {
      for (uint32_t c = lane; c < chunks; c += 64) {
        const uint32_t l = div_magic(c, magic_c);
        const uint32_t* s = wslot + (size_t)l * sdw + 4 * (c - l * hw);
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(u4{s[0], s[1], s[2], s[3]}, reinterpret_cast<u4*>(dst + 2 * c));
      }
    }
    if (!(MORPH & 2)) __builtin_amdgcn_s_waitcnt(0x0f70);
    return;
  }
  const uint32_t hw = sw >> 1, chunks = 64 * hw;
  uint64_t* dst = out + first * sw;
  for (uint32_t c = lane; c < chunks; c += 64) {
    const uint32_t l = div_magic(c, magic_c);
    const uint32_t* s = wslot + (size_t)l * sdw + 4 * (c - l * hw);
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(u4{s[0], s[1], s[2], s[3]}, reinterpret_cast<u4*>(dst + 2 * c));
  }
}

// round 4: the product kernel plus an L2/MALL prefetch of the field rows of
// the workgroup DIST launches later (on the same XCD when DIST % 8 == 0):
// LDS-DMA loads into a 1 KB dummy area (no VGPRs held), so that workgroup's
// own loads hit on-die caches.
template <uint32_t DIST, int PRIO, int WPG = 4, bool GUARD = false, int MORPH = 0>
__global__ __launch_bounds__(64 * WPG, 3) void enc_pf(const float* __restrict__ data, Geometry g, CodecParams cp,
                                               uint64_t* __restrict__ out, uint32_t sw, uint32_t sdw, uint32_t magic_c)
{
  __shared__ uint32_t lut[512];
  __shared__ uint32_t dummy[256];
  extern __shared__ uint32_t ldsw[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint32_t* wslot = ldsw + (size_t)wv * 64 * sdw;
  const uint64_t w = (uint64_t)blockIdx.x * WPG + wv;
  const uint64_t first = w * 64;
  const uint64_t b = first + lane;
  float v[64];
  if (PRIO) __builtin_amdgcn_s_setprio(PRIO);
  BlockPos p{};
  if (!GUARD || b < g.nblocks) {
    p = block_pos(g, b, 3);
    gather3<float, true>(v, data, g, p);
  }
  if (PRIO) __builtin_amdgcn_s_setprio(0);
  {
    const uint4* src = reinterpret_cast<const uint4*>(&kCoderTables);
    uint4* dst = reinterpret_cast<uint4*>(lut);
    dst[lane] = src[lane];
    dst[lane + 64] = src[lane + 64];
  }
  const uint64_t bp = b + (uint64_t)DIST * 256;
  if (DIST && first + (uint64_t)DIST * 256 < g.nblocks) {
    const BlockPos pp = block_pos(g, bp, 3);
    const float* o = data + pp.off;
#pragma unroll
    for (int k = 0; k < 4; k++)
#pragma unroll
      for (int j = 0; j < 4; j++)
        __builtin_amdgcn_global_load_lds((const void*)(o + j * g.s[1] + k * g.s[2]),
                                         (__attribute__((address_space(3))) void*)dummy, 16, 0, 0);
  }
  {
    uint4* z = reinterpret_cast<uint4*>(wslot);
    for (uint32_t i = lane; i < 16 * sdw; i += 64)
      z[i] = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  }
  if (!(MORPH & 4) || b < g.nblocks) {
    OrSlot os{reinterpret_cast<uint64_t*>(wslot + (size_t)lane * sdw), sdw - 1};
    encode_block3<float, false, true>(os, lut, v, cp, [&](float (&r)[64]) { gather3<float, true>(r, data, g, p); });
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (MORPH & 1) {
    if (first >= g.nblocks)
      return;
    const uint64_t nb = (g.nblocks - first) < 64 ? (g.nblocks - first) : 64;
    const uint32_t hw = sw >> 1, chunks = (uint32_t)nb * hw;
    uint64_t* dst = out + first * sw;
    if ((sw & 1) == 0) {
      for (uint32_t c = lane; c < chunks; c += 64) {
        const uint32_t l = div_magic(c, magic_c);
        const uint32_t* s = wslot + (size_t)l * sdw + 4 * (c - l * hw);
        typedef uint32_t u4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(u4{s[0], s[1], s[2], s[3]}, reinterpret_cast<u4*>(dst + 2 * c));
      }
    }
    if (!(MORPH & 2)) __builtin_amdgcn_s_waitcnt(0x0f70);
    return;
  }
  const uint32_t hw = sw >> 1, chunks = 64 * hw;
  uint64_t* dst = out + first * sw;
  for (uint32_t c = lane; c < chunks; c += 64) {
    const uint32_t l = div_magic(c, magic_c);
    const uint32_t* s = wslot + (size_t)l * sdw + 4 * (c - l * hw);
    typedef uint32_t u4 __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(u4{s[0], s[1], s[2], s[3]}, reinterpret_cast<u4*>(dst + 2 * c));
  }
  if (!(MORPH & 2)) __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0): the prefetch has landed before the workgroup's LDS is released
}

// round 4: interleaved (conflict-free) LDS slots, each lane stores its own
// block with 16-byte strided stores (ilv.h)
template <int PRIO, int OWN>
__global__ __launch_bounds__(256, 3) void enc_ilv(const float* __restrict__ data, Geometry g, CodecParams cp,
                                                uint64_t* __restrict__ out, uint32_t rows)
{
  __shared__ uint32_t lut[512];
  extern __shared__ uint32_t ldsw[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint32_t* wreg = ldsw + (size_t)wv * 64 * rows;
  const uint64_t w = (uint64_t)blockIdx.x * kWavesPerGroup + wv;
  const uint64_t first = w * 64;
  const uint64_t b = first + lane;
  float v[64];
  if (PRIO) __builtin_amdgcn_s_setprio(PRIO);
  BlockPos p = block_pos(g, b, 3);
  gather3<float, true>(v, data, g, p);
  if (PRIO) __builtin_amdgcn_s_setprio(0);
  {
    const uint4* src = reinterpret_cast<const uint4*>(&kCoderTables);
    uint4* dst = reinterpret_cast<uint4*>(lut);
    dst[lane] = src[lane];
    dst[lane + 64] = src[lane + 64];
    uint4* z = reinterpret_cast<uint4*>(wreg);
    for (uint32_t i = lane; i < 16 * rows; i += 64)
      z[i] = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
  }
  const uint32_t lanebase = lds_off(wreg) + 4u * lane;
  ilv::encode_block_fixed_f32(lanebase, rows - 1, lut, v, cp, [&](float (&r)[64]) { gather3<float, true>(r, data, g, p); });
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  if (OWN) {
    u4* dst = reinterpret_cast<u4*>(out + b * 16);
#pragma unroll
    for (int c = 0; c < 8; c++) {
      const uint32_t* s = wreg + lane + 256 * c;
      __builtin_nontemporal_store(u4{s[0], s[64], s[128], s[192]}, dst + c);
    }
  } else {
    // coalesced: chunk t of the wave's run = dwords 4(t%8) .. of block t/8
    u4* dst = reinterpret_cast<u4*>(out + first * 16);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t t = lane + 64 * i, l = t >> 3, c = t & 7;
      const uint32_t* s = wreg + l + 256 * c;
      __builtin_nontemporal_store(u4{s[0], s[64], s[128], s[192]}, dst + t);
    }
  }
}

template <typename K>
static float time_it(K launch, int reps)
{
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int r = 0; r < 5; r++) launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; r++) launch();
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv)
{
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const char* tag = argc > 1 ? argv[1] : "base";
  const bool stages = argc > 2;
  const uint32_t n = 1024;
  const size_t N = (size_t)n * n * n;
  float* d; uint64_t* o; unsigned long long* cs;
  CK(hipMalloc(&d, N * 4)); CK(hipMalloc(&o, N * 2 + 4096)); CK(hipMalloc(&cs, 8));
  hipLaunchKernelGGL(fill_f1, dim3((unsigned)(N / 256)), dim3(256), 0, 0, d, n);
  Geometry g{};
  for (int a = 0; a < 4; a++) { g.n[a] = a < 3 ? n : 1; g.f[a] = 0; g.nb[a] = a < 3 ? n / 4 : 1; }
  g.s[0] = 1; g.s[1] = n; g.s[2] = (int64_t)n * n; g.s[3] = 0;
  g.nblocks = (uint64_t)(n / 4) * (n / 4) * (n / 4);
  for (int a = 0; a < 3; a++) g.dv[a] = make_fastdiv(g.nb[a]);
  CodecParams cp{1024, 1024, 64, -1074};
  const uint32_t sw = 16, sdw = slot_dwords_for(1024) | 1u;
  const uint32_t magic_w = (uint32_t)((0x100000000ull + sw - 1) / sw), magic_c = (uint32_t)((0x100000000ull + sw / 2 - 1) / (sw / 2));
  const size_t lds = 4 * 64 * sdw * 4;
  dim3 grid((unsigned)(g.nblocks / 256)), block(256);
  const double gb = N * 6.0 / 1e9;
  auto full = [&] {
    hipLaunchKernelGGL((encode3_aligned<float, true, false>), grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_w, magic_c, 0u,
                       (Partial*)nullptr);
  };
  if (argc > 1 && std::string(argv[1]) == "pmc") {  // a few launches for counter passes
    for (int r = 0; r < 5; r++) full();
    CK(hipDeviceSynchronize());
    return 0;
  }
  for (int r = 0; r < 3; r++) {
    float t = time_it(full, 20);
    printf("%-10s full      %.4f ms  %.0f GB/s(alg)  frac %.4f\n", tag, t, gb / t * 1e3, gb / t * 1e3 / 8000.0);
  }
  CK(hipMemset(cs, 0, 8));
  full();
  hipLaunchKernelGGL(checksum, dim3(1024), dim3(256), 0, 0, o, (uint64_t)(N / 4), cs);
  unsigned long long h = 0;
  CK(hipMemcpy(&h, cs, 8, hipMemcpyDeviceToHost));
  printf("%-10s checksum %016llx\n", tag, h);
  for (int r = 0; r < 0; r++) {
    float t;
    t = time_it([&] { hipLaunchKernelGGL(enc_gate<1>, grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c); }, 20);
    printf("%-10s gate1     %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
    t = time_it([&] { hipLaunchKernelGGL(enc_gate<2>, grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c); }, 20);
    printf("%-10s gate2     %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
    t = time_it([&] { hipLaunchKernelGGL(enc_gate<4>, grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c); }, 20);
    printf("%-10s gate4     %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
    t = time_it([&] { hipLaunchKernelGGL((enc_gate<4, false, true>), grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c); }, 20);
    printf("%-10s nosync-w0 %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
    t = time_it([&] { hipLaunchKernelGGL((enc_gate<4, true, false>), grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c); }, 20);
    printf("%-10s sync-lazy %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
    t = time_it([&] { hipLaunchKernelGGL((enc_gate<4, false, false>), grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c); }, 20);
    printf("%-10s nosync-lazy %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
  }
  for (int r = 0; r < 2; r++) {
    float t;
    t = time_it([&] { hipLaunchKernelGGL((encode3_aligned<float, true, false, 2>), dim3((unsigned)(g.nblocks / 128)), dim3(128),
                                         2 * 64 * sdw * 4, 0, d, g, cp, o, sw, sdw, magic_w, magic_c, 0u, (Partial*)nullptr); }, 20);
    printf("%-10s wpg2      %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
    t = time_it([&] { hipLaunchKernelGGL((encode3_aligned<float, true, false, 1>), dim3((unsigned)(g.nblocks / 64)), dim3(64),
                                         1 * 64 * sdw * 4, 0, d, g, cp, o, sw, sdw, magic_w, magic_c, 0u, (Partial*)nullptr); }, 20);
    printf("%-10s wpg1      %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
    t = time_it([&] { hipLaunchKernelGGL((encode3_aligned<float, true, false, 8>), dim3((unsigned)(g.nblocks / 512)), dim3(512),
                                         8 * 64 * sdw * 4, 0, d, g, cp, o, sw, sdw, magic_w, magic_c, 0u, (Partial*)nullptr); }, 20);
    printf("%-10s wpg8      %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
  }
  for (int r = 0; r < 2; r++) {
    float t;
#define PF(D, P) \
    t = time_it([&] { hipLaunchKernelGGL((enc_pf<D, P>), grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c); }, 20); \
    printf("%-10s pf%-4d p%d %.4f ms  frac %.4f\n", tag, D, P, t, gb / t * 1e3 / 8000.0);
    PF(0, 0) PF(0, 1)
#define MO(M) \
    t = time_it([&] { hipLaunchKernelGGL((enc_pf<0, 0, 4, false, M>), grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c); }, 20); \
    printf("%-10s morph%d %.4f ms  frac %.4f\n", tag, M, t, gb / t * 1e3 / 8000.0);
    MO(1) MO(2) MO(3) MO(4) MO(7)
    t = time_it([&] { hipLaunchKernelGGL((enc_pf<0, 1, 4, true>), grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c); }, 20);
    printf("%-10s pf0 p1 guard %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
    t = time_it([&] { hipLaunchKernelGGL((enc_pf<0, 1, 2>), dim3((unsigned)(g.nblocks / 128)), dim3(128), 2 * 64 * sdw * 4, 0, d, g, cp, o, sw, sdw, magic_c); }, 20);
    printf("%-10s pf0 p1 wpg2 %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
    t = time_it([&] { hipLaunchKernelGGL((enc_pf<0, 2, 2>), dim3((unsigned)(g.nblocks / 128)), dim3(128), 2 * 64 * sdw * 4, 0, d, g, cp, o, sw, sdw, magic_c); }, 20);
    printf("%-10s pf0 p2 wpg2 %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
    t = time_it([&] { hipLaunchKernelGGL((enc_pf<0, 3, 4>), grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c); }, 20);
    printf("%-10s pf0 p3      %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
  }
  {
    CK(hipMemset(cs, 0, 8));
    hipLaunchKernelGGL((enc_pf<0, 1, 2>), dim3((unsigned)(g.nblocks / 128)), dim3(128), 2 * 64 * sdw * 4, 0, d, g, cp, o, sw, sdw, magic_c);
    hipLaunchKernelGGL(checksum, dim3(1024), dim3(256), 0, 0, o, (uint64_t)(N / 4), cs);
    unsigned long long h2 = 0;
    CK(hipMemcpy(&h2, cs, 8, hipMemcpyDeviceToHost));
    printf("%-10s pf checksum %016llx\n", tag, h2);
  }
  {
    const uint32_t rows = slot_dwords_for(1024);  // 35
    const size_t ilds = 4 * 64 * rows * 4;
    for (int r = 0; r < 2; r++) {
      float t;
      t = time_it([&] { hipLaunchKernelGGL((enc_ilv<0, 1>), grid, block, ilds, 0, d, g, cp, o, rows); }, 20);
      printf("%-10s ilv own p0 %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
      t = time_it([&] { hipLaunchKernelGGL((enc_ilv<1, 1>), grid, block, ilds, 0, d, g, cp, o, rows); }, 20);
      printf("%-10s ilv own p1 %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
      t = time_it([&] { hipLaunchKernelGGL((enc_ilv<1, 0>), grid, block, ilds, 0, d, g, cp, o, rows); }, 20);
      printf("%-10s ilv coa p1 %.4f ms  frac %.4f\n", tag, t, gb / t * 1e3 / 8000.0);
    }
    for (int own = 0; own < 2; own++) {
      CK(hipMemset(cs, 0, 8));
      if (own) hipLaunchKernelGGL((enc_ilv<1, 1>), grid, block, ilds, 0, d, g, cp, o, rows);
      else hipLaunchKernelGGL((enc_ilv<1, 0>), grid, block, ilds, 0, d, g, cp, o, rows);
      hipLaunchKernelGGL(checksum, dim3(1024), dim3(256), 0, 0, o, (uint64_t)(N / 4), cs);
      unsigned long long h2 = 0;
      CK(hipMemcpy(&h2, cs, 8, hipMemcpyDeviceToHost));
      printf("%-10s ilv%d checksum %016llx\n", tag, own, h2);
    }
  }
  for (int G : {1, 2}) {
    CK(hipMemset(cs, 0, 8));
    if (G == 1) hipLaunchKernelGGL(enc_gate<1>, grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c);
    else hipLaunchKernelGGL(enc_gate<2>, grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c);
    hipLaunchKernelGGL(checksum, dim3(1024), dim3(256), 0, 0, o, (uint64_t)(N / 4), cs);
    unsigned long long h2 = 0;
    CK(hipMemcpy(&h2, cs, 8, hipMemcpyDeviceToHost));
    printf("%-10s gate%d checksum %016llx\n", tag, G, h2);
  }
  if (stages) {
    float t;
    t = time_it([&] { hipLaunchKernelGGL(enc_stage<1>, grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c); }, 20);
    printf("%-10s load+copy %.4f ms\n", tag, t);
    t = time_it([&] { hipLaunchKernelGGL(enc_stage<2>, grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c); }, 20);
    printf("%-10s no-coder  %.4f ms\n", tag, t);
    t = time_it([&] { hipLaunchKernelGGL(enc_stage<3>, grid, block, lds, 0, d, g, cp, o, sw, sdw, magic_c); }, 20);
    printf("%-10s light-coder %.4f ms\n", tag, t);
  }
  return 0;
}
