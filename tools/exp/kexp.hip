// Experiment harness (not product code): variants of the fixed-rate 3D encode
// kernel with parts removed, timed with HIP events
// on a device-resident 1024^3 f32 field.  Build: make -C tools/exp; run: tools/exp/kexp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kernels3.h"
using namespace zfp_amd;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// MODE 0: full; 1: no coder (planes folded into one word); 2: coder on synthetic planes; 3: load+max only;
// 4: load + cast + lift (no planes, no coder)
#ifndef KEXP_WPS
#define KEXP_WPS 3
#endif
template <int MODE>
__global__ __launch_bounds__(256, KEXP_WPS) void enc_var(const float* __restrict__ data, Geometry g, CodecParams cp,
                                                 uint64_t* __restrict__ out, uint32_t sw, uint32_t swp, uint32_t magic)
{
  __shared__ uint32_t lut[256];
  extern __shared__ uint64_t lds[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint64_t* wslot = lds + (size_t)wv * 64 * swp;
  encode_prologue(lut, wslot, 64 * swp);
  const uint64_t w = (uint64_t)blockIdx.x * kWavesPerGroup + wv;
  const uint64_t first = w * 64;
  const uint64_t b = first + lane;
  if (b < g.nblocks) {
    OrSlot os{wslot + (size_t)lane * swp, 2 * swp - 1};
    if (MODE == 2) {
      uint32_t Pl[32], Ph[32];
      uint32_t h = (uint32_t)b * 2654435761u;
#pragma unroll
      for (int k = 0; k < 32; k++) {
        h ^= h << 13; h ^= h >> 17; h ^= h << 5;
        uint32_t keep = k > 20 ? 0x0000000fu : (k > 12 ? 0x0000ffffu : ~0u);
        Pl[k] = h & keep;
        Ph[k] = (h * 7u) & (k > 12 ? 0u : ~0u);
      }
      code_planes<32, false>(os, lut, 9, cp.maxbits, 32, Pl, Ph);
    } else {
      float v[64];
      BlockPos p = block_pos(g, b, 3);
      gather3<float, true>(v, data, g, p);
      if (MODE == 0) {
        encode_block3<float, false, true>(os, lut, v, cp, [&](float (&r)[64]) { gather3<float, true>(r, data, g, p); });
      } else if (MODE == 4) {
        int32_t q[64];
        uint32_t mp;
        lossy_emax_cast(q, v, cp, mp, [&](float (&r)[64]) { gather3<float, true>(r, data, g, p); });
        xform<3, false, false>(q);
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < 64; k++) acc ^= (uint32_t)q[k] + k;
        os.head(acc);
      } else if (MODE == 1) {
        int32_t q[64];
        uint32_t mp;
        lossy_emax_cast(q, v, cp, mp, [&](float (&r)[64]) { gather3<float, true>(r, data, g, p); });
        xform<3, false, false>(q);
        uint32_t Pl[32], Ph[32];
        planes_from_coeffs(Pl, Ph, q);
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < 32; k++) acc ^= Pl[k] + 3u * Ph[k] + k;
        os.head(acc);
      } else {
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < 64; i++) acc = max(acc, __float_as_uint(v[i]) & 0x7fffffffu);
        os.head(acc);
      }
    }
  }
  if (first >= g.nblocks) return;
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  const uint32_t total = 64 * sw;
  uint64_t* dst = out + first * sw;
  for (uint32_t i = 2 * lane; i < total; i += 128) {
    const uint32_t l = div_magic(i, magic);
    const uint64_t* src = wslot + (size_t)l * swp + (i - l * sw);
    ulonglong2 q; q.x = src[0]; q.y = src[1];
    *reinterpret_cast<ulonglong2*>(dst + i) = q;
  }
}


// persistent + software-pipelined full encoder (prefetch of the next batch's
// field into registers once the planes are built)
#ifndef KEXP_PIPE_WPS
#define KEXP_PIPE_WPS 3
#endif
__global__ __launch_bounds__(256, KEXP_PIPE_WPS) void enc_pipe(const float* __restrict__ data, Geometry g, CodecParams cp,
                                                    uint64_t* __restrict__ out, uint32_t sw, uint32_t swp, uint32_t magic)
{
  __shared__ uint32_t lut[256];
  extern __shared__ uint64_t lds[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint64_t* wslot = lds + (size_t)wv * 64 * swp;
  lut[threadIdx.x] = dbl_entry(threadIdx.x);
  __syncthreads();
  const uint64_t nw = (g.nblocks + 63) / 64;
  const uint64_t step = (uint64_t)gridDim.x * kWavesPerGroup;
  uint64_t w = (uint64_t)blockIdx.x * kWavesPerGroup + wv;
  if (w >= nw) return;
  uint64_t* slot = wslot + (size_t)lane * swp;
  float v[64];
  gather3<float, true>(v, data, g, block_pos(g, w * 64 + lane, 3));
  for (;;) {
    for (uint32_t i = 0; i + 1 < swp; i += 2)
      *reinterpret_cast<ulonglong2*>(slot + i) = make_ulonglong2(0, 0);
    slot[swp - 1] = 0;
    const uint64_t wn = w + step;
    const uint64_t b = w * 64 + lane;
    if (b < g.nblocks) {
      const BlockPos p = block_pos(g, b, 3);
      OrSlot os{slot, 2 * swp - 1};
      encode_block3_fixed(os, lut, v, cp, [&](float (&r)[64]) { gather3<float, true>(r, data, g, p); },
                          [&] {
                            if (wn < nw)
                              gather3<float, true>(v, data, g, block_pos(g, wn * 64 + lane, 3));
                          });
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t total = 64 * sw;
    uint64_t* dst = out + w * 64 * sw;
    for (uint32_t i = 2 * lane; i < total; i += 128) {
      const uint32_t l = div_magic(i, magic);
      const uint64_t* src = wslot + (size_t)l * swp + (i - l * sw);
      ulonglong2 q; q.x = src[0]; q.y = src[1];
      *reinterpret_cast<ulonglong2*>(dst + i) = q;
    }
    __builtin_amdgcn_wave_barrier();
    w = wn;
    if (w >= nw) break;
  }
}


// persistent (one batch at a time, no prefetch) with an optional start stagger
// so the load phases of the waves sharing a SIMD fall at different times
template <int STAGGER>
__global__ __launch_bounds__(256, 4) void enc_persist(const float* __restrict__ data, Geometry g, CodecParams cp,
                                                    uint64_t* __restrict__ out, uint32_t sw, uint32_t swp, uint32_t magic)
{
  __shared__ uint32_t lut[256];
  extern __shared__ uint64_t lds[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint64_t* wslot = lds + (size_t)wv * 64 * swp;
  lut[threadIdx.x] = dbl_entry(threadIdx.x);
  __syncthreads();
  const uint64_t nw = (g.nblocks + 63) / 64;
  const uint64_t step = (uint64_t)gridDim.x * kWavesPerGroup;
  uint64_t w = (uint64_t)blockIdx.x * kWavesPerGroup + wv;
  if (STAGGER) {
    const uint32_t h = (blockIdx.x * 2654435761u) >> 29;  // 0..7
    for (uint32_t i = 0; i < h * STAGGER; i++)
      __builtin_amdgcn_s_sleep(127);
  }
  uint64_t* slot = wslot + (size_t)lane * swp;
  for (; w < nw; w += step) {
    for (uint32_t i = 0; i + 1 < swp; i += 2)
      *reinterpret_cast<ulonglong2*>(slot + i) = make_ulonglong2(0, 0);
    slot[swp - 1] = 0;
    const uint64_t b = w * 64 + lane;
    if (b < g.nblocks) {
      float v[64];
      const BlockPos p = block_pos(g, b, 3);
      gather3<float, true>(v, data, g, p);
      OrSlot os{slot, 2 * swp - 1};
      encode_block3_fixed(os, lut, v, cp, [&](float (&r)[64]) { gather3<float, true>(r, data, g, p); }, [] {});
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t total = 64 * sw;
    uint64_t* dst = out + w * 64 * sw;
    for (uint32_t i = 2 * lane; i < total; i += 128) {
      const uint32_t l = div_magic(i, magic);
      const uint64_t* src = wslot + (size_t)l * swp + (i - l * sw);
      ulonglong2 q; q.x = src[0]; q.y = src[1];
      *reinterpret_cast<ulonglong2*>(dst + i) = q;
    }
    __builtin_amdgcn_wave_barrier();
  }
}


// persistent, prefetching the first two z-slabs (8 float4 = 32 VGPRs) of the
// next batch while the current one is coded; 96 + 32 VGPRs keeps 4 waves/SIMD
__global__ __launch_bounds__(256, 4) void enc_half(const float* __restrict__ data, Geometry g, CodecParams cp,
                                                  uint64_t* __restrict__ out, uint32_t sw, uint32_t swp, uint32_t magic)
{
  __shared__ uint32_t lut[256];
  extern __shared__ uint64_t lds[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint64_t* wslot = lds + (size_t)wv * 64 * swp;
  lut[threadIdx.x] = dbl_entry(threadIdx.x);
  __syncthreads();
  const uint64_t nw = (g.nblocks + 63) / 64;
  const uint64_t step = (uint64_t)gridDim.x * kWavesPerGroup;
  uint64_t w = (uint64_t)blockIdx.x * kWavesPerGroup + wv;
  uint64_t* slot = wslot + (size_t)lane * swp;
  const int64_t sy = g.s[1], sz = g.s[2];
  float4 pre[8];
  if (w < nw) {
    const float* o = data + block_pos(g, w * 64 + lane, 3).off;
#pragma unroll
    for (int k = 0; k < 2; k++)
#pragma unroll
      for (int j = 0; j < 4; j++) pre[4 * k + j] = *reinterpret_cast<const float4*>(o + j * sy + k * sz);
  }
  for (; w < nw; w += step) {
    for (uint32_t i = 0; i + 1 < swp; i += 2)
      *reinterpret_cast<ulonglong2*>(slot + i) = make_ulonglong2(0, 0);
    slot[swp - 1] = 0;
    const uint64_t b = w * 64 + lane;
    const uint64_t wn = w + step;
    float v[64];
    const BlockPos p = block_pos(g, b, 3);
    {
      const float* o = data + p.off;
#pragma unroll
      for (int k = 2; k < 4; k++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
          float4 q = *reinterpret_cast<const float4*>(o + j * sy + k * sz);
          v[16 * k + 4 * j] = q.x; v[16 * k + 4 * j + 1] = q.y; v[16 * k + 4 * j + 2] = q.z; v[16 * k + 4 * j + 3] = q.w;
        }
#pragma unroll
      for (int k = 0; k < 2; k++)
#pragma unroll
        for (int j = 0; j < 4; j++) {
          float4 q = pre[4 * k + j];
          v[16 * k + 4 * j] = q.x; v[16 * k + 4 * j + 1] = q.y; v[16 * k + 4 * j + 2] = q.z; v[16 * k + 4 * j + 3] = q.w;
        }
    }
    OrSlot os{slot, 2 * swp - 1};
    encode_block3_fixed(os, lut, v, cp, [&](float (&r)[64]) { gather3<float, true>(r, data, g, p); },
                        [&] {
                          if (wn < nw) {
                            const float* o = data + block_pos(g, wn * 64 + lane, 3).off;
#pragma unroll
                            for (int k = 0; k < 2; k++)
#pragma unroll
                              for (int j = 0; j < 4; j++) pre[4 * k + j] = *reinterpret_cast<const float4*>(o + j * sy + k * sz);
                          }
                        });
    __builtin_amdgcn_wave_barrier();
    const uint32_t total = 64 * sw;
    uint64_t* dst = out + w * 64 * sw;
    for (uint32_t i = 2 * lane; i < total; i += 128) {
      const uint32_t l = div_magic(i, magic);
      const uint64_t* src = wslot + (size_t)l * swp + (i - l * sw);
      ulonglong2 q; q.x = src[0]; q.y = src[1];
      *reinterpret_cast<ulonglong2*>(dst + i) = q;
    }
    __builtin_amdgcn_wave_barrier();
  }
}

template <typename K>
static float time_it(K launch, int reps)
{
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  launch();
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
  const bool quick = argc > 1;
  const uint64_t n = 1024;
  const size_t N = n * n * n;
  float* d; uint64_t* o;
  CK(hipMalloc(&d, N * 4)); CK(hipMalloc(&o, N * 2 + 4096));
  {
    std::vector<float> h(n * n);
    for (uint64_t z = 0; z < n; z++) {
      for (uint64_t y = 0; y < n; y++)
        for (uint64_t x = 0; x < n; x++)
          h[y * n + x] = (float)(sin(0.05 * x) * cos(0.03 * y) + 0.5 * sin(0.02 * z + 0.01 * x * y / n));
      CK(hipMemcpy(d + z * n * n, h.data(), n * n * 4, hipMemcpyHostToDevice));
    }
  }
  Geometry g{};
  for (int a = 0; a < 4; a++) { g.n[a] = a < 3 ? n : 1; g.f[a] = 0; g.nb[a] = a < 3 ? n / 4 : 1; }
  g.s[0] = 1; g.s[1] = n; g.s[2] = n * n; g.s[3] = 0;
  g.nblocks = (n / 4) * (n / 4) * (n / 4);
  for (int a = 0; a < 3; a++) g.dv[a] = make_fastdiv(g.nb[a]);
  CodecParams cp{1024, 1024, 64, -1074};
  const uint32_t sw = 16, swp = 19, magic = (uint32_t)((0x100000000ull + sw - 1) / sw);
  const size_t lds = 4 * 64 * swp * 8;
  dim3 grid((unsigned)(g.nblocks / 256)), block(256);
  const double gb = N * 6.0 / 1e9;
  float t;
  t = time_it([&] { hipLaunchKernelGGL(enc_var<0>, grid, block, lds, 0, d, g, cp, o, sw, swp, magic); }, 10);
  printf("full        %.3f ms  %.0f GB/s(alg)\n", t, gb / t * 1e3);
  if (quick) {
    int per_cu = 0, cus = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)enc_persist<0>, 256, lds));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    dim3 pg((unsigned)(per_cu * cus));
    for (int r = 0; r < 3; r++) {
      t = time_it([&] { hipLaunchKernelGGL(enc_var<0>, grid, block, lds, 0, d, g, cp, o, sw, swp, magic); }, 20);
      printf("one-shot      %.3f ms\n", t);
      t = time_it([&] { hipLaunchKernelGGL(enc_persist<0>, pg, block, lds, 0, d, g, cp, o, sw, swp, magic); }, 20);
      printf("persist       %.3f ms (%d/CU)\n", t, per_cu);
      t = time_it([&] { hipLaunchKernelGGL(enc_half, pg, block, lds, 0, d, g, cp, o, sw, swp, magic); }, 20);
      printf("persist+half  %.3f ms\n", t);
      t = time_it([&] { hipLaunchKernelGGL(enc_persist<2>, pg, block, lds, 0, d, g, cp, o, sw, swp, magic); }, 20);
      printf("persist+stag2 %.3f ms\n", t);
    }
    std::vector<uint64_t> a(N / 4), b2(N / 4);
    hipLaunchKernelGGL(enc_var<0>, grid, block, lds, 0, d, g, cp, o, sw, swp, magic);
    CK(hipMemcpy(a.data(), o, N * 2, hipMemcpyDeviceToHost));
    hipLaunchKernelGGL(enc_half, pg, block, lds, 0, d, g, cp, o, sw, swp, magic);
    CK(hipMemcpy(b2.data(), o, N * 2, hipMemcpyDeviceToHost));
    printf("persist stream identical: %s\n", a == b2 ? "yes" : "NO");
    return 0;
  }
  t = time_it([&] { hipLaunchKernelGGL(enc_var<1>, grid, block, lds, 0, d, g, cp, o, sw, swp, magic); }, 10);
  printf("no-coder    %.3f ms\n", t);
  t = time_it([&] { hipLaunchKernelGGL(enc_var<2>, grid, block, lds, 0, d, g, cp, o, sw, swp, magic); }, 10);
  printf("coder-only  %.3f ms\n", t);
  t = time_it([&] { hipLaunchKernelGGL(enc_var<3>, grid, block, lds, 0, d, g, cp, o, sw, swp, magic); }, 10);
  printf("load-only   %.3f ms\n", t);
  t = time_it([&] { hipLaunchKernelGGL(enc_var<4>, grid, block, lds, 0, d, g, cp, o, sw, swp, magic); }, 10);
  printf("cast+lift   %.3f ms\n", t);
  {
    int per_cu = 0, cus = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)enc_pipe, 256, lds));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    for (int mult = 1; mult <= 2; mult++) {
      dim3 pg((unsigned)(per_cu * cus * mult));
      t = time_it([&] { hipLaunchKernelGGL(enc_pipe, pg, block, lds, 0, d, g, cp, o, sw, swp, magic); }, 10);
      printf("pipelined   %.3f ms  (%d groups/CU x %d CUs x %d)  %.0f GB/s(alg)\n", t, per_cu, cus, mult, gb / t * 1e3);
    }
    // check: same stream as the one-shot kernel
    std::vector<uint64_t> a(N / 4), b2(N / 4);
    hipLaunchKernelGGL(enc_var<0>, grid, block, lds, 0, d, g, cp, o, sw, swp, magic);
    CK(hipMemcpy(a.data(), o, N * 2, hipMemcpyDeviceToHost));
    hipLaunchKernelGGL(enc_pipe, dim3(per_cu * cus), block, lds, 0, d, g, cp, o, sw, swp, magic);
    CK(hipMemcpy(b2.data(), o, N * 2, hipMemcpyDeviceToHost));
    printf("pipelined stream identical: %s\n", a == b2 ? "yes" : "NO");
  }
  return 0;
}
