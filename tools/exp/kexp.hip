// Experiment harness (not product code): variants of the fixed-rate 3D encode
// kernel with parts removed, plus VALU/LDS micro-kernels, timed with HIP events
// on a device-resident 1024^3 f32 field.  Build: make -C tools/exp; run: tools/exp/kexp
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "kernels3.h"
using namespace zfp_amd;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// MODE 0: full; 1: no coder (planes folded into one word); 2: coder on synthetic planes; 3: load+max only
template <int MODE>
__global__ __launch_bounds__(256, 4) void enc_var(const float* __restrict__ data, Geometry g, CodecParams cp,
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
    OrSlot os{wslot + (size_t)lane * swp, sw};
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
      code_planes<32>(os, lut, 9, cp.maxbits, 32, Pl, Ph);
    } else {
      float v[64];
      BlockPos p = block_pos(g, b, 3);
      gather3<float, true>(v, data, g, p);
      if (MODE == 0) {
        encode_block3<float, false>(os, lut, v, cp, [&](float (&r)[64]) { gather3<float, true>(r, data, g, p); });
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
        os.put(0, acc, 32);
      } else {
        uint32_t acc = 0;
#pragma unroll
        for (int i = 0; i < 64; i++) acc = max(acc, __float_as_uint(v[i]) & 0x7fffffffu);
        os.put(0, acc, 32);
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

// Persistent waves: each wave loops over sets of 64 blocks; the next set's
// block is loaded into registers right after the current block's cast, so its
// loads are in flight during the transform and the coder.
template <int WPS>
__global__ __launch_bounds__(256, WPS) void enc_persist(const float* __restrict__ data, Geometry g, CodecParams cp,
                                                       uint64_t* __restrict__ out, uint32_t sw, uint32_t swp,
                                                       uint32_t magic, uint64_t nsets)
{
  __shared__ uint32_t lut[256];
  extern __shared__ uint64_t lds[];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  uint64_t* wslot = lds + (size_t)wv * 64 * swp;
  lut[threadIdx.x] = dbl_entry(threadIdx.x);
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * kWavesPerGroup;
  uint64_t set = (uint64_t)blockIdx.x * kWavesPerGroup + wv;
  float v[64];
  if (set < nsets) {
    BlockPos p = block_pos(g, set * 64 + lane, 3);
    gather3<float, true>(v, data, g, p);
  }
  for (; set < nsets; set += stride) {
    // zero the slots
    uint4* z = reinterpret_cast<uint4*>(wslot);
    for (uint32_t i = lane; i < 64 * swp / 2; i += 64) z[i] = make_uint4(0, 0, 0, 0);
    if (((64 * swp) & 1) && lane == 0) wslot[64 * swp - 1] = 0;
    const uint64_t b = set * 64 + lane;
    OrSlot os{wslot + (size_t)lane * swp, sw};
    BlockPos p = block_pos(g, b, 3);
    int32_t q[64];
    uint32_t mp;
    int emax = lossy_emax_cast(q, v, cp, mp, [&](float (&r)[64]) { gather3<float, true>(r, data, g, p); });
    // prefetch the next set's block (v is dead after the cast)
    const uint64_t nset = set + stride;
    if (nset < nsets) {
      BlockPos pn = block_pos(g, nset * 64 + lane, 3);
      gather3<float, true>(v, data, g, pn);
    }
    const uint32_t e = mp ? (uint32_t)(emax + 127) : 0u;
    if (e) {
      os.put(0, 2 * (uint64_t)e + 1, 9);
      xform<3, false, false>(q);
      encode_ints3(os, lut, q, 9, cp.maxbits, mp);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t total = 64 * sw;
    uint64_t* dst = out + set * 64 * sw;
    for (uint32_t i = 2 * lane; i < total; i += 128) {
      const uint32_t l = div_magic(i, magic);
      const uint64_t* src = wslot + (size_t)l * swp + (i - l * sw);
      ulonglong2 qq; qq.x = src[0]; qq.y = src[1];
      *reinterpret_cast<ulonglong2*>(dst + i) = qq;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// micro: N dependent-free chains of 64-bit shifts / 32-bit adds / ds_or
template <int OP>
__global__ __launch_bounds__(256) void micro(uint64_t* out, uint32_t iters)
{
  __shared__ uint64_t s[256 * 9];
  uint64_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;
  uint32_t sh = threadIdx.x & 31;
  s[threadIdx.x * 9] = 0;
  for (uint32_t i = 0; i < iters; i++) {
    if (OP == 0) {  // 64-bit shifts
      a0 = (a0 << sh) ^ i; a1 = (a1 << sh) ^ i; a2 = (a2 << sh) ^ i; a3 = (a3 << sh) ^ i;
      a4 = (a4 << sh) ^ i; a5 = (a5 << sh) ^ i; a6 = (a6 << sh) ^ i; a7 = (a7 << sh) ^ i;
    } else if (OP == 1) {  // 32-bit add+xor (same op count on 32-bit values)
      uint32_t* p = reinterpret_cast<uint32_t*>(&a0);
      a0 = (uint32_t)((uint32_t)a0 + sh) ^ i; a1 = (uint32_t)((uint32_t)a1 + sh) ^ i;
      a2 = (uint32_t)((uint32_t)a2 + sh) ^ i; a3 = (uint32_t)((uint32_t)a3 + sh) ^ i;
      a4 = (uint32_t)((uint32_t)a4 + sh) ^ i; a5 = (uint32_t)((uint32_t)a5 + sh) ^ i;
      a6 = (uint32_t)((uint32_t)a6 + sh) ^ i; a7 = (uint32_t)((uint32_t)a7 + sh) ^ i;
      (void)p;
    } else {  // ds_or_b64, 4 per iteration, per-lane slot (odd stride)
      uint64_t* q = s + threadIdx.x * 9;
      lds_or(q + (i & 7), a0 ^ i); lds_or(q + ((i + 1) & 7), a1 ^ i);
      lds_or(q + ((i + 2) & 7), a2 ^ i); lds_or(q + ((i + 3) & 7), a3 ^ i);
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ s[threadIdx.x * 9];
}

// shader clock during a VALU-bound loop: s_memtime (core clock) vs s_memrealtime (100 MHz)
__global__ __launch_bounds__(256) void clockprobe(uint64_t* out, uint32_t iters)
{
  uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7;
  for (uint32_t i = 0; i < iters; i++) {
    a0 = (a0 + i) ^ a1; a1 = (a1 + i) ^ a2; a2 = (a2 + i) ^ a3; a3 = (a3 + i) ^ a0;
  }
  uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) { out[2 * blockIdx.x] = t1 - t0; out[2 * blockIdx.x + 1] = r1 - r0; }
  if (a0 == 12345) out[0] = a0 + a1 + a2 + a3;
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

int main()
{
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
  CodecParams cp{1024, 1024, 64, -1074};
  const uint32_t sw = 16, swp = 17, magic = (uint32_t)((0x100000000ull + sw - 1) / sw);
  const size_t lds = 4 * 64 * swp * 8;
  dim3 grid((unsigned)(g.nblocks / 256)), block(256);
  const double gb = N * 6.0 / 1e9;
  float t;
  t = time_it([&] { hipLaunchKernelGGL(enc_var<0>, grid, block, lds, 0, d, g, cp, o, sw, swp, magic); }, 10);
  printf("full        %.3f ms  %.0f GB/s(alg)\n", t, gb / t * 1e3);
  t = time_it([&] { hipLaunchKernelGGL(enc_var<1>, grid, block, lds, 0, d, g, cp, o, sw, swp, magic); }, 10);
  printf("no-coder    %.3f ms\n", t);
  t = time_it([&] { hipLaunchKernelGGL(enc_var<2>, grid, block, lds, 0, d, g, cp, o, sw, swp, magic); }, 10);
  printf("coder-only  %.3f ms\n", t);
  {
    int ncu = 256;
    uint64_t nsets = g.nblocks / 64;
    for (int wps : {2, 3, 4}) {
      for (int gpc : {1, 2, 4}) {
        dim3 pg(ncu * gpc);
        if (wps == 2) t = time_it([&] { hipLaunchKernelGGL(enc_persist<2>, pg, block, lds, 0, d, g, cp, o, sw, swp, magic, nsets); }, 10);
        if (wps == 3) t = time_it([&] { hipLaunchKernelGGL(enc_persist<3>, pg, block, lds, 0, d, g, cp, o, sw, swp, magic, nsets); }, 10);
        if (wps == 4) t = time_it([&] { hipLaunchKernelGGL(enc_persist<4>, pg, block, lds, 0, d, g, cp, o, sw, swp, magic, nsets); }, 10);
        printf("persist wps=%d groups/CU=%d  %.3f ms  %.0f GB/s(alg)\n", wps, gpc, t, gb / t * 1e3);
      }
    }
  }
  t = time_it([&] { hipLaunchKernelGGL(enc_var<3>, grid, block, lds, 0, d, g, cp, o, sw, swp, magic); }, 10);
  printf("load-only   %.3f ms\n", t);
  const uint32_t it = 4096;
  dim3 mg(1024 * 4);
  t = time_it([&] { hipLaunchKernelGGL(micro<0>, mg, block, 0, 0, o, it); }, 5);
  printf("micro shl64: %.3f ms -> %.2f cycles/instr/SIMD\n", t, t * 1e-3 * 2.4e9 / (double)(mg.x * 4.0 / 1024 * it * 16));
  t = time_it([&] { hipLaunchKernelGGL(micro<1>, mg, block, 0, 0, o, it); }, 5);
  printf("micro add32: %.3f ms -> %.2f cycles/instr/SIMD\n", t, t * 1e-3 * 2.4e9 / (double)(mg.x * 4.0 / 1024 * it * 16));
  t = time_it([&] { hipLaunchKernelGGL(micro<2>, mg, block, 0, 0, o, it); }, 5);
  printf("micro ds_or: %.3f ms -> %.2f cycles/ds_or/CU\n", t, t * 1e-3 * 2.4e9 / (double)(mg.x * 4.0 / 256 * it * 4));
  {
    const unsigned nb = 4096;
    t = time_it([&] { hipLaunchKernelGGL(clockprobe, dim3(nb), block, 0, 0, o, 200000u); }, 1);
    std::vector<uint64_t> h(2 * nb);
    CK(hipMemcpy(h.data(), o, 16 * nb, hipMemcpyDeviceToHost));
    double sc = 0, sr = 0;
    for (unsigned i = 0; i < nb; i++) { sc += h[2 * i]; sr += h[2 * i + 1]; }
    printf("clockprobe: %.3f ms, core clock during VALU loop = %.0f MHz\n", t, sc / sr * 100.0);
  }
  return 0;
}
