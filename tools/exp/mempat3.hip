// Experiment harness (not product code), round 4 (mempat3: occupancy and burst-length sweep): why the C2 encoder's block
// access pattern (1.13 ms) is slower than a linear stream of the same bytes
// (1.02 ms).  1024^3 f32 field read once, 2 GiB written, no coding.
//   lin     linear float4 stream: lane reads two float4, writes one (2:1)
//   lin16   burst shape of the encoder on linear addresses: a wave reads 16 KB
//           contiguous as 16 float4 per lane (1 KB per instruction), writes
//           8 KB contiguous (8 float4 per lane)
//   blk     the encoder's mapping (lane = 4x4x4 block, 16 float4 row loads,
//           128 B out per block through an LDS slot, 16-byte coalesced stores)
//   blkpad  blk on a field whose z-plane pitch is padded by 4 KB (is the 4 MiB
//           power-of-two plane stride the cost?)
//   blkyz   blk with the 16 loads issued y-outer, z-inner
//   blkdma  blk with the rows landed in LDS by global_load_lds_dwordx4 (16 KB
//           tile per wave, slots alias the tile after the reads)
//   blk8    blk with 8 loads, wait, 8 loads (two halves)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u4 ld(const u4* p) { return __builtin_nontemporal_load(p); }
__device__ __forceinline__ void st(u4* p, u4 v) { __builtin_nontemporal_store(v, p); }

constexpr uint32_t N = 1024;
constexpr uint32_t SDW = 37;

__global__ __launch_bounds__(256) void lin(const u4* __restrict__ in, u4* __restrict__ out, uint64_t n4)
{
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4 / 2) return;
  const u4 a = ld(in + 2 * i), b = ld(in + 2 * i + 1);
  st(out + i, a ^ b);
}

__global__ __launch_bounds__(256) void lin16(const u4* __restrict__ in, u4* __restrict__ out)
{
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t w = (uint64_t)blockIdx.x * 4 + wv;
  const u4* src = in + w * 1024;
  u4 v[16];
#pragma unroll
  for (int i = 0; i < 16; i++) v[i] = ld(src + i * 64 + lane);
  u4* dst = out + w * 512;
#pragma unroll
  for (int i = 0; i < 8; i++) st(dst + i * 64 + lane, v[i] ^ v[i + 8]);
}

template <int K>
__global__ __launch_bounds__(256) void linK(const u4* __restrict__ in, u4* __restrict__ out)
{
  extern __shared__ uint32_t lds[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t w = (uint64_t)blockIdx.x * 4 + wv;
  const u4* src = in + w * 64 * K;
  u4 v[K];
#pragma unroll
  for (int i = 0; i < K; i++) v[i] = ld(src + i * 64 + lane);
  u4* dst = out + w * 32 * K;
#pragma unroll
  for (int i = 0; i < K / 2; i++) st(dst + i * 64 + lane, v[i] ^ v[i + K / 2]);
  if (lane == 1000) lds[0] = 0;
}

template <int ORDER>
__device__ __forceinline__ void gather(u4 (&v)[16], const u4* in, uint64_t b, uint64_t pitch4)
{
  const uint32_t bx = (uint32_t)(b % (N / 4)), by = (uint32_t)((b / (N / 4)) % (N / 4)), bz = (uint32_t)(b / ((N / 4) * (N / 4)));
  const u4* o = in + (uint64_t)(4 * bz) * pitch4 + ((uint64_t)(4 * by) * N + 4 * bx) / 4;
  if (ORDER == 0) {
#pragma unroll
    for (int z = 0; z < 4; z++)
#pragma unroll
      for (int y = 0; y < 4; y++) v[4 * z + y] = ld(o + (uint64_t)z * pitch4 + (uint64_t)y * N / 4);
  } else {
#pragma unroll
    for (int y = 0; y < 4; y++)
#pragma unroll
      for (int z = 0; z < 4; z++) v[4 * z + y] = ld(o + (uint64_t)z * pitch4 + (uint64_t)y * N / 4);
  }
}

__device__ __forceinline__ void slot_out(const u4 (&v)[16], uint32_t* ws, int lane, u4* dst)
{
  uint32_t* slot = ws + lane * SDW;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const u4 r = v[i] ^ v[i + 8];
    slot[4 * i] = r.x; slot[4 * i + 1] = r.y; slot[4 * i + 2] = r.z; slot[4 * i + 3] = r.w;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int c = lane; c < 512; c += 64) {
    const uint32_t l = c >> 3;
    const uint32_t* s = ws + l * SDW + 4 * (c & 7);
    st(dst + c, u4{s[0], s[1], s[2], s[3]});
  }
}

template <int ORDER>
__global__ __launch_bounds__(256) void blk(const u4* __restrict__ in, u4* __restrict__ out, uint64_t pitch4)
{
  extern __shared__ uint32_t lds[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t first = ((uint64_t)blockIdx.x * 4 + wv) * 64, b = first + lane;
  u4 v[16];
  gather<ORDER>(v, in, b, pitch4);
  slot_out(v, lds + (size_t)wv * 64 * SDW, lane, out + first * 8);
}

__global__ __launch_bounds__(256) void blk8(const u4* __restrict__ in, u4* __restrict__ out, uint64_t pitch4)
{
  extern __shared__ uint32_t lds[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t first = ((uint64_t)blockIdx.x * 4 + wv) * 64, b = first + lane;
  const uint32_t bx = (uint32_t)(b % (N / 4)), by = (uint32_t)((b / (N / 4)) % (N / 4)), bz = (uint32_t)(b / ((N / 4) * (N / 4)));
  const u4* o = in + (uint64_t)(4 * bz) * pitch4 + ((uint64_t)(4 * by) * N + 4 * bx) / 4;
  u4 v[16];
#pragma unroll
  for (int z = 0; z < 2; z++)
#pragma unroll
    for (int y = 0; y < 4; y++) v[4 * z + y] = ld(o + (uint64_t)z * pitch4 + (uint64_t)y * N / 4);
  u4 a[4];
#pragma unroll
  for (int i = 0; i < 4; i++) a[i] = v[i] ^ v[i + 4];
  __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
  for (int z = 2; z < 4; z++)
#pragma unroll
    for (int y = 0; y < 4; y++) v[4 * z + y] = ld(o + (uint64_t)z * pitch4 + (uint64_t)y * N / 4);
#pragma unroll
  for (int i = 0; i < 4; i++) v[i] = a[i];
  slot_out(v, lds + (size_t)wv * 64 * SDW, lane, out + first * 8);
}

// rows landed in LDS by the DMA path: piece i (row (y,z) = (i%4, i/4)) of
// the wave's 64 blocks is 1 KB, lane l's 16 bytes at l*16
__global__ __launch_bounds__(256) void blkdma(const u4* __restrict__ in, u4* __restrict__ out, uint64_t pitch4)
{
  extern __shared__ uint32_t lds[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t first = ((uint64_t)blockIdx.x * 4 + wv) * 64, b = first + lane;
  const uint32_t bx = (uint32_t)(b % (N / 4)), by = (uint32_t)((b / (N / 4)) % (N / 4)), bz = (uint32_t)(b / ((N / 4) * (N / 4)));
  const u4* o = in + (uint64_t)(4 * bz) * pitch4 + ((uint64_t)(4 * by) * N + 4 * bx) / 4;
  uint32_t* tile = lds + (size_t)wv * 4096;  // 16 KB per wave
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int z = i >> 2, y = i & 3;
    __builtin_amdgcn_global_load_lds((const void*)(o + (uint64_t)z * pitch4 + (uint64_t)y * N / 4),
                                     (__attribute__((address_space(3))) void*)(tile + i * 256), 16, 0, 2);
  }
  __builtin_amdgcn_s_waitcnt(0x0f70);  // vmcnt(0)
  __builtin_amdgcn_wave_barrier();
  u4 v[16];
#pragma unroll
  for (int i = 0; i < 16; i++) v[i] = *reinterpret_cast<const u4*>(tile + i * 256 + lane * 4);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  slot_out(v, tile, lane, out + first * 8);
}

template <typename K>
static float time_it(K launch, int reps)
{
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int r = 0; r < 10; r++) launch();
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
  setvbuf(stdout, nullptr, _IOLBF, 0);
  const uint64_t nf = (uint64_t)N * N * N, n4 = nf / 4, nb = nf / 64;
  const uint64_t pitch = (uint64_t)N * N;
  u4 *in, *out;
  CK(hipMalloc(&in, nf * 4)); CK(hipMalloc(&out, nf * 2));
  CK(hipMemset(in, 1, nf * 4));
  const double gb = nf * 6.0 / 1e9;
  auto rep = [&](const char* name, int occ, float t) { printf("%-7s occ %d  %.4f ms  %.0f GB/s  frac %.3f\n", name, occ, t, gb / t * 1e3, gb / t * 1e3 / 8000.0); };
  for (int r = 0; r < 200; r++) hipLaunchKernelGGL(lin, dim3((unsigned)(n4 / 2 / 256)), dim3(256), 0, 0, in, out, n4);
  CK(hipDeviceSynchronize());
  const unsigned g = (unsigned)(nb / 256);
  // LDS bytes that allow `occ` 256-thread workgroups per CU (160 KiB)
  auto ldsfor = [](int occ) -> size_t { return occ >= 8 ? 0 : (size_t)(163840 / occ) & ~(size_t)1023; };
  for (int r = 0; r < 2; r++) {
    rep("lin", 0, time_it([&] { hipLaunchKernelGGL(lin, dim3((unsigned)(n4 / 2 / 256)), dim3(256), 0, 0, in, out, n4); }, 20));
    rep("lin2", 8, time_it([&] { hipLaunchKernelGGL(linK<2>, dim3(g * 8), dim3(256), 0, 0, in, out); }, 20));
    rep("lin4", 8, time_it([&] { hipLaunchKernelGGL(linK<4>, dim3(g * 4), dim3(256), 0, 0, in, out); }, 20));
    rep("lin8", 8, time_it([&] { hipLaunchKernelGGL(linK<8>, dim3(g * 2), dim3(256), 0, 0, in, out); }, 20));
    for (int occ : {8, 6, 4, 3, 2})
      rep("lin16", occ, time_it([&] { hipLaunchKernelGGL(linK<16>, dim3(g), dim3(256), ldsfor(occ), 0, in, out); }, 20));
    for (int occ : {4, 3, 2})
      rep("lin8", occ, time_it([&] { hipLaunchKernelGGL(linK<8>, dim3(g * 2), dim3(256), ldsfor(occ), 0, in, out); }, 20));
    for (int occ : {4, 3, 2})
      rep("blk", occ, time_it([&] { hipLaunchKernelGGL(blk<0>, dim3(g), dim3(256), ldsfor(occ), 0, in, out, pitch / 4); }, 20));
    for (int occ : {2, 1})
      rep("blkdma", occ, time_it([&] { hipLaunchKernelGGL(blkdma, dim3(g), dim3(256), ldsfor(occ), 0, in, out, pitch / 4); }, 20));
  }
  return 0;
}
