// Experiment harness (not product code): what the C2 encoder's memory pattern
// alone costs on MI355X.  1024^3 f32 field (4 GiB) read once, 2 GiB written,
// no coding:
//   lin      linear float4 stream: lane reads two float4, writes one (2:1)
//   blk      the encoder's mapping: lane = one 4x4x4 block, a wave = 64 blocks
//            along x, 16 float4 row loads per lane; 128 B per block written
//            through an LDS slot as 16-byte coalesced stores (as encode3_aligned)
//   blkd     blk with each lane storing its own 128 B directly (8 strided
//            uint4 stores, no LDS)
//   blk2     blk with two blocks per lane in sequence (half the waves)
// Loads/stores non-temporal unless built with -DPLAIN.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

typedef uint32_t u4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u4 ld(const u4* p)
{
#ifdef PLAIN
  return *p;
#else
  return __builtin_nontemporal_load(p);
#endif
}
__device__ __forceinline__ void st(u4* p, u4 v)
{
#ifdef PLAIN
  *p = v;
#else
  __builtin_nontemporal_store(v, p);
#endif
}

constexpr uint32_t N = 1024;

__global__ __launch_bounds__(256) void lin(const u4* __restrict__ in, u4* __restrict__ out, uint64_t n4)
{
  const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4 / 2) return;
  const u4 a = ld(in + 2 * i), b = ld(in + 2 * i + 1);
  st(out + i, a ^ b);
}

// block b (raster: x fastest over 256 blocks per row): rows (y, z) of 16 B
__device__ __forceinline__ void gather(u4 (&v)[16], const u4* in, uint64_t b)
{
  const uint32_t bx = (uint32_t)(b % (N / 4)), by = (uint32_t)((b / (N / 4)) % (N / 4)), bz = (uint32_t)(b / ((N / 4) * (N / 4)));
  const u4* o = in + ((uint64_t)(4 * bz) * N * N + (uint64_t)(4 * by) * N + 4 * bx) / 4;
#pragma unroll
  for (int z = 0; z < 4; z++)
#pragma unroll
    for (int y = 0; y < 4; y++)
      v[4 * z + y] = ld(o + ((uint64_t)z * N * N + (uint64_t)y * N) / 4);
}

template <int LDS>
__global__ __launch_bounds__(256) void blk(const u4* __restrict__ in, u4* __restrict__ out)
{
  extern __shared__ uint32_t lds[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t first = ((uint64_t)blockIdx.x * 4 + wv) * 64, b = first + lane;
  u4 v[16];
  gather(v, in, b);
  u4 r[8];
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = v[i] ^ v[i + 8];
  if (LDS) {
    constexpr uint32_t sdw = 37;  // odd slot stride (dwords), as the encoder
    uint32_t* slot = lds + (size_t)wv * 64 * sdw + lane * sdw;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      slot[4 * i] = r[i].x; slot[4 * i + 1] = r[i].y; slot[4 * i + 2] = r[i].z; slot[4 * i + 3] = r[i].w;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t* ws = lds + (size_t)wv * 64 * sdw;
    u4* dst = out + first * 8;
#pragma unroll
    for (int c = lane; c < 512; c += 64) {
      const uint32_t l = c >> 3;
      const uint32_t* s = ws + l * sdw + 4 * (c & 7);
      st(dst + c, u4{s[0], s[1], s[2], s[3]});
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; i++) st(out + b * 8 + i, r[i]);
  }
}

__global__ __launch_bounds__(256) void blk2(const u4* __restrict__ in, u4* __restrict__ out)
{
  extern __shared__ uint32_t lds[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int h = 0; h < 2; h++) {
    const uint64_t first = (((uint64_t)blockIdx.x * 2 + h) * 4 + wv) * 64, b = first + lane;
    u4 v[16];
    gather(v, in, b);
    constexpr uint32_t sdw = 37;
    uint32_t* slot = lds + (size_t)wv * 64 * sdw + lane * sdw;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const u4 r = v[i] ^ v[i + 8];
      slot[4 * i] = r.x; slot[4 * i + 1] = r.y; slot[4 * i + 2] = r.z; slot[4 * i + 3] = r.w;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint32_t* ws = lds + (size_t)wv * 64 * sdw;
    u4* dst = out + first * 8;
#pragma unroll
    for (int c = lane; c < 512; c += 64) {
      const uint32_t l = c >> 3;
      const uint32_t* s = ws + l * sdw + 4 * (c & 7);
      st(dst + c, u4{s[0], s[1], s[2], s[3]});
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
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
  u4 *in, *out;
  CK(hipMalloc(&in, nf * 4)); CK(hipMalloc(&out, nf * 2));
  CK(hipMemset(in, 1, nf * 4));
  const double gb = nf * 6.0 / 1e9;
  const size_t lds = 4 * 64 * 37 * 4;
  auto rep = [&](const char* name, float t) { printf("%-6s %.4f ms  %.0f GB/s  frac %.3f\n", name, t, gb / t * 1e3, gb / t * 1e3 / 8000.0); };
  for (int r = 0; r < 2; r++) {
    rep("lin", time_it([&] { hipLaunchKernelGGL(lin, dim3((unsigned)(n4 / 2 / 256)), dim3(256), 0, 0, in, out, n4); }, 20));
    rep("blk", time_it([&] { hipLaunchKernelGGL(blk<1>, dim3((unsigned)(nb / 256)), dim3(256), lds, 0, in, out); }, 20));
    rep("blkd", time_it([&] { hipLaunchKernelGGL(blk<0>, dim3((unsigned)(nb / 256)), dim3(256), 0, 0, in, out); }, 20));
    rep("blk2", time_it([&] { hipLaunchKernelGGL(blk2, dim3((unsigned)(nb / 512)), dim3(256), lds, 0, in, out); }, 20));
  }
  return 0;
}
