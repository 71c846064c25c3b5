// Experiment (not product code): sustained issue cost of single VALU instruction
// kinds on gfx950 with many waves per SIMD.  Each kernel runs ITERS x 16
// independent instructions of one kind per lane (8 register chains x 2).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int K>
__global__ __launch_bounds__(256) void vk(uint32_t* out, uint32_t iters)
{
  uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11, a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;
  uint32_t b0 = a0 ^ 1, b1 = a1 ^ 1, b2 = a2 ^ 1, b3 = a3 ^ 1, b4 = a4 ^ 1, b5 = a5 ^ 1, b6 = a6 ^ 1, b7 = a7 ^ 1;
  uint32_t s = threadIdx.x & 31;
  uint64_t m = __ballot(threadIdx.x & 1), m2 = 0;
  for (uint32_t i = 0; i < iters; i++) {
#define OP(r)                                                                                              \
    if (K == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##r) : "v"(s));                               \
    if (K == 1) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(*(uint64_t*)&a##r) : "v"(s));               \
    if (K == 2) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(a##r) : "v"(s), "v"(b##r));                \
    if (K == 3) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a##r) : "v"(b##r), "v"(s));               \
    if (K == 4) asm volatile("v_bcnt_u32_b32 %0, %0, %1" : "+v"(a##r) : "v"(b##r));                       \
    if (K == 5) asm volatile("v_ffbh_u32 %0, %0" : "+v"(a##r));                                           \
    if (K == 6) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(a##r) : "v"(b##r), "v"(s));           \
    if (K == 7) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a##r) : "v"(b##r), "v"(s));               \
    if (K == 8) asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(a##r));                                        \
    if (K == 9) asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(a##r) : "v"(s));                           \
    if (K == 10) asm volatile("v_mov_b32 %0, %1" : "=v"(a##r) : "v"(b##r));                               \
    if (K == 11) asm volatile("v_lshl_or_b32 %0, %0, %1, %2" : "+v"(a##r) : "v"(s), "v"(b##r));           \
    if (K == 12) asm volatile("v_bfe_u32 %0, %0, %1, %2" : "+v"(a##r) : "v"(s), "v"(b##r));               \
    if (K == 13) asm volatile("v_lshlrev_b32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "+v"(a##r) : "v"(s)); \
    if (K == 14) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a##r) : "v"(b##r));                  \
    if (K == 15) asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(a##r) : "v"(b##r), "v"(s));               \
    if (K == 16) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a##r) : "v"(b##r), "s"(m));        \
    if (K == 17) asm volatile("v_cmp_gt_u32 %1, %0, %2\n v_cndmask_b32_e64 %0, %0, %2, %1" : "+v"(a##r), "=s"(m2) : "v"(b##r)); \
    if (K == 18) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a##r) : "v"(b##r));                           \
    if (K == 19) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a##r) : "v"(b##r));                           \
    if (K == 20) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(a##r) : "v"(b##r));                           \
    if (K == 21) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a##r) : "v"(b##r));                           \
    if (K == 22) asm volatile("v_cmp_gt_u32 %1, %0, %2" : "+v"(a##r), "=s"(m2) : "v"(b##r));             \
    if (K == 23) asm volatile("v_lshrrev_b64 %0, %1, %0" : "+v"(*(uint64_t*)&a##r) : "v"(s));               \
    if (K == 24) asm volatile("v_ashrrev_i32 %0, %1, %0" : "+v"(a##r) : "v"(s));                          \
    if (K == 25) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(a##r) : "v"(b##r), "v"(s));               \
    if (K == 26) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a##r) : "v"(b##r));                           \
    if (K == 27) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(a##r) : "v"(b##r), "v"(s));               \
    if (K == 28) asm volatile("v_ashrrev_i64 %0, %1, %0" : "+v"(*(uint64_t*)&a##r) : "v"(s));               \
    if (K == 29) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a##r) : "v"(b##r) : "vcc"); \
    if (K == 30) asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(*(uint64_t*)&a##r) : "v"(*(uint64_t*)&b##r)); \
    if (K == 31) asm volatile("v_mov_b64 %0, %1" : "=v"(*(uint64_t*)&a##r) : "v"(*(uint64_t*)&b##r));
    REP8(OP)
    REP8(OP)
#undef OP
  }
  out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ (uint32_t)m2;
}

// LDS: ds_or_b64 / ds_read_b32 / ds_write_b64 streams at per-lane odd-stride slots
template <int K>
__global__ __launch_bounds__(256) void lk(uint32_t* out, uint32_t iters)
{
  __shared__ uint64_t s[256 * 17];
  uint64_t* q = s + threadIdx.x * 17;
  for (int i = 0; i < 17; i++) q[i] = 0;
  uint64_t v = threadIdx.x;
  uint32_t acc = 0;
  for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (K == 0) __hip_atomic_fetch_or(q + ((i + j) & 15), v ^ j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
      if (K == 1) acc += ((volatile uint32_t*)s)[(threadIdx.x * 37 + i * 8 + j) & 1023];
      if (K == 2) ((volatile uint64_t*)q)[(i + j) & 15] = v ^ j;
    }
  }
  out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)q[threadIdx.x & 15] + acc;
}

template <typename F>
static float time_it(F f)
{
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  f(); CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0)); for (int r = 0; r < 3; r++) f(); CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / 3;
}

int main()
{
  uint32_t* o; CK(hipMalloc(&o, 64 << 20));
  const char* names[] = {"add_u32", "lshlrev_b64", "bfi", "perm", "bcnt", "ffbh", "alignbit", "add3", "cvt_i32_f32",
                         "lshlrev_b32", "mov", "lshl_or", "bfe_u32", "lshl_sdwa", "cndmask", "max3_i32",
                         "cndmask_sgpr", "cmp+cndmask", "xor", "and", "sub", "min_u32", "cmp_gt", "lshrrev_b64", "ashrrev", "or3", "mul_f32", "xad", "ashrrev_i64", "add_co+addc(2)", "lshl_add_u64", "mov_b64"};
  const uint32_t it = 2048;
  for (int waves_per_simd : {4}) {
    dim3 g(256 * waves_per_simd), b(256);  // 4 waves per group -> 1 per SIMD
    double instr_per_simd = (double)waves_per_simd * it * 16;
    float t;
#define RUN(K) t = time_it([&] { hipLaunchKernelGGL(vk<K>, g, b, 0, 0, o, it); }); \
    printf("w/simd=%d %-12s %.3f ms  %.2f ns/instr/SIMD\n", waves_per_simd, names[K], t, t * 1e6 / instr_per_simd);
    RUN(0) RUN(1) RUN(2) RUN(3) RUN(4) RUN(5) RUN(6) RUN(7) RUN(8) RUN(9) RUN(10) RUN(11) RUN(12) RUN(13) RUN(14) RUN(15)
    RUN(16) RUN(17) RUN(18) RUN(19) RUN(20) RUN(21) RUN(22) RUN(23) RUN(24) RUN(25) RUN(26) RUN(27) RUN(28) RUN(29) RUN(30) RUN(31)
#undef RUN
    double lds_per_cu = (double)waves_per_simd * 4 * it * 8;
    t = time_it([&] { hipLaunchKernelGGL(lk<0>, g, b, 0, 0, o, it); });
    printf("w/simd=%d ds_or_b64    %.3f ms  %.2f ns/instr/CU\n", waves_per_simd, t, t * 1e6 / lds_per_cu);
    t = time_it([&] { hipLaunchKernelGGL(lk<1>, g, b, 0, 0, o, it); });
    printf("w/simd=%d ds_read_b32  %.3f ms  %.2f ns/instr/CU\n", waves_per_simd, t, t * 1e6 / lds_per_cu);
    t = time_it([&] { hipLaunchKernelGGL(lk<2>, g, b, 0, 0, o, it); });
    printf("w/simd=%d ds_write_b64 %.3f ms  %.2f ns/instr/CU\n", waves_per_simd, t, t * 1e6 / lds_per_cu);
  }
  return 0;
}
