// Host (single-lane) stand-in for the HIP device API, so the device-side codec
// headers compile with g++ for logic tests (tests/emu).  A "wave" is one lane:
// __any(x) == x (or true, see emu_any_all) and readfirstlane is the identity.
#pragma once
#include <cstdint>
#include <cstring>
#include <type_traits>
#define __device__
#define __host__
#define __global__
#define __constant__
#define __shared__ static
#define __forceinline__ inline
#define __launch_bounds__(...)
// With emu_any_all set, every wave-level test passes as if some other lane
// needed the branch: per-lane predication inside such branches is exercised.
inline bool emu_any_all = false;
static inline int __any(int x) { return x != 0 || emu_any_all; }
static inline uint64_t __builtin_amdgcn_ballot_w64(bool x) { return (x || emu_any_all) ? 1u : 0u; }
// llvm.amdgcn.icmp (unsigned): the wave mask of one compare (predicates EQ 32,
// NE 33, UGT 34, UGE 35, ULT 36, ULE 37), one lane here
static inline uint64_t __builtin_amdgcn_uicmp(uint32_t a, uint32_t b, int pred)
{
  const bool c = pred == 32 ? a == b : pred == 33 ? a != b : pred == 34 ? a > b : pred == 35 ? a >= b
               : pred == 36 ? a < b : a <= b;
  return (c || emu_any_all) ? 1u : 0u;
}
static inline int __popc(uint32_t x) { return __builtin_popcount(x); }
static inline int __popcll(uint64_t x) { return __builtin_popcountll(x); }
static inline int __clzll(long long x) { return x ? __builtin_clzll((uint64_t)x) : 64; }
static inline int __clz(int x) { return x ? __builtin_clz((uint32_t)x) : 32; }
static inline uint32_t __float_as_uint(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
static inline float __uint_as_float(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
static inline long long __double_as_longlong(double d) { long long u; std::memcpy(&u, &d, 8); return u; }
static inline double __longlong_as_double(long long u) { double d; std::memcpy(&d, &u, 8); return d; }
static inline int __builtin_amdgcn_readfirstlane(int x) { return x; }
// v_alignbit_b32: ({a,b} >> (c & 31)) low 32 bits
static inline uint32_t __builtin_amdgcn_alignbit(uint32_t a, uint32_t b, uint32_t c)
{
  return (uint32_t)((((uint64_t)a << 32) | b) >> (c & 31));
}
// v_bitop3_b32: result bit = ttbl bit (s0 << 2 | s1 << 1 | s2) of the inputs' bits
static inline uint32_t __builtin_amdgcn_bitop3_b32(uint32_t s0, uint32_t s1, uint32_t s2, uint32_t ttbl)
{
  uint32_t r = 0;
  for (int i = 0; i < 32; i++) {
    uint32_t idx = (((s0 >> i) & 1u) << 2) | (((s1 >> i) & 1u) << 1) | ((s2 >> i) & 1u);
    r |= ((ttbl >> idx) & 1u) << i;
  }
  return r;
}
// v_perm_b32: bytes 0-3 from src1, 4-7 from src0
static inline uint32_t __builtin_amdgcn_perm(uint32_t s0, uint32_t s1, uint32_t sel)
{
  uint64_t v = ((uint64_t)s0 << 32) | s1;
  uint32_t r = 0;
  for (int i = 0; i < 4; i++) {
    uint32_t b = (sel >> (8 * i)) & 0xff;
    r |= (uint32_t)((v >> (8 * (b & 7))) & 0xff) << (8 * i);
  }
  return r;
}
#define __ATOMIC_RELAXED_STUB 0
#define __HIP_MEMORY_SCOPE_WAVEFRONT 1
// atomic: the 4-lane emulation (quad_emu.cpp) ORs into one slot from four threads
template <typename T> static inline T __hip_atomic_fetch_or(T* p, T v, int, int) { return __atomic_fetch_or(p, v, __ATOMIC_RELAXED); }
static inline uint32_t __umulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
struct float4 { float x, y, z, w; };
struct double2 { double x, y; };
static inline float4 make_float4(float a, float b, float c, float d) { return float4{a, b, c, d}; }
static inline double2 make_double2(double a, double b) { return double2{a, b}; }
#include <cmath>
using std::fabs;
#include <math.h>
#include <algorithm>
using std::max;
using std::min;
// plain read-modify-write: the scan emulation runs lanes one after another
static inline uint32_t atomicAdd(uint32_t* p, uint32_t v) { uint32_t o = *p; *p = o + v; return o; }
// kernel built-ins, so headers that define kernels compile (the emulations
// call the per-lane device functions, not the kernels)
// (quad_emu.cpp brings its own per-thread threadIdx and barrier)
#ifdef EMU_KERNEL_BUILTINS
struct emu_dim3 { uint32_t x = 0, y = 0, z = 0; };
inline emu_dim3 threadIdx, blockIdx, blockDim;
static inline void __syncthreads() {}
#endif
