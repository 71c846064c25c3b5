// Experiment (not product code): the fixed-rate f32 coder of codec_dev.h
// (code_planes_fr32 / code_planes_fru / expand_event) with lane-interleaved
// LDS slots -- dword j of lane l at wave_base + 256 j + 4 l -- so the 64 lanes'
// ds_or writes of a plane always hit 64 different banks whatever their bit
// positions (the product's per-lane slots, an odd 35 dwords apart, collide
// whenever two lanes of a half-wave sit at positions whose dword indices
// differ by a multiple of 32 mod the stride: 368 conflict cycles per wave).
// The position is kept as Q = -(bit position within the lane's slot): the row
// of a write starting at bit p = -Q is ceil(p/32) - 1 = ~(Q >> 5), its byte
// address lanebase | (~(Q | 31)) << 3 (one v_bitop3 + one v_lshl_or, as the
// product's), and the funnel shift Q mod 32.
#pragma once
#include "codec_dev.h"

namespace ilv {
using namespace zfp_amd;

constexpr uint32_t kRow = 256;  // bytes between a lane's consecutive dwords

__device__ __forceinline__ uint32_t row_addr(uint32_t lanebase, int32_t Q)
{
  // ~(Q | 31) as one v_bitop3 (truth table 0x03 = ~(a | b)), then one v_lshl_or
  return (__builtin_amdgcn_bitop3_b32((uint32_t)Q, 31u, 0u, 0x03) << 3) | lanebase;
}

__device__ __forceinline__ void w32(uint32_t lanebase, int32_t Q, uint32_t v)
{
  const uint32_t a = row_addr(lanebase, Q);
  ZFP_LDS_OR(lds_at(a), __builtin_amdgcn_alignbit(v, 0u, (uint32_t)Q));
  ZFP_LDS_OR(lds_at(a + kRow), __builtin_amdgcn_alignbit(0u, v, (uint32_t)Q));
}

__device__ __forceinline__ void w64(uint32_t lanebase, int32_t Q, uint32_t v0, uint32_t v1)
{
  const uint32_t a = row_addr(lanebase, Q);
  ZFP_LDS_OR(lds_at(a), __builtin_amdgcn_alignbit(v0, 0u, (uint32_t)Q));
  ZFP_LDS_OR(lds_at(a + kRow), __builtin_amdgcn_alignbit(v1, v0, (uint32_t)Q));
  ZFP_LDS_OR(lds_at(a + 2 * kRow), __builtin_amdgcn_alignbit(0u, v1, (uint32_t)Q));
}

// clamped writes (rows <= jmax) of the rare extension branch, at bit p >= 1
struct Slot {
  uint32_t lanebase;
  uint32_t jmax;
  __device__ __forceinline__ void row_or(uint32_t j, uint32_t v) { ZFP_LDS_OR(lds_at(lanebase + j * kRow), v); }
  __device__ __forceinline__ void put64_clamped(uint32_t p, uint32_t v0, uint32_t v1)
  {
    uint32_t j = (p + 31u) >> 5;
    j = j < jmax - 1 ? j : jmax - 1;
    const uint32_t t = 0u - p;
    row_or(j - 1, __builtin_amdgcn_alignbit(v0, 0u, t));
    row_or(j, __builtin_amdgcn_alignbit(v1, v0, t));
    row_or(j + 1, __builtin_amdgcn_alignbit(0u, v1, t));
  }
  __device__ __forceinline__ void put32_clamped(uint32_t p, uint32_t v)
  {
    uint32_t j = (p + 31u) >> 5;
    j = j < jmax ? j : jmax;
    const uint32_t t = 0u - p;
    row_or(j - 1, __builtin_amdgcn_alignbit(v, 0u, t));
    row_or(j, __builtin_amdgcn_alignbit(0u, v, t));
  }
};

__device__ __forceinline__ void expand_event(Slot& s, const uint32_t* lut, const ExtEvent& e)
{
  const uint32_t h = e.hb & 63u, impl = (e.hb >> 6) & 1u;
  const uint64_t xs = ((uint64_t)e.xh << 32) | e.xl;
  uint32_t D = 16u + (uint32_t)__popc(e.xl & 0xffffu);
#pragma unroll
  for (int j = 1; j < 4; j++) {
    const bool unit = h >= 16u * j;
    if (__any(unit)) {
      const uint32_t u = (uint32_t)(xs >> (16 * j)) & 0xffffu;
      const uint32_t cu = (uint32_t)__popc(u);
      uint32_t dj = dbl16(lut, u);
      if (h < 16u * (j + 1))
        dj -= (2u + impl) << ((h - 16u * j + cu - 1u) & 31u);
      if (unit) {
        if (j == 1)
          s.put64_clamped(e.gp + D, (dj << 1) | (e.hb >> 7), dj >> 31);
        else
          s.put32_clamped(e.gp + 1u + D, dj);
      }
      D += 16u + cu;
    }
  }
}

__device__ __forceinline__ void code_planes_fru(Slot& os, const uint32_t* lut, int32_t Q, int32_t Qlim, uint32_t n,
                                                int kstart, const uint32_t (&Pl)[32], const uint32_t (&Ph)[32])
{
  const uint32_t tdbl = lds_off(lut), tlead = tdbl + 1024u;
  uint32_t Sh = n > 32u ? ~0u >> ((0u - n) & 31u) : 0u;
#pragma unroll
  for (int k = 31; k >= 0; k--) {
    if (k > kstart)
      continue;
    if (k < ZFP_FR_EXIT_PLANES && __builtin_amdgcn_ballot_w64(Q > Qlim) == 0)
      break;
    const uint32_t pl = Pl[k], ph = Ph[k];
    const bool hi = n >= 32u;
    const uint32_t Nh = ph & ~Sh;
    const uint32_t t = Nh >> (n & 31u);
    const uint32_t x0 = hi ? t : __builtin_amdgcn_alignbit(Nh, pl, n);
    const uint32_t x1 = hi ? 0u : t;
    const uint32_t l0 = *lds_at(tlead + byte0_x4(x0));
    const uint32_t l1 = *lds_at(tdbl + byte1_x4(x0));
    const uint32_t bl = 31u - (uint32_t)__clz((int)((x0 << 1) | 1u));
    const uint32_t e1 = (uint32_t)__popc(x0) + bl;
    const uint32_t impl = Nh >> 31;
    uint32_t n1 = n + bl;
    const uint32_t d = (l1 << (l0 & 31u)) | (l0 >> 5);
    uint32_t g = ubfe(d, 0u, e1 - impl);
    uint32_t L = e1 - impl + 1u - (n1 >> 6);
    const bool ext = x0 > 0xfffeu || x1 != 0u;
    const int32_t Qg = Q - (int32_t)n;
    if (__builtin_amdgcn_ballot_w64(ext) != 0) {
      uint32_t hb = 0;
      if (ext) {
        const uint32_t hx = x1 ? 63u - (uint32_t)__clz((int)x1) : 31u - (uint32_t)__clz((int)x0);
        const uint32_t c = (uint32_t)__popc(x0) + (uint32_t)__popc(x1);
        n1 = n + hx + 1u;
        const uint32_t im = n1 >> 6;
        L = hx + c + 2u - 2u * im;
        g = hx < 16u ? d & ~(im << 31) : d;
        hb = hx | (im << 6) | ((x0 & 0xffffu) == 0xffffu ? 0x80u : 0u);
      }
      expand_event(os, lut, ExtEvent{(uint32_t)(-Qg), x0, x1, hb});
    }
    w64(os.lanebase, Q, hi ? pl : ubfe(pl, 0u, n), ph & Sh);
    w32(os.lanebase, Qg, g);
    const int32_t Qn = Qg - (int32_t)L;
    Q = Qn > Qlim ? Qn : Qlim;
    n = n1;
    Sh = n > 32u ? ~0u >> ((0u - n) & 31u) : 0u;
  }
}

// lanebase: byte address of the lane's dword 0 (wave base 256-aligned + 4 lane)
__device__ __forceinline__ void code_planes_fr32(uint32_t lanebase, uint32_t jmax, const uint32_t* lut, uint32_t pos,
                                                 uint32_t lim, const uint32_t (&Pl)[32], const uint32_t (&Ph)[32])
{
  Slot os{lanebase, jmax};
  const uint32_t tdbl = lds_off(lut), tlead = tdbl + 1024u;
  int32_t Q = -(int32_t)pos;
  const int32_t Qlim = -(int32_t)lim;
  uint32_t n = 0;
  bool m32 = true;
  int ksw = 0;
#pragma unroll
  for (int k = 31; k >= 0; k--) {
    if (m32) {
      if (__builtin_amdgcn_ballot_w64(Ph[k] != 0u || n > 31u) != 0) {
        m32 = false;
        ksw = k;
      } else {
        const uint32_t pl = Pl[k];
        const uint32_t xs = pl >> n;
        const uint32_t l0 = *lds_at(tlead + byte0_x4(xs));
        const uint32_t l1 = *lds_at(tdbl + byte1_x4(xs));
        const uint32_t bl = 32u - (uint32_t)__clz((int)xs);
        const uint32_t e1 = (uint32_t)__popc(xs) + bl;
        if (k < 31)  // n == 0 at the first plane: no verbatim bits
          w32(lanebase, Q, ubfe(pl, 0u, n));
        const int32_t Qg = Q - (int32_t)n;
        const uint32_t d = (l1 << (l0 & 31u)) | (l0 >> 5);
        uint32_t g = d - (1u << (e1 & 31u));
        const bool ext = xs > 0xfffeu;
        if (__builtin_amdgcn_ballot_w64(ext) != 0) {
          const uint32_t h = 31u - (uint32_t)__clz((int)xs);
          const uint32_t gp = (uint32_t)(-Qg);
          const uint32_t g32 = (xs & 0xffffu) == 0xffffu ? 1u : 0u;
          g = ext ? d : g;
          expand_event(os, lut, ExtEvent{gp, xs, 0u, ext ? h | (g32 << 7) : 0u});
        }
        w32(lanebase, Qg, g);
        const int32_t Qn = Qg - (int32_t)e1 - 1;
        Q = Qn > Qlim ? Qn : Qlim;
        n += bl;
      }
    }
  }
  if (!m32)
    code_planes_fru(os, lut, Q, Qlim, n, ksw, Pl, Ph);
}

// encode_block3_fixed (block3.h) for f32 with the interleaved coder
template <typename Reload>
__device__ __forceinline__ void encode_block_fixed_f32(uint32_t lanebase, uint32_t jmax, const uint32_t* lut,
                                                       float (&v)[64], const CodecParams& cp, Reload&& reload)
{
  int32_t q[64];
  uint32_t mp;
  const int emax = lossy_emax_cast(q, v, cp, mp, reload);
  const uint32_t e = mp ? (uint32_t)(emax + 127) : 0u;
  if (e)
    ZFP_LDS_OR(lds_at(lanebase), 2 * e + 1);
  ZFP_PHASE_BARRIER();
  xform<3, false, false>(q);
  ZFP_PHASE_BARRIER();
  uint32_t Pl[32], Ph[32];
  planes_from_coeffs(Pl, Ph, q);
  ZFP_PHASE_BARRIER();
  pin_registers(Pl);
  pin_registers(Ph);
  code_planes_fr32(lanebase, jmax, lut, e ? 9u : cp.maxbits, cp.maxbits, Pl, Ph);
}

}  // namespace ilv
