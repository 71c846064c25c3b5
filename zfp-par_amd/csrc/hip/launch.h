// Launchers of the tuned f32/f64 kernels, one translation unit per scalar type
// and block dimensionality (zfp_k3f.hip, zfp_k3d.hip, zfp_k4f.hip,
// zfp_k4d.hip) plus the index scan (zfp_scan.hip), so the instantiations
// compile in parallel and the host shim (zfp_hip.hip) instantiates none.
// Every launcher enumerates the template arguments it dispatches on, so a
// kernel the host can select is always instantiated next to its launch.
#pragma once

#include "kernels4.h"
#include "scan.h"

namespace zfp_amd {

struct Launch {
  dim3 grid, block;
  size_t lds;
  hipStream_t stream;
};

// 3D (kernels3.h).  hi: f64 kernels that code planes 32..63 only (maxprec <=
// 32); shrt: decode3 with short staging slots (f64 hi, lossy only).
#define ZFP_DECL3(S)                                                                                                 \
  void launch_encode3_aligned(const Launch& l, bool vec, const S* f, const Geometry& g, const CodecParams& cp,       \
                              uint64_t* out, uint32_t sw, uint32_t sdw, uint32_t magic_w, uint32_t magic_c,          \
                              uint32_t r0, Partial* parts);                                                         \
  void launch_encode3_general(const Launch& l, bool vec, bool rev, bool hi, const S* f, const Geometry& g,           \
                              const CodecParams& cp, const GeneralArgs& a);                                         \
  void launch_decode3(const Launch& l, bool vec, bool rev, bool hi, bool shrt, S* f, const Geometry& g,              \
                      const CodecParams& cp, const DecodeArgs& a);
ZFP_DECL3(float)
ZFP_DECL3(double)
#undef ZFP_DECL3

// 4D (kernels4.h).  half: exchange areas shared by quad pairs.
#define ZFP_DECL4(S)                                                                                                 \
  void launch_encode4(const Launch& l, bool vec, bool rev, bool half, const S* f, const Geometry& g,                 \
                      const CodecParams& cp, const GeneralArgs& a);                                                 \
  void launch_encode4_patch(const Launch& l, bool vec, bool rev, const S* f, const Geometry& g,                     \
                            const CodecParams& cp, uint64_t* out, const OvfEntry* list, uint32_t n, uint32_t swp);  \
  void launch_decode4(const Launch& l, bool vec, bool rev, S* f, const Geometry& g, const CodecParams& cp,           \
                      const DecodeArgs& a);
ZFP_DECL4(float)
ZFP_DECL4(double)
#undef ZFP_DECL4

// index scan pass (scan.h) for zfp_type `type` (1 int32, 2 int64, 3 float,
// 4 double), dims 1..4
void launch_scan_pass(int type, int dims, bool rev, dim3 grid, hipStream_t stream, const ScanArgs& a);
void launch_scan_window(int type, int dims, bool rev, hipStream_t stream, const ScanArgs& a, int32_t* win);

}  // namespace zfp_amd
