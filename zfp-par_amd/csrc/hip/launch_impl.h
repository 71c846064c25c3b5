// Bodies of the launchers declared in launch.h; each zfp_k*.hip translation
// unit instantiates them for its scalar type.
#pragma once

#include "launch.h"

namespace zfp_amd {

template <typename S>
void enc3_aligned_impl(const Launch& l, bool vec, const S* f, const Geometry& g, const CodecParams& cp, uint64_t* out,
                       uint32_t sw, uint32_t sdw, uint32_t mw, uint32_t mc, uint32_t r0, Partial* parts)
{
  // whole workgroups, word-aligned start, even words per block (16-byte chunks)
  const bool full = r0 == 0 && (sw & 1) == 0 && sw >= 2 && g.nblocks % (64u * kWavesPerGroup) == 0 &&
                    (reinterpret_cast<uintptr_t>(out) & 15) == 0 && l.block.x == 64u * kWavesPerGroup;
  if (full && vec)
    hipLaunchKernelGGL((encode3_aligned_full<S, true>), l.grid, l.block, l.lds, l.stream, f, g, cp, out, sw, sdw, mc);
  else if (full)
    hipLaunchKernelGGL((encode3_aligned_full<S, false>), l.grid, l.block, l.lds, l.stream, f, g, cp, out, sw, sdw, mc);
  else if (vec)
    hipLaunchKernelGGL((encode3_aligned<S, true, false>), l.grid, l.block, l.lds, l.stream, f, g, cp, out, sw, sdw, mw,
                       mc, r0, parts);
  else
    hipLaunchKernelGGL((encode3_aligned<S, false, false>), l.grid, l.block, l.lds, l.stream, f, g, cp, out, sw, sdw, mw,
                       mc, r0, parts);
}

template <typename S, bool HI>
void enc3_general_impl(const Launch& l, bool vec, bool rev, const S* f, const Geometry& g, const CodecParams& cp,
                       const GeneralArgs& a)
{
  if (vec && rev)
    hipLaunchKernelGGL((encode3_general<S, true, true, HI>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
  else if (vec)
    hipLaunchKernelGGL((encode3_general<S, true, false, HI>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
  else if (rev)
    hipLaunchKernelGGL((encode3_general<S, false, true, HI>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
  else
    hipLaunchKernelGGL((encode3_general<S, false, false, HI>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
}

template <typename S, bool HI>
void dec3_impl(const Launch& l, bool vec, bool rev, bool shrt, S* f, const Geometry& g, const CodecParams& cp,
               const DecodeArgs& a)
{
  if constexpr (HI) {
    if (shrt && !rev) {  // short staging slots (the only short-slot decoder)
      if (vec)
        hipLaunchKernelGGL((decode3<S, true, false, true, 3, true>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
      else
        hipLaunchKernelGGL((decode3<S, false, false, true, 3, true>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
      return;
    }
  }
  if (vec && rev)
    hipLaunchKernelGGL((decode3<S, true, true, HI>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
  else if (vec)
    hipLaunchKernelGGL((decode3<S, true, false, HI>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
  else if (rev)
    hipLaunchKernelGGL((decode3<S, false, true, HI>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
  else
    hipLaunchKernelGGL((decode3<S, false, false, HI>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
}

template <typename S, bool HALF>
void enc4_impl(const Launch& l, bool vec, bool rev, const S* f, const Geometry& g, const CodecParams& cp,
               const GeneralArgs& a)
{
  if (vec && rev)
    hipLaunchKernelGGL((encode4<S, true, true, HALF>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
  else if (vec)
    hipLaunchKernelGGL((encode4<S, true, false, HALF>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
  else if (rev)
    hipLaunchKernelGGL((encode4<S, false, true, HALF>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
  else
    hipLaunchKernelGGL((encode4<S, false, false, HALF>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
}

template <typename S>
void enc4_patch_impl(const Launch& l, bool vec, bool rev, const S* f, const Geometry& g, const CodecParams& cp,
                     uint64_t* out, const OvfEntry* list, uint32_t n, uint32_t swp)
{
  if (vec && rev)
    hipLaunchKernelGGL((encode4_patch<S, true, true>), l.grid, l.block, l.lds, l.stream, f, g, cp, out, list, n, swp);
  else if (vec)
    hipLaunchKernelGGL((encode4_patch<S, true, false>), l.grid, l.block, l.lds, l.stream, f, g, cp, out, list, n, swp);
  else if (rev)
    hipLaunchKernelGGL((encode4_patch<S, false, true>), l.grid, l.block, l.lds, l.stream, f, g, cp, out, list, n, swp);
  else
    hipLaunchKernelGGL((encode4_patch<S, false, false>), l.grid, l.block, l.lds, l.stream, f, g, cp, out, list, n, swp);
}

// f32/f64 4D decoding always shares exchange areas between quad pairs
template <typename S>
void dec4_impl(const Launch& l, bool vec, bool rev, S* f, const Geometry& g, const CodecParams& cp, const DecodeArgs& a)
{
  if (vec && rev)
    hipLaunchKernelGGL((decode4<S, true, true, true>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
  else if (vec)
    hipLaunchKernelGGL((decode4<S, true, false, true>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
  else if (rev)
    hipLaunchKernelGGL((decode4<S, false, true, true>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
  else
    hipLaunchKernelGGL((decode4<S, false, false, true>), l.grid, l.block, l.lds, l.stream, f, g, cp, a);
}

// the launch.h overloads for one 3D scalar type (f64: hi selects the planes
// 32..63 kernels; f32 has none)
#define ZFP_DEFINE3(S)                                                                                               \
  void launch_encode3_aligned(const Launch& l, bool vec, const S* f, const Geometry& g, const CodecParams& cp,       \
                              uint64_t* out, uint32_t sw, uint32_t sdw, uint32_t magic_w, uint32_t magic_c,          \
                              uint32_t r0, Partial* parts)                                                          \
  {                                                                                                                  \
    enc3_aligned_impl<S>(l, vec, f, g, cp, out, sw, sdw, magic_w, magic_c, r0, parts);                              \
  }                                                                                                                  \
  void launch_encode3_general(const Launch& l, bool vec, bool rev, bool hi, const S* f, const Geometry& g,           \
                              const CodecParams& cp, const GeneralArgs& a)                                          \
  {                                                                                                                  \
    if (sizeof(S) == 8 && hi)                                                                                        \
      enc3_general_impl<S, sizeof(S) == 8>(l, vec, rev, f, g, cp, a);                                               \
    else                                                                                                             \
      enc3_general_impl<S, false>(l, vec, rev, f, g, cp, a);                                                         \
  }                                                                                                                  \
  void launch_decode3(const Launch& l, bool vec, bool rev, bool hi, bool shrt, S* f, const Geometry& g,              \
                      const CodecParams& cp, const DecodeArgs& a)                                                   \
  {                                                                                                                  \
    if (sizeof(S) == 8 && hi)                                                                                        \
      dec3_impl<S, sizeof(S) == 8>(l, vec, rev, shrt, f, g, cp, a);                                                 \
    else                                                                                                             \
      dec3_impl<S, false>(l, vec, rev, false, f, g, cp, a);                                                          \
  }

#define ZFP_DEFINE4(S)                                                                                               \
  void launch_encode4(const Launch& l, bool vec, bool rev, bool half, const S* f, const Geometry& g,                 \
                      const CodecParams& cp, const GeneralArgs& a)                                                  \
  {                                                                                                                  \
    if (half)                                                                                                        \
      enc4_impl<S, true>(l, vec, rev, f, g, cp, a);                                                                  \
    else                                                                                                             \
      enc4_impl<S, false>(l, vec, rev, f, g, cp, a);                                                                 \
  }                                                                                                                  \
  void launch_encode4_patch(const Launch& l, bool vec, bool rev, const S* f, const Geometry& g,                     \
                            const CodecParams& cp, uint64_t* out, const OvfEntry* list, uint32_t n, uint32_t swp)   \
  {                                                                                                                  \
    enc4_patch_impl<S>(l, vec, rev, f, g, cp, out, list, n, swp);                                                    \
  }                                                                                                                  \
  void launch_decode4(const Launch& l, bool vec, bool rev, S* f, const Geometry& g, const CodecParams& cp,           \
                      const DecodeArgs& a)                                                                          \
  {                                                                                                                  \
    dec4_impl<S>(l, vec, rev, f, g, cp, a);                                                                          \
  }

}  // namespace zfp_amd
