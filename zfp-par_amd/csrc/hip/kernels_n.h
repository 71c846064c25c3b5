// Launchers of the generic per-lane kernels (1D/2D blocks of every type, 3D
// integer blocks: encode3_general / decode3 with D < 3 or an integer scalar),
// defined in zfp_hip_n32.hip (float, int32) and zfp_hip_n64.hip (double,
// int64) so that their instantiations compile in parallel with zfp_hip.hip.
#pragma once

#include "kernels3.h"
#include "kernels4.h"

namespace zfp_amd {

// type: zfp_type (1 int32, 2 int64, 3 float, 4 double); dims 1..3
void launch_encode_n(int type, int dims, bool rev, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                     const void* field, const Geometry& g, const CodecParams& cp, const GeneralArgs& a);
void launch_decode_n(int type, int dims, bool rev, hipStream_t stream, dim3 grid, dim3 block, size_t lds, void* field,
                     const Geometry& g, const CodecParams& cp, const DecodeArgs& a);
// the same per element width (4: float, int32; 8: double, int64)
void launch_encode_n32(int type, int dims, bool rev, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                       const void* field, const Geometry& g, const CodecParams& cp, const GeneralArgs& a);
void launch_decode_n32(int type, int dims, bool rev, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                       void* field, const Geometry& g, const CodecParams& cp, const DecodeArgs& a);
void launch_encode_n64(int type, int dims, bool rev, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                       const void* field, const Geometry& g, const CodecParams& cp, const GeneralArgs& a);
void launch_decode_n64(int type, int dims, bool rev, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                       void* field, const Geometry& g, const CodecParams& cp, const DecodeArgs& a);

// 4D integer fields (encode4 / decode4 with an integer scalar)
void launch_encode4_int(int type, bool rev, bool vec, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                        const void* field, const Geometry& g, const CodecParams& cp, const GeneralArgs& a);
void launch_decode4_int(int type, bool rev, bool vec, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                        void* field, const Geometry& g, const CodecParams& cp, const DecodeArgs& a);

void launch_encode4_int64(bool rev, bool vec, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                          const void* field, const Geometry& g, const CodecParams& cp, const GeneralArgs& a);
void launch_decode4_int64(bool rev, bool vec, hipStream_t stream, dim3 grid, dim3 block, size_t lds, void* field,
                          const Geometry& g, const CodecParams& cp, const DecodeArgs& a);

inline void launch_encode_n(int type, int dims, bool rev, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                            const void* field, const Geometry& g, const CodecParams& cp, const GeneralArgs& a)
{
  if (type == 1 || type == 3)
    launch_encode_n32(type, dims, rev, stream, grid, block, lds, field, g, cp, a);
  else
    launch_encode_n64(type, dims, rev, stream, grid, block, lds, field, g, cp, a);
}

inline void launch_decode_n(int type, int dims, bool rev, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                            void* field, const Geometry& g, const CodecParams& cp, const DecodeArgs& a)
{
  if (type == 1 || type == 3)
    launch_decode_n32(type, dims, rev, stream, grid, block, lds, field, g, cp, a);
  else
    launch_decode_n64(type, dims, rev, stream, grid, block, lds, field, g, cp, a);
}

// body of zfp_hip_n32.hip / zfp_hip_n64.hip: kernels for the scalar types
// A (integer) and B (float) of one width
template <typename A, typename B>
struct GenericKernels {
  template <typename S, int D>
  static void enc(bool rev, hipStream_t st, dim3 grid, dim3 block, size_t lds, const void* f, const Geometry& g,
                  const CodecParams& cp, const GeneralArgs& a)
  {
    if (rev)
      hipLaunchKernelGGL((encode3_general<S, false, true, false, D>), grid, block, lds, st, (const S*)f, g, cp, a);
    else
      hipLaunchKernelGGL((encode3_general<S, false, false, false, D>), grid, block, lds, st, (const S*)f, g, cp, a);
  }
  template <typename S, int D>
  static void dec(bool rev, hipStream_t st, dim3 grid, dim3 block, size_t lds, void* f, const Geometry& g,
                  const CodecParams& cp, const DecodeArgs& a)
  {
    if (rev)
      hipLaunchKernelGGL((decode3<S, false, true, false, D>), grid, block, lds, st, (S*)f, g, cp, a);
    else
      hipLaunchKernelGGL((decode3<S, false, false, false, D>), grid, block, lds, st, (S*)f, g, cp, a);
  }
  static void encode4i(bool rev, bool vec, hipStream_t st, dim3 grid, dim3 block, size_t lds, const void* f,
                       const Geometry& g, const CodecParams& cp, const GeneralArgs& a)
  {
    const A* d = (const A*)f;
    if (vec && rev) hipLaunchKernelGGL((encode4<A, true, true>), grid, block, lds, st, d, g, cp, a);
    else if (vec) hipLaunchKernelGGL((encode4<A, true, false>), grid, block, lds, st, d, g, cp, a);
    else if (rev) hipLaunchKernelGGL((encode4<A, false, true>), grid, block, lds, st, d, g, cp, a);
    else hipLaunchKernelGGL((encode4<A, false, false>), grid, block, lds, st, d, g, cp, a);
  }
  static void decode4i(bool rev, bool vec, hipStream_t st, dim3 grid, dim3 block, size_t lds, void* f,
                       const Geometry& g, const CodecParams& cp, const DecodeArgs& a)
  {
    A* d = (A*)f;
    if (vec && rev) hipLaunchKernelGGL((decode4<A, true, true>), grid, block, lds, st, d, g, cp, a);
    else if (vec) hipLaunchKernelGGL((decode4<A, true, false>), grid, block, lds, st, d, g, cp, a);
    else if (rev) hipLaunchKernelGGL((decode4<A, false, true>), grid, block, lds, st, d, g, cp, a);
    else hipLaunchKernelGGL((decode4<A, false, false>), grid, block, lds, st, d, g, cp, a);
  }
  static void encode(int type, int dims, bool rev, hipStream_t st, dim3 grid, dim3 block, size_t lds, const void* f,
                     const Geometry& g, const CodecParams& cp, const GeneralArgs& a)
  {
    if (type <= 2) {
      if (dims == 1) enc<A, 1>(rev, st, grid, block, lds, f, g, cp, a);
      else if (dims == 2) enc<A, 2>(rev, st, grid, block, lds, f, g, cp, a);
      else enc<A, 3>(rev, st, grid, block, lds, f, g, cp, a);
    } else {
      if (dims == 1) enc<B, 1>(rev, st, grid, block, lds, f, g, cp, a);
      else enc<B, 2>(rev, st, grid, block, lds, f, g, cp, a);
    }
  }
  static void decode(int type, int dims, bool rev, hipStream_t st, dim3 grid, dim3 block, size_t lds, void* f,
                     const Geometry& g, const CodecParams& cp, const DecodeArgs& a)
  {
    if (type <= 2) {
      if (dims == 1) dec<A, 1>(rev, st, grid, block, lds, f, g, cp, a);
      else if (dims == 2) dec<A, 2>(rev, st, grid, block, lds, f, g, cp, a);
      else dec<A, 3>(rev, st, grid, block, lds, f, g, cp, a);
    } else {
      if (dims == 1) dec<B, 1>(rev, st, grid, block, lds, f, g, cp, a);
      else dec<B, 2>(rev, st, grid, block, lds, f, g, cp, a);
    }
  }
};

}  // namespace zfp_amd
