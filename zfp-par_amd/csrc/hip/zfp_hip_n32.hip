// Generic per-lane kernels for 4-byte scalars (float 1D/2D, int32 1D/2D/3D);
// see kernels_n.h.
#include "kernels_n.h"

namespace zfp_amd {

void launch_encode_n32(int type, int dims, bool rev, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                       const void* field, const Geometry& g, const CodecParams& cp, const GeneralArgs& a)
{
  GenericKernels<int32_t, float>::encode(type, dims, rev, stream, grid, block, lds, field, g, cp, a);
}

void launch_decode_n32(int type, int dims, bool rev, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                       void* field, const Geometry& g, const CodecParams& cp, const DecodeArgs& a)
{
  GenericKernels<int32_t, float>::decode(type, dims, rev, stream, grid, block, lds, field, g, cp, a);
}

void launch_encode4_int(int type, bool rev, bool vec, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                        const void* field, const Geometry& g, const CodecParams& cp, const GeneralArgs& a)
{
  if (type == 1)
    GenericKernels<int32_t, float>::encode4i(rev, vec, stream, grid, block, lds, field, g, cp, a);
  else
    launch_encode4_int64(rev, vec, stream, grid, block, lds, field, g, cp, a);
}

void launch_decode4_int(int type, bool rev, bool vec, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                        void* field, const Geometry& g, const CodecParams& cp, const DecodeArgs& a)
{
  if (type == 1)
    GenericKernels<int32_t, float>::decode4i(rev, vec, stream, grid, block, lds, field, g, cp, a);
  else
    launch_decode4_int64(rev, vec, stream, grid, block, lds, field, g, cp, a);
}

}  // namespace zfp_amd
