// Generic per-lane kernels for 8-byte scalars (double 1D/2D, int64 1D/2D/3D);
// see kernels_n.h.
#include "kernels_n.h"

namespace zfp_amd {

void launch_encode_n64(int type, int dims, bool rev, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                       const void* field, const Geometry& g, const CodecParams& cp, const GeneralArgs& a)
{
  GenericKernels<int64_t, double>::encode(type, dims, rev, stream, grid, block, lds, field, g, cp, a);
}

void launch_decode_n64(int type, int dims, bool rev, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                       void* field, const Geometry& g, const CodecParams& cp, const DecodeArgs& a)
{
  GenericKernels<int64_t, double>::decode(type, dims, rev, stream, grid, block, lds, field, g, cp, a);
}

void launch_encode4_int64(bool rev, bool vec, hipStream_t stream, dim3 grid, dim3 block, size_t lds,
                          const void* field, const Geometry& g, const CodecParams& cp, const GeneralArgs& a)
{
  GenericKernels<int64_t, double>::encode4i(rev, vec, stream, grid, block, lds, field, g, cp, a);
}

void launch_decode4_int64(bool rev, bool vec, hipStream_t stream, dim3 grid, dim3 block, size_t lds, void* field,
                          const Geometry& g, const CodecParams& cp, const DecodeArgs& a)
{
  GenericKernels<int64_t, double>::decode4i(rev, vec, stream, grid, block, lds, field, g, cp, a);
}

}  // namespace zfp_amd
