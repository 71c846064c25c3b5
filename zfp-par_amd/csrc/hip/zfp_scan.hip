// Index scan passes (scan.h) for every scalar type, dimensionality and mode,
// compiled apart from the host shim.
#include "launch.h"

namespace zfp_amd {

template <typename S>
static void scan_typed(int dims, bool rev, dim3 grid, hipStream_t st, const ScanArgs& a)
{
  const dim3 block(256);
  switch (dims) {
    case 1:
      if (rev) hipLaunchKernelGGL((scan_pass<S, 1, true>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((scan_pass<S, 1, false>), grid, block, 0, st, a);
      break;
    case 2:
      if (rev) hipLaunchKernelGGL((scan_pass<S, 2, true>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((scan_pass<S, 2, false>), grid, block, 0, st, a);
      break;
    case 3:
      if (rev) hipLaunchKernelGGL((scan_pass<S, 3, true>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((scan_pass<S, 3, false>), grid, block, 0, st, a);
      break;
    default:
      if (rev) hipLaunchKernelGGL((scan_pass<S, 4, true>), grid, block, 0, st, a);
      else hipLaunchKernelGGL((scan_pass<S, 4, false>), grid, block, 0, st, a);
      break;
  }
}

template <typename S>
static void window_typed(int dims, bool rev, hipStream_t st, const ScanArgs& a, int32_t* win)
{
  const dim3 one(1), block(64);
  switch (dims) {
    case 1:
      if (rev) hipLaunchKernelGGL((scan_window<S, 1, true>), one, block, 0, st, a, win);
      else hipLaunchKernelGGL((scan_window<S, 1, false>), one, block, 0, st, a, win);
      break;
    case 2:
      if (rev) hipLaunchKernelGGL((scan_window<S, 2, true>), one, block, 0, st, a, win);
      else hipLaunchKernelGGL((scan_window<S, 2, false>), one, block, 0, st, a, win);
      break;
    case 3:
      if (rev) hipLaunchKernelGGL((scan_window<S, 3, true>), one, block, 0, st, a, win);
      else hipLaunchKernelGGL((scan_window<S, 3, false>), one, block, 0, st, a, win);
      break;
    default:
      if (rev) hipLaunchKernelGGL((scan_window<S, 4, true>), one, block, 0, st, a, win);
      else hipLaunchKernelGGL((scan_window<S, 4, false>), one, block, 0, st, a, win);
      break;
  }
}

// the exponent window of pass 1's plausible chain starts (float types only)
void launch_scan_window(int type, int dims, bool rev, hipStream_t stream, const ScanArgs& a, int32_t* win)
{
  if (type == 3)
    window_typed<float>(dims, rev, stream, a, win);
  else if (type == 4)
    window_typed<double>(dims, rev, stream, a, win);
}

void launch_scan_pass(int type, int dims, bool rev, dim3 grid, hipStream_t stream, const ScanArgs& a)
{
  switch (type) {
    case 1: scan_typed<int32_t>(dims, rev, grid, stream, a); break;
    case 2: scan_typed<int64_t>(dims, rev, grid, stream, a); break;
    case 3: scan_typed<float>(dims, rev, grid, stream, a); break;
    default: scan_typed<double>(dims, rev, grid, stream, a); break;
  }
}

}  // namespace zfp_amd
