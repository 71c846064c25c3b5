// PCIe copy rates on the box: pageable vs pinned, each direction alone and both
// at once from two threads on two streams (design input for the host pipeline).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s failed: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main()
{
  const size_t A = (size_t)4 << 30, B = (size_t)2 << 30, CH = (size_t)128 << 20;
  char *ha = (char*)malloc(A), *hb = (char*)malloc(B);
  memset(ha, 1, A); memset(hb, 2, B);
  char *da, *db, *pa, *pb;
  CK(hipMalloc(&da, A)); CK(hipMalloc(&db, B));
  CK(hipHostMalloc(&pa, CH * 2)); CK(hipHostMalloc(&pb, CH * 2));
  hipStream_t s1, s2; CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  auto h2d = [&](bool chunked) { for (size_t o = 0; o < A; o += CH) { CK(hipMemcpyAsync(da + o, ha + o, CH, hipMemcpyHostToDevice, s1)); } CK(hipStreamSynchronize(s1)); };
  auto d2h = [&]() { for (size_t o = 0; o < B; o += CH) { CK(hipMemcpyAsync(hb + o, db + o, CH, hipMemcpyDeviceToHost, s2)); } CK(hipStreamSynchronize(s2)); };
  for (int rep = 0; rep < 2; rep++) {
    double t0 = now(); h2d(true); double t1 = now(); d2h(); double t2 = now();
    std::thread th([&] { h2d(true); }); double t3 = now(); d2h(); th.join(); double t4 = now();
    printf("pageable: H2D %.1f GB/s, D2H %.1f GB/s, both at once %.1f ms (%.1f GB/s total)\n", A / (t1 - t0) / 1e9,
           B / (t2 - t1) / 1e9, (t4 - t3) * 1e3, (A + B) / (t4 - t3) / 1e9);
  }
  // pinned staging: DMA only (no CPU copy) rates
  for (int rep = 0; rep < 2; rep++) {
    double t0 = now();
    for (size_t o = 0; o < A; o += CH) CK(hipMemcpyAsync(da + o, pa, CH, hipMemcpyHostToDevice, s1));
    CK(hipStreamSynchronize(s1));
    double t1 = now();
    for (size_t o = 0; o < B; o += CH) CK(hipMemcpyAsync(pb, db + o, CH, hipMemcpyDeviceToHost, s2));
    CK(hipStreamSynchronize(s2));
    double t2 = now();
    for (size_t o = 0; o < A; o += CH) CK(hipMemcpyAsync(da + o, pa, CH, hipMemcpyHostToDevice, s1));
    for (size_t o = 0; o < B; o += CH) CK(hipMemcpyAsync(pb, db + o, CH, hipMemcpyDeviceToHost, s2));
    CK(hipStreamSynchronize(s1)); CK(hipStreamSynchronize(s2));
    double t3 = now();
    printf("pinned DMA: H2D %.1f GB/s, D2H %.1f GB/s, both at once %.1f GB/s total\n", A / (t1 - t0) / 1e9,
           B / (t2 - t1) / 1e9, (A + B) / (t3 - t2) / 1e9);
  }
  // CPU memcpy rate, 1 and 8 threads
  for (int nt : {1, 4, 8, 16}) {
    double t0 = now();
    std::vector<std::thread> ts;
    for (int i = 0; i < nt; i++)
      ts.emplace_back([&, i] { size_t per = B / nt; memcpy(hb + i * per, ha + i * per, per); });
    for (auto& t : ts) t.join();
    double t1 = now();
    printf("host memcpy %d threads: %.1f GB/s\n", nt, B / (t1 - t0) / 1e9);
  }
  // hipHostRegister cost of the 4 GB buffer
  double t0 = now();
  CK(hipHostRegister(ha, A, hipHostRegisterDefault));
  double t1 = now();
  for (size_t o = 0; o < A; o += CH) CK(hipMemcpyAsync(da + o, ha + o, CH, hipMemcpyHostToDevice, s1));
  CK(hipStreamSynchronize(s1));
  double t2 = now();
  CK(hipHostUnregister(ha));
  double t3 = now();
  printf("hipHostRegister 4 GiB: %.1f ms, registered H2D %.1f GB/s, unregister %.1f ms\n", (t1 - t0) * 1e3,
         A / (t2 - t1) / 1e9, (t3 - t2) * 1e3);
  return 0;
}
