// libzfp_hip.so -- MI355X codec library behind include/zfp_hip.h.
//
// Host side of the C-ABI: validates a job, works out where the field and the
// stream live (host or device), stages host buffers through per-thread device
// scratch on a per-thread HIP stream, picks a kernel path and launches it.
//
//   fixed rate, block size a multiple of 64 bits  -> encode3_aligned (+ one
//        funnel-shift pass when the stream offset is not word aligned)
//   everything else (variable rate, odd block sizes) -> encode3_general with
//        decoupled look-back, then fixup_zero/fixup_or for words shared by waves
//   decode: decode3 (fixed-rate offsets analytic, variable rate from the index)
//   4D: encode4 / decode4 (one block per quad of lanes, 16 blocks per wave),
//        every mode through the packing path of encode3_general
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <numeric>
#include <string>
#include <thread>
#include <vector>

#include "kernels_n.h"
#include "launch.h"
#include "zfp_hip.h"

using namespace zfp_amd;

// ---------------------------------------------------------------------------
// errors
static thread_local std::string g_err;

static int fail(const char* fmt, ...)
{
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return 0;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return fail("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

// ---------------------------------------------------------------------------
// block index (variable-rate streams)
// An index describes one stream: it records the codec settings, the layout
// and a fingerprint of the stream's words (stream_fingerprint), and is used
// only for a stream that matches all of them (index_matches) -- another
// stream of the same shape, a changed mode or a rewritten buffer is scanned.
struct zfp_hip_index {
  int device = -1;
  uint64_t nblocks = 0;
  uint64_t nwaves = 0;
  uint32_t per_wave = 0;       // blocks per wave of the layout it was made for (64: 3D, 16: 4D)
  uint64_t start_bit = ~0ull;  // stream bit offset of block 0 it was made for
  uint64_t total_bits = 0;
  uint64_t fp = 0;             // stream_fingerprint of the stream it was made for
  uint32_t minbits = 0, maxbits = 0, maxprec = 0;
  int32_t minexp = 0;
  int32_t type = 0, dims = 0;
  uint16_t* d_len = nullptr;   // per-block bit length
  uint64_t* d_base = nullptr;  // per-wave start bit relative to the stream's first block
  size_t cap_blocks = 0, cap_waves = 0;
};

static int index_reserve(zfp_hip_index* x, uint64_t nblocks, uint64_t nwaves)
{
  if (x->cap_blocks < nblocks) {
    if (x->d_len) (void)hipFree(x->d_len);
    x->d_len = nullptr;
    x->cap_blocks = 0;
    if (hipMalloc(&x->d_len, std::max<uint64_t>(nblocks, 1) * sizeof(uint16_t)) != hipSuccess)
      return fail("hipMalloc of the block index (%llu blocks) failed", (unsigned long long)nblocks);
    x->cap_blocks = nblocks;
  }
  if (x->cap_waves < nwaves) {
    if (x->d_base) (void)hipFree(x->d_base);
    x->d_base = nullptr;
    x->cap_waves = 0;
    if (hipMalloc(&x->d_base, std::max<uint64_t>(nwaves, 1) * sizeof(uint64_t)) != hipSuccess)
      return fail("hipMalloc of the block index (%llu waves) failed", (unsigned long long)nwaves);
    x->cap_waves = nwaves;
  }
  return 1;
}

static void index_release(zfp_hip_index* x)
{
  if (x->d_len) (void)hipFree(x->d_len);
  if (x->d_base) (void)hipFree(x->d_base);
  x->d_len = nullptr;
  x->d_base = nullptr;
  x->cap_blocks = x->cap_waves = 0;
  x->nblocks = x->nwaves = 0;
  x->start_bit = ~0ull;
  x->fp = 0;
}

// Fingerprint of the stream bits [start_bit, start_bit + total_bits): a hash
// of the bit count and of 16 words spread evenly over the range (the first
// and last masked to the range).  Two streams of one field and mode whose
// block lengths differ anywhere differ in the words after that block, so an
// index is not used for a stream it does not describe (a stream that matches
// in every sampled word and in length has, in practice, the same block
// offsets).  Host streams are read in place; device streams through a small
// gather kernel.
constexpr int kFpWords = 16;

static __global__ void fp_gather(const uint64_t* __restrict__ w, uint64_t W0, uint64_t n, uint64_t* __restrict__ out)
{
  const uint32_t i = threadIdx.x;
  if (i < kFpWords)
    out[i] = w[W0 + (n - 1) * i / (kFpWords - 1)];
}

static uint64_t fp_mix(uint64_t h, uint64_t v)
{
  h ^= v + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
  return h * 0xff51afd7ed558ccdull;
}

// ---------------------------------------------------------------------------
// device contexts: a HIP stream, events and reusable scratch.  Calls borrow a
// context from a process-wide pool and return it when they finish, so the
// number of contexts (and their device memory) is bounded by the peak number
// of concurrent calls, whatever threads make them (zfpy builds a new thread
// pool per call).  zfp_hip_release_scratch() frees the idle ones.
struct Scratch {
  void* p = nullptr;
  size_t bytes = 0;
};

struct Ctx {
  int device = -1;
  hipStream_t stream = nullptr;
  hipStream_t side[2] = {nullptr, nullptr};  // host slab pipeline: uploads, downloads
  hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};  // [4], [5]: index scan
  Scratch field, words, status, partials, misc, ovf, fpbuf;
  Scratch scan_bm, scan_seg, scan_tiles, scan_pos;  // index scan of a stream without index
  zfp_hip_index scan_index;                         // index built by the scan
  Scratch chk;                                      // index verification word (DecodeArgs::idx_bad)
  uint32_t* idx_chk = nullptr;                      // set while a caller's index is being verified
};

struct Timing {
  double kernel_ms = 0, total_ms = 0, scan_ms = 0;
  int scan_passes = 0;
  bool timed = false;
  bool stale_index = false;  // the last decompress found its index stale and scanned (zfp_hip_last_stale_index)
};
static thread_local Timing t_timing;

static std::mutex g_pool_mu;
static std::vector<Ctx*> g_idle;

static void free_scratch(Scratch& s)
{
  if (s.p)
    (void)hipFree(s.p);
  s.p = nullptr;
  s.bytes = 0;
}

static void destroy_ctx(Ctx* c)
{
  (void)hipSetDevice(c->device);
  for (Scratch* s : {&c->field, &c->words, &c->status, &c->partials, &c->misc, &c->ovf, &c->fpbuf, &c->scan_bm,
                     &c->scan_seg, &c->scan_tiles, &c->scan_pos, &c->chk})
    free_scratch(*s);
  index_release(&c->scan_index);
  for (auto& e : c->ev)
    if (e) (void)hipEventDestroy(e);
  if (c->stream)
    (void)hipStreamDestroy(c->stream);
  for (auto& q : c->side)
    if (q) (void)hipStreamDestroy(q);
  delete c;
}

static int ensure(Scratch& s, size_t bytes)
{
  if (s.bytes >= bytes)
    return 1;
  free_scratch(s);
  // size classes (powers of two up to 256 MiB, then 64 MiB steps): calls of
  // slightly different sizes reuse a context's buffers instead of regrowing them
  size_t want = 64 << 10;
  if (bytes > ((size_t)256 << 20))
    want = (bytes + ((size_t)64 << 20) - 1) & ~(((size_t)64 << 20) - 1);
  else
    while (want < bytes) want <<= 1;
  hipError_t e = hipMalloc(&s.p, want);
  if (e != hipSuccess) {
    s.p = nullptr;
    return fail("hipMalloc(%zu) failed: %s", want, hipGetErrorString(e));
  }
  s.bytes = want;
  return 1;
}

static Ctx* acquire_ctx(int device)
{
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess)
      device = 0;
  }
  if (hipSetDevice(device) != hipSuccess) {
    fail("hipSetDevice(%d) failed", device);
    return nullptr;
  }
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t i = g_idle.size(); i-- > 0;)  // most recently returned first
      if (g_idle[i]->device == device) {
        Ctx* c = g_idle[i];
        g_idle.erase(g_idle.begin() + (long)i);
        return c;
      }
  }
  Ctx* c = new Ctx;
  c->device = device;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    fail("hipStreamCreate failed");
    delete c;
    return nullptr;
  }
  for (auto& e : c->ev)
    (void)hipEventCreate(&e);
  return c;
}

static void release_ctx(Ctx* c)
{
  if (!c)
    return;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  g_idle.push_back(c);
}

// borrows a context for the lifetime of one API call
struct CtxLease {
  Ctx* c;
  explicit CtxLease(int device) : c(acquire_ctx(device)) {}
  ~CtxLease() { release_ctx(c); }
  CtxLease(const CtxLease&) = delete;
  CtxLease& operator=(const CtxLease&) = delete;
};

static bool is_device_ptr(const void* p)
{
  if (!p)
    return false;
  hipPointerAttribute_t attr;
  hipError_t e = hipPointerGetAttributes(&attr, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeDevice;
}

static int stream_fingerprint(Ctx* c, const uint64_t* words, bool dev, uint64_t start_bit, uint64_t total_bits,
                              uint64_t* fp)
{
  const uint64_t W0 = start_bit >> 6, end = start_bit + total_bits;
  const uint64_t n = total_bits ? ((end + 63) >> 6) - W0 : 1;
  uint64_t v[kFpWords];
  if (dev) {
    if (!ensure(c->fpbuf, kFpWords * 8))
      return 0;
    hipLaunchKernelGGL(fp_gather, dim3(1), dim3(64), 0, c->stream, words, W0, n, (uint64_t*)c->fpbuf.p);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(v, c->fpbuf.p, sizeof v, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
  } else {
    for (int i = 0; i < kFpWords; i++)
      v[i] = words[W0 + (n - 1) * (uint64_t)i / (kFpWords - 1)];
  }
  uint64_t h = fp_mix(0x7a6670ull, total_bits);
  for (int i = 0; i < kFpWords; i++) {
    const uint64_t wi = W0 + (n - 1) * (uint64_t)i / (kFpWords - 1);
    uint64_t m = ~0ull;
    if (wi == W0)
      m &= ~0ull << (start_bit & 63);
    if (total_bits && wi == ((end - 1) >> 6) && (end & 63))
      m &= (1ull << (end & 63)) - 1;
    if (!total_bits)
      m = 0;
    h = fp_mix(h, v[i] & m);
  }
  *fp = h;
  return 1;
}

// ---------------------------------------------------------------------------
// job analysis
struct Plan {
  int dims = 0;
  int type = 0;      // zfp_type: 1 int32, 2 int64, 3 float, 4 double
  size_t es = 0;     // bytes per value
  bool dbl = false;  // double (the f64 float kernels)
  Geometry g{};
  CodecParams cp{};
  bool fixed = false;        // every block exactly maxbits bits
  bool vec = false;          // 16-byte row loads/stores possible
  uint32_t bound_bits = 0;   // max bits a block writes (excl. padding)
  uint32_t max_len = 0;      // max block length incl. padding
  int64_t span_lo = 0, span_hi = 0;  // element offsets touched by the box
};

static int plan_job(const zfp_hip_job* j, const void* field_base, Plan& p)
{
  if (!j)
    return fail("null job");
  if (j->type < 1 || j->type > 4)
    return fail("zfp_hip: scalar type %d not supported", j->type);
  if (j->dims < 1 || j->dims > 4)
    return fail("zfp_hip: %dD fields are not supported", j->dims);
  p.dims = j->dims;
  p.type = j->type;
  p.dbl = j->type == 4;
  p.es = (j->type == 2 || j->type == 4) ? 8 : 4;
  p.cp.minbits = j->minbits;
  p.cp.maxbits = j->maxbits;
  p.cp.maxprec = j->maxprec;
  p.cp.minexp = j->minexp;
  if (p.cp.maxprec == 0 || p.cp.maxprec > 64)
    return fail("zfp_hip: invalid maxprec %u", p.cp.maxprec);
  p.g.nblocks = 1;
  p.span_lo = p.span_hi = 0;
  for (int a = 0; a < 4; a++) {
    p.g.n[a] = a < p.dims ? j->n[a] : 1;
    p.g.s[a] = a < p.dims ? j->s[a] : 0;
    p.g.f[a] = a < p.dims ? j->f[a] : 0;
    uint64_t e = a < p.dims ? j->e[a] : 1;
    uint64_t nb = (a < p.dims) ? (e > p.g.f[a] ? (e - p.g.f[a] + 3) / 4 : 0) : 1;
    if (a < p.dims && e > p.g.n[a])
      return fail("zfp_hip: chunk end %llu exceeds field extent %llu on axis %d", (unsigned long long)e,
                  (unsigned long long)p.g.n[a], a);
    if (nb > 0xffffffffull)
      return fail("zfp_hip: too many blocks along axis %d", a);
    p.g.nb[a] = (uint32_t)nb;
    p.g.nblocks *= nb;
    if (a < p.dims && e > p.g.f[a]) {
      int64_t d0 = (int64_t)p.g.f[a] * p.g.s[a];
      // a block reads whole 4-blocks past a chunk end that is not block aligned
      // (up to the field edge, compress.c:127-133): the span covers them
      const uint64_t eb = std::min<uint64_t>(p.g.n[a], p.g.f[a] + 4 * nb);
      int64_t d1 = (int64_t)(eb - 1) * p.g.s[a];
      p.span_lo += std::min(d0, d1);
      p.span_hi += std::max(d0, d1);
    }
  }
  if (p.g.nblocks >> 32)
    return fail("zfp_hip: %llu blocks in one call (at most 2^32 - 1)", (unsigned long long)p.g.nblocks);
  for (int a = 0; a < 3; a++)
    p.g.dv[a] = make_fastdiv(p.g.nb[a]);
  const bool integer = p.type <= 2;
  const int ebits = integer ? 0 : p.dbl ? 11 : 8, pbits = p.es == 8 ? 6 : 5, intprec = p.es == 8 ? 64 : 32;
  const bool rev = p.cp.minexp < kMinExp;
  // header bits (zfp.c block bounds): integers have none in lossy modes
  const uint32_t hdr = integer ? (rev ? pbits : 0) : (rev ? 2 + ebits + pbits : 1 + ebits);
  const uint64_t bvals = 1ull << (2 * p.dims);  // values per block
  uint64_t body = hdr + (bvals - 1) + bvals * std::min<uint32_t>(p.cp.maxprec, intprec);
  uint64_t bound = body;
  if (p.cp.maxbits >= hdr)
    bound = std::min<uint64_t>(bound, p.cp.maxbits);
  p.bound_bits = (uint32_t)bound;
  p.max_len = std::max<uint32_t>(p.bound_bits, p.cp.minbits);
  p.fixed = !rev && p.cp.minbits == p.cp.maxbits && p.cp.maxbits >= (uint32_t)(integer ? 1 : 1 + ebits);
  const size_t es = p.es;
  p.vec = p.g.s[0] == 1 && (p.g.s[1] % 4) == 0 && (p.g.s[2] % 4) == 0 && (p.g.f[0] % 4) == 0 &&
          (p.dims < 4 || (p.g.s[3] % 4) == 0) && ((uintptr_t)field_base % (4 * es)) == 0;
  if (!p.fixed && p.max_len > 0xffff)
    return fail("zfp_hip: block length bound %u bits exceeds the block index (16-bit lengths)", p.max_len);
  return 1;
}

// the codec settings and layout an index is made for
static void index_stamp(zfp_hip_index* x, const Plan& p)
{
  x->minbits = p.cp.minbits;
  x->maxbits = p.cp.maxbits;
  x->maxprec = p.cp.maxprec;
  x->minexp = p.cp.minexp;
  x->type = p.type;
  x->dims = p.dims;
}

static size_t slot_words_odd(uint32_t bits)
{
  return slot_words_for(bits) | 1;  // odd stride: fewer LDS bank collisions between lanes
}

// ---------------------------------------------------------------------------
// launchers

// The stream word holding an encode's first bit (bits below g0 belong to what
// precedes it): `val` ORed in (the host's pending bits), or with `keep` the bits
// already in the device word are kept (a host slab pipeline: what the previous
// slab wrote).  `idx_add` is added to the per-wave index bases (the launch's
// bit offset within its chunk).
struct Head {
  uint64_t val = 0;
  bool keep = false;
  uint64_t idx_add = 0;
};

// f(tag) with a null pointer of the field's scalar type
template <typename F>
static int by_type(const Plan& p, F&& f)
{
  switch (p.type) {
    case 1: return f((int32_t*)nullptr);
    case 2: return f((int64_t*)nullptr);
    case 3: return f((float*)nullptr);
    default: return f((double*)nullptr);
  }
}

static uint64_t head_keep_mask(const Head& h, uint32_t g0) { return h.keep && g0 ? (1ull << g0) - 1 : 0ull; }

// double with maxprec <= 32: the kernels that code planes 32..63 only
template <typename S>
static bool hi_planes(const Plan& p)
{
  return std::is_same<S, double>::value && p.dims == 3 && p.cp.maxprec <= 32;
}

// 1D/2D blocks and integer fields: the generic per-lane codec (blockn.h),
// instantiated in zfp_hip_n32.hip / zfp_hip_n64.hip (separate translation
// units, compiled in parallel)
template <typename S, int D>
static void launch_enc_generic(Ctx* c, const Plan& p, const S* d_field, dim3 grid, dim3 block, size_t lds,
                               const GeneralArgs& a)
{
  launch_encode_n(p.type, D, p.cp.minexp < kMinExp, c->stream, grid, block, lds, d_field, p.g, p.cp, a);
}

template <typename S, int D>
static void launch_dec_generic(Ctx* c, const Plan& p, S* d_field, dim3 grid, dim3 block, size_t lds,
                               const DecodeArgs& a)
{
  launch_decode_n(p.type, D, p.cp.minexp < kMinExp, c->stream, grid, block, lds, d_field, p.g, p.cp, a);
}

template <typename S, bool HI>
static void launch_general3(Ctx* c, const Plan& p, const S* d_field, dim3 grid, dim3 block, size_t lds,
                            const GeneralArgs& a)
{
  if constexpr (kIntField<S>) {
    if (p.dims == 1) launch_enc_generic<S, 1>(c, p, d_field, grid, block, lds, a);
    else if (p.dims == 2) launch_enc_generic<S, 2>(c, p, d_field, grid, block, lds, a);
    else launch_enc_generic<S, 3>(c, p, d_field, grid, block, lds, a);
  } else {
    if (p.dims == 1) return launch_enc_generic<S, 1>(c, p, d_field, grid, block, lds, a);
    if (p.dims == 2) return launch_enc_generic<S, 2>(c, p, d_field, grid, block, lds, a);
    launch_encode3_general(Launch{grid, block, lds, c->stream}, p.vec, p.cp.minexp < kMinExp, HI, d_field, p.g,
                           p.cp, a);
  }
}

template <typename S, bool HI>
static void run_decode3(Ctx* c, const Plan& p, S* d_field, dim3 grid, dim3 block, size_t lds, const DecodeArgs& a)
{
  if constexpr (kIntField<S>) {
    if (p.dims == 1) launch_dec_generic<S, 1>(c, p, d_field, grid, block, lds, a);
    else if (p.dims == 2) launch_dec_generic<S, 2>(c, p, d_field, grid, block, lds, a);
    else launch_dec_generic<S, 3>(c, p, d_field, grid, block, lds, a);
  } else {
    if (p.dims == 1) return launch_dec_generic<S, 1>(c, p, d_field, grid, block, lds, a);
    if (p.dims == 2) return launch_dec_generic<S, 2>(c, p, d_field, grid, block, lds, a);
    // short staging slots (a.ovf) exist for the f64 planes-32..63 decoder only
    launch_decode3(Launch{grid, block, lds, c->stream}, p.vec, p.cp.minexp < kMinExp, HI, HI && a.ovf != nullptr,
                   d_field, p.g, p.cp, a);
  }
}

// Arguments of the packing encoders (encode3_general, encode4) for `nwaves`
// waves: fix-up partials, look-back state and, for a variable-rate stream with
// an index, the index buffers.  Queues the look-back resets on the stream.
static int general_args(Ctx* c, const Plan& p, uint64_t nwaves, uint32_t swp, uint64_t* d_out, uint32_t g0,
                        zfp_hip_index* index, uint64_t idx_add, GeneralArgs& a)
{
  const bool var = !p.fixed;
  // misc: [0] total bits, [1] ticket|error
  if (!ensure(c->partials, nwaves * 2 * sizeof(Partial)) || !ensure(c->misc, 64) ||
      (var && !ensure(c->status, nwaves * 8)))
    return 0;
  a = GeneralArgs{};
  a.out = d_out;
  a.g0 = g0;
  a.swp = swp;
  a.var = var ? 1 : 0;
  a.maxbits = p.cp.maxbits;
  a.status = (uint64_t*)c->status.p;
  a.total_bits = (uint64_t*)c->misc.p;
  a.ticket = (uint32_t*)((char*)c->misc.p + 8);
  a.error = (uint32_t*)((char*)c->misc.p + 12);
  a.partials = (Partial*)c->partials.p;
  a.idx_add = idx_add;
  if (var && index) {
    if (!index_reserve(index, p.g.nblocks, nwaves))
      return 0;
    index->device = c->device;
    index->nblocks = p.g.nblocks;
    index->nwaves = nwaves;
    index->per_wave = p.dims == 4 ? kBlocks4PerWave : 64u;
    index->start_bit = ~0ull;  // set by the caller once the encode succeeded
    a.idx_len = index->d_len;
    a.idx_base = index->d_base;
  }
  HIP_TRY(hipMemsetAsync(c->misc.p, 0, 64, c->stream));
  if (var)
    HIP_TRY(hipMemsetAsync(c->status.p, 0, nwaves * 8, c->stream));
  return 1;
}

// After a packing encoder: merge the words shared by neighbouring waves; for a
// variable-rate stream read back its length (and the look-back health flag).
// kRedoFullSlots: the overflow pool of a short-slot launch ran out, the launch
// must be repeated with full-size slots.
constexpr int kRedoFullSlots = 2;
static int finish_general(Ctx* c, const Plan& p, uint64_t nwaves, uint64_t* d_out, uint32_t g0, const Head& head,
                          const GeneralArgs& a, zfp_hip_index* index, uint64_t* total_bits)
{
  unsigned fg = (unsigned)((2 * nwaves + 255) / 256);
  hipLaunchKernelGGL(fixup_zero, dim3(fg), dim3(256), 0, c->stream, a.partials, 2 * nwaves, d_out, 0ull,
                     g0 ? head.val : 0ull, head_keep_mask(head, g0));
  hipLaunchKernelGGL(fixup_or, dim3(fg), dim3(256), 0, c->stream, a.partials, 2 * nwaves, d_out);
  HIP_TRY(hipGetLastError());
  if (!p.fixed) {
    uint64_t host[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(host, c->misc.p, 16, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const uint32_t err = (uint32_t)(host[1] >> 32);
    if (err & 1u)
      return fail("zfp_hip: look-back timed out (GPU scheduling anomaly)");
    if (err & 2u)
      return kRedoFullSlots;
    *total_bits = host[0];
    if (index)
      index->total_bits = host[0];
  } else {
    *total_bits = p.g.nblocks * (uint64_t)p.cp.maxbits;
  }
  return 1;
}

// Short LDS slots for the variable-rate 3D encoders.  A slot sized for the
// block's worst case (C3: 2,123 bits, 35 words) limits the CU to two
// workgroups; the kernels' registers allow three (f64 planes 32..63: <= 168
// VGPRs) or four (f32 lossy).  The slot is cut to what that
// many workgroups can hold; blocks that code longer take the overflow pool.
// Fixed rate, 1D/2D and integer fields keep full-size slots.
template <typename S>
static uint32_t short_slot_words(const Plan& p)
{
  if (p.fixed || p.dims != 3 || kIntField<S> || getenv("ZFP_HIP_FULL_SLOTS"))
    return ~0u;
  const bool rev = p.cp.minexp < kMinExp;
  // f32 reversible: 177 VGPRs (two waves per SIMD whatever the slots); measured
  // slower at three with spills
  int groups;
  if (sizeof(S) == 4)
    groups = rev ? 2 : 4;
  else
    groups = hi_planes<S>(p) ? 3 : 2;
  if (const char* e = getenv("ZFP_HIP_SLOT_WORDS"))  // tests: force overflows
    return (uint32_t)atoi(e) | 1u;
  const int64_t words = ((int64_t)(160 * 1024) / groups - (int64_t)kLutBytes) / 8 / kWavesPerGroup;
  int64_t swp = (words - 96) / 64;
  if ((swp & 1) == 0)
    swp--;
  return swp < 3 ? ~0u : (uint32_t)swp;
}

// Short slots for the variable-rate 4D encoder (f32 fields): the region of 16
// slots sized for the worst case (f32 reversible: 8,462 bits, 17.3 KB) limits
// the CU to 8 one-wave workgroups (2 waves per SIMD), where the registers allow
// 3 (f32 reversible).  f32 reversible slots are cut to what 12 waves per CU
// leave (93 words, 5,856 intact bits); a block that codes longer -- on the C5 field,
// the blocks that fail the reversible cast test, about 8,300 bits each -- is
// packed with its first bits and listed, and encode4_patch codes it again with
// a full slot.  The overflow pool holds a quarter of the blocks (the round-4
// first try sized it for 1/16 of them: more overflowed on C5 and the launch
// was redone with full slots, 46 -> 90 ms).  C5 chunk 46.4 -> 43.1 ms;
// 128^4 1.51 -> 1.55 ms (profiles/r4o_4d_slots.txt).  Lossy f32 modes keep
// full slots (not measured).  ZFP_HIP_SLOT_WORDS=n forces n-word slots (tests
// of the overflow and patch path), ZFP_HIP_FULL_SLOTS=1 full ones.
// Data whose blocks mostly overflow (noise-like fields) would pay the redo on
// every call: after a redo the next kFullSlotCalls4 calls of the same thread
// take full slots directly, then short slots are tried again.  The backoff is
// per thread (a caller looping over its own noisy data), so calls of other
// threads -- other zfp_parallel chunks, other devices -- are not slowed.
constexpr uint32_t kShortSlotWords4 = 93;
constexpr int kFullSlotCalls4 = 16;
static thread_local int t_full_slot_calls4 = 0;
template <typename S>
static uint32_t short_slot_words4(const Plan& p)
{
  if (p.fixed || kIntField<S> || sizeof(S) == 8 || getenv("ZFP_HIP_FULL_SLOTS"))
    return ~0u;
  if (const char* e = getenv("ZFP_HIP_SLOT_WORDS"))  // tests: force overflows
    return (uint32_t)atoi(e) | 1u;
  if (p.cp.minexp >= kMinExp)
    return ~0u;
  if (t_full_slot_calls4 > 0) {
    t_full_slot_calls4--;
    return ~0u;
  }
  return kShortSlotWords4;
}

template <typename S>
static void launch_encode4_kernel(Ctx* c, const Plan& p, const S* d_field, dim3 grid, size_t lds, const GeneralArgs& a,
                                  bool half)
{
  const bool rev = p.cp.minexp < kMinExp;
  if constexpr (kIntField<S>) {
    launch_encode4_int(p.type, rev, p.vec, c->stream, grid, dim3(64), lds, d_field, p.g, p.cp, a);
  } else {
    launch_encode4(Launch{grid, dim3(64), lds, c->stream}, p.vec, rev, half, d_field, p.g, p.cp, a);
  }
}

// 4D: encode4 for every mode (one 64-thread workgroup per 16 blocks)
template <typename S>
static int run_encode4(Ctx* c, const Plan& p, const S* d_field, uint64_t* d_out, uint32_t g0,
                          const Head& head, zfp_hip_index* index, uint64_t* total_bits)
{
  using Int = typename Traits<S>::Int;
  const uint64_t nwaves = (p.g.nblocks + kBlocks4PerWave - 1) / kBlocks4PerWave;
  if (nwaves > 0x7fffffffull)
    return fail("zfp_hip: field too large for one launch");
  const uint32_t swp_full = slot_words4(p.bound_bits);
  const size_t xfull = (size_t)kBlocks4PerWave * kXStride * sizeof(Int);
  const bool half = !kIntField<S>;  // f32/f64: exchange areas shared by two quads
  const uint32_t swp_short = short_slot_words4<S>(p);
  for (int attempt = 0; attempt < 2; attempt++) {
    const uint32_t swp = attempt == 0 ? std::min(swp_full, swp_short) : swp_full;
    const size_t region = std::max<size_t>((size_t)kBlocks4PerWave * swp * 8, half ? xfull / 2 : xfull);
    const size_t lds = (size_t)kEnc4HeadWords * 8 + region;
    if (lds > 160 * 1024)
      return fail("zfp_hip: 4D block bound %u bits too large for LDS", p.bound_bits);
    GeneralArgs a{};
    if (!general_args(c, p, nwaves, swp, d_out, g0, index, head.idx_add, a))
      return 0;
    if (swp < swp_full) {
      // a quarter of the blocks (C5: about 1/20 overflow); more makes the
      // launch redo itself with full slots (correct, slower)
      uint64_t cap = std::min<uint64_t>(p.g.nblocks, std::max<uint64_t>(65536, p.g.nblocks / 4));
      if (const char* e = getenv("ZFP_HIP_OVF_POOL"))  // tests: force the full-slot redo
        cap = std::max<uint64_t>(1, std::min<uint64_t>(p.g.nblocks, (uint64_t)atoll(e)));
      if (!ensure(c->ovf, cap * sizeof(OvfEntry)))
        return 0;
      a.ovf = (uint64_t*)c->ovf.p;
      a.ovf_count = (uint32_t*)((char*)c->misc.p + 16);
      a.ovf_cap = (uint32_t)cap;
      a.ovf_swp = swp_full;
      a.cap_bits = slot_cap_bits4(swp);  // clamped writes of an outrun slot land in its last three dwords
    }
#ifdef ZFP_EXP4_TRACE
    const size_t ntr = (nwaves + 63) / 64 * 8;
    uint64_t* d_tr = nullptr;
    if (getenv("ZFP_HIP_TRACE4")) {
      HIP_TRY(hipMalloc(&d_tr, ntr * 8));
      HIP_TRY(hipMemsetAsync(d_tr, 0, ntr * 8, c->stream));
    }
    a.trace = d_tr;
#endif
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    launch_encode4_kernel<S>(c, p, d_field, dim3((unsigned)nwaves), lds, a, half);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev[2], c->stream));
#ifdef ZFP_EXP4_TRACE
    if (d_tr) {
      std::vector<uint64_t> h(ntr);
      HIP_TRY(hipMemcpyAsync(h.data(), d_tr, ntr * 8, hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      HIP_TRY(hipFree(d_tr));
      // phases: 0 ticket, 1 gather landed, 2 cast+lifts+exchange, 3 transposes+coder, 4 look-back, 5 pack
      double sum[6] = {0}, t0min = 1e30, t0max = 0;
      size_t cnt = 0;
      for (size_t i = 0; i + 8 <= ntr; i += 8) {
        if (!h[i + 6]) continue;
        cnt++;
        uint64_t prev = 0;
        for (int k = 0; k < 6; k++) { sum[k] += (double)(h[i + k] - prev); prev = h[i + k]; }
        t0min = std::min(t0min, (double)h[i + 6]);
        t0max = std::max(t0max, (double)h[i + 6]);
      }
      fprintf(stderr, "trace4 waves %zu (100 MHz ticks, mean): ticket %.1f gather %.1f cast+lift+xchg %.1f coder %.1f lookback %.1f pack %.1f | launch span %.0f\n",
              cnt, sum[0] / cnt, sum[1] / cnt, sum[2] / cnt, sum[3] / cnt, sum[4] / cnt, sum[5] / cnt, t0max - t0min);
    }
#endif
    const int rc = finish_general(c, p, nwaves, d_out, g0, head, a, index, total_bits);
    if (rc == kRedoFullSlots) {
      if (!getenv("ZFP_HIP_SLOT_WORDS") && !getenv("ZFP_HIP_OVF_POOL"))
        t_full_slot_calls4 = kFullSlotCalls4;
      continue;
    }
    if (rc != 1 || !a.ovf)
      return rc;
    if constexpr (!kIntField<S>) {
      uint32_t n = 0;
      HIP_TRY(hipMemcpyAsync(&n, a.ovf_count, 4, hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      if (n) {
        const size_t plds = (size_t)kEnc4HeadWords * 8 + std::max<size_t>((size_t)kBlocks4PerWave * swp_full * 8, xfull);
        const dim3 pg((n + kBlocks4PerWave - 1) / kBlocks4PerWave), pb(64);
        const OvfEntry* list = (const OvfEntry*)a.ovf;
        launch_encode4_patch(Launch{pg, pb, plds, c->stream}, p.vec, p.cp.minexp < kMinExp, d_field, p.g, p.cp, d_out,
                             list, n, swp_full);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(c->ev[2], c->stream));
      }
    }
    return 1;
  }
  return fail("zfp_hip: overflow pool exhausted with full-size slots");
}

template <typename S>
static int launch_encode(Ctx* c, const Plan& p, const S* d_field, uint64_t* d_out, uint32_t g0,
                         const Head& head, zfp_hip_index* index, uint64_t* total_bits)
{
  if (p.dims == 4)
    return run_encode4<S>(c, p, d_field, d_out, g0, head, index, total_bits);
  const uint64_t nwaves = (p.g.nblocks + 63) / 64;
  const uint64_t ngroups = (nwaves + kWavesPerGroup - 1) / kWavesPerGroup;
  if (ngroups > 0x7fffffffull)
    return fail("zfp_hip: field too large for one launch");
  dim3 grid((unsigned)ngroups), block(256);
  // aligned fixed-rate kernel: word-multiple blocks and no precision limit
  // below the integer width (its coder runs every plane until the budget)
  if constexpr (!kIntField<S>)
  if (p.fixed && (p.cp.maxbits % 64) == 0 && p.cp.maxprec >= (p.dbl ? 64u : 32u) && p.dims == 3) {
    const uint32_t sw = p.cp.maxbits / 64;
    const uint32_t sdw = slot_dwords_for(p.cp.maxbits) | 1u;  // dwords from 2 sw on are spare
    auto magic_of = [](uint32_t d) { return d > 1 ? (uint32_t)((0x100000000ull + d - 1) / d) : 0u; };
    const uint32_t magic_w = magic_of(sw), magic_c = (sw & 1) ? 0u : magic_of(sw / 2);
    size_t lds = (size_t)kWavesPerGroup * 64 * sdw * 4;
    if (lds + 2 * kLutBytes > 160 * 1024)
      return fail("zfp_hip: block size %u bits too large for LDS", p.cp.maxbits);
    Partial* parts = nullptr;
    if (g0) {
      if (!ensure(c->partials, nwaves * 2 * sizeof(Partial)))
        return 0;
      parts = (Partial*)c->partials.p;
    }
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    launch_encode3_aligned(Launch{grid, block, lds, c->stream}, p.vec, d_field, p.g, p.cp, d_out, sw, sdw, magic_w,
                           magic_c, g0, parts);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev[2], c->stream));
    if (g0) {
      unsigned fg = (unsigned)((2 * nwaves + 255) / 256);
      hipLaunchKernelGGL(fixup_zero, dim3(fg), dim3(256), 0, c->stream, parts, 2 * nwaves, d_out, 0ull, head.val,
                         head_keep_mask(head, g0));
      hipLaunchKernelGGL(fixup_or, dim3(fg), dim3(256), 0, c->stream, parts, 2 * nwaves, d_out);
      HIP_TRY(hipGetLastError());
    }
    *total_bits = p.g.nblocks * (uint64_t)p.cp.maxbits;
    return 1;
  }
  // general path
  const uint32_t swp_full = (uint32_t)slot_words_odd(p.bound_bits);
  const uint32_t swp_short = short_slot_words<S>(p);
  for (int attempt = 0; attempt < 2; attempt++) {
    const uint32_t swp = attempt == 0 ? std::min(swp_full, swp_short) : swp_full;
    size_t lds = (size_t)kWavesPerGroup * gen_wave_words(swp) * 8;
    if (lds + kLutBytes > 160 * 1024)
      return fail("zfp_hip: block bound %u bits too large for LDS", p.bound_bits);
    GeneralArgs a{};
    if (!general_args(c, p, nwaves, swp, d_out, g0, index, head.idx_add, a))
      return 0;
    if (swp < swp_full) {
      // overflow pool: a sixteenth of the blocks (at least 64K, at most all)
      uint64_t cap = std::min<uint64_t>(p.g.nblocks, std::max<uint64_t>(65536, p.g.nblocks / 16));
      if (const char* e = getenv("ZFP_HIP_OVF_POOL"))  // tests: force the full-slot redo
        cap = std::max<uint64_t>(1, std::min<uint64_t>(cap, (uint64_t)atoll(e)));
      if (!ensure(c->ovf, cap * swp_full * 8))
        return 0;
      a.ovf = (uint64_t*)c->ovf.p;
      a.ovf_count = (uint32_t*)((char*)c->misc.p + 16);
      a.ovf_cap = (uint32_t)cap;
      a.ovf_swp = swp_full;
      a.cap_bits = 64 * swp - 96;  // the clamped writes of an outrun slot land in its last three dwords
    }
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    if constexpr (sizeof(S) == 8) {
      if (hi_planes<S>(p))
        launch_general3<S, true>(c, p, d_field, grid, block, lds, a);
      else
        launch_general3<S, false>(c, p, d_field, grid, block, lds, a);
    } else {
      launch_general3<S, false>(c, p, d_field, grid, block, lds, a);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev[2], c->stream));
    const int rc = finish_general(c, p, nwaves, d_out, g0, head, a, index, total_bits);
    if (rc != kRedoFullSlots)
      return rc;
  }
  return fail("zfp_hip: overflow pool exhausted with full-size slots");
}

template <typename S>
static int run_decode4(Ctx* c, const Plan& p, S* d_field, const uint64_t* d_in, uint64_t in_words, uint32_t g0,
                          const zfp_hip_index* index)
{
  using Int = typename Traits<S>::Int;
  const uint64_t nwaves = (p.g.nblocks + kBlocks4PerWave - 1) / kBlocks4PerWave;
  if (nwaves > 0x7fffffffull)
    return fail("zfp_hip: field too large for one launch");
  DecodeArgs a{};
  a.in = d_in;
  a.in_words = in_words;
  a.g0 = g0;
  a.var = p.fixed ? 0 : 1;
  a.maxbits = p.cp.maxbits;
  a.idx_bad = p.fixed ? nullptr : c->idx_chk;
  const uint32_t per_block = p.fixed ? p.cp.maxbits : p.max_len;
  a.W = (per_block + 63) / 64 + 1;  // peek64 at the budget end reads one word past it
  a.swp = a.W | 1;
  a.wmagic = (uint32_t)((0x100000000ull + a.W - 1) / a.W);
  if (!p.fixed) {
    if (index->nwaves != nwaves)
      return fail("zfp_hip: block index has %llu waves, the 4D layout needs %llu", (unsigned long long)index->nwaves,
                  (unsigned long long)nwaves);
    a.idx_len = index->d_len;
    a.idx_base = index->d_base;
  }
  // f32/f64: exchange areas shared by quad pairs (HALF), as in the encoder
  const bool half = !kIntField<S>;
  const size_t xfull = (size_t)kBlocks4PerWave * kXStride * sizeof(Int);
  // variable rate, f32/f64: the wave's segment (its 16 blocks, contiguous in
  // the stream) staged back to back in what the kernel's VGPR-bound number of
  // waves per CU leaves of the LDS (kDec4WavesPerCu); the staging reads only
  // the segment's words, where padded slots read 16 worst-case blocks' worth
  // for every wave.  A wave whose segment does not fit (runs of long blocks: on
  // the C5 field 2.6 % of the waves at 16 waves per CU) goes on a list that a
  // second launch decodes with padded slots.  ZFP_HIP_PACK_WORDS=n stages n words instead
  // (tests: many waves take the second launch); ZFP_HIP_FULL_SLOTS=1 padded
  // slots only.
  uint32_t packw = 0;
  if (!p.fixed && half && !getenv("ZFP_HIP_FULL_SLOTS")) {
    const uint32_t waves_per_cu = kDec4WavesPerCu<S>;
    const uint32_t fit = (uint32_t)(((160u * 1024u) / waves_per_cu - kDec4HeadWords * 8) / 8);
    const uint32_t worst = (uint32_t)((126ull + (uint64_t)kBlocks4PerWave * per_block) / 64 + 1);
    packw = std::min(fit, worst);
    if (const char* e = getenv("ZFP_HIP_PACK_WORDS"))
      packw = (uint32_t)atoi(e);
    if ((size_t)packw * 8 < xfull / 2)
      packw = (uint32_t)(xfull / 16);  // the exchange areas need that much anyway
    if ((size_t)kDec4HeadWords * 8 + (size_t)packw * 8 > 160 * 1024)
      packw = 0;
  }
  const bool rev = p.cp.minexp < kMinExp;
  auto launch = [&](uint32_t pw, dim3 grid) -> int {
    a.packw = pw;
    const size_t region = pw ? std::max<size_t>((size_t)pw * 8, xfull / 2)
                             : std::max<size_t>((size_t)kBlocks4PerWave * a.swp * 8, half ? xfull / 2 : xfull);
    const size_t lds = (size_t)kDec4HeadWords * 8 + region;
    if (lds > 160 * 1024)
      return fail("zfp_hip: 4D block size too large for LDS staging (%u bits)", per_block);
    if constexpr (kIntField<S>)
      launch_decode4_int(p.type, rev, p.vec, c->stream, grid, dim3(64), lds, d_field, p.g, p.cp, a);
    else
      launch_decode4(Launch{grid, dim3(64), lds, c->stream}, p.vec, rev, d_field, p.g, p.cp, a);
    HIP_TRY(hipGetLastError());
    return 1;
  };
#ifdef ZFP_EXP4_TRACE
  const size_t ntr = (nwaves + 63) / 64 * 8;
  uint64_t* d_tr = nullptr;
  if (getenv("ZFP_HIP_TRACE4")) {
    HIP_TRY(hipMalloc(&d_tr, ntr * 8));
    HIP_TRY(hipMemsetAsync(d_tr, 0, ntr * 8, c->stream));
  }
  a.trace = d_tr;
  struct TraceDump {
    Ctx* c; uint64_t* d; size_t n;
    ~TraceDump() {
      if (!d) return;
      std::vector<uint64_t> h(n);
      if (hipMemcpyAsync(h.data(), d, n * 8, hipMemcpyDeviceToHost, c->stream) == hipSuccess &&
          hipStreamSynchronize(c->stream) == hipSuccess) {
        // slots: 0 staged, 2..5 decode_block4 marks (parse, planes->coefficients, exchange, lift),
        // 1 decoded, 7 scattered
        const int order[7] = {0, 2, 3, 4, 5, 1, 7};
        double sum[7] = {0};
        size_t cnt = 0;
        for (size_t i = 0; i + 8 <= n; i += 8) {
          if (!h[i + 6]) continue;
          cnt++;
          uint64_t prev = 0;
          for (int k = 0; k < 7; k++) { sum[k] += (double)(h[i + order[k]] - prev); prev = h[i + order[k]]; }
        }
        if (cnt)
          fprintf(stderr, "dtrace4 waves %zu (100 MHz ticks, mean): stage %.1f parse %.1f planes->coeffs %.1f "
                  "exchange %.1f lift %.1f cast %.1f scatter %.1f\n", cnt, sum[0] / cnt, sum[1] / cnt,
                  sum[2] / cnt, sum[3] / cnt, sum[4] / cnt, sum[5] / cnt, sum[6] / cnt);
      }
      (void)hipFree(d);
    }
  } dump{c, d_tr, ntr};
#endif
  HIP_TRY(hipEventRecord(c->ev[1], c->stream));
  if (!packw) {
    if (!launch(0, dim3((unsigned)nwaves)))
      return 0;
    HIP_TRY(hipEventRecord(c->ev[2], c->stream));
    return 1;
  }
  // misc: [12] error, [16] list count; ovf: the wave list
  if (!ensure(c->misc, 64) || !ensure(c->ovf, nwaves * 4))
    return 0;
  HIP_TRY(hipMemsetAsync(c->misc.p, 0, 64, c->stream));
  a.error = (uint32_t*)((char*)c->misc.p + 12);
  a.ovf_count = (uint32_t*)((char*)c->misc.p + 16);
  a.wave_ovf = (uint32_t*)c->ovf.p;
  a.ovf_cap = (uint32_t)nwaves;
  if (!launch(packw, dim3((unsigned)nwaves)))
    return 0;
  uint32_t n = 0;
  HIP_TRY(hipMemcpyAsync(&n, a.ovf_count, 4, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (n) {
    // the listed waves again, their segments staged whole: sized for sixteen
    // worst-case blocks, so every segment fits (a wave that still did not --
    // an index entry past the block bound -- flags an error instead of
    // listing itself); fewer waves per CU, but only the segment's words are
    // read, where padded slots read sixteen worst-case blocks' worth
    const uint32_t worst = (uint32_t)((126ull + (uint64_t)kBlocks4PerWave * per_block) / 64 + 1);
    const bool packed2 = packw && (size_t)kDec4HeadWords * 8 + (size_t)worst * 8 <= 160 * 1024 &&
                         !getenv("ZFP_HIP_OVF_PADDED");
    if (getenv("ZFP_HIP_VERBOSE"))
      fprintf(stderr, "zfp_hip: decode4: %u of %llu wave segments past %u staged words, decoded %s\n", n,
              (unsigned long long)nwaves, packw, packed2 ? "from whole segments" : "with padded slots");
    a.wave_list = a.wave_ovf;
    a.ovf_cap = 0;
    if (!launch(packed2 ? worst : 0u, dim3(n)))
      return 0;
    a.wave_list = nullptr;
  }
  HIP_TRY(hipEventRecord(c->ev[2], c->stream));
  return 1;
}


// Short staging slots for the variable-rate 3D decoder (the encoder's rule,
// short_slot_words): words staged per block such that the kernel's VGPR-bound
// number of workgroups fits the CU's LDS; longer blocks are staged in global
// memory.  ~0u: full size.
template <typename S>
static uint32_t short_stage_words(const Plan& p)
{
  if (p.fixed || p.dims != 3 || kIntField<S> || getenv("ZFP_HIP_FULL_SLOTS"))
    return ~0u;
  if (!hi_planes<S>(p))  // the only decoder instantiated with short slots
    return ~0u;
  if (const char* e = getenv("ZFP_HIP_SLOT_WORDS"))  // tests: force overflows
    return (uint32_t)atoi(e) | 1u;
  const int groups = 3;
  const int64_t words = ((int64_t)(160 * 1024) / groups - (int64_t)kLutBytes - kWavesPerGroup * 64 * 4) / 8 /
                        (kWavesPerGroup * 64);
  const int64_t W = (words & 1) ? words : words - 1;
  return W < 3 ? ~0u : (uint32_t)W;
}

template <typename S>
static int launch_decode(Ctx* c, const Plan& p, S* d_field, const uint64_t* d_in, uint64_t in_words, uint32_t g0,
                         const zfp_hip_index* index)
{
  if (p.dims == 4)
    return run_decode4<S>(c, p, d_field, d_in, in_words, g0, index);
  const uint64_t nwaves = (p.g.nblocks + 63) / 64;
  if (!p.fixed && index->nwaves != nwaves)
    return fail("zfp_hip: block index has %llu waves, the 3D layout needs %llu", (unsigned long long)index->nwaves,
                (unsigned long long)nwaves);
  const uint64_t ngroups = (nwaves + kWavesPerGroup - 1) / kWavesPerGroup;
  const uint32_t per_block = p.fixed ? p.cp.maxbits : p.max_len;
  const uint32_t W_full = (per_block + 63) / 64 + 1;  // peek64 at the budget end reads one word past it
  const uint32_t W_short = short_stage_words<S>(p);
  for (int attempt = 0; attempt < 2; attempt++) {
    DecodeArgs a{};
    a.in = d_in;
    a.in_words = in_words;
    a.g0 = g0;
    a.var = p.fixed ? 0 : 1;
    a.maxbits = p.cp.maxbits;
    a.idx_bad = p.fixed ? nullptr : c->idx_chk;
    a.W = attempt == 0 ? std::min(W_full, W_short) : W_full;
    a.swp = a.W | 1;
    a.wmagic = (uint32_t)((0x100000000ull + a.W - 1) / a.W);
    if (!p.fixed) {
      a.idx_len = index->d_len;
      a.idx_base = index->d_base;
    }
    size_t lds = (size_t)kWavesPerGroup * 64 * a.swp * 8;
    if (lds + kLutBytes + kWavesPerGroup * 64 * 4 > 160 * 1024)
      return fail("zfp_hip: block size too large for LDS staging (%u bits)", per_block);
    if (a.W < W_full) {
      uint64_t cap = std::min<uint64_t>(p.g.nblocks, std::max<uint64_t>(65536, p.g.nblocks / 16));
      if (const char* e = getenv("ZFP_HIP_OVF_POOL"))
        cap = std::max<uint64_t>(1, std::min<uint64_t>(cap, (uint64_t)atoll(e)));
      if (!ensure(c->ovf, cap * W_full * 8) || !ensure(c->misc, 64))
        return 0;
      HIP_TRY(hipMemsetAsync(c->misc.p, 0, 64, c->stream));
      a.ovf = (uint64_t*)c->ovf.p;
      a.ovf_count = (uint32_t*)((char*)c->misc.p + 16);
      a.error = (uint32_t*)((char*)c->misc.p + 12);
      a.ovf_cap = (uint32_t)cap;
      a.ovf_W = W_full;
      a.cap_bits = (a.W - 1) * 64;
    }
    dim3 grid((unsigned)ngroups), block(256);
    HIP_TRY(hipEventRecord(c->ev[1], c->stream));
    if constexpr (sizeof(S) == 8) {
      if (hi_planes<S>(p))
        run_decode3<S, true>(c, p, d_field, grid, block, lds, a);
      else
        run_decode3<S, false>(c, p, d_field, grid, block, lds, a);
    } else {
      run_decode3<S, false>(c, p, d_field, grid, block, lds, a);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev[2], c->stream));
    if (!a.ovf)
      return 1;
    uint32_t err = 0;
    HIP_TRY(hipMemcpyAsync(&err, a.error, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (!(err & 2u))
      return 1;
  }
  return fail("zfp_hip: decode overflow pool exhausted with full-size slots");
}

static void record_timing(Ctx* c)
{
  float k = 0, t = 0;
  if (hipEventElapsedTime(&k, c->ev[1], c->ev[2]) == hipSuccess &&
      hipEventElapsedTime(&t, c->ev[0], c->ev[3]) == hipSuccess) {
    t_timing.kernel_ms = k;
    t_timing.total_ms = t;
    t_timing.timed = true;
  }
}

// Device-to-host copy of `bytes` into user memory that other threads may be
// filling at the same time (zfpy decompresses the chunks of one array from a
// thread pool, and chunk boundaries need not fall on pages).  The pageable
// copy path of the runtime may write whole pages, so only whole pages of the
// destination are copied directly; the partial pages at either end go through
// a private buffer and a CPU copy of exactly their bytes.
static int copy_to_host_exact(void* h, const void* d, size_t bytes, hipStream_t q)
{
  constexpr uintptr_t kPage = 4096;
  const uintptr_t a = (uintptr_t)h, e = a + bytes;
  const uintptr_t a1 = (a + kPage - 1) & ~(kPage - 1), e1 = e & ~(kPage - 1);
  if (a1 >= e1) {  // no whole page inside
    std::vector<char> tmp(bytes);
    HIP_TRY(hipMemcpyAsync(tmp.data(), d, bytes, hipMemcpyDeviceToHost, q));
    HIP_TRY(hipStreamSynchronize(q));
    memcpy(h, tmp.data(), bytes);
    return 1;
  }
  const size_t head = a1 - a, tail = e - e1;
  HIP_TRY(hipMemcpyAsync((void*)a1, (const char*)d + head, e1 - a1, hipMemcpyDeviceToHost, q));
  if (head || tail) {
    std::vector<char> tmp(head + tail);
    if (head)
      HIP_TRY(hipMemcpyAsync(tmp.data(), d, head, hipMemcpyDeviceToHost, q));
    if (tail)
      HIP_TRY(hipMemcpyAsync(tmp.data() + head, (const char*)d + (e1 - a), tail, hipMemcpyDeviceToHost, q));
    HIP_TRY(hipStreamSynchronize(q));
    memcpy(h, tmp.data(), head);
    memcpy((void*)e1, tmp.data() + head, tail);
  }
  return 1;
}

// copy the box of elements between a host field and a device image of its
// span (device pointer d_base corresponds to host pointer h_base)
static int copy_box(Ctx* c, const Plan& p, void* h_base, void* d_base, size_t es, bool to_host,
                    hipStream_t q = nullptr)
{
  if (!q)
    q = c->stream;
  // whole span contiguous?  (full x/y extents, default strides)
  const Geometry& g = p.g;
  bool contiguous = true;
  int64_t expect = 1;
  for (int a = 0; a < p.dims; a++) {
    if (g.s[a] != expect)
      contiguous = false;
    expect *= (int64_t)g.n[a];
  }
  uint64_t e[4];
  for (int a = 0; a < 4; a++)
    e[a] = a < p.dims ? std::min<uint64_t>(g.n[a], g.f[a] + 4ull * g.nb[a]) : 1;
  bool full_lower = true;
  for (int a = 0; a < p.dims - 1; a++)
    if (g.f[a] != 0 || e[a] != g.n[a])
      full_lower = false;
  hipMemcpyKind kind = to_host ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice;
  if ((contiguous && full_lower) || !to_host) {
    // one copy of the span (reading extra elements is harmless)
    size_t off = (size_t)p.span_lo * es;
    size_t bytes = (size_t)(p.span_hi - p.span_lo + 1) * es;
    if (to_host)
      return copy_to_host_exact((char*)h_base + off, (char*)d_base + off, bytes, q);
    else
      HIP_TRY(hipMemcpyAsync((char*)d_base + off, (char*)h_base + off, bytes, kind, q));
    return 1;
  }
  if (g.s[0] != 1)
    return fail("zfp_hip: host-resident decompression of a non-slab chunk needs unit x stride");
  // to host: the box's rows, (z, w) slice by slice, into a private dense
  // buffer (2D copies), then row by row into the field (neighbouring boxes of
  // the same array may be written concurrently, and the pageable copy path may
  // write whole pages)
  if (to_host) {
    const size_t w0 = (size_t)(e[0] - g.f[0]) * es;
    const size_t nrows = p.dims >= 2 ? (size_t)(e[1] - g.f[1]) : 1;
    const size_t pitch = nrows > 1 ? (size_t)g.s[1] * es : w0;
    const uint64_t z0 = p.dims >= 3 ? g.f[2] : 0, z1 = p.dims >= 3 ? e[2] : 1;
    const uint64_t v0 = p.dims >= 4 ? g.f[3] : 0, v1 = p.dims >= 4 ? e[3] : 1;
    std::vector<char> tmp(w0 * nrows * (size_t)((z1 - z0) * (v1 - v0)));
    auto slice_off = [&](uint64_t z, uint64_t w) {
      return (int64_t)g.f[0] * g.s[0] + (int64_t)(p.dims >= 2 ? g.f[1] : 0) * (p.dims >= 2 ? g.s[1] : 0) +
             (int64_t)z * (p.dims >= 3 ? g.s[2] : 0) + (int64_t)w * (p.dims >= 4 ? g.s[3] : 0);
    };
    size_t k = 0;
    for (uint64_t w = v0; w < v1; w++)
      for (uint64_t z = z0; z < z1; z++, k++)
        HIP_TRY(hipMemcpy2DAsync(tmp.data() + k * w0 * nrows, w0, (char*)d_base + slice_off(z, w) * (int64_t)es, pitch,
                                 w0, nrows, hipMemcpyDeviceToHost, q));
    HIP_TRY(hipStreamSynchronize(q));
    k = 0;
    for (uint64_t w = v0; w < v1; w++)
      for (uint64_t z = z0; z < z1; z++, k++)
        for (size_t y = 0; y < nrows; y++)
          memcpy((char*)h_base + (slice_off(z, w) + (int64_t)y * (p.dims >= 2 ? g.s[1] : 0)) * (int64_t)es,
                 tmp.data() + (k * nrows + y) * w0, w0);
    return 1;
  }
  // row-wise 2D copies, one per (z, w) slice
  size_t width = (size_t)(e[0] - g.f[0]) * es;
  size_t rows = p.dims >= 2 ? (size_t)(e[1] - g.f[1]) : 1;
  size_t pitch = (size_t)(p.dims >= 2 ? g.s[1] : 1) * es;
  for (uint64_t w = (p.dims >= 4 ? g.f[3] : 0); w < (p.dims >= 4 ? e[3] : 1); w++)
    for (uint64_t z = (p.dims >= 3 ? g.f[2] : 0); z < (p.dims >= 3 ? e[2] : 1); z++) {
      int64_t off = (int64_t)g.f[0] * g.s[0] + (int64_t)(p.dims >= 2 ? g.f[1] : 0) * (p.dims >= 2 ? g.s[1] : 0) +
                    (int64_t)z * (p.dims >= 3 ? g.s[2] : 0) + (int64_t)w * (p.dims >= 4 ? g.s[3] : 0);
      HIP_TRY(hipMemcpy2DAsync((char*)h_base + off * (int64_t)es, pitch, (char*)d_base + off * (int64_t)es, pitch,
                               width, rows, kind, q));
    }
  return 1;
}

// ---------------------------------------------------------------------------
// Index scan (scan.h): block starts of a variable-rate stream resident on the
// device at d_in (word 0 holds bit g0 of the first block), written into `x`.
// Segment length and pass-1 lead-in (ZFP_HIP_SCAN_SEG_BITS / _LEAD_BITS):
// a speculative chain resynchronises after ~116-205 Kbit on average (DESIGN.md
// §3.5), so short segments cost one pass per segment of every unsynchronised
// stretch.  A lead-in cuts the passes of f64 precision-32 streams (512^3: 18 ->
// 5 at 128 Kbit segments and 512 Kbit lead-in, 45 -> 41 ms) but not of 4D
// reversible ones, whose unsynchronised stretches run for megabits (128^4: 91
// passes at 64 Kbit without, 42 at 128 Kbit with, 145 -> 236 ms), so it is off
// by default (profiles/r3_scan_lead.txt).  Since pass 1 starts chains at
// plausible block starts (round 5) almost every segment is settled in pass 1,
// whose time is the slowest lane's start search plus its parse: 32 Kbit
// segments measured faster than 64 (128^4 reversible 38.2-39.6 -> 36.4-37.5 ms,
// 512^3 f64 precision 32 9.7-9.8 -> 7.8-8.0 ms) and 16 Kbit slower again
// (profiles/r5sg_scan_seg.txt, r5sg2_scan_seg_ab.txt).
#ifndef ZFP_SCAN_MIN_SEG_BITS
#define ZFP_SCAN_MIN_SEG_BITS 32768
#endif
#ifndef ZFP_SCAN_LEAD_BITS
#define ZFP_SCAN_LEAD_BITS 0
#endif
constexpr uint64_t kScanMinSegBits = ZFP_SCAN_MIN_SEG_BITS, kScanLeadBits = ZFP_SCAN_LEAD_BITS;

static uint64_t scan_seg_bits(uint64_t limit)
{
  if (const char* e = getenv("ZFP_HIP_SCAN_SEG_BITS")) {
    const uint64_t v = strtoull(e, nullptr, 10);
    if (v >= 64)
      return v & ~63ull;
  }
  // about 2^18 lanes at most
  uint64_t L = (limit + (1ull << 18) - 1) >> 18;
  L = std::max<uint64_t>(L, kScanMinSegBits);
  return (L + 63) & ~63ull;
}

// pass-1 lead-in (scan.h): long enough that a speculative chain has almost
// always met the true one before its segment starts
static uint64_t scan_lead_bits()
{
  if (const char* e = getenv("ZFP_HIP_SCAN_LEAD_BITS"))
    return strtoull(e, nullptr, 10);
  return kScanLeadBits;
}

static void launch_scan_dispatch(Ctx* c, const Plan& p, const ScanArgs& a)
{
  launch_scan_pass(p.type, p.dims, p.cp.minexp < kMinExp, dim3((unsigned)((a.nseg + 255) / 256)), c->stream, a);
}

static int scan_index(Ctx* c, const Plan& p, const uint64_t* d_in, uint64_t in_words, uint32_t g0,
                      zfp_hip_index* x)
{
  const uint64_t nb = p.g.nblocks;
  const uint32_t per_wave = p.dims == 4 ? kBlocks4PerWave : 64u;
  const uint64_t nwaves = (nb + per_wave - 1) / per_wave;
  const uint64_t avail = in_words * 64 > g0 ? in_words * 64 - g0 : 0;
  const uint64_t extent = std::min<uint64_t>(avail, nb * (uint64_t)p.max_len);
  const uint64_t limit = extent + 1;  // bit positions 0..extent may start a block (or end the last)
  const uint64_t seg = scan_seg_bits(limit);
  const uint64_t nseg = (limit + seg - 1) / seg;
  const uint64_t bm_words = (limit + 63) / 64;
  const uint64_t ntiles = (bm_words + kTileWords - 1) / kTileWords;
  if (!ensure(c->scan_bm, bm_words * 8) || !ensure(c->scan_seg, nseg * 4 * 8 + 64) ||
      !ensure(c->scan_tiles, ntiles * 8 + 64) || !ensure(c->scan_pos, (nb + 1) * 8) ||
      !index_reserve(x, nb, nwaves))
    return 0;
  hipEvent_t e0 = c->ev[4], e1 = c->ev[5];
  HIP_TRY(hipEventRecord(e0, c->stream));
  uint64_t* bm = (uint64_t*)c->scan_bm.p;
  uint64_t* used = (uint64_t*)c->scan_seg.p;
  uint64_t* xs = used + nseg;
  uint64_t* xsnap = xs + nseg;
  uint64_t* plaus = xsnap + nseg;
  uint32_t* moved = (uint32_t*)(plaus + nseg);
  uint32_t* refused = moved + 1;
  HIP_TRY(hipMemsetAsync(bm, 0, bm_words * 8, c->stream));
  HIP_TRY(hipMemsetAsync(used, 0xff, nseg * 8, c->stream));
  ScanArgs a{};
  a.in = d_in;
  a.in_words = in_words;
  a.g0 = g0;
  a.first = 1;
  a.seg_bits = seg;
  a.lead = scan_lead_bits();
  a.nseg = nseg;
  a.limit = limit;
  a.bm = bm;
  a.entry_used = used;
  a.xsnap = xsnap;
  a.x = xs;
  a.moved = moved;
  a.sp = ScanParams{p.cp.minbits, p.cp.maxbits, p.cp.maxprec, p.cp.minexp};
  // float streams: pass 1 starts each chain at a plausible block start (scan.h);
  // ZFP_HIP_SCAN_PLAUSIBLE=0 starts them at the segment's first bit instead
  const char* pl = getenv("ZFP_HIP_SCAN_PLAUSIBLE");
  if ((p.type == 3 || p.type == 4) && !(pl && pl[0] == '0')) {
    int32_t* win = reinterpret_cast<int32_t*>(moved + 2);
    launch_scan_window(p.type, p.dims, p.cp.minexp < kMinExp, c->stream, a, win);
    HIP_TRY(hipGetLastError());
    a.win = win;
    a.plaus = plaus;
    a.refused = refused;
  }
  launch_scan_dispatch(c, p, a);
  HIP_TRY(hipGetLastError());
  a.first = 0;
  int passes = 1;
  // ZFP_HIP_SCAN_TRACE=1: per-pass wall time and moved exits on stderr (diagnostics)
  const bool trace = getenv("ZFP_HIP_SCAN_TRACE") != nullptr;
  auto tp = std::chrono::steady_clock::now();
  if (trace) {
    HIP_TRY(hipStreamSynchronize(c->stream));
    fprintf(stderr, "scan: %llu segments of %llu bits, pass 1 %.3f ms\n", (unsigned long long)nseg,
            (unsigned long long)seg, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tp).count());
    tp = std::chrono::steady_clock::now();
  }
  // phase A (plausible starts only): passes that refuse implausible chains at
  // segments still holding their plausible chain; phase B: ordinary passes,
  // which settle whatever phase A left inconsistent (scan.h)
  a.refuse = a.plaus ? 1u : 0u;
  for (;;) {
    uint32_t host_cnt[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(xsnap, xs, nseg * 8, hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMemsetAsync(moved, 0, 8, c->stream));
    launch_scan_dispatch(c, p, a);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(host_cnt, moved, 8, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    passes++;
    if (trace) {
      const auto t = std::chrono::steady_clock::now();
      fprintf(stderr, "scan: pass %d%s %.3f ms, %u exits moved, %u refused\n", passes, a.refuse ? " (A)" : "",
              std::chrono::duration<double, std::milli>(t - tp).count(), host_cnt[0], host_cnt[1]);
      tp = t;
    }
    if (!host_cnt[0]) {
      if (!a.refuse || !host_cnt[1])
        break;
      a.refuse = 0;  // phase A settled with refusals outstanding: ordinary passes
      continue;
    }
    if ((uint64_t)passes > 2 * nseg + 4)
      return fail("zfp_hip: index scan did not converge after %d passes", passes);
  }
  // bitmap -> positions -> index
  uint64_t* tiles = (uint64_t*)c->scan_tiles.p;
  uint64_t* sum = tiles + ntiles;
  uint64_t* pos = (uint64_t*)c->scan_pos.p;
  hipLaunchKernelGGL(bm_tile_count, dim3((unsigned)ntiles), dim3(256), 0, c->stream, bm, bm_words, tiles);
  hipLaunchKernelGGL(tile_scan, dim3(1), dim3(1024), 0, c->stream, tiles, ntiles, sum);
  hipLaunchKernelGGL(bm_tile_emit, dim3((unsigned)ntiles), dim3(256), 0, c->stream, bm, bm_words, tiles, nb, pos);
  hipLaunchKernelGGL(index_from_pos, dim3((unsigned)((nb + 255) / 256)), dim3(256), 0, c->stream, pos, nb, per_wave,
                     x->d_len, x->d_base);
  HIP_TRY(hipGetLastError());
  uint64_t host[2] = {0, 0};
  HIP_TRY(hipMemcpyAsync(&host[0], sum, 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(&host[1], pos + nb, 8, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipEventRecord(e1, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (host[0] < nb + 1)
    return fail("zfp_hip: stream holds %llu of %llu blocks (truncated or not a stream of this field/mode)",
                (unsigned long long)(host[0] ? host[0] - 1 : 0), (unsigned long long)nb);
  float ms = 0;
  if (hipEventElapsedTime(&ms, e0, e1) == hipSuccess)
    t_timing.scan_ms = ms;
  t_timing.scan_passes = passes;
  x->device = c->device;
  x->nblocks = nb;
  x->nwaves = nwaves;
  x->per_wave = per_wave;
  x->total_bits = host[1];
  return 1;
}

// the index was made for this stream: same codec settings, layout, bit offset
// and device, and the stream's fingerprint over the index's bit count agrees
static bool index_matches(Ctx* c, const zfp_hip_index* x, const Plan& p, const uint64_t* words, bool dev_stream,
                          uint64_t capacity_words, uint64_t bit_offset)
{
  if (!(x && x->d_len && x->nblocks == p.g.nblocks && x->start_bit == bit_offset && x->device == c->device &&
        x->per_wave == (p.dims == 4 ? kBlocks4PerWave : 64u) && x->minbits == p.cp.minbits &&
        x->maxbits == p.cp.maxbits && x->maxprec == p.cp.maxprec && x->minexp == p.cp.minexp && x->type == p.type &&
        x->dims == p.dims))
    return false;
  if (((bit_offset + x->total_bits + 63) >> 6) > capacity_words)
    return false;
  uint64_t fp = 0;
  if (!stream_fingerprint(c, words, dev_stream, bit_offset, x->total_bits, &fp)) {
    (void)hipGetLastError();
    return false;
  }
  return fp == x->fp;
}

// ---------------------------------------------------------------------------
// Host-resident field and stream: slab pipeline.  The chunk is
// cut along its outermost axis into slabs of whole block layers (default about
// 128 MB of field each).  Three host threads drive three HIP streams:
//   uploads    field slab s (compress) / stream words of slab s (decompress)
//   kernels    slab s once its upload is done (a device-side event wait)
//   downloads  stream words / field slab s once its kernel is done
// so the two PCIe directions run at once (pageable copies from two threads: 83
// GB/s together on the box, 57 and 55 alone) and the kernels hide under them.
// Slab s is an ordinary chunk encode at bit offset O_s: fixed rate O_s is
// analytic; variable rate O_s = O_{s-1} + its length, known when slab s-1's
// kernel returns (the look-back runs within a slab).  The word holding O_s is
// shared by two slabs: slab s keeps the bits slab s-1 left below its first bit
// (Head::keep), and slab s-1's download stops before that word.  Every slab has
// its own region of the device images, so no buffer is reused while a copy of
// it may be in flight.
static uint64_t env_mb(const char* name, uint64_t dflt)
{
  if (const char* e = getenv(name)) {
    const uint64_t v = strtoull(e, nullptr, 10);
    if (v)
      return v << 20;
  }
  return dflt << 20;
}

struct Slab {
  zfp_hip_job job;
  Plan p;
  uint64_t b0;  // first block of the slab within the chunk
};

// Slabs of whole block layers along the outermost axis; false: the chunk is
// not worth (or not fit for) the pipeline.  `align`: slabs hold whole waves of
// this many blocks (variable rate: the chunk's block index layout).
static bool make_slabs(const zfp_hip_job* job, const void* field_base, const Plan& p, uint64_t align,
                       std::vector<Slab>& out)
{
  const size_t es = p.es;
  const uint64_t field_bytes = (uint64_t)(p.span_hi - p.span_lo + 1) * es;
  if (field_bytes < env_mb("ZFP_HIP_PIPE_MIN_MB", 256))
    return false;
  // contiguous layout: each slab's span is its own range of the field
  int64_t expect = 1;
  for (int a = 0; a < p.dims; a++) {
    if (p.g.s[a] != expect)
      return false;
    expect *= (int64_t)p.g.n[a];
  }
  const int ao = p.dims - 1;
  const uint64_t nbo = p.g.nb[ao];
  if (nbo < 2)
    return false;
  const uint64_t layer = p.g.nblocks / nbo;
  const uint64_t layer_bytes = layer * (1ull << (2 * p.dims)) * es;
  uint64_t L = std::max<uint64_t>(1, env_mb("ZFP_HIP_PIPE_SLAB_MB", 128) / layer_bytes);
  if (align > 1) {
    const uint64_t q = align / std::gcd(layer, align);
    L = (L + q - 1) / q * q;
  }
  if (L >= nbo)
    return false;
  for (uint64_t l0 = 0; l0 < nbo; l0 += L) {
    Slab sl;
    sl.job = *job;
    sl.job.f[ao] = job->f[ao] + 4 * l0;
    sl.job.e[ao] = std::min<uint64_t>(job->e[ao], job->f[ao] + 4 * (l0 + L));
    if (!plan_job(&sl.job, field_base, sl.p))
      return false;
    sl.b0 = l0 * layer;
    out.push_back(sl);
  }
  return true;
}

static int ensure_side_streams(Ctx* c)
{
  for (auto& q : c->side)
    if (!q)
      HIP_TRY(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
  return 1;
}

// Hand-off between the pipeline's host threads: `done[k]` counts the slabs
// whose stage-k event is recorded (a stream can only wait for a recorded event).
struct PipeSync {
  std::mutex mu;
  std::condition_variable cv;
  size_t done[2] = {0, 0};
  bool failed = false;
  std::string err;
  void post(int k, size_t n)
  {
    { std::lock_guard<std::mutex> l(mu); done[k] = n; }
    cv.notify_all();
  }
  void fail_with(const char* what)
  {
    { std::lock_guard<std::mutex> l(mu); if (!failed) { failed = true; err = what; } }
    cv.notify_all();
  }
  bool wait(int k, size_t n)  // false: another stage failed
  {
    std::unique_lock<std::mutex> l(mu);
    cv.wait(l, [&] { return failed || done[k] >= n; });
    return !failed;
  }
};

struct EventSet {
  std::vector<hipEvent_t> ev;
  explicit EventSet(size_t n) : ev(n, nullptr)
  {
    for (auto& e : ev)
      (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  }
  ~EventSet()
  {
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
  }
};

template <typename S>
static int compress_slabs(Ctx* c, const Plan& p, const std::vector<Slab>& sl, const void* field_base,
                          uint64_t* words, uint64_t capacity_words, uint64_t bit_offset, uint64_t head_word,
                          zfp_hip_index* index, uint64_t* end_bit)
{
  const size_t es = sizeof(S);
  const size_t ns = sl.size();
  const uint64_t W0 = bit_offset >> 6;
  const uint64_t worst_bits = (bit_offset & 63) + p.g.nblocks * (uint64_t)(p.fixed ? p.cp.maxbits : p.max_len);
  const uint64_t worst_words = (worst_bits + 63) / 64 + 1;
  if (!ensure(c->field, (size_t)(p.span_hi - p.span_lo + 1) * es) || !ensure(c->words, worst_words * 8) ||
      !ensure_side_streams(c))
    return 0;
  char* d_img = (char*)c->field.p - p.span_lo * (int64_t)es;
  uint64_t* d_words = (uint64_t*)c->words.p;
  const uint32_t per_wave = p.dims == 4 ? kBlocks4PerWave : 64u;
  const bool var_index = !p.fixed && index;
  if (var_index) {
    // the index describes no stream until this one is complete
    index->start_bit = ~0ull;
    index->nblocks = 0;
    if (!index_reserve(index, p.g.nblocks, (p.g.nblocks + per_wave - 1) / per_wave))
      return 0;
  }
  EventSet ev_in(ns), ev_k(ns);
  std::vector<uint64_t> wa(ns), wb(ns);  // stream words [wa, wb) of slab s, relative to W0
  PipeSync ps;
  std::thread up([&] {
    if (hipSetDevice(c->device) != hipSuccess)
      return ps.fail_with("hipSetDevice failed (upload thread)");
    for (size_t s = 0; s < ns; s++) {
      if (!copy_box(c, sl[s].p, (void*)field_base, d_img, es, false, c->side[0]) ||
          hipEventRecord(ev_in.ev[s], c->side[0]) != hipSuccess)
        return ps.fail_with("field upload failed");
      ps.post(0, s + 1);
    }
  });
  std::thread down([&] {
    if (hipSetDevice(c->device) != hipSuccess)
      return ps.fail_with("hipSetDevice failed (download thread)");
    for (size_t s = 0; s < ns; s++) {
      if (!ps.wait(1, s + 1))
        return;
      if (hipStreamWaitEvent(c->side[1], ev_k.ev[s], 0) != hipSuccess ||
          hipMemcpyAsync(words + W0 + wa[s], d_words + wa[s], (wb[s] - wa[s]) * 8, hipMemcpyDeviceToHost,
                         c->side[1]) != hipSuccess)
        return ps.fail_with("stream download failed");
    }
    if (hipStreamSynchronize(c->side[1]) != hipSuccess)
      ps.fail_with("stream download failed");
  });
  uint64_t off = bit_offset;
  int ok = 1;
  for (size_t s = 0; s < ns && ok; s++) {
    if (!ps.wait(0, s + 1)) {
      ok = 0;
      break;
    }
    if (hipStreamWaitEvent(c->stream, ev_in.ev[s], 0) != hipSuccess) {
      ok = fail("hipStreamWaitEvent failed");
      break;
    }
    const uint64_t Ws = off >> 6;
    Head h;
    h.val = s == 0 ? head_word : 0ull;
    h.keep = s > 0;
    h.idx_add = off - bit_offset;
    zfp_hip_index view;  // the slab's part of the chunk's index
    if (var_index) {
      view.device = c->device;
      view.d_len = index->d_len + sl[s].b0;
      view.d_base = index->d_base + sl[s].b0 / per_wave;
      view.cap_blocks = view.cap_waves = ~(size_t)0;
    }
    uint64_t total = 0;
    ok = launch_encode<S>(c, sl[s].p, (const S*)d_img, d_words + (Ws - W0), (uint32_t)(off & 63), h,
                          var_index ? &view : nullptr, &total);
    view.d_len = nullptr;  // a view: nothing to free
    view.d_base = nullptr;
    if (!ok)
      break;
    const uint64_t next = off + total;
    wa[s] = Ws - W0;
    wb[s] = (s + 1 < ns ? next >> 6 : (next + 63) >> 6) - W0;
    if (W0 + wb[s] > capacity_words) {
      ok = fail("zfp_hip_compress: compressed stream (%llu words) exceeds capacity %llu",
                (unsigned long long)(W0 + wb[s]), (unsigned long long)capacity_words);
      break;
    }
    if (hipEventRecord(ev_k.ev[s], c->stream) != hipSuccess) {
      ok = fail("hipEventRecord failed");
      break;
    }
    ps.post(1, s + 1);
    off = next;
  }
  if (!ok)
    ps.fail_with(g_err.c_str());
  up.join();
  down.join();
  // every queued copy has finished before the call returns, failed or not
  (void)hipStreamSynchronize(c->stream);
  (void)hipStreamSynchronize(c->side[0]);
  (void)hipStreamSynchronize(c->side[1]);
  if (!ok)
    return 0;
  if (ps.failed)
    return fail("zfp_hip_compress: %s", ps.err.c_str());
  if (var_index) {
    index->device = c->device;
    index->nblocks = p.g.nblocks;
    index->nwaves = (p.g.nblocks + per_wave - 1) / per_wave;
    index->per_wave = per_wave;
    index->total_bits = off - bit_offset;
    index_stamp(index, p);
    if (!stream_fingerprint(c, words, false, bit_offset, index->total_bits, &index->fp))
      return 0;
    index->start_bit = bit_offset;
  }
  *end_bit = off;
  return 1;
}

// Slab s's stream words are known before any kernel runs: fixed rate
// analytically, variable rate from the block index (the start of the slab's
// first wave; slabs hold whole waves), whose per-slab bases are read back
// first.  Every slab decodes against the chunk's whole stream image, with its
// view of the index, once its own words have arrived.
template <typename S>
static int decompress_slabs(Ctx* c, const Plan& p, const std::vector<Slab>& sl, void* field_base,
                            const uint64_t* words, uint64_t capacity_words, uint64_t bit_offset,
                            const zfp_hip_index* index, uint64_t* end_bit)
{
  const size_t es = sizeof(S);
  const size_t ns = sl.size();
  const uint64_t W0 = bit_offset >> 6;
  const uint32_t g0 = (uint32_t)(bit_offset & 63);
  const uint64_t avail = capacity_words > W0 ? capacity_words - W0 : 0;
  const uint64_t mb = p.cp.maxbits;
  const uint32_t per_wave = p.dims == 4 ? kBlocks4PerWave : 64u;
  const uint64_t total = p.fixed ? p.g.nblocks * mb : index->total_bits;
  const uint64_t nwords = std::min<uint64_t>((g0 + total + 63) / 64 + 1, avail);
  if (!ensure(c->field, (size_t)(p.span_hi - p.span_lo + 1) * es) || !ensure(c->words, nwords * 8 + 8) ||
      !ensure_side_streams(c))
    return 0;
  char* d_img = (char*)c->field.p - p.span_lo * (int64_t)es;
  uint64_t* d_words = (uint64_t*)c->words.p;
  EventSet ev_in(ns), ev_k(ns);
  // bit offset of slab s's first block relative to the chunk's first block
  std::vector<uint64_t> base(ns + 1, total);
  for (size_t s = 0; s < ns; s++) {
    if (p.fixed)
      base[s] = sl[s].b0 * mb;
    else
      HIP_TRY(hipMemcpyAsync(&base[s], index->d_base + sl[s].b0 / per_wave, 8, hipMemcpyDeviceToHost, c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  // stream words [wa, wb) relative to W0 read by slab s (one word of lookahead)
  std::vector<uint64_t> wa(ns), wb(ns);
  for (size_t s = 0; s < ns; s++) {
    if (base[s] > base[s + 1] || base[s + 1] > total)
      return fail("zfp_hip_decompress: block index inconsistent with the slab layout");
    wa[s] = (g0 + base[s]) >> 6;
    wb[s] = std::min<uint64_t>(((g0 + base[s + 1] + 63) >> 6) + 1, nwords);
  }
  PipeSync ps;
  std::thread up([&] {
    if (hipSetDevice(c->device) != hipSuccess)
      return ps.fail_with("hipSetDevice failed (upload thread)");
    for (size_t s = 0; s < ns; s++) {
      if (hipMemcpyAsync(d_words + wa[s], words + W0 + wa[s], (wb[s] - wa[s]) * 8, hipMemcpyHostToDevice,
                         c->side[0]) != hipSuccess ||
          hipEventRecord(ev_in.ev[s], c->side[0]) != hipSuccess)
        return ps.fail_with("stream upload failed");
      ps.post(0, s + 1);
    }
  });
  std::thread down([&] {
    if (hipSetDevice(c->device) != hipSuccess)
      return ps.fail_with("hipSetDevice failed (download thread)");
    for (size_t s = 0; s < ns; s++) {
      if (!ps.wait(1, s + 1))
        return;
      if (hipStreamWaitEvent(c->side[1], ev_k.ev[s], 0) != hipSuccess ||
          !copy_box(c, sl[s].p, field_base, d_img, es, true, c->side[1]))
        return ps.fail_with("field download failed");
    }
    if (hipStreamSynchronize(c->side[1]) != hipSuccess)
      ps.fail_with("field download failed");
  });
  int ok = 1;
  for (size_t s = 0; s < ns && ok; s++) {
    if (!ps.wait(0, s + 1)) {
      ok = 0;
      break;
    }
    if (hipStreamWaitEvent(c->stream, ev_in.ev[s], 0) != hipSuccess) {
      ok = fail("hipStreamWaitEvent failed");
      break;
    }
    if (p.fixed) {
      const uint64_t o = bit_offset + sl[s].b0 * mb;
      ok = launch_decode<S>(c, sl[s].p, (S*)d_img, d_words + wa[s], wb[s] - wa[s], (uint32_t)(o & 63), nullptr);
    } else {
      // the slab's part of the chunk's index (bases stay relative to the chunk)
      zfp_hip_index view;
      view.device = c->device;
      view.nblocks = sl[s].p.g.nblocks;
      view.nwaves = (sl[s].p.g.nblocks + per_wave - 1) / per_wave;
      view.per_wave = per_wave;
      view.total_bits = base[s + 1] - base[s];
      view.d_len = index->d_len + sl[s].b0;
      view.d_base = index->d_base + sl[s].b0 / per_wave;
      ok = launch_decode<S>(c, sl[s].p, (S*)d_img, d_words, nwords, g0, &view);
      view.d_len = nullptr;  // a view: nothing to free
      view.d_base = nullptr;
    }
    if (!ok)
      break;
    if (hipEventRecord(ev_k.ev[s], c->stream) != hipSuccess) {
      ok = fail("hipEventRecord failed");
      break;
    }
    ps.post(1, s + 1);
  }
  if (!ok)
    ps.fail_with(g_err.c_str());
  up.join();
  down.join();
  // every queued copy has finished before the call returns, failed or not
  (void)hipStreamSynchronize(c->stream);
  (void)hipStreamSynchronize(c->side[0]);
  (void)hipStreamSynchronize(c->side[1]);
  if (!ok)
    return 0;
  if (ps.failed)
    return fail("zfp_hip_decompress: %s", ps.err.c_str());
  *end_bit = bit_offset + total;
  return 1;
}

// ---------------------------------------------------------------------------
extern "C" {

int zfp_hip_device_count(void)
{
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

const char* zfp_hip_last_error(void) { return g_err.c_str(); }

int zfp_hip_is_device_ptr(const void* p)
{
  static int ndev = -1;  // benign race: every thread computes the same value
  if (ndev < 0)
    ndev = zfp_hip_device_count();
  return ndev > 0 && is_device_ptr(p) ? 1 : 0;
}

int zfp_hip_memcpy(void* dst, const void* src, size_t bytes)
{
  if (hipMemcpy(dst, src, bytes, hipMemcpyDefault) != hipSuccess)
    return fail("hipMemcpy(%zu) failed", bytes);
  return 1;
}

int zfp_hip_compress(const zfp_hip_job* job, const void* field_base, uint64_t* words, uint64_t capacity_words,
                     uint64_t bit_offset, uint64_t head_word, int device, zfp_hip_index* index, uint64_t* end_bit)
{
  Plan p;
  if (!plan_job(job, field_base, p))
    return 0;
  if (!field_base || !words)
    return fail("zfp_hip_compress: null field or stream pointer");
  if (zfp_hip_device_count() <= 0)
    return fail("zfp_hip_compress: no HIP device available");
  CtxLease lease(device);
  Ctx* c = lease.c;
  if (!c)
    return 0;
  t_timing = Timing{};
  const size_t es = p.es;
  const uint64_t W0 = bit_offset >> 6;
  const uint32_t g0 = (uint32_t)(bit_offset & 63);
  if (p.g.nblocks == 0) {
    *end_bit = bit_offset;
    return 1;
  }
  const uint64_t worst_bits = (uint64_t)g0 + p.g.nblocks * (uint64_t)(p.fixed ? p.cp.maxbits : p.max_len);
  const uint64_t worst_words = (worst_bits + 63) / 64 + 1;
  const bool dev_field = is_device_ptr(field_base);
  const bool dev_stream = is_device_ptr(words);
  if (p.fixed && W0 + (worst_bits + 63) / 64 > capacity_words)
    return fail("zfp_hip_compress: stream capacity %llu words < %llu needed", (unsigned long long)capacity_words,
                (unsigned long long)(W0 + (worst_bits + 63) / 64));
  if (!dev_field && !dev_stream && !getenv("ZFP_HIP_NO_PIPE")) {
    std::vector<Slab> sl;
    if (make_slabs(job, field_base, p, p.fixed ? 1 : (p.dims == 4 ? kBlocks4PerWave : 64u), sl)) {
      const auto t0 = std::chrono::steady_clock::now();
      const int ok = by_type(p, [&](auto tag) {
        using S = std::remove_pointer_t<decltype(tag)>;
        return compress_slabs<S>(c, p, sl, field_base, words, capacity_words, bit_offset, head_word, index, end_bit);
      });
      t_timing.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      t_timing.kernel_ms = 0;
      t_timing.timed = ok != 0;
      return ok;
    }
  }
  HIP_TRY(hipEventRecord(c->ev[0], c->stream));
  // field
  const void* d_field = field_base;
  if (!dev_field) {
    size_t bytes = (size_t)(p.span_hi - p.span_lo + 1) * es;
    if (!ensure(c->field, bytes))
      return 0;
    char* d_img = (char*)c->field.p - p.span_lo * (int64_t)es;
    if (!copy_box(c, p, (void*)field_base, d_img, es, false))
      return 0;
    d_field = d_img;
  }
  // stream
  uint64_t* d_out;
  const bool direct = dev_stream && W0 + worst_words <= capacity_words;
  if (direct) {
    d_out = words + W0;
  } else {
    if (!ensure(c->words, worst_words * 8))
      return 0;
    d_out = (uint64_t*)c->words.p;
  }
  uint64_t total = 0;
  Head head;
  head.val = head_word;
  int ok = by_type(p, [&](auto tag) {
    using S = std::remove_pointer_t<decltype(tag)>;
    return launch_encode<S>(c, p, (const S*)d_field, d_out, g0, head, index, &total);
  });
  if (!ok)
    return 0;
  const uint64_t end = bit_offset + total;
  const uint64_t nwords = (g0 + total + 63) / 64;
  if (W0 + nwords > capacity_words)
    return fail("zfp_hip_compress: compressed stream (%llu words) exceeds capacity %llu",
                (unsigned long long)(W0 + nwords), (unsigned long long)capacity_words);
  if (!direct) {
    hipMemcpyKind kind = dev_stream ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    HIP_TRY(hipMemcpyAsync(words + W0, d_out, nwords * 8, kind, c->stream));
  }
  HIP_TRY(hipEventRecord(c->ev[3], c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  record_timing(c);
  if (index && !p.fixed) {
    index_stamp(index, p);
    if (!stream_fingerprint(c, words, dev_stream, bit_offset, total, &index->fp))
      return 0;
    index->start_bit = bit_offset;
  }
  *end_bit = end;
  return 1;
}

// One decompression with the given index (nullptr: the stream is scanned).
// *stale: the decoded block lengths disagreed with a caller's index that had
// passed index_matches -- the index belongs to another stream; the output is
// garbage and the caller decodes again with a scan.
static int decompress_once(Ctx* c, const Plan& p, const zfp_hip_job* job, void* field_base, const uint64_t* words,
                           uint64_t capacity_words, uint64_t bit_offset, const zfp_hip_index* index,
                           uint64_t* end_bit, bool* stale)
{
  const size_t es = p.es;
  const uint64_t W0 = bit_offset >> 6;
  const uint32_t g0 = (uint32_t)(bit_offset & 63);
  const bool dev_field = is_device_ptr(field_base);
  const bool dev_stream = is_device_ptr(words);
  // a variable-rate stream without a matching index (made by another
  // process, another library, or for another stream or position) is scanned
  const bool have_index = !p.fixed && index_matches(c, index, p, words, dev_stream, capacity_words, bit_offset);
  const bool scan = !p.fixed && !have_index;
  // a caller's index that passed the (sampled) fingerprint is verified exactly
  // by the decode kernels: every block's decoded length against its entry
  c->idx_chk = nullptr;
  if (have_index) {
    if (!ensure(c->chk, 8))
      return 0;
    HIP_TRY(hipMemsetAsync(c->chk.p, 0, 4, c->stream));
    c->idx_chk = (uint32_t*)c->chk.p;
  }
  auto verified = [&]() -> int {
    if (!c->idx_chk)
      return 1;
    uint32_t bad = 0;
    c->idx_chk = nullptr;
    HIP_TRY(hipMemcpyAsync(&bad, c->chk.p, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (bad)
      *stale = true;
    return 1;
  };
  const uint64_t avail = capacity_words > W0 ? capacity_words - W0 : 0;
  uint64_t nwords;
  if (p.fixed)
    nwords = (g0 + p.g.nblocks * (uint64_t)p.cp.maxbits + 63) / 64 + 1;
  else if (have_index)
    nwords = (g0 + index->total_bits + 63) / 64 + 1;
  else
    nwords = (g0 + p.g.nblocks * (uint64_t)p.max_len + 63) / 64 + 1;
  nwords = std::min<uint64_t>(nwords, avail);
  if ((p.fixed || have_index) && !dev_field && !dev_stream && !getenv("ZFP_HIP_NO_PIPE")) {
    std::vector<Slab> sl;
    if (make_slabs(job, field_base, p, p.fixed ? 1 : (p.dims == 4 ? kBlocks4PerWave : 64u), sl)) {
      const auto t0 = std::chrono::steady_clock::now();
      const int ok = by_type(p, [&](auto tag) {
        using S = std::remove_pointer_t<decltype(tag)>;
        return decompress_slabs<S>(c, p, sl, field_base, words, capacity_words, bit_offset, index, end_bit);
      });
      t_timing.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      t_timing.kernel_ms = 0;
      t_timing.timed = ok != 0;
      if (!ok) {
        c->idx_chk = nullptr;
        return 0;
      }
      return verified();
    }
  }
  HIP_TRY(hipEventRecord(c->ev[0], c->stream));
  const uint64_t* d_in = words + W0;
  if (!dev_stream) {
    if (!ensure(c->words, nwords * 8 + 8))
      return 0;
    HIP_TRY(hipMemcpyAsync(c->words.p, words + W0, nwords * 8, hipMemcpyHostToDevice, c->stream));
    d_in = (const uint64_t*)c->words.p;
  }
  if (scan) {
    if (!scan_index(c, p, d_in, nwords, g0, &c->scan_index))
      return 0;
    c->scan_index.start_bit = bit_offset;
    index = &c->scan_index;
  }
  const uint64_t total = p.fixed ? p.g.nblocks * (uint64_t)p.cp.maxbits : index->total_bits;
  void* d_field = field_base;
  char* d_img = nullptr;
  if (!dev_field) {
    size_t bytes = (size_t)(p.span_hi - p.span_lo + 1) * es;
    if (!ensure(c->field, bytes))
      return 0;
    d_img = (char*)c->field.p - p.span_lo * (int64_t)es;
    d_field = d_img;
  }
  int ok = by_type(p, [&](auto tag) {
    using S = std::remove_pointer_t<decltype(tag)>;
    return launch_decode<S>(c, p, (S*)d_field, d_in, nwords, g0, index);
  });
  if (!ok) {
    c->idx_chk = nullptr;
    return 0;
  }
  if (!dev_field && !copy_box(c, p, field_base, d_img, es, true))
    return 0;
  HIP_TRY(hipEventRecord(c->ev[3], c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  record_timing(c);
  *end_bit = bit_offset + total;
  return verified();
}

int zfp_hip_decompress(const zfp_hip_job* job, void* field_base, const uint64_t* words, uint64_t capacity_words,
                       uint64_t bit_offset, int device, const zfp_hip_index* index, uint64_t* end_bit)
{
  Plan p;
  if (!plan_job(job, field_base, p))
    return 0;
  if (!field_base || !words)
    return fail("zfp_hip_decompress: null field or stream pointer");
  if (zfp_hip_device_count() <= 0)
    return fail("zfp_hip_decompress: no HIP device available");
  CtxLease lease(device);
  Ctx* c = lease.c;
  if (!c)
    return 0;
  t_timing = Timing{};
  if (p.g.nblocks == 0) {
    *end_bit = bit_offset;
    return 1;
  }
  bool stale = false;
  int ok = decompress_once(c, p, job, field_base, words, capacity_words, bit_offset, index, end_bit, &stale);
  if (ok && stale) {
    // the caller's index passed the fingerprint but not the block lengths:
    // decode again with the block starts found by the scan
    ok = decompress_once(c, p, job, field_base, words, capacity_words, bit_offset, nullptr, end_bit, &stale);
    t_timing.stale_index = true;
  }
  return ok;
}

int zfp_hip_index_build(const zfp_hip_job* job, const uint64_t* words, uint64_t capacity_words, uint64_t bit_offset,
                        int device, zfp_hip_index* index)
{
  Plan p;
  if (!index)
    return fail("zfp_hip_index_build: null index");
  if (!plan_job(job, nullptr, p))
    return 0;
  if (p.fixed)
    return fail("zfp_hip_index_build: fixed-rate streams need no index");
  if (!words)
    return fail("zfp_hip_index_build: null stream");
  if (zfp_hip_device_count() <= 0)
    return fail("zfp_hip_index_build: no HIP device available");
  CtxLease lease(device);
  Ctx* c = lease.c;
  if (!c)
    return 0;
  t_timing = Timing{};
  const uint64_t W0 = bit_offset >> 6;
  const uint32_t g0 = (uint32_t)(bit_offset & 63);
  const uint64_t avail = capacity_words > W0 ? capacity_words - W0 : 0;
  const uint64_t nwords = std::min<uint64_t>((g0 + p.g.nblocks * (uint64_t)p.max_len + 63) / 64 + 1, avail);
  const uint64_t* d_in = words + W0;
  if (!is_device_ptr(words)) {
    if (!ensure(c->words, nwords * 8 + 8))
      return 0;
    HIP_TRY(hipMemcpyAsync(c->words.p, words + W0, nwords * 8, hipMemcpyHostToDevice, c->stream));
    d_in = (const uint64_t*)c->words.p;
  }
  if (p.g.nblocks == 0) {
    index->nblocks = 0;
    index->nwaves = 0;
    index->total_bits = 0;
  } else if (!scan_index(c, p, d_in, nwords, g0, index)) {
    return 0;
  }
  index_stamp(index, p);
  if (!stream_fingerprint(c, words, is_device_ptr(words), bit_offset, index->total_bits, &index->fp))
    return 0;
  index->start_bit = bit_offset;
  return 1;
}

zfp_hip_index* zfp_hip_index_create(void) { return new zfp_hip_index; }

void zfp_hip_index_free(zfp_hip_index* index)
{
  if (!index)
    return;
  index_release(index);
  delete index;
}

uint64_t zfp_hip_index_blocks(const zfp_hip_index* index) { return index ? index->nblocks : 0; }

// exported index: a 10-word head (tag, layout, bit count, fingerprint, codec
// settings), the per-block lengths, the per-wave bases
constexpr size_t kIndexHead = 80;
constexpr uint64_t kIndexTag = 0x337a6678646e69ull;  // "indxfz3"

size_t zfp_hip_index_export(const zfp_hip_index* index, void* buffer, size_t capacity)
{
  if (!index)
    return 0;
  size_t need = kIndexHead + index->nblocks * 2 + index->nwaves * 8;
  if (!buffer)
    return need;
  if (capacity < need)
    return 0;
  uint64_t* h = (uint64_t*)buffer;
  h[0] = kIndexTag;
  h[1] = index->nblocks;
  h[2] = index->nwaves;
  h[3] = index->total_bits;
  h[4] = index->per_wave;
  h[5] = index->start_bit;
  h[6] = index->fp;
  h[7] = ((uint64_t)index->maxbits << 32) | index->minbits;
  h[8] = ((uint64_t)(uint32_t)index->minexp << 32) | index->maxprec;
  h[9] = ((uint64_t)(uint32_t)index->dims << 32) | (uint32_t)index->type;
  char* q = (char*)buffer + kIndexHead;
  if (index->nblocks && hipMemcpy(q, index->d_len, index->nblocks * 2, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  q += index->nblocks * 2;
  if (index->nwaves && hipMemcpy(q, index->d_base, index->nwaves * 8, hipMemcpyDeviceToHost) != hipSuccess)
    return 0;
  return need;
}

zfp_hip_index* zfp_hip_index_import(const void* buffer, size_t bytes)
{
  if (!buffer || bytes < kIndexHead)
    return nullptr;
  const uint64_t* h = (const uint64_t*)buffer;
  if (h[0] != kIndexTag || h[1] > (1ull << 32) || h[2] > h[1] || bytes < kIndexHead + h[1] * 2 + h[2] * 8)
    return nullptr;
  zfp_hip_index* x = new zfp_hip_index;
  x->nblocks = h[1];
  x->nwaves = h[2];
  x->total_bits = h[3];
  x->per_wave = (uint32_t)h[4];
  x->start_bit = h[5];
  x->fp = h[6];
  x->minbits = (uint32_t)h[7];
  x->maxbits = (uint32_t)(h[7] >> 32);
  x->maxprec = (uint32_t)h[8];
  x->minexp = (int32_t)(uint32_t)(h[8] >> 32);
  x->type = (int32_t)(uint32_t)h[9];
  x->dims = (int32_t)(uint32_t)(h[9] >> 32);
  (void)hipGetDevice(&x->device);
  const char* q = (const char*)buffer + kIndexHead;
  if ((x->nblocks && hipMalloc(&x->d_len, x->nblocks * 2) != hipSuccess) ||
      (x->nwaves && hipMalloc(&x->d_base, x->nwaves * 8) != hipSuccess)) {
    zfp_hip_index_free(x);
    return nullptr;
  }
  x->cap_blocks = x->nblocks;
  x->cap_waves = x->nwaves;
  if (x->nblocks)
    (void)hipMemcpy(x->d_len, q, x->nblocks * 2, hipMemcpyHostToDevice);
  if (x->nwaves)
    (void)hipMemcpy(x->d_base, q + x->nblocks * 2, x->nwaves * 8, hipMemcpyHostToDevice);
  return x;
}

int zfp_hip_last_timing(double* kernel_ms, double* total_ms)
{
  if (!t_timing.timed)
    return 0;
  if (kernel_ms) *kernel_ms = t_timing.kernel_ms;
  if (total_ms) *total_ms = t_timing.total_ms;
  return 1;
}

int zfp_hip_last_stale_index(void) { return t_timing.stale_index ? 1 : 0; }

int zfp_hip_last_scan(double* scan_ms, int* passes)
{
  if (!t_timing.scan_passes)
    return 0;
  if (scan_ms) *scan_ms = t_timing.scan_ms;
  if (passes) *passes = t_timing.scan_passes;
  return 1;
}

size_t zfp_hip_scratch_bytes(void)
{
  std::lock_guard<std::mutex> lk(g_pool_mu);
  size_t b = 0;
  for (Ctx* c : g_idle) {
    for (const Scratch* s : {&c->field, &c->words, &c->status, &c->partials, &c->misc, &c->ovf, &c->scan_bm, &c->scan_seg,
                             &c->scan_tiles, &c->scan_pos})
      b += s->bytes;
    b += c->scan_index.cap_blocks * 2 + c->scan_index.cap_waves * 8;
  }
  return b;
}

int zfp_hip_release_scratch(void)
{
  std::vector<Ctx*> idle;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    idle.swap(g_idle);
  }
  for (Ctx* c : idle)
    destroy_ctx(c);
  return (int)idle.size();
}

}  // extern "C"
