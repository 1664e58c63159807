// MI355X (gfx950 / CDNA4) kernels of the GPU-share stack.  See gsx_kernels.h.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "gsx_kernels.h"

extern "C" int gsx_gemm_bf16_nt_launch_cfg(void* stream, const void* A, const void* B, void* C, int M, int N, int K,
                                           int cfg);

namespace {

thread_local std::string g_err;

int fail(hipError_t e, const char* what) {
  char buf[256];
  std::snprintf(buf, sizeof(buf), "%s: %s (%d)", what, hipGetErrorString(e), static_cast<int>(e));
  g_err = buf;
  return static_cast<int>(e);
}

int fail_arg(const char* what) {
  g_err = what;
  return static_cast<int>(hipErrorInvalidValue);
}

#define GSX_CHECK(call)                       \
  do {                                        \
    hipError_t _e = (call);                   \
    if (_e != hipSuccess) return fail(_e, #call); \
  } while (0)

// ------------------------------------------------------------------ CU probe

__global__ __launch_bounds__(64) void cuprobe_kernel(uint32_t* out, int spin) {
  uint32_t hw, xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  // keep the workgroup resident for a while so the dispatcher spreads the
  // grid over every CU the queue's mask allows
  float x = static_cast<float>(threadIdx.x);
  for (int i = 0; i < spin; ++i) x = __builtin_fmaf(x, 1.0000001f, 0.5f);
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = hw;
    out[2 * blockIdx.x + 1] = xcc | (x == -1.0f ? 0x80000000u : 0u);
  }
}

// ------------------------------------------------------------------ HBM stamp / verify / fill

// 16-B aligned: one dwordx4 load / store per stamp.  With 8-B alignment the compiler split each access into two
// dwordx2, and both halves of a stamp missed L2 together: two DRAM reads per stamp (rocprofv3 PMC,
// profiles/r02_pmc_admit/)
struct alignas(16) Stamp {
  uint64_t tag;
  uint64_t off;
};
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));  // a stamp read as one 16-B vector

typedef const __attribute__((address_space(1))) u64x2* global_stamp_ptr;  // slice addresses are device memory

typedef __attribute__((address_space(1))) u64x2* global_stamp_wptr;

__device__ __forceinline__ u64x2 load_stamp(const char* p) { return *(global_stamp_ptr)(p); }
__device__ __forceinline__ void store_stamp(char* p, uint64_t tag, uint64_t off) {
  u64x2 v;
  v.x = tag;
  v.y = off;
  *(global_stamp_wptr)(p) = v;  // one global_store_dwordx4
}

__global__ __launch_bounds__(256) void stamp_kernel(char* base, uint64_t n, uint64_t stride, uint64_t tag) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    store_stamp(base + i * stride, tag, i * stride);
  }
}

__global__ __launch_bounds__(256) void verify_kernel(const char* base, uint64_t n, uint64_t stride, uint64_t tag,
                                                     unsigned long long* bad) {
  uint32_t mine = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const u64x2 s = load_stamp(base + i * stride);
    mine += (s.x != tag || s.y != i * stride) ? 1u : 0u;
  }
  // wave64 reduction, one atomic per wave
  for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
  if ((threadIdx.x & 63) == 0 && mine) atomicAdd(bad, static_cast<unsigned long long>(mine));
}

constexpr int kMaxSlices = 32;
struct SliceTable {
  gsx_slice s[kMaxSlices];
  int n;
};

// grid.y = slice; each block strides over that slice's stamps
__global__ __launch_bounds__(256) void verify_slices_kernel(SliceTable t, uint64_t stride, unsigned long long* bad) {
  const gsx_slice sl = t.s[blockIdx.y];
  const uint64_t n = sl.bytes / stride;
  const char* base = reinterpret_cast<const char*>(sl.addr);
  uint32_t mine = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const u64x2 st = load_stamp(base + i * stride);
    mine += (st.x != sl.tag || st.y != i * stride) ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
  if ((threadIdx.x & 63) == 0 && mine) atomicAdd_system(bad, static_cast<unsigned long long>(mine));
}

// grid.y = slice; each block strides over that slice's stamp positions
__global__ __launch_bounds__(256) void stamp_slices_kernel(SliceTable t, uint64_t stride) {
  const gsx_slice sl = t.s[blockIdx.y];
  const uint64_t n = sl.bytes / stride;
  char* base = reinterpret_cast<char*>(sl.addr);
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    store_stamp(base + i * stride, sl.tag, i * stride);
  }
}

// One launch per admission: grid.y rows [0, n_stamp) stamp the new extents, the other rows verify the resident
// ones.  Only used when the host has checked that no two extents of the table overlap, so the two kinds of block
// touch disjoint memory and need no ordering between them; with an overlap the two-launch path runs instead, and the
// verify launch counts the overwritten stamps.  The stamp rows do not read back what they wrote (the two-launch
// path verifies fresh stamps in its second launch): in this mode a fresh slice is first verified by the next
// admission on the device, so the two modes' bad counts differ by the current admission's own new stamps.
__global__ __launch_bounds__(256) void admit_slices_kernel(SliceTable t, int n_stamp, uint64_t stride,
                                                           unsigned long long* bad) {
  const gsx_slice sl = t.s[blockIdx.y];
  const uint64_t n = sl.bytes / stride;
  char* base = reinterpret_cast<char*>(sl.addr);
  if (static_cast<int>(blockIdx.y) < n_stamp) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
      store_stamp(base + i * stride, sl.tag, i * stride);
    }
    return;  // the whole block leaves together: blockIdx.y is uniform
  }
  uint32_t mine = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const u64x2 st = load_stamp(base + i * stride);
    mine += (st.x != sl.tag || st.y != i * stride) ? 1u : 0u;
  }
  for (int o = 32; o > 0; o >>= 1) mine += __shfl_xor(mine, o, 64);
  if ((threadIdx.x & 63) == 0 && mine) atomicAdd_system(bad, static_cast<unsigned long long>(mine));
}

__global__ __launch_bounds__(256) void fill_kernel(uint4* p, uint64_t n16, uint32_t pat) {
  uint4 v = make_uint4(pat, pat, pat, pat);
  uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t step = gridDim.x * 256ull;
  // 4 independent 16-B stores in flight per lane
  for (; i + 3 * step < n16; i += 4 * step) {
    p[i] = v;
    p[i + step] = v;
    p[i + 2 * step] = v;
    p[i + 3 * step] = v;
  }
  for (; i < n16; i += step) p[i] = v;
}

// ------------------------------------------------------------------ bf16 MFMA GEMM
// The kernels live in gemm.hip (templated tile family); gsx_gemm_bf16_nt
// picks the measured-best tile for the shape (profiles/r01_kernels.json).

std::mutex g_mu;
unsigned long long* g_counter[64] = {nullptr};
unsigned long long* g_host_counter[64] = {nullptr};  // pinned, device-visible
// One bad-stamp counter per device: its reset -> kernel launch -> readback sequence is held under the
// device's mutex, so concurrent callers on one device (e.g. two Python threads) never mix their counts.
std::mutex g_dev_mu[64];

hipStream_t S(void* s) { return reinterpret_cast<hipStream_t>(s); }

int grid_for(uint64_t n, int per_block, int max_blocks) {
  uint64_t g = (n + per_block - 1) / per_block;
  if (g > static_cast<uint64_t>(max_blocks)) g = max_blocks;
  return g < 1 ? 1 : static_cast<int>(g);
}

}  // namespace

extern "C" {

const char* gsx_last_error(void) { return g_err.c_str(); }

int gsx_device_count(int* n) {
  GSX_CHECK(hipGetDeviceCount(n));
  return 0;
}

int gsx_device_info(int dev, gsx_devinfo* out) {
  hipDeviceProp_t p;
  GSX_CHECK(hipGetDeviceProperties(&p, dev));
  std::memset(out, 0, sizeof(*out));
  std::snprintf(out->name, sizeof(out->name), "%s", p.name);
  std::snprintf(out->arch, sizeof(out->arch), "%s", p.gcnArchName);
  GSX_CHECK(hipDeviceGetPCIBusId(out->pci_bus_id, sizeof(out->pci_bus_id), dev));
  out->total_mem = p.totalGlobalMem;
  out->cu_count = p.multiProcessorCount;
  out->clock_khz = p.clockRate;
  out->wave_size = p.warpSize;
  out->lds_per_block = p.sharedMemPerBlock;
  return 0;
}

int gsx_mem_info(int dev, uint64_t* free_b, uint64_t* total_b) {
  GSX_CHECK(hipSetDevice(dev));
  size_t f = 0, t = 0;
  GSX_CHECK(hipMemGetInfo(&f, &t));
  *free_b = f;
  *total_b = t;
  return 0;
}

int gsx_set_device(int dev) {
  GSX_CHECK(hipSetDevice(dev));
  return 0;
}

int gsx_synchronize(int dev) {
  GSX_CHECK(hipSetDevice(dev));
  GSX_CHECK(hipDeviceSynchronize());
  return 0;
}

int gsx_stream_create(int dev, const uint32_t* cu_mask, int mask_words, void** stream) {
  GSX_CHECK(hipSetDevice(dev));
  hipStream_t s;
  if (mask_words > 0) {
    GSX_CHECK(hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(mask_words), cu_mask));
  } else {
    GSX_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  }
  *stream = s;
  return 0;
}

int gsx_stream_get_mask(void* stream, uint32_t* cu_mask, int mask_words) {
  GSX_CHECK(hipExtStreamGetCUMask(S(stream), static_cast<uint32_t>(mask_words), cu_mask));
  return 0;
}

int gsx_stream_destroy(void* stream) {
  GSX_CHECK(hipStreamDestroy(S(stream)));
  return 0;
}

int gsx_stream_sync(void* stream) {
  GSX_CHECK(hipStreamSynchronize(S(stream)));
  return 0;
}

int gsx_malloc(int dev, uint64_t bytes, void** ptr) {
  GSX_CHECK(hipSetDevice(dev));
  GSX_CHECK(hipMalloc(ptr, bytes));
  return 0;
}

int gsx_free(void* ptr) {
  GSX_CHECK(hipFree(ptr));
  return 0;
}

int gsx_memcpy_d2h(void* dst, const void* src, uint64_t bytes) {
  GSX_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return 0;
}

int gsx_memcpy_h2d(void* dst, const void* src, uint64_t bytes) {
  GSX_CHECK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
  return 0;
}

int gsx_cuprobe(void* stream, int blocks, int spin, uint32_t* out_host) {
  if (blocks <= 0 || blocks > (1 << 20) || spin < 0) return fail_arg("gsx_cuprobe: bad blocks/spin");
  uint32_t* d = nullptr;
  GSX_CHECK(hipMallocAsync(reinterpret_cast<void**>(&d), sizeof(uint32_t) * 2 * blocks, S(stream)));
  hipLaunchKernelGGL(cuprobe_kernel, dim3(blocks), dim3(64), 0, S(stream), d, spin);
  GSX_CHECK(hipGetLastError());
  GSX_CHECK(hipMemcpyAsync(out_host, d, sizeof(uint32_t) * 2 * blocks, hipMemcpyDeviceToHost, S(stream)));
  GSX_CHECK(hipFreeAsync(d, S(stream)));
  GSX_CHECK(hipStreamSynchronize(S(stream)));
  return 0;
}

int gsx_hbm_stamp(void* stream, void* base, uint64_t bytes, uint64_t stride, uint64_t tag) {
  if (!base || stride < sizeof(Stamp) || stride % 16) return fail_arg("gsx_hbm_stamp: stride must be >=16, %16");
  if (reinterpret_cast<uintptr_t>(base) % 16) return fail_arg("gsx_hbm_stamp: base not 16-B aligned");
  uint64_t n = bytes / stride;
  if (!n) return 0;
  hipLaunchKernelGGL(stamp_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0, S(stream), static_cast<char*>(base),
                     n, stride, tag);
  GSX_CHECK(hipGetLastError());
  return 0;
}

int gsx_hbm_verify(void* stream, const void* base, uint64_t bytes, uint64_t stride, uint64_t tag, uint64_t* bad) {
  if (!base || stride < sizeof(Stamp) || stride % 16) return fail_arg("gsx_hbm_verify: stride must be >=16, %16");
  if (reinterpret_cast<uintptr_t>(base) % 16) return fail_arg("gsx_hbm_verify: base not 16-B aligned");
  uint64_t n = bytes / stride;
  *bad = 0;
  if (!n) return 0;
  int dev = 0;
  GSX_CHECK(hipGetDevice(&dev));
  unsigned long long* ctr;
  {
    std::lock_guard<std::mutex> g(g_mu);
    if (dev < 0 || dev >= 64) return fail_arg("gsx_hbm_verify: device index");
    if (!g_counter[dev]) GSX_CHECK(hipMalloc(reinterpret_cast<void**>(&g_counter[dev]), 64));
    ctr = g_counter[dev];
  }
  std::lock_guard<std::mutex> dl(g_dev_mu[dev]);
  GSX_CHECK(hipMemsetAsync(ctr, 0, sizeof(unsigned long long), S(stream)));
  hipLaunchKernelGGL(verify_kernel, dim3(grid_for(n, 256, 8192)), dim3(256), 0, S(stream),
                     static_cast<const char*>(base), n, stride, tag, ctr);
  GSX_CHECK(hipGetLastError());
  unsigned long long h = 0;
  GSX_CHECK(hipMemcpyAsync(&h, ctr, sizeof(h), hipMemcpyDeviceToHost, S(stream)));
  GSX_CHECK(hipStreamSynchronize(S(stream)));
  *bad = h;
  return 0;
}

int gsx_hbm_admit(void* stream, const gsx_slice* slices, int n, int stamp_idx, uint64_t stride, uint64_t* bad) {
  *bad = 0;
  if (n < 0 || stride < sizeof(Stamp) || stride % 16) return fail_arg("gsx_hbm_admit: bad n/stride");
  for (int i = 0; i < n; ++i) {
    if (!slices[i].addr || slices[i].addr % 16) return fail_arg("gsx_hbm_admit: slice base not 16-B aligned");
  }
  if (stamp_idx >= n) return fail_arg("gsx_hbm_admit: stamp_idx out of range");
  if (stamp_idx >= 0) {
    const gsx_slice& s0 = slices[stamp_idx];
    uint64_t ns = s0.bytes / stride;
    if (ns) {
      hipLaunchKernelGGL(stamp_kernel, dim3(grid_for(ns, 256, 8192)), dim3(256), 0, S(stream),
                         reinterpret_cast<char*>(s0.addr), ns, stride, s0.tag);
      GSX_CHECK(hipGetLastError());
    }
  }
  if (n == 0) return 0;
  int dev = 0;
  GSX_CHECK(hipGetDevice(&dev));
  unsigned long long* hc;
  {
    std::lock_guard<std::mutex> g(g_mu);
    if (dev < 0 || dev >= 64) return fail_arg("gsx_hbm_admit: device index");
    if (!g_host_counter[dev]) {
      GSX_CHECK(hipHostMalloc(reinterpret_cast<void**>(&g_host_counter[dev]), 64, hipHostMallocCoherent));
    }
    hc = g_host_counter[dev];
  }
  std::lock_guard<std::mutex> dl(g_dev_mu[dev]);
  __atomic_store_n(hc, 0ull, __ATOMIC_SEQ_CST);
  uint64_t maxn = 0;
  for (int i = 0; i < n; ++i) maxn = std::max<uint64_t>(maxn, slices[i].bytes / stride);
  // one stamp per lane (up to 1024 blocks per slice).  Measured on MI355X: verifying 4 x 64 GiB at a
  // 1 MiB stride takes ~12 us with 64 or with 1024 blocks per slice -- every read opens its own DRAM page
  // and TLB entry, so translation, not per-lane latency, bounds it (profiles/r01_session7_gpu.md)
  const int gx = grid_for(maxn, 256, 1024);
  for (int base = 0; base < n; base += kMaxSlices) {
    SliceTable t;
    t.n = std::min(kMaxSlices, n - base);
    for (int i = 0; i < t.n; ++i) t.s[i] = slices[base + i];
    hipLaunchKernelGGL(verify_slices_kernel, dim3(gx, t.n), dim3(256), 0, S(stream), t, stride, hc);
    GSX_CHECK(hipGetLastError());
  }
  GSX_CHECK(hipStreamSynchronize(S(stream)));
  *bad = __atomic_load_n(hc, __ATOMIC_SEQ_CST);
  return 0;
}

int gsx_hbm_admit_n(void* stream, const gsx_slice* slices, int n, int n_stamp, int verify, uint64_t stride,
                    uint64_t* bad) {
  *bad = 0;
  if (n < 0 || n_stamp < 0 || n_stamp > n || stride < sizeof(Stamp) || stride % 16)
    return fail_arg("gsx_hbm_admit_n: bad n/n_stamp/stride");
  for (int i = 0; i < n; ++i) {
    if (!slices[i].addr || slices[i].addr % 16) return fail_arg("gsx_hbm_admit_n: slice base not 16-B aligned");
  }
  auto table_grid = [&](int from, int count, SliceTable* t) {
    t->n = count;
    uint64_t maxn = 0;
    for (int i = 0; i < count; ++i) {
      t->s[i] = slices[from + i];
      maxn = std::max<uint64_t>(maxn, slices[from + i].bytes / stride);
    }
    return grid_for(maxn, 256, 1024);
  };
  // one table, extents pairwise disjoint: stamp and verify can share one launch
  // (every pair: two new extents that overlap each other must be caught by the verify launch as well)
  // opt-in (GSX_ADMIT_ONE_LAUNCH=1): it cuts GPU time per admission (6.5 vs 10.2 us) but not the wall-clock of an
  // admission, and its kernel-time tail is longer; interleaved A/Bs of the driver's bench showed no gain
  // (profiles/r02_fused_admit/), so two launches stay the default.  Its contract is weaker: the fresh stamps are
  // written, not read back (the rows of one launch are unordered), so a bad count covers the resident slices only,
  // where the default path also verifies every new extent it just stamped
  static const bool one_launch = [] {
    const char* e = std::getenv("GSX_ADMIT_ONE_LAUNCH");
    return e && e[0] == '1';
  }();
  bool disjoint = one_launch && verify && n > 0 && n <= kMaxSlices;
  for (int i = 0; disjoint && i < n; ++i) {
    for (int j = i + 1; j < n; ++j) {
      const uint64_t a0 = slices[i].addr, a1 = a0 + slices[i].bytes;
      const uint64_t b0 = slices[j].addr, b1 = b0 + slices[j].bytes;
      if (a0 < b1 && b0 < a1) {
        disjoint = false;
        break;
      }
    }
  }
  if (disjoint) {
    int dev = 0;
    GSX_CHECK(hipGetDevice(&dev));
    unsigned long long* hc;
    {
      std::lock_guard<std::mutex> g(g_mu);
      if (dev < 0 || dev >= 64) return fail_arg("gsx_hbm_admit_n: device index");
      if (!g_host_counter[dev]) {
        GSX_CHECK(hipHostMalloc(reinterpret_cast<void**>(&g_host_counter[dev]), 64, hipHostMallocCoherent));
      }
      hc = g_host_counter[dev];
    }
    std::lock_guard<std::mutex> dl(g_dev_mu[dev]);
    __atomic_store_n(hc, 0ull, __ATOMIC_SEQ_CST);
    SliceTable t;
    const int gx = table_grid(0, n, &t);
    hipLaunchKernelGGL(admit_slices_kernel, dim3(gx, t.n), dim3(256), 0, S(stream), t, n_stamp, stride, hc);
    GSX_CHECK(hipGetLastError());
    GSX_CHECK(hipStreamSynchronize(S(stream)));
    *bad = __atomic_load_n(hc, __ATOMIC_SEQ_CST);
    return 0;
  }
  for (int base = 0; base < n_stamp; base += kMaxSlices) {
    SliceTable t;
    const int gx = table_grid(base, std::min(kMaxSlices, n_stamp - base), &t);
    hipLaunchKernelGGL(stamp_slices_kernel, dim3(gx, t.n), dim3(256), 0, S(stream), t, stride);
    GSX_CHECK(hipGetLastError());
  }
  if (!verify || n == 0) {
    GSX_CHECK(hipStreamSynchronize(S(stream)));
    return 0;
  }
  int dev = 0;
  GSX_CHECK(hipGetDevice(&dev));
  unsigned long long* hc;
  {
    std::lock_guard<std::mutex> g(g_mu);
    if (dev < 0 || dev >= 64) return fail_arg("gsx_hbm_admit_n: device index");
    if (!g_host_counter[dev]) {
      GSX_CHECK(hipHostMalloc(reinterpret_cast<void**>(&g_host_counter[dev]), 64, hipHostMallocCoherent));
    }
    hc = g_host_counter[dev];
  }
  std::lock_guard<std::mutex> dl(g_dev_mu[dev]);
  __atomic_store_n(hc, 0ull, __ATOMIC_SEQ_CST);
  for (int base = 0; base < n; base += kMaxSlices) {
    SliceTable t;
    const int gx = table_grid(base, std::min(kMaxSlices, n - base), &t);
    hipLaunchKernelGGL(verify_slices_kernel, dim3(gx, t.n), dim3(256), 0, S(stream), t, stride, hc);
    GSX_CHECK(hipGetLastError());
  }
  GSX_CHECK(hipStreamSynchronize(S(stream)));
  *bad = __atomic_load_n(hc, __ATOMIC_SEQ_CST);
  return 0;
}

int gsx_hbm_fill(void* stream, void* base, uint64_t bytes, uint32_t pattern) {
  if (!base || bytes % 16 || reinterpret_cast<uintptr_t>(base) % 16) return fail_arg("gsx_hbm_fill: need 16-B multiple");
  uint64_t n16 = bytes / 16;
  if (!n16) return 0;
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n16, 256 * 4, 256 * 16)), dim3(256), 0, S(stream),
                     static_cast<uint4*>(base), n16, pattern);
  GSX_CHECK(hipGetLastError());
  return 0;
}

int gsx_gemm_bf16_nt(void* stream, const void* A, const void* B, void* C, int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0 || M % 128 || N % 128 || K % 64)
    return fail_arg("gsx_gemm_bf16_nt: need M%128==0, N%128==0, K%64==0");
  if ((reinterpret_cast<uintptr_t>(A) | reinterpret_cast<uintptr_t>(B) | reinterpret_cast<uintptr_t>(C)) % 16)
    return fail_arg("gsx_gemm_bf16_nt: operands must be 16-B aligned");
  // phased 256x256 / 8 waves (prefetch in flight across barriers): 1.39-1.46 PFLOP/s on MI355X at
  // 4k-16k (the __syncthreads 256x256 tile: 1.12-1.21); 128x128 grouped otherwise
  const int cfg = (M % 256 == 0 && N % 256 == 0) ? 5 : 0;
  int rc = gsx_gemm_bf16_nt_launch_cfg(stream, A, B, C, M, N, K, cfg);
  if (rc != 0) return fail(static_cast<hipError_t>(rc), "gemm launch");
  return 0;
}

int gsx_event_time_gemm(void* stream, const void* A, const void* B, void* C, int M, int N, int K, int iters,
                        float* ms) {
  hipEvent_t e0, e1;
  GSX_CHECK(hipEventCreate(&e0));
  GSX_CHECK(hipEventCreate(&e1));
  GSX_CHECK(hipEventRecord(e0, S(stream)));
  for (int i = 0; i < iters; ++i) {
    int rc = gsx_gemm_bf16_nt(stream, A, B, C, M, N, K);
    if (rc) return rc;
  }
  GSX_CHECK(hipEventRecord(e1, S(stream)));
  GSX_CHECK(hipEventSynchronize(e1));
  GSX_CHECK(hipEventElapsedTime(ms, e0, e1));
  GSX_CHECK(hipEventDestroy(e0));
  GSX_CHECK(hipEventDestroy(e1));
  return 0;
}

}  // extern "C"
