// C ABI of libgsx_kernels.so: the MI355X (gfx950) device-side pieces of the
// GPU-share stack.  The reference has no GPU code at all;
// these are new capabilities that make the shares verifiable on hardware:
//
//  * CU probe            — every workgroup records the hardware XCC / SE / CU /
//                          SIMD it ran on (s_getreg HW_ID, XCC_ID), so a CU
//                          mask (the MPS stand-in of BASELINE.json) can be
//                          checked against what the hardware actually used;
//  * HBM stamp / verify  — a pod's gpu-mem slice is stamped with its tag and
//                          verified later: proves co-resident pods placed by
//                          the binpack allocator really fit and never overlap;
//  * HBM scrub           — full-bandwidth 16 B/lane fill used to wipe a slice
//                          when a pod leaves (and as the HBM roofline probe);
//  * bf16 MFMA GEMM      — the pod workload used to measure isolation
//                          (throughput under per-pod CU partitions);
//  * CU-masked streams   — hipExtStreamCreateWithCUMask.
//
// All functions return 0 or a hipError_t value; gsx_last_error() has text.
#pragma once

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  char name[64];
  char arch[32];
  char pci_bus_id[32];
  uint64_t total_mem;
  int32_t cu_count;
  int32_t xcc_count;  // not reported by HIP; filled from the probe by callers
  int32_t clock_khz;
  int32_t wave_size;
  uint64_t lds_per_block;
} gsx_devinfo;

const char* gsx_last_error(void);
int gsx_device_count(int* n);
int gsx_device_info(int dev, gsx_devinfo* out);
int gsx_mem_info(int dev, uint64_t* free_b, uint64_t* total_b);
int gsx_synchronize(int dev);
// Make `dev` current on the calling thread (native runtime threads launch admission kernels).
int gsx_set_device(int dev);

// streams (mask_words == 0: plain stream)
int gsx_stream_create(int dev, const uint32_t* cu_mask, int mask_words, void** stream);
int gsx_stream_get_mask(void* stream, uint32_t* cu_mask, int mask_words);
int gsx_stream_destroy(void* stream);
int gsx_stream_sync(void* stream);

// memory
int gsx_malloc(int dev, uint64_t bytes, void** ptr);
int gsx_free(void* ptr);
int gsx_memcpy_d2h(void* dst, const void* src, uint64_t bytes);
int gsx_memcpy_h2d(void* dst, const void* src, uint64_t bytes);

// CU probe: `blocks` workgroups of 64 threads each spin `spin` iterations and
// record (HW_ID, XCC_ID) into out[2*b] / out[2*b+1].  Runs on `stream`
// (may be a CU-masked stream) and synchronises it.
int gsx_cuprobe(void* stream, int blocks, int spin, uint32_t* out_host);

// HBM stamp/verify: 16-byte stamps {tag, offset} every `stride` bytes of
// [base, base+bytes).  verify returns the number of bad stamps in *bad.
int gsx_hbm_stamp(void* stream, void* base, uint64_t bytes, uint64_t stride, uint64_t tag);
int gsx_hbm_verify(void* stream, const void* base, uint64_t bytes, uint64_t stride, uint64_t tag, uint64_t* bad);
// Batched pod admission: optionally stamp slice `stamp_idx` (-1: none), then
// verify every slice in ONE launch; *bad = total bad stamps.  The bad-stamp
// counter lives in pinned host memory, so there is no memset / copy kernel
// and exactly one stream sync per call.
typedef struct {
  uint64_t addr;
  uint64_t bytes;
  uint64_t tag;
} gsx_slice;
int gsx_hbm_admit(void* stream, const gsx_slice* slices, int n, int stamp_idx, uint64_t stride, uint64_t* bad);
// Admission of a pod made of several extents (its slice is not contiguous when the arena is
// fragmented): stamp slices[0, n_stamp) in one launch, then (verify != 0) verify all n slices;
// one stream sync.
int gsx_hbm_admit_n(void* stream, const gsx_slice* slices, int n, int n_stamp, int verify, uint64_t stride,
                    uint64_t* bad);

// Fill [base, base+bytes) with a 32-bit pattern (bytes % 16 == 0).
int gsx_hbm_fill(void* stream, void* base, uint64_t bytes, uint32_t pattern);

// C[M][N] (bf16) = A[M][K] (bf16, row-major) * B[N][K]^T (bf16, row-major).
// Requires M % 128 == 0, N % 128 == 0, K % 64 == 0.  Dispatches to the best
// tile of the templated family in gemm.hip (256x256 when M, N % 256 == 0).
int gsx_gemm_bf16_nt(void* stream, const void* A, const void* B, void* C, int M, int N, int K);

// elapsed milliseconds of running `fn` on stream via hip events (for benches)
int gsx_event_time_gemm(void* stream, const void* A, const void* B, void* C, int M, int N, int K, int iters,
                        float* ms);

#ifdef __cplusplus
}
#endif
