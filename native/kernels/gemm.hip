// bf16 MFMA GEMM family for the pod workload: C[M][N] = A[M][K] * B[N][K]^T (bf16 in/out, fp32 accumulate).
//
// One template, several tile shapes (BM x BN with WM x WN waves, BK = 64),
// selected at launch.  Structure per K-tile (see gsx_kernels.hip for the
// 128x128 original and the reasoning):
//   * global -> LDS with global_load_lds (16 B/lane), lane-linear LDS image,
//     XOR swizzle folded into the per-lane *global* source address;
//   * two LDS buffers: tile k+1 in flight while the MFMAs consume tile k;
//     one barrier per K-tile;
//   * v_mfma_f32_16x16x32_bf16, each wave owns a (BM/WM) x (BN/WN) C tile;
//   * s_setprio around the MFMA burst so the partner wave's loads issue;
//   * grouped, XCD-aware tile order (GROUP_M tile-rows per group; workgroup
//     ids remapped bijectively so one XCD's blocks share A/B panels in L2);
//   * epilogue through LDS: 16-B coalesced row stores.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace gsxgemm {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef const void __attribute__((address_space(1)))* gptr_t;
typedef void __attribute__((address_space(3)))* lptr_t;

constexpr int BK = 64;

__device__ __forceinline__ uint32_t swz(int row, int chunk) {
  return static_cast<uint32_t>(row * (BK * 2) + ((chunk ^ ((row >> 1) & 7)) << 4));
}

__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return static_cast<uint16_t>((u >> 16) | ((u & 0xffff) ? 0x40 : 0));
  u += 0x7fffu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}

template <int BM, int BN, int WM, int WN, int GROUP_M>
__global__ __launch_bounds__(WM * WN * 64) void gemm_kernel(const uint16_t* __restrict__ A,
                                                           const uint16_t* __restrict__ B,
                                                           uint16_t* __restrict__ C, int M, int N, int K) {
  constexpr int NW = WM * WN;
  constexpr int TA = BM * BK * 2, TB = BN * BK * 2;  // bytes per operand tile
  constexpr int MR = BM / WM / 16, NR = BN / WN / 16;
  constexpr int RA = TA / 1024 / NW, RB = TB / 1024 / NW;  // glds rounds per wave (1 KiB each)
  static_assert(RA >= 1 && RB >= 1 && TA % (1024 * NW) == 0 && TB % (1024 * NW) == 0, "tile/wave mismatch");
  constexpr int WTM = BM / WM, WTN = BN / WN;  // wave tile
  static_assert(NW * WTM * WTN * 2 <= 2 * (TA + TB), "epilogue staging must fit in LDS");
  extern __shared__ __attribute__((aligned(16))) char lds[];  // [buf][A|B], reused by the epilogue

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid / WN, wc = wid % WN;

  // XCD-aware bijective remap, then grouped tile order
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int ntm = M / BM, ntn = N / BN;
  const int per_group = GROUP_M * ntn;
  const int g = wg / per_group;
  const int first_m = g * GROUP_M;
  const int gm = (ntm - first_m) < GROUP_M ? (ntm - first_m) : GROUP_M;
  const int tm = first_m + (wg % per_group) % gm;
  const int tn = (wg % per_group) / gm;
  const int row0 = tm * BM, col0 = tn * BN;

  int offA[RA], offB[RB];
#pragma unroll
  for (int i = 0; i < RA; ++i) {
    const int p = (i * NW + wid) * 64 + lane;
    const int rr = p >> 3, slot = p & 7;
    offA[i] = rr * K + ((slot ^ ((rr >> 1) & 7)) * 8);
  }
#pragma unroll
  for (int i = 0; i < RB; ++i) {
    const int p = (i * NW + wid) * 64 + lane;
    const int rr = p >> 3, slot = p & 7;
    offB[i] = rr * K + ((slot ^ ((rr >> 1) & 7)) * 8);
  }
  const uint16_t* Ab = A + static_cast<size_t>(row0) * K;
  const uint16_t* Bb = B + static_cast<size_t>(col0) * K;

  auto stage = [&](int kt, int buf) {
    char* la = lds + buf * (TA + TB);
    char* lb = la + TA;
#pragma unroll
    for (int i = 0; i < RA; ++i)
      __builtin_amdgcn_global_load_lds((gptr_t)(Ab + offA[i] + kt * BK), (lptr_t)(la + (i * NW + wid) * 1024), 16,
                                       0, 0);
#pragma unroll
    for (int i = 0; i < RB; ++i)
      __builtin_amdgcn_global_load_lds((gptr_t)(Bb + offB[i] + kt * BK), (lptr_t)(lb + (i * NW + wid) * 1024), 16,
                                       0, 0);
  };

  f32x4 acc[MR][NR];
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  stage(0, 0);
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) stage(kt + 1, buf ^ 1);
    const char* la = lds + buf * (TA + TB);
    const char* lb = la + TA;
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      const int ch = kk * 4 + fq;
      bf16x8 bfr[NR];
#pragma unroll
      for (int n = 0; n < NR; ++n) bfr[n] = *reinterpret_cast<const bf16x8*>(lb + swz(wc * WTN + n * 16 + fr, ch));
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(la + swz(wr * WTM + m * 16 + fr, ch));
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int n = 0; n < NR; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[n], acc[m][n], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    __syncthreads();
  }
  // epilogue through LDS (wave-private region): bf16 tile, then 16-B row stores
  uint16_t* ct = reinterpret_cast<uint16_t*>(lds + wid * (WTM * WTN * 2));
#pragma unroll
  for (int m = 0; m < MR; ++m)
#pragma unroll
    for (int n = 0; n < NR; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j) ct[(m * 16 + fq * 4 + j) * WTN + n * 16 + fr] = f2bf(acc[m][n][j]);
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  constexpr int LPR = WTN / 8;   // lanes per row (16 B each)
  constexpr int RPI = 64 / LPR;  // rows per store instruction
#pragma unroll
  for (int i = 0; i < WTM / RPI; ++i) {
    const int rr = i * RPI + lane / LPR, cc = (lane % LPR) * 8;
    const uint4 v = *reinterpret_cast<const uint4*>(ct + rr * WTN + cc);
    *reinterpret_cast<uint4*>(C + static_cast<size_t>(row0 + wr * WTM + rr) * N + col0 + wc * WTN + cc) = v;
  }
}

// ---------------------------------------------------------------------------
// Phased 256x256 kernel: the prefetch stays in flight across barriers.
//
// The kernel above ends every K-tile with __syncthreads(), which hipcc lowers
// to `s_waitcnt vmcnt(0); s_barrier`: the next tile's loads are drained every
// 64 K, and at one 512-thread block per CU nothing hides that.  Here a K-tile
// is four phases; each phase MFMAs one quadrant of the wave's 128x64 C tile
// (16 MFMAs) and issues one *half-tile* (16 KiB: 128 rows x 64 k of A or B)
// two K-tiles ahead.  Waits are counted (`vmcnt(8)` = four half-tiles may stay
// in flight), barriers are raw s_barrier, and the two wave groups (wr = 0/1,
// one of each per SIMD) run one barrier apart so that one wave's ds_reads
// overlap the other's MFMAs.
//
// Half-tiles (LDS regions of 16 KiB, [buffer = tile & 1][half]):
//   0: A rows {0-63, 128-191}  1: A rows {64-127, 192-255}   (m-half of each wave row)
//   2: B cols {wc*64 + 0..31}  3: B cols {wc*64 + 32..63}     (n-half of each wave col)
// Per K-tile phases (reads -> MFMA quadrant, and what is staged):
//   p0: read A0,B2 -> (m0,n0)   stage tile t+1 half 3
//   p1: read B3    -> (m0,n1)   stage tile t+1 half 1
//   p2: read A1    -> (m1,n1)   stage tile t+2 half 0
//   p3: -          -> (m1,n0)   stage tile t+2 half 2
// Every half is restaged >= 2 phases after its last read (WAR across the
// staggered groups) and waited for (vmcnt(8) before the first barrier of the
// phase) one phase before it is read (RAW).  Tiles past the end are clamped to
// the last tile so the counts stay uniform; those loads land in dead buffers.
// ---------------------------------------------------------------------------
constexpr int PH_HALF = 128 * BK * 2;  // 16 KiB

__device__ __forceinline__ void ph_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// M32: the same schedule on v_mfma_f32_32x32x16_bf16 (per quadrant 2 x 1 blocks of 32x32 over 4 k-steps: 8 MFMAs
// of twice the work instead of 16), for the A/B the MFMA-shape rule asks for (the chip may hold a different clock
// on the other shape; same LDS bytes, same registers).
template <int GROUP_M, bool M32 = false>
__global__ __launch_bounds__(512) void gemm_phased_kernel(const uint16_t* __restrict__ A,
                                                         const uint16_t* __restrict__ B, uint16_t* __restrict__ C,
                                                         int M, int N, int K) {
  constexpr int BM = 256, BN = 256, WTM = 128, WTN = 64;
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;

  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int ntm = M / BM, ntn = N / BN;
  const int per_group = GROUP_M * ntn;
  const int g = wg / per_group;
  const int first_m = g * GROUP_M;
  const int gm = (ntm - first_m) < GROUP_M ? (ntm - first_m) : GROUP_M;
  const int tm = first_m + (wg % per_group) % gm;
  const int tn = (wg % per_group) / gm;
  const uint16_t* Ab = A + static_cast<size_t>(tm * BM) * K;
  const uint16_t* Bb = B + static_cast<size_t>(tn * BN) * K;

  // per-lane source offsets of the two 8-KiB rounds of each half
  int off[4][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = (i * 8 + wid) * 64 + lane;
    const int lr = p >> 3, slot = p & 7;
    const int sw = (slot ^ ((lr >> 1) & 7)) * 8;
    off[0][i] = ((lr >> 6) * 128 + (lr & 63)) * K + sw;
    off[1][i] = ((lr >> 6) * 128 + 64 + (lr & 63)) * K + sw;
    off[2][i] = ((lr >> 5) * 64 + (lr & 31)) * K + sw;
    off[3][i] = ((lr >> 5) * 64 + 32 + (lr & 31)) * K + sw;
  }
  const int nk = K / BK;
  auto stage = [&](int tile, int half) {
    const int kt = tile < nk ? tile : nk - 1;
    const uint16_t* src = (half < 2 ? Ab : Bb) + kt * BK;
    char* dst = lds + ((tile & 1) * 4 + half) * PH_HALF + wid * 1024;
    __builtin_amdgcn_global_load_lds((gptr_t)(src + off[half][0]), (lptr_t)dst, 16, 0, 0);
    __builtin_amdgcn_global_load_lds((gptr_t)(src + off[half][1]), (lptr_t)(dst + 8 * 1024), 16, 0, 0);
  };

  f32x4 acc[8][4];
  f32x16 acc32[4][2];  // M32: [32-row block][32-col block] of the wave's 128x64 tile
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc32[m][n][j] = 0.f;

  const int fr = lane & 15, fq = lane >> 4;
  const int r32 = lane & 31, h32 = lane >> 5;  // M32 operand maps: row / column lane & 31, k = 8 (lane >> 5) + j
  bf16x8 af[4][2], bf[2][2][2];  // A: [m][kk]; B: [nh][n][kk]  (M32: A [b][kk], B [nh][kk], k-steps of 16)

  auto read_a = [&](const char* base, int mh) {
    const char* h = base + mh * PH_HALF;
    if constexpr (M32) {
#pragma unroll
      for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk)
          af[b * 2 + (kk >> 1)][kk & 1] =
              *reinterpret_cast<const bf16x8*>(h + swz(wr * 64 + b * 32 + r32, kk * 2 + h32));
    } else {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          af[m][kk] = *reinterpret_cast<const bf16x8*>(h + swz(wr * 64 + m * 16 + fr, kk * 4 + fq));
    }
  };
  auto read_b = [&](const char* base, int nh) {
    const char* h = base + (2 + nh) * PH_HALF;
    if constexpr (M32) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
        bf[nh][kk >> 1][kk & 1] = *reinterpret_cast<const bf16x8*>(h + swz(wc * 32 + r32, kk * 2 + h32));
    } else {
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          bf[nh][n][kk] = *reinterpret_cast<const bf16x8*>(h + swz(wc * 32 + n * 16 + fr, kk * 4 + fq));
    }
  };
  auto mma = [&](int mh, int nh) {
    __builtin_amdgcn_s_setprio(1);
    if constexpr (M32) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int b = 0; b < 2; ++b)
          acc32[mh * 2 + b][nh] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
              af[b * 2 + (kk >> 1)][kk & 1], bf[nh][kk >> 1][kk & 1], acc32[mh * 2 + b][nh], 0, 0, 0);
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int n = 0; n < 2; ++n)
            acc[mh * 4 + m][nh * 2 + n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m][kk], bf[nh][n][kk],
                                                                                 acc[mh * 4 + m][nh * 2 + n], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  };

  // prologue: what the steady state has issued before tile 0, phase 0
  stage(0, 0);
  stage(0, 2);
  stage(0, 3);
  stage(0, 1);
  stage(1, 0);
  stage(1, 2);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  ph_barrier();
  if (wr == 1) ph_barrier();  // stagger the groups by one barrier

  for (int t = 0; t < nk; ++t) {
    const char* base = lds + (t & 1) * 4 * PH_HALF;
    // p0
    read_a(base, 0);
    read_b(base, 0);
    stage(t + 1, 3);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    ph_barrier();
    mma(0, 0);
    ph_barrier();
    // p1
    read_b(base, 1);
    stage(t + 1, 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    ph_barrier();
    mma(0, 1);
    ph_barrier();
    // p2
    read_a(base, 1);
    stage(t + 2, 0);
    ph_barrier();
    mma(1, 1);
    ph_barrier();
    // p3
    stage(t + 2, 2);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    ph_barrier();
    mma(1, 0);
    ph_barrier();
  }
  if (wr == 0) ph_barrier();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  ph_barrier();

  uint16_t* ct = reinterpret_cast<uint16_t*>(lds + wid * (WTM * WTN * 2));
  if constexpr (M32) {
    // 32x32 C map: column lane & 31, row (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 2; ++n)
#pragma unroll
        for (int j = 0; j < 16; ++j)
          ct[(m * 32 + (j & 3) + 8 * (j >> 2) + 4 * h32) * WTN + n * 32 + r32] = f2bf(acc32[m][n][j]);
  } else {
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) ct[(m * 16 + fq * 4 + j) * WTN + n * 16 + fr] = f2bf(acc[m][n][j]);
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  constexpr int LPR = WTN / 8, RPI = 64 / LPR;
  const int row0 = tm * BM + wr * WTM, col0 = tn * BN + wc * WTN;
#pragma unroll
  for (int i = 0; i < WTM / RPI; ++i) {
    const int rr = i * RPI + lane / LPR, cc = (lane % LPR) * 8;
    const uint4 v = *reinterpret_cast<const uint4*>(ct + rr * WTN + cc);
    *reinterpret_cast<uint4*>(C + static_cast<size_t>(row0 + rr) * N + col0 + cc) = v;
  }
}

template <int GM, bool M32 = false>
hipError_t launch_phased(hipStream_t s, const void* A, const void* B, void* C, int M, int N, int K) {
  constexpr int lds = 8 * PH_HALF;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_phased_kernel<GM, M32>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  if (M % 256 || N % 256 || K % BK) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm_phased_kernel<GM, M32>), dim3((M / 256) * (N / 256)), dim3(512), lds, s,
                     static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), M,
                     N, K);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// 4-wave 256x256 kernel: one wave per SIMD, 128x128 C per wave.
//
// rocprofv3 on the 8-wave kernels showed 1.57x the LDS instructions of
// hipBLASLt's 256x256 kernel: a 128x64 wave tile re-reads A once per 64
// columns.  A 128x128 wave tile halves that (LDS bytes per FLOP 0.75x), at
// the price of 256 fp32 accumulators per lane — AGPRs, which gfx950 has when
// a wave owns its SIMD (waves_per_eu = 1, 512 registers per lane).
//
// With no partner wave on the SIMD, latency is hidden inside the wave: the
// K loop runs in k32 sub-steps, and the fragments of sub-step s+1 (16
// ds_read_b128) are issued before the 64 MFMAs of sub-step s (register
// double buffer).  LDS holds two K-tiles (2 x 64 KiB); tile t+2 is staged
// into tile t's buffer as soon as every wave has read it, and waited for
// with a counted vmcnt(16) (one tile of loads stays in flight) one sub-step
// before it is read.  Past-the-end tiles are clamped (dead buffers).
//
// Measured (MI355X, random bf16, profiles/r01_rocprof_bench_gemm.md): LDS
// instructions drop to hipBLASLt's level (18.0M vs 16.8M at 8192^3; the
// 8-wave kernels issue 26.4M), but the kernel runs at 1.04-1.18 PFLOP/s, below
// the phased 8-wave kernel (1.41-1.47): hipcc (ROCm 7.2) keeps 256
// accumulators in AGPRs only with v_accvgpr_mov copies and s_nops between the
// MFMAs of the inner loop.  With the MFMAs in inline asm ("+a" pins the
// accumulators, ASM=true) the loop is clean — 8 MFMAs, 16 prefetch ds_reads,
// 56 MFMAs per sub-step, no copies — and reaches 1.11-1.22 PFLOP/s: with one
// wave per SIMD nothing fills the MFMA pipe across the two barriers per
// K-tile, which the staggered 8-wave kernel hides.  Kept as ablations; not
// dispatched by default.
// ---------------------------------------------------------------------------
template <int GROUP_M, bool ASM>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_w4_kernel(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, uint16_t* __restrict__ C, int M, int N, int K) {
  constexpr int BM = 256, BN = 256, WT = 128;
  constexpr int TILE = 256 * BK * 2;  // 32 KiB per operand per K-tile
  extern __shared__ __attribute__((aligned(16))) char lds[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;

  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int xcd = orig & 7;
  const int q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int ntm = M / BM, ntn = N / BN;
  const int per_group = GROUP_M * ntn;
  const int g = wg / per_group;
  const int first_m = g * GROUP_M;
  const int gm = (ntm - first_m) < GROUP_M ? (ntm - first_m) : GROUP_M;
  const int tm = first_m + (wg % per_group) % gm;
  const int tn = (wg % per_group) / gm;
  const uint16_t* Ab = A + static_cast<size_t>(tm * BM) * K;
  const uint16_t* Bb = B + static_cast<size_t>(tn * BN) * K;

  int off[8];  // 8 rounds of 4 KiB (256 lanes x 16 B) cover one 256-row operand tile
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int p = (i * 4 + wid) * 64 + lane;
    const int row = p >> 3, slot = p & 7;
    off[i] = row * K + (slot ^ ((row >> 1) & 7)) * 8;
  }
  const int nk = K / BK;
  auto stage = [&](int tile) {
    const int kt = tile < nk ? tile : nk - 1;
    char* la = lds + (tile & 1) * 2 * TILE;
    char* lb = la + TILE;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      __builtin_amdgcn_global_load_lds((gptr_t)(Ab + off[i] + kt * BK), (lptr_t)(la + (i * 4 + wid) * 1024), 16, 0,
                                       0);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      __builtin_amdgcn_global_load_lds((gptr_t)(Bb + off[i] + kt * BK), (lptr_t)(lb + (i * 4 + wid) * 1024), 16, 0,
                                       0);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  bf16x8 af[2][8], bfr[2][8];
  auto read = [&](int set, int tile, int kk) {
    const char* la = lds + (tile & 1) * 2 * TILE;
    const char* lb = la + TILE;
#pragma unroll
    for (int m = 0; m < 8; ++m)
      af[set][m] = *reinterpret_cast<const bf16x8*>(la + swz(wr * WT + m * 16 + fr, kk * 4 + fq));
#pragma unroll
    for (int n = 0; n < 8; ++n)
      bfr[set][n] = *reinterpret_cast<const bf16x8*>(lb + swz(wc * WT + n * 16 + fr, kk * 4 + fq));
  };
  // 64 MFMAs of one k32 sub-step; `prefetch` (the next sub-step's ds_reads) is issued after the
  // first row of 8, so the wait for this sub-step's fragments never covers the prefetch
  auto mma = [&](int set, int pf_tile, int pf_kk) {
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        if (m == 1 && n == 0) {
          __builtin_amdgcn_sched_barrier(0);
          read(set ^ 1, pf_tile, pf_kk);
          __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (ASM) {
          // accumulator pinned to AGPRs ("+a"): no accumulator copies between the MFMAs
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[m][n]) : "v"(af[set][m]), "v"(bfr[set][n]));
        } else {
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[set][m], bfr[set][n], acc[m][n], 0, 0, 0);
        }
      }
  };

  stage(0);
  stage(1);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  ph_barrier();
  read(0, 0, 0);
  for (int t = 0; t < nk; ++t) {
    // sub-step (t, k 0..31): fragments of (t, k 32..63) in flight under the MFMAs
    mma(0, t, 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ph_barrier();  // every wave is done with tile t's buffer
    stage(t + 2);
    // sub-step (t, k 32..63): tile t+1 must have landed (tile t+2's 16 loads stay in flight)
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    ph_barrier();
    // unconditional (no phi copies); the last one reads a dead buffer, never used
    mma(1, t + 1, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (ASM) {
    // the compiler cannot see the asm MFMAs: cover the MFMA-write -> VALU-read (v_accvgpr_read) hazard
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  }
  ph_barrier();

  // epilogue: wave-private 128x128 bf16 staging (32 KiB per wave), 16-B row stores
  uint16_t* ct = reinterpret_cast<uint16_t*>(lds + wid * (WT * WT * 2));
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int n = 0; n < 8; ++n)
#pragma unroll
      for (int j = 0; j < 4; ++j) ct[(m * 16 + fq * 4 + j) * WT + n * 16 + fr] = f2bf(acc[m][n][j]);
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  constexpr int LPR = WT / 8, RPI = 64 / LPR;
  const int row0 = tm * BM + wr * WT, col0 = tn * BN + wc * WT;
#pragma unroll
  for (int i = 0; i < WT / RPI; ++i) {
    const int rr = i * RPI + lane / LPR, cc = (lane % LPR) * 8;
    const uint4 v = *reinterpret_cast<const uint4*>(ct + rr * WT + cc);
    *reinterpret_cast<uint4*>(C + static_cast<size_t>(row0 + rr) * N + col0 + cc) = v;
  }
}

template <int GM, bool ASM>
hipError_t launch_w4(hipStream_t s, const void* A, const void* B, void* C, int M, int N, int K) {
  constexpr int lds = 4 * 256 * BK * 2;  // 128 KiB
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_w4_kernel<GM, ASM>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  if (M % 256 || N % 256 || K % BK) return hipErrorInvalidValue;
  hipLaunchKernelGGL((gemm_w4_kernel<GM, ASM>), dim3((M / 256) * (N / 256)), dim3(256), lds, s,
                     static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), M,
                     N, K);
  return hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int GM>
hipError_t launch(hipStream_t s, const void* A, const void* B, void* C, int M, int N, int K) {
  constexpr int lds = 2 * (BM + BN) * BK * 2;
  static bool attr = false;
  if (!attr) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_kernel<BM, BN, WM, WN, GM>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
    attr = true;
  }
  const int tiles = (M / BM) * (N / BN);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, WM, WN, GM>), dim3(tiles), dim3(WM * WN * 64), lds, s,
                     static_cast<const uint16_t*>(A), static_cast<const uint16_t*>(B), static_cast<uint16_t*>(C), M,
                     N, K);
  return hipGetLastError();
}

}  // namespace gsxgemm

// Tile configurations (index -> BM x BN, waves).  Exposed for benchmarking.
extern "C" int gsx_gemm_cfg_tile(int cfg, int* bm, int* bn) {
  static const int t[][2] = {{128, 128}, {256, 128}, {128, 256}, {256, 256}, {128, 128},
                             {256, 256}, {256, 256}, {256, 256}, {256, 256}, {256, 256}, {256, 256}};
  if (cfg < 0 || cfg > 10) return -1;
  *bm = t[cfg][0];
  *bn = t[cfg][1];
  return 0;
}

extern "C" int gsx_gemm_bf16_nt_launch_cfg(void* stream, const void* A, const void* B, void* C, int M, int N, int K,
                                           int cfg) {
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (cfg) {
    case 0: return static_cast<int>(gsxgemm::launch<128, 128, 2, 2, 8>(s, A, B, C, M, N, K));
    case 1: return static_cast<int>(gsxgemm::launch<256, 128, 4, 2, 4>(s, A, B, C, M, N, K));
    case 2: return static_cast<int>(gsxgemm::launch<128, 256, 2, 4, 8>(s, A, B, C, M, N, K));
    case 3: return static_cast<int>(gsxgemm::launch<256, 256, 2, 4, 4>(s, A, B, C, M, N, K));
    case 4: return static_cast<int>(gsxgemm::launch<128, 128, 2, 2, 1>(s, A, B, C, M, N, K));
    case 5: return static_cast<int>(gsxgemm::launch_phased<4>(s, A, B, C, M, N, K));
    case 6: return static_cast<int>(gsxgemm::launch_phased<8>(s, A, B, C, M, N, K));
    case 7: return static_cast<int>(gsxgemm::launch_w4<4, false>(s, A, B, C, M, N, K));
    case 8: return static_cast<int>(gsxgemm::launch_w4<8, false>(s, A, B, C, M, N, K));
    case 9: return static_cast<int>(gsxgemm::launch_w4<4, true>(s, A, B, C, M, N, K));
    case 10: return static_cast<int>(gsxgemm::launch_phased<4, true>(s, A, B, C, M, N, K));
    default: return static_cast<int>(hipErrorInvalidValue);
  }
}
