// A kernel whose every lane keeps SCRATCH_INTS ints in private memory (scratch): built once per size as its own
// code object (gsx-scratch-<KiB>.hsaco, native/build.py tools) and loaded by `gsx-memprobe --scratch KIB`, so
// that the isolation library's load-time scratch check (native/isolate/gsx_isolate.cc: hook_freeze) judges
// each size on its own.
#include <hip/hip_runtime.h>

#ifndef SCRATCH_INTS
#define SCRATCH_INTS 256
#endif

extern "C" __global__ void __launch_bounds__(256) gsx_scratch_kernel(int* out, int seed) {
  volatile int a[SCRATCH_INTS];  // volatile + a data-dependent index: the array cannot live in registers
  const int t = static_cast<int>(threadIdx.x);
  for (int i = t % 64; i < SCRATCH_INTS; i += 64) a[i] = seed + i + t;
  int s = 0;
  for (int i = 0; i < SCRATCH_INTS; i += 64) s += a[(i + seed * t) & (SCRATCH_INTS - 1)];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
