// gsx-memprobe: how much device memory does this process (pod) get?
//
//   gsx-memprobe [--device N] [--alloc BYTES[,BYTES...]] [--hold-ms MS] [--touch]
//
// Prints hipMemGetInfo before and after, then tries each allocation in turn (kept until exit) and prints one
// JSON line.  Operators run it inside a pod to see the HBM share the device plugin's isolation library enforces
// (native/isolate/gsx_isolate.cc); tests/test_gpu_isolate.py drives it against the share and past it.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

int main(int argc, char** argv) {
  int dev = 0, hold_ms = 0;
  bool touch = false;
  std::vector<size_t> sizes;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--device") && i + 1 < argc) {
      dev = std::atoi(argv[++i]);
    } else if (!std::strcmp(argv[i], "--alloc") && i + 1 < argc) {
      std::string s(argv[++i]);
      size_t p = 0;
      while (p < s.size()) {
        size_t q = s.find(',', p);
        if (q == std::string::npos) q = s.size();
        sizes.push_back(std::strtoull(s.substr(p, q - p).c_str(), nullptr, 10));
        p = q + 1;
      }
    } else if (!std::strcmp(argv[i], "--hold-ms") && i + 1 < argc) {
      hold_ms = std::atoi(argv[++i]);
    } else if (!std::strcmp(argv[i], "--touch")) {
      touch = true;
    } else {
      std::fprintf(stderr, "usage: %s [--device N] [--alloc B,...] [--hold-ms MS] [--touch]\n", argv[0]);
      return 2;
    }
  }
  if (hipSetDevice(dev) != hipSuccess) {
    std::fprintf(stderr, "hipSetDevice(%d) failed\n", dev);
    return 1;
  }
  size_t free0 = 0, total0 = 0;
  hipError_t e = hipMemGetInfo(&free0, &total0);
  if (e != hipSuccess) {
    std::fprintf(stderr, "hipMemGetInfo: %s\n", hipGetErrorString(e));
    return 1;
  }
  std::vector<void*> held;
  std::string rows;
  for (size_t b : sizes) {
    void* p = nullptr;
    hipError_t r = hipMalloc(&p, b);
    if (r == hipSuccess && touch) r = hipMemset(p, 0x5a, b);
    if (r == hipSuccess) r = hipDeviceSynchronize();
    bool ok = r == hipSuccess && p != nullptr;
    if (ok) held.push_back(p);
    (void)hipGetLastError();  // an OOM is sticky in some HIP versions' last-error slot
    char buf[256];
    std::snprintf(buf, sizeof buf, "%s{\"bytes\":%zu,\"ok\":%s,\"err\":\"%s\"}", rows.empty() ? "" : ",", b,
                  ok ? "true" : "false", ok ? "" : hipGetErrorName(r));
    rows += buf;
  }
  size_t free1 = 0, total1 = 0;
  (void)hipMemGetInfo(&free1, &total1);
  std::printf("{\"device\":%d,\"total\":%zu,\"free\":%zu,\"allocs\":[%s],\"free_after\":%zu,\"total_after\":%zu}\n",
              dev, total0, free0, rows.c_str(), free1, total1);
  std::fflush(stdout);
  if (hold_ms > 0) usleep(static_cast<useconds_t>(hold_ms) * 1000u);
  for (void* p : held) (void)hipFree(p);
  return 0;
}
