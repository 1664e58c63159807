// gsx-cuprobe: which compute units does a (CU-masked) queue actually use?
//
//   gsx-cuprobe [--device N] [--mask 0-63,128-191] [--blocks 8192] [--spin 20000] [--list]
//
// Launches the probe kernel (every workgroup records s_getreg HW_ID / XCC_ID)
// on a stream created with hipExtStreamCreateWithCUMask (or a plain stream,
// which still honours a process-wide HSA_CU_MASK), and prints one JSON line:
// distinct physical CUs in total and per XCD.  Operators run it inside a pod
// to check the partition the device plugin handed out; --list adds every CU as [xcc,se,sh,cu].
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#include "gsx_kernels.h"

static std::vector<uint32_t> parse_mask(const char* s, int cus) {
  std::vector<uint32_t> w(static_cast<size_t>((cus + 31) / 32), 0u);
  std::string str(s);
  size_t i = 0;
  while (i < str.size()) {
    size_t j = str.find(',', i);
    if (j == std::string::npos) j = str.size();
    std::string tok = str.substr(i, j - i);
    int a, b;
    size_t dash = tok.find('-');
    a = std::atoi(tok.c_str());
    b = dash == std::string::npos ? a : std::atoi(tok.c_str() + dash + 1);
    for (int c = a; c <= b && c < cus; ++c) w[static_cast<size_t>(c / 32)] |= 1u << (c % 32);
    i = j + 1;
  }
  return w;
}

int main(int argc, char** argv) {
  int dev = 0, blocks = 8192, spin = 20000;
  const char* mask = nullptr;
  bool list = false;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--device") && i + 1 < argc) dev = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--mask") && i + 1 < argc) mask = argv[++i];
    else if (!std::strcmp(argv[i], "--blocks") && i + 1 < argc) blocks = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--spin") && i + 1 < argc) spin = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--list")) list = true;
    // a program that drops a variable before its first HIP call (tests of the isolation library's hsa_init)
    else if (!std::strcmp(argv[i], "--unsetenv") && i + 1 < argc) unsetenv(argv[++i]);
    else {
      std::fprintf(stderr, "usage: %s [--device N] [--mask LIST] [--blocks N] [--spin N] [--list] [--unsetenv NAME]\n",
                   argv[0]);
      return 2;
    }
  }
  gsx_devinfo info;
  if (gsx_device_info(dev, &info) != 0) {
    std::fprintf(stderr, "device %d: %s\n", dev, gsx_last_error());
    return 1;
  }
  void* stream = nullptr;
  std::vector<uint32_t> words;
  if (mask) words = parse_mask(mask, info.cu_count);
  if (gsx_stream_create(dev, words.empty() ? nullptr : words.data(), static_cast<int>(words.size()), &stream) != 0) {
    std::fprintf(stderr, "stream: %s\n", gsx_last_error());
    return 1;
  }
  std::vector<uint32_t> rec(static_cast<size_t>(2 * blocks));
  if (gsx_cuprobe(stream, blocks, spin, rec.data()) != 0) {
    std::fprintf(stderr, "probe: %s\n", gsx_last_error());
    return 1;
  }
  std::set<std::tuple<int, int, int, int>> cus;
  std::vector<std::set<std::tuple<int, int, int>>> per_xcc(16);
  for (int b = 0; b < blocks; ++b) {
    uint32_t hw = rec[static_cast<size_t>(2 * b)], xcc = rec[static_cast<size_t>(2 * b + 1)] & 0xF;
    int cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
    cus.insert(std::make_tuple(static_cast<int>(xcc), se, sh, cu));
    per_xcc[xcc].insert(std::make_tuple(se, sh, cu));
  }
  std::printf("{\"device\":%d,\"arch\":\"%s\",\"cu_count\":%d,\"mask\":\"%s\",\"hsa_cu_mask\":\"%s\",\"distinct_cus\":%zu,"
              "\"per_xcd\":[",
              dev, info.arch, info.cu_count, mask ? mask : "", std::getenv("HSA_CU_MASK") ? std::getenv("HSA_CU_MASK") : "",
              cus.size());
  for (int x = 0; x < 8; ++x) std::printf("%s%zu", x ? "," : "", per_xcc[static_cast<size_t>(x)].size());
  std::printf("]");
  if (list) {
    std::printf(",\"cus\":[");
    bool first = true;
    for (const auto& t : cus) {
      std::printf("%s[%d,%d,%d,%d]", first ? "" : ",", std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t));
      first = false;
    }
    std::printf("]");
  }
  std::printf("}\n");
  gsx_stream_destroy(stream);
  return 0;
}
