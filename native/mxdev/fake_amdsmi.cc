// A stand-in for libamd_smi.so (test only, never shipped): the amdsmi C entry points libmxdev uses, over a topology
// in which amdsmi's enumeration order (PCI order) is NOT the HIP ordinal order -- what some MI355X platforms show
// (HIP numbers GPUs in KFD node order).  libmxdev must index devices by HIP ordinal (amdsmi_get_gpu_enumeration_info
// hip_id), so that "GPU i" means one device everywhere: the rank whose HBM arena lives on HIP device i, the
// device plugin's inventory entry i, and the /dev/dri/renderD node a container of GPU i is given.
//
//   GSX_FAKE_AMDSMI="<hip_id of amdsmi device 0>,<of device 1>,..."  (default "3,1,0,2,7,5,4,6": 8 GPUs, shuffled)
//
// amdsmi device k: BDF 0000:<0x11 + 0x10 k>:00.0, UUID "fake-smi-<k>", renderD<128 + k>, card<k>, hsa_id k + 1,
// VRAM 288 GiB - k MiB (every device's total tells which one it is).
#include <amd_smi/amdsmi.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {

std::vector<int> g_hip;     // amdsmi order -> hip_id
int g_socket = 0;           // one socket handle
std::vector<int> g_handles;  // processor handles: &g_handles[k]

int device_of(amdsmi_processor_handle h) {
  for (size_t k = 0; k < g_handles.size(); ++k)
    if (h == &g_handles[k]) return static_cast<int>(k);
  return -1;
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_init(uint64_t) {
  const char* s = std::getenv("GSX_FAKE_AMDSMI");
  std::string spec = s && *s ? s : "3,1,0,2,7,5,4,6";
  g_hip.clear();
  for (size_t i = 0; i < spec.size();) {
    size_t j = spec.find(',', i);
    if (j == std::string::npos) j = spec.size();
    g_hip.push_back(std::atoi(spec.substr(i, j - i).c_str()));
    i = j + 1;
  }
  g_handles.assign(g_hip.size(), 0);
  return AMDSMI_STATUS_SUCCESS;
}

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_shut_down() { return AMDSMI_STATUS_SUCCESS; }

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_socket_handles(uint32_t* n, amdsmi_socket_handle* out) {
  if (out && *n >= 1) out[0] = &g_socket;
  *n = 1;
  return AMDSMI_STATUS_SUCCESS;
}

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_processor_handles(amdsmi_socket_handle,
                                                                                       uint32_t* n,
                                                                                       amdsmi_processor_handle* out) {
  if (out) {
    for (uint32_t k = 0; k < *n && k < g_handles.size(); ++k) out[k] = &g_handles[k];
  }
  *n = static_cast<uint32_t>(g_handles.size());
  return AMDSMI_STATUS_SUCCESS;
}

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_processor_type(amdsmi_processor_handle,
                                                                                    processor_type_t* t) {
  *t = AMDSMI_PROCESSOR_TYPE_AMD_GPU;
  return AMDSMI_STATUS_SUCCESS;
}

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_gpu_device_bdf(amdsmi_processor_handle h,
                                                                                    amdsmi_bdf_t* b) {
  int k = device_of(h);
  if (k < 0) return AMDSMI_STATUS_INVAL;
  b->as_uint = 0;
  b->bus_number = static_cast<uint64_t>(0x11 + 0x10 * k);
  return AMDSMI_STATUS_SUCCESS;
}

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_gpu_device_uuid(amdsmi_processor_handle h,
                                                                                     unsigned int* len, char* uuid) {
  int k = device_of(h);
  if (k < 0) return AMDSMI_STATUS_INVAL;
  std::snprintf(uuid, *len, "fake-smi-%d", k);
  return AMDSMI_STATUS_SUCCESS;
}

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_gpu_enumeration_info(amdsmi_processor_handle h,
                                                                                          amdsmi_enumeration_info_t* e) {
  int k = device_of(h);
  if (k < 0) return AMDSMI_STATUS_INVAL;
  std::memset(e, 0, sizeof(*e));
  e->drm_render = static_cast<uint32_t>(128 + k);
  e->drm_card = static_cast<uint32_t>(k);
  e->hsa_id = static_cast<uint32_t>(k + 1);
  e->hip_id = static_cast<uint32_t>(g_hip[static_cast<size_t>(k)]);
  return AMDSMI_STATUS_SUCCESS;
}

__attribute__((visibility("default"))) amdsmi_status_t amdsmi_get_gpu_memory_total(amdsmi_processor_handle h,
                                                                                      amdsmi_memory_type_t,
                                                                                      uint64_t* total) {
  int k = device_of(h);
  if (k < 0) return AMDSMI_STATUS_INVAL;
  *total = (uint64_t{288} << 30) - (static_cast<uint64_t>(k) << 20);
  return AMDSMI_STATUS_SUCCESS;
}

}  // extern "C"
