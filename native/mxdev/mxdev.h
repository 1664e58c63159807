// mxdev: MI355X device discovery / health / topology over amdsmi.
//
// Replaces the NVML (cgo) layer of the upstream gpushare device plugin
// (docs/designs/designs.md:57-61): per-GPU VRAM total for the gpu-mem
// capacity, BDF / UUID / render+card minors for the /dev nodes handed to
// containers, KFD ids, compute/memory partition mode, RAS/ECC counters and
// reset / fault events for device health, and xGMI link types between GPUs.
//
// libamd_smi is dlopen()ed at run time with RTLD_DEEPBIND|RTLD_LOCAL, so the
// module loads on CPU-only hosts (the driver's build check), and the symbols
// never bind to the ROCm-SMI copy bundled inside the torch wheel.  A "fake"
// backend (e.g. "8x288GB") serves CPU tests with the same record layout.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace mxdev {

struct DeviceRec {
  int index = 0;           // HIP enumeration order
  std::string name;        // market name
  std::string arch = "gfx950";
  std::string bdf;         // dddd:bb:dd.f
  std::string uuid;
  uint64_t total_bytes = 0;  // VRAM total
  uint64_t used_bytes = 0;
  int cu_count = 0;
  int xcc_count = 8;
  int render_minor = -1;
  int card_minor = -1;
  int64_t kfd_id = -1;
  int hsa_id = -1;
  std::string partition = "SPX";
  std::string memory_partition;  // NPS1 / NPS2 / NPS4 / NPS8 (memory pools per physical GPU)
  int partition_id = 0;          // compute-partition index on its physical GPU (KFD current_partition_id)
  std::string pool;              // physical GPU key (BDF without the function): partitions of one GPU share it
  bool healthy = true;
  uint64_t ecc_uncorrectable = 0;
  uint64_t ecc_correctable = 0;
  // RAS: uncorrectable errors of the blocks a pod's work depends on (HBM/UMC, GFX, SDMA, xGMI WAFL)
  uint64_t ras_umc_uncorrectable = 0, ras_gfx_uncorrectable = 0, ras_sdma_uncorrectable = 0;
  uint64_t ras_xgmi_uncorrectable = 0, ras_xgmi_correctable = 0;
  int xgmi_error = 0;            // amdsmi_xgmi_status_t: 0 none, 1 error, 2 multiple errors
  bool thermal_throttle = false; // prochot / socket / HBM / VR thermal violation active
  bool power_throttle = false;   // package power tracking violation active
  std::string reason;            // why unhealthy ("" when healthy)
  int numa_node = -1;
  std::vector<std::string> link_types;  // per peer index: XGMI / PCIE / SELF / UNKNOWN
};

struct Event {
  int index;        // device index
  int type;         // amdsmi_evt_notification_type_t
  std::string name; // VMFAULT / THERMAL_THROTTLE / GPU_PRE_RESET / GPU_POST_RESET / ...
  std::string message;
};

class Backend {
 public:
  virtual ~Backend() = default;
  virtual std::string name() const = 0;
  virtual bool enumerate(std::vector<DeviceRec>* out, std::string* err) = 0;
  // refresh health counters of one device (ECC); false on error
  virtual bool health(int index, DeviceRec* rec, std::string* err) = 0;
  // start listening for reset / fault events on every device
  virtual bool watch_events(std::string* err) = 0;
  // wait up to timeout_ms for events
  virtual std::vector<Event> poll_events(int timeout_ms) = 0;
  // fake backend only: inject a fault / change ("ecc_uncorrectable=3", "xgmi_error=1", "thermal_throttle=1",
  // "partition=CPX", "memory_partition=NPS2", "event=GPU_PRE_RESET"); false + *err elsewhere
  virtual bool inject(int index, const std::string& what, std::string* err) {
    *err = "fault injection is only supported by the fake backend";
    return false;
  }
};

// healthy = no uncorrectable ECC / RAS error in HBM, GFX, SDMA or xGMI, and no xGMI link error; a thermal or
// power throttle is reported but does not make a device unhealthy (it slows pods, it does not corrupt them)
void classify(DeviceRec* r);

// "amdsmi", "fake:<spec>", or "auto" (amdsmi, error if unavailable).
Backend* make_backend(const std::string& kind, std::string* err);

// Parse "NxSIZE{GB,GiB,MiB,MB}[:SPX|DPX|QPX|CPX[:NPS1|NPS2|NPS4|NPS8]]" into fake device records.
// With a compute-partition mode every physical GPU appears as 1/2/4/8 logical devices (function number =
// partition id), each reporting the VRAM of the memory pool it sits in, as KFD does.
// XCDs per logical device on MI355X (8 XCDs per physical GPU) for a compute-partition mode.
int xcds_for_partition(const std::string& mode);
// Logical devices per physical GPU for a compute-partition mode.
int partitions_for_mode(const std::string& mode);

bool fake_spec(const std::string& spec, std::vector<DeviceRec>* out, std::string* err);

}  // namespace mxdev
