// Wire-level model: naming profile, PodView / NodeView extraction.
//
// Mirrors the accessors of the reference's pkg/utils (pod.go, node.go,
// const.go) but works directly on the JSON tape of a v1.Pod / v1.Node so the
// extender never builds Python dicts on its hot paths.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "json.h"

namespace gsx {

// Resource / annotation names.  Default = the reference's "shared-gpu"
// profile (pkg/utils/const.go:4-12); the "aliyun" profile swaps the domain
// (aliyun.com/gpu-mem, ALIYUN_COM_GPU_MEM_*) as in docs/designs/bind.jpg.
struct Profile {
  std::string resource = "shared-gpu/gpu-mem";
  std::string count = "shared-gpu/gpu-count";
  std::string a_idx = "SHARED_GPU_MEM_IDX";
  std::string a_pod = "SHARED_GPU_MEM_POD";
  std::string a_dev = "SHARED_GPU_MEM_DEV";
  std::string a_assigned = "SHARED_GPU_MEM_ASSIGNED";
  std::string a_assume = "SHARED_GPU_MEM_ASSUME_TIME";
  // Node annotation published by our device plugin with per-device totals
  // ("268,268,...") so heterogeneous / partitioned devices are exact instead
  // of capacity/count integer division (reference pkg/cache/nodeinfo.go:34).
  std::string a_node_devs = "gpushare.amd.com/device-memory";
  // container env with the container's share (samples/docker/run.sh:3-6)
  std::string env_container = "SHARED_GPU_MEM_CONTAINER";
};

// "shared-gpu" (default, pkg/utils/const.go) or "aliyun" (docs/designs/bind.jpg).
Profile profile_by_name(const std::string& name);

struct PodView {
  std::string uid, name, ns, node, phase, rv;
  bool deleting = false;     // metadata.deletionTimestamp set
  int64_t request = 0;       // sum of container limits[resource] (pod.go:146-155)
  int64_t dev_idx = -1;      // annotation IDX, -1 if absent/invalid (pod.go:45-60)
  int64_t annot_mem = 0;     // annotation POD, clamped >= 0 (pod.go:94-113)
  bool has_annot_mem = false;
  int64_t annot_dev_total = -1;
  int assigned = -1;         // annotation ASSIGNED: -1 absent, 0 false, 1 true
  int64_t assume_time = -1;  // annotation ASSUME_TIME (unix ns)
  std::string cu_mask;       // optional per-pod CU mask annotation (isolation)
  // gpushare.amd.com/hold-idx: a second device the pod is charged on while the device plugin moves its
  // allocation record to the GPU kubelet really gave it (deviceplugin/reconcile.py); -1 if absent
  int64_t hold_idx = -1;

  bool terminal() const { return phase == "Succeeded" || phase == "Failed"; }
  // pod.go:28-37 IsCompletePod
  bool complete() const { return deleting || terminal(); }
  // pod.go:13-25 AssignedNonTerminatedPod
  bool assigned_non_terminated() const { return !deleting && !node.empty() && !terminal(); }
};

struct NodeView {
  std::string name;
  int64_t total = 0;  // capacity[resource] (node.go:14-22)
  int64_t count = 0;  // capacity[count] (node.go:24-30)
  std::vector<int64_t> dev_totals;  // optional per-device totals annotation
  std::string address;              // first InternalIP (kubectl-inspect output)
  // the node's device plugin matches Allocates in landing order (annotation gpushare.amd.com/allocate-order
  // = "landing", published by deviceplugin/plugin.py): binds need no ASSUME_TIME order there (ledger.h)
  bool landing_order = false;
  // the node's device plugin publishes its unaccounted GPU use to the extender (POST .../physical; annotation
  // gpushare.amd.com/physical-publication = "true", deviceplugin/plugin.py publish_node): after an extender (re)start
  // or a leader change, binds to the node wait for its first publication (ledger.h publication_wait)
  bool publishes = false;
};

inline constexpr const char* kAllocateOrderAnnotation = "gpushare.amd.com/allocate-order";
inline constexpr const char* kPhysicalPublicationAnnotation = "gpushare.amd.com/physical-publication";

// Extract a PodView from the pod object at tape index `pod`.
bool parse_pod(const json::Doc& d, uint32_t pod, const Profile& p, PodView* out);
// Same for a node object.
bool parse_node(const json::Doc& d, uint32_t node, const Profile& p, NodeView* out);

// A resource.Quantity (string or number) at tape index idx (-1: absent) as an integer (Quantity.Value()).
bool quantity_of(const json::Doc& d, int64_t idx, int64_t* out);

// Sum of container limits[name] of a pod object (init containers ignored,
// exactly like pod.go:146-155).
int64_t pod_limits_sum(const json::Doc& d, uint32_t pod, const std::string& name);

}  // namespace gsx
