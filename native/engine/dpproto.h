// Protobuf wire format of the kubelet device-plugin API v1beta1 (the messages this repo serves and calls), hand
// written like deviceplugin/api.py's descriptor: field numbers follow k8s.io/kubelet/pkg/apis/deviceplugin/
// v1beta1/api.proto.  Unknown fields are skipped on decode; maps are repeated {1: key, 2: value} entries.
#pragma once

#include <cstdint>
#include <functional>
#include <map>
#include <string>
#include <string_view>
#include <vector>

namespace gsx::dp {

struct DeviceMsg {
  std::string id, health;
  std::vector<int64_t> numa;
};

struct MountMsg {
  std::string container_path, host_path;
  bool read_only = false;
};

struct DeviceSpecMsg {
  std::string container_path, host_path, permissions;
};

struct ContainerResponse {
  std::map<std::string, std::string> envs, annotations;
  std::vector<MountMsg> mounts;
  std::vector<DeviceSpecMsg> devices;
};

struct PreferredRequest {
  std::vector<std::string> available, must_include;
  int32_t size = 0;
};
// The same, as views into the request message (kubelet sends every free ID of the node: hundreds of strings)
struct PreferredRequestView {
  std::vector<std::string_view> available, must_include;
  int32_t size = 0;
};

// kubelet PodResources API v1 (k8s.io/kubelet/pkg/apis/podresources/v1/api.proto, deviceplugin/podresources.py):
// the devices of one container of one pod
struct PodDevicesMsg {
  std::string ns, name, container, resource;
  std::vector<std::string> ids;
};

// ---- encode
// ListPodResourcesResponse: one PodResources per (ns, name) in first-seen order, one ContainerResources per entry
std::string encode_pod_resources_list(const std::vector<PodDevicesMsg>& entries);
bool decode_pod_resources_list(const std::string& msg, std::vector<PodDevicesMsg>* entries);
std::string encode_options(bool pre_start_required, bool preferred_available);
// DevicePluginOptions -> (pre_start_required, get_preferred_allocation_available)
bool decode_options(const std::string& msg, bool* pre_start_required, bool* preferred_available);
std::string encode_list_and_watch(const std::vector<DeviceMsg>& devs);
std::string encode_preferred_response(const std::vector<std::vector<std::string>>& per_container);
std::string encode_allocate_response(const std::vector<ContainerResponse>& per_container);
bool encode_allocate_response_selfcheck(const std::vector<ContainerResponse>& per_container);  // tests
std::string encode_allocate_request(const std::vector<std::vector<std::string>>& ids_per_container);
std::string encode_preferred_request(const std::vector<PreferredRequest>& reqs);

// ---- decode (false: malformed)
bool decode_allocate_request(const std::string& msg, std::vector<std::vector<std::string>>* ids_per_container);
bool decode_preferred_request(std::string_view msg, std::vector<PreferredRequestView>* reqs);  // views into msg
// kubelet's usual GetPreferredAllocation: one container, no must_include.  Its size and the container message (whose
// available IDs for_each_available walks in order, stopping when `fn` returns false); false for any other shape.
bool preferred_single(std::string_view msg, int32_t* size, std::string_view* container);
bool for_each_available(std::string_view container, const std::function<bool(std::string_view)>& fn);
// The same request in one walk: `size` read first from the container's tail (kubelet's Go protobuf writes
// allocation_size, field 3, last), then every entry is walked once -- `fn` sees each available ID, and the walk
// checks there is no must_include and that field 3 says `size`.  false (use preferred_single) for any other shape.
bool preferred_single_size(std::string_view msg, int32_t* size, std::string_view* container);
// One walk over the container's available IDs: the first `size` that start with `prefix` go to *mine, the first
// `size` others to *other (both in list order); false if the container has must_include, a field 3 that is not
// `size`, or is malformed.
bool pick_available(std::string_view container, int32_t size, std::string_view prefix,
                    std::vector<std::string_view>* mine, std::vector<std::string_view>* other);
bool decode_list_and_watch(const std::string& msg, std::vector<DeviceMsg>* devs);
bool decode_preferred_response(const std::string& msg, std::vector<std::vector<std::string>>* per_container);
bool decode_allocate_response(const std::string& msg, std::vector<ContainerResponse>* per_container);

}  // namespace gsx::dp
