#include "dpcore.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>

#include "json.h"

namespace gsx {
namespace {

const char kCuMaskAnn[] = "gpushare.amd.com/cu-mask";
const char kAssignTimeAnn[] = "gpushare.amd.com/assign-time";
const char kPodAnn[] = "gpushare.amd.com/pod";  // container annotation: which pod the allocation was built for
const char kContainerDir[] = "/run/gsx";

double mono_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

double wall_s() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

int64_t wall_ns() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return static_cast<int64_t>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

bool mkdirs(const std::string& path) {
  std::string cur;
  size_t i = 0;
  while (i <= path.size()) {
    size_t j = path.find('/', i);
    if (j == std::string::npos) j = path.size();
    cur = path.substr(0, j);
    if (!cur.empty() && ::mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return false;
    i = j + 1;
  }
  return true;
}

bool write_atomic(const std::string& path, const std::string& text, mode_t mode, std::string* err) {
  std::string tmp = path + ".tmp";
  ::chmod(tmp.c_str(), 0644);  // a previous attempt's read-only leftover
  int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) {
    *err = "open " + tmp + ": " + std::strerror(errno);
    return false;
  }
  size_t off = 0;
  while (off < text.size()) {
    ssize_t n = ::write(fd, text.data() + off, text.size() - off);
    if (n < 0 && errno == EINTR) continue;
    if (n <= 0) {
      *err = "write " + tmp + ": " + std::strerror(errno);
      ::close(fd);
      return false;
    }
    off += static_cast<size_t>(n);
  }
  ::close(fd);
  if (::chmod(tmp.c_str(), mode) != 0 || ::rename(tmp.c_str(), path.c_str()) != 0) {
    *err = "install " + path + ": " + std::strerror(errno);
    return false;
  }
  return true;
}

}  // namespace

dp::ContainerResponse build_response(const AllocPod& pod, const DpDevice& d, int64_t container_units,
                                     const std::vector<int>& cus, const std::string& mount_mode, const Profile& p) {
  // deviceplugin/allocator.py documents the contract; both call this
  dp::ContainerResponse r;
  const int64_t dev_total = pod.dev_total > 0 ? pod.dev_total : 0;
  const bool isolated = mount_mode == "isolated";
  const std::string visible = isolated ? "0" : std::to_string(d.index);
  double frac = dev_total ? static_cast<double>(container_units) / static_cast<double>(dev_total) : 0.0;
  if (d.share_bytes && d.total_bytes > d.share_bytes) {
    // a partition that shares its HBM pool sees the whole pool as device memory: scale to the pool
    frac *= static_cast<double>(d.share_bytes) / static_cast<double>(d.total_bytes);
  }
  char fbuf[32];
  std::snprintf(fbuf, sizeof fbuf, "%.6f", frac);
  r.envs["HIP_VISIBLE_DEVICES"] = visible;
  r.envs["ROCR_VISIBLE_DEVICES"] = visible;
  r.envs[p.a_idx] = std::to_string(d.index);
  r.envs[p.a_dev] = std::to_string(dev_total);
  r.envs[p.a_pod] = std::to_string(pod.request);
  r.envs[p.env_container] = std::to_string(container_units);
  r.envs["GSX_GPU_MEM_FRACTION"] = fbuf;
  r.envs["GSX_GPU_BDF"] = d.bdf;
  if (!cus.empty()) {
    std::string words = cu_words(cus, d.cu_count);
    r.envs["GSX_CU_MASK"] = words;
    r.envs["HSA_CU_MASK"] = visible + ":" + cu_ranges(cus);
    r.annotations[kCuMaskAnn] = words;
  }
  if (isolated) {
    for (const auto& n : d.nodes) r.devices.push_back(dp::DeviceSpecMsg{n, n, "rw"});
  }
  return r;
}

std::string isolation_config_text(const std::vector<int>& cus, int cu_count, int64_t limit_bytes) {
  std::string t = "# written by the gpushare device plugin; read by libgsx_isolate.so\n";
  if (!cus.empty()) t += "cu_mask=" + cu_words(cus, cu_count) + "\n";
  if (limit_bytes > 0) t += "hbm_limit_bytes=" + std::to_string(limit_bytes) + "\n";
  t += std::string("ledger=") + kContainerDir + "/hbm.ledger\n";
  return t;
}

bool isolation_prepare(const std::string& host_dir, const std::string& uid, const std::vector<int>& cus, int cu_count,
                       int64_t limit_bytes, bool host_process, std::vector<dp::MountMsg>* mounts,
                       std::map<std::string, std::string>* envs, std::string* err) {
  if (uid.empty() || uid.find('/') != std::string::npos || uid == "." || uid == "..") {
    *err = "bad pod uid for the isolation directory";
    return false;
  }
  const std::string d = host_dir + "/pods/" + uid;
  if (!mkdirs(d)) {
    *err = "mkdir " + d + ": " + std::strerror(errno);
    return false;
  }
  std::string conf = isolation_config_text(cus, cu_count, limit_bytes);
  const std::string ledger = d + "/hbm.ledger";
  if (host_process) {  // no mount namespace: the ledger is named by its host path
    std::string from = std::string("ledger=") + kContainerDir + "/hbm.ledger";
    size_t at = conf.find(from);
    if (at != std::string::npos) conf.replace(at, from.size(), "ledger=" + ledger);
  }
  if (!write_atomic(d + "/isolation.conf", conf, 0444, err)) return false;
  if (::access(ledger.c_str(), F_OK) != 0) {
    int fd = ::open(ledger.c_str(), O_CREAT | O_RDWR | O_CLOEXEC, 0666);
    if (fd < 0) {
      *err = "create " + ledger + ": " + std::strerror(errno);
      return false;
    }
    ::close(fd);
    ::chmod(ledger.c_str(), 0666);  // the container's user is not ours
  }
  if (host_process) {
    (*envs)["HSA_TOOLS_LIB"] = host_dir + "/libgsx_isolate.so";
    (*envs)["GSX_ISOLATION_CONFIG"] = d + "/isolation.conf";
    return true;
  }
  const std::string c = kContainerDir;
  mounts->push_back(dp::MountMsg{c + "/isolation.conf", d + "/isolation.conf", true});
  mounts->push_back(dp::MountMsg{c + "/hbm.ledger", ledger, false});
  mounts->push_back(dp::MountMsg{c + "/libgsx_isolate.so", host_dir + "/libgsx_isolate.so", true});
  mounts->push_back(dp::MountMsg{"/etc/ld.so.preload", host_dir + "/ld.so.preload", true});
  (*envs)["HSA_TOOLS_LIB"] = c + "/libgsx_isolate.so";
  return true;
}

DpCore::DpCore(DpConfig cfg, AllocState* state) : cfg_(std::move(cfg)), state_(state) {
  if (!cfg_.api.server.empty()) api_ = std::make_unique<ApiClient>(cfg_.api);
  if (cfg_.early_answer && !cfg_.journal.empty()) {
    std::string err;
    int fd = ::open(cfg_.journal.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0644);
    if (fd < 0 || !journal_map(fd, &err)) {
      if (fd < 0) err = std::strerror(errno);
      std::fprintf(stderr, "[gsx-dpcore] journal %s: %s; answering after the ASSIGNED patch instead\n",
                   cfg_.journal.c_str(), err.c_str());
      if (fd >= 0) ::close(fd);
      cfg_.early_answer = false;  // no durable record before the answer: keep the synchronous commit
    }
  }
}

DpCore::~DpCore() { journal_unmap(true); }

bool DpCore::journal_map(int fd, std::string* err) {
  struct stat st {};
  if (::fstat(fd, &st) != 0) {
    *err = std::string("fstat: ") + std::strerror(errno);
    return false;
  }
  size_t used = static_cast<size_t>(st.st_size);
  size_t cap = std::max(kJournalChunk, (used / kJournalChunk + 1) * kJournalChunk);
  if (::ftruncate(fd, static_cast<off_t>(cap)) != 0) {
    *err = std::string("ftruncate: ") + std::strerror(errno);
    return false;
  }
  // blocks reserved up front: a store into a mapped page the filesystem cannot back raises SIGBUS (a full disk would
  // kill the plugin inside an Allocate); a reservation that fails is an error here, where the caller can fall back
  if (int fe = ::posix_fallocate(fd, 0, static_cast<off_t>(cap)); fe != 0) {
    *err = std::string("posix_fallocate: ") + std::strerror(fe);
    (void)!::ftruncate(fd, static_cast<off_t>(used));
    return false;
  }
  // not prefaulted: a rotation runs under the state lock, and populating 1 MiB there would hold an Allocate up;
  // the pages fault in as lines reach them (one 4 KiB page per ~4 Allocates)
  void* m = ::mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) {
    *err = std::string("mmap: ") + std::strerror(errno);
    (void)!::ftruncate(fd, static_cast<off_t>(used));
    return false;
  }
  // what an earlier process left: its whole lines (zeros past them, or a line torn by a crash mid-copy -- its
  // Allocate was never answered -- are written over)
  char* b = static_cast<char*>(m);
  while (used > 0 && b[used - 1] != '\n') --used;
  // a torn tail is cleared, so a shorter line written over it leaves no fragment behind
  std::memset(b + used, 0, static_cast<size_t>(st.st_size) - used);
  jfd_ = fd;
  jmap_ = static_cast<char*>(m);
  jcap_ = cap;
  jlen_ = used;
  return true;
}

void DpCore::journal_unmap(bool trim) {
  if (jmap_) ::munmap(jmap_, jcap_);
  if (jfd_ >= 0) {
    if (trim) (void)!::ftruncate(jfd_, static_cast<off_t>(jlen_));
    ::close(jfd_);
  }
  jmap_ = nullptr;
  jfd_ = -1;
  jcap_ = jlen_ = 0;
}

bool DpCore::journal_append(const AllocRecord& r) {
  if (jfd_ < 0) return true;
  // one line per Allocate, the record's fields as the plugin's checkpoint has them (AllocRecord.to_dict)
  size_t est = 256 + r.aid.size() + r.uid.size() + r.cu_mask.size() + r.iso.size();
  for (const auto& id : r.ids) est += id.size() + 3;
  std::string line;
  line.reserve(est);
  line.append("{\"aid\":");
  json::append_quoted(&line, r.aid);
  line.append(",\"uid\":");
  json::append_quoted(&line, r.uid);
  line.append(",\"ids\":[");
  for (size_t i = 0; i < r.ids.size(); ++i) {
    if (i) line.push_back(',');
    json::append_quoted(&line, r.ids[i]);
  }
  line.append("],\"dev\":").append(std::to_string(r.dev)).append(",\"units\":").append(std::to_string(r.units));
  line.append(",\"cu_mask\":");
  json::append_quoted(&line, r.cu_mask);
  line.append(",\"owner\":\"\",\"t\":").append(std::to_string(r.t)).append(",\"iso\":");
  json::append_quoted(&line, r.iso);
  line.append(",\"on_gpu\":").append(r.on_gpu ? "true" : "false").append("}\n");
  if (jlen_ + line.size() > jcap_) {
    // grow by whole chunks (a syscall pair per ~1,000 Allocates): the mapping is re-made over the longer file
    const size_t cap = ((jlen_ + line.size()) / kJournalChunk + 1) * kJournalChunk;
    // the new chunk's blocks are reserved before it is mapped (see journal_map: no SIGBUS on a full disk)
    void* m = (::ftruncate(jfd_, static_cast<off_t>(cap)) == 0 &&
               ::posix_fallocate(jfd_, static_cast<off_t>(jcap_), static_cast<off_t>(cap - jcap_)) == 0)
                  ? ::mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_SHARED, jfd_, 0)
                  : MAP_FAILED;
    if (m == MAP_FAILED) {
      (void)!::ftruncate(jfd_, static_cast<off_t>(std::max(jcap_, jlen_)));  // no unreserved tail left mapped later
      // the line still goes to the file (past the mapped bytes), where a full disk fails the write, not the process;
      // the next append retries the growth
      ssize_t n = ::pwrite(jfd_, line.data(), line.size(), static_cast<off_t>(jlen_));
      if (n == static_cast<ssize_t>(line.size())) {
        jlen_ += line.size();
        return true;
      }
      return false;
    }
    ::munmap(jmap_, jcap_);
    jmap_ = static_cast<char*>(m);
    jcap_ = cap;
  }
  // the page cache outlives this process: once copied, the line survives a crash of the plugin like a write(2)
  std::memcpy(jmap_ + jlen_, line.data(), line.size());
  jlen_ += line.size();
  return true;
}

bool DpCore::journal_rotate(std::string* err) {
  if (jfd_ < 0) return true;
  const std::string& path = cfg_.journal;
  const std::string old = path + ".old";
  if (::access(old.c_str(), F_OK) != 0) {
    // the common case: the journal (trimmed to its lines) becomes .old, a fresh journal takes the next Allocates
    int nfd = -1;
    std::string e2;
    if (::rename(path.c_str(), old.c_str()) != 0) {
      *err = "rename " + path + ": " + std::strerror(errno);
      return false;
    }
    nfd = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (nfd < 0) {
      *err = "open " + path + ": " + std::strerror(errno);
      (void)::rename(old.c_str(), path.c_str());  // keep appending where we were
      return false;
    }
    const int ofd = jfd_;
    char* omap = jmap_;
    const size_t ocap = jcap_, olen = jlen_;
    jfd_ = -1;
    jmap_ = nullptr;
    if (!journal_map(nfd, &e2)) {
      ::close(nfd);
      (void)::rename(old.c_str(), path.c_str());
      jfd_ = ofd;
      jmap_ = omap;
      jcap_ = ocap;
      jlen_ = olen;
      *err = "map " + path + ": " + e2;
      return false;
    }
    // .old is not trimmed: the checkpoint that covers it deletes it, and its readers skip the zeros (a shrinking
    // truncate under the state lock could wait for the pages' writeback)
    (void)olen;
    ::munmap(omap, ocap);
    ::close(ofd);
    return true;
  }
  // a previous checkpoint did not land: .old still holds records it was to cover; append this generation to it
  // (read back from the file: lines past the mapping, written when growing it failed, are in the file only).  .old is
  // a renamed journal and keeps its zero padding: trimmed back to its last whole line first, or the appended
  // generation's first line would follow a run of NULs
  int out = ::open(old.c_str(), O_RDWR | O_CLOEXEC);
  bool ok = out >= 0;
  if (ok) {
    struct stat ost {};
    ok = ::fstat(out, &ost) == 0;
    off_t end = ok ? ost.st_size : 0;
    char tail[4096];
    while (ok && end > 0) {
      const off_t from = std::max<off_t>(0, end - static_cast<off_t>(sizeof tail));
      ssize_t n = ::pread(out, tail, static_cast<size_t>(end - from), from);
      if (n < 0 && errno == EINTR) continue;
      if (n <= 0) {
        ok = false;
        break;
      }
      ssize_t k = n;
      while (k > 0 && tail[k - 1] != '\n') --k;
      if (k > 0) {
        end = from + k;
        break;
      }
      end = from;
    }
    ok = ok && ::ftruncate(out, end) == 0 && ::lseek(out, 0, SEEK_END) == end;
  }
  size_t off = 0;
  char buf[65536];
  while (ok && off < jlen_) {
    ssize_t n = ::pread(jfd_, buf, std::min(sizeof buf, jlen_ - off), static_cast<off_t>(off));
    if (n < 0 && errno == EINTR) continue;
    ok = n > 0 && ::write(out, buf, static_cast<size_t>(n)) == n;
    if (ok) off += static_cast<size_t>(n);
  }
  if (out >= 0) ::close(out);
  if (!ok) {
    *err = "appending " + path + " to " + old + ": " + std::strerror(errno);
    return false;
  }
  std::memset(jmap_, 0, std::min(jlen_, jcap_));  // the generation lives in .old now
  if (jlen_ > jcap_) (void)!::ftruncate(jfd_, static_cast<off_t>(jcap_));  // the unmapped lines went too
  jlen_ = 0;
  return true;
}

void DpCore::set_devices(std::vector<DpDevice> devs, std::map<std::string, int> id_owner) {
  devs_.clear();
  for (auto& d : devs) devs_[d.index] = std::move(d);
  id_owner_ = std::unordered_map<std::string, int>(id_owner.begin(), id_owner.end());
  id_owner_view_.clear();
  for (const auto& kv : id_owner_) id_owner_view_.emplace(std::string_view(kv.first), kv.second);
  // the plugin's IDs are "<device base><sep><k>" (deviceplugin/plugin.py: fake_ids): when every ID of a device
  // shares one prefix that no other device's IDs start with, "is this ID on GPU g" is a prefix compare instead of a
  // hash lookup per ID (kubelet lists every free ID of the node: ~2,300 on an 8-GPU node)
  id_prefix_.clear();
  std::map<int, std::string> pre;
  bool ok = true;
  for (const auto& kv : id_owner_) {
    size_t cut = kv.first.rfind(kIdSep);
    if (cut == std::string::npos) {
      ok = false;
      break;
    }
    std::string p = kv.first.substr(0, cut + kIdSep.size());
    auto it = pre.find(kv.second);
    if (it == pre.end()) {
      pre.emplace(kv.second, std::move(p));
    } else if (it->second != p) {
      ok = false;
      break;
    }
  }
  for (const auto& a : pre) {
    for (const auto& b : pre) {
      if (a.first != b.first && b.second.compare(0, a.second.size(), a.second) == 0) ok = false;
    }
  }
  if (ok) id_prefix_ = std::unordered_map<int, std::string>(pre.begin(), pre.end());
}

bool DpCore::id_on(std::string_view id, int dev) const {
  if (!id_prefix_.empty()) {
    auto p = id_prefix_.find(dev);
    return p != id_prefix_.end() && id.size() > p->second.size() && id.compare(0, p->second.size(), p->second) == 0;
  }
  auto o = id_owner_view_.find(id);
  return o != id_owner_view_.end() && o->second == dev;
}

int64_t DpCore::physical_used(int dev) const { return state_->physical_used(dev); }

bool DpCore::ids_on(const std::vector<std::string>& ids, int dev) const {
  for (const auto& id : ids) {
    if (!id_on(id, dev)) return false;
  }
  return !ids.empty();
}

bool DpCore::preferred(const std::string& req, std::string* resp, std::string* why) {
  int32_t size = 0;
  std::string_view container;
  if (!id_prefix_.empty() && dp::preferred_single_size(std::string_view(req), &size, &container)) {
    // one walk over kubelet's free IDs (~2,300 on 8 GPUs): the size is read off the container's tail, so the pod's
    // GPU is known before the walk, which picks its IDs (then others, in order, if it has too few) and validates
    // the request as it goes
    const int64_t want = state_->preferred_device(size);
    if (want < 0) {
      stats_.slow_preferred++;
      *why = "no pending pod of that size known yet";
      return false;
    }
    auto pre = id_prefix_.find(static_cast<int>(want));
    const std::string_view prefix = pre != id_prefix_.end() ? std::string_view(pre->second) : std::string_view();
    std::vector<std::string_view> mine, other;
    mine.reserve(static_cast<size_t>(size));
    const size_t cap = static_cast<size_t>(size);
    const bool ok = dp::pick_available(container, size, prefix, &mine, &other);
    if (ok) {
      std::vector<std::vector<std::string>> out(1);
      std::vector<std::string>& chosen = out[0];
      chosen.reserve(cap);
      for (auto id : mine) chosen.emplace_back(id);
      for (size_t k = 0; chosen.size() < cap && k < other.size(); ++k) chosen.emplace_back(other[k]);
      *resp = dp::encode_preferred_response(out);
      stats_.fast_preferred++;
      return true;
    }
    // another shape after all (must_include, a size that is not the tail's): the general walks below
  }
  if (dp::preferred_single(std::string_view(req), &size, &container)) {
    // kubelet's usual request (one container, nothing it must include): the free-ID list (~2,300 on 8 GPUs) is
    // walked in place, without a view per ID, and only until `size` IDs of the pod's GPU are found
    const int64_t want = state_->preferred_device(size);
    if (want < 0) {
      stats_.slow_preferred++;
      *why = "no pending pod of that size known yet";
      return false;
    }
    std::vector<std::vector<std::string>> out(1);
    std::vector<std::string>& chosen = out[0];
    chosen.reserve(static_cast<size_t>(std::max<int32_t>(size, 0)));
    // the GPU's ID prefix looked up once, not per listed ID (the walk passes ~2,000 IDs of other GPUs)
    auto pre = id_prefix_.find(static_cast<int>(want));
    const std::string_view prefix = pre != id_prefix_.end() ? std::string_view(pre->second) : std::string_view();
    auto on = [&](std::string_view id) {
      if (id_prefix_.empty()) return id_on(id, static_cast<int>(want));
      return !prefix.empty() && id.size() > prefix.size() && id.compare(0, prefix.size(), prefix) == 0;
    };
    for (int pass = 0; pass < 2 && static_cast<int32_t>(chosen.size()) < size; ++pass) {
      dp::for_each_available(container, [&](std::string_view id) {
        if (on(id) == (pass == 0)) chosen.emplace_back(id);
        return static_cast<int32_t>(chosen.size()) < size;
      });
    }
    *resp = dp::encode_preferred_response(out);
    stats_.fast_preferred++;
    return true;
  }
  std::vector<dp::PreferredRequestView> reqs;  // views into `req`: no string per ID
  if (!dp::decode_preferred_request(std::string_view(req), &reqs)) {
    *why = "malformed request";
    return false;
  }
  std::vector<std::vector<std::string>> out;
  for (const auto& r : reqs) {
    int64_t want = state_->preferred_device(r.size);
    if (want < 0) {
      stats_.slow_preferred++;
      *why = "no pending pod of that size known yet";
      return false;
    }
    // kubelet sends every free ID of the node (hundreds): pick the first `size` of them, the pod's GPU's first,
    // copying only what is chosen
    std::vector<std::string> chosen;
    for (auto id : r.must_include) chosen.emplace_back(id);
    std::set<std::string_view> taken(r.must_include.begin(), r.must_include.end());
    for (int pass = 0; pass < 2 && static_cast<int32_t>(chosen.size()) < r.size; ++pass) {
      for (auto id : r.available) {
        if (static_cast<int32_t>(chosen.size()) >= r.size) break;
        const bool on_gpu = id_on(id, static_cast<int>(want));
        if (on_gpu != (pass == 0) || (!taken.empty() && taken.count(id))) continue;
        chosen.emplace_back(id);
      }
    }
    if (static_cast<int32_t>(chosen.size()) > r.size) chosen.resize(static_cast<size_t>(r.size));
    out.push_back(std::move(chosen));
  }
  *resp = dp::encode_preferred_response(out);
  stats_.fast_preferred++;
  return true;
}

DpStep DpCore::allocate(const std::string& req, std::string* resp, DpEvent* ev, std::unique_ptr<DpPending>* pend,
                        std::string* why) {
  const double t0 = mono_s();
  std::vector<std::vector<std::string>> ids_per;
  if (!dp::decode_allocate_request(req, &ids_per) || ids_per.size() != 1 || ids_per[0].empty()) {
    stats_.slow_allocate++;
    *why = "not a single-container request";
    return DpStep::Slow;
  }
  const std::vector<std::string>& ids = ids_per[0];
  const int64_t units = static_cast<int64_t>(ids.size());
  const double td = mono_s();
  auto m = state_->match(units);
  const double tm = mono_s();

  if (!m.first) {
    stats_.slow_allocate++;
    *why = "no candidate";
    return DpStep::Slow;
  }
  const AllocPod pod = *m.first;  // a copy: observe() later replaces the state's
  bool ambiguous = false;
  if (devs_.size() > 1) {
    for (const AllocPod* c : state_->candidates()) {
      if (c->uid != pod.uid && c->request == pod.request && c->dev != pod.dev) {
        ambiguous = true;
        break;
      }
    }
  }
  auto dit = devs_.find(static_cast<int>(pod.dev));
  if (dit == devs_.end() || pod.hold_idx >= 0 || !pod.hold_partner.empty()) {
    stats_.slow_allocate++;
    *why = dit == devs_.end() ? "GPU not on this node" : "pod in a reconciliation exchange";
    return DpStep::Slow;
  }
  const DpDevice& dev = dit->second;
  const bool later = pod.assigned == "true";
  // kubelet hands out each fake ID once and GetPreferredAllocation steers a pod's IDs onto its GPU: when this
  // Allocate's IDs all lie on the pod's GPU and so do those of every recorded allocation whose container runs
  // there, kubelet's own per-ID accounting bounds what runs on that GPU (each unit there holds one of its IDs),
  // whatever the records of pods it has since freed still say.  Otherwise the records decide (the Python guard
  // repairs and waits).  A record off its GPU elsewhere on the node does not matter to this GPU.
  const bool on_gpu = ids_on(ids, dev.index);

  if (!later && cfg_.guard && physical_used(dev.index) + units > dev.units) {
    if (!on_gpu || state_->off_gpu_records_on(dev.index) != 0) {
      stats_.slow_allocate++;
      *why = "GPU physically full by the records";
      return DpStep::Slow;
    }
    stats_.guard_by_ids++;
  }
  if (!later && !api_) {
    stats_.slow_allocate++;
    *why = "no apiserver client";
    return DpStep::Slow;
  }
  CuPartitioner* cp = state_->cus(dev.index);
  const bool had_cus = cp && cp->holds(pod.uid);
  if (!later) state_->set_inflight(pod.uid, true);
  std::vector<int> cus;
  std::string err;
  auto undo = [&] {
    if (!later) {
      if (cp && !had_cus) cp->release(pod.uid);
      state_->set_inflight(pod.uid, false);
    }
  };
  if (!state_->claim_cus(pod.uid, &cus, &err)) {
    undo();
    stats_.slow_allocate++;
    *why = "CU partition: " + err;
    return DpStep::Slow;
  }
  const double tc = mono_s();
  auto p = std::make_unique<DpPending>();
  p->pod = pod;
  p->whole = m.second;
  p->had_cus = had_cus;
  p->units = units;
  p->ids = std::move(ids_per[0]);  // `ids` is not read after this point
  p->on_gpu = on_gpu;
  p->ambiguous = ambiguous;
  p->cr = build_response(pod, dev, units, cus, cfg_.mount_mode, cfg_.profile);
  const double tb = mono_s();
  p->t0 = t0;
  p->tm = tm;
  p->ti0 = mono_s();
  if (!cfg_.iso_dir.empty()) {
    if (!isolation_prepare(cfg_.iso_dir, pod.uid, cus, dev.cu_count, pod.request * cfg_.unit_bytes,
                           cfg_.mount_mode == "all", &p->cr.mounts, &p->cr.envs, &err)) {
      undo();
      stats_.slow_allocate++;
      *why = "isolation files: " + err;
      return DpStep::Slow;
    }
    p->iso = pod.uid;
  }
  p->ti1 = p->tp0 = p->tp1 = mono_s();
  p->cr.annotations[kPodAnn] = pod.key + "/" + pod.uid;
  if (later) {
    state_->later_container_allocated(pod.uid, units);
    p->ok = true;
    finish(*p, resp, ev, why);
    return DpStep::Answered;
  }
  // The precondition: synchronous answer -- the resourceVersion the match was made on (the commit IS the claim:
  // a stale view loses with 409 and the slow path re-decides).  Early answer -- the pod's UID: kubelet already
  // has this allocation, so the commit must land on whatever version the pod has by then (kubelet's status
  // updates move it), but never on a pod re-created under the same name.
  std::string patch = cfg_.early_answer ? "{\"metadata\":{\"uid\":" : "{\"metadata\":{\"resourceVersion\":";
  json::append_quoted(&patch, cfg_.early_answer ? pod.uid : pod.rv);
  patch.append(",\"annotations\":{");
  json::append_quoted(&patch, cfg_.profile.a_assigned);
  patch.append(":\"true\",");
  json::append_quoted(&patch, kAssignTimeAnn);
  patch.append(":\"").append(std::to_string(wall_ns())).append("\"");
  auto cm = p->cr.annotations.find(kCuMaskAnn);
  if (cm != p->cr.annotations.end()) {
    patch.push_back(',');
    json::append_quoted(&patch, kCuMaskAnn);
    patch.push_back(':');
    json::append_quoted(&patch, cm->second);
  }
  patch.append("}}}");
  p->body = std::move(patch);
  p->path = "/api/v1/namespaces/" + pod.ns + "/pods/" + pod.name;
  if (cfg_.early_answer) {
    p->answered = true;
    p->ok = true;
    state_->first_container_committed(pod.uid, units, p->whole);  // claimed (in flight) until the patch lands
    const double tbody = mono_s();
    record_and_answer(*p, resp, ev);
    stats_.ph_decode += td - t0;
    stats_.ph_match += tm - td;
    stats_.ph_claim += tc - tm;
    stats_.ph_build += tb - tc;
    stats_.ph_body += tbody - tb;
    stats_.phased++;
    ev->committed = true;
    *pend = std::move(p);
    return DpStep::AnsweredPending;
  }
  *pend = std::move(p);
  return DpStep::Pending;
}

void DpCore::run_patch(DpPending& p) {
  p.tp0 = mono_s();
  p.ok = api_->request("PATCH", p.path, p.body, "application/merge-patch+json", &p.status, &p.resp, &p.err);
  p.tp1 = mono_s();
}

bool DpCore::finish(DpPending& p, std::string* resp, DpEvent* ev, std::string* why) {
  const bool later = p.path.empty();
  if (p.answered) {
    p.retry = false;
    json::Doc d;
    AllocPod committed;
    std::string perr;
    if (p.ok && p.status < 300 && d.parse(p.resp, &perr) && parse_alloc_pod(d, 0, cfg_.profile, &committed)) {
      committed.raw = p.resp;
      state_->observe(committed);
      state_->set_inflight(p.pod.uid, false);
      ev->uid = p.pod.uid;
      ev->key = p.pod.key;
      ev->patch_only = true;
      ev->pod_json = std::move(p.resp);
      return true;
    }
    // re-created under its name: kube-apiserver refuses the changed metadata.uid of the patched object (422 Invalid);
    // a UID-precondition 409 is what a PUT or Binding would get, accepted too
    const bool recreated = p.ok && ((p.status == 422 && p.resp.find("metadata.uid") != std::string::npos) ||
                                    (p.status == 409 && p.resp.find("UID in precondition") != std::string::npos));
    if ((p.ok && p.status == 404) || recreated || !state_->pod(p.pod.uid)) {
      // the pod went away (deleted, or re-created under its name): nothing to commit.  It is released now, not when
      // the pod feed delivers the deletion: unclaimed but still pending ASSIGNED=false in the state, it would be the
      // next Allocate's match (kubelet has already started its container and is admitting the next pod)
      state_->set_inflight(p.pod.uid, false);
      state_->deleted(p.pod.uid);
      stats_.commits_gone++;
      return true;
    }
    // transport error, 5xx, an injected or transient 409: the commit is retried with capped exponential backoff
    // for as long as the pod exists -- kubelet has its answer, so giving up would leave the pod ASSIGNED=false
    // (claimed here, but a match candidate for a restarted plugin) with its container running
    stats_.patch_failures++;
    p.attempts++;
    p.retry = true;
    p.not_before = mono_s() + std::min(1.0, 0.002 * static_cast<double>(1 << std::min(p.attempts, 10)));
    if (p.attempts == 1 || p.attempts % 32 == 0) {
      *why = p.ok ? "ASSIGNED patch answered " + std::to_string(p.status) : "ASSIGNED patch: " + p.err;
      std::fprintf(stderr, "[gsx-dpcore] %s: %s (attempt %d; the Allocate was answered, retrying)\n",
                   p.pod.key.c_str(), why->c_str(), p.attempts);
    }
    return true;
  }
  if (!later) {
    json::Doc d;
    AllocPod committed;
    std::string perr;
    bool good = p.ok && p.status < 300 && d.parse(p.resp, &perr) && parse_alloc_pod(d, 0, cfg_.profile, &committed);
    if (good) committed.raw = p.resp;
    if (!good) {
      CuPartitioner* cp = state_->cus(static_cast<int>(p.pod.dev));
      if (cp && !p.had_cus) cp->release(p.pod.uid);
      state_->set_inflight(p.pod.uid, false);
      stats_.patch_failures++;
      stats_.slow_allocate++;
      *why = p.ok ? "ASSIGNED patch answered " + std::to_string(p.status) : "ASSIGNED patch: " + p.err;
      return false;
    }
    state_->observe(committed);
    state_->set_inflight(p.pod.uid, false);
    state_->first_container_committed(p.pod.uid, p.units, p.whole);
    ev->pod_json = std::move(p.resp);
    ev->committed = true;
  }
  record_and_answer(p, resp, ev);
  return true;
}

void DpCore::record_and_answer(DpPending& p, std::string* resp, DpEvent* ev) {
  char aid[64];
  std::snprintf(aid, sizeof aid, "%llx-%x-n%llu", static_cast<unsigned long long>(wall_ns() / 1000000),
                static_cast<unsigned>(::getpid()), static_cast<unsigned long long>(++aid_));
  auto cm = p.cr.annotations.find(kCuMaskAnn);
  const double tr0 = mono_s();
  AllocRecord& rec = state_->record(p.pod.uid, p.ids, p.units,
                                    cm != p.cr.annotations.end() ? cm->second : p.pod.cu_mask, aid, wall_s(), p.on_gpu);
  rec.iso = p.iso;
  const double tr1 = mono_s();
  if (p.answered && !journal_append(rec)) {  // durable before kubelet has the answer
    // the disk is full (or the journal unwritable): later Allocates answer after their commit instead, as when the
    // journal could not be opened at all
    stats_.journal_failures++;
    cfg_.early_answer = false;
    std::fprintf(stderr, "[gsx-dpcore] journal %s: write failed (%s); answering after the ASSIGNED patch from now on\n",
                 cfg_.journal.c_str(), std::strerror(errno));
  }
  const double tj = mono_s();
  *resp = dp::encode_allocate_response({p.cr});
  stats_.ph_record += tr1 - tr0;
  stats_.ph_journal += tj - tr1;
  stats_.ph_encode += mono_s() - tj;
  stats_.fast_allocate++;
  ev->uid = p.pod.uid;
  ev->key = p.pod.key;
  ev->aid = aid;
  ev->iso = p.iso;
  ev->ambiguous = p.ambiguous;
  const double t1 = mono_s();
  ev->t_handler = t1 - p.t0;
  ev->t_match = p.tm - p.t0;
  ev->t_isolate = p.ti1 - p.ti0;
  ev->t_patch = p.tp1 - p.tp0;
}

}  // namespace gsx
