// Native reflector: LIST + WATCH of one Kubernetes resource on its own thread.
//
// The reference consumes pods and nodes through client-go shared informers
// (pkg/gpushare/controller.go:76-128, cmd/main.go:103): a reflector LISTs,
// then WATCHes from the list's resourceVersion, re-watches when a stream
// ends and re-lists on "410 Gone".  This is the same protocol in C++ so the
// extender's per-event work (decode, filter, ledger update) never reaches
// Python: watch lines are parsed with the tape parser straight out of the
// socket buffer and handed to the owner's callbacks.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "apiclient.h"
#include "json.h"

namespace gsx {

enum class Ev : int { Added = 0, Modified = 1, Deleted = 2 };

struct ReflectorConfig {
  std::string path;  // collection path, e.g. "/api/v1/pods" or "/api/v1/namespaces/ns/pods"
  std::string label_selector, field_selector;
  int watch_timeout_s = 300;       // server-side watch timeout (then re-watch)
  double backoff_max_s = 5.0;      // reconnect backoff cap
  // LIST in pages of this many objects (`limit` / `continue`, client-go's pager default 500); 0 = one
  // unpaginated request.  Keeps each apiserver response (and etcd range read) bounded in a large cluster.
  int list_page_size = 500;
};

// One complete LIST, possibly assembled from several pages.  Objects are addressed as
// (page, tape index); the pages' bodies live as long as the view.
struct ListView {
  std::vector<std::unique_ptr<std::string>> bodies;
  std::vector<json::Doc> pages;
  std::vector<std::pair<uint32_t, uint32_t>> items;
  size_t size() const { return items.size(); }
  const json::Doc& doc(size_t i) const { return pages[items[i].first]; }
  uint32_t obj(size_t i) const { return items[i].second; }
};

// Callbacks run serially on the reflector thread.
struct ReflectorHandler {
  // A complete LIST.  The owner replaces its view (and diffs it to emit deletes, like client-go's
  // Replace()).
  std::function<void(const ListView& list)> on_list;
  // One watch event; `obj` is the tape index of the object in `doc`.
  std::function<void(Ev type, const json::Doc& doc, uint32_t obj)> on_event;
};

class Reflector {
 public:
  Reflector(const ApiConfig& cfg, ReflectorConfig rc, ReflectorHandler h);
  ~Reflector();
  void start();
  void stop();
  // Blocks until the first LIST was delivered (true) or the timeout expired.
  bool wait_synced(double timeout_s);
  bool synced() const { return synced_.load(); }
  uint64_t events() const { return events_.load(); }
  uint64_t relists() const { return relists_.load(); }
  uint64_t rewatches() const { return rewatches_.load(); }
  uint64_t errors() const { return errors_.load(); }
  std::string last_error() const;
  std::string resource_version() const;
  uint64_t list_pages() const { return list_pages_.load(); }
  // Steady-clock seconds at which the last successfully applied LIST was *sent* (0: none yet).  Any write
  // acknowledged before this instant is reflected in that LIST.
  double last_list_start() const { return last_list_start_.load(); }
  // End the current watch (even one the apiserver never answered) and LIST again.
  void request_relist();

 private:
  void run();
  bool do_list(std::string* err);
  // 0: stream ended (re-watch), 1: resourceVersion gone (re-list), -1: error.
  int do_watch(std::string* err);
  bool on_line(std::string_view line, int* verdict);
  void set_error(const std::string& e);
  std::string query(bool watch, const std::string& cont) const;

  ApiClient api_;
  ReflectorConfig rc_;
  ReflectorHandler h_;
  std::thread th_;
  std::atomic<bool> stop_{false};
  std::atomic<bool> synced_{false};
  std::atomic<uint64_t> events_{0}, relists_{0}, rewatches_{0}, errors_{0}, list_pages_{0};
  std::atomic<double> last_list_start_{0.0};
  std::atomic<bool> relist_req_{false};
  StreamHandle stream_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::string rv_;
  std::string last_err_;
};

// Percent-encode a query parameter value (RFC 3986 unreserved kept).
std::string url_escape(std::string_view s);

}  // namespace gsx
