#include "informer.h"
#include "introspect.h"

#include <sys/socket.h>

#include <chrono>
#include <cstdio>

namespace gsx {

std::string url_escape(std::string_view s) {
  static const char* hex = "0123456789ABCDEF";
  std::string o;
  o.reserve(s.size());
  for (unsigned char c : s) {
    if ((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '-' || c == '_' ||
        c == '.' || c == '~') {
      o.push_back(static_cast<char>(c));
    } else {
      o.push_back('%');
      o.push_back(hex[c >> 4]);
      o.push_back(hex[c & 15]);
    }
  }
  return o;
}

Reflector::Reflector(const ApiConfig& cfg, ReflectorConfig rc, ReflectorHandler h)
    : api_(cfg), rc_(std::move(rc)), h_(std::move(h)) {}

Reflector::~Reflector() { stop(); }

void Reflector::start() {
  if (th_.joinable()) return;
  stop_.store(false);
  stream_.aborted.store(false);
  th_ = std::thread([this] {
    std::string res = rc_.path.substr(rc_.path.rfind('/') + 1);
    introspect::name_thread("refl-" + res);
    run();
  });
}

void Reflector::stop() {
  stop_.store(true);
  stream_.abort();
  cv_.notify_all();
  if (th_.joinable()) th_.join();
}

bool Reflector::wait_synced(double timeout_s) {
  std::unique_lock<std::mutex> lk(mu_);
  return cv_.wait_for(lk, std::chrono::duration<double>(timeout_s),
                      [this] { return synced_.load() || stop_.load(); }) &&
         synced_.load();
}

std::string Reflector::last_error() const {
  std::lock_guard<std::mutex> g(mu_);
  return last_err_;
}

std::string Reflector::resource_version() const {
  std::lock_guard<std::mutex> g(mu_);
  return rv_;
}

void Reflector::set_error(const std::string& e) {
  errors_++;
  std::lock_guard<std::mutex> g(mu_);
  last_err_ = e;
}

void Reflector::request_relist() {
  relist_req_.store(true);
  // shut the socket down without marking the handle aborted: the watch ends, the loop re-lists
  int fd = stream_.fd.load();
  if (fd >= 0) ::shutdown(fd, SHUT_RDWR);
  cv_.notify_all();
}

std::string Reflector::query(bool watch, const std::string& cont) const {
  std::string q = rc_.path;
  char sep = '?';
  auto add = [&](const char* k, const std::string& v) {
    q.push_back(sep);
    sep = '&';
    q.append(k).push_back('=');
    q.append(url_escape(v));
  };
  if (!rc_.label_selector.empty()) add("labelSelector", rc_.label_selector);
  if (!rc_.field_selector.empty()) add("fieldSelector", rc_.field_selector);
  if (!watch && rc_.list_page_size > 0) {
    add("limit", std::to_string(rc_.list_page_size));
    if (!cont.empty()) add("continue", cont);
  }
  if (watch) {
    add("watch", "true");
    add("allowWatchBookmarks", "true");
    std::string rv;
    {
      std::lock_guard<std::mutex> g(mu_);
      rv = rv_;
    }
    if (!rv.empty()) add("resourceVersion", rv);
    if (rc_.watch_timeout_s > 0) add("timeoutSeconds", std::to_string(rc_.watch_timeout_s));
  }
  return q;
}

bool Reflector::do_list(std::string* err) {
  const double started = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  ListView lv;
  std::string cont, list_rv;
  for (int page = 0;; ++page) {
    int status = 0;
    lv.bodies.emplace_back(new std::string());
    std::string& body = *lv.bodies.back();
    if (!api_.request("GET", query(false, cont), std::string(), nullptr, &status, &body, err)) return false;
    if (status == 410 && page > 0) {
      // the continue token outlived the apiserver's history: start the LIST over
      *err = "LIST " + rc_.path + ": continue token expired";
      return false;
    }
    if (status != 200) {
      *err = "LIST " + rc_.path + ": HTTP " + std::to_string(status) + ": " + body.substr(0, 200);
      return false;
    }
    lv.pages.emplace_back();
    json::Doc& d = lv.pages.back();
    if (!d.parse(body, err)) return false;
    int64_t it = d.find(0, "items");
    if (it >= 0 && d.at(static_cast<uint32_t>(it)).type == json::T::Array) {
      uint32_t end = d.at(static_cast<uint32_t>(it)).skip;
      for (uint32_t i = static_cast<uint32_t>(it) + 1; i < end; i = d.next(i)) {
        if (d.at(i).type == json::T::Object) lv.items.emplace_back(static_cast<uint32_t>(page), i);
      }
    }
    // the whole LIST is consistent at the first page's resourceVersion
    if (page == 0) {
      int64_t rv = d.path(0, {"metadata", "resourceVersion"});
      list_rv = rv >= 0 ? d.str(static_cast<uint32_t>(rv)) : std::string();
    }
    list_pages_++;
    int64_t c = d.path(0, {"metadata", "continue"});
    cont = c >= 0 ? d.str(static_cast<uint32_t>(c)) : std::string();
    if (cont.empty() || rc_.list_page_size <= 0) break;
  }
  {
    std::lock_guard<std::mutex> g(mu_);
    rv_ = list_rv;
  }
  if (h_.on_list) h_.on_list(lv);
  last_list_start_.store(started);
  relists_++;
  return true;
}

bool Reflector::on_line(std::string_view line, int* verdict) {
  json::Doc d;
  std::string perr;
  if (!d.parse(line, &perr)) {
    set_error("bad watch event: " + perr);
    *verdict = -1;
    return false;
  }
  int64_t t = d.find(0, "type");
  int64_t o = d.find(0, "object");
  if (t < 0 || o < 0) return true;
  std::string_view type;
  std::string tbuf;
  if (!d.str_view(static_cast<uint32_t>(t), &type)) {
    tbuf = d.str(static_cast<uint32_t>(t));
    type = tbuf;
  }
  uint32_t obj = static_cast<uint32_t>(o);
  if (type == "ERROR") {
    int64_t code = 0;
    int64_t c = d.find(obj, "code");
    if (c >= 0) d.as_int(static_cast<uint32_t>(c), &code);
    if (code == 410) {
      *verdict = 1;
    } else {
      int64_t m = d.find(obj, "message");
      set_error("watch error " + std::to_string(code) + ": " + (m >= 0 ? d.str(static_cast<uint32_t>(m)) : ""));
      *verdict = -1;
    }
    return false;
  }
  int64_t rv = d.path(obj, {"metadata", "resourceVersion"});
  if (type == "BOOKMARK") {
    if (rv >= 0) {
      std::lock_guard<std::mutex> g(mu_);
      rv_ = d.str(static_cast<uint32_t>(rv));
    }
    return true;
  }
  Ev ev;
  if (type == "ADDED") {
    ev = Ev::Added;
  } else if (type == "MODIFIED") {
    ev = Ev::Modified;
  } else if (type == "DELETED") {
    ev = Ev::Deleted;
  } else {
    return true;
  }
  events_++;
  if (h_.on_event) h_.on_event(ev, d, obj);
  if (rv >= 0) {
    std::lock_guard<std::mutex> g(mu_);
    rv_ = d.str(static_cast<uint32_t>(rv));
  }
  return true;
}

int Reflector::do_watch(std::string* err) {
  std::string buf;
  size_t off = 0;
  int verdict = 0;
  int status = 0;
  std::string ebody;
  auto on_data = [&](std::string_view piece) -> bool {
    buf.append(piece.data(), piece.size());
    while (true) {
      size_t nl = buf.find('\n', off);
      if (nl == std::string::npos) break;
      std::string_view line(buf.data() + off, nl - off);
      off = nl + 1;
      if (line.find_first_not_of(" \r\t") == std::string_view::npos) continue;
      if (!on_line(line, &verdict)) return false;
      if (stop_.load()) return false;
    }
    if (off > 0 && off == buf.size()) {
      buf.clear();
      off = 0;
    } else if (off > (1u << 20)) {
      buf.erase(0, off);
      off = 0;
    }
    return true;
  };
  double idle = rc_.watch_timeout_s > 0 ? rc_.watch_timeout_s + 60.0 : 3600.0;
  if (!api_.stream(query(true, std::string()), &status, &ebody, on_data, err, &stream_, idle)) return -1;
  if (status == 410) return 1;
  if (status >= 400) {
    *err = "WATCH " + rc_.path + ": HTTP " + std::to_string(status) + ": " + ebody.substr(0, 200);
    return -1;
  }
  if (verdict != 0) {
    if (verdict < 0) *err = last_error();
    return verdict;
  }
  return 0;
}

void Reflector::run() {
  double backoff = 0.05;
  bool need_list = true;
  auto sleep_backoff = [&] {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait_for(lk, std::chrono::duration<double>(backoff), [this] { return stop_.load() || relist_req_.load(); });
    backoff = std::min(rc_.backoff_max_s, backoff * 2);
  };
  while (!stop_.load()) {
    std::string err;
    try {
      if (relist_req_.exchange(false)) need_list = true;
      if (need_list) {
        if (!do_list(&err)) {
          set_error(err);
          sleep_backoff();
          continue;
        }
        need_list = false;
        if (!synced_.exchange(true)) {
          std::lock_guard<std::mutex> g(mu_);
          cv_.notify_all();
        }
      }
      int r = do_watch(&err);
      if (stop_.load()) break;
      if (relist_req_.load()) continue;  // ended on purpose: LIST next
      if (r == 1) {
        need_list = true;  // 410 Gone: history compacted past our resourceVersion
        continue;
      }
      if (r < 0) {
        set_error(err);
        sleep_backoff();
        continue;
      }
      backoff = 0.05;
      rewatches_++;
    } catch (const std::exception& e) {
      // a handler or a decode that throws must not end the process from this thread: start over from a LIST
      set_error(std::string("reflector: ") + e.what());
      need_list = true;
      sleep_backoff();
    }
  }
}

}  // namespace gsx
