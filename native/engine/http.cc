#include "http.h"

#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>

namespace gsx {
namespace http {

namespace {

std::string lower(std::string_view s) {
  std::string o(s);
  for (char& c : o) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return o;
}

std::string_view trim(std::string_view s) {
  while (!s.empty() && (s.front() == ' ' || s.front() == '\t')) s.remove_prefix(1);
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\r')) s.remove_suffix(1);
  return s;
}

bool contains_token(std::string_view v, std::string_view tok) {
  // comma-separated, case-insensitive
  size_t i = 0;
  while (i <= v.size()) {
    size_t j = v.find(',', i);
    if (j == std::string_view::npos) j = v.size();
    std::string_view t = trim(v.substr(i, j - i));
    if (t.size() == tok.size()) {
      bool eq = true;
      for (size_t k = 0; k < t.size(); ++k) {
        if (std::tolower(static_cast<unsigned char>(t[k])) != std::tolower(static_cast<unsigned char>(tok[k]))) {
          eq = false;
          break;
        }
      }
      if (eq) return true;
    }
    i = j + 1;
  }
  return false;
}

}  // namespace

bool parse_chunk_size(std::string_view hex, size_t limit, size_t* out) {
  // 1*HEXDIG only: no sign, no "0x", no whitespace; anything above `limit` is refused before it can wrap
  if (hex.empty() || hex.size() > 16) return false;
  size_t v = 0;
  for (char c : hex) {
    int d;
    if (c >= '0' && c <= '9') {
      d = c - '0';
    } else if (c >= 'a' && c <= 'f') {
      d = c - 'a' + 10;
    } else if (c >= 'A' && c <= 'F') {
      d = c - 'A' + 10;
    } else {
      return false;
    }
    if (static_cast<size_t>(d) > limit || v > (limit - static_cast<size_t>(d)) / 16) return false;
    v = v * 16 + static_cast<size_t>(d);
  }
  *out = v;
  return true;
}

const std::string* Message::header(std::string_view name) const {
  for (const auto& h : headers) {
    if (h.first == name) return &h.second;
  }
  return nullptr;
}

std::string_view Message::path() const {
  std::string_view t(target);
  size_t q = t.find('?');
  return q == std::string_view::npos ? t : t.substr(0, q);
}

long parse_head(const char* buf, size_t n, bool is_request, Message* out, std::string* err, long* content_length,
                bool* chunked) {
  std::string_view s(buf, n);
  size_t hend = s.find("\r\n\r\n");
  if (hend == std::string_view::npos) {
    if (n > (64u << 10)) {
      *err = "header too large";
      return -1;
    }
    return 0;
  }
  *out = Message();
  std::string_view head = s.substr(0, hend);
  size_t le = head.find("\r\n");
  std::string_view start = head.substr(0, le);
  // start line
  if (is_request) {
    size_t a = start.find(' ');
    size_t b = a == std::string_view::npos ? a : start.find(' ', a + 1);
    if (a == std::string_view::npos || b == std::string_view::npos) {
      *err = "bad request line";
      return -1;
    }
    out->method = std::string(start.substr(0, a));
    out->target = std::string(start.substr(a + 1, b - a - 1));
    std::string_view ver = start.substr(b + 1);
    if (ver.size() != 8 || ver.substr(0, 5) != "HTTP/") {
      *err = "bad http version";
      return -1;
    }
    out->minor_version = ver[7] - '0';
  } else {
    if (start.size() < 12 || start.substr(0, 5) != "HTTP/") {
      *err = "bad status line";
      return -1;
    }
    out->minor_version = start[7] - '0';
    out->status = std::atoi(std::string(start.substr(9, 3)).c_str());
    out->reason = start.size() > 13 ? std::string(start.substr(13)) : std::string();
  }
  // headers
  size_t pos = le == std::string_view::npos ? head.size() : le + 2;
  *content_length = -1;
  *chunked = false;
  bool conn_close = false, conn_keep = false;
  while (pos < head.size()) {
    size_t e = head.find("\r\n", pos);
    if (e == std::string_view::npos) e = head.size();
    std::string_view line = head.substr(pos, e - pos);
    size_t c = line.find(':');
    if (c == std::string_view::npos) {
      *err = "bad header line";
      return -1;
    }
    std::string name = lower(trim(line.substr(0, c)));
    std::string_view val = trim(line.substr(c + 1));
    if (name == "content-length") {
      char* endp = nullptr;
      std::string v(val);
      long cl = std::strtol(v.c_str(), &endp, 10);
      if (!endp || *endp || cl < 0) {
        *err = "bad content-length";
        return -1;
      }
      *content_length = cl;
    } else if (name == "transfer-encoding") {
      *chunked = contains_token(val, "chunked");
    } else if (name == "connection") {
      conn_close = contains_token(val, "close");
      conn_keep = contains_token(val, "keep-alive");
    }
    out->headers.emplace_back(std::move(name), std::string(val));
    pos = e + 2;
  }
  out->keep_alive = out->minor_version >= 1 ? !conn_close : conn_keep;
  return static_cast<long>(hend + 4);
}

long parse(const char* buf, size_t n, bool is_request, Message* out, std::string* err, bool eof, size_t max_body) {
  std::string_view s(buf, n);
  long content_length = -1;
  bool chunked = false;
  long hl = parse_head(buf, n, is_request, out, err, &content_length, &chunked);
  if (hl <= 0) return hl;
  size_t body_start = static_cast<size_t>(hl);
  if (chunked) {
    size_t p = body_start;
    std::string body;
    while (true) {
      size_t e = s.find("\r\n", p);
      if (e == std::string_view::npos) return 0;
      std::string_view szs = s.substr(p, e - p);
      size_t semi = szs.find(';');
      if (semi != std::string_view::npos) szs = szs.substr(0, semi);
      szs = trim(szs);
      size_t sz = 0;
      if (!parse_chunk_size(szs, max_body, &sz)) {
        *err = "bad chunk size";
        return -1;
      }
      p = e + 2;
      if (sz == 0) {
        // trailers until empty line
        while (true) {
          size_t e2 = s.find("\r\n", p);
          if (e2 == std::string_view::npos) return 0;
          if (e2 == p) {
            p += 2;
            break;
          }
          p = e2 + 2;
        }
        out->body = std::move(body);
        return static_cast<long>(p);
      }
      // invariant body.size() <= max_body and sz <= max_body: no subtraction or sum below can wrap
      if (sz > max_body - body.size()) {
        *err = "body too large";
        return -1;
      }
      if (p > n || n - p < sz + 2) return 0;
      body.append(buf + p, sz);
      p += sz + 2;
    }
  }
  if (content_length >= 0) {
    if (static_cast<size_t>(content_length) > max_body) {
      *err = "body too large";
      return -1;
    }
    if (n < body_start + static_cast<size_t>(content_length)) return 0;
    out->body.assign(buf + body_start, static_cast<size_t>(content_length));
    return static_cast<long>(body_start + static_cast<size_t>(content_length));
  }
  if (is_request || out->status == 204 || out->status == 304 || (out->status >= 100 && out->status < 200)) {
    return static_cast<long>(body_start);
  }
  // response delimited by connection close
  out->body_until_close = true;
  out->keep_alive = false;
  if (!eof) return 0;
  out->body.assign(buf + body_start, n - body_start);
  return static_cast<long>(n);
}

void MessageParser::reset() {
  scanned_ = 0;
  head_len_ = 0;
  head_ = Message();
  content_length_ = -1;
  chunked_ = false;
  cpos_ = 0;
  body_.clear();
}

long MessageParser::parse(const char* buf, size_t n, Message* out, std::string* err, size_t max_body, bool eof) {
  constexpr size_t kMaxHead = 64u << 10;
  std::string_view s(buf, n);
  if (head_len_ == 0) {
    size_t hend = s.find("\r\n\r\n", scanned_ > 3 ? scanned_ - 3 : 0);
    if (hend == std::string_view::npos) {
      scanned_ = n;
      if (n > kMaxHead) {
        *err = "header too large";
        reset();
        return -1;
      }
      return 0;
    }
    long hl = parse_head(buf, n, is_request_, &head_, err, &content_length_, &chunked_);
    if (hl <= 0) {
      reset();
      return -1;  // the terminator is there, so 0 cannot happen
    }
    head_len_ = hl;
    cpos_ = static_cast<size_t>(hl);
  }
  size_t used = static_cast<size_t>(head_len_);
  if (chunked_) {
    size_t p = cpos_;
    while (true) {
      size_t e = s.find("\r\n", p);
      if (e == std::string_view::npos) {
        if (n - p > kMaxHead) {  // a size line (or trailers) that never ends
          *err = "bad chunk size";
          reset();
          return -1;
        }
        return 0;
      }
      std::string_view szs = s.substr(p, e - p);
      size_t semi = szs.find(';');
      if (semi != std::string_view::npos) szs = szs.substr(0, semi);
      szs = trim(szs);
      size_t sz = 0;
      if (!parse_chunk_size(szs, max_body, &sz)) {
        *err = "bad chunk size";
        reset();
        return -1;
      }
      size_t q = e + 2;
      if (sz == 0) {
        while (true) {  // trailers until the empty line; resumed from the 0-size line if incomplete
          size_t e2 = s.find("\r\n", q);
          if (e2 == std::string_view::npos) {
            if (n - p > kMaxHead) {
              *err = "trailers too large";
              reset();
              return -1;
            }
            cpos_ = p;
            return 0;
          }
          if (e2 == q) {
            q += 2;
            break;
          }
          q = e2 + 2;
        }
        used = q;
        break;
      }
      if (sz > max_body - body_.size()) {  // body_.size() <= max_body, sz <= max_body: no wrap
        *err = "body too large";
        reset();
        return -1;
      }
      if (q > n || n - q < sz + 2) {
        cpos_ = p;  // this chunk is re-read once its data is in; the ones before stay decoded
        return 0;
      }
      body_.append(buf + q, sz);
      p = q + sz + 2;
      cpos_ = p;
    }
    *out = std::move(head_);
    out->body = std::move(body_);
  } else if (content_length_ >= 0) {
    if (static_cast<size_t>(content_length_) > max_body) {
      *err = "body too large";
      reset();
      return -1;
    }
    if (n < used + static_cast<size_t>(content_length_)) return 0;
    *out = std::move(head_);
    out->body.assign(buf + used, static_cast<size_t>(content_length_));
    used += static_cast<size_t>(content_length_);
  } else if (is_request_ || head_.status == 204 || head_.status == 304 || (head_.status >= 100 && head_.status < 200)) {
    *out = std::move(head_);  // no body
  } else {
    // a response delimited by the connection closing
    if (!eof) return 0;
    *out = std::move(head_);
    out->body_until_close = true;
    out->keep_alive = false;
    out->body.assign(buf + used, n - used);
    used = n;
  }
  reset();
  return static_cast<long>(used);
}

int Dechunker::feed(const char* data, size_t n, const std::function<void(std::string_view)>& out) {
  size_t i = 0;
  while (i < n) {
    switch (state_) {
      case State::Size: {
        char c = data[i++];
        if (c == '\n') {
          // size line complete (ignore extensions after ';')
          size_t semi = line_.find(';');
          if (semi != std::string::npos) line_.resize(semi);
          while (!line_.empty() && (line_.back() == '\r' || line_.back() == ' ')) line_.pop_back();
          size_t sz = 0;
          if (!parse_chunk_size(line_, size_t{1} << 40, &sz)) return -1;
          line_.clear();
          remaining_ = sz;
          state_ = sz == 0 ? State::Trailer : State::Data;
        } else {
          if (line_.size() > 64) return -1;
          line_.push_back(c);
        }
        break;
      }
      case State::Data: {
        size_t take = static_cast<size_t>(std::min<unsigned long long>(remaining_, n - i));
        out(std::string_view(data + i, take));
        i += take;
        remaining_ -= take;
        if (remaining_ == 0) state_ = State::DataEnd;
        break;
      }
      case State::DataEnd: {
        char c = data[i++];
        if (c == '\n') {
          state_ = State::Size;
        } else if (c != '\r') {
          return -1;
        }
        break;
      }
      case State::Trailer: {
        char c = data[i++];
        if (c == '\n') {
          if (line_.empty() || line_ == "\r") {
            state_ = State::Done;
            return 1;
          }
          line_.clear();
        } else {
          line_.push_back(c);
        }
        break;
      }
      case State::Done:
        return 1;
    }
  }
  return state_ == State::Done ? 1 : 0;
}

const char* reason_phrase(int status) {
  switch (status) {
    case 200: return "OK";
    case 201: return "Created";
    case 204: return "No Content";
    case 400: return "Bad Request";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 413: return "Payload Too Large";
    case 500: return "Internal Server Error";
    case 502: return "Bad Gateway";
    case 503: return "Service Unavailable";
    default: return "Status";
  }
}

std::string response(int status, std::string_view content_type, std::string_view body, bool keep_alive,
                     std::string_view extra_headers) {
  std::string o;
  o.reserve(160 + body.size());
  char line[96];
  int k = std::snprintf(line, sizeof(line), "HTTP/1.1 %d %s\r\n", status, reason_phrase(status));
  o.append(line, static_cast<size_t>(k));
  if (!content_type.empty()) {
    o.append("Content-Type: ");
    o.append(content_type);
    o.append("\r\n");
  }
  k = std::snprintf(line, sizeof(line), "Content-Length: %zu\r\n", body.size());
  o.append(line, static_cast<size_t>(k));
  if (!keep_alive) o.append("Connection: close\r\n");
  o.append(extra_headers);
  o.append("\r\n");
  o.append(body);
  return o;
}

bool parse_url(const std::string& s, Url* out) {
  *out = Url();
  std::string rest;
  if (s.rfind("https://", 0) == 0) {
    out->tls = true;
    out->port = 443;
    rest = s.substr(8);
  } else if (s.rfind("http://", 0) == 0) {
    rest = s.substr(7);
  } else {
    return false;
  }
  size_t slash = rest.find('/');
  std::string hostport = rest.substr(0, slash);
  if (slash != std::string::npos) {
    out->prefix = rest.substr(slash);
    while (!out->prefix.empty() && out->prefix.back() == '/') out->prefix.pop_back();
  }
  if (!hostport.empty() && hostport[0] == '[') {
    size_t rb = hostport.find(']');
    if (rb == std::string::npos) return false;
    out->host = hostport.substr(1, rb - 1);
    if (rb + 1 < hostport.size()) {
      if (hostport[rb + 1] != ':') return false;
      out->port = std::atoi(hostport.c_str() + rb + 2);
    }
  } else {
    size_t c = hostport.rfind(':');
    if (c != std::string::npos) {
      out->host = hostport.substr(0, c);
      out->port = std::atoi(hostport.c_str() + c + 1);
    } else {
      out->host = hostport;
    }
  }
  return !out->host.empty() && out->port > 0 && out->port < 65536;
}

}  // namespace http
}  // namespace gsx
