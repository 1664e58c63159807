// Minimal HTTP/1.1 message parsing / serialisation for the native extender
// server and its apiserver client.
//
// The reference serves kube-scheduler with Go's net/http
// (pkg/routes/routes.go, cmd/main.go:128) and talks to kube-apiserver with
// client-go.  The native equivalents only need: request/response start lines,
// headers, Content-Length and chunked bodies, keep-alive.
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <string_view>
#include <utility>
#include <vector>

namespace gsx {
namespace http {

struct Message {
  // request
  std::string method;
  std::string target;  // path + optional ?query
  // response
  int status = 0;
  std::string reason;
  // both
  int minor_version = 1;
  std::vector<std::pair<std::string, std::string>> headers;  // names lower-cased
  std::string body;
  bool keep_alive = true;
  bool body_until_close = false;  // response without length: read to EOF

  const std::string* header(std::string_view lower_name) const;
  std::string_view path() const;  // target without query
};

// Parse one complete message from buf[0..n).  Returns the number of bytes
// consumed (> 0), 0 if more input is needed, -1 on a malformed message.
// `eof` tells the parser the peer closed (completes read-to-close bodies).
long parse(const char* buf, size_t n, bool is_request, Message* out, std::string* err, bool eof = false,
           size_t max_body = 64u << 20);

// Parse only the start line + headers.  Returns the head length (> 0), 0 if
// more input is needed, -1 if malformed.  *content_length = -1 when absent.
long parse_head(const char* buf, size_t n, bool is_request, Message* out, std::string* err, long* content_length,
                bool* chunked);

// A chunk-size token (1*HEXDIG, extensions already stripped) no larger than
// `limit`.  Rejects signs, prefixes, empty and over-long input, and any value
// above `limit` before it can wrap.
bool parse_chunk_size(std::string_view hex, size_t limit, size_t* out);

// Incremental Transfer-Encoding: chunked decoder for streamed bodies (watch
// responses).  feed() passes decoded bytes to `out`; returns 1 once the
// terminating chunk (and trailers) were consumed, 0 if more input is needed,
// -1 on malformed framing.
class Dechunker {
 public:
  int feed(const char* data, size_t n, const std::function<void(std::string_view)>& out);
  bool done() const { return state_ == State::Done; }

 private:
  enum class State { Size, Data, DataEnd, Trailer, Done };
  State state_ = State::Size;
  std::string line_;
  unsigned long long remaining_ = 0;
};

// Resumable parser for one connection's input buffer.  Same contract as
// parse(), but the work done on an incomplete message is kept: the head search
// resumes where it stopped and complete chunks stay decoded, so a message that
// arrives in many small reads costs O(bytes), not O(bytes^2) (one re-parse of
// the whole buffer per read).  `buf` must always start at the current message;
// after a return != 0 the parser is ready for the next one.
class MessageParser {
 public:
  explicit MessageParser(bool is_request = true) : is_request_(is_request) {}
  long parse(const char* buf, size_t n, Message* out, std::string* err, size_t max_body = 64u << 20,
             bool eof = false);
  void reset();

 private:
  bool is_request_;
  size_t scanned_ = 0;  // bytes already searched for the end of the head
  long head_len_ = 0;   // > 0 once the head is parsed
  Message head_;
  long content_length_ = -1;
  bool chunked_ = false;
  size_t cpos_ = 0;  // offset of the next chunk-size line
  std::string body_;
};

// Serialise a response.
std::string response(int status, std::string_view content_type, std::string_view body, bool keep_alive,
                     std::string_view extra_headers = {});

const char* reason_phrase(int status);

// scheme://host[:port][/prefix] -> parts.  Returns false if malformed.
struct Url {
  bool tls = false;
  std::string host;  // without brackets
  int port = 80;
  std::string prefix;  // path prefix without trailing slash
};
bool parse_url(const std::string& s, Url* out);

}  // namespace http
}  // namespace gsx
