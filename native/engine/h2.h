// Minimal gRPC-over-HTTP/2 transport for the kubelet device-plugin API (unix sockets, no TLS), on the system's
// libnghttp2 (dlopen'ed: framing, HPACK, flow control) — the device plugin's hot RPCs without grpcio's
// ~0.2-0.4 ms per call (profiles/r03b/README.md).
//
//  * Server: poll-driven (no threads of its own).  Its epoll fd is handed to the owner's event loop (the
//    plugin's asyncio loop, via loop.add_reader); poll() accepts, reads, dispatches complete requests to the
//    handler and writes.  A handler answers at once (respond) or later (the call id stays valid until then);
//    server-streaming calls (ListAndWatch) stay open and get messages with stream_send().
//  * Client: blocking unary / server-streaming calls on one connection (the compiled kubelet stand-in).
//
// gRPC framing: a message is a 1-byte compressed flag (always 0 here) + 4-byte big-endian length + payload;
// status travels in trailers (grpc-status, grpc-message), or in a trailers-only response for errors.
#pragma once

#include <cstdint>
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace gsx::h2 {

// dlopen libnghttp2 once; false (with *err) if the library is not on this system
bool available(std::string* err = nullptr);

std::string grpc_frame(const std::string& payload);
// Splits complete gRPC messages off the front of `buf` (consumed); false on a malformed / compressed frame.
bool grpc_unframe(std::string* buf, std::vector<std::string>* out);

struct Call {
  uint64_t id = 0;
  std::string path;     // "/v1beta1.DevicePlugin/Allocate"
  std::string message;  // the request message (unary / server-streaming: exactly one)
};

class Server {
 public:
  using Handler = std::function<void(Server&, const Call&)>;

  // Listens on `unix_path` (replacing a stale socket file).  ok() false: *init_error says why.
  Server(const std::string& unix_path, Handler handler);
  ~Server();
  Server(const Server&) = delete;
  Server& operator=(const Server&) = delete;

  bool ok() const { return ok_; }
  const std::string& init_error() const { return err_; }
  int fd() const { return ep_; }  // readable when poll() has work
  void watch_fd(int fd);          // another fd that should wake the owner (poll() leaves it alone)

  // Non-blocking: accept, read, dispatch, write.  Returns the number of requests dispatched.
  int poll();

  // Unary answer (status 0 + message) or error (status != 0, message = grpc-message).  false: the call is gone.
  bool respond(uint64_t call, int status, const std::string& payload_or_message);
  // Server streaming: one more message / the end (trailers).
  bool stream_send(uint64_t call, const std::string& payload);
  bool stream_end(uint64_t call, int status, const std::string& message);
  std::vector<uint64_t> open_streams(const std::string& path) const;

  uint64_t calls() const { return calls_; }
  uint64_t connections() const { return conns_total_; }

  struct Conn;
  struct Stream;

 private:
  friend struct Callbacks;
  void accept_all();
  bool read_conn(Conn* c);
  bool flush_conn(Conn* c);
  void close_conn(int fd);
  Stream* find(uint64_t call, Conn** conn);
  void dispatch(Conn* c, Stream* s);
  void submit(Conn* c, Stream* s);

  std::string path_;
  Handler handler_;
  int lfd_ = -1, ep_ = -1;
  bool ok_ = false;
  std::string err_;
  std::map<int, std::unique_ptr<Conn>> conns_;
  std::map<uint64_t, std::pair<int, int32_t>> calls_by_id_;  // call id -> (conn fd, stream id)
  uint64_t next_call_ = 1, calls_ = 0, conns_total_ = 0;
  std::vector<std::pair<Conn*, Stream*>> ready_;  // complete requests found during one read
};

class Client {
 public:
  explicit Client(const std::string& unix_path);
  ~Client();
  Client(const Client&) = delete;
  Client& operator=(const Client&) = delete;

  // Unary call: true + *resp on grpc-status 0; false: *status (grpc or -1 transport) and *err.
  bool call(const std::string& path, const std::string& req, std::string* resp, int* status, std::string* err,
            double timeout_s = 10.0);
  // Server streaming: reads until `max_messages` arrived (or the stream ends / timeout), then cancels.
  bool stream(const std::string& path, const std::string& req, size_t max_messages, std::vector<std::string>* out,
              int* status, std::string* err, double timeout_s = 10.0);

  struct Impl;

 private:
  std::unique_ptr<Impl> impl_;
};

}  // namespace gsx::h2
