"""Lean HTTP/1.1 server + client on raw asyncio (protocols / streams), for the control plane's many small calls.

Every hop of a pod's life (create -> watch -> filter -> bind -> watch ->
Allocate -> status -> watch) is a small JSON request on a keep-alive
connection.  aiohttp spends most of its per-request budget in machinery we do
not need (middlewares, multipart, cookie jars, tracing signals).  This module
keeps only: request line + headers, Content-Length / chunked bodies,
keep-alive, chunked streaming responses (watch), TLS via ``ssl`` contexts, and
a connection pool on the client.  The fake apiserver, the Kubernetes client,
the scheduler simulator and the runtime shims all use it.
"""
from __future__ import annotations

import asyncio
import json
import ssl as _ssl
from urllib.parse import parse_qsl, unquote, urlsplit

REASONS = {200: "OK", 201: "Created", 202: "Accepted", 204: "No Content", 400: "Bad Request", 401: "Unauthorized",
           403: "Forbidden", 404: "Not Found", 405: "Method Not Allowed", 409: "Conflict", 410: "Gone",
           415: "Unsupported Media Type", 422: "Unprocessable Entity", 429: "Too Many Requests",
           500: "Internal Server Error", 502: "Bad Gateway", 503: "Service Unavailable"}


class HTTPError(Exception):
    """Raise from a handler to answer with ``status`` and a JSON (or text) body."""

    def __init__(self, status: int, body: bytes | str | dict = b"", content_type: str = "application/json"):
        super().__init__(status)
        self.status = status
        if isinstance(body, dict):
            body = json.dumps(body, separators=(",", ":"))
        self.body = body.encode() if isinstance(body, str) else body
        self.content_type = content_type


class Request:
    __slots__ = ("method", "target", "path", "query_string", "headers", "body", "match_info", "transport", "_query")

    def __init__(self, method: str, target: str, headers: dict, body: bytes, transport):
        self.method = method
        self.target = target
        p, _, q = target.partition("?")
        self.path = unquote(p)
        self.query_string = q
        self.headers = headers
        self.body = body
        self.match_info: dict = {}
        self.transport = transport
        self._query = None

    @property
    def query(self) -> dict:
        if self._query is None:
            self._query = dict(parse_qsl(self.query_string, keep_blank_values=True))
        return self._query

    def json(self):
        return json.loads(self.body) if self.body else None

    @property
    def closed(self) -> bool:
        return self.transport is None or self.transport.is_closing()


class Response:
    __slots__ = ("status", "body", "content_type", "headers")

    def __init__(self, body: bytes | str = b"", status: int = 200, content_type: str = "application/json",
                 headers: dict | None = None):
        self.status = status
        self.body = body.encode() if isinstance(body, str) else body
        self.content_type = content_type
        self.headers = headers

    @staticmethod
    def json(obj, status: int = 200) -> "Response":
        return Response(json.dumps(obj, separators=(",", ":")).encode(), status)


class Stream:
    """Chunked streaming response (a watch).  Write with :meth:`write`; the handler returns when done."""

    def __init__(self, transport, content_type: str = "application/json"):
        self.transport = transport
        self.content_type = content_type
        self.started = False

    def start(self):
        if not self.started:
            self.transport.write(b"HTTP/1.1 200 OK\r\nContent-Type: " + self.content_type.encode() +
                                 b"\r\nTransfer-Encoding: chunked\r\n\r\n")
            self.started = True

    def write(self, data: bytes):
        self.start()
        if data and not self.transport.is_closing():
            self.transport.write(b"%x\r\n%s\r\n" % (len(data), data))

    def finish(self):
        self.start()
        if not self.transport.is_closing():
            self.transport.write(b"0\r\n\r\n")

    @property
    def closed(self) -> bool:
        return self.transport.is_closing()


def _serialize(resp: Response, keep_alive: bool) -> bytes:
    head = [b"HTTP/1.1 %d %s\r\n" % (resp.status, REASONS.get(resp.status, "Status").encode())]
    if resp.content_type:
        head.append(b"Content-Type: " + resp.content_type.encode() + b"\r\n")
    head.append(b"Content-Length: %d\r\n" % len(resp.body))
    if resp.headers:
        for k, v in resp.headers.items():
            head.append(f"{k}: {v}\r\n".encode())
    if not keep_alive:
        head.append(b"Connection: close\r\n")
    head.append(b"\r\n")
    head.append(resp.body)
    return b"".join(head)


class Router:
    """Exact paths plus ``/a/{x}/b`` templates (segment captures)."""

    def __init__(self):
        self.exact: dict[tuple[str, str], object] = {}
        self.templates: dict[tuple[str, int], list] = {}

    def add(self, method: str, path: str, handler):
        if "{" not in path:
            self.exact[(method, path)] = handler
            return
        segs = path.strip("/").split("/")
        self.templates.setdefault((method, len(segs)), []).append((segs, handler))

    def resolve(self, method: str, path: str):
        h = self.exact.get((method, path))
        if h is not None:
            return h, {}
        segs = path.strip("/").split("/")
        for tsegs, handler in self.templates.get((method, len(segs)), ()):
            m = {}
            for t, s in zip(tsegs, segs):
                if t.startswith("{"):
                    m[t[1:-1]] = s
                elif t != s:
                    break
            else:
                return handler, m
        return None, None


class _ServerProtocol(asyncio.Protocol):
    def __init__(self, server: "Server"):
        self.server = server
        self.buf = bytearray()
        self.transport = None
        self.busy = False
        self.closed = False

    def connection_made(self, transport):
        self.transport = transport
        self.server.conns.add(self)

    def connection_lost(self, exc):
        self.closed = True
        self.server.conns.discard(self)

    def data_received(self, data: bytes):
        self.buf += data
        if not self.busy:
            self._process()

    def _process(self):
        while not self.busy and not self.closed:
            i = self.buf.find(b"\r\n\r\n")
            if i < 0:
                if len(self.buf) > 1 << 16:
                    self._fail(400, b"header too large")
                return
            head = bytes(self.buf[:i]).decode("latin-1")
            lines = head.split("\r\n")
            try:
                method, target, version = lines[0].split(" ", 2)
            except ValueError:
                self._fail(400, b"bad request line")
                return
            headers = {}
            for ln in lines[1:]:
                k, _, v = ln.partition(":")
                headers[k.strip().lower()] = v.strip()
            start = i + 4
            te = headers.get("transfer-encoding", "")
            if "chunked" in te.lower():
                body, used = _dechunk(self.buf, start)
                if body is None:
                    return
                end = used
            else:
                n = int(headers.get("content-length", "0") or 0)
                if len(self.buf) < start + n:
                    return
                body = bytes(self.buf[start:start + n])
                end = start + n
            del self.buf[:end]
            conn = headers.get("connection", "").lower()
            keep = ("close" not in conn) if version == "HTTP/1.1" else ("keep-alive" in conn)
            req = Request(method, target, headers, body, self.transport)
            handler, match = self.server.router.resolve(method, req.path)
            if handler is None:
                self._write(Response(b"404 page not found\n", 404, "text/plain"), keep)
                continue
            req.match_info = match
            try:
                res = handler(req)
            except HTTPError as e:
                self._write(Response(e.body, e.status, e.content_type), keep)
                continue
            except Exception as e:  # noqa: BLE001
                self._write(Response(repr(e).encode(), 500, "text/plain"), keep)
                continue
            if asyncio.iscoroutine(res):
                self.busy = True
                t = asyncio.get_running_loop().create_task(self._finish(res, req, keep))
                self.server.tasks.add(t)
                t.add_done_callback(self.server.tasks.discard)
                # a task cancelled before its first step (the server closing) never awaits the handler's coroutine
                t.add_done_callback(lambda _t, c=res: c.close())
                return
            self._write(res, keep)

    async def _finish(self, coro, req, keep):
        try:
            res = await coro
        except HTTPError as e:
            res = Response(e.body, e.status, e.content_type)
        except asyncio.CancelledError:
            res = None
        except Exception as e:  # noqa: BLE001
            res = Response(repr(e).encode(), 500, "text/plain")
        self.busy = False
        if isinstance(res, Stream) or res is None:
            # a finished watch stream: the connection cannot carry another request cleanly unless finished
            if isinstance(res, Stream) and not self.closed:
                res.finish()
                if not keep:
                    self.transport.close()
            return
        self._write(res, keep)
        if self.buf and not self.closed:
            self._process()

    def _write(self, res: Response, keep: bool):
        if self.closed:
            return
        self.transport.write(_serialize(res, keep))
        if not keep:
            self.transport.close()
            self.closed = True

    def _fail(self, status: int, msg: bytes):
        self._write(Response(msg, status, "text/plain"), False)


def _dechunk(buf, pos: int):
    """Decode a chunked body starting at ``pos``; returns (body, end) or (None, None) if incomplete."""
    out = bytearray()
    while True:
        e = buf.find(b"\r\n", pos)
        if e < 0:
            return None, None
        size = int(bytes(buf[pos:e]).split(b";", 1)[0], 16)
        pos = e + 2
        if size == 0:
            while True:
                e = buf.find(b"\r\n", pos)
                if e < 0:
                    return None, None
                if e == pos:
                    return bytes(out), pos + 2
                pos = e + 2
        if len(buf) < pos + size + 2:
            return None, None
        out += buf[pos:pos + size]
        pos += size + 2


class Server:
    def __init__(self, router: Router | None = None):
        self.router = router or Router()
        self.conns: set[_ServerProtocol] = set()
        self.tasks: set[asyncio.Task] = set()
        self._srv: asyncio.AbstractServer | None = None
        self.port = 0

    def route(self, method: str, path: str, handler):
        self.router.add(method, path, handler)

    async def start(self, host: str = "127.0.0.1", port: int = 0, ssl_context=None) -> int:
        loop = asyncio.get_running_loop()
        self._srv = await loop.create_server(lambda: _ServerProtocol(self), host, port, backlog=1024,
                                             reuse_address=True, ssl=ssl_context)
        self.port = self._srv.sockets[0].getsockname()[1]
        return self.port

    async def stop(self):
        if self._srv is not None:
            self._srv.close()
        for t in list(self.tasks):
            t.cancel()
        for c in list(self.conns):
            if c.transport is not None:
                c.transport.close()
        if self._srv is not None:
            try:
                await asyncio.wait_for(self._srv.wait_closed(), 2.0)
            except asyncio.TimeoutError:
                pass


# ---------------------------------------------------------------- client

class ClientResponse:
    __slots__ = ("status", "headers", "body")

    def __init__(self, status: int, headers: dict, body: bytes):
        self.status = status
        self.headers = headers
        self.body = body

    def json(self):
        return json.loads(self.body) if self.body else None


class _Conn:
    __slots__ = ("reader", "writer")

    def __init__(self, reader, writer):
        self.reader = reader
        self.writer = writer

    def close(self):
        try:
            self.writer.close()
        except Exception:  # noqa: BLE001
            pass


async def _read_head(reader) -> tuple[int, dict]:
    head = await reader.readuntil(b"\r\n\r\n")
    lines = head[:-4].decode("latin-1").split("\r\n")
    parts = lines[0].split(" ", 2)
    status = int(parts[1])
    headers = {}
    for ln in lines[1:]:
        k, _, v = ln.partition(":")
        headers[k.strip().lower()] = v.strip()
    return status, headers


async def _read_body(reader, headers: dict) -> tuple[bytes, bool]:
    """Returns (body, reusable)."""
    if "chunked" in headers.get("transfer-encoding", "").lower():
        out = bytearray()
        while True:
            ln = await reader.readuntil(b"\r\n")
            size = int(ln[:-2].split(b";", 1)[0], 16)
            if size == 0:
                while (await reader.readuntil(b"\r\n")) != b"\r\n":
                    pass
                return bytes(out), True
            out += await reader.readexactly(size + 2)
            del out[-2:]
    if "content-length" in headers:
        n = int(headers["content-length"])
        return (await reader.readexactly(n)) if n else b"", True
    return await reader.read(), False


class Client:
    """Keep-alive HTTP/1.1 client bound to one base URL (``http://`` or ``https://``)."""

    def __init__(self, base_url: str, *, ssl_context=None, headers: dict | None = None, limit: int = 256,
                 timeout: float | None = 30.0):
        u = urlsplit(base_url)
        self.scheme = u.scheme
        self.host = u.hostname or "127.0.0.1"
        self.port = u.port or (443 if u.scheme == "https" else 80)
        self.prefix = u.path.rstrip("/")
        self.ssl = ssl_context if u.scheme == "https" else None
        if u.scheme == "https" and self.ssl is None:
            self.ssl = _ssl.create_default_context()
        hostport = self.host if self.port in (80, 443) else f"{self.host}:{self.port}"
        self._base = {"Host": hostport, "Accept": "application/json"}
        self._base.update(headers or {})
        self._base_head = "".join(f"{k}: {v}\r\n" for k, v in self._base.items()).encode()
        self.idle: list[_Conn] = []
        self.limit = limit
        self.timeout = timeout
        self.closed = False

    def set_header(self, name: str, value: str) -> None:
        """Replace a header sent with every request (e.g. a rotated bearer token)."""
        self._base[name] = value
        self._base_head = "".join(f"{k}: {v}\r\n" for k, v in self._base.items()).encode()

    async def _open(self) -> _Conn:
        r, w = await asyncio.open_connection(self.host, self.port, ssl=self.ssl, limit=1 << 22)
        return _Conn(r, w)

    def _req_bytes(self, method: str, path: str, body: bytes | None, content_type: str | None,
                   extra: dict | None) -> bytes:
        h = [f"{method} {self.prefix}{path} HTTP/1.1\r\n".encode(), self._base_head]
        if extra:
            h.append("".join(f"{k}: {v}\r\n" for k, v in extra.items()).encode())
        if body is not None:
            h.append(b"Content-Type: " + (content_type or "application/json").encode() + b"\r\n")
            h.append(b"Content-Length: %d\r\n" % len(body))
        h.append(b"\r\n")
        if body:
            h.append(body)
        return b"".join(h)

    async def request(self, method: str, path: str, body: bytes | None = None, content_type: str | None = None,
                      headers: dict | None = None, timeout: float | None = -1.0) -> ClientResponse:
        data = self._req_bytes(method, path, body, content_type, headers)
        tmo = self.timeout if timeout == -1.0 else timeout
        # one timer that cancels this task (asyncio.wait_for would wrap every read in a new task)
        timer = fired = None
        if tmo:
            task = asyncio.current_task()
            fired = []

            def _expire():
                fired.append(True)
                task.cancel()
            timer = asyncio.get_running_loop().call_later(tmo, _expire)
        try:
            return await self._request(method, path, data)
        except asyncio.CancelledError:
            if fired:
                raise asyncio.TimeoutError(f"{method} {path}: no response in {tmo}s") from None
            raise
        finally:
            if timer is not None:
                timer.cancel()

    async def _request(self, method: str, path: str, data: bytes) -> "ClientResponse":
        for attempt in range(2):
            reused = bool(self.idle)
            c = self.idle.pop() if reused else await self._open()
            try:
                c.writer.write(data)
                status, hdrs = await _read_head(c.reader)
                rbody, reusable = await _read_body(c.reader, hdrs)
            except (asyncio.IncompleteReadError, ConnectionError, OSError) as e:
                c.close()
                if reused and attempt == 0:
                    continue  # stale keep-alive connection
                raise ConnectionError(f"{method} {path}: {e!r}") from e
            except BaseException:
                c.close()
                raise
            if reusable and "close" not in hdrs.get("connection", "").lower() and len(self.idle) < self.limit \
                    and not self.closed:
                self.idle.append(c)
            else:
                c.close()
            return ClientResponse(status, hdrs, rbody)
        raise ConnectionError(f"{method} {path}: failed")

    async def stream(self, method: str, path: str, headers: dict | None = None):
        """Open a streaming request; returns (status, headers, async iterator of body chunks, closer)."""
        c = await self._open()
        c.writer.write(self._req_bytes(method, path, None, None, headers))
        status, hdrs = await _read_head(c.reader)
        chunked = "chunked" in hdrs.get("transfer-encoding", "").lower()

        async def chunks():
            try:
                if not chunked:
                    if "content-length" in hdrs:
                        yield await c.reader.readexactly(int(hdrs["content-length"]))
                        return
                    while True:
                        d = await c.reader.read(65536)
                        if not d:
                            return
                        yield d
                while True:
                    ln = await c.reader.readuntil(b"\r\n")
                    size = int(ln[:-2].split(b";", 1)[0], 16)
                    if size == 0:
                        return
                    d = await c.reader.readexactly(size + 2)
                    yield d[:-2]
            finally:
                c.close()
        return status, hdrs, chunks(), c.close

    async def close(self):
        self.closed = True
        for c in self.idle:
            c.close()
        self.idle.clear()
