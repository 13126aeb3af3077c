"""HTTP management interface: /healthz /readyz /metrics / (+ /debug, REST, WS).

Parity: internal/httpserver/server.go
  * New / Start / Stop / SetReady / Addr / ServeError ...... server.go:81-168
  * /healthz "ok\\n"; /readyz "ready\\n" 200 | "not ready\\n" 503;
    /metrics text/plain; version=0.0.4; / index; 404 elsewhere  server.go:172-206
  * pprof mount (opt-in) -> /debug/pprof/{,goroutine,profile,heap}
    (Python equivalents: thread stacks, cProfile sample, gc/tracemalloc)
  * /debug/stats: raw native device counters + stripe/fault/stall state (JSON; MI355X
    addition), served whenever the owner registers a ``debug_stats`` provider
  * timeouts: 5 s header read / 10 s read / 10 s write / 60 s idle
Additions for the north star's "REST/WS API": GET /api/v1/{stats,devices,pool,node}
(JSON from provider callbacks) and a minimal RFC 6455 WebSocket at /ws that
pushes the stats JSON once per second. Unauthenticated: bind to loopback.
"""
from __future__ import annotations

import base64
import hashlib
import io
import json
import socket
import struct
import sys
import threading
import time
import traceback
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Callable

from otedama_amd.metrics import Registry

INDEX_HTML = """<!DOCTYPE html>
<html>
<head><title>Otedama</title></head>
<body>
<h1>Otedama</h1>
<p>MI355X mining engine and Stratum pool &mdash; HTTP management interface.</p>
<ul>
<li><a href="/metrics">/metrics</a> &mdash; Prometheus scrape endpoint</li>
<li><a href="/healthz">/healthz</a> &mdash; liveness probe</li>
<li><a href="/readyz">/readyz</a> &mdash; readiness probe</li>
<li><a href="/api/v1/stats">/api/v1/stats</a> &mdash; live stats (JSON); <code>/ws</code> streams them</li>
<li><a href="/debug/stats">/debug/stats</a> &mdash; per-device native counters, stripes, faults, stalls</li>
</ul>
</body>
</html>
"""

WS_GUID = "258EAFA5-E914-47DA-95CA-C5AB0DC85B11"
ApiProvider = Callable[[], object]


class _Handler(BaseHTTPRequestHandler):
    server_version = "otedama"
    sys_version = ""
    protocol_version = "HTTP/1.1"
    timeout = 10  # read/write timeout per socket op

    def log_message(self, fmt, *args):  # quiet; the engine logger owns stdout/stderr
        return

    @property
    def app(self) -> "HTTPServer":
        return self.server.app  # type: ignore[attr-defined]

    def _send(self, code: int, body: bytes, ctype: str) -> None:
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        if self.command != "HEAD":
            self.wfile.write(body)

    def do_HEAD(self):  # noqa: N802
        self.do_GET()

    def do_GET(self):  # noqa: N802
        path = self.path.split("?", 1)[0]
        app = self.app
        if path == "/healthz":
            return self._send(200, b"ok\n", "text/plain; charset=utf-8")
        if path == "/readyz":
            if app.ready:
                return self._send(200, b"ready\n", "text/plain; charset=utf-8")
            return self._send(503, b"not ready\n", "text/plain; charset=utf-8")
        if path == "/metrics":
            if app.registry is None:
                return self._send(500, b"metrics registry not configured\n", "text/plain; charset=utf-8")
            return self._send(200, app.registry.render().encode(), "text/plain; version=0.0.4; charset=utf-8")
        if path == "/":
            return self._send(200, INDEX_HTML.encode(), "text/html; charset=utf-8")
        if path.startswith("/api/v1/"):
            name = path[len("/api/v1/"):].strip("/")
            fn = app.api.get(name)
            if fn is None:
                return self._send(404, b'{"error":"not found"}\n', "application/json")
            try:
                body = json.dumps(fn(), default=_json_default).encode() + b"\n"
            except Exception as exc:  # noqa: BLE001
                return self._send(500, json.dumps({"error": str(exc)}).encode(), "application/json")
            return self._send(200, body, "application/json")
        if path == "/ws" and "stats" in app.api:
            return self._websocket(app.api["stats"])
        if path == "/debug/stats" and "debug_stats" in app.api:
            try:
                body = json.dumps(app.api["debug_stats"](), default=_json_default).encode() + b"\n"
            except Exception as exc:  # noqa: BLE001
                return self._send(500, json.dumps({"error": str(exc)}).encode(), "application/json")
            return self._send(200, body, "application/json")
        if app.pprof and path.startswith("/debug/pprof"):
            return self._pprof(path)
        return self._send(404, b"404 page not found\n", "text/plain; charset=utf-8")

    # ------------------------------------------------------------ debug
    def _pprof(self, path: str) -> None:
        name = path[len("/debug/pprof"):].strip("/")
        if name in ("", "index"):
            body = "/debug/pprof/goroutine (thread stacks)\n/debug/pprof/profile?seconds=N (cProfile)\n" \
                   "/debug/pprof/heap (gc counts; live allocations by line under PYTHONTRACEMALLOC=1)\n/debug/pprof/cmdline\n"
            return self._send(200, body.encode(), "text/plain; charset=utf-8")
        if name in ("goroutine", "threads"):
            frames = sys._current_frames()
            out = io.StringIO()
            for t in threading.enumerate():
                out.write(f"thread {t.name} (daemon={t.daemon}):\n")
                f = frames.get(t.ident)
                if f is not None:
                    out.write("".join(traceback.format_stack(f)))
                out.write("\n")
            return self._send(200, out.getvalue().encode(), "text/plain; charset=utf-8")
        if name == "cmdline":
            return self._send(200, "\x00".join(sys.argv).encode(), "text/plain; charset=utf-8")
        if name == "heap":
            import gc

            heap = {"gc_counts": gc.get_count(), "gc_stats": gc.get_stats(), "objects": len(gc.get_objects())}
            import tracemalloc

            if tracemalloc.is_tracing():  # PYTHONTRACEMALLOC=1 at start-up: the live allocations by source line
                snap = tracemalloc.take_snapshot().filter_traces(
                    (tracemalloc.Filter(False, tracemalloc.__file__), tracemalloc.Filter(False, "<frozen *>")))
                stats = snap.statistics("lineno")
                heap["traced_kib"] = round(sum(st.size for st in stats) / 1024, 1)
                heap["top"] = [{"where": f"{st.traceback[0].filename}:{st.traceback[0].lineno}",
                                "kib": round(st.size / 1024, 1), "blocks": st.count} for st in stats[:40]]
            body = json.dumps(heap)
            return self._send(200, body.encode(), "application/json")
        if name == "profile":
            import cProfile
            import pstats
            from urllib.parse import parse_qs, urlparse

            secs = float(parse_qs(urlparse(self.path).query).get("seconds", ["5"])[0])
            prof = cProfile.Profile()
            prof.enable()
            time.sleep(min(max(secs, 0.1), 60.0))
            prof.disable()
            out = io.StringIO()
            pstats.Stats(prof, stream=out).sort_stats("cumulative").print_stats(50)
            return self._send(200, out.getvalue().encode(), "text/plain; charset=utf-8")
        return self._send(404, b"404 page not found\n", "text/plain; charset=utf-8")

    # ------------------------------------------------------------ websocket
    def _websocket(self, fn: ApiProvider) -> None:
        key = self.headers.get("Sec-WebSocket-Key")
        if not key or self.headers.get("Upgrade", "").lower() != "websocket":
            return self._send(400, b"expected websocket upgrade\n", "text/plain; charset=utf-8")
        accept = base64.b64encode(hashlib.sha1((key + WS_GUID).encode()).digest()).decode()
        self.send_response(101, "Switching Protocols")
        self.send_header("Upgrade", "websocket")
        self.send_header("Connection", "Upgrade")
        self.send_header("Sec-WebSocket-Accept", accept)
        self.end_headers()
        self.wfile.flush()
        self.close_connection = True
        sock = self.connection
        sock.settimeout(1.0)
        while not self.app.stopping.is_set():
            try:
                payload = json.dumps(fn(), default=_json_default).encode()
                sock.sendall(ws_frame(payload))
                try:  # drain client frames (close / ping) without blocking long
                    data = sock.recv(4096)
                    if not data or (data[0] & 0x0F) == 0x8:
                        break
                except socket.timeout:
                    pass
            except OSError:
                break


def ws_frame(payload: bytes, opcode: int = 0x1) -> bytes:
    n = len(payload)
    if n < 126:
        hdr = struct.pack("!BB", 0x80 | opcode, n)
    elif n < 65536:
        hdr = struct.pack("!BBH", 0x80 | opcode, 126, n)
    else:
        hdr = struct.pack("!BBQ", 0x80 | opcode, 127, n)
    return hdr + payload


def _json_default(o):
    if isinstance(o, bytes):
        return o.hex()
    if hasattr(o, "to_dict"):
        return o.to_dict()
    if hasattr(o, "__dict__"):
        return o.__dict__
    return str(o)


class _Server(ThreadingHTTPServer):
    daemon_threads = True
    allow_reuse_address = True

    def __init__(self, addr, handler, app):
        self.app = app
        super().__init__(addr, handler)

    def get_request(self):
        sock, addr = super().get_request()
        sock.settimeout(_Handler.timeout)
        return sock, addr


class HTTPServer:
    def __init__(self, addr: str, registry: Registry | None, enable_pprof: bool = False,
                 api: dict[str, ApiProvider] | None = None):
        self.addr_config = addr
        self.registry = registry
        self.pprof = enable_pprof
        self.api: dict[str, ApiProvider] = dict(api or {})
        self._ready = threading.Event()
        self.stopping = threading.Event()
        self._srv: _Server | None = None
        self._thread: threading.Thread | None = None
        self._bound: str | None = None
        self._serve_error: BaseException | None = None

    @property
    def ready(self) -> bool:
        return self._ready.is_set()

    def set_ready(self, ready: bool) -> None:
        (self._ready.set if ready else self._ready.clear)()

    def start(self) -> None:
        host, _, port = self.addr_config.rpartition(":")
        host = host.strip("[]") or "0.0.0.0"
        try:
            self._srv = _Server((host, int(port or 0)), _Handler, self)
        except OSError as exc:
            raise OSError(f"httpserver: listen on {self.addr_config}: {exc}") from exc
        h, p = self._srv.server_address[:2]
        self._bound = f"{h}:{p}"

        def serve():
            try:
                self._srv.serve_forever(poll_interval=0.2)
            except BaseException as exc:  # noqa: BLE001
                self._serve_error = exc

        self._thread = threading.Thread(target=serve, name="otedama-http", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self.stopping.set()
        if self._srv is not None:
            self._srv.shutdown()
            self._srv.server_close()
        if self._thread is not None:
            self._thread.join(timeout=5.0)

    @property
    def addr(self) -> str:
        return self._bound or self.addr_config

    def serve_error(self) -> BaseException | None:
        return self._serve_error
