"""A torch-free host for the node's rendezvous store: the server side of torch.distributed's TCPStore protocol.

The node supervisor (parallel/launch.py ``supervise_node``) hosts the store that outlives any rank: the RCCL/gloo
rendezvous of every process-group generation and the node's op log live in it (parallel/node.py). Hosting it with
``torch.distributed.TCPStore`` cost the supervisor an ``import torch``: 570-600 MiB RSS, ~250 MiB of it anonymous,
for a process that never touches a tensor. This server speaks the same wire protocol from the standard library, so
the ranks keep using plain ``dist.TCPStore`` clients (``is_master=False``) and the supervisor stays at ~25 MiB.

Wire format (client -> server, little endian, as torch's TCPStore client writes it): one query-type byte, then
strings and byte vectors as a uint64 length + bytes, counts as uint64, ADD deltas as int64, VALIDATE's magic and
PING's nonce as uint32. Responses: GET/COMPARE_SET a vector, ADD/DELETE_KEY/GETNUMKEYS an int64, CHECK one
status byte, WAIT one byte when every key exists (or WAIT_CANCELED after CANCEL_WAIT), PING the nonce back.
ADD keeps its counter as decimal text, as torch's server does (a GET of an added key returns b"3").

Reference analogue: the reference has no multi-process store (one Go process per host); its closest piece is the
engine's shared job state (internal/engine/run.go). Parity is with torch's TCPStore semantics, pinned by
tests/test_kvstore.py against torch's own clients.
"""
from __future__ import annotations

import selectors
import socket
import struct
import threading
from collections import defaultdict

VALIDATE, SET, COMPARE_SET, GET, ADD, CHECK, WAIT, GETNUMKEYS, DELETE_KEY, APPEND, MULTI_GET, MULTI_SET, \
    CANCEL_WAIT, PING, QUEUE_PUSH, QUEUE_POP, QUEUE_LEN, LIST_KEYS = range(18)
MAGIC = 0x3C85F7CE
READY, NOT_READY = 0, 1
STOP_WAITING, WAIT_CANCELED = 0, 1

_U8, _U32, _U64, _I64 = struct.Struct("<B"), struct.Struct("<I"), struct.Struct("<Q"), struct.Struct("<q")
TX_CAP = 16 << 20  # replies queued for one peer that is not reading; past this the peer is dropped


class _Incomplete(Exception):
    pass


class _Reader:
    """Cursor over a connection's receive buffer; raises _Incomplete when a request is not all there yet."""

    __slots__ = ("buf", "pos")

    def __init__(self, buf: bytearray):
        self.buf, self.pos = buf, 0

    def take(self, n: int) -> bytes:
        if self.pos + n > len(self.buf):
            raise _Incomplete
        b = bytes(self.buf[self.pos:self.pos + n])
        self.pos += n
        return b

    def u32(self) -> int:
        return _U32.unpack(self.take(4))[0]

    def u64(self) -> int:
        return _U64.unpack(self.take(8))[0]

    def i64(self) -> int:
        return _I64.unpack(self.take(8))[0]

    def blob(self) -> bytes:
        return self.take(self.u64())


def _vec(b: bytes) -> bytes:
    return _U64.pack(len(b)) + b


class _Conn:
    __slots__ = ("sock", "rx", "tx", "validated", "waiting")

    def __init__(self, sock: socket.socket):
        self.sock, self.rx, self.tx = sock, bytearray(), bytearray()
        self.validated = False
        self.waiting: list[set[bytes]] = []  # outstanding WAITs, in arrival order (answered in order)


class StoreServer:
    """TCPStore-protocol server on a background thread. ``set`` / ``get`` / ``delete_key`` / ``add`` are also
    callable in-process (the supervisor marks dead ranks and the stop flag with them). They take the keys a client
    passes: torch's client puts "/" in front of every key on the wire, and so do they."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, backlog: int = 256):
        self._lsock = socket.create_server((host, port), backlog=backlog, reuse_port=False)
        self._lsock.setblocking(False)
        self.port = self._lsock.getsockname()[1]
        self._data: dict[bytes, bytes] = {}
        self._waiters: dict[bytes, list[_Conn]] = defaultdict(list)  # key -> conns with a WAIT that names it
        self._lock = threading.Lock()
        self._sel = selectors.DefaultSelector()
        self._sel.register(self._lsock, selectors.EVENT_READ, None)
        self._wake_r, self._wake_w = socket.socketpair()
        self._wake_r.setblocking(False)
        self._sel.register(self._wake_r, selectors.EVENT_READ, "wake")
        self._dirty: set[_Conn] = set()  # connections with replies to send
        self.refused = 0  # peers dropped for a bad magic, a query before VALIDATE or a query type not served here
        self._stop = False
        self._thread = threading.Thread(target=self._run, name="otd-store", daemon=True)
        self._thread.start()

    # ---- in-process API (same semantics as the wire ops) ----
    def set(self, key: str | bytes, value: str | bytes) -> None:
        with self._lock:
            self._set(_k(key), _b(value))
        self._kick()

    def get(self, key: str | bytes) -> bytes | None:
        with self._lock:
            return self._data.get(_k(key))

    def add(self, key: str | bytes, delta: int) -> int:
        with self._lock:
            v = self._add(_k(key), delta)
        self._kick()
        return v

    def delete_key(self, key: str | bytes) -> bool:
        with self._lock:
            return self._data.pop(_k(key), None) is not None

    def num_keys(self) -> int:
        with self._lock:
            return len(self._data)

    def close(self) -> None:
        self._stop = True
        self._kick()
        self._thread.join(timeout=5)
        for key in list(self._sel.get_map().values()):
            try:
                key.fileobj.close()
            except OSError:
                pass
        self._sel.close()
        self._wake_w.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # ---- internals (the data lock is held) ----
    def _set(self, key: bytes, value: bytes) -> None:
        self._data[key] = value
        self._wake_waiters(key)

    def _add(self, key: bytes, delta: int) -> int:
        v = int(self._data.get(key, b"0")) + delta
        self._set(key, str(v).encode())
        return v

    def _wake_waiters(self, key: bytes) -> None:
        conns = self._waiters.pop(key, None)
        if not conns:
            return
        for c in conns:
            self._answer_waits(c)

    def _answer_waits(self, c: _Conn) -> None:
        # WAITs on one connection are answered in order: a later WAIT never overtakes an earlier one
        while c.waiting and all(k in self._data for k in c.waiting[0]):
            c.waiting.pop(0)
            c.tx += _U8.pack(STOP_WAITING)
            self._dirty.add(c)
        if c.waiting:
            for k in c.waiting[0]:
                if k not in self._data and c not in self._waiters[k]:
                    self._waiters[k].append(c)

    def _kick(self) -> None:
        try:
            self._wake_w.send(b"x")
        except OSError:
            pass

    def _run(self) -> None:
        conns: dict[int, _Conn] = {}
        while not self._stop:
            for key, ev in self._sel.select(timeout=1.0):
                if key.data is None:
                    self._accept(conns)
                elif key.data == "wake":
                    try:
                        while self._wake_r.recv(4096):
                            pass
                    except BlockingIOError:
                        pass
                else:
                    c = key.data
                    if ev & selectors.EVENT_READ:
                        self._read(c, conns)
                    if ev & selectors.EVENT_WRITE and c.sock.fileno() in conns:
                        self._flush(c, conns)  # a slow reader's socket drained: send the rest
            if self._dirty:
                with self._lock:
                    dirty, self._dirty = self._dirty, set()
                for c in dirty:
                    if c.sock.fileno() in conns:
                        self._flush(c, conns)

    def _accept(self, conns: dict) -> None:
        while True:
            try:
                s, _ = self._lsock.accept()
            except (BlockingIOError, InterruptedError):
                return
            s.setblocking(False)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            c = _Conn(s)
            conns[s.fileno()] = c
            self._sel.register(s, selectors.EVENT_READ, c)

    def _drop(self, c: _Conn, conns: dict) -> None:
        with self._lock:
            for k in list(self._waiters):
                lst = self._waiters[k]
                if c in lst:
                    lst.remove(c)
                    if not lst:
                        del self._waiters[k]
        conns.pop(c.sock.fileno(), None)
        try:
            self._sel.unregister(c.sock)
        except (KeyError, ValueError):
            pass
        c.sock.close()

    def _read(self, c: _Conn, conns: dict) -> None:
        try:
            d = c.sock.recv(1 << 16)
        except (BlockingIOError, InterruptedError):
            return
        except OSError:
            d = b""
        if not d:
            self._drop(c, conns)
            return
        c.rx += d
        ok = True
        with self._lock:
            while c.rx:
                r = _Reader(c.rx)
                try:
                    ok = self._handle(c, r)
                except _Incomplete:
                    break
                del c.rx[:r.pos]
                if c.tx:
                    self._dirty.add(c)
                if not ok:
                    c.tx.clear()
                    self._dirty.discard(c)
                    break
        if not ok:
            self.refused += 1
            self._drop(c, conns)

    def _flush(self, c: _Conn, conns: dict) -> None:
        """Send what the connection has queued without ever blocking: the bytes are taken out under the data lock
        (an in-process set() on the supervisor's thread appends WAIT replies to c.tx), sent outside it, and what the
        socket did not take goes back in front and waits for EVENT_WRITE. A peer that stops reading (a process frozen
        after a GPU fault) can therefore never stall this thread, the supervisor's set('otd/dead/r') or any other
        rank's heartbeat; one whose backlog passes TX_CAP is dropped."""
        with self._lock:
            data, c.tx = bytes(c.tx), bytearray()
        ok, n = True, 0
        try:
            n = c.sock.send(data) if data else 0
        except (BlockingIOError, InterruptedError):
            n = 0
        except OSError:
            ok = False
        if ok and n < len(data):
            with self._lock:
                c.tx[:0] = data[n:]
                backlog = len(c.tx)
            ok = backlog <= TX_CAP
        if ok:
            want = selectors.EVENT_READ | (selectors.EVENT_WRITE if c.tx else 0)
            try:
                if self._sel.get_key(c.sock).events != want:
                    self._sel.modify(c.sock, want, c)
            except (KeyError, ValueError):
                pass
        else:
            self._drop(c, conns)

    def _handle(self, c: _Conn, r: _Reader) -> bool:
        """Parse and serve one request (raises _Incomplete before changing any state). False = drop the peer."""
        q = r.take(1)[0]
        if q == VALIDATE:
            if r.u32() != MAGIC:
                return False
            c.validated = True
            return True
        if not c.validated:
            return False
        if q == PING:
            c.tx += _U32.pack(r.u32())
        elif q == SET:
            k, v = r.blob(), r.blob()
            self._set(k, v)
        elif q == COMPARE_SET:
            k, expected, desired = r.blob(), r.blob(), r.blob()
            cur = self._data.get(k)
            if cur is None:
                if expected == b"":
                    self._set(k, desired)
                    c.tx += _vec(desired)
                else:
                    c.tx += _vec(expected)
            else:
                if cur == expected:
                    self._set(k, desired)
                    cur = desired
                c.tx += _vec(cur)
        elif q == GET:
            k = r.blob()
            c.tx += _vec(self._data.get(k, b""))
        elif q == ADD:
            k, delta = r.blob(), r.i64()
            c.tx += _I64.pack(self._add(k, delta))
        elif q == CHECK:
            keys = [r.blob() for _ in range(r.u64())]
            c.tx += _U8.pack(READY if all(k in self._data for k in keys) else NOT_READY)
        elif q == WAIT:
            keys = {r.blob() for _ in range(r.u64())}
            c.waiting.append(keys)
            self._answer_waits(c)
        elif q == CANCEL_WAIT:
            for k in list(self._waiters):
                lst = self._waiters[k]
                if c in lst:
                    lst.remove(c)
                    if not lst:
                        del self._waiters[k]
            c.waiting.clear()
            c.tx += _U8.pack(WAIT_CANCELED)
        elif q == GETNUMKEYS:
            c.tx += _I64.pack(len(self._data))
        elif q == DELETE_KEY:
            k = r.blob()
            c.tx += _I64.pack(1 if self._data.pop(k, None) is not None else 0)
        elif q == APPEND:
            k, v = r.blob(), r.blob()
            self._set(k, self._data.get(k, b"") + v)
        elif q == MULTI_GET:
            keys = [r.blob() for _ in range(r.u64())]
            for k in keys:
                c.tx += _vec(self._data.get(k, b""))
        elif q == MULTI_SET:
            n = r.u64()
            kv = [(r.blob(), r.blob()) for _ in range(n)]
            for k, v in kv:
                self._set(k, v)
        else:  # the QUEUE_* and LIST_KEYS ops are not used by the node; an unknown query desynchronises the stream
            return False
        return True


def _b(x: str | bytes) -> bytes:
    return x.encode() if isinstance(x, str) else bytes(x)


def _k(key: str | bytes) -> bytes:
    return b"/" + _b(key)  # torch's TCPStore client sends every key as "/" + key
