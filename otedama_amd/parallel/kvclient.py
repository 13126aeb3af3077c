"""A torch-free client of torch.distributed's TCPStore protocol (the node's rendezvous store).

The node's rank processes run the native RCCL data plane (parallel/rcclcomm.py) and never import torch, yet they
share one store with the supervisor (parallel/kvstore.py, our server) or with torchrun's agent (torch's C++ server).
This client speaks the same wire protocol as torch's ``TCPStore`` client (parallel/kvstore.py's docstring has the
format) and offers the subset of its API the node uses: ``set``, ``get`` (waits for the key, like torch's),
``add``, ``check``, ``delete_key``, ``wait``, ``clone``, ``set_timeout`` / ``timeout``. Every key goes on the wire
as "/" + key, as torch's client sends it, so both kinds of client see the same keys.

Reference analogue: none (one Go process per host); parity is with torch's TCPStore client, pinned by
tests/test_kvclient.py against both servers.
"""
from __future__ import annotations

import datetime
import socket
import struct
import threading

from otedama_amd.parallel.kvstore import (ADD, CANCEL_WAIT, CHECK, DELETE_KEY, GET, MAGIC, PING, READY, SET,
                                          STOP_WAITING, VALIDATE, WAIT, WAIT_CANCELED)

_U8, _U32, _U64, _I64 = struct.Struct("<B"), struct.Struct("<I"), struct.Struct("<Q"), struct.Struct("<q")


def _b(x) -> bytes:
    return x.encode() if isinstance(x, str) else bytes(x)


def _key(k) -> bytes:
    return b"/" + _b(k)


def _vec(b: bytes) -> bytes:
    return _U64.pack(len(b)) + b


class StoreClient:
    """One TCP connection to a TCPStore-protocol server. Thread-safe (one request at a time); use ``clone()`` for a
    connection per thread, as the node does with torch's client."""

    def __init__(self, host: str, port: int, timeout: float | datetime.timedelta = 300.0,
                 connect_timeout: float | None = None):
        self.host, self.port = host, int(port)
        self._timeout = timeout.total_seconds() if isinstance(timeout, datetime.timedelta) else float(timeout)
        self._lock = threading.Lock()
        self._sock = self._connect(connect_timeout if connect_timeout is not None else self._timeout)

    def _connect(self, within: float) -> socket.socket:
        """Connect, retrying while the server is not up yet (a rank may start before the rendezvous host)."""
        import time

        end = time.monotonic() + within
        while True:
            try:
                s = socket.create_connection((self.host, self.port), timeout=max(0.1, min(5.0, within)))
                break
            except OSError:
                if time.monotonic() >= end:
                    raise
                time.sleep(0.05)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        s.settimeout(self._timeout)
        s.sendall(_U8.pack(VALIDATE) + _U32.pack(MAGIC))
        return s

    # ---------------------------------------------------------------- torch.distributed.Store-like API
    @property
    def timeout(self) -> datetime.timedelta:
        return datetime.timedelta(seconds=self._timeout)

    def set_timeout(self, timeout: float | datetime.timedelta) -> None:
        self._timeout = timeout.total_seconds() if isinstance(timeout, datetime.timedelta) else float(timeout)
        if self._sock is not None:
            self._sock.settimeout(self._timeout)

    def clone(self) -> "StoreClient":
        return StoreClient(self.host, self.port, self._timeout)

    def set(self, key, value) -> None:
        self._rpc(_U8.pack(SET) + _vec(_key(key)) + _vec(_b(value)), lambda: None)

    def get(self, key) -> bytes:
        """The key's value, waiting for it to be set up to the client's timeout (TimeoutError), as torch's get()."""
        self.wait([key])
        return self._rpc(_U8.pack(GET) + _vec(_key(key)), self._read_vec)

    def add(self, key, delta: int) -> int:
        return self._rpc(_U8.pack(ADD) + _vec(_key(key)) + _I64.pack(int(delta)), lambda: _I64.unpack(self._read(8))[0])

    def check(self, keys) -> bool:
        return self._rpc(_U8.pack(CHECK) + _U64.pack(len(keys)) + b"".join(_vec(_key(k)) for k in keys),
                         lambda: self._read(1)[0] == READY)

    def delete_key(self, key) -> bool:
        return self._rpc(_U8.pack(DELETE_KEY) + _vec(_key(key)), lambda: _I64.unpack(self._read(8))[0] == 1)

    def wait(self, keys, timeout: float | datetime.timedelta | None = None) -> None:
        """Block until every key exists (TimeoutError after ``timeout``, default the client's)."""
        t = self._timeout if timeout is None else (
            timeout.total_seconds() if isinstance(timeout, datetime.timedelta) else float(timeout))
        with self._lock:
            sock = self._conn()
            canceled = False  # the wait timed out and was withdrawn: the connection is back in sync
            try:
                sock.sendall(_U8.pack(WAIT) + _U64.pack(len(keys)) + b"".join(_vec(_key(k)) for k in keys))
                sock.settimeout(t)
                try:
                    got = self._read(1)[0]
                except socket.timeout:
                    # withdraw the wait: the server answers WAIT_CANCELED (after a STOP_WAITING that crossed it)
                    sock.settimeout(self._timeout)
                    sock.sendall(_U8.pack(CANCEL_WAIT))
                    while self._read(1)[0] != WAIT_CANCELED:
                        pass
                    canceled = True
                    raise TimeoutError(f"wait timeout after {t:.1f} s, keys: {list(keys)}") from None
                sock.settimeout(self._timeout)
            except BaseException:
                if canceled:
                    sock.settimeout(self._timeout)
                else:
                    self._drop()
                raise
            if got != STOP_WAITING:
                self._drop()
                raise RuntimeError(f"store: unexpected WAIT reply {got}")

    def ping(self) -> bool:
        return self._rpc(_U8.pack(PING) + _U32.pack(0x0D7E), lambda: _U32.unpack(self._read(4))[0] == 0x0D7E)

    def close(self) -> None:
        self._drop()

    # ---------------------------------------------------------------- wire
    def _conn(self) -> socket.socket:
        if self._sock is None:  # the previous request failed part way: a fresh connection, in protocol sync
            self._sock = self._connect(self._timeout)
        return self._sock

    def _drop(self) -> None:
        sock, self._sock = self._sock, None
        if sock is not None:
            try:
                sock.close()
            except OSError:
                pass

    def _rpc(self, payload: bytes, read):
        """One request and its reply. A request that fails part way (a timeout, a reset) may leave a reply in flight
        that the next request would read as its own, so the connection is dropped and the next request reconnects."""
        with self._lock:
            sock = self._conn()
            try:
                sock.sendall(payload)
                return read()
            except BaseException:
                self._drop()
                raise

    def _read(self, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = self._sock.recv(n - len(buf))  # type: ignore[union-attr]
            if not chunk:
                raise ConnectionError("store closed the connection")
            buf += chunk
        return bytes(buf)

    def _read_vec(self) -> bytes:
        return self._read(_U64.unpack(self._read(8))[0])


class PrefixClient:
    """Keys under ``prefix/`` of a StoreClient (torch's PrefixStore)."""

    def __init__(self, prefix: str, store: StoreClient):
        self.prefix, self.store = prefix, store

    def _p(self, k) -> str:
        return f"{self.prefix}/{k if isinstance(k, str) else _b(k).decode()}"

    def set(self, key, value) -> None:
        self.store.set(self._p(key), value)

    def get(self, key) -> bytes:
        return self.store.get(self._p(key))

    def check(self, keys) -> bool:
        return self.store.check([self._p(k) for k in keys])

    def wait(self, keys, timeout=None) -> None:
        self.store.wait([self._p(k) for k in keys], timeout)
