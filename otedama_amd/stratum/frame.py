"""Stratum V2 binary framing.

Parity: internal/stratum/frame.go
  * 6-byte header: u16 extension_type (bit 15 = channel_msg) | u8 msg_type |
    u24 msg_length, little-endian ...................... frame.go:57-86,172-186
  * Header.validate (U24 bound, channel payload >= 4) ... frame.go:108-136
  * Frame.channel_id ................................... frame.go:153-161
  * encode_frame / decode_header ....................... frame.go:194-231
  * Decoder: max frame (16 MiB) checked BEFORE
    allocating the payload (anti-DoS) .................. frame.go:238-302
An asyncio reader (``read_frame_async``) is provided for the client/pool loops.

``FrameScanner`` / ``FrameReader`` are the bulk path used by the pool server and the SV2 client: one socket
read is split into frames by the native scanner (``csrc/cpu/sv2_frame.cpp``) in one call, instead of two
``readexactly`` awaits per frame. The size checks are the same and run before any payload is buffered past
the offending header.
"""
from __future__ import annotations

import asyncio
import collections
import struct
from typing import BinaryIO, NamedTuple

HEADER_SIZE = 6
MAX_MESSAGE_LENGTH = (1 << 24) - 1
DEFAULT_MAX_FRAME_SIZE = 16 * 1024 * 1024
MINIMUM_CHANNEL_PAYLOAD = 4
CHANNEL_MSG_BIT = 0x8000


class FrameError(ValueError):
    pass


class Header(NamedTuple):
    # NamedTuple rather than a frozen dataclass: a pool decodes one of these per share, and tuple construction
    # is ~5x cheaper than a frozen dataclass __init__.
    extension_type: int = 0
    msg_type: int = 0
    msg_length: int = 0

    @property
    def channel_msg(self) -> bool:
        return bool(self.extension_type & CHANNEL_MSG_BIT)

    @property
    def extension_id(self) -> int:
        return self.extension_type & ~CHANNEL_MSG_BIT & 0xFFFF

    def validate(self) -> None:
        if self.msg_length > MAX_MESSAGE_LENGTH:
            raise FrameError(f"stratum: MsgLength {self.msg_length} exceeds U24 maximum {MAX_MESSAGE_LENGTH}")
        if self.channel_msg and self.msg_length < MINIMUM_CHANNEL_PAYLOAD:
            raise FrameError(f"stratum: channel message requires payload >= {MINIMUM_CHANNEL_PAYLOAD} bytes, "
                             f"got {self.msg_length}")

    def encode(self) -> bytes:
        self.validate()
        n = self.msg_length
        return struct.pack("<HB", self.extension_type & 0xFFFF, self.msg_type & 0xFF) + bytes(
            (n & 0xFF, (n >> 8) & 0xFF, (n >> 16) & 0xFF))


class Frame(NamedTuple):
    header: Header
    payload: bytes

    def channel_id(self) -> int:
        if not self.header.channel_msg:
            raise FrameError("stratum: frame is not a channel message")
        if len(self.payload) < MINIMUM_CHANNEL_PAYLOAD:
            raise FrameError(f"stratum: channel message payload is {len(self.payload)} bytes, need at least "
                             f"{MINIMUM_CHANNEL_PAYLOAD}")
        return struct.unpack_from("<I", self.payload, 0)[0]


def decode_header(src: bytes) -> Header:
    if len(src) < HEADER_SIZE:
        raise FrameError(f"stratum: header truncated: need {HEADER_SIZE} bytes, got {len(src)}")
    ext, mt = struct.unpack_from("<HB", src, 0)
    return Header(ext, mt, src[3] | (src[4] << 8) | (src[5] << 16))


def encode_frame(f: Frame) -> bytes:
    if len(f.payload) > MAX_MESSAGE_LENGTH:
        raise FrameError(f"stratum: payload length {len(f.payload)} exceeds U24 maximum {MAX_MESSAGE_LENGTH}")
    h = Header(f.header.extension_type, f.header.msg_type, len(f.payload))
    return h.encode() + bytes(f.payload)


def _check_size(h: Header, max_frame: int) -> None:
    h.validate()
    total = HEADER_SIZE + h.msg_length
    if total > max_frame:
        raise FrameError(f"stratum: frame size {total} exceeds MaxFrameSize {max_frame}")


class Decoder:
    """Blocking frame reader over a file-like object (reads exactly)."""

    def __init__(self, r: BinaryIO, max_frame_size: int = DEFAULT_MAX_FRAME_SIZE):
        self.r = r
        self.max_frame_size = max_frame_size

    def _read_exact(self, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = self.r.read(n - len(buf))
            if not chunk:
                raise EOFError("unexpected EOF" if buf else "EOF")
            buf += chunk
        return bytes(buf)

    def read_frame(self) -> Frame:
        if self.max_frame_size <= 0:
            raise FrameError("stratum: Decoder.MaxFrameSize must be positive")
        h = decode_header(self._read_exact(HEADER_SIZE))
        _check_size(h, self.max_frame_size)
        payload = self._read_exact(h.msg_length) if h.msg_length else b""
        return Frame(h, payload)


async def read_frame_async(reader: asyncio.StreamReader, max_frame_size: int = DEFAULT_MAX_FRAME_SIZE) -> Frame:
    raw = await reader.readexactly(HEADER_SIZE)
    h = decode_header(raw)
    _check_size(h, max_frame_size)
    payload = await reader.readexactly(h.msg_length) if h.msg_length else b""
    return Frame(h, payload)


def iter_frames(buf: bytes, max_frame_size: int = DEFAULT_MAX_FRAME_SIZE):
    """Parse back-to-back frames from a byte string (tests / fuzzing)."""
    off = 0
    while off < len(buf):
        h = decode_header(buf[off:off + HEADER_SIZE])
        _check_size(h, max_frame_size)
        end = off + HEADER_SIZE + h.msg_length
        if end > len(buf):
            raise EOFError("unexpected EOF")
        yield Frame(h, bytes(buf[off + HEADER_SIZE:end]))
        off = end


def _scan_py(buf, max_frame_size: int):
    """Pure-Python twin of the native ``sv2_scan`` (used when the extension is not built)."""
    out, off, n = [], 0, len(buf)
    while n - off >= HEADER_SIZE:
        ext = buf[off] | (buf[off + 1] << 8)
        ln = buf[off + 3] | (buf[off + 4] << 8) | (buf[off + 5] << 16)
        if HEADER_SIZE + ln > max_frame_size:
            return out, off, 1
        if ext & CHANNEL_MSG_BIT and ln < MINIMUM_CHANNEL_PAYLOAD:
            return out, off, 2
        end = off + HEADER_SIZE + ln
        if end > n:
            break
        out.append((ext, buf[off + 2], off + HEADER_SIZE, ln))
        off = end
    return out, off, 0


def _scanner():
    """The native splitter when the extension is already in this process (the pool server loads it at start),
    else the Python one: a miner engine reads a few frames a second and must not load the HIP runtime for them."""
    from otedama_amd.ops.native import loaded

    mod = loaded()
    return mod.sv2_scan if mod is not None and hasattr(mod, "sv2_scan") else _scan_py


class FrameScanner:
    """Incremental frame splitter: ``feed(bytes)`` returns every frame completed by the new bytes.

    A bad header (too large, short channel payload) raises ``FrameError`` once the frames before it have been
    returned, and every later ``feed`` raises it again.
    """

    def __init__(self, max_frame_size: int = DEFAULT_MAX_FRAME_SIZE, native: bool = True):
        if max_frame_size <= 0:
            raise FrameError("stratum: Decoder.MaxFrameSize must be positive")
        self.max_frame_size = max_frame_size
        self._buf = bytearray()
        self._err: FrameError | None = None
        self._scan = _scanner() if native else _scan_py

    @property
    def pending(self) -> int:
        """Bytes held for a frame that is not complete yet."""
        return len(self._buf)

    @property
    def error(self) -> FrameError | None:
        """The bad-header error found after the frames the last ``feed`` returned (raised by the next ``feed``)."""
        return self._err

    def feed(self, data: bytes) -> list[Frame]:
        if self._err is not None:
            raise self._err
        self._buf += data
        recs, consumed, status = self._scan(self._buf, self.max_frame_size)
        buf = self._buf
        frames = [Frame(Header(e, t, ln), bytes(buf[o:o + ln])) for e, t, o, ln in recs]
        del buf[:consumed]
        if status:
            try:
                _check_size(decode_header(bytes(buf[:HEADER_SIZE])), self.max_frame_size)
            except FrameError as exc:
                self._err = exc
            if not frames:
                raise self._err
        return frames


class FrameReader:
    """Asyncio frame reader over anything with ``read(n)`` (a ``StreamReader`` or the Noise ``EncryptedReader``).

    EOF mid-frame raises ``asyncio.IncompleteReadError`` like ``readexactly`` does in ``read_frame_async``.
    """

    def __init__(self, reader, max_frame_size: int = DEFAULT_MAX_FRAME_SIZE, chunk: int = 1 << 16):
        self.reader = reader
        self.chunk = chunk
        self._scanner = FrameScanner(max_frame_size)
        self._ready: collections.deque[Frame] = collections.deque()

    async def read_frame(self) -> Frame:
        while not self._ready:
            if self._scanner.error is not None:
                # a bad header arrived in the same read as the frames already returned: fail now instead of
                # waiting on the socket for data that would only be rejected
                raise self._scanner.error
            data = await self.reader.read(self.chunk)
            if not data:
                raise asyncio.IncompleteReadError(b"", self._scanner.pending or HEADER_SIZE)
            self._ready.extend(self._scanner.feed(data))
        return self._ready.popleft()
