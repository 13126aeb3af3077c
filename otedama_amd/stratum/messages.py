"""Stratum V2 mining-protocol messages: encode / decode / dispatch.

Parity (reference byte layouts):
  * STR0_255 / B0_255 / B0_32 / U16 / U32 LE primitives ..... stratum/wire.go:28-126
    (encode strict, decode lenient: B0_32 is read as B0_255)
  * message ids ............................................. stratum/messages.go:45-58
  * SetupConnection(+Success/Error), OpenMiningChannel(+Success/Error)
                                                              stratum/handshake.go:33-290
  * NewMiningJob (OPTION[u32] min_ntime), SetNewPrevHash, SetTarget,
    SubmitSharesStandard/Success/Error ...................... stratum/messages.go:89-348
  * WrapMessage / DispatchFrame (switch on msg_type only;
    unknown types -> UnknownMessage) ........................ stratum/messages.go:357-485
  * ValidateSetupConnection ................................. stratum/messages.go:492-500

Two dialects: ``REFERENCE`` reproduces the reference encoders byte
for byte (its own test pools agree with them); ``SPEC`` follows the SV2 spec
where the reference deviates (SubmitSharesError = 0x1d, endpoint_port in
SetupConnection, max_target in OpenMiningChannel, group_channel_id in
OpenMiningChannelSuccess, u64 new_shares_sum). Extra messages the pool side
needs (Reconnect, UpdateChannel, CloseChannel, SetExtranoncePrefix) are added.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from typing import ClassVar

from otedama_amd.stratum.frame import CHANNEL_MSG_BIT, Frame, FrameError, Header

MSG_SETUP_CONNECTION = 0x00
MSG_SETUP_CONNECTION_SUCCESS = 0x01
MSG_SETUP_CONNECTION_ERROR = 0x02
MSG_CHANNEL_ENDPOINT_CHANGED = 0x03
MSG_RECONNECT = 0x04
MSG_OPEN_MINING_CHANNEL = 0x10
MSG_OPEN_MINING_CHANNEL_SUCCESS = 0x11
MSG_OPEN_MINING_CHANNEL_ERROR = 0x12
MSG_OPEN_EXTENDED_MINING_CHANNEL = 0x13
MSG_OPEN_EXTENDED_MINING_CHANNEL_SUCCESS = 0x14
MSG_NEW_MINING_JOB = 0x15
MSG_UPDATE_CHANNEL = 0x16
MSG_CLOSE_CHANNEL = 0x18
MSG_SET_EXTRANONCE_PREFIX = 0x19
MSG_SUBMIT_SHARES_STANDARD = 0x1A
MSG_SUBMIT_SHARES_EXTENDED = 0x1B
MSG_SUBMIT_SHARES_SUCCESS = 0x1C
MSG_SUBMIT_SHARES_ERROR = 0x1E          # reference id (spec: 0x1d)
MSG_SUBMIT_SHARES_ERROR_SPEC = 0x1D
MSG_NEW_EXTENDED_MINING_JOB = 0x1F
MSG_SET_NEW_PREV_HASH = 0x20
MSG_SET_TARGET = 0x21

MINING_PROTOCOL = 0

# SetupConnection flags (mining protocol, spec §5.3.2)
FLAG_REQUIRES_STANDARD_JOBS = 1 << 0
FLAG_REQUIRES_WORK_SELECTION = 1 << 1
FLAG_REQUIRES_VERSION_ROLLING = 1 << 2

REFERENCE = "reference"
SPEC = "spec"


class MessageError(FrameError):
    pass


class _R:
    """Bounds-checked little-endian reader."""

    __slots__ = ("b", "pos", "ctx")

    def __init__(self, b: bytes, ctx: str):
        self.b, self.pos, self.ctx = b, 0, ctx

    def take(self, n: int, what: str) -> bytes:
        if self.pos + n > len(self.b):
            raise MessageError(f"stratum: {self.ctx}.{what}: unexpected EOF")
        v = self.b[self.pos:self.pos + n]
        self.pos += n
        return v

    def u8(self, w):
        return self.take(1, w)[0]

    def u16(self, w):
        return struct.unpack("<H", self.take(2, w))[0]

    def u32(self, w):
        return struct.unpack("<I", self.take(4, w))[0]

    def u64(self, w):
        return struct.unpack("<Q", self.take(8, w))[0]

    def f32(self, w):
        return struct.unpack("<f", self.take(4, w))[0]

    def str0_255(self, w):
        n = self.u8(w)
        return self.take(n, w).decode("utf-8", "replace") if n else ""

    def b0_255(self, w):
        n = self.u8(w)
        return bytes(self.take(n, w)) if n else b""

    def rest(self) -> bytes:
        return self.b[self.pos:]


def str0_255(s: str) -> bytes:
    b = s.encode()
    if len(b) > 255:
        raise MessageError(f"stratum: string too long ({len(b)} > 255 bytes)")
    return bytes([len(b)]) + b


def b0_255(v: bytes) -> bytes:
    if len(v) > 255:
        raise MessageError(f"stratum: byte slice too long ({len(v)} > 255)")
    return bytes([len(v)]) + v


def b0_32(v: bytes) -> bytes:
    if len(v) > 32:
        raise MessageError(f"stratum: byte slice too long for B0_32 ({len(v)} > 32)")
    return bytes([len(v)]) + v


def b0_64k(v: bytes) -> bytes:
    if len(v) > 0xFFFF:
        raise MessageError(f"stratum: byte slice too long for B0_64K ({len(v)} > 65535)")
    return struct.pack("<H", len(v)) + v


def _b0_64k(r: "_R", what: str) -> bytes:
    n = r.u16(what)
    return bytes(r.take(n, what)) if n else b""


def _u256(v: bytes, what: str) -> bytes:
    if len(v) != 32:
        raise MessageError(f"stratum: {what} must be 32 bytes")
    return bytes(v)


@dataclass
class Message:
    MSG_TYPE: ClassVar[int] = -1
    CHANNEL_MSG: ClassVar[bool] = False

    def encode(self, dialect: str = REFERENCE) -> bytes:
        raise NotImplementedError

    @classmethod
    def decode(cls, payload: bytes, dialect: str = REFERENCE):
        raise NotImplementedError

    def msg_type(self, dialect: str = REFERENCE) -> int:
        return self.MSG_TYPE


@dataclass
class SetupConnection(Message):
    MSG_TYPE: ClassVar[int] = MSG_SETUP_CONNECTION
    protocol: int = MINING_PROTOCOL
    min_version: int = 2
    max_version: int = 2
    flags: int = 0
    endpoint: str = ""
    vendor: str = ""
    hardware_version: str = ""
    firmware: str = ""
    device_id: str = ""
    endpoint_port: int = 0  # SPEC dialect only

    def encode(self, dialect=REFERENCE):
        b = struct.pack("<BHHI", self.protocol, self.min_version, self.max_version, self.flags & 0xFFFFFFFF)
        b += str0_255(self.endpoint)
        if dialect == SPEC:
            b += struct.pack("<H", self.endpoint_port)
        for s in (self.vendor, self.hardware_version, self.firmware, self.device_id):
            b += str0_255(s)
        return b

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        r = _R(payload, "SetupConnection")
        m = cls(r.u8("Protocol"), r.u16("MinVersion"), r.u16("MaxVersion"), r.u32("Flags"), r.str0_255("Endpoint"))
        if dialect == SPEC:
            m.endpoint_port = r.u16("EndpointPort")
        m.vendor = r.str0_255("Vendor")
        m.hardware_version = r.str0_255("HardwareVersion")
        m.firmware = r.str0_255("Firmware")
        m.device_id = r.str0_255("DeviceID")
        return m


@dataclass
class SetupConnectionSuccess(Message):
    MSG_TYPE: ClassVar[int] = MSG_SETUP_CONNECTION_SUCCESS
    used_version: int = 2
    flags: int = 0

    def encode(self, dialect=REFERENCE):
        return struct.pack("<HI", self.used_version, self.flags & 0xFFFFFFFF)

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        if len(payload) < 6:
            raise MessageError(f"stratum: SetupConnectionSuccess: short payload ({len(payload)} < 6)")
        return cls(*struct.unpack_from("<HI", payload, 0))


@dataclass
class SetupConnectionError(Message):
    MSG_TYPE: ClassVar[int] = MSG_SETUP_CONNECTION_ERROR
    flags: int = 0
    error: str = ""

    def encode(self, dialect=REFERENCE):
        return struct.pack("<I", self.flags & 0xFFFFFFFF) + str0_255(self.error)

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        r = _R(payload, "SetupConnectionError")
        return cls(r.u32("Flags"), r.str0_255("Error"))


@dataclass
class Reconnect(Message):
    MSG_TYPE: ClassVar[int] = MSG_RECONNECT
    new_host: str = ""
    new_port: int = 0

    def encode(self, dialect=REFERENCE):
        return str0_255(self.new_host) + struct.pack("<H", self.new_port)

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        r = _R(payload, "Reconnect")
        return cls(r.str0_255("NewHost"), r.u16("NewPort"))


@dataclass
class OpenMiningChannel(Message):
    MSG_TYPE: ClassVar[int] = MSG_OPEN_MINING_CHANNEL
    req_id: int = 0
    user: str = ""
    nominal_hashrate: float = 0.0
    max_target: bytes = field(default=b"\xff" * 32)  # SPEC dialect only

    def encode(self, dialect=REFERENCE):
        b = struct.pack("<I", self.req_id) + str0_255(self.user) + struct.pack("<f", self.nominal_hashrate)
        if dialect == SPEC:
            b += _u256(self.max_target, "max_target")
        return b

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        r = _R(payload, "OpenMiningChannel")
        m = cls(r.u32("ReqID"), r.str0_255("User"), r.f32("NominalHashrate"))
        if dialect == SPEC:
            m.max_target = bytes(r.take(32, "MaxTarget"))
        return m


@dataclass
class OpenMiningChannelSuccess(Message):
    MSG_TYPE: ClassVar[int] = MSG_OPEN_MINING_CHANNEL_SUCCESS
    req_id: int = 0
    channel_id: int = 0
    target: bytes = field(default=b"\xff" * 32)
    extranonce: bytes = b""
    extranonce2_size: int = 0     # REFERENCE dialect
    group_channel_id: int = 0     # SPEC dialect

    def encode(self, dialect=REFERENCE):
        b = struct.pack("<II", self.req_id, self.channel_id) + _u256(self.target, "target") + b0_32(self.extranonce)
        if dialect == SPEC:
            return b + struct.pack("<I", self.group_channel_id)
        return b + struct.pack("<H", self.extranonce2_size)

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        r = _R(payload, "OpenMiningChannelSuccess")
        m = cls(r.u32("ReqID"), r.u32("ChannelID"), bytes(r.take(32, "Target")), r.b0_255("Extranonce"))
        if dialect == SPEC:
            m.group_channel_id = r.u32("GroupChannelID")
        else:
            m.extranonce2_size = r.u16("ExtraNonce2Size")
        return m


@dataclass
class OpenMiningChannelError(Message):
    MSG_TYPE: ClassVar[int] = MSG_OPEN_MINING_CHANNEL_ERROR
    req_id: int = 0
    error: str = ""

    def encode(self, dialect=REFERENCE):
        return struct.pack("<I", self.req_id) + str0_255(self.error)

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        if len(payload) < 4:
            raise MessageError(f"stratum: OpenMiningChannelError: short payload ({len(payload)} < 4)")
        m = cls(struct.unpack_from("<I", payload)[0])
        if len(payload) > 4:
            m.error = _R(payload[4:], "OpenMiningChannelError").str0_255("Error")
        return m


@dataclass
class OpenExtendedMiningChannel(Message):
    MSG_TYPE: ClassVar[int] = MSG_OPEN_EXTENDED_MINING_CHANNEL
    req_id: int = 0
    user: str = ""
    nominal_hashrate: float = 0.0
    max_target: bytes = field(default=b"\xff" * 32)
    min_extranonce_size: int = 0

    def encode(self, dialect=REFERENCE):
        return (struct.pack("<I", self.req_id) + str0_255(self.user) + struct.pack("<f", self.nominal_hashrate)
                + _u256(self.max_target, "max_target") + struct.pack("<H", self.min_extranonce_size))

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        r = _R(payload, "OpenExtendedMiningChannel")
        return cls(r.u32("ReqID"), r.str0_255("User"), r.f32("NominalHashrate"), bytes(r.take(32, "MaxTarget")),
                   r.u16("MinExtranonceSize"))


@dataclass
class OpenExtendedMiningChannelSuccess(Message):
    MSG_TYPE: ClassVar[int] = MSG_OPEN_EXTENDED_MINING_CHANNEL_SUCCESS
    req_id: int = 0
    channel_id: int = 0
    target: bytes = field(default=b"\xff" * 32)
    extranonce_size: int = 0          # bytes the miner rolls after the prefix
    extranonce_prefix: bytes = b""

    def encode(self, dialect=REFERENCE):
        return (struct.pack("<II", self.req_id, self.channel_id) + _u256(self.target, "target")
                + struct.pack("<H", self.extranonce_size) + b0_32(self.extranonce_prefix))

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        r = _R(payload, "OpenExtendedMiningChannelSuccess")
        return cls(r.u32("ReqID"), r.u32("ChannelID"), bytes(r.take(32, "Target")), r.u16("ExtranonceSize"),
                   r.b0_255("ExtranoncePrefix"))


@dataclass
class NewExtendedMiningJob(Message):
    MSG_TYPE: ClassVar[int] = MSG_NEW_EXTENDED_MINING_JOB
    CHANNEL_MSG: ClassVar[bool] = True
    channel_id: int = 0
    job_id: int = 0
    has_min_ntime: bool = False
    min_ntime: int = 0
    version: int = 0
    version_rolling_allowed: bool = True
    merkle_path: list = field(default_factory=list)   # U256 branch hashes, leaf (coinbase) side first
    coinbase_prefix: bytes = b""
    coinbase_suffix: bytes = b""

    def encode(self, dialect=REFERENCE):
        if len(self.merkle_path) > 255:
            raise MessageError("stratum: NewExtendedMiningJob: merkle path longer than 255")
        b = struct.pack("<II", self.channel_id, self.job_id)
        b += (b"\x01" + struct.pack("<I", self.min_ntime)) if self.has_min_ntime else b"\x00"
        b += struct.pack("<IB", self.version & 0xFFFFFFFF, 1 if self.version_rolling_allowed else 0)
        b += bytes([len(self.merkle_path)]) + b"".join(_u256(h, "merkle_path") for h in self.merkle_path)
        return b + b0_64k(self.coinbase_prefix) + b0_64k(self.coinbase_suffix)

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        r = _R(payload, "NewExtendedMiningJob")
        m = cls(r.u32("ChannelID"), r.u32("JobID"))
        opt = r.u8("MinNTime")
        if opt == 1:
            m.has_min_ntime, m.min_ntime = True, r.u32("MinNTime")
        elif opt != 0:
            raise MessageError(f"stratum: NewExtendedMiningJob: invalid OPTION count {opt} for min_ntime")
        m.version = r.u32("Version")
        m.version_rolling_allowed = r.u8("VersionRollingAllowed") != 0
        m.merkle_path = [bytes(r.take(32, "MerklePath")) for _ in range(r.u8("MerklePath"))]
        m.coinbase_prefix = _b0_64k(r, "CoinbaseTxPrefix")
        m.coinbase_suffix = _b0_64k(r, "CoinbaseTxSuffix")
        return m


@dataclass
class NewMiningJob(Message):
    MSG_TYPE: ClassVar[int] = MSG_NEW_MINING_JOB
    CHANNEL_MSG: ClassVar[bool] = True
    channel_id: int = 0
    job_id: int = 0
    has_min_ntime: bool = False
    min_ntime: int = 0
    version: int = 0
    merkle_root: bytes = field(default=bytes(32))

    def encode(self, dialect=REFERENCE):
        b = struct.pack("<II", self.channel_id, self.job_id)
        b += (b"\x01" + struct.pack("<I", self.min_ntime)) if self.has_min_ntime else b"\x00"
        return b + struct.pack("<I", self.version & 0xFFFFFFFF) + _u256(self.merkle_root, "merkle_root")

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        need = 4 + 4 + 1 + 4 + 32
        if len(payload) < need:
            raise MessageError(f"stratum: NewMiningJob: short payload ({len(payload)} < {need})")
        ch, jid = struct.unpack_from("<II", payload, 0)
        off = 8
        opt = payload[off]
        m = cls(ch, jid)
        if opt == 0:
            off += 1
        elif opt == 1:
            off += 1
            if len(payload) < off + 4 + 4 + 32:
                raise MessageError(f"stratum: NewMiningJob: short payload for present min_ntime ({len(payload)})")
            m.has_min_ntime = True
            m.min_ntime = struct.unpack_from("<I", payload, off)[0]
            off += 4
        else:
            raise MessageError(f"stratum: NewMiningJob: invalid OPTION count {opt} for min_ntime")
        m.version = struct.unpack_from("<I", payload, off)[0]
        m.merkle_root = bytes(payload[off + 4:off + 36])
        return m


@dataclass
class UpdateChannel(Message):
    MSG_TYPE: ClassVar[int] = MSG_UPDATE_CHANNEL
    CHANNEL_MSG: ClassVar[bool] = True
    channel_id: int = 0
    nominal_hashrate: float = 0.0
    maximum_target: bytes = field(default=b"\xff" * 32)

    def encode(self, dialect=REFERENCE):
        return struct.pack("<If", self.channel_id, self.nominal_hashrate) + _u256(self.maximum_target, "max_target")

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        r = _R(payload, "UpdateChannel")
        return cls(r.u32("ChannelID"), r.f32("NominalHashrate"), bytes(r.take(32, "MaximumTarget")))


@dataclass
class CloseChannel(Message):
    MSG_TYPE: ClassVar[int] = MSG_CLOSE_CHANNEL
    CHANNEL_MSG: ClassVar[bool] = True
    channel_id: int = 0
    reason: str = ""

    def encode(self, dialect=REFERENCE):
        return struct.pack("<I", self.channel_id) + str0_255(self.reason)

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        r = _R(payload, "CloseChannel")
        return cls(r.u32("ChannelID"), r.str0_255("Reason"))


@dataclass
class SetExtranoncePrefix(Message):
    MSG_TYPE: ClassVar[int] = MSG_SET_EXTRANONCE_PREFIX
    CHANNEL_MSG: ClassVar[bool] = True
    channel_id: int = 0
    extranonce_prefix: bytes = b""

    def encode(self, dialect=REFERENCE):
        return struct.pack("<I", self.channel_id) + b0_32(self.extranonce_prefix)

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        r = _R(payload, "SetExtranoncePrefix")
        return cls(r.u32("ChannelID"), r.b0_255("ExtranoncePrefix"))


@dataclass
class SetNewPrevHash(Message):
    MSG_TYPE: ClassVar[int] = MSG_SET_NEW_PREV_HASH
    CHANNEL_MSG: ClassVar[bool] = True
    channel_id: int = 0
    job_id: int = 0
    prev_hash: bytes = field(default=bytes(32))
    min_ntime: int = 0
    nbits: int = 0

    def encode(self, dialect=REFERENCE):
        return (struct.pack("<II", self.channel_id, self.job_id) + _u256(self.prev_hash, "prev_hash")
                + struct.pack("<II", self.min_ntime, self.nbits))

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        if len(payload) < 48:
            raise MessageError(f"stratum: SetNewPrevHash: short payload ({len(payload)} < 48)")
        ch, jid = struct.unpack_from("<II", payload, 0)
        mt, nb = struct.unpack_from("<II", payload, 40)
        return cls(ch, jid, bytes(payload[8:40]), mt, nb)


@dataclass
class SetTarget(Message):
    MSG_TYPE: ClassVar[int] = MSG_SET_TARGET
    CHANNEL_MSG: ClassVar[bool] = True
    channel_id: int = 0
    max_target: bytes = field(default=b"\xff" * 32)

    def encode(self, dialect=REFERENCE):
        return struct.pack("<I", self.channel_id) + _u256(self.max_target, "max_target")

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        if len(payload) < 36:
            raise MessageError(f"stratum: SetTarget: short payload ({len(payload)} < 36)")
        return cls(struct.unpack_from("<I", payload)[0], bytes(payload[4:36]))


@dataclass
class SubmitSharesStandard(Message):
    MSG_TYPE: ClassVar[int] = MSG_SUBMIT_SHARES_STANDARD
    CHANNEL_MSG: ClassVar[bool] = True
    channel_id: int = 0
    sequence_number: int = 0
    job_id: int = 0
    nonce: int = 0
    ntime: int = 0
    nversion: int = 0

    def encode(self, dialect=REFERENCE):
        return struct.pack("<6I", self.channel_id, self.sequence_number, self.job_id, self.nonce & 0xFFFFFFFF,
                           self.ntime & 0xFFFFFFFF, self.nversion & 0xFFFFFFFF)

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        if len(payload) < 24:
            raise MessageError(f"stratum: SubmitSharesStandard: short payload ({len(payload)} < 24)")
        return cls(*struct.unpack_from("<6I", payload, 0))


@dataclass
class SubmitSharesExtended(Message):
    MSG_TYPE: ClassVar[int] = MSG_SUBMIT_SHARES_EXTENDED
    CHANNEL_MSG: ClassVar[bool] = True
    channel_id: int = 0
    sequence_number: int = 0
    job_id: int = 0
    nonce: int = 0
    ntime: int = 0
    nversion: int = 0
    extranonce: bytes = b""

    def encode(self, dialect=REFERENCE):
        return struct.pack("<6I", self.channel_id, self.sequence_number, self.job_id, self.nonce & 0xFFFFFFFF,
                           self.ntime & 0xFFFFFFFF, self.nversion & 0xFFFFFFFF) + b0_32(self.extranonce)

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        r = _R(payload, "SubmitSharesExtended")
        vals = [r.u32(w) for w in ("ChannelID", "SequenceNumber", "JobID", "Nonce", "NTime", "Version")]
        return cls(*vals, r.b0_255("Extranonce"))


@dataclass
class SubmitSharesSuccess(Message):
    MSG_TYPE: ClassVar[int] = MSG_SUBMIT_SHARES_SUCCESS
    CHANNEL_MSG: ClassVar[bool] = True
    channel_id: int = 0
    last_sequence_number: int = 0
    new_submits_accepted: int = 0
    new_shares_summed: int = 0

    def encode(self, dialect=REFERENCE):
        b = struct.pack("<III", self.channel_id, self.last_sequence_number, self.new_submits_accepted)
        if dialect == SPEC:
            return b + struct.pack("<Q", self.new_shares_summed)
        return b + struct.pack("<I", self.new_shares_summed & 0xFFFFFFFF)

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        need = 20 if dialect == SPEC else 16
        if len(payload) < need:
            raise MessageError(f"stratum: SubmitSharesSuccess: short payload ({len(payload)} < {need})")
        a, b, c = struct.unpack_from("<III", payload, 0)
        d = struct.unpack_from("<Q" if dialect == SPEC else "<I", payload, 12)[0]
        return cls(a, b, c, d)


@dataclass
class SubmitSharesError(Message):
    MSG_TYPE: ClassVar[int] = MSG_SUBMIT_SHARES_ERROR
    CHANNEL_MSG: ClassVar[bool] = True
    channel_id: int = 0
    sequence_number: int = 0
    error: str = ""

    def msg_type(self, dialect=REFERENCE):
        return MSG_SUBMIT_SHARES_ERROR_SPEC if dialect == SPEC else MSG_SUBMIT_SHARES_ERROR

    def encode(self, dialect=REFERENCE):
        return struct.pack("<II", self.channel_id, self.sequence_number) + str0_255(self.error)

    @classmethod
    def decode(cls, payload, dialect=REFERENCE):
        if len(payload) < 8:
            raise MessageError(f"stratum: SubmitSharesError: short payload ({len(payload)} < 8)")
        m = cls(*struct.unpack_from("<II", payload, 0))
        if len(payload) > 8:
            m.error = _R(payload[8:], "SubmitSharesError").str0_255("Error")
        return m


@dataclass
class UnknownMessage(Message):
    msg_type_value: int = 0
    payload: bytes = b""

    def msg_type(self, dialect=REFERENCE):
        return self.msg_type_value

    def encode(self, dialect=REFERENCE):
        return self.payload


_BY_TYPE = {cls.MSG_TYPE: cls for cls in (
    SetupConnection, SetupConnectionSuccess, SetupConnectionError, Reconnect, OpenMiningChannel,
    OpenMiningChannelSuccess, OpenMiningChannelError, NewMiningJob, UpdateChannel, CloseChannel,
    SetExtranoncePrefix, SetNewPrevHash, SetTarget, SubmitSharesStandard, SubmitSharesSuccess, SubmitSharesError,
    OpenExtendedMiningChannel, OpenExtendedMiningChannelSuccess, NewExtendedMiningJob, SubmitSharesExtended)}


def wrap_message(msg: Message, dialect: str = REFERENCE) -> Frame:
    payload = msg.encode(dialect)
    h = Header(CHANNEL_MSG_BIT if msg.CHANNEL_MSG else 0, msg.msg_type(dialect), len(payload))
    h.validate()
    return Frame(h, payload)


def encode_message(msg: Message, dialect: str = REFERENCE) -> bytes:
    f = wrap_message(msg, dialect)
    return f.header.encode() + f.payload


def dispatch_frame(f: Frame, dialect: str = REFERENCE) -> Message:
    mt = f.header.msg_type
    if dialect == SPEC:
        if mt == MSG_SUBMIT_SHARES_ERROR_SPEC:
            return SubmitSharesError.decode(f.payload, dialect)
        if mt == MSG_SUBMIT_SHARES_ERROR:
            return UnknownMessage(mt, f.payload)
    cls = _BY_TYPE.get(mt)
    if cls is None:
        return UnknownMessage(mt, bytes(f.payload))
    return cls.decode(bytes(f.payload), dialect)


def validate_setup_connection(m: SetupConnection) -> None:
    if m.protocol != MINING_PROTOCOL:
        raise MessageError(f"stratum: unsupported protocol {m.protocol} (only MiningProtocol=0 supported)")
    if m.min_version > m.max_version:
        raise MessageError(f"stratum: MinVersion {m.min_version} > MaxVersion {m.max_version}")
