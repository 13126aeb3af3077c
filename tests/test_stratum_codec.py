"""SV2 frame codec, wire primitives and messages: golden bytes, round trips in both dialects, truncation at
every byte, bounds (U24, 16 MiB, channel payload >= 4), dispatch of unknown / dialect-specific types.

Mirrors internal/stratum/{frame,wire,messages,handshake}_test.go (TestEncodeHeader_*, TestDecodeHeader_*,
TestDecoder_*, TestFrame_ChannelID_*, TestAppendStr0_255_*, TestB0_32_*, Test<Message>_RoundTrip,
Test<Message>_Decode_Truncated, TestDispatchFrame_*, TestValidateSetupConnection_*) and the golden frames of
SURVEY Appendix A.2.
"""
from __future__ import annotations

import asyncio
import io
import struct

import pytest

from otedama_amd.stratum import frame as F
from otedama_amd.stratum import messages as M

U256 = bytes(range(32))


def _all_messages():
    return [
        M.SetupConnection(0, 2, 2, 0x6, "pool.example:3336", "Otedama", "v3.0.0", "main", "gfx950", endpoint_port=3336),
        M.SetupConnectionSuccess(2, 0x4),
        M.SetupConnectionError(1, "unsupported-protocol"),
        M.Reconnect("pool2.example", 3337),
        M.OpenMiningChannel(7, "bc1q.rig", 1.5e12, max_target=b"\x7f" * 32),
        M.OpenMiningChannelSuccess(7, 3, U256, b"\x01\x02\x03\x04", extranonce2_size=8, group_channel_id=9),
        M.OpenMiningChannelError(7, "unknown-user"),
        M.OpenExtendedMiningChannel(8, "bc1q.rig", 2.0e12, b"\x3f" * 32, 4),
        M.OpenExtendedMiningChannelSuccess(8, 4, U256, 6, b"\xaa\xbb"),
        M.NewMiningJob(3, 100, True, 1_700_000_000, 0x20000000, U256),
        M.NewMiningJob(3, 101, False, 0, 0x20000004, U256[::-1]),
        M.NewExtendedMiningJob(4, 5, True, 1_700_000_001, 0x20000000, True, [U256, bytes(32)], b"\x01" * 40,
                               b"\x02" * 60),
        M.UpdateChannel(3, 3.0e12, b"\x0f" * 32),
        M.CloseChannel(3, "bye"),
        M.SetExtranoncePrefix(4, b"\x09" * 8),
        M.SetNewPrevHash(3, 100, U256, 1_700_000_000, 0x1703A30C),
        M.SetTarget(3, b"\x00" * 28 + b"\xff" * 4),
        M.SubmitSharesStandard(3, 11, 100, 0xDEADBEEF, 0x60000000, 0x20000004),
        M.SubmitSharesExtended(4, 12, 5, 0xCAFEBABE, 0x60000001, 0x20002000, b"\x01\x02\x03\x04\x05\x06"),
        M.SubmitSharesSuccess(3, 11, 5, 5000),
        M.SubmitSharesError(3, 12, "stale-share"),
    ]


# ------------------------------------------------------------------ golden frames
def test_golden_submit_shares_standard():
    got = M.encode_message(M.SubmitSharesStandard(1, 1, 1, 0xDEADBEEF, 0x60000000, 0x20000004))
    assert got.hex() == "00801a180000010000000100000001000000efbeadde0000006004000020"


def test_golden_setup_connection():
    m = M.SetupConnection(0, 2, 2, 0, "pool.example:3336", "Otedama", "v3.0.0", "main", "cpu")
    assert M.encode_message(m).hex() == ("00000033000000020002000000000011706f6f6c2e6578616d706c653a33333336074f74"
                                         "6564616d610676332e302e30046d61696e03637075")


def test_golden_open_mining_channel():
    m = M.OpenMiningChannel(1, "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq", 0.0)
    assert M.encode_message(m).hex() == ("000010330000010000002a62633171617230737272723778666b7679356c3634336c79646e7739"
                                         "7265353967747a7a7766356d647100000000")


def test_golden_new_mining_job_future():
    m = M.NewMiningJob(1, 100, False, 0, 0x20000000, U256)
    raw = M.encode_message(m)
    assert raw[:6].hex() == "0080152d0000" and len(raw) == 6 + 45
    assert raw[6:].hex().startswith("01000000640000000000000020") and raw[-32:] == U256


def test_golden_new_mining_job_with_min_ntime_is_49_bytes():
    assert len(M.NewMiningJob(1, 1, True, 5, 0, U256).encode()) == 49


@pytest.mark.parametrize("m,size", [(M.SetNewPrevHash(1, 2, U256, 3, 4), 48), (M.SetTarget(1, U256), 36),
                                    (M.SubmitSharesSuccess(1, 2, 3, 4), 16), (M.SetupConnectionSuccess(2, 0), 6)])
def test_fixed_message_sizes(m, size):
    assert len(m.encode()) == size


def test_spec_dialect_sizes_differ_where_the_reference_deviates():
    assert len(M.SubmitSharesSuccess(1, 2, 3, 4).encode(M.SPEC)) == 20
    assert M.SubmitSharesError(1, 2, "x").msg_type(M.SPEC) == 0x1D
    assert M.SubmitSharesError(1, 2, "x").msg_type(M.REFERENCE) == 0x1E
    sc = M.SetupConnection(endpoint="h", endpoint_port=1)
    assert len(sc.encode(M.SPEC)) == len(sc.encode(M.REFERENCE)) + 2
    omc = M.OpenMiningChannel(1, "u", 0.0)
    assert len(omc.encode(M.SPEC)) == len(omc.encode(M.REFERENCE)) + 32


# ------------------------------------------------------------------ round trips
@pytest.mark.parametrize("dialect", [M.REFERENCE, M.SPEC])
@pytest.mark.parametrize("m", _all_messages(), ids=lambda m: type(m).__name__)
def test_every_message_round_trips_through_a_frame(m, dialect):
    raw = M.encode_message(m, dialect)
    (f,) = list(F.iter_frames(raw))
    assert f.header.msg_type == m.msg_type(dialect)
    assert f.header.channel_msg is m.CHANNEL_MSG
    got = M.dispatch_frame(f, dialect)
    if dialect == M.REFERENCE:
        if isinstance(m, M.SetupConnection):
            m = M.SetupConnection(**{**m.__dict__, "endpoint_port": 0})
        if isinstance(m, M.OpenMiningChannel):
            m = M.OpenMiningChannel(m.req_id, m.user, m.nominal_hashrate)
        if isinstance(m, M.OpenMiningChannelSuccess):
            m = M.OpenMiningChannelSuccess(m.req_id, m.channel_id, m.target, m.extranonce, m.extranonce2_size)
    elif isinstance(m, M.OpenMiningChannelSuccess):
        m = M.OpenMiningChannelSuccess(m.req_id, m.channel_id, m.target, m.extranonce, 0, m.group_channel_id)
    if hasattr(m, "nominal_hashrate"):
        assert got.nominal_hashrate == pytest.approx(m.nominal_hashrate, rel=1e-6)
        got.nominal_hashrate = m.nominal_hashrate
    assert got == m


@pytest.mark.parametrize("m", [x for x in _all_messages() if x.CHANNEL_MSG], ids=lambda m: type(m).__name__)
def test_channel_messages_expose_the_channel_id(m):
    f = M.wrap_message(m)
    assert f.channel_id() == m.channel_id


# ------------------------------------------------------------------ truncation at every byte
@pytest.mark.parametrize("dialect", [M.REFERENCE, M.SPEC])
@pytest.mark.parametrize("m", _all_messages(), ids=lambda m: type(m).__name__)
def test_truncated_payloads_raise_message_error_only(m, dialect):
    payload = m.encode(dialect)
    cls = type(m)
    lenient_tail = isinstance(m, (M.SetupConnectionError, M.OpenMiningChannelError, M.SubmitSharesError,
                                  M.CloseChannel))
    for n in range(len(payload)):
        try:
            cls.decode(payload[:n], dialect)
        except M.MessageError:
            continue
        # only a trailing optional/variable string may be cut at its length prefix
        assert lenient_tail or n == len(payload), (cls.__name__, n)


@pytest.mark.parametrize("cls", [M.NewMiningJob, M.NewExtendedMiningJob])
def test_invalid_option_count_is_rejected(cls):
    m = cls(1, 2, True, 3, 4) if cls is M.NewMiningJob else cls(1, 2, True, 3, 4, True, [], b"", b"")
    raw = bytearray(m.encode())
    raw[8] = 2
    with pytest.raises(M.MessageError, match="OPTION"):
        cls.decode(bytes(raw))


# ------------------------------------------------------------------ wire primitives
@pytest.mark.parametrize("s", ["", "a", "x" * 255, "日本"])
def test_str0_255_round_trip(s):
    b = M.str0_255(s)
    assert b[0] == len(s.encode()) and M._R(b, "t").str0_255("s") == s


def test_str0_255_too_long():
    with pytest.raises(M.MessageError, match="too long"):
        M.str0_255("x" * 256)
    with pytest.raises(M.MessageError):
        M.str0_255("é" * 128)  # 256 bytes in UTF-8


def test_b0_32_encode_strict_decode_lenient():
    assert M.b0_32(b"\x01" * 32)[0] == 32
    with pytest.raises(M.MessageError, match="B0_32"):
        M.b0_32(b"\x01" * 33)
    # a 40-byte extranonce in an incoming OpenMiningChannelSuccess is still read (read as B0_255)
    payload = struct.pack("<II", 1, 2) + U256 + bytes([40]) + b"\x05" * 40 + struct.pack("<H", 4)
    got = M.OpenMiningChannelSuccess.decode(payload)
    assert got.extranonce == b"\x05" * 40 and got.extranonce2_size == 4


def test_b0_255_and_b0_64k_bounds():
    assert M.b0_255(b"\x00" * 255)[0] == 255
    with pytest.raises(M.MessageError):
        M.b0_255(b"\x00" * 256)
    assert M.b0_64k(b"\x00" * 0xFFFF)[:2] == b"\xff\xff"
    with pytest.raises(M.MessageError):
        M.b0_64k(b"\x00" * 0x10000)


@pytest.mark.parametrize("cls,field", [(M.SetTarget, "max_target"), (M.SetNewPrevHash, "prev_hash"),
                                       (M.NewMiningJob, "merkle_root")])
def test_u256_fields_must_be_32_bytes(cls, field):
    m = cls()
    setattr(m, field, b"\x00" * 31)
    with pytest.raises(M.MessageError, match="32 bytes"):
        m.encode()


def test_merkle_path_longer_than_255_is_rejected():
    with pytest.raises(M.MessageError, match="255"):
        M.NewExtendedMiningJob(merkle_path=[U256] * 256).encode()


def test_integers_are_masked_to_u32():
    m = M.SubmitSharesStandard(1, 2, 3, nonce=(1 << 32) + 5, ntime=-1 & 0xFFFFFFFF, nversion=(1 << 33) | 7)
    got = M.SubmitSharesStandard.decode(m.encode())
    assert (got.nonce, got.ntime, got.nversion) == (5, 0xFFFFFFFF, 7)


# ------------------------------------------------------------------ header / frame
@pytest.mark.parametrize("ext,mt,ln", [(0, 0, 0), (0x8000, 0x1A, 24), (0x0001, 0xFF, 0xFFFFFF), (0x8003, 0x20, 48)])
def test_header_encode_decode(ext, mt, ln):
    h = F.Header(ext, mt, ln)
    raw = h.encode()
    assert len(raw) == F.HEADER_SIZE and F.decode_header(raw) == h
    assert h.channel_msg is bool(ext & 0x8000) and h.extension_id == ext & 0x7FFF


def test_header_u24_bound_and_channel_minimum():
    with pytest.raises(F.FrameError, match="U24"):
        F.Header(0, 1, 1 << 24).encode()
    with pytest.raises(F.FrameError, match="payload >= 4"):
        F.Header(F.CHANNEL_MSG_BIT, 0x21, 3).encode()
    F.Header(0, 0x21, 3).encode()  # non-channel short payloads are fine


@pytest.mark.parametrize("n", range(6))
def test_decode_header_truncated(n):
    with pytest.raises(F.FrameError, match="truncated"):
        F.decode_header(b"\x00" * n)


def test_frame_channel_id_errors():
    with pytest.raises(F.FrameError, match="not a channel message"):
        F.Frame(F.Header(0, 1, 4), b"\x01\x00\x00\x00").channel_id()
    with pytest.raises(F.FrameError, match="at least"):
        F.Frame(F.Header(F.CHANNEL_MSG_BIT, 1, 2), b"\x01\x00").channel_id()
    assert F.Frame(F.Header(F.CHANNEL_MSG_BIT, 1, 4), b"\x07\x00\x00\x00").channel_id() == 7


def test_encode_frame_recomputes_length():
    raw = F.encode_frame(F.Frame(F.Header(0, 0x10, 999), b"abc"))
    assert F.decode_header(raw).msg_length == 3 and raw[6:] == b"abc"


def test_encode_frame_rejects_oversized_payload():
    class Big(bytes):
        def __len__(self):
            return 1 << 24

    with pytest.raises(F.FrameError, match="U24"):
        F.encode_frame(F.Frame(F.Header(0, 0, 0), Big()))


def test_decoder_reads_back_to_back_frames_and_eof():
    raw = b"".join(M.encode_message(m) for m in _all_messages())
    d = F.Decoder(io.BytesIO(raw))
    got = [M.dispatch_frame(d.read_frame()) for _ in _all_messages()]
    assert [type(g) for g in got] == [type(m) for m in _all_messages()]
    with pytest.raises(EOFError, match="^EOF$"):
        d.read_frame()


def test_decoder_unexpected_eof_mid_frame():
    raw = M.encode_message(M.SetTarget(1, U256))
    with pytest.raises(EOFError, match="unexpected"):
        F.Decoder(io.BytesIO(raw[:-1])).read_frame()
    with pytest.raises(EOFError, match="unexpected"):
        F.Decoder(io.BytesIO(raw[:3])).read_frame()


def test_decoder_max_frame_checked_before_payload_is_read():
    class Tripwire(io.BytesIO):
        reads = 0

        def read(self, n=-1):
            Tripwire.reads += 1
            if Tripwire.reads > 1:
                raise AssertionError("payload read after an oversized header")
            return super().read(n)

    hdr = F.Header(0, 0x15, 1 << 20).encode()
    with pytest.raises(F.FrameError, match="MaxFrameSize"):
        F.Decoder(Tripwire(hdr + b"\x00" * 16), max_frame_size=1024).read_frame()


@pytest.mark.parametrize("size", [0, -1])
def test_decoder_requires_positive_max_frame(size):
    with pytest.raises(F.FrameError, match="positive"):
        F.Decoder(io.BytesIO(b""), max_frame_size=size).read_frame()
    with pytest.raises(F.FrameError, match="positive"):
        F.FrameScanner(size)


def test_default_max_frame_is_16_mib():
    assert F.DEFAULT_MAX_FRAME_SIZE == 16 << 20
    ok = F.Header(0, 0, F.DEFAULT_MAX_FRAME_SIZE - F.HEADER_SIZE)
    F._check_size(ok, F.DEFAULT_MAX_FRAME_SIZE)
    with pytest.raises(F.FrameError):
        F._check_size(F.Header(0, 0, F.DEFAULT_MAX_FRAME_SIZE - F.HEADER_SIZE + 1), F.DEFAULT_MAX_FRAME_SIZE)


def test_read_frame_async():
    raw = M.encode_message(M.SubmitSharesSuccess(1, 2, 3, 4)) + M.encode_message(M.SetTarget(1, U256))

    async def go():
        r = asyncio.StreamReader()
        r.feed_data(raw)
        r.feed_eof()
        a = await F.read_frame_async(r)
        b = await F.read_frame_async(r)
        with pytest.raises(asyncio.IncompleteReadError):
            await F.read_frame_async(r)
        return a, b

    a, b = asyncio.run(go())
    assert isinstance(M.dispatch_frame(a), M.SubmitSharesSuccess) and isinstance(M.dispatch_frame(b), M.SetTarget)


# ------------------------------------------------------------------ dispatch
@pytest.mark.parametrize("mt", [0x05, 0x17, 0x22, 0x70, 0xFF])
def test_unknown_types_dispatch_to_unknown_message(mt):
    f = F.Frame(F.Header(0, mt, 3), b"xyz")
    got = M.dispatch_frame(f)
    assert isinstance(got, M.UnknownMessage) and got.msg_type() == mt and got.payload == b"xyz"
    assert got.encode() == b"xyz"


def test_dispatch_ignores_the_extension_type():
    raw = bytearray(M.encode_message(M.SetTarget(5, U256)))
    raw[0:2] = struct.pack("<H", 0x8000 | 0x0042)
    (f,) = F.iter_frames(bytes(raw))
    assert f.header.extension_id == 0x42 and M.dispatch_frame(f) == M.SetTarget(5, U256)


def test_submit_shares_error_id_per_dialect():
    spec = F.Frame(F.Header(F.CHANNEL_MSG_BIT, 0x1D, 10), M.SubmitSharesError(1, 2, "x").encode())
    ref = F.Frame(F.Header(F.CHANNEL_MSG_BIT, 0x1E, 10), spec.payload)
    assert isinstance(M.dispatch_frame(spec, M.SPEC), M.SubmitSharesError)
    assert isinstance(M.dispatch_frame(ref, M.SPEC), M.UnknownMessage)
    assert isinstance(M.dispatch_frame(ref, M.REFERENCE), M.SubmitSharesError)


def test_error_messages_without_a_reason_string():
    assert M.SubmitSharesError.decode(struct.pack("<II", 1, 2)).error == ""
    assert M.OpenMiningChannelError.decode(struct.pack("<I", 9)).error == ""


# ------------------------------------------------------------------ SetupConnection validation
@pytest.mark.parametrize("proto,mn,mx,ok", [(0, 2, 2, True), (0, 1, 3, True), (1, 2, 2, False), (3, 2, 2, False),
                                            (0, 3, 2, False)])
def test_validate_setup_connection(proto, mn, mx, ok):
    m = M.SetupConnection(proto, mn, mx)
    if ok:
        M.validate_setup_connection(m)
    else:
        with pytest.raises(M.MessageError):
            M.validate_setup_connection(m)


def test_setup_connection_flag_bits():
    assert (M.FLAG_REQUIRES_STANDARD_JOBS, M.FLAG_REQUIRES_WORK_SELECTION, M.FLAG_REQUIRES_VERSION_ROLLING) == (1, 2, 4)


def test_non_utf8_strings_decode_with_replacement():
    payload = struct.pack("<I", 1) + bytes([3]) + b"\xff\xfe\xfd"
    assert M.SetupConnectionError.decode(payload).error == "�" * 3


def test_frame_reader_raises_a_buffered_bad_header_without_waiting_for_more_data():
    good = M.encode_message(M.SetTarget(1, U256))
    bad = F.Header(0, 0x15, F.MAX_MESSAGE_LENGTH).encode()

    async def go():
        r = asyncio.StreamReader()
        r.feed_data(good + bad)  # one socket read carries a good frame and an oversized header; no EOF follows
        fr = F.FrameReader(r)
        assert M.dispatch_frame(await fr.read_frame()) == M.SetTarget(1, U256)
        with pytest.raises(F.FrameError, match="MaxFrameSize"):
            await asyncio.wait_for(fr.read_frame(), 1.0)

    asyncio.run(go())


def test_frame_scanner_does_not_load_the_hip_runtime():
    """A GPU-free engine must not page in the extension (and with it libamdhip64) to split a few SV2 frames a
    second: on a cold GPU host that cost ~1.4 s before the first job (profiles/r3/j_startup)."""
    import subprocess
    import sys

    code = ("import sys; from otedama_amd.stratum.frame import FrameScanner; "
            "FrameScanner().feed(b''); print('otedama_amd._native' in sys.modules)")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert out.stdout.strip() == "False", out.stdout + out.stderr
