"""Noise NX (stratum/noise_test.go, noise_pool_test.go): handshake, transport, framing."""
import asyncio
import struct

import pytest

from otedama_amd.stratum import noise as N
from otedama_amd.stratum.frame import Frame, Header, encode_frame, read_frame_async


SUITES = pytest.mark.parametrize("suite", N.SUITES)


def _pair(static_priv=12345, payload=b"cert", suite=N.DEFAULT_SUITE):
    r = N.Responder(static_priv)
    i = N.Initiator(suite=suite)
    r.read_message1(i.write_message1())
    got = i.read_message2(r.write_message2(payload))
    return i, r, got


def test_hkdf_rfc5869_like():
    a, b = N.hkdf(b"\x00" * 32, b"ikm", 2)
    assert len(a) == len(b) == 32 and a != b
    assert N.hkdf(b"\x00" * 32, b"ikm", 3)[:2] == [a, b]


@SUITES
def test_handshake_roundtrip(suite):
    i, r, payload = _pair(suite=suite)
    assert r.suite == suite
    assert payload == b"cert"
    assert i.handshake_hash == r.handshake_hash
    assert i.remote_static_wire == r.s_pub and i.remote_static == r.s_xonly
    assert i.remote_static == N.keypair(12345)[1]  # the x-only key in both suites
    for msg in (b"", b"hello", bytes(1000)):
        assert r.recv.decrypt(b"", i.send.encrypt(b"", msg)) == msg
        assert i.recv.decrypt(b"", r.send.encrypt(b"", msg)) == msg
    assert i.send.n == 3 and r.recv.n == 3


@SUITES
def test_pinned_static_key(suite):
    _, pub = N.keypair(777)
    r = N.Responder(777)
    i = N.Initiator(expected_static=pub, suite=suite)
    r.read_message1(i.write_message1())
    i.read_message2(r.write_message2())
    r2 = N.Responder(778)
    i2 = N.Initiator(expected_static=pub, suite=suite)
    r2.read_message1(i2.write_message1())
    with pytest.raises(N.NoiseError, match="pinned"):
        i2.read_message2(r2.write_message2())


@SUITES
def test_tamper_and_replay_rejected(suite):
    for pos in (5, 40, 70, -1):  # ephemeral key, static key, tag
        r = N.Responder(999)
        i = N.Initiator(suite=suite)
        r.read_message1(i.write_message1())
        m2 = bytearray(r.write_message2(b"x"))
        m2[pos] ^= 1
        with pytest.raises(N.NoiseError):
            i.read_message2(bytes(m2))
    i, r, _ = _pair(suite=suite)
    ct = i.send.encrypt(b"", b"once")
    assert r.recv.decrypt(b"", ct) == b"once"
    with pytest.raises(N.NoiseError):
        r.recv.decrypt(b"", ct)  # nonce advanced: replay fails


def test_message_size_checks():
    with pytest.raises(N.NoiseError):
        N.Initiator().read_message2(b"\x00" * 10)
    with pytest.raises(N.NoiseError):
        N.Responder(5).read_message1(b"\x00" * 31)
    with pytest.raises(N.NoiseError, match="64"):
        N.Responder(5, suite="ellswift").read_message1(b"\x00" * 32)  # a fixed suite refuses the other
    with pytest.raises(N.NoiseError, match="32"):
        N.Responder(5, suite="legacy").read_message1(b"\x00" * 64)
    with pytest.raises(N.NoiseError, match="unknown suite"):
        N.Initiator(suite="p256")
    i, _, _ = _pair()
    with pytest.raises(N.NoiseError, match="too large"):
        N.encode_frame(i.send, bytes(N.MAX_FRAME))


def test_certificate():
    auth_priv, auth_pub = N.keypair(4242)
    _, static_pub = N.keypair(31337)
    cert = N.certificate_payload(static_pub, auth_priv, 100, 200)
    assert N.verify_certificate(cert, static_pub, auth_pub, 150)
    assert not N.verify_certificate(cert, static_pub, auth_pub, 250)
    assert not N.verify_certificate(cert, b"\x01" * 32, auth_pub, 150)


@SUITES
def test_async_stream_carries_sv2_frames(suite):
    async def main():
        got = []

        async def handle(reader, writer):
            er, ew = await N.server_handshake(reader, writer, 5555, b"pool-cert")
            f = await read_frame_async(er)
            got.append(f)
            ew.write(encode_frame(Frame(Header(0, 0x1B, 4), b"pong")))
            big = bytes(range(256)) * 400  # > one Noise frame
            ew.write(big)
            await ew.drain()
            writer.close()

        srv = await asyncio.start_server(handle, "127.0.0.1", 0)
        port = srv.sockets[0].getsockname()[1]
        reader, writer = await asyncio.open_connection("127.0.0.1", port)
        _, pub = N.keypair(5555)
        er, ew, payload, rs = await N.client_handshake(reader, writer, expected_static=pub, suite=suite)
        assert payload == b"pool-cert" and rs == pub
        ew.write(encode_frame(Frame(Header(0, 0x1A, 4), b"ping")))
        await ew.drain()
        f = await read_frame_async(er)
        assert f.payload == b"pong" and f.header.msg_type == 0x1B
        assert await er.readexactly(256 * 400) == bytes(range(256)) * 400
        writer.close()
        srv.close()
        await srv.wait_closed()
        assert got[0].payload == b"ping"

    asyncio.run(main())


def test_wire_is_encrypted():
    i, _, _ = _pair()
    fr = N.encode_frame(i.send, b"mining.submit secret")
    (n,) = struct.unpack("<H", fr[:2])
    assert n == len(fr) - 2 == 20 + 16 and b"secret" not in fr


def test_ellswift_wire_sizes_match_sv2():
    """SV2 (EllSwift suite): message 1 is the 64-byte encoded ephemeral key; message 2 with the 74-byte
    SignatureNoiseMessage is 64 + 80 + 90 = 234 bytes. The legacy suite's are 32 and 32 + 48 + 90."""
    auth_priv, _ = N.keypair(4242)
    for suite, m1_len, m2_len in (("ellswift", 64, 234), ("legacy", 32, 170)):
        r = N.Responder(31337)
        i = N.Initiator(suite=suite)
        m1 = i.write_message1()
        r.read_message1(m1)
        cert = N.certificate_payload(N.keypair(31337)[1], auth_priv, 0, 2**32 - 1)
        m2 = r.write_message2(cert)
        assert (len(m1), len(m2)) == (m1_len, m2_len)
        assert i.read_message2(m2) == cert


def test_ellswift_protocol_name_hash():
    """The 45-byte protocol name is longer than 32: h0 = SHA-256(name) (Noise spec §5.2)."""
    import hashlib

    assert N.PROTOCOL_NAME_ELLSWIFT == b"Noise_NX_Secp256k1+EllSwift_ChaChaPoly_SHA256"
    assert N.SymmetricState(N.PROTOCOL_NAME_ELLSWIFT).h == hashlib.sha256(N.PROTOCOL_NAME_ELLSWIFT).digest()
