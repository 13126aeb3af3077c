"""internal/stratum/noise*_test.go, case by case, against the spec Noise NX here (secp256k1, ChaCha20-Poly1305,
SHA-256) instead of the reference's P-256 variant: HKDF outputs, SymmetricState initialisation / MixHash /
MixKey / Split, CipherState nonce and authentication rules, the handshake state machine's size checks, and
the encrypted stream framing (round trips, truncation, tampering, small reads, oversize writes)."""
from __future__ import annotations

import asyncio
import hashlib
import hmac
import struct

import pytest

from otedama_amd.stratum import noise as N


# ------------------------------------------------------------------ HKDF / HMAC
def test_hmac_sha256_rfc4231_case2():
    # the Noise HKDF is built on HMAC-SHA256; RFC 4231 test case 2
    d = hmac.new(b"Jefe", b"what do ya want for nothing?", hashlib.sha256).hexdigest()
    assert d == "5bdcc146bf60754e6a042426089575c75a003f089d2739839dec58b964ec3843"


@pytest.mark.parametrize("n", [2, 3])
def test_hkdf_outputs_are_32_bytes_deterministic_and_distinct(n):
    ck, ikm = b"\x01" * 32, b"input key material"
    a = N.hkdf(ck, ikm, n)
    assert len(a) == n and all(len(x) == 32 for x in a)
    assert a == N.hkdf(ck, ikm, n)
    assert len(set(a)) == n


def test_hkdf_depends_on_ikm_and_chaining_key():
    base = N.hkdf(b"\x01" * 32, b"a", 2)
    assert N.hkdf(b"\x01" * 32, b"b", 2) != base
    assert N.hkdf(b"\x02" * 32, b"a", 2) != base


def test_hkdf_matches_the_noise_spec_definition():
    ck, ikm = bytes(range(32)), b"ikm"
    tk = hmac.new(ck, ikm, hashlib.sha256).digest()
    o1 = hmac.new(tk, b"\x01", hashlib.sha256).digest()
    o2 = hmac.new(tk, o1 + b"\x02", hashlib.sha256).digest()
    o3 = hmac.new(tk, o2 + b"\x03", hashlib.sha256).digest()
    assert N.hkdf(ck, ikm, 3) == [o1, o2, o3]


# ------------------------------------------------------------------ SymmetricState
def test_initialize_short_name_is_padded_long_name_is_hashed():
    short = N.SymmetricState(b"Noise_NN")
    assert short.h == b"Noise_NN".ljust(32, b"\x00") and short.ck == short.h
    long_ = N.SymmetricState(N.PROTOCOL_NAME)
    assert len(N.PROTOCOL_NAME) > 32 and long_.h == hashlib.sha256(N.PROTOCOL_NAME).digest()


def test_mix_hash_changes_state_and_is_deterministic():
    a, b = N.SymmetricState(), N.SymmetricState()
    h0 = a.h
    a.mix_hash(b"data")
    b.mix_hash(b"data")
    assert a.h != h0 and a.h == b.h == hashlib.sha256(h0 + b"data").digest()


def test_mix_key_updates_chaining_key_and_enables_encryption():
    s = N.SymmetricState()
    ck0 = s.ck
    assert s.cs.k is None and s.encrypt_and_hash(b"plain") == b"plain"  # no key yet: passthrough
    s.mix_key(b"\x07" * 32)
    assert s.ck != ck0 and s.cs.k is not None and s.cs.n == 0
    assert s.encrypt_and_hash(b"plain") != b"plain"


def test_split_populates_two_distinct_ciphers_with_zero_nonces():
    s = N.SymmetricState()
    s.mix_key(b"\x09" * 32)
    c1, c2 = s.split()
    assert c1.k and c2.k and c1.k != c2.k and c1.n == c2.n == 0


# ------------------------------------------------------------------ CipherState
def _cs():
    return N.CipherState(b"\x42" * 32), N.CipherState(b"\x42" * 32)


def test_cipherstate_roundtrip_and_nonce_increments():
    tx, rx = _cs()
    for i in range(5):
        ct = tx.encrypt(b"ad", b"hello %d" % i)
        assert len(ct) == len(b"hello %d" % i) + N.TAG
        assert rx.decrypt(b"ad", ct) == b"hello %d" % i
        assert tx.n == rx.n == i + 1


def test_many_encrypts_produce_different_ciphertexts():
    tx, _ = _cs()
    cts = {tx.encrypt(b"", b"same plaintext") for _ in range(16)}
    assert len(cts) == 16


def test_decrypt_with_a_different_or_skipped_nonce_fails():
    tx, rx = _cs()
    c0 = tx.encrypt(b"", b"zero")
    c1 = tx.encrypt(b"", b"one")
    with pytest.raises(N.NoiseError):
        rx.decrypt(b"", c1)  # receiver expects nonce 0
    assert rx.n == 0  # a failed decrypt does not advance the nonce
    assert rx.decrypt(b"", c0) == b"zero"
    tx2, rx2 = _cs()
    tx2.encrypt(b"", b"skipped")
    c = tx2.encrypt(b"", b"second")
    with pytest.raises(N.NoiseError):
        rx2.decrypt(b"", c)


def test_tampered_ciphertext_and_wrong_ad_fail():
    tx, rx = _cs()
    ct = bytearray(tx.encrypt(b"ad", b"payload"))
    ct[0] ^= 1
    with pytest.raises(N.NoiseError):
        rx.decrypt(b"ad", bytes(ct))
    tx, rx = _cs()
    ct = tx.encrypt(b"ad", b"payload")
    with pytest.raises(N.NoiseError):
        rx.decrypt(b"other ad", ct)
    tag = bytearray(ct)
    tag[-1] ^= 0x80
    with pytest.raises(N.NoiseError):
        rx.decrypt(b"ad", bytes(tag))


def test_nonce_exhaustion_is_refused():
    tx, _ = _cs()
    tx.n = 2 ** 64 - 1
    with pytest.raises(N.NoiseError, match="exhausted"):
        tx.encrypt(b"", b"x")


def test_empty_key_is_passthrough():
    cs = N.CipherState()
    assert cs.encrypt(b"ad", b"abc") == b"abc" and cs.decrypt(b"ad", b"abc") == b"abc" and cs.n == 0


# ------------------------------------------------------------------ handshake state machine
@pytest.mark.parametrize("suite,klen", [("ellswift", 64), ("legacy", 32)])
def test_initiator_message1_and_transport_before_completion(suite, klen):
    hs = N.Initiator(suite=suite)
    m1 = hs.write_message1()
    assert len(m1) == klen and m1 == hs.e_pub
    assert hs.send is None and hs.recv is None  # no transport ciphers before message 2


@pytest.mark.parametrize("suite,klen", [("ellswift", 64), ("legacy", 32)])
def test_read_message2_too_short(suite, klen):
    hs = N.Initiator(suite=suite)
    hs.write_message1()
    with pytest.raises(N.NoiseError, match="too short"):
        hs.read_message2(b"\x00" * (klen + klen + 2 * N.TAG - 1))


def test_message1_must_be_32_or_64_bytes():
    r = N.Responder(12345)
    for n in (0, 31, 33, 63, 65):
        with pytest.raises(N.NoiseError):
            r.read_message1(b"\x02" * n)


def test_message2_with_invalid_ephemeral_key():
    """Legacy suite: x >= p is no curve point. (EllSwift has no invalid encodings: every 64 bytes decode.)"""
    r = N.Responder(12345)
    i = N.Initiator(suite="legacy")
    r.read_message1(i.write_message1())
    m2 = bytearray(r.write_message2(b"p"))
    m2[:32] = b"\xff" * 32  # x >= p: not on the curve
    with pytest.raises(N.NoiseError):
        i.read_message2(bytes(m2))


@pytest.mark.parametrize("suite", N.SUITES)
def test_completed_handshake_transport_keys_cross_over(suite):
    r = N.Responder(987654321)
    i = N.Initiator(expected_static=r.s_xonly, suite=suite)
    r.read_message1(i.write_message1())
    assert i.read_message2(r.write_message2(b"cert")) == b"cert"
    assert i.handshake_hash == r.handshake_hash and i.remote_static == r.s_xonly
    assert i.send.k == r.recv.k and i.recv.k == r.send.k and i.send.k != i.recv.k
    assert r.recv.decrypt(b"", i.send.encrypt(b"", b"up")) == b"up"
    assert i.recv.decrypt(b"", r.send.encrypt(b"", b"down")) == b"down"


# ------------------------------------------------------------------ encrypted streams
class _SinkWriter:
    def __init__(self):
        self.buf = bytearray()

    def write(self, b):
        self.buf += b

    async def drain(self):
        pass


def _pair():
    tx, rx = _cs()
    sink = _SinkWriter()
    return N.EncryptedWriter(sink, tx), sink, rx


def _reader(data: bytes, rx, eof=True):
    r = asyncio.StreamReader()
    r.feed_data(data)
    if eof:
        r.feed_eof()
    return N.EncryptedReader(r, rx)


def test_multiple_messages_round_trip_and_byte_count():
    w, sink, rx = _pair()
    msgs = [b"first", b"", b"x" * 1000, bytes(range(256))]
    for m in msgs:
        w.write(m)

    async def go():
        r = _reader(bytes(sink.buf), rx)
        return [await r.readexactly(len(m)) for m in msgs]

    assert asyncio.run(go()) == msgs


def test_read_reassembles_across_small_reads():
    w, sink, rx = _pair()
    w.write(b"0123456789" * 10)

    async def go():
        r = _reader(bytes(sink.buf), rx)
        out = b""
        while len(out) < 100:
            out += await r.read(7)
        return out

    assert asyncio.run(go()) == b"0123456789" * 10


def test_read_from_truncated_and_empty_streams():
    w, sink, rx = _pair()
    w.write(b"payload")

    async def truncated():
        r = _reader(bytes(sink.buf[:-3]), rx)
        return await r.readexactly(7)

    with pytest.raises(asyncio.IncompleteReadError):
        asyncio.run(truncated())

    async def empty():
        return await _reader(b"", N.CipherState(b"\x42" * 32)).read(10)

    assert asyncio.run(empty()) == b""


def test_tampered_frame_is_detected():
    w, sink, rx = _pair()
    w.write(b"secret share")
    data = bytearray(sink.buf)
    data[5] ^= 0x01

    async def go():
        return await _reader(bytes(data), rx).readexactly(12)

    with pytest.raises(N.NoiseError):
        asyncio.run(go())


def test_oversize_write_is_split_into_max_frames():
    w, sink, rx = _pair()
    big = bytes(range(256)) * 600  # 153600 bytes > one 65535-byte frame
    w.write(big)
    # walk the length prefixes: every frame fits the 16-bit length, and there are several of them
    off, frames = 0, 0
    while off < len(sink.buf):
        n = struct.unpack_from("<H", sink.buf, off)[0]
        assert n <= N.MAX_FRAME
        off += 2 + n
        frames += 1
    assert off == len(sink.buf) and frames == 3

    async def go():
        return await _reader(bytes(sink.buf), rx).readexactly(len(big))

    assert asyncio.run(go()) == big


def test_encode_frame_rejects_oversize_plaintext():
    tx, _ = _cs()
    with pytest.raises(N.NoiseError, match="too large"):
        N.encode_frame(tx, b"\x00" * (N.MAX_FRAME - N.TAG + 1))
    assert tx.n == 0  # the refused frame did not consume a nonce
    assert len(N.encode_frame(N.CipherState(b"\x42" * 32), b"\x00" * (N.MAX_FRAME - N.TAG))) == 2 + N.MAX_FRAME


def test_libcrypto_aead_matches_the_native_binding():
    """The ctypes libcrypto binding (used by a GPU-free engine that must not load the extension) and the native
    extension's binding produce identical ciphertexts and tags and reject the same tampering."""
    import os

    from otedama_amd.ops.native import require_native
    from otedama_amd.utils import aead

    lc = aead.libcrypto()
    if lc is None:
        pytest.skip("libcrypto not loadable")
    nat = require_native()
    for kind in (aead.AES256GCM, aead.CHACHA20POLY1305):
        for n in (0, 1, 31, 1000):
            key, nonce, pt, ad = os.urandom(32), os.urandom(12), os.urandom(n), os.urandom(n % 7)
            a = lc.seal(kind, key, nonce, pt, ad)
            assert a == nat.aead_seal(kind, key, nonce, pt, ad)
            assert lc.open_(kind, key, nonce, a, ad) == pt == nat.aead_open(kind, key, nonce, a, ad)
            bad = bytearray(a)
            bad[-1] ^= 1
            assert lc.open_(kind, key, nonce, bytes(bad), ad) is None
            assert lc.open_(kind, key, nonce, a, ad + b"x") is None


def test_aead_does_not_load_the_extension():
    import subprocess
    import sys

    code = ("import sys; from otedama_amd.utils import aead; c = aead.seal(aead.CHACHA20POLY1305, bytes(32), "
            "bytes(12), b'hi'); assert aead.open_(aead.CHACHA20POLY1305, bytes(32), bytes(12), c) == b'hi'; "
            "print('otedama_amd._native' in sys.modules)")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert out.stdout.strip() == "False", out.stdout + out.stderr
