"""X11 (K6) acceptance vector, pinned ahead of the kernels (no offline per-stage KATs).

The Dash genesis header is rebuilt here from its coinbase transaction and checked against the published
merkle root, so the fixture's 80 bytes are independently verified. An X11 implementation must map them to
the published genesis hash before the algorithm is offered (models/algorithms.py keeps "x11" unregistered
until then; docs/PARITY.md K6)."""
import hashlib
import json
import struct
from pathlib import Path

import pytest

KAT = json.loads((Path(__file__).parent / "fixtures" / "x11_dash_genesis.json").read_text())


def _sha256d(b: bytes) -> bytes:
    return hashlib.sha256(hashlib.sha256(b).digest()).digest()


def _push(data: bytes) -> bytes:
    return (b"\x4c" if len(data) > 75 else b"") + bytes([len(data)]) + data


def test_genesis_header_rebuilds_from_coinbase():
    msg = KAT["coinbase_timestamp"].encode()
    pub = bytes.fromhex(KAT["coinbase_pubkey"])
    script_sig = bytes.fromhex("04ffff001d0104") + _push(msg)   # nBits 0x1d00ffff, CScriptNum(4), timestamp
    spk = _push(pub) + b"\xac"                                  # <pubkey> OP_CHECKSIG
    tx = (struct.pack("<I", 1) + b"\x01" + bytes(32) + b"\xff" * 4 + bytes([len(script_sig)]) + script_sig
          + b"\xff" * 4 + b"\x01" + struct.pack("<q", KAT["reward_sats"]) + bytes([len(spk)]) + spk + bytes(4))
    root = _sha256d(tx)
    assert root[::-1].hex() == KAT["merkle_root_display"]
    hdr = (struct.pack("<I", KAT["version"]) + bytes(32) + root
           + struct.pack("<III", KAT["time"], int(KAT["bits"], 16), KAT["nonce"]))
    assert hdr.hex() == KAT["header_hex"]
    # The published hash meets the header's own compact target (sanity of the pinned digest).
    bits = int(KAT["bits"], 16)
    target = (bits & 0xFFFFFF) << (8 * ((bits >> 24) - 3))
    assert int(KAT["x11_hash_display"], 16) <= target


def test_x11_not_offered_without_a_passing_kat():
    from otedama_amd.models.algorithms import get

    try:
        algo = get("x11")
    except (KeyError, ValueError):
        pytest.skip("x11 not implemented (docs/PARITY.md K6)")
    digest = algo.hash(bytes.fromhex(KAT["header_hex"]))
    assert digest[::-1].hex() == KAT["x11_hash_display"]


def test_x11_cpu_chain_trace_regression_pins():
    """Every intermediate digest of the CPU chain on the genesis header (regression pins; only the final digest
    is independently known, so a change here must come with the genesis test still passing)."""
    from otedama_amd.ops.native import load

    n = load(build_if_missing=False)
    if n is None:
        pytest.skip("native extension not built")
    pins = json.loads((Path(__file__).parent / "fixtures" / "x11_genesis_trace.json").read_text())
    trace = n.x11_trace(bytes.fromhex(pins["header_hex"]))
    for i, (name, want) in enumerate(pins["stages"].items()):
        assert trace[64 * i : 64 * i + 64].hex() == want, name
    assert trace[640:672][::-1].hex() == KAT["x11_hash_display"]


def test_x11_stage_functions_accept_any_length():
    """Each stage is a full hash (padding for any length), not only the 64-byte chain step."""
    from otedama_amd.ops.native import load

    n = load(build_if_missing=False)
    if n is None:
        pytest.skip("native extension not built")
    for st in range(11):
        outs = {n.x11_stage(st, bytes(range(256))[:L]) for L in (0, 1, 63, 64, 65, 127, 128, 129, 200)}
        assert len(outs) == 9 and all(len(o) == 64 for o in outs)
    with pytest.raises(ValueError):
        n.x11_stage(11, b"")


def test_x11_cpu_luffa_bitsliced_sbox_matches_table():
    from otedama_amd.ops.native import load

    n = load(build_if_missing=False)
    if n is None:
        pytest.skip("native extension not built")
    assert n.x11_luffa_sbox_selfcheck()
