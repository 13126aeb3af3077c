"""Share previews (parallel/node.py): a follower sends each new share record to the leader's preview port, and the
leader submits it on arrival instead of waiting for the R2 gather. R2 still carries every share. The leader admits
each share once, whichever path brings it first. On the MI355X the gather waits for a wave slot under a saturating
miner (profiles/r5/e_reserve_cus). Reference: the fan-in never makes a producer wait
(internal/engine/fanin.go:22-58)."""
import os

import pytest

from otedama_amd.parallel.commbase import SHARE_SLOTS
from otedama_amd.parallel.node import parse_share_preview, share_key, share_preview_msgs


def _share(i):
    return {"epoch": (3 << 40) + i, "nonce": 0xFFFFFFF0 + (i % 16), "ntime": 1_700_000_000 + i,
            "version": 0x20000000 | (i << 13), "extranonce2": (1 << 63) + i, "found_at": 1234.5 + i,
            "device_found_at": 1234.25 + i}


def test_preview_datagrams_round_trip_every_field():
    shares = [_share(i) for i in range(SHARE_SLOTS + 6)]
    msgs = share_preview_msgs(shares, orig_rank=5)
    assert len(msgs) == 2 and all(len(m) < 60000 for m in msgs)
    got = [s for m in msgs for s in parse_share_preview(m)]
    assert len(got) == len(shares)
    for a, b in zip(shares, got):
        assert b["orig_rank"] == 5
        for k in ("epoch", "nonce", "ntime", "version", "extranonce2"):
            assert b[k] == a[k], k
        assert abs(b["found_at"] - a["found_at"]) < 1e-6 and abs(b["device_found_at"] - a["device_found_at"]) < 1e-6
    assert share_key(got[0]) != share_key(got[1])


@pytest.mark.parametrize("msg", [b"", b"p", b"p\x01\x00", b"p\x01\x00" + b"x" * 79, b"o\x01\x00" + bytes(80)])
def test_malformed_previews_are_ignored(msg):
    assert parse_share_preview(msg) == []


@pytest.mark.timeout(300)
@pytest.mark.parametrize("drop", [False, True])
def test_node_submits_previews_and_admits_each_share_once(drop, monkeypatch):
    """A 3-rank CPU node against a pool process: with the datagrams flowing, the followers' shares are admitted from
    their previews. With every datagram dropped (fault injection), R2 delivers them all. The pool re-hashes every
    share and rejects none: no share was submitted twice."""
    from otedama_amd.parallel.node_probe import measure_node

    if drop:
        monkeypatch.setenv("OTEDAMA_FAULT_BELL_DROP", "1")
    r = measure_node(3, seconds=3, warmup=1, cpu=True, algorithm="sha256d", switches=0)
    assert r["exit_code"] == 0 and r["pool_rejected"] == 0 and r["accepted_remote_in_window"] > 0, r
    if drop:
        assert r["share_previews"] == 0 and r["share_gathered_first"] > 0, r
    else:
        assert r["share_previews"] > 0, r
        assert r["share_gathered_first"] <= max(2, r["share_previews"] // 20), r  # a datagram is rarely late
