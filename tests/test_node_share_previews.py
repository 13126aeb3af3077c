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


def test_leader_admits_each_share_once_and_forgets_old_keys(monkeypatch):
    """NodeMinerSet._take: a share seen from a preview is skipped when its R2 copy arrives; the remembered keys are
    pruned past SEEN_TTL and capped at SEEN_MAX (the leader's heap stays flat on a long run)."""
    import collections
    import os as _os
    import threading
    import types

    from otedama_amd.parallel import node as nodemod

    clock = [1000.0]
    monkeypatch.setattr(nodemod.time, "monotonic", lambda: clock[0])
    monkeypatch.setattr(nodemod, "SEEN_MAX", 4)
    ms = types.SimpleNamespace(
        comm=types.SimpleNamespace(info=types.SimpleNamespace(orig_rank=0)), _take_lock=threading.Lock(),
        _seen=collections.OrderedDict(), _jobs={(3 << 40) + i: {"job_id": str(i)} for i in range(16)},
        remote_stale=0, _remote=collections.deque(), share_previews=0, share_gathered_first=0,
        _remote_efd=_os.eventfd(0, _os.EFD_NONBLOCK), _gather_wanted=False)
    take = nodemod.NodeMinerSet._take

    def share(i):
        return dict(_share(i), orig_rank=1)

    take(ms, [share(0)], preview=True)
    take(ms, [share(0)])  # its R2 copy
    assert len(ms._remote) == 1 and ms.share_previews == 1 and ms.share_gathered_first == 0
    for i in range(1, 6):
        take(ms, [share(i)], preview=True)
    assert len(ms._seen) <= 5 and len(ms._remote) == 6  # capped (pruned before each batch)
    clock[0] += nodemod.SEEN_TTL + 1
    take(ms, [share(7)], preview=True)
    assert list(ms._seen.values()) == [clock[0]]  # everything older than the TTL is gone
    _os.close(ms._remote_efd)


def test_previews_are_taken_only_from_the_ranks_doorbell_socket():
    """The leader's preview reader accepts a datagram only from the doorbell socket its rank published
    (otd/bell/<rank>); a datagram from any other local socket is refused and counted."""
    import socket
    import threading
    import time as _time
    import types

    from otedama_amd.parallel import node as nodemod
    from otedama_amd.parallel.kvclient import StoreClient
    from otedama_amd.parallel.kvstore import StoreServer

    with StoreServer() as srv:
        store = StoreClient("127.0.0.1", srv.port, timeout=10)
        leader_bell, follower_bell = nodemod._Bell(store, 0), nodemod._Bell(store, 1)
        spv = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        spv.bind(("127.0.0.1", 0))
        spv.setblocking(False)
        taken = []
        ms = types.SimpleNamespace(_bell=leader_bell, _spv=spv, _stop=False, previews_refused=0,
                                   log=lambda *a: None, _take=lambda sh, preview: taken.extend(sh))
        th = threading.Thread(target=nodemod.NodeMinerSet._spv_loop, args=(ms,), daemon=True)
        th.start()
        port = spv.getsockname()[1]
        msg = nodemod.share_preview_msgs([_share(1)], 1)[0]
        rogue = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        rogue.sendto(msg, ("127.0.0.1", port))            # right format, wrong socket
        assert follower_bell.send_port(port, msg)          # the rank's own doorbell socket
        end = _time.monotonic() + 5
        while (not taken or ms.previews_refused < 1) and _time.monotonic() < end:
            _time.sleep(0.01)
        ms._stop = True
        th.join(timeout=2)
        assert len(taken) == 1 and taken[0]["orig_rank"] == 1 and ms.previews_refused == 1
        for sock in (rogue, spv):
            sock.close()
        leader_bell.close()
        follower_bell.close()
