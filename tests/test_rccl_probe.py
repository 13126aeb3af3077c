"""The bench's data-plane probe (otedama_amd/parallel/rccl_probe.py): its arrival barrier, on a dict-backed store.

The injected "fail" fault makes the child exit before it imports torch, so these run in about a second each.
"""
import json
import threading
import time

from otedama_amd.parallel import rccl_probe


class _Store(dict):
    def set(self, k, v):
        self[k] = v

    def get(self, k):
        return self[k]

    def check(self, keys):
        return all(k in self for k in keys)


def test_probe_child_starts_after_every_rank_arrived():
    store, prefix = _Store(), rccl_probe._prefix()

    def peer():  # rank 1 reaches the probe a second late (a slower cold start), then reports
        time.sleep(1.0)
        store.set(f"{prefix}/arrive/1", "1")
        time.sleep(0.3)
        store.set(f"{prefix}/result/1", json.dumps({"ok": True, "s": 0.3}))

    threading.Thread(target=peer, daemon=True).start()
    r = rccl_probe.run_probe(store, 0, 2, timeout=30, fault="fail")
    assert r["arrive_s"] >= 0.9, r
    assert not r["ok"] and r["ranks"]["0"]["reason"].startswith("exit code 3"), r
    assert r["ranks"]["1"]["ok"]


def test_probe_starts_anyway_when_a_peer_never_arrives():
    store, prefix = _Store(), rccl_probe._prefix()
    store.set(f"{prefix}/result/1", json.dumps({"ok": False, "reason": "peer gone"}))
    t0 = time.monotonic()
    r = rccl_probe.run_probe(store, 0, 2, timeout=30, fault="fail", arrive_timeout=0.5)
    assert 0.4 <= r["arrive_s"] < 5.0 and time.monotonic() - t0 < 20.0, r
    assert not r["ok"] and r["ranks"]["1"]["reason"] == "peer gone"


def test_plan_fits_the_budget():
    """the probe's worst case (a full arrival wait, a hung child, the verdict wait) fits the time the
    pre-flight has left."""
    for budget in (20.0, 60.0, 137.0, 400.0):
        a, t, v = rccl_probe.plan(budget, 60.0, 120.0)
        assert a + t + v <= max(budget, 20.0) + 1e-6 and t >= 10.0 and a >= 1.0 and v >= 5.0, (budget, a, t, v)
    assert rccl_probe.plan(None, 60.0, 120.0) == (120.0, 60.0, 90.0)


def test_followers_take_rank0s_decision_not_their_own_reading():
    """every rank uses rank 0's one decision. A follower whose own child succeeded still falls back when
    rank 0 decided gloo (another rank failed), so no two ranks pick different backends."""
    store, prefix = _Store(), rccl_probe._prefix()
    store.set(f"{prefix}/arrive/0", "1")
    store.set(f"{prefix}/decision", json.dumps({"ok": False, "ranks": {"0": {"ok": False, "reason": "x"},
                                                                       "1": {"ok": True}}}))
    r = rccl_probe.run_probe(store, 1, 2, timeout=30, fault="fail", arrive_timeout=0.5)
    assert not r["ok"] and r["impl"] == "gloo" and r["ranks"]["0"]["reason"] == "x"
    store2, _ = _Store(), None
    store2.set(f"{prefix}/arrive/0", "1")
    store2.set(f"{prefix}/decision", json.dumps({"ok": True, "ranks": {"0": {"ok": True}, "1": {"ok": True}}}))
    r = rccl_probe.run_probe(store2, 1, 2, timeout=30, fault="fail", arrive_timeout=0.5)
    assert r["ok"] and r["impl"] == "rccl-native"  # rank 0's decision stands for every rank
