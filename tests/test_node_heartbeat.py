"""A follower's heartbeat survives a failed store write (parallel/node.py _Heartbeat): the write is retried on a fresh
connection at the next beat. Before, the heartbeat thread returned on the first failure, and the leader then saw a live
rank as dead for good (stale heartbeat, never re-admitted)."""
import json
import time

from otedama_amd.parallel import node as nodemod


class _FlakyStore:
    """Fails the first writes of the first connections, then works."""

    def __init__(self, shared, fail_first=2):
        self.shared = shared
        self.fail_first = fail_first

    def clone(self):
        self.shared["clones"] += 1
        return _FlakyStore(self.shared, 0 if self.shared["clones"] > 2 else self.fail_first)

    def set(self, key, value):
        if self.fail_first > 0:
            self.fail_first -= 1
            raise TimeoutError("store stalled")
        self.shared["data"][key] = value


class _Local:
    epoch = 7

    def device_stats(self):
        return {"gpu-0": {"hashes": 10, "shares": 1, "dropped": 0, "faulted": False, "hashes_done_at_s": 1.0}}

    def high_water(self):
        return 3


def test_heartbeat_retries_a_failed_write_on_a_fresh_connection(monkeypatch):
    monkeypatch.setattr(nodemod, "HB_INTERVAL", 0.01)
    shared = {"clones": 0, "data": {}}
    hb = nodemod._Heartbeat(_FlakyStore(shared), 3, _Local())
    hb.start()
    try:
        end = time.monotonic() + 5
        while "otd/hb/3" not in shared["data"] and time.monotonic() < end:
            time.sleep(0.01)
    finally:
        hb.stop.set()
        hb.th.join(timeout=2)
    assert "otd/hb/3" in shared["data"], shared
    assert hb.failures >= 1 and shared["clones"] >= 2
    assert json.loads(shared["data"]["otd/hb/3"])["hashes"] == 10
