"""Native CPU mining worker, case by case: mirrors internal/miner/worker_test.go against `_native.CpuMiner`.

Reference behaviour (file:line in /root/reference/internal/miner/worker.go) and where it differs by design:
  * Stats before Start are zero; Start/Stop lifecycle ............. :127-164, :194-211
  * easy target finds shares on every thread ....................... :216-282
  * SetWork switches the job: later shares carry the new job ........ :171-176
  * shares carry the configured device id (empty when unset) ........ :33-43
  * non-blocking share send, drops counted when the queue is full ... :266-275
  * HashRateString .................................................. :285-298
Differences: Start twice is a no-op instead of a panic (worker_test.go TestWorker_StartTwicePanics pins the Go panic);
threads claim 64 Ki-nonce chunks from a shared cursor instead of a fixed stride, so no two threads ever hash the same
nonce of the same work (the reference's stride scheme, worker.go:220-221,279, gives the same guarantee per job).
"""
import os
import struct
import threading
import time

import pytest

from otedama_amd.engine.stats import hashrate_string
from otedama_amd.models.header import GENESIS_HEADER_HEX, int_to_hash, sha256d
from otedama_amd.ops.native import require_native

N = require_native()
GEN = bytes.fromhex(GENESIS_HEADER_HEX)
EASY = int_to_hash((1 << 248) - 1)  # ~1 share per 256 hashes
NEVER = bytes(32)                   # target 0: no share in practice


def job(**kw):
    j = {"header": GEN, "target": EASY, "epoch": 1, "job_id": "j1"}
    j.update(kw)
    return j


def collect(m, want: int, timeout: float = 5.0) -> list[dict]:
    out, deadline = [], time.time() + timeout
    while time.time() < deadline and len(out) < want:
        out += m.poll(256)
        time.sleep(0.01)
    return out


def verify(s: dict, header: bytes, target: bytes) -> None:
    hdr = bytearray(header)
    struct.pack_into("<I", hdr, 0, s["version"])
    struct.pack_into("<I", hdr, 68, s["ntime"])
    struct.pack_into("<I", hdr, 76, s["nonce"])
    h = sha256d(bytes(hdr))
    assert h == s["hash"]
    assert int.from_bytes(h, "little") <= int.from_bytes(target, "little")


@pytest.fixture
def miner():
    made = []

    def make(threads=2, device_id="cpu-0", queue_cap=1024):
        m = N.CpuMiner(threads, device_id, queue_cap)
        made.append(m)
        return m
    yield make
    for m in made:
        m.stop()


def test_worker_stats_before_start(miner):
    st = miner().stats()
    assert st["hashes"] == 0 and st["shares"] == 0 and st["dropped"] == 0 and st["candidates"] == 0
    assert not st["faulted"]


def test_worker_start_twice_is_a_noop(miner):
    m = miner(threads=2)
    m.set_job(job())
    m.start()
    m.start()
    assert collect(m, 2)
    m.stop()
    m.stop()  # idempotent as well


def test_worker_stop_without_start(miner):
    miner().stop()


def test_worker_start_and_stop(miner):
    m = miner(threads=2)
    m.set_job(job(target=NEVER))
    m.start()
    time.sleep(0.2)
    m.stop()
    h = m.stats()["hashes"]
    assert h > 0 and h % (1 << 16) == 0  # whole 64 Ki-nonce chunks
    time.sleep(0.1)
    assert m.stats()["hashes"] == h  # no thread survives Stop


def test_worker_restart_after_stop(miner):
    m = miner(threads=1)
    m.set_job(job())
    m.start()
    assert collect(m, 1)
    m.stop()
    m.start()
    assert collect(m, 1)


def test_worker_finds_shares_with_easy_target(miner):
    m = miner(threads=1)
    m.set_job(job())
    m.start()
    shares = collect(m, 10)
    m.stop()
    assert len(shares) >= 10
    for s in shares:
        verify(s, GEN, EASY)
        assert s["job_id"] == "j1" and s["epoch"] == 1


def test_worker_multiple_threads_find_distinct_shares(miner):
    m = miner(threads=4)
    m.set_job(job())
    m.start()
    shares = collect(m, 64)
    m.stop()
    keys = [(s["version"], s["ntime"], s["nonce"]) for s in shares]
    assert len(keys) >= 64 and len(set(keys)) == len(keys)  # no nonce searched twice
    for s in shares:
        verify(s, GEN, EASY)


def test_worker_set_work_job_change(miner):
    m = miner(threads=2)
    m.set_job(job(job_id="old", epoch=1))
    m.start()
    assert collect(m, 1)
    other = bytes(reversed(GEN[:76])) + GEN[76:]
    m.set_job(job(header=other, job_id="new", epoch=2))
    time.sleep(0.05)
    m.poll(100000)  # drain anything found before the switch
    shares = collect(m, 8)
    m.stop()
    fresh = [s for s in shares if s["job_id"] == "new"]
    assert len(fresh) >= 8 * len(shares) // 10
    for s in fresh:
        assert s["epoch"] == 2
        verify(s, other, EASY)


def test_worker_pause_with_none_and_resume(miner):
    m = miner(threads=2)
    m.set_job(job(target=NEVER))
    m.start()
    time.sleep(0.05)
    m.set_job(None)
    time.sleep(0.05)
    h0 = m.stats()["hashes"]
    time.sleep(0.15)
    assert m.stats()["hashes"] == h0
    m.set_job(job(target=NEVER))
    time.sleep(0.15)
    assert m.stats()["hashes"] > h0


def test_worker_stats_after_work(miner):
    m = miner(threads=2)
    m.set_job(job())
    m.start()
    shares = collect(m, 20)
    m.stop()
    shares += m.poll(100000)
    st = m.stats()
    assert st["hashes"] >= 1 << 16 and st["busy_seconds"] > 0
    assert st["shares"] == st["candidates"] == len(shares) + st["dropped"]
    assert st["launches"] == 0 and not st["faulted"]  # CPU: no device launches
    rate = st["hashes"] / st["busy_seconds"]
    assert rate > 1e5  # H/s per busy thread-second (SHA-NI or portable path)


def test_worker_full_queue_drops_are_counted(miner):
    m = miner(threads=2, queue_cap=4)
    m.set_job(job())
    m.start()
    deadline = time.time() + 5
    while time.time() < deadline and m.stats()["dropped"] == 0:
        time.sleep(0.01)
    m.stop()
    st = m.stats()
    assert st["dropped"] > 0
    kept = m.poll(100000)
    assert len(kept) == 4 and st["shares"] == len(kept) + st["dropped"]


def test_share_device_id_propagated_from_config(miner):
    m = miner(threads=1, device_id="cpu-7")
    assert m.device_id == "cpu-7"
    m.set_job(job())
    m.start()
    shares = collect(m, 2)
    assert shares and all(s["device_id"] == "cpu-7" for s in shares)


def test_share_device_id_empty_when_not_set(miner):
    m = miner(threads=1, device_id="")
    assert m.device_id == ""
    m.set_job(job())
    m.start()
    shares = collect(m, 1)
    assert shares and shares[0]["device_id"] == ""


def test_worker_zero_threads_defaults_to_one(miner):
    m = miner(threads=0)
    m.set_job(job())
    m.start()
    assert collect(m, 1)


def test_default_worker_threads_use_all_cores():
    from otedama_amd.hal import CPUDriver
    devs = CPUDriver().enumerate()
    assert len(devs) == 1 and devs[0].identity().id == "cpu-0"
    assert devs[0].capabilities().sha256d
    assert os.cpu_count() >= 1


def test_worker_version_rolling_shares_stay_in_mask(miner):
    mask = 0x1FFFE000
    m = miner(threads=2)
    m.set_job(job(version_mask=mask))
    m.start()
    shares = collect(m, 16)
    m.stop()
    base = struct.unpack_from("<I", GEN, 0)[0]
    for s in shares:
        assert (s["version"] ^ base) & ~mask == 0
        verify(s, GEN, EASY)


def test_worker_poll_is_thread_safe(miner):
    m = miner(threads=2)
    m.set_job(job())
    m.start()
    got, lock = [], threading.Lock()

    def drain():
        end = time.time() + 0.5
        while time.time() < end:
            batch = m.poll(8)
            with lock:
                got.extend(batch)
    ts = [threading.Thread(target=drain) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    m.stop()
    got += m.poll(100000)
    keys = [(s["version"], s["nonce"]) for s in got]
    assert len(keys) == len(set(keys)) == m.stats()["shares"] - m.stats()["dropped"]


@pytest.mark.parametrize("hps,want", [(500, "500 H/s"), (1500, "1.50 kH/s"), (2.5e6, "2.50 MH/s"),
                                      (3.7e9, "3.70 GH/s"), (120e12, "120.00 TH/s")])
def test_hash_rate_string(hps, want):
    assert hashrate_string(hps) == want  # worker_test.go TestHashRateString table
