"""Device processes on a real MI355X (engine/devproc.py): the GPU-side half of the fault-containment contract.

A device process is SIGKILLed while its 2^32-hash SHA-256d launch runs on the GPU. The parent (GPU-free) must
survive, retire the device, start a fresh process on the same GPU after the 1 s backoff (the killed process's
queues and memory are torn down by the driver) and resume hashing with verified shares. A real kernel page fault is
not injected on purpose: on this pool it can reset every GPU of the host; SIGKILL is the same process death the
supervisor sees after one.

Also: KFD-topology enumeration (what the GPU-free engine uses) names the same devices, with the same CU counts and
architecture, as the HIP runtime.
"""
import os
import signal
import time

import pytest

from otedama_amd import hal
from otedama_amd.engine.miners import MinerSet
from otedama_amd.models.header import int_to_hash, sha256d

pytestmark = pytest.mark.gpu


def _job(target):
    hdr = bytes([1, 0, 0, 0]) + os.urandom(64) + (1700000000).to_bytes(4, "little") + bytes.fromhex("ffff001d") + \
        bytes(4)
    return {"header": hdr, "target": int_to_hash(target), "job_id": "gpu-A", "algo": "sha256d",
            "version_mask": 0x1FFFE000}


def _verify(job, s, target):
    hdr = bytearray(job["header"])
    hdr[0:4] = int(s["version"]).to_bytes(4, "little")
    hdr[76:80] = int(s["nonce"]).to_bytes(4, "little")
    return int.from_bytes(sha256d(bytes(hdr)), "little") <= target


def _wait(pred, timeout):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        if pred():
            return True
        time.sleep(0.02)
    return pred()


def test_kfd_enumeration_matches_the_hip_runtime():
    kfd = hal.KFDDriver().enumerate()
    hip = hal.HIPDriver().enumerate()
    assert kfd and len(kfd) == len(hip)
    for a, b in zip(sorted(kfd, key=lambda d: d.index), sorted(hip, key=lambda d: d.index)):
        assert (a.index, a.identity().id, a.identity().model) == (b.index, b.identity().id, b.identity().model)
        assert a.extra["arch"] == b.extra["arch"] == "gfx950" and a.extra["cus"] == b.extra["cus"] > 0
        assert a.capabilities() == b.capabilities()


def test_sigkilled_gpu_device_process_restarts_and_resumes():
    devs = [d for d in hal.KFDDriver().enumerate() if d.index == 0]
    assert devs
    logs = []
    ms = MinerSet(devs, "sha256d", isolation="process", log=lambda lvl, msg: logs.append((lvl, msg)))
    target = (1 << 226) - 1  # ~1 share per 2^30 hashes: ~18 shares/s at 19 GH/s
    job = _job(target)
    shares = []
    ms.start()
    try:
        m = ms.miners[0]
        assert _wait(lambda: m.native.ready_at > 0, 120), logs
        ms.set_job(job)
        assert _wait(lambda: len(shares.extend(ms.poll(256)) or shares) >= 5, 30), logs
        old_pid = m.native.pid
        time.sleep(0.1)  # inside a running 2^32-hash launch
        t_kill = time.monotonic()
        os.kill(old_pid, signal.SIGKILL)
        assert _wait(lambda: m.retired, 5.0), logs
        # the fresh process (1 s backoff) opens the same GPU and reports in
        assert _wait(lambda: not m.retired and m.native.pid != old_pid, 60), logs
        t_back = time.monotonic() - t_kill
        n0 = len(shares)
        assert _wait(lambda: len(shares.extend(ms.poll(256)) or shares) >= n0 + 5, 60), logs
        t_shares = time.monotonic() - t_kill
        st = m.native.stats()
        print(f"device process back after {t_back:.2f} s, shares again after {t_shares:.2f} s; restarts "
              f"{m.native.restarts}; startup {st.get('native_startup_ms')}")
        assert m.native.restarts == 1
        assert not st.get("faulted"), st
    finally:
        ms.stop()
    assert all(_verify(job, s, target) for s in shares)
    assert len({(s["version"], s["nonce"]) for s in shares}) == len(shares)  # nothing searched twice


def test_device_process_starts_hashing_within_a_second():
    """process start -> first GPU hash under 1 s (a warm page cache; bench.py records it)."""
    from otedama_amd.engine.latency_probe import measure_device_startup

    res = measure_device_startup(0)
    print("device process start-up:", res)
    assert res["spawn_to_first_batch_s"] < 1.0, res
    assert res["native_phases_ms"].get("first_batch") is not None, res


def test_share_latency_pool_in_its_own_process():
    """device hit -> pool accept p50 under 2 ms, with the pool in a separate process and the GPU in
    a device process (the production layout)."""
    from otedama_amd.engine.latency_probe import measure_share_latency

    res = measure_share_latency(device_index=0, seconds=4.0)
    print("share latency:", {k: v for k, v in res.items() if k.endswith("_ms") or k.startswith("pool_")})
    assert res["accepted"] >= 5 and res["rejected"] == 0 and res["pool_rejected"] == 0, res
    assert res["device_hit_to_accept_p50_ms"] is not None and res["device_hit_to_accept_p50_ms"] < 2.0, res
    assert res["p50_ms"] < 2.0, res
