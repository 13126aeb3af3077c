"""Native GPU runtime on a real MI355X: in-kernel hit publication, the device abort word, target-only updates.

* Hits reach the host while the launch that found them is still running (host-coherent ring polled by the
  miner thread), each carrying the kernel's own s_memrealtime stamp mapped to the host clock.
* New work moves the device abort word: the running batch stops within a grid-stride trip and the switch
  (set_job -> first batch of the new work running) is timed.
* A target-only update (same work, SV2 SetTarget / V1 set_difficulty) reaches the share filter at the next launch
  of the cached variant group (the version-parallel path used to keep the old target for the group).
Every share is re-hashed on the CPU (hashlib) against the header it claims.
"""
import hashlib
import os
import struct
import time

import pytest

pytestmark = pytest.mark.gpu


def _native():
    from otedama_amd.ops.native import require_native

    return require_native()


def _check_share(hdr: bytes, s: dict, target_int: int, algo: str = "sha256d") -> None:
    h80 = bytearray(hdr)
    struct.pack_into("<I", h80, 0, s["version"])
    struct.pack_into("<I", h80, 76, s["nonce"])
    if algo == "scrypt":
        d = hashlib.scrypt(bytes(h80), salt=bytes(h80), n=1024, r=1, p=1, dklen=32)
    else:
        d = hashlib.sha256(hashlib.sha256(bytes(h80)).digest()).digest()
    assert d == s["hash"] and int.from_bytes(d, "little") <= target_int


def _job(hdr, target_int, epoch, job_id, **kw):
    from otedama_amd.models.header import int_to_hash

    return dict({"header": hdr, "target": int_to_hash(target_int), "epoch": epoch, "job_id": job_id,
                 "version_mask": 0x1FFFE000}, **kw)


def test_hits_arrive_while_the_launch_runs():
    N = _native()
    hdr = os.urandom(76) + bytes(4)
    target = (1 << 232) - 1  # ~256 hits per 2^32-hash launch
    m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 32)  # one launch = 2^32 hashes (~0.22 s)
    m.set_job(_job(hdr, target, 7, "j7"))
    m.start()
    try:
        deadline = time.monotonic() + 10
        first = []
        while time.monotonic() < deadline and not first:
            first = m.poll(256)
            time.sleep(0.0005)
        st_first = m.stats()
        time.sleep(0.6)
        rest = m.poll(4096)
    finally:
        m.stop()
    st = m.stats()
    assert not st["faulted"], st
    assert first, st
    assert st_first["launches"] == 0, st_first  # delivered before any batch completed
    assert st["ring_hits"] > 0
    for s in first + rest:
        _check_share(hdr, s, target)
        assert s["epoch"] == 7 and s["job_id"] == "j7"
        # device clock mapped to the host clock: the hit precedes its verification by well under a launch
        assert 0 < s["device_found_at"] <= s["found_at"] + 0.002, s
        assert s["found_at"] - s["device_found_at"] < 0.05, s
    assert st["clock_calib_rtt_us"] > 0


def test_new_work_aborts_the_running_batch():
    N = _native()
    hdr_a, hdr_b = os.urandom(76) + bytes(4), os.urandom(76) + bytes(4)
    target = (1 << 236) - 1
    m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 32)  # ~0.22 s launches: a switch without abort waits for two
    m.set_job(_job(hdr_a, target, 1, "a"))
    m.start()
    try:
        time.sleep(0.5)
        m.poll(4096)
        m.set_job(_job(hdr_b, target, 2, "b"))
        time.sleep(0.05)
        st_switch = m.stats()
        time.sleep(0.4)
        shares = m.poll(4096)
    finally:
        m.stop()
    st = m.stats()
    assert not st["faulted"], st
    assert st_switch["job_switches"] >= 2, st_switch  # the first job and the switch to b
    assert st_switch["last_job_switch_ms"] < 20.0, st_switch
    assert st["aborted_launches"] >= 1, st
    b = [s for s in shares if s["job_id"] == "b"]
    assert b
    for s in shares:
        _check_share(hdr_b if s["job_id"] == "b" else hdr_a, s, target)


@pytest.mark.parametrize("host_abort", ["1", "0"])
def test_abort_word_store_paths(monkeypatch, host_abort):
    """The CPU stores the abort word straight into VRAM on the MI355X (no control stream); with
    OTEDAMA_HOST_ABORT=0 the store goes through a high-priority stream. Both stop the running batch for new work,
    and the per-launch clock probes keep the device -> host clock mapping (shares stamped before their host
    verification, within a launch)."""
    monkeypatch.setenv("OTEDAMA_HOST_ABORT", host_abort)
    N = _native()
    hdr_a, hdr_b = os.urandom(76) + bytes(4), os.urandom(76) + bytes(4)
    target = (1 << 236) - 1
    m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 32)
    m.set_job(_job(hdr_a, target, 1, "a"))
    m.start()
    try:
        time.sleep(0.5)
        m.poll(4096)
        m.set_job(_job(hdr_b, target, 2, "b"))
        time.sleep(0.5)
        shares = m.poll(4096)
    finally:
        m.stop()
    st = m.stats()
    assert not st["faulted"], st
    assert st["host_abort"] is (host_abort == "1"), st
    assert st["last_job_switch_ms"] < 20.0 and st["aborted_launches"] >= 1, st
    assert st["clock_samples"] >= 2, st
    b = [s for s in shares if s["job_id"] == "b"]
    assert b
    for s in b:
        _check_share(hdr_b, s, target)
        assert 0 < s["device_found_at"] <= s["found_at"] + 0.002 and s["found_at"] - s["device_found_at"] < 0.05, s


def test_target_only_update_reaches_the_running_group():
    """Same work, easier target, partway through a 128-variant group: shares at the new target appear within a
    couple of 2^29-nonce launches (the version-parallel variant table stays cached; its target must not)."""
    N = _native()
    hdr = os.urandom(76) + bytes(4)
    hard, easy = (1 << 190) - 1, (1 << 234) - 1
    m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 29)
    m.set_job(_job(hdr, hard, 1, "t"))
    m.start()
    try:
        time.sleep(0.4)
        assert m.poll(256) == []
        t0 = time.monotonic()
        m.set_job(_job(hdr, easy, 2, "t"))
        shares = []
        while time.monotonic() - t0 < 2.0 and not shares:
            shares = m.poll(256)
            time.sleep(0.001)
        dt = time.monotonic() - t0
        st = m.stats()
    finally:
        m.stop()
    assert not st["faulted"], st
    assert shares, st
    assert dt < 0.2, dt
    assert st["job_switches"] == 1  # a target-only update is not new work: no abort, no cursor reset
    for s in shares:
        _check_share(hdr, s, easy)
        assert s["epoch"] == 2


def test_scrypt_switch_stops_the_romix_batch():
    """New scrypt work stops the running batches: polls at both ROMix phase boundaries and, from the scalar unit,
    every 64 iterations of the write loop; the two half-grid batches run half a hash apart, so one of them is always
    writing and frees its half within ~1 ms (under 10 ms p50; round 3 took 12-17 ms)."""
    import statistics

    N = _native()
    hdrs = [os.urandom(76) + bytes(4) for _ in range(6)]
    target = (1 << 240) - 1  # ~16 hits per 1 Mi-hash batch
    m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 29)
    m.set_job(_job(hdrs[0], target, 1, "j0", algo="scrypt"))
    m.start()
    shares = []
    try:
        t0 = time.monotonic()
        while m.stats()["job_switches"] < 1 and time.monotonic() - t0 < 30:  # 128 GiB scratch + first batch
            time.sleep(0.01)
        for k in range(1, 6):
            time.sleep(0.3)
            m.set_job(_job(hdrs[k], target, k + 1, f"j{k}", algo="scrypt"))
            shares += m.poll(4096)
        time.sleep(0.4)
        shares += m.poll(4096)
    finally:
        m.stop()
    st = m.stats()
    assert not st["faulted"], st
    sw = st["job_switch_ms"][-5:]
    print("scrypt switch ms:", sw)
    assert st["job_switches"] >= 6 and statistics.median(sw) < 10.0 and max(sw) < 45.0, st
    assert st["aborted_launches"] >= 1
    by_id = {f"j{k}": h for k, h in enumerate(hdrs)}
    for s in shares[:40]:
        _check_share(by_id[s["job_id"]], s, target, "scrypt")


def test_startup_phases_are_recorded():
    """The device thread times its own start-up (start -> first GPU hash): HIP context, streams,
    control words, buffers, clock calibration, the wait for the first job and the first batch (set_job -> running,
    incl. code-object load), with the resident set after each."""
    N = _native()
    hdr = os.urandom(76) + bytes(4)
    t0 = time.monotonic()
    m = N.GpuMiner(0, "gpu-0")
    m.start()
    try:
        m.set_job(_job(hdr, (1 << 190) - 1, 1, "t"))
        while time.monotonic() - t0 < 20 and m.stats()["job_switches"] < 1:
            time.sleep(0.002)
        wall = time.monotonic() - t0
        st = m.stats()
    finally:
        m.stop()
    assert not st["faulted"], st
    ph = st["startup_ms"]
    print("startup phases ms:", {k: round(v, 2) for k, v in ph.items()}, "construct->first batch s:", round(wall, 3))
    assert list(ph) == ["hip_set_device", "streams", "control_words", "buffers", "clock_calibration",
                        "wait_first_job", "first_batch"]
    print("resident MiB after each phase:", st["startup_rss_mb"])
    assert list(st["startup_rss_mb"])[:5] == list(ph)[:5]
    assert all(v >= 0 for v in ph.values())
    assert sum(ph.values()) <= wall * 1e3 + 50


def test_job_switch_with_other_streams_in_the_process():
    """The abort-word write must not queue behind a search kernel when the process holds more HIP streams than the
    runtime has hardware queues (torch's streams plus the miner's two search streams): bench.py measured ~110 ms
    switches at 2^32-hash launches before the control stream got a high-priority queue of its own."""
    import torch

    from otedama_amd.engine.latency_probe import measure_job_switch

    extra = [torch.cuda.Stream() for _ in range(6)]
    for s in extra:  # give each stream a queue (first use) and keep them alive
        with torch.cuda.stream(s):
            torch.ones(1, device="cuda").add_(1)
    torch.cuda.synchronize()
    res = measure_job_switch(0, "sha256d", switches=6, batch_nonces=1 << 32)
    print("job switch at 2^32:", res)
    assert res["path"] == "devproc"
    assert res["p50_ms"] is not None and res["p50_ms"] < 20.0, res  # engine -> device process -> new batch
    assert res["max_ms"] < 50.0, res
    inproc = res["in_process"]  # the miner in this process, next to torch's streams
    assert inproc["p50_ms"] is not None and inproc["p50_ms"] < 20.0, inproc
    assert inproc["max_ms"] < 50.0, inproc


def _drain(m, seconds):
    shares, end = [], time.monotonic() + seconds
    while time.monotonic() < end:
        shares += m.poll(1 << 16)
        time.sleep(0.002)
    return shares


def test_launches_are_sized_from_the_share_target_and_nothing_is_lost():
    """at a target giving ~4000 candidates per 2^32 hashes, launches shrink (powers of two) until
    the expected candidates per launch are <= hit-ring capacity / 8, so no candidate overflows the ring: every
    candidate the kernels counted is a verified share or a counted top-word tie, and the share count matches the
    Poisson expectation of the hashes searched."""
    N = _native()
    hdr = os.urandom(76) + bytes(4)
    target = (4000 << 224) - 1
    m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 32, queue_cap=1 << 22)
    m.set_job(_job(hdr, target, 1, "d"))
    m.start()
    try:
        shares = _drain(m, 1.5)
    finally:
        m.stop()
    shares += m.poll(1 << 22)
    st = m.stats()
    assert not st["faulted"], st
    assert st["launch_hashes"] <= 1 << 29, st["launch_hashes"]  # 2^32 cut to keep <= 512 expected candidates
    assert st["ring_overflow"] == 0 and st["dropped"] == 0, st
    assert st["candidates"] == st["shares"] + st["rejected_candidates"], st
    assert len(shares) == st["shares"]
    expected = st["hashes"] * (target + 1) / 2.0 ** 256
    assert abs(len(shares) - expected) < 6 * expected ** 0.5 + 0.01 * expected, (len(shares), expected)
    keys = {(s["version"], s["nonce"]) for s in shares}
    assert len(keys) == len(shares)  # no duplicate
    for s in shares[:400]:
        _check_share(hdr, s, target)


def test_ring_overflow_is_counted_exactly(monkeypatch):
    """With launch sizing off (OTEDAMA_LAUNCH_CAP=0: 2^32-hash launches) at ~16000 candidates per launch, the 4096-
    record hit ring overflows; every candidate past it is counted in ring_overflow, so candidates = verified shares +
    top-word ties + ring_overflow exactly, and the engine-facing counter reports the loss."""
    N = _native()
    monkeypatch.setenv("OTEDAMA_LAUNCH_CAP", "0")
    hdr = os.urandom(76) + bytes(4)
    target = (16000 << 224) - 1
    m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 32, queue_cap=1 << 22)
    m.set_job(_job(hdr, target, 1, "o"))
    m.start()
    try:
        shares = _drain(m, 1.2)
    finally:
        m.stop()
    shares += m.poll(1 << 22)
    st = m.stats()
    assert not st["faulted"], st
    assert st["launch_hashes"] == 1 << 32
    assert st["ring_overflow"] > 0, st
    assert st["candidates"] == st["shares"] + st["rejected_candidates"] + st["ring_overflow"], st
    assert len(shares) == st["shares"] and st["dropped"] == 0
    for s in shares[:200]:
        _check_share(hdr, s, target)
