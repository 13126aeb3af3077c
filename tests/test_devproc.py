"""One process per device (engine/devproc.py) on the CPU: the same parent/child protocol, re-split and respawn
path as the GPU processes, with native CpuMiner children (a dead device must not stop the
node). A child is SIGKILLed mid-job: within ~2 s the survivors are re-striped past every cursor so the dead
device's residue class keeps being searched, verified shares keep flowing, a fresh process replaces the dead one
and rejoins the stripe plan, and nothing hangs."""
import os
import signal
import time

import pytest

from otedama_amd import hal
from otedama_amd.engine.miners import MinerSet
from otedama_amd.models.header import int_to_hash, sha256d


def _devs(n):
    return [hal.SimpleDevice(hal.Identity(f"cpu-{i}", hal.Family.CPU, "t", "cpu"),
                             hal.Capabilities(sha256d=True, general_compute=True), threads=1) for i in range(n)]


def _job():
    hdr = bytes([1, 0, 0, 0]) + bytes(range(32)) + bytes(range(32, 64)) + (1700000000).to_bytes(4, "little") + \
        bytes.fromhex("ffff001d") + bytes(4)
    return {"header": hdr, "target": int_to_hash(1 << 241), "job_id": "job-A", "algo": "sha256d",
            "version_mask": 0x1FFFE000}


def _verify(s):
    hdr = bytearray(_job()["header"])
    hdr[0:4] = int(s["version"]).to_bytes(4, "little")
    hdr[76:80] = int(s["nonce"]).to_bytes(4, "little")
    return int.from_bytes(sha256d(bytes(hdr)), "little") <= 1 << 241


def _wait(pred, timeout):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        if pred():
            return True
        time.sleep(0.02)
    return pred()


def test_sigkilled_device_process_is_resplit_and_replaced():
    logs = []
    ms = MinerSet(_devs(4), "sha256d", isolation="process", log=lambda lvl, msg: logs.append((lvl, msg)))
    ms.start()
    shares = []
    try:
        assert _wait(lambda: all(m.native.ready_at > 0 for m in ms.miners), 60), logs
        ep = ms.set_job(_job())
        assert _wait(lambda: len({s["device_id"] for s in (shares.extend(ms.poll(256)) or shares)}) == 4, 60)
        victim = ms.miners[2]
        old_pid = victim.native.pid
        # cursors are reported at 2 Hz; wait for one with the current epoch
        assert _wait(lambda: victim.native.stats().get("variant_epoch", 0) >= ep, 5)
        hw_before = ms.high_water()
        t_kill = time.monotonic()
        os.kill(old_pid, signal.SIGKILL)
        assert _wait(lambda: victim.retired and ms.resplits >= 1, 2.0), logs
        t_resplit = time.monotonic() - t_kill
        assert t_resplit < 2.0
        # survivors: stride 3, starting past every cursor (the dead device's class is covered from there on)
        jobs = [m.native._job for m in ms.miners if m is not victim]
        starts = sorted(j["variant_start"] for j in jobs)
        assert all(j["variant_stride"] == 3 for j in jobs)
        assert starts == [starts[0], starts[0] + 1, starts[0] + 2] and starts[0] > hw_before
        assert victim.native.stats()["faulted"]
        # verified shares keep flowing from the survivors
        n0 = len(shares)
        assert _wait(lambda: len(shares.extend(ms.poll(256)) or shares) >= n0 + 6, 20)
        # the replacement process (backoff 1 s) reports in and is re-striped back in
        assert _wait(lambda: not victim.retired, 20), logs
        assert victim.native.pid != old_pid and victim.native.restarts == 1
        assert _wait(lambda: ms.resplits >= 2, 5)
        jobs = [m.native._job for m in ms.miners]
        assert all(j["variant_stride"] == 4 for j in jobs)
        n1 = len(shares)
        assert _wait(lambda: any(s["device_id"] == "cpu-2" for s in (shares.extend(ms.poll(256)) or shares)[n1:]), 30)
    finally:
        t0 = time.monotonic()
        ms.stop()
        assert time.monotonic() - t0 < 15  # nothing hangs
    assert shares and all(_verify(s) for s in shares)
    assert all(s["job_id"] == "job-A" for s in shares)
    # nothing searched twice: the replacement starts on a fresh stripe, not the dead process's old one
    assert len({(s["version"], s["nonce"]) for s in shares}) == len(shares)
    assert any("lost" in m for _, m in logs) and any("back" in m for _, m in logs)


def test_device_process_startup_and_counters_survive_restart():
    ms = MinerSet(_devs(1), "sha256d", isolation="process")
    ms.start()
    try:
        dp = ms.miners[0].native
        assert _wait(lambda: dp.ready_at > 0, 60)
        assert 0 < dp.startup_seconds < 30
        ms.set_job(_job())
        assert _wait(lambda: dp.stats()["hashes"] > 0, 20)
        h = dp.stats()["hashes"]
        fds = len(os.listdir("/proc/self/fd"))
        dp.kill(signal.SIGKILL)
        assert _wait(lambda: not ms.miners[0].retired and dp.restarts == 1 and dp.alive, 20)
        assert dp.stats()["hashes"] >= h  # cumulative across the restart
        assert len(os.listdir("/proc/self/fd")) <= fds  # the dead child's socket was closed, the new one replaces it
    finally:
        ms.stop()


def test_kfd_topology_enumeration_without_a_runtime(tmp_path, monkeypatch):
    """The engine names GPUs from the KFD topology (no HIP runtime in the parent); CPU nodes are skipped, the
    arch comes from gfx_target_version, CUs from simd_count / simd_per_cu, and *_VISIBLE_DEVICES re-numbers."""
    nodes = {0: "cpu_cores_count 64\nsimd_count 0\ngfx_target_version 0\n",
             1: "simd_count 1024\nsimd_per_cu 4\ngfx_target_version 90500\n",
             2: "simd_count 1024\nsimd_per_cu 4\ngfx_target_version 90500\n",
             3: "simd_count 440\nsimd_per_cu 4\ngfx_target_version 90010\n"}
    for n, text in nodes.items():
        d = tmp_path / str(n)
        d.mkdir()
        (d / "properties").write_text(text)
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    devs = hal.KFDDriver(str(tmp_path)).enumerate()
    assert [(d.identity().id, d.index, d.extra["arch"], d.extra["cus"]) for d in devs] == \
        [("gpu-0", 0, "gfx950", 256), ("gpu-1", 1, "gfx950", 256), ("gpu-2", 2, "gfx90a", 110)]
    assert devs[0].capabilities().sha256d and not devs[2].capabilities().sha256d
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1,2")
    devs = hal.KFDDriver(str(tmp_path)).enumerate()
    assert [(d.index, d.extra["arch"]) for d in devs] == [(0, "gfx950"), (1, "gfx90a")]


def test_kfd_topology_skips_nodes_whose_render_device_is_not_openable(tmp_path, monkeypatch):
    """A container given some of the host's GPUs sees every KFD node but can open only its own render devices;
    the runtime skips the others, so the KFD list must too or ordinal i names another GPU."""
    topo, dri = tmp_path / "topo", tmp_path / "dri"
    topo.mkdir()
    dri.mkdir()
    for n, minor in ((1, 128), (2, 129), (3, 130)):
        d = topo / str(n)
        d.mkdir()
        (d / "properties").write_text(f"simd_count 1024\nsimd_per_cu 4\ngfx_target_version 90500\n"
                                      f"drm_render_minor {minor}\n")
    (dri / "renderD128").write_text("")
    (dri / "renderD130").write_text("")  # renderD129 is another container's GPU: absent here
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    devs = hal.KFDDriver(str(topo), dri_path=str(dri)).enumerate()
    assert [(d.identity().id, d.index) for d in devs] == [("gpu-0", 0), ("gpu-1", 1)]
    os.chmod(dri / "renderD130", 0)  # present but not openable (root ignores modes: only check when it matters)
    if not os.access(dri / "renderD130", os.R_OK | os.W_OK):
        assert len(hal.KFDDriver(str(topo), dri_path=str(dri)).enumerate()) == 1


def test_process_isolation_engine_side_does_not_load_the_extension():
    """The engine of a GPU node hands every GPU to a device process: building its MinerSet must not import the
    native extension (which links the HIP runtime; ~1 GB of RSS once a GPU context exists)."""
    import subprocess
    import sys

    code = (
        "import sys\n"
        "from otedama_amd import hal\n"
        "from otedama_amd.engine.miners import MinerSet, variant_space\n"
        "gpu = hal.SimpleDevice(hal.Identity('gpu-0', hal.Family.GPU, 'AMD', 'AMD Instinct MI355X 256CU gfx950'),\n"
        "                       hal.KERNEL_ISAS['gfx950'], index=0, extra={'arch': 'gfx950', 'cus': 256})\n"
        "ms = MinerSet([gpu], 'sha256d', isolation='process')\n"
        "assert len(ms.miners) == 1 and variant_space({'version_mask': 0x1FFFE000}) == 65536\n"
        "print('otedama_amd._native' in sys.modules)\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60,
                         env=dict(os.environ, OTEDAMA_NO_TORCH="1"))
    assert out.stdout.strip() == "False", out.stdout + out.stderr


@pytest.mark.parametrize("env,want", [({"OTEDAMA_DEVICE_HW_QUEUES": "1"}, "1"),
                                      ({"OTEDAMA_DEVICE_HW_QUEUES": "1", "GPU_MAX_HW_QUEUES": "3"}, "3"),
                                      ({}, None)])
def test_device_process_hardware_queue_cap(env, want):
    """OTEDAMA_DEVICE_HW_QUEUES reaches the child as GPU_MAX_HW_QUEUES (an explicit GPU_MAX_HW_QUEUES wins); by
    default the runtime's own cap stays (the two search streams need their own queues, docs/RUNTIME.md)."""
    from otedama_amd.engine.devproc import DeviceProcess

    base = {k: v for k, v in os.environ.items() if k not in ("OTEDAMA_DEVICE_HW_QUEUES", "GPU_MAX_HW_QUEUES")}
    dp = DeviceProcess(0, "cpu-q", cpu_threads=1, env=dict(base, **env))
    dp.start()
    try:
        with open(f"/proc/{dp.pid}/environ", "rb") as f:
            child = dict(kv.split(b"=", 1) for kv in f.read().split(b"\0") if b"=" in kv)
    finally:
        dp.stop()
    got = child.get(b"GPU_MAX_HW_QUEUES")
    assert (got.decode() if got is not None else None) == want
