"""GPU-fault handling and per-device stall detection.

A faulted device is retired and its rank's variant class (parallel/partition.py) is re-split among
the survivors at once, starting past the high-water mark of every device's cursor on the current work
(never re-searching a variant, so no duplicate shares); when that jump does not fit in the job's
variant space the re-split waits for the next NEW work. A live device with work whose hash counter
stops is reported as stalled."""
import time
from types import SimpleNamespace

import pytest

from otedama_amd.engine import miners as miners_mod
from otedama_amd.engine.miners import DeviceMiner, MinerSet
from otedama_amd.parallel.partition import stripe_for


class FakeNative:
    def __init__(self):
        self.jobs, self.hashes, self.fault, self.stopped = [], 0, "", False
        self.done_at = 0.0  # device-timeline completion time of `hashes` (0: none reported)
        self.cursor = (0, 0)  # (variant_next, variant_epoch) as the native miners report them

    def start(self):
        pass

    def stop(self):
        self.stopped = True

    def set_job(self, t):
        self.jobs.append(t)

    def poll(self, n):
        return []

    def stats(self):
        return {"hashes": self.hashes, "shares": 0, "dropped": 0, "faulted": bool(self.fault), "error": self.fault,
                "candidates": 0, "launches": 0, "variant_next": self.cursor[0], "variant_epoch": self.cursor[1],
                "hashes_done_at_s": self.done_at}


def _dev(name):
    return SimpleNamespace(identity=lambda: SimpleNamespace(id=name))


def _set(n, rank=0, world=1, log=None):
    from otedama_amd.ops.native import require_native

    ms = MinerSet.__new__(MinerSet)
    ms.algorithm, ms.log = "sha256d", log or (lambda lvl, msg: None)
    ms.N, ms._variant_base, ms._work_epoch0, ms.resplits, ms._stopped = require_native(), 0, 0, 0, False
    ms.miners = [DeviceMiner(_dev(f"gpu{i}"), FakeNative()) for i in range(n)]
    ms.rank, ms.world_size, ms.stall_samples, ms._restripe_pending = rank, world, 3, False
    ms._restripe()
    import threading
    import time
    ms._lock, ms._epoch, ms._template, ms._t_last = threading.RLock(), 0, None, time.monotonic()
    return ms


def _covered(stripes, n):
    seen = []
    for st in stripes:
        seen += [v for v in st.variants(n) if v < n]
    return sorted(seen)


@pytest.mark.parametrize("world,local", [(1, 1), (1, 4), (2, 3), (8, 1), (4, 2)])
def test_two_level_stripes_are_a_partition(world, local):
    n = 240
    stripes = [stripe_for(r, world, i, local) for r in range(world) for i in range(local)]
    assert _covered(stripes, n) == list(range(n))  # disjoint (no repeats) and complete


def test_rank_resplits_its_own_class_after_a_fault():
    world, n = 4, 400
    plan = {r: [stripe_for(r, world, i, 3) for i in range(3)] for r in range(world)}
    plan[2] = [stripe_for(2, world, i, 2) for i in range(2)]  # rank 2 lost one of 3 devices
    assert _covered([s for ss in plan.values() for s in ss], n) == list(range(n))


def _tmpl(prev=b"\x01", target="ff" * 32, job="j1"):
    return {"algo": "sha256d", "header": (prev * 80)[:80].hex(), "target": target, "job_id": job}


def test_faulted_device_retired_and_stripe_resplit_on_next_new_work():
    """A template whose variant space cannot take the jump (here: not even parseable) defers the re-split."""
    logs = []
    ms = _set(3, log=lambda lvl, msg: logs.append((lvl, msg)))
    ms.set_job(_tmpl())
    assert [(m.native.jobs[-1]["variant_start"], m.native.jobs[-1]["variant_stride"]) for m in ms.miners] == \
        [(0, 3), (1, 3), (2, 3)]
    ms.miners[1].native.fault = "hipErrorLaunchFailure"
    assert ms.retire_faulted() == [("gpu1", "hipErrorLaunchFailure")]
    assert ms.miners[1].native.stopped and ms.miners[1].retired
    assert ms.retire_faulted() == []                     # reported once
    assert any("retired" in m for _, m in logs)
    n1 = len(ms.miners[1].native.jobs)
    # same work, new target (SetTarget): stripes must NOT move (cursor keeps going, no duplicates)
    ms.set_job(_tmpl(target="7f" + "ff" * 31, job="j2"))
    assert [(m.native.jobs[-1]["variant_start"], m.native.jobs[-1]["variant_stride"]) for m in (ms.miners[0],
            ms.miners[2])] == [(0, 3), (2, 3)]
    # new work: survivors take the whole class
    ms.set_job(_tmpl(prev=b"\x02", job="j3"))
    assert [(m.native.jobs[-1]["variant_start"], m.native.jobs[-1]["variant_stride"]) for m in (ms.miners[0],
            ms.miners[2])] == [(0, 2), (1, 2)]
    assert len(ms.miners[1].native.jobs) == n1           # retired device gets no more work
    assert ms.stripe_total == 2 and [m.id for m in ms.live()] == ["gpu0", "gpu2"]


def test_per_device_stall_detection():
    logs = []
    ms = _set(2, log=lambda lvl, msg: logs.append((lvl, msg)))
    for _ in range(5):                                   # no work: idle is not a stall
        ms.update_hashrates()
    assert ms.stalled() == []
    ms.set_job(_tmpl())
    for k in range(3):
        ms.miners[0].native.hashes += 1 << 29             # gpu0 progresses, gpu1 is hung
        ms.update_hashrates()
    assert ms.stalled() == ["gpu1"]
    assert sum("no hash progress" in m for _, m in logs) == 1
    ms.pause_device("gpu1", True)
    ms.update_hashrates()
    assert ms.stalled() == []                            # paused on purpose
    ms.pause_device("gpu1", False)
    ms.miners[1].native.hashes += 5
    ms.update_hashrates()
    assert ms.stalled() == []


def test_engine_metrics_track_device_health():
    from otedama_amd.engine.metrics import EngineMetrics
    from otedama_amd.metrics import Registry

    m = EngineMetrics(Registry())
    m.devices_active.set(7)
    m.devices_faulted.set(1)
    assert m.devices_active.value() == 7 and m.devices_faulted.value() == 1
    assert miners_mod._work_key(_tmpl(target="00" * 32)) == miners_mod._work_key(_tmpl())


def _real_tmpl(prev=b"\x01", target=b"\xff" * 32, job="j1", mask=0x1FFFE000):
    return {"algo": "sha256d", "header": (prev * 80)[:80], "target": target, "job_id": job, "version_mask": mask}


def test_fault_resplits_at_once_past_every_cursor():
    """Real template (2^16 BIP320 variants): the survivors get the whole class immediately, starting past the
    highest cursor any device reported (dead one included) plus two 128-variant groups of the old stride."""
    ms = _set(3)
    ep = ms.set_job(_real_tmpl())
    assert [(j["variant_start"], j["variant_stride"]) for j in (m.native.jobs[-1] for m in ms.miners)] == \
        [(0, 3), (1, 3), (2, 3)]
    # cursors: gpu0 started variants 0,3 (next 6); gpu1 up to 7 (next 10, then died); gpu2 next 5
    ms.miners[0].native.cursor, ms.miners[1].native.cursor, ms.miners[2].native.cursor = (6, ep), (10, ep), (5, ep)
    ms.miners[1].native.fault = "device process killed by signal 9"
    assert [d for d, _ in ms.retire_faulted()] == ["gpu1"]
    base = 10 + 2 * 128 * 3
    survivors = [m.native.jobs[-1] for m in (ms.miners[0], ms.miners[2])]
    assert [(j["variant_start"], j["variant_stride"]) for j in survivors] == [(base, 2), (base + 1, 2)]
    assert ms.resplits == 1
    # the dead device's residue class (1 mod 3) is covered going forward, and nothing below base repeats
    covered = sorted(v for j in survivors for v in range(j["variant_start"], base + 600, j["variant_stride"]))
    assert covered == list(range(base, base + 600))
    # cursors of an older job epoch are ignored: new work restarts from 0
    ms.miners[0].native.cursor = (9000, ep)
    ep2 = ms.set_job(_real_tmpl(prev=b"\x02", job="j2"))
    assert ep2 > ep and [m.native.jobs[-1]["variant_start"] for m in (ms.miners[0], ms.miners[2])] == [0, 1]


def test_node_variant_base_adds_to_the_local_resplit():
    ms = _set(2, rank=1, world=4)
    ms.set_job(dict(_real_tmpl(), variant_base=4096))
    assert [(m.native.jobs[-1]["variant_start"], m.native.jobs[-1]["variant_stride"]) for m in ms.miners] == \
        [(4096 + 1, 8), (4096 + 5, 8)]
    assert "variant_base" not in ms.miners[0].native.jobs[-1]


@pytest.mark.parametrize("rank,world", [(1, 2), (1, 4), (3, 4), (5, 8)])
def test_local_resplit_keeps_the_rank_residue_class(rank, world):
    """a device cursor sits in the rank's class (rank mod world), so the re-split offset must be a
    multiple of world_size; otherwise rank 1 of 2 moved to even variants (rank 0's class: duplicate shares) and left
    its own class unsearched. Every new start stays congruent to rank mod world and the survivors cover the class."""
    ms = _set(2, rank=rank, world=world)
    ep = ms.set_job(dict(_real_tmpl(), variant_base=4096))
    first = [m.native.jobs[-1]["variant_start"] for m in ms.miners]
    assert all(v % world == rank for v in first)
    # device cursors as the native miners report them: the next unstarted variant of their own stripe
    ms.miners[0].native.cursor = (first[0] + 37 * ms.miners[0].stripe_stride, ep)
    ms.miners[1].native.cursor = (first[1] + 41 * ms.miners[1].stripe_stride, ep)
    ms.miners[1].native.fault = "hipErrorLaunchFailure"
    ms.retire_faulted()
    survivor = ms.miners[0].native.jobs[-1]
    assert survivor["variant_start"] % world == rank, survivor
    assert survivor["variant_stride"] == world
    assert survivor["variant_start"] >= max(c for c, _ in (ms.miners[0].native.cursor, ms.miners[1].native.cursor))


def test_python_variant_space_matches_native():
    from otedama_amd.engine.miners import variant_space
    from otedama_amd.ops.native import require_native

    N = require_native()
    base = {"header": bytes(80), "target": bytes(32), "algo": "sha256d"}
    cases = [{}, {"version_mask": 0x1FFFE000}, {"version_mask": 0xFFFFFFFF}, {"ntime_roll": 7},
             {"version_mask": 0x1FFFE000, "ntime_roll": 3},
             {"coinb1": b"a", "coinb2": b"b", "extranonce1": b"e", "extranonce2_size": 4, "merkle_branches": []},
             {"coinb1": b"a", "coinb2": b"b", "extranonce1": b"e", "extranonce2_size": 8, "merkle_branches": [],
              "version_mask": 0x1FFFE000},
             {"coinb1": b"a", "coinb2": b"b", "extranonce1": b"e", "extranonce2_size": 0, "merkle_branches": []}]
    for c in cases:
        t = dict(base, **c)
        assert variant_space(t) == N.variant_space(t), c


def test_total_hashrate_from_device_timeline_spans():
    """GPU counters move a whole launch at a time: the node total is the sum of the exact device-timeline rates, not
    a wall-clock sample (which read 25.7 GH/s for a 19.3 GH/s device over a 1 s window)."""
    ms = _set(2)
    ms.set_job(_tmpl())
    ms.update_hashrates()
    assert ms.exact_total() is None                     # no device-timeline completion yet: wall window
    for m in ms.miners:                                 # first completions: still no span to divide by
        m.native.hashes, m.native.done_at = 1 << 32, 10.0
    ms.update_hashrates()
    assert ms.exact_total() is None
    ms.miners[0].native.hashes, ms.miners[0].native.done_at = 6 << 32, 11.0   # 5 launches in 1.0 device-s
    ms.miners[1].native.hashes, ms.miners[1].native.done_at = 4 << 32, 11.5   # 3 launches in 1.5 device-s
    ms.update_hashrates()
    assert ms.exact_total() == pytest.approx((5 << 32) / 1.0 + (3 << 32) / 1.5)
    ms.miners[1].retired = True                         # a retired device no longer counts
    ms.miners[0].native.hashes, ms.miners[0].native.done_at = 7 << 32, 11.25
    ms.update_hashrates()
    assert ms.exact_total() == pytest.approx((1 << 32) / 0.25)


def test_node_total_hashrate_from_each_ranks_device_timeline():
    """The node leader's total: local device-timeline rates plus each member rank's rate over its heartbeat's
    device-timeline completion span; a rank without one puts the node back on the wall-clock window."""
    from otedama_amd.parallel.node import NodeMinerSet

    local = _set(1)
    local.set_job(_tmpl())
    node = NodeMinerSet.__new__(NodeMinerSet)
    node.local, node.capacity, node._blob, node._paused = local, 3, None, set()
    node.comm = SimpleNamespace(info=SimpleNamespace(members=[0, 1, 2]))
    node._rows_by_orig, node._prev_rows, node._hb_pairs, node._prev_pairs, node._exact = {}, {}, {}, {}, {}
    node.row_done_at, node._rates, node._remote_idle, node._t_last = {}, {}, {}, time.monotonic()

    def tick(local_h, local_t, rows):
        local.miners[0].native.hashes, local.miners[0].native.done_at = local_h, local_t
        for r, (h, t) in rows.items():  # as the heartbeat reader stores them
            node._rows_by_orig[r], node.row_done_at[r], node._hb_pairs[r] = [h, 0, 0, 0], t, (h, t)
        node.update_hashrates()

    tick(1 << 32, 1.0, {1: (1 << 32, 50.0), 2: (1 << 32, 7.0)})
    tick(3 << 32, 1.5, {1: (4 << 32, 51.0), 2: (2 << 32, 7.5)})
    assert node.exact_total() == pytest.approx((2 << 32) / 0.5 + (3 << 32) / 1.0 + (1 << 32) / 0.5)
    tick(4 << 32, 1.75, {1: (5 << 32, 51.25), 2: (2 << 32, 7.5)})   # rank 2 counted nothing new
    assert node.exact_total() is None


def test_total_hashrate_adds_continuous_cpu_rates_to_exact_gpu_rates():
    ms = _set(2)
    ms.set_job(_tmpl())
    gpu, cpu = ms.miners
    gpu.native.hashes, gpu.native.done_at = 1 << 32, 5.0
    ms.update_hashrates()
    gpu.native.hashes, gpu.native.done_at = 3 << 32, 5.5
    cpu.native.hashes = 1_000_000                       # no device timeline: a continuous counter
    ms.update_hashrates()
    assert ms.exact_total() == pytest.approx((2 << 32) / 0.5 + cpu.hashrate)
    assert not cpu.exact and not cpu.timeline and gpu.exact
