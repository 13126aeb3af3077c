"""parallel/node_probe.py: the node object of bench.py — exact window rates from (hashes, device-timeline time)
pairs, nearest-rank quantiles with sample counts, and the per-role RSS map."""
import os

import pytest

from otedama_amd.parallel.node_probe import _quantiles, _rank_of, process_rss, window_rates


def test_window_rates_use_the_device_timeline_span():
    # rank0: a GPU whose counter moves a launch at a time; the wall times of the samples are irregular, the
    # device-timeline completion times are what the hashes belong to
    samples = [
        (10.0, {"rank0": (1000, 5.0), "rank1": (0, 0.0)}),
        (10.5, {"rank0": (1000, 5.0), "rank1": (50, 0.0)}),
        (11.2, {"rank0": (3000, 7.0), "rank1": (120, 0.0)}),
        (12.0, {"rank0": (5000, 9.0), "rank1": (200, 0.0)}),
        (30.0, {"rank0": (9999, 99.0), "rank1": (999, 0.0)}),  # outside the window
    ]
    r = window_rates(samples, 10.0, 12.0)
    assert r["rank0"] == pytest.approx((5000 - 1000) / (9.0 - 5.0))
    # no device timeline (a CPU miner): the wall span of the samples
    assert r["rank1"] == pytest.approx(200 / 2.0)


def test_window_rates_need_two_samples():
    assert window_rates([(1.0, {"rank0": (10, 1.0)})], 0.0, 5.0) == {}
    assert window_rates([], 0.0, 5.0) == {}


def test_nearest_rank_quantiles_report_their_sample_count():
    q = _quantiles([float(x) for x in range(1, 201)])
    assert q == {"p50_ms": 100.0, "p95_ms": 190.0, "p99_ms": 198.0, "samples": 200}
    assert _quantiles([]) == {"p50_ms": None, "p95_ms": None, "p99_ms": None, "samples": 0}
    assert _quantiles([3.0])["p99_ms"] == 3.0


def test_rank_keys_and_rss_roles():
    assert _rank_of("rank7") == 7 and _rank_of("gpu-0") == 0
    rss = process_rss(os.getpid())  # this process as the "supervisor": its children (if any) are not ranks here
    assert rss.get("supervisor", 0) > 0


@pytest.mark.parametrize("gpus,want", [
    (1, [(0, "sha256d"), (0, "scrypt")]),
    (2, [(0, "sha256d"), (1, "scrypt")]),
    (8, [(0, "sha256d"), (1, "sha256d"), (2, "sha256d"), (3, "sha256d"),
         (4, "scrypt"), (5, "scrypt"), (6, "scrypt"), (7, "scrypt")]),
])
def test_mixed_pool_layout(gpus, want):
    """BASELINE config 5: both algorithms on GPU 0 at N=1, else the first ceil(N/2) GPUs SHA-256d, the rest scrypt."""
    from otedama_amd.pool.pool_probe import layout

    assert layout(gpus) == want


def test_job_switch_stats_per_rank_and_worst():
    """Node-wide job switch: for each forced block, each rank's first work start after the pool's
    send within the window; worst-rank p50 / max, the node's per-block slowest rank, and missing starts."""
    from otedama_amd.parallel.node_probe import job_switch_stats

    blocks = [10.0, 11.0, 12.0]
    ws = {"rank0": [(1, 10.0005), (2, 11.0004), (3, 12.0006)],
          "rank1": [(1, 10.0020), (2, 11.0030), (3, 12.0010)],
          "rank2": [(1, 10.0010), (3, 12.0200)]}  # missed block 2 (e.g. a lost heartbeat sample)
    js = job_switch_stats(blocks, ws, 3, job_set_at=[(1, 10.0002), (2, 11.0002), (3, 12.0003)],
                          job_bcast_at=[(1, 10.0008)], job_applied={"rank1": [(1, 10.0011)]})
    assert js["blocks"] == 3 and js["missing"] == 1
    r = js["per_rank"]
    assert r["rank0"]["samples"] == 3 and r["rank2"]["samples"] == 2
    assert abs(r["rank1"]["p50_ms"] - 2.0) < 1e-6 and abs(r["rank2"]["max_ms"] - 20.0) < 1e-6
    assert abs(js["worst_rank_max_ms"] - 20.0) < 1e-6 and abs(js["worst_rank_p50_ms"] - 20.0) < 1e-6
    assert abs(js["node_p50_ms"] - 3.0) < 1e-6  # per block slowest: 2.0, 3.0, 20.0
    assert abs(js["pool_to_leader_p50_ms"] - 0.2) < 1e-6 and abs(js["pool_to_r1_done_p50_ms"] - 0.8) < 1e-6
    assert abs(js["pool_to_follower_apply_p50_ms"]["rank1"] - 1.1) < 1e-6
    # a start before the block or after the window is not this block's
    js2 = job_switch_stats([10.0], {"rank0": [(1, 9.9), (2, 13.0)]}, 1)
    assert js2["missing"] == 1 and js2["worst_rank_p50_ms"] is None
