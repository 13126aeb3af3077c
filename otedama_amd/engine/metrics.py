"""The engine's otedama_* metric bundle.

Parity: internal/engine/metrics.go:22-581 — every series name, type and label
set is kept so existing dashboards and alerts keep working; lazily created
label sets (reject reason, per-device shares, payout info, last reject) are
bounded exactly as there. MI355X additions are per-device series
(otedama_device_hashrate_hashes_per_second{device}, otedama_device_busy_ratio{device},
otedama_device_kernel_launches_total{device}), the node's collective tick (otedama_node_*) and the
local-pool series in otedama_amd.pool.server. docs/METRICS.md lists every name
(enforced by tests/test_metrics_doc.py, the analogue of metrics_doc_test.go).
"""
from __future__ import annotations

import threading

from otedama_amd import version as _version
from otedama_amd.engine.stats import REJECT_CATEGORIES, acceptance_rate
from otedama_amd.metrics import Registry


class EngineMetrics:
    def __init__(self, reg: Registry):
        self.reg = reg
        C, G = reg.new_counter, reg.new_gauge
        self.hashrate = G("otedama_hashrate_hashes_per_second", "Current aggregate hashrate in hashes per second.")
        self.shares_found = C("otedama_shares_found_total", "Total shares found locally by all workers.")
        self.shares_submitted = C("otedama_shares_submitted_total",
                                  "Total shares actually transmitted to the pool (mining.submit / "
                                  "SubmitSharesStandard), incremented at send time regardless of the verdict.")
        self.shares_accepted = C("otedama_shares_total", "Total shares reported by the pool.", {"status": "accepted"})
        self.shares_rejected = C("otedama_shares_total", "Total shares reported by the pool.", {"status": "rejected"})
        self.pool_connect_attempts = C("otedama_pool_connect_attempts_total",
                                       "Total pool-connection attempts, including reconnects.")
        self.pool_connect_failures = C("otedama_pool_connect_failures_total", "Total pool-connection failures.")
        self.arbitration_switches = C("otedama_arbitration_switches_total",
                                      "Total arbitration workload switches (mining <-> AI).")
        self.arbitration_holds = C("otedama_arbitration_holds_total",
                                   "Total decisions where a higher-yielding stream existed but hysteresis kept the "
                                   "current assignment.")
        self.arbitration_foregone = G("otedama_arbitration_foregone_sats_per_second",
                                      "Instantaneous opportunity cost of the current allocation: raw sats/s left on "
                                      "the table by hysteresis holds.")
        self.arbitration_expected_yield = G("otedama_arbitration_expected_yield_sats_per_second",
                                            "The engine's forecast earning rate: summed ExpectedYield of the chosen "
                                            "assignments.")
        self.effective_yield = G("otedama_effective_yield_sats_per_second",
                                 "Gross-minus-losses yield: otedama_arbitration_expected_yield_sats_per_second "
                                 "scaled by the productive fraction of uptime.")
        self.active_streams = G("otedama_active_streams",
                                "Number of live revenue streams in arbitration after pruning stale providers.")
        self.devices_idle = G("otedama_devices_idle",
                              "Number of devices left idle this arbitration cycle (no compatible stream above the "
                              "yield floor).")
        self.devices_active = G("otedama_devices_active",
                                "Local devices hashing: not retired after a fault and not stalled.")
        self.devices_faulted = G("otedama_devices_faulted",
                                 "Devices whose miner thread died on a HIP error (retired; survivors re-split "
                                 "their search stripe at the next job).")
        self.devices_stalled = G("otedama_devices_stalled",
                                 "Live devices with work assigned whose hash counter stopped advancing for "
                                 "several stats ticks.")
        self.btc_usd_rate = G("otedama_btc_usd_rate", "Current BTC/USD rate from provider consensus.")
        self.uptime = G("otedama_uptime_seconds", "Seconds since engine start.")
        self.start_time = G("otedama_start_time_seconds", "Unix timestamp at which engine started.")
        lat_help = "Share-submission round-trip latency (submit->accept)."
        self.submit_latency_p50 = G("otedama_submit_latency_milliseconds", lat_help, {"quantile": "0.5"})
        self.submit_latency_p95 = G("otedama_submit_latency_milliseconds", lat_help, {"quantile": "0.95"})
        self.submit_latency_p99 = G("otedama_submit_latency_milliseconds", lat_help, {"quantile": "0.99"})
        hit_help = ("Device hit -> pool accept latency: from the kernel's own hit time (s_memrealtime mapped to the "
                    "host clock) to the pool's acceptance.")
        self.hit_latency_p50 = G("otedama_share_hit_to_accept_milliseconds", hit_help, {"quantile": "0.5"})
        self.hit_latency_p95 = G("otedama_share_hit_to_accept_milliseconds", hit_help, {"quantile": "0.95"})
        self.hit_latency_p99 = G("otedama_share_hit_to_accept_milliseconds", hit_help, {"quantile": "0.99"})
        self.job_switch_ms = G("otedama_job_switch_milliseconds",
                               "Most recent work switch on a GPU: new work handed to the device -> the first batch "
                               "of it running (obsolete batches stop at the device abort word). Max over devices.")
        self.share_acceptance_rate = G("otedama_share_acceptance_rate",
                                       "Accepted shares / total judged shares (1.0 = all accepted).")
        self.shares_unaccounted = G("otedama_shares_unaccounted",
                                    "Shares found locally but not yet judged by the pool (found - accepted - "
                                    "rejected).")
        self.productive_seconds = C("otedama_productive_seconds_total",
                                    "Cumulative wall-clock seconds the miner actually produced hashrate.")
        self.reject_rate = G("otedama_reject_rate",
                             "Rejected shares / total judged shares (complement of acceptance_rate).")
        self.stale_rate = G("otedama_stale_rate",
                            "Stale-rejected shares / total judged shares. High values indicate network latency or "
                            "a pool that is too far away.")
        self.up = G("otedama_up", "1 when the engine is hashing (or intentionally curtailed), 0 when stalled.")
        self.curtailed = G("otedama_curtailed", "1 while mining is paused by the BTC/USD curtailment rule.")
        self.power_watts = G("otedama_power_watts",
                             "Configured total system power draw in watts (from power_watts config). 0 when not set.")
        self.joules_per_terahash = G("otedama_joules_per_terahash",
                                     "Energy efficiency: watts x 1e12 / hashrate. 0 when power_watts is not "
                                     "configured.")
        self.power_cost_usd_per_hour = G("otedama_power_cost_usd_per_hour",
                                         "Estimated electricity cost: power_watts/1000 x electricity_price_per_kwh.")
        self.pool_connection_state = G("otedama_pool_connection_state",
                                       "Pool connection state: 0=disconnected, 1=connecting, 2=connected.")
        self.pool_active_index = G("otedama_pool_active_index", "Index of the pool currently in use (0-based).")
        self.payout_active_index = G("otedama_payout_active_index",
                                     "Index of the payout address currently in use (0-based).")
        info = _version.get()
        G("otedama_build_info", "Build information (constant 1); version/commit/goversion are labels.",
          {"version": info.version, "commit": info.commit, "goversion": "python" + info.python_version}).set(1)
        self.last_job_received = G("otedama_last_job_received_seconds",
                                   "Unix timestamp of the most recent mining job received from the pool.")
        self.clock_skew_seconds = G("otedama_clock_skew_seconds",
                                    "Maximum absolute offset (s) between the local system clock and the price "
                                    "sources' HTTP Date headers.")
        self.btc_rate_age_seconds = G("otedama_btc_rate_age_seconds",
                                      "Seconds since the BTC/USD rate was last successfully fetched.")
        self.rate_sources_ok = G("otedama_rate_sources_ok",
                                 "Number of BTC/USD price sources that returned a usable in-band reading.")
        self.rate_sources_total = G("otedama_rate_sources_total",
                                    "Number of BTC/USD price sources configured. The denominator for "
                                    "otedama_rate_sources_ok.")
        self.pool_difficulty = G("otedama_pool_difficulty", "Current share difficulty assigned by the pool.")
        self.estimated_share_interval_seconds = G("otedama_estimated_share_interval_seconds",
                                                  "Expected wall-clock seconds between consecutive shares: "
                                                  "difficulty x 2^32 / hashrate.")
        self.stale_skipped = C("otedama_shares_stale_skipped_total",
                               "Shares found for a job the pool already invalidated (not submitted).")
        self.below_target_skipped = C("otedama_shares_below_target_skipped_total",
                                      "Shares found under a share target the pool has since raised (SV2 SetTarget "
                                      "re-issues the job; not submitted, the pool would reject them).")
        self.node_collective_seconds = G("otedama_node_collective_seconds",
                                         "Multi-GPU node: median wall time of rank 0's node ops (R1 job broadcast, R2 "
                                         "share gather, R3 counters, re-forms); 0 outside node mode.")
        self.node_collective_p99 = G("otedama_node_collective_p99_seconds",
                                     "Multi-GPU node: 99th-percentile wall time of rank 0's node ops.")
        self.node_collectives = G("otedama_node_device_collectives",
                                  "Multi-GPU node: device collectives (RCCL) issued by rank 0 since start.")
        self.node_ranks = G("otedama_node_ranks", "Multi-GPU node: ranks (one per GPU) in the torchrun job; 1 when "
                                                  "running standalone.")
        self.node_ranks.set(1)
        self.node_generation = G("otedama_node_generation",
                                 "Multi-GPU node: process-group generation (each re-form after a lost or rejoining "
                                 "rank starts the next one); 0 outside node mode.")
        self.node_lost_ranks = G("otedama_node_lost_ranks",
                                 "Multi-GPU node: ranks currently out of the node (lost, not yet re-admitted).")
        self.node_share_previews = G("otedama_node_share_previews",
                                     "Multi-GPU node: remote shares the leader admitted from a follower's preview "
                                     "datagram, ahead of the R2 gather, since start.")
        self.node_remote_stale = G("otedama_node_remote_stale_shares",
                                   "Multi-GPU node: remote shares of a job the leader no longer knows (dropped).")
        self._lock = threading.Lock()
        self._reject_reason: dict[str, object] = {}
        self._last_reject: dict[str, object] = {}
        self._device_found: dict[str, object] = {}
        self._device_hashrate: dict[str, object] = {}
        self._device_busy: dict[str, object] = {}
        self._device_launches: dict[str, object] = {}
        self._device_lost: dict[tuple[str, str], object] = {}
        self._payout_info: dict[str, object] = {}

    def reject_reason(self, category: str):
        if category not in REJECT_CATEGORIES:
            category = "other"
        with self._lock:
            c = self._reject_reason.get(category)
            if c is None:
                c = self.reg.new_counter("otedama_shares_rejected_by_reason_total",
                                         "Rejected shares broken down by inferred root cause.", {"reason": category})
                self._reject_reason[category] = c
            return c

    def touch_last_reject(self, category: str, unix: float) -> None:
        if category not in REJECT_CATEGORIES:
            category = "other"
        with self._lock:
            g = self._last_reject.get(category)
            if g is None:
                g = self.reg.new_gauge("otedama_last_reject_seconds",
                                       "Unix timestamp of the most recent share rejection of this category.",
                                       {"reason": category})
                self._last_reject[category] = g
        g.set(unix)

    def inc_shares_found_for_device(self, device: str) -> None:
        if not device:
            return
        with self._lock:
            c = self._device_found.get(device)
            if c is None:
                if len(self._device_found) >= 64:  # bounded label set
                    return
                c = self.reg.new_counter("otedama_device_shares_found_total",
                                         "Total shares found by this device. Per-device breakdown of "
                                         "otedama_shares_found_total.", {"device": device})
                self._device_found[device] = c
        c.inc()

    def set_device_hashrate(self, device: str, hps: float) -> None:
        with self._lock:
            g = self._device_hashrate.get(device)
            if g is None:
                if len(self._device_hashrate) >= 64:
                    return
                g = self.reg.new_gauge("otedama_device_hashrate_hashes_per_second",
                                       "Per-device hashrate (GPU kernel or CPU threads).", {"device": device})
                self._device_hashrate[device] = g
        g.set(hps)

    def set_device_busy(self, device: str, ratio: float) -> None:
        with self._lock:
            g = self._device_busy.get(device)
            if g is None:
                if len(self._device_busy) >= 64:
                    return
                g = self.reg.new_gauge("otedama_device_busy_ratio",
                                       "Fraction of the last stats interval the device spent executing search "
                                       "kernels (GPU: HIP event time of its launches; CPU: thread time / threads).",
                                       {"device": device})
                self._device_busy[device] = g
        g.set(ratio)

    def add_device_launches(self, device: str, n: int) -> None:
        if n <= 0:
            return
        with self._lock:
            c = self._device_launches.get(device)
            if c is None:
                if len(self._device_launches) >= 64:
                    return
                c = self.reg.new_counter("otedama_device_kernel_launches_total",
                                         "Search-kernel launches (batches) completed by the device.", {"device": device})
                self._device_launches[device] = c
        c.add(n)

    def add_device_candidates_lost(self, device: str, reason: str, n: int) -> None:
        """Candidates a device found but never queued as shares: ``ring_overflow`` (past a launch's hit-ring
        capacity) or ``verify_queue_full`` (scrypt host-verifier queue bound)."""
        if n <= 0:
            return
        with self._lock:
            c = self._device_lost.get((device, reason))
            if c is None:
                if len(self._device_lost) >= 128:
                    return
                c = self.reg.new_counter("otedama_device_candidates_lost_total",
                                         "Kernel candidates lost before host verification, by cause (ring_overflow: "
                                         "more hits than a launch's hit ring holds; verify_queue_full: scrypt "
                                         "verifier queue at its bound).", {"device": device, "reason": reason})
                self._device_lost[(device, reason)] = c
        c.add(n)

    def set_active_payout(self, masked: str) -> None:
        if not masked:  # metrics.go:513: an empty address never creates a series
            return
        with self._lock:
            for addr, g in self._payout_info.items():
                g.set(1 if addr == masked else 0)
            if masked not in self._payout_info:
                g = self.reg.new_gauge("otedama_payout_info",
                                       "Active payout destination (masked). The series valued 1 is the address "
                                       "currently mined to.", {"address": masked})
                g.set(1)
                self._payout_info[masked] = g

    def update_share_rates(self) -> tuple[float, int]:
        acc, rej = self.shares_accepted.value(), self.shares_rejected.value()
        judged = acc + rej
        rate = acceptance_rate(acc, rej)
        self.share_acceptance_rate.set(rate)
        self.reject_rate.set(0.0 if judged == 0 else rej / judged)
        stale = self._reject_reason.get("stale")
        self.stale_rate.set(0.0 if judged == 0 or stale is None else stale.value() / judged)
        self.shares_unaccounted.set(max(self.shares_found.value() - judged, 0))
        return rate, judged
