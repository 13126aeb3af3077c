"""bench.py always reports: a stuck rank, a stuck section or a dead rank 0 must still
end in one well-formed JSON line inside the deadline, never in a silent timeout.

The CPU rehearsal (gloo + the native CPU scanner) runs the real launcher, rank guard and sections; the fault hook
OTEDAMA_BENCH_FAULT=stuck:<rank>:<section> hangs one rank at the start of one section (parallel/guard.py).
Reference rule: nothing in the engine waits without a deadline (internal/engine/run.go:1251).
"""
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import pytest

from benchjson import detail_env, result

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "OTEDAMA_BENCH_FAULT"):
        e.pop(k, None)
    e.update(extra)
    return e


def _bench(*args, env=None, timeout=240):
    t0 = time.monotonic()
    denv, detail = detail_env(tempfile.mkdtemp(prefix="otd-bench-"))
    res = subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout,
                         env=_env(**denv, **(env or {})), cwd=ROOT)
    res.detail = detail
    return res, time.monotonic() - t0


def _json(res) -> dict:
    return result(res, res.detail)


@pytest.mark.timeout(300)
def test_world8_stuck_rank_in_preflight_prints_an_error_json():
    """A rank that never reaches the rendezvous: rank 0 reports at the pre-flight deadline with every rank's phase
    and stderr tail, stops the others, and exits non-zero."""
    res, took = _bench("--gpus", "8", "--steps", "2", "--warmup", "1", "--cpu-rehearsal", "--cpu-seconds", "0",
                       "--preflight-timeout", "25", env={"OTEDAMA_BENCH_FAULT": "stuck:3:preflight"}, timeout=200)
    assert res.returncode != 0
    d = _json(res)
    assert d["value"] is None and d["n_gpus"] == 8
    assert "preflight" in d["error"] or "preflight" in json.dumps(d["errors"])
    diag = d["diagnosis"]
    assert diag["world_size"] == 8 and set(diag["ranks_checked_in"]) == set(range(8))
    assert diag["ranks"]["3"]["phase"] == "section:preflight"  # never got past the start of the pre-flight
    assert all(diag["ranks"][str(r)]["phase"] in ("rendezvous", "first-collective", "exit:stopped by rank 0")
               or diag["ranks"][str(r)]["phase"].startswith("exit") for r in (1, 2, 4, 5, 6, 7))
    assert d["error"].startswith(d["summary"]["error"]) and list(d)[-1] == "summary"
    assert took < 120, took


@pytest.mark.timeout(300)
def test_stuck_node_section_keeps_the_full_json():
    """Rank 0 hangs in the node section: the section records its timeout and every earlier result is printed."""
    res, took = _bench("--gpus", "2", "--steps", "2", "--warmup", "1", "--cpu-rehearsal", "--cpu-seconds", "0.3",
                       "--node-seconds", "3", "--section-timeouts", "node=12",
                       env={"OTEDAMA_BENCH_FAULT": "stuck:0:node"}, timeout=200)
    assert res.returncode == 0, res.stderr[-3000:]
    d = _json(res)
    assert d["value"] > 0 and d["n_gpus"] == 2 and d["rccl_ranks_seen"] == [0, 1]
    assert d["errors"]["node"] == "timeout after 12 s"
    assert d["sections"]["node"]["status"] == "timeout" and d["sections"]["cpu"]["status"] == "ok"
    assert d["cpu_single_thread_hashes_per_sec"] > 0
    s = d["summary"]
    assert list(d)[-1] == "summary" and s["errors"]["node"] == "timeout after 12 s" and s["cfg2_version_rolled_hps"] > 0
    assert took < 100, took


@pytest.mark.timeout(300)
def test_dead_rank0_still_gets_a_json_from_the_launcher():
    """Rank 0 dies before it can print: the launcher prints the error JSON with the ranks' diagnosis."""
    res, _ = _bench("--gpus", "2", "--steps", "1", "--warmup", "0", "--cpu-rehearsal", "--cpu-seconds", "0",
                    env={"OTEDAMA_BENCH_FAULT": "exit:0:sha256d"}, timeout=200)
    assert res.returncode != 0
    d = _json(res)
    assert d["value"] is None and "rank 0 printed no result" in d["error"]
    assert d["diagnosis"]["ranks_checked_in"] == [0, 1]


@pytest.mark.timeout(300)
def test_torchrun_stuck_follower_in_the_headline():
    """The driver's torchrun command line with a follower stuck in the headline section: rank 0 (blocked in a
    collective with it) reports at the section deadline, and torchrun's job ends instead of hanging."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    denv = detail_env(tempfile.mkdtemp(prefix="otd-bench-"))[0]
    t0 = time.monotonic()
    res = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), BENCH, "--gpus", "2",
                          "--steps", "2", "--warmup", "1", "--cpu-rehearsal", "--cpu-seconds", "0",
                          "--section-timeouts", "sha256d=15"],
                         capture_output=True, text=True, timeout=240,
                         env=_env(OTEDAMA_BENCH_FAULT="stuck:1:sha256d", **denv), cwd=ROOT)
    res.detail = denv["OTEDAMA_BENCH_DETAIL"]
    took = time.monotonic() - t0
    d = _json(res)
    assert d["value"] is None and "sha256d" in json.dumps(d["errors"])
    assert d["diagnosis"]["ranks"]["1"]["phase"] == "section:sha256d"
    assert took < 120, took


def test_run_ranks_deadline_stops_hung_ranks():
    from otedama_amd.parallel.launch import run_ranks

    t0 = time.monotonic()
    rc = run_ranks([sys.executable, "-c", "import time; time.sleep(120)"], 2, deadline=2.0)
    assert rc == 124 and time.monotonic() - t0 < 30


def test_run_ranks_forwards_rank0_lines():
    from otedama_amd.parallel.launch import run_ranks

    seen = []
    rc = run_ranks([sys.executable, "-c", "import os; print('{\"metric\": %s}' % os.environ['RANK'])"], 2,
                   on_rank0_line=seen.append)
    assert rc == 0 and seen == ['{"metric": 0}\n']


# ------------------------------------------------------------------ unit level
def test_fault_spec_parsing():
    from otedama_amd.parallel.guard import fault_for

    env = {"OTEDAMA_BENCH_FAULT": "stuck:3:preflight, exit:0:node,bogus,stuck:x:y"}
    assert fault_for(3, "preflight", env) == "stuck"
    assert fault_for(0, "node", env) == "exit"
    assert fault_for(1, "preflight", env) is None and fault_for(3, "node", env) is None


def test_guard_section_timeout_emits_once(tmp_path):
    """In-process: a section that overruns calls emit with the section's error (the exit is stubbed out)."""
    from otedama_amd.parallel import guard as G

    calls = []

    class Stop(Exception):
        pass

    g = G.RankGuard(0, 1, deadline_s=60, emit=lambda errors, reason: calls.append((errors, reason)) or 0,
                    run_dir=str(tmp_path), poll_s=0.05)
    left = []
    g._leave = lambda code, why: left.append(code)
    g.stop_children = lambda grace=5.0: None
    g.start()
    with g.section("fast", 5):
        pass
    with g.section("slow", 0.2):
        time.sleep(1.0)
    assert len(calls) == 1 and calls[0][0]["slow"] == "timeout after 0 s" and left == [0]
    assert g.sections["fast"]["status"] == "ok" and g.sections["slow"]["status"] == "timeout"
    assert g.finish() is False  # fired first: the main thread must not print a second line


def test_guard_records_section_errors_and_finish_blocks_firing(tmp_path):
    from otedama_amd.parallel import guard as G

    g = G.RankGuard(0, 1, deadline_s=60, emit=lambda e, r: 0, run_dir=str(tmp_path), poll_s=0.05)
    with g.section("broken", 5):
        raise ValueError("boom")
    assert g.errors["broken"] == "ValueError: boom" and g.sections["broken"]["status"] == "error"
    with pytest.raises(KeyError):
        with g.section("critical", 5, critical=True):
            raise KeyError("x")
    assert g.finish() is True
    st = json.loads((tmp_path / "rank0.json").read_text())
    assert st["exited"] is True and st["phase"] == "done"


def test_diagnose_ignores_stale_status_files(tmp_path):
    from otedama_amd.parallel import guard as G

    (tmp_path / "rank1.json").write_text(json.dumps({"rank": 1, "t_start": time.time() - 3600, "pid": 1}))
    (tmp_path / "rank0.json").write_text(json.dumps({"rank": 0, "t_start": time.time(), "pid": os.getpid(),
                                                     "phase": "rendezvous", "t_wall": time.time()}))
    (tmp_path / "rank0.stderr").write_text("x" * 2000 + "the last words")
    d = G.diagnose_run_dir(str(tmp_path), 2, time.time())
    assert d["ranks_checked_in"] == [0] and d["ranks"]["1"]["checked_in"] is False
    assert d["ranks"]["0"]["stderr_tail"].endswith("the last words") and len(d["ranks"]["0"]["stderr_tail"]) <= 600


@pytest.mark.timeout(300)
@pytest.mark.parametrize("fault", ["", "fail:2:probe", "hang:1:probe", "fail:3:native"])
def test_data_plane_probe_falls_back_together_and_still_measures(fault):
    """The pre-flight's data-plane probe (parallel/rccl_probe.py): every rank checks in a child process that the
    native RCCL module forms a group of all ranks and an all_reduce completes, under a deadline; rank 0 publishes one
    decision. All ok: the bench's R1 / R2 / R3 run on the native module (``impl: rccl-native``). If any rank's check
    fails or hangs, or one rank's in-process init fails after a good probe, every rank runs the bench over gloo
    together and the headline is still measured. Rehearsed with the module's CPU stand-in (tests/loopback_rccl.py)."""
    env = {"OTEDAMA_RCCL_MODULE": "loopback_rccl", "PYTHONPATH": os.path.join(ROOT, "tests"),
           "OTEDAMA_PROBE_TIMEOUT": "8"}
    if fault:
        env["OTEDAMA_BENCH_FAULT"] = fault
    res, took = _bench("--gpus", "4", "--steps", "2", "--warmup", "1", "--cpu-rehearsal", "--cpu-seconds", "0",
                       "--comm-ops", "20", env=env, timeout=240)
    assert res.returncode == 0, res.stderr[-3000:]
    d = _json(res)
    dp = d["preflight"]["data_plane"]
    assert d["value"] and d["value"] > 0 and d["hits_r2_gathered"] == d["hits_found"] > 0
    native = fault == ""
    assert dp["impl"] == ("rccl-native" if native else "gloo") == d.line["summary"]["data_plane"], dp
    assert (d.line["summary"]["data_plane_note"] is None) is native
    assert dp["backend"] == ("rccl" if native else "gloo")
    assert dp["probe"]["ok"] is (not fault.endswith(":probe")), dp
    assert d["comm"]["idle"]["R2"]["samples"] == 20 and d["comm"]["busbw"]["blocks_ok"]
    if fault.endswith(":probe"):
        bad = fault.split(":")[1]
        assert not dp["probe"]["ranks"][bad]["ok"]
        assert ("injected" if fault.startswith("fail") else "killed") in dp["probe"]["ranks"][bad]["reason"]
        # the group needs every rank: the others' children waited for it until their deadline
        assert all(v["ok"] is False for v in dp["probe"]["ranks"].values()), dp
    elif fault:
        assert "3" in dp["native_error"] or "injected" in dp["native_error"], dp


@pytest.mark.timeout(300)
def test_probe_with_default_deadlines_fits_the_preflight_under_skew_and_a_hang():
    """the probe's deadlines come from the pre-flight budget (no OTEDAMA_PROBE_TIMEOUT override here). One
    rank reaches the probe 25 s late (a cold-start skew past the derived arrival wait) and another rank's child hangs:
    the probe still decides inside the pre-flight, every rank falls back to gloo together, and the headline is
    measured. --preflight-timeout 90 keeps the test short; the derivation is the same as at the default 240 s."""
    env = {"OTEDAMA_RCCL_MODULE": "loopback_rccl", "PYTHONPATH": os.path.join(ROOT, "tests"),
           "OTEDAMA_BENCH_FAULT": "slow:2:arrive,hang:1:probe", "OTEDAMA_FAULT_SLOW_S": "25"}
    res, took = _bench("--gpus", "4", "--steps", "2", "--warmup", "1", "--cpu-rehearsal", "--cpu-seconds", "0",
                       "--comm-ops", "10", "--preflight-timeout", "90", env=env, timeout=280)
    assert res.returncode == 0, res.stderr[-3000:]
    d = _json(res)
    dp = d["preflight"]["data_plane"]
    assert d["value"] > 0 and dp["impl"] == "gloo" and not dp["probe"]["ok"], dp
    a, t, v = dp["probe"]["deadlines_s"]
    assert a + t + v <= 90.0 - 40.0 + 1.0, dp["probe"]  # inside the budget minus the fallback's reserve
    assert d["sections"]["preflight"]["status"] == "ok" and d["sections"]["preflight"]["s"] < 90.0
    assert "killed" in dp["probe"]["ranks"]["1"]["reason"]


@pytest.mark.timeout(300)
def test_a_rank_stuck_in_the_comm_section_costs_only_that_section():
    """The comm section is the last one every rank takes part in, and its collectives are bounded: when one rank
    never joins, the others' ops raise (CollectiveTimeout) well inside the section's budget. The section is recorded
    as an error, and rank 0 goes on with its own sections (here the CPU miner) and prints the full line. Rehearsed on
    the native data plane's CPU stand-in."""
    env = {"OTEDAMA_RCCL_MODULE": "loopback_rccl", "PYTHONPATH": os.path.join(ROOT, "tests"),
           "OTEDAMA_BENCH_FAULT": "stuck:2:comm"}
    res, took = _bench("--gpus", "4", "--steps", "2", "--warmup", "1", "--cpu-rehearsal", "--cpu-seconds", "0.3",
                       "--comm-ops", "10", "--section-timeouts", "comm=24", env=env, timeout=280)
    assert res.returncode == 0, res.stderr[-3000:]
    d = _json(res)
    assert d["value"] > 0 and d.line["summary"]["data_plane"] == "rccl-native"
    assert d["sections"]["comm"]["status"] == "error" and "comm" in d["errors"], d["sections"]
    assert d["sections"]["cpu"]["status"] == "ok" and d["cpu_single_thread_hashes_per_sec"] > 0


@pytest.mark.timeout(300)
def test_a_failed_headline_section_prints_a_capped_error_line():
    """bench.fail(): the headline section raises on rank 0 (not a hang) at world 8. Rank 0 prints the error line
    under the driver's cap, with the section's error in ``summary``, stops its peers and exits non-zero."""
    res, took = _bench("--gpus", "8", "--steps", "2", "--warmup", "1", "--cpu-rehearsal", "--cpu-seconds", "0",
                       "--comm-ops", "0", env={"OTEDAMA_BENCH_FAULT": "fail:0:sha256d"}, timeout=240)
    assert res.returncode != 0
    d = _json(res)
    assert d["value"] is None and "injected failure in section sha256d" in d["error"]
    assert "sha256d" in d.line["summary"]["errors"]
    assert took < 150, took
