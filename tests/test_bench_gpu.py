"""bench.py's multi-rank GPU path on the one-GPU box: two ranks share GPU 0 over gloo (OTEDAMA_DIST_BACKEND=gloo).

The driver's 8-GPU run uses RCCL with one GPU per rank; everything else of that run (the launcher, the rank guard,
the kernel sections with their R1 / R2 / R3, the hit re-verification, the JSON and its summary) runs here on the
real kernels, so a multi-rank bug in the GPU code path shows up before that run.
"""
import os
import subprocess
import sys
import tempfile

import pytest

from benchjson import detail_env, result

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_bench_two_ranks_share_the_gpu_over_gloo():
    denv, detail = detail_env(tempfile.mkdtemp(prefix="otd-bench-"))
    env = dict(os.environ, OTEDAMA_DIST_BACKEND="gloo", **denv)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    res = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                          "--single-midstate-headers", "1", "--scrypt-steps", "2", "--x11-steps", "2",
                          "--miner-seconds", "0", "--no-latency", "--cpu-seconds", "0", "--node-seconds", "0",
                          "--pool-seconds", "0"], capture_output=True, text=True, timeout=220, env=env, cwd=ROOT)
    assert res.returncode == 0, res.stderr[-4000:]
    d = result(res, detail)
    assert d["n_gpus"] == 2 and d["rehearsal"] == "gloo-shared-gpu" and d["rccl_ranks_seen"] == [0, 1]
    assert d["value"] > 1e10 and len(d["per_rank_hashes_per_sec"]) == 2
    assert d["hits_verified"] == d["hits_found"] > 0 and d["hits_duplicate"] == 0 and d["hits_outside_window"] == 0
    assert d["hits_r2_gathered"] == d["hits_found"]
    assert d["scrypt"]["hits_verified"] == d["scrypt"]["hits_checked"] > 0
    assert d["x11"]["hits_verified"] == d["x11"]["hits_found"] > 0
    assert d["errors"] is None and all(v["status"] == "ok" for v in d["sections"].values()), d["sections"]
    assert list(d)[-1] == "summary" and d["summary"]["cfg2_version_rolled_hps"] > 1e10 and d["summary"]["world_size"] == 2
