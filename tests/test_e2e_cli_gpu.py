"""SURVEY §7.3 minimum end-to-end slice on a real MI355X, through the real CLI:
`otedama run` (separate process, GPU miner) -> local validating SV2 pool -> accepted shares ->
/metrics shows hashrate, accepted shares and a populated submit-latency p50; SIGTERM exits 0.
"""
import asyncio
import os
import re
import signal
import subprocess
import sys
import threading
import time
import urllib.request
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
ADDR = "bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq"


class _PoolThread:
    def __init__(self, difficulty: float, algorithm: str = "sha256d"):
        from otedama_amd.pool.server import PoolOptions, PoolServer

        self.pool = PoolServer(PoolOptions(algorithm=algorithm, initial_difficulty=difficulty, payout_address=ADDR,
                                           target_share_seconds=0.2, retarget_seconds=5))
        self.loop = asyncio.new_event_loop()
        self.ready = threading.Event()
        self.t = threading.Thread(target=self._run, daemon=True)

    def _run(self):
        asyncio.set_event_loop(self.loop)
        self.loop.run_until_complete(self.pool.start())
        self.ready.set()
        self.loop.run_forever()

    def __enter__(self):
        self.t.start()
        assert self.ready.wait(30)
        return self.pool

    def __exit__(self, *exc):
        asyncio.run_coroutine_threadsafe(self.pool.stop(), self.loop).result(30)
        self.loop.call_soon_threadsafe(self.loop.stop)
        self.t.join(10)


def _metric(body: str, name: str, labels: str = "") -> float | None:
    m = re.search(rf"^{re.escape(name)}{re.escape(labels)} (\S+)$", body, re.M)
    return float(m.group(1)) if m else None


@pytest.mark.gpu
@pytest.mark.parametrize("algorithm,difficulty,min_hashrate,extended", [
    ("sha256d", 0.25, 1e9, False),   # ~16 GH/s per GPU: ~15 shares/s before vardiff settles
    ("scrypt", 16.0, 1e6, False),    # ~16.7 MH/s per GPU, scrypt diff1 = 0xffff << 224: ~16 shares/s
    ("x11", 0.005, 1e8, False),      # ~390 MH/s per GPU, Bitcoin diff1: ~18 shares/s, validated by the pool's CPU chain
    ("sha256d", 0.25, 1e9, True),    # SV2 extended channel: the GPU miner rolls extranonce in the coinbase
])
def test_cli_run_mines_against_local_pool(tmp_path, algorithm, difficulty, min_hashrate, extended):
    with _PoolThread(difficulty, algorithm) as pool:
        cfg = tmp_path / "config.yaml"
        ext = "    sv2_extended_channel: true\n" if extended else ""
        cfg.write_text(f"bitcoin_address: {ADDR}\npools:\n  - url: stratum+v2://{pool.addr_sv2}\n{ext}"
                       f"mining:\n  algorithm: {algorithm}\n  batch_nonces: 134217728\n")
        env = dict(os.environ, HOME=str(tmp_path), PYTHONPATH=str(ROOT), OTEDAMA_DATA_DIR=str(tmp_path / "d"))
        proc = subprocess.Popen([sys.executable, "-m", "otedama_amd", "run", "--config", str(cfg), "--no-tui",
                                 "--http-addr", "127.0.0.1:0", "--gpus", "0"],
                                stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, cwd=ROOT)
        lines, http = [], None
        try:
            deadline = time.time() + 120
            while time.time() < deadline and http is None:
                line = proc.stdout.readline()
                if not line:
                    break
                lines.append(line)
                m = re.search(r"http: listening on (\S+)", line)
                if m:
                    http = m.group(1)
            assert http, "".join(lines)
            threading.Thread(target=lambda: [lines.append(x) for x in proc.stdout], daemon=True).start()
            body = ""
            deadline = time.time() + 60
            while time.time() < deadline:
                time.sleep(2)
                with urllib.request.urlopen(f"http://{http}/metrics", timeout=5) as r:
                    body = r.read().decode()
                acc = _metric(body, "otedama_shares_total", '{status="accepted"}') or 0
                p50 = _metric(body, "otedama_submit_latency_milliseconds", '{quantile="0.5"}') or 0
                hr = _metric(body, "otedama_hashrate_hashes_per_second") or 0
                if acc >= 10 and p50 > 0 and hr > min_hashrate:
                    break
            assert acc >= 10 and p50 > 0, body + "".join(lines[-40:])
            assert hr > min_hashrate, f"hashrate {hr}"
            with urllib.request.urlopen(f"http://{http}/readyz", timeout=5) as r:
                assert r.status == 200
            assert pool.m_accepted.value() >= acc  # every engine-side accept was validated by the pool
        finally:
            proc.send_signal(signal.SIGTERM)
            try:
                rc = proc.wait(60)
            except subprocess.TimeoutExpired:
                proc.kill()
                rc = proc.wait(10)
        assert rc == 0, "".join(lines[-40:])


@pytest.mark.gpu
def test_cli_node_mode_two_ranks_share_one_gpu(tmp_path):
    """torchrun node mode through the real CLI: rank 0 runs the engine (pool session, HTTP), rank 1 a NodeWorker;
    on this 1-GPU box both ranks hash disjoint variant stripes on GPU 0 and talk over gloo (an 8-GPU node uses
    RCCL, one GPU per rank). Rank 1's shares reach the pool through rank 0 (R2) and are accepted."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    with _PoolThread(0.25, "sha256d") as pool:
        cfg = tmp_path / "config.yaml"
        cfg.write_text(f"bitcoin_address: {ADDR}\npools:\n  - url: stratum+v2://{pool.addr_sv2}\n"
                       f"mining:\n  batch_nonces: 134217728\n")
        env = dict(os.environ, HOME=str(tmp_path), PYTHONPATH=str(ROOT), OTEDAMA_DATA_DIR=str(tmp_path / "d"),
                   OTEDAMA_DIST_BACKEND="gloo")
        proc = subprocess.Popen([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                                 "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "otedama_amd", "run",
                                 "--config", str(cfg), "--no-tui", "--http-addr", "127.0.0.1:0"],
                                stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env, cwd=ROOT,
                                start_new_session=True)
        lines, http = [], None
        try:
            deadline = time.time() + 150
            while time.time() < deadline and http is None:
                line = proc.stdout.readline()
                if not line:
                    break
                lines.append(line)
                m = re.search(r"http: listening on (\S+)", line)
                if m:
                    http = m.group(1)
            assert http, "".join(lines)
            threading.Thread(target=lambda: [lines.append(x) for x in proc.stdout], daemon=True).start()
            body, rank1 = "", 0
            deadline = time.time() + 60
            while time.time() < deadline:
                time.sleep(2)
                with urllib.request.urlopen(f"http://{http}/metrics", timeout=5) as r:
                    body = r.read().decode()
                acc = _metric(body, "otedama_shares_total", '{status="accepted"}') or 0
                rank1 = _metric(body, "otedama_device_shares_found_total", '{device="rank1"}') or 0
                if acc >= 10 and rank1 >= 2:
                    break
            assert acc >= 10 and rank1 >= 2, body + "".join(lines[-40:])
            assert any("node: rank 1 of 2 mining on GPU 0 (1 device(s))" in x for x in lines), "".join(lines[-40:])
            assert pool.m_accepted.value() >= acc
        finally:
            os.killpg(proc.pid, signal.SIGTERM)
            try:
                proc.wait(60)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
                proc.wait(10)
