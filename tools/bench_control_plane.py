"""Control-plane microbenchmarks against the reference's secondary published numbers.

* SV2 header decode / 1 KB full-frame decode: the native scanner (``tools/bench_sv2.cpp``, built here with g++)
  and the Python ``FrameScanner`` end to end (Frame objects included).
* ``/metrics`` text render with 200 labelled series (reference CHANGELOG.md:1654-1657: 1.12 ms/op).
* Startup: wall time of ``otedama version`` and ``otedama config validate`` in a fresh interpreter, and the RSS
  of the imported control plane.

Usage: ``python tools/bench_control_plane.py [--out profiles/r1/control_plane.json]``. CPU only.
"""
from __future__ import annotations

import argparse
import io
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def native_frames() -> dict:
    exe = Path("/tmp/otedama_bench_sv2")
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{ROOT / 'csrc/include'}", str(ROOT / "tools/bench_sv2.cpp"),
                    str(ROOT / "csrc/cpu/sv2_frame.cpp"), "-o", str(exe)], check=True)
    out = json.loads(subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout)
    out.pop("sink", None)
    return out


def python_frames() -> dict:
    from otedama_amd.stratum.frame import Frame, FrameScanner, Header, decode_header, encode_frame

    res = {}
    for name, size, n in (("header", 4, 200_000), ("full1k", 1024, 50_000)):
        raw = b"".join(encode_frame(Frame(Header(0, 0x15, size), bytes(size))) for _ in range(n))
        best = 1e9
        for _ in range(3):
            sc = FrameScanner()
            t0 = time.perf_counter()
            for off in range(0, len(raw), 1 << 16):  # 64 KiB socket reads
                sc.feed(raw[off:off + (1 << 16)])
            best = min(best, (time.perf_counter() - t0) / n)
        res[f"scanner_{name}_ns"] = round(best * 1e9, 1)
    hdr = encode_frame(Frame(Header(0, 0x15, 4), bytes(4)))[:6]
    t0 = time.perf_counter()
    for _ in range(200_000):
        decode_header(hdr)
    res["decode_header_py_ns"] = round((time.perf_counter() - t0) / 200_000 * 1e9, 1)
    return res


def metrics_render() -> dict:
    from otedama_amd import metrics as M

    reg = M.Registry()
    gs = [reg.new_gauge("otedama_bench_series", "bench", {"device": f"gpu-{i}"}) for i in range(200)]
    for i, g in enumerate(gs):
        g.set(i * 1.5)
    buf = io.StringIO()
    reg.write_text(buf)
    res = {"series": 200, "bytes": len(buf.getvalue())}
    for name, changing in (("ms_per_render_static", False), ("ms_per_render_all_changed", True)):
        n, best = 200, 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            for k in range(n):
                if changing:  # every series gets a new value before each scrape (worst case)
                    for i, g in enumerate(gs):
                        g.set(k + i * 1.37e-3)
                reg.write_text(io.StringIO())
            best = min(best, (time.perf_counter() - t0) / n)
        res[name] = round(best * 1e3, 3)
    return res


def startup() -> dict:
    env = dict(os.environ, OTEDAMA_NO_AUTOBUILD="1")
    res = {}
    for name, args in (("version_s", ["version"]), ("config_validate_s", ["config", "validate"])):
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            subprocess.run([sys.executable, "-m", "otedama_amd", *args], cwd=ROOT, env=env, capture_output=True)
            best = min(best, time.perf_counter() - t0)
        res[name] = round(best, 3)
    first = ("import time; from otedama_amd.models.header import GENESIS_HEADER_HEX;"
             "from otedama_amd.ops.native import require_native; N = require_native();"
             "m = N.CpuMiner(1, 'cpu-0'); m.set_job({'header': bytes.fromhex(GENESIS_HEADER_HEX),"
             "'target': bytes(32)}); m.start()\n"
             "while m.stats()['hashes'] == 0: time.sleep(0.0005)\n"
             "m.stop()")
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        subprocess.run([sys.executable, "-c", first], cwd=ROOT, env=env, check=True)
        best = min(best, time.perf_counter() - t0)
    res["process_start_to_first_cpu_hash_s"] = round(best, 3)
    # VmHWM, not ru_maxrss: on Linux ru_maxrss survives exec and would report this (forked) parent's peak.
    code = ("import otedama_amd.engine.run, otedama_amd.httpserver, otedama_amd.tui;"
            "print([l.split()[1] for l in open('/proc/self/status') if l.startswith('VmHWM')][0])")
    rss = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, check=True)
    res["control_plane_rss_mb"] = round(int(rss.stdout.strip()) / 1024, 1)
    return res


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    res = {"sv2_native": native_frames(), "sv2_python": python_frames(), "metrics": metrics_render(),
           "startup": startup(),
           "reference": {"header_ns": 20, "full1k_ns": 200, "metrics_ms_per_render": 1.12, "startup_s": 1.0,
                         "rss_mb_full_stack": 25}}
    line = json.dumps(res)
    print(line)
    if a.out:
        Path(a.out).write_text(json.dumps(res, indent=1) + "\n")


if __name__ == "__main__":
    main()
