"""Job switch (engine -> device process -> first batch of the new work running) for one algorithm under two
environments, each in fresh processes: e.g. the X11 stage polls / scrypt staggered halves (A, the default) against
the round-3 behaviour (B). Prints one JSON line per (variant, algorithm)."""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CHILD = r'''
import json, sys
sys.path.insert(0, sys.argv[1])
from otedama_amd.engine.latency_probe import measure_job_switch
r = measure_job_switch(0, sys.argv[2], switches=int(sys.argv[3]))
r.pop("in_process", None)
print(json.dumps(r))
'''


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", required=True)
    ap.add_argument("--switches", type=int, default=10)
    ap.add_argument("--env-b", default="")
    a = ap.parse_args()
    for name, spec in (("a", ""), ("b", a.env_b)):
        env = dict(os.environ)
        for kv in filter(None, spec.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v
        out = subprocess.run([sys.executable, "-c", CHILD, ROOT, a.algo, str(a.switches)], capture_output=True,
                             text=True, timeout=170, env=env)
        line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
        if out.returncode != 0 or not line:
            print(json.dumps({"variant": name, "error": out.returncode, "stderr": out.stderr[-1500:]}), flush=True)
            return 1
        print(json.dumps({"variant": name, "algo": a.algo, "env": spec, **json.loads(line[0])}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
