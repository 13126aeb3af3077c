#!/usr/bin/env python3
"""Local-pool throughput (BASELINE.json config 5): the command-line wrapper of otedama_amd/pool/load.py.

Usage: python tools/bench_pool.py [--algo sha256d|scrypt|x11|mixed] [--miners 16] [--seconds 10]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from otedama_amd.pool.load import _miner, _run_pool, main, main_async  # noqa: E402,F401

if __name__ == "__main__":
    sys.exit(main())
