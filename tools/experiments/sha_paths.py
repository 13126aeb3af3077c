"""SHA-256d on one GPU through each launch path, same process, same kernel (otd_sha256d_search_vn<2,0>):

  ops_2^35     torch-stream launches of 128 variants x 2^28 nonces (what bench.py times), back to back
  ops_2^32     the same with 128 x 2^25 (the production launch size)
  ops_2^32_2s  2^32-hash launches alternating over two torch streams (the production overlap)
  miner        the native GpuMiner (hit ring, abort word, 2 streams, 2^32 launches)

python tools/sha_paths.py  -> one JSON line of hashes/s per path (two rounds, interleaved)."""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from otedama_amd.models.header import int_to_hash  # noqa: E402
from otedama_amd.ops import search as S  # noqa: E402


def main() -> int:
    N = S.require_native()
    dev = "cuda:0"
    hdr = bytes(range(76)) + bytes(4)
    s = S.Sha256dSearchV(dev, grid=S.default_grid(dev, S.SHA256D_V2_BLOCKS_PER_CU), chains=2, occupancy8=False)
    hs = [((0x20000000 | (v << 13)) & 0xFFFFFFFF).to_bytes(4, "little") + hdr[4:] for v in range(128)]
    prep = s.prepare(hs, (1 << 200).to_bytes(32, "little"))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]

    def ops(per_variant: int, seconds: float, two: bool) -> float:
        n = max(2, int(seconds * 19.5e9 / (128 * per_variant)))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(n):
            if two:
                with torch.cuda.stream(streams[i % 2]):
                    s.launch(prep, (i * per_variant) & 0xFFFFFFFF, per_variant)
            else:
                s.launch(prep, (i * per_variant) & 0xFFFFFFFF, per_variant)
        torch.cuda.synchronize()
        return 128 * per_variant * n / (time.perf_counter() - t0)

    def miner(seconds: float) -> float:
        m = N.GpuMiner(0, "gpu-0", batch_nonces=1 << 32, grid=N.gpu_cu_count(0) * 6, queue_cap=4096,
                       sha_variants=128)
        m.set_job({"header": hdr, "target": int_to_hash((1 << 224) - 1), "job_id": "p", "epoch": 1,
                   "algo": "sha256d", "version_mask": 0x1FFFE000})
        m.start()
        time.sleep(2.0)

        def edge():  # counter moves only when a launch retires: time the window between two moves
            h = m.stats()["hashes"]
            while True:
                h2 = m.stats()["hashes"]
                if h2 != h:
                    return h2, time.monotonic()
                time.sleep(0.0002)

        h0, t0 = edge()
        time.sleep(seconds)
        h1, t1 = edge()
        m.stop()
        return (h1 - h0) / (t1 - t0)

    ops(1 << 25, 1.0, False)  # warm-up
    res: dict = {"ops_2^35": [], "ops_2^32": [], "ops_2^32_2s": [], "miner": []}
    for _ in range(2):
        res["ops_2^35"].append(ops(1 << 28, 8.0, False))
        res["ops_2^32"].append(ops(1 << 25, 8.0, False))
        res["ops_2^32_2s"].append(ops(1 << 25, 8.0, True))
        res["miner"].append(miner(8.0))
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(main())
