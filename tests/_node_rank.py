"""One rank of a CPU (gloo) node for tests/test_node_faults.py: rank 0 drives the node and reports to out_dir."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def job(target_bits: int) -> dict:
    from otedama_amd.models.header import int_to_hash

    hdr = bytes([1, 0, 0, 0]) + bytes(range(32)) + bytes(range(32, 64)) + (1700000000).to_bytes(4, "little") + \
        bytes.fromhex("ffff001d") + bytes(4)
    return {"header": hdr, "target": int_to_hash((1 << target_bits) - 1), "job_id": "job-A", "algo": "sha256d",
            "version_mask": 0x1FFFE000}


def main(out_dir: str, mode: str) -> int:
    from otedama_amd import hal
    from otedama_amd.engine.miners import MinerSet
    from otedama_amd.parallel.comm import NodeComm, init_from_env, join_from_env, shutdown
    from otedama_amd.parallel.node import NodeMinerSet, NodeWorker

    joining = os.environ.get("OTEDAMA_NODE_JOIN") == "1"
    info = join_from_env("gloo", use_gpu=False) if joining else init_from_env("gloo", use_gpu=False)
    dev = [hal.SimpleDevice(hal.Identity("cpu-0", hal.Family.CPU, "t", "cpu"),
                            hal.Capabilities(sha256d=True, general_compute=True), threads=1)]
    local = MinerSet(dev, "sha256d", rank=max(info.rank, 0), world_size=max(info.world_size, 1))
    comm = NodeComm(info)
    logs = []
    log = lambda lvl, msg: logs.append(msg)  # noqa: E731
    if info.orig_rank > 0:
        NodeWorker(local, comm, log=log, joining=joining).run()
        shutdown(info)
        return 0
    stats_interval = 10.0 if mode == "quiet" else 0.5
    node = NodeMinerSet(local, comm, log=log, stats_interval=stats_interval)
    node.start()
    world = info.world_size
    shares = []
    res = {"world": world}
    try:
        if mode == "quiet":  # no shares, no job churn: count device collectives per rank over a window
            node.set_job(job(160))
            time.sleep(2.0)
            c0, t0 = comm.collectives, time.monotonic()
            time.sleep(4.0)
            res["collectives_per_s"] = (comm.collectives - c0) / (time.monotonic() - t0)
            res["tick_p50_s"], res["tick_p99_s"] = node.link.tick_quantile(0.5), node.link.tick_quantile(0.99)
            return 0
        if mode == "trim":  # job churn past the op log's retention, a follower stopped meanwhile, then resumed
            from otedama_amd.parallel.node import _k

            def churn(seconds):
                nonlocal shares
                end = time.monotonic() + seconds
                i = 0
                while time.monotonic() < end:
                    j = job(236)
                    j["job_id"] = f"churn-{time.monotonic_ns()}-{i}"
                    node.set_job(j)
                    i += 1
                    shares += node.poll(256)
                    time.sleep(0.02)

            churn(2.0)
            with open(os.path.join(out_dir, "phase1.json.tmp"), "w") as f:
                json.dump({"op_k": node._op_k}, f)
            os.replace(os.path.join(out_dir, "phase1.json.tmp"), os.path.join(out_dir, "phase1.json"))
            resumed = os.path.join(out_dir, "killed.json")
            while not os.path.exists(resumed):
                churn(0.2)
            ep_resume = node.epoch
            end = time.monotonic() + 40
            got = False
            while time.monotonic() < end and not got:
                new = node.poll(256)
                shares += new
                got = any(s["device_id"] == "rank1" and s["epoch"] >= ep_resume for s in new)
                time.sleep(0.02)
            store = comm.info.store
            res.update(ops_posted=node._op_k, victim_shares_after_resume=got, reforms=node.link.reforms,
                       ops_kept=sum(1 for j in range(node._op_k) if store.check([_k("op", j)])))
            return 0
        ep0 = node.set_job(job(236))
        end = time.monotonic() + 60
        while time.monotonic() < end:
            shares += node.poll(256)
            ranks = {s["device_id"] for s in shares}
            if len(ranks) >= world:
                break
            time.sleep(0.02)
        res["phase1_devices"] = sorted({s["device_id"] for s in shares})
        with open(os.path.join(out_dir, "phase1.json.tmp"), "w") as f:
            json.dump({"n": len(shares)}, f)
        os.replace(os.path.join(out_dir, "phase1.json.tmp"), os.path.join(out_dir, "phase1.json"))
        killed = os.path.join(out_dir, "killed.json")
        end = time.monotonic() + 60
        while not os.path.exists(killed) and time.monotonic() < end:
            shares += node.poll(256)
            time.sleep(0.01)
        with open(killed) as f:
            k = json.load(f)
        n_before = len(shares)
        t_reform = None
        end = time.monotonic() + 30
        post = []
        while time.monotonic() < end:
            new = node.poll(256)
            shares += new
            if t_reform is None and node.link.reforms >= 1 and node.epoch > ep0:  # re-form done, job re-issued
                t_reform = time.time()
                base, members = node._variant_base, list(comm.info.members)
            if t_reform is not None:  # shares of the re-issued job (older ones may still arrive late)
                post += [s for s in new if s["device_id"] != "cpu-0" and s["epoch"] > ep0]
                if len({s["device_id"] for s in post}) >= min(2, world - 2) and len(post) >= 3:
                    break
            time.sleep(0.01)
        res.update(reform_after_s=(t_reform - k["t"]) if t_reform else None, base=base if t_reform else None,
                   members=members if t_reform else None, lost=node.lost_ranks,
                   post=[{"dev": s["device_id"], "version": s["version"], "nonce": s["nonce"], "epoch": s["epoch"]}
                         for s in post], n_before=n_before)
        if mode == "rejoin":  # the harness restarts the killed rank: it must be re-admitted and mine again
            end = time.monotonic() + 60
            while time.monotonic() < end and node.link.reforms < 2:
                shares += node.poll(256)
                time.sleep(0.02)
            res["members_after_rejoin"] = list(comm.info.members)
            victim = f"rank{k['rank']}"
            t1 = time.monotonic()
            got = False
            while time.monotonic() - t1 < 30 and not got:
                new = node.poll(256)
                shares += new
                got = any(s["device_id"] == victim for s in new)
                time.sleep(0.02)
            res["victim_shares_after_rejoin"] = got
    finally:
        node.stop()
        res["shares"] = [{"dev": s["device_id"], "version": s["version"], "nonce": s["nonce"]} for s in shares]
        res["logs"] = logs[-50:]
        res["collectives"] = comm.collectives
        with open(os.path.join(out_dir, "result.json"), "w") as f:
            json.dump(res, f)
        shutdown(comm.info)
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "kill"))
