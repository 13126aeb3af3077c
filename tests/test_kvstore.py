"""parallel/kvstore.py: the supervisor's torch-free store against torch's own TCPStore clients.

Parity is pinned by running one op sequence through a torch client against torch's server and against ours and
comparing every result; then the cases only a server can show (waits woken by another client or in-process,
cancelled waits, a gloo process group's rendezvous, many clients) run against ours."""
from __future__ import annotations

import datetime
import os
import subprocess
import sys
import threading
import time

import pytest
import torch
import torch.distributed as dist

from otedama_amd.parallel.kvstore import StoreServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TD = datetime.timedelta


def _client(port, timeout=5.0):
    return dist.TCPStore("127.0.0.1", port, None, False, TD(seconds=timeout), wait_for_workers=False)


def _sequence(c):
    out = []
    c.set("a", "1")
    out.append(c.get("a"))
    out += [c.add("n", 3), c.add("n", -1), c.get("n")]
    out += [c.compare_set("x", "", "v1"), c.compare_set("x", "bad", "v2"), c.compare_set("x", "v1", "v3"), c.get("x")]
    out += [c.compare_set("y", "nope", "z"), c.check(["y"])]
    out += [c.check(["a", "n"]), c.check(["a", "missing"])]
    out += [c.num_keys()]
    out += [c.delete_key("a"), c.delete_key("a"), c.check(["a"])]
    c.append("ap", "x")
    c.append("ap", "yz")
    out.append(c.get("ap"))
    c.multi_set(["m1", "m2"], ["A", b"\x00\xff"])
    out.append(c.multi_get(["m1", "m2", "ap"]))
    c.set("big", os.urandom(1) * (3 << 20))  # a 3 MiB value arrives in many recv() chunks
    out.append(len(c.get("big")))
    p = dist.PrefixStore("otd-g3", c)
    p.set("k", "v")
    out += [p.get("k"), p.add("c", 5), c.get("otd-g3/c")]
    c.set_timeout(TD(seconds=0.3))
    try:
        c.wait(["never"])
        out.append("no timeout")
    except dist.DistStoreError:
        out.append("timeout")
    c.set("after", "ok")  # the connection is still in step after a cancelled wait
    out.append(c.get("after"))
    out.append(c.num_keys())
    return out


def test_same_results_as_torchs_own_server():
    ref_srv = dist.TCPStore("127.0.0.1", 0, None, True, TD(seconds=5), wait_for_workers=False)
    ref = _sequence(_client(ref_srv.port))
    with StoreServer() as ours:
        got = _sequence(_client(ours.port))
    assert got == ref
    assert "timeout" in ref and ref[-2] == b"ok"


def test_waits_are_woken_by_other_clients_and_in_process():
    with StoreServer() as srv:
        a, b = _client(srv.port), _client(srv.port)
        t = threading.Timer(0.2, lambda: b.set("k1", "v1"))
        t.start()
        t0 = time.monotonic()
        assert a.get("k1") == b"v1" and time.monotonic() - t0 < 3
        t = threading.Timer(0.2, lambda: srv.set("otd/dead/3", "137"))  # the supervisor marks a rank dead
        t.start()
        a.wait(["otd/dead/3"])
        assert a.get("otd/dead/3") == b"137"
        assert srv.get("k1") == b"v1" and srv.add("n", 2) == 2 and a.add("n", 1) == 3
        assert srv.delete_key("otd/dead/3") and not a.check(["otd/dead/3"])
        # several clients blocked on one key are all released by one set
        got = []
        ths = [threading.Thread(target=lambda: got.append(_client(srv.port).get("go"))) for _ in range(6)]
        for th in ths:
            th.start()
        time.sleep(0.2)
        srv.set("go", "1")
        for th in ths:
            th.join(10)
        assert got == [b"1"] * 6


def test_a_bad_magic_or_unknown_query_drops_only_that_peer():
    import socket
    import struct

    with StoreServer() as srv:
        good = _client(srv.port)
        s = socket.create_connection(("127.0.0.1", srv.port))
        s.sendall(b"\x00" + struct.pack("<I", 0xDEADBEEF))
        s.settimeout(3)
        assert s.recv(16) == b""  # closed
        s2 = socket.create_connection(("127.0.0.1", srv.port))
        s2.sendall(b"\x00" + struct.pack("<I", 0x3C85F7CE) + b"\x63")
        s2.settimeout(3)
        assert s2.recv(16) == b""
        good.set("still", "here")
        assert good.get("still") == b"here"
        assert srv.refused == 2


_GLOO = r"""
import datetime, os, sys, torch, torch.distributed as dist
r, w, port = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
st = dist.TCPStore("127.0.0.1", port, None, False, datetime.timedelta(seconds=30), wait_for_workers=False)
for gen in range(2):  # two process-group generations, as a node re-form creates
    dist.init_process_group("gloo", store=dist.PrefixStore(f"otd-g{gen}", st), rank=r, world_size=w)
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    assert t.item() == w * (w + 1) / 2, t
    dist.destroy_process_group()
print("ok")
"""


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_process_groups_rendezvous_through_it(world):
    with StoreServer() as srv:
        env = dict(os.environ, PYTHONPATH=ROOT)
        procs = [subprocess.Popen([sys.executable, "-c", _GLOO, str(r), str(world), str(srv.port)], env=env,
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
        outs = [p.communicate(timeout=120) for p in procs]
        refused = srv.refused
    assert [p.returncode for p in procs] == [0] * world, [o[1][-2000:] for o in outs]
    assert refused == 0  # gloo's rendezvous used only query types the server implements
    assert all(o[0].strip().endswith("ok") for o in outs)  # gloo prints its own connection lines first


def test_the_node_supervisor_does_not_import_torch():
    """`otedama node` runs its supervisor with the store above and a sysfs GPU count: no torch in that process
    (570-600 MiB RSS before; the ranks and device processes are where torch lives)."""
    code = ("import sys; from otedama_amd.parallel import launch, kvstore; import otedama_amd.cli.node_cmd; "
            "s = kvstore.StoreServer(); s.set('otd/stopping', '1'); s.close(); "
            "print('torch' in sys.modules)")
    out = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, PYTHONPATH=ROOT), capture_output=True,
                         text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "False"
    assert torch  # the test process itself uses torch's clients


def test_in_process_sets_race_client_waits_without_desync():
    """The supervisor's thread sets keys (waking WAITs, which queues replies) while the server thread answers the
    same connections: 4 clients x 300 wait/get rounds on keys another thread publishes stay in step."""
    with StoreServer() as srv:
        errors = []

        def publisher():
            for i in range(300):
                srv.set(f"k{i}", str(i))

        def consumer(cid):
            c = _client(srv.port, timeout=20)
            try:
                for i in range(300):
                    assert c.get(f"k{i}") == str(i).encode()
                    c.set(f"ack{cid}/{i}", "1")
                assert c.check([f"ack{cid}/299"])  # SET has no reply: a round trip orders it before the count below
            except Exception as exc:  # noqa: BLE001
                errors.append(repr(exc))

        ths = [threading.Thread(target=consumer, args=(j,)) for j in range(4)] + [threading.Thread(target=publisher)]
        for th in ths:
            th.start()
        for th in ths:
            th.join(60)
        assert not errors, errors[:3]
        assert srv.num_keys() == 300 + 4 * 300


def test_garbage_from_one_peer_never_disturbs_another():
    """Property: whatever bytes a validated peer sends (truncated requests, huge lengths, unknown query types), the
    server thread survives, and a well-formed client on another connection keeps getting correct answers."""
    import socket
    import struct

    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as st

    with StoreServer() as srv:
        good = _client(srv.port)

        @settings(max_examples=60, deadline=None, suppress_health_check=list(HealthCheck))
        @given(st.binary(min_size=0, max_size=96))
        def one(blob):
            s = socket.create_connection(("127.0.0.1", srv.port))
            try:
                s.sendall(b"\x00" + struct.pack("<I", 0x3C85F7CE) + blob)
            finally:
                s.close()
            good.set("probe", blob.hex() or "-")
            assert good.get("probe") == (blob.hex() or "-").encode()

        one()
        assert srv._thread.is_alive()


def test_supervisor_counts_gpus_from_sysfs_without_torch(tmp_path):
    """`otedama node` checks --gpus against the KFD topology (parallel/launch.py visible_gpus), so the supervisor never
    imports torch; *_VISIBLE_DEVICES re-numbering applies as for the engine. Fixture topology: a CPU node and two
    gfx950 GPUs."""
    code = (
        "import sys, json; from otedama_amd import hal; hal.KFD_TOPOLOGY_PATH = sys.argv[1]; "
        "from otedama_amd.parallel.launch import visible_gpus; "
        "print(json.dumps([visible_gpus(), 'torch' in sys.modules]))")
    for n, text in {0: "simd_count 0\ngfx_target_version 0\n",
                    1: "simd_count 1024\nsimd_per_cu 4\ngfx_target_version 90500\n",
                    2: "simd_count 1024\nsimd_per_cu 4\ngfx_target_version 90500\n"}.items():
        (tmp_path / str(n)).mkdir()
        (tmp_path / str(n) / "properties").write_text(text)
    env = {k: v for k, v in os.environ.items() if not k.endswith("VISIBLE_DEVICES")}
    env["PYTHONPATH"] = ROOT
    out = subprocess.run([sys.executable, "-c", code, str(tmp_path)], env=env, capture_output=True, text=True,
                         timeout=60)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "[2, false]"
    env["HIP_VISIBLE_DEVICES"] = "1"
    out = subprocess.run([sys.executable, "-c", code, str(tmp_path)], env=env, capture_output=True, text=True,
                         timeout=60)
    assert out.stdout.strip() == "[1, false]", out.stderr


def test_a_peer_that_stops_reading_never_stalls_the_store():
    """a client whose socket buffer is full (a rank frozen after a GPU fault) must not block the server
    thread: other clients and the supervisor's in-process calls stay served at once, and the stalled peer is dropped
    when its backlog passes TX_CAP."""
    import socket
    import struct

    from otedama_amd.parallel import kvstore as K

    with StoreServer() as srv:
        srv.set("big", b"x" * (1 << 20))
        raw = socket.create_connection(("127.0.0.1", srv.port))
        key = b"/big"
        get = bytes([K.GET]) + struct.pack("<Q", len(key)) + key
        raw.sendall(bytes([K.VALIDATE]) + struct.pack("<I", K.MAGIC) + get * 40)  # 40 MiB of replies, never read
        time.sleep(0.5)
        c = _client(srv.port)
        t0 = time.monotonic()
        for i in range(20):
            c.set(f"k{i}", str(i))
            assert c.get(f"k{i}") == str(i).encode()
        srv.set("otd/dead/3", "137")  # the supervisor's in-process call
        assert time.monotonic() - t0 < 2.0
        # the stalled peer was dropped once its backlog passed TX_CAP: only the listener, the wake-up pipe and the
        # torch client are still registered
        end = time.monotonic() + 5
        while len(srv._sel.get_map()) > 3 and time.monotonic() < end:
            time.sleep(0.05)
        assert len(srv._sel.get_map()) == 3
        raw.close()
