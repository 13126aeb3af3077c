"""The torch-free TCPStore client (parallel/kvclient.py) against both servers the node meets: ours
(parallel/kvstore.py, hosted by the supervisor) and torch's own (torchrun's agent store), and interleaved with
torch's client on the same keys (a node may mix them: the bench's torch ranks and a native node)."""
import datetime
import threading
import time

import pytest
import torch.distributed as dist

from otedama_amd.parallel.kvclient import PrefixClient, StoreClient
from otedama_amd.parallel.kvstore import StoreServer


@pytest.fixture(params=["ours", "torch"])
def server(request):
    if request.param == "ours":
        srv = StoreServer()
        yield srv.port
        srv.close()
    else:
        master = dist.TCPStore("127.0.0.1", 0, None, True, datetime.timedelta(seconds=30), wait_for_workers=False)
        yield master.port
        del master


def test_basic_ops(server):
    c = StoreClient("127.0.0.1", server, timeout=5)
    c.set("a", "1")
    assert c.get("a") == b"1" and c.check(["a"]) and not c.check(["a", "nope"])
    assert c.add("n", 2) == 2 and c.add("n", 3) == 5 and c.get("n") == b"5"
    assert c.delete_key("a") and not c.delete_key("a") and not c.check(["a"])
    assert c.ping()
    c2 = c.clone()
    c2.set("b", b"\x00\xff")
    assert c.get("b") == b"\x00\xff"
    p = PrefixClient("otd-g3", c)
    p.set("rcclid", b"x" * 128)
    assert c.get("otd-g3/rcclid") == b"x" * 128 and p.get("rcclid") == b"x" * 128


def test_get_waits_for_the_key_and_times_out(server):
    c = StoreClient("127.0.0.1", server, timeout=5)
    other = c.clone()
    threading.Timer(0.3, lambda: other.set("late", "v")).start()
    t0 = time.monotonic()
    assert c.get("late") == b"v" and time.monotonic() - t0 >= 0.25
    c.set_timeout(0.3)
    with pytest.raises(TimeoutError):
        c.get("never")
    c.set_timeout(5)
    c.set("after", "ok")  # the connection is still in sync after the cancelled wait
    assert c.get("after") == b"ok" and c.add("n2", 1) == 1


def test_interleaves_with_torchs_client(server):
    mine = StoreClient("127.0.0.1", server, timeout=5)
    theirs = dist.TCPStore("127.0.0.1", server, None, False, datetime.timedelta(seconds=5), wait_for_workers=False)
    mine.set("k1", "from-native")
    assert theirs.get("k1") == b"from-native"
    theirs.set("k2", "from-torch")
    assert mine.get("k2") == b"from-torch"
    assert theirs.add("c", 1) == 1 and mine.add("c", 1) == 2 and theirs.add("c", 0) == 2
    assert theirs.check(["k1", "k2"]) and mine.check(["k1", "k2"])


def test_a_request_that_fails_part_way_reconnects_in_sync():
    """A reply that arrives after its request gave up must not be read as the next request's reply: the client drops
    the connection on a failed request and the next one reconnects."""
    import socket as _socket

    from otedama_amd.parallel.kvclient import StoreClient
    from otedama_amd.parallel.kvstore import StoreServer

    with StoreServer() as srv:
        c = StoreClient("127.0.0.1", srv.port, timeout=5.0)
        c.set("a", b"1")
        real = c._sock
        c._sock.settimeout(1e-9)  # the next reply cannot arrive in time
        try:
            c.check(["a"])
        except (_socket.timeout, TimeoutError, BlockingIOError, OSError):
            pass
        else:  # the reply beat the clock: nothing to test on this host
            return
        assert c._sock is None and real.fileno() == -1  # dropped, not reused with a reply in flight
        assert c.get("a") == b"1" and c.check(["a"]) and c.add("n", 2) == 2
        with pytest.raises(TimeoutError):
            c.wait(["missing"], timeout=0.1)
        assert c._sock is not None and c.get("a") == b"1"  # a withdrawn wait keeps the connection in sync
        c.close()
