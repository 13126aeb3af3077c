"""Stratum V1 client session against scripted loopback pools (the reference's runFakeServer pattern,
poolproto/stratumv1/stratumv1_test.go:1438-1500): BIP310 negotiation, subscribe/authorize, difficulty and job
delivery, submit accept/reject, show_message, client.reconnect (closes, never follows), oversize-line guard."""
import asyncio
import json

import pytest

from otedama_amd.models.header import hash_to_int, target_from_difficulty
from otedama_amd.poolproto.base import Credentials, FatalPoolError, ShareSubmission
from otedama_amd.poolproto.stratumv1 import BIP320_MASK, MAX_LINE_BYTES, V1Dialer, prevhash_to_stratum

PREV = prevhash_to_stratum(bytes(range(32)))
NOTIFY = ["1a", PREV, "01000000", "ffffffff", [], "20000000", "1d00ffff", "5f5e1000", True]


class ScriptedPool:
    def __init__(self, authorize=True, after_auth=(), submit_replies=(True,)):
        self.authorize = authorize
        self.after_auth = list(after_auth)
        self.submit_replies = list(submit_replies)
        self.submits: list[list] = []
        self.methods: list[str] = []
        self.server = None
        self.writers = []

    async def start(self):
        self.server = await asyncio.start_server(self._handle, "127.0.0.1", 0)
        return self.server.sockets[0].getsockname()[1]

    async def stop(self):
        for w in self.writers:
            w.close()
        self.server.close()
        await self.server.wait_closed()

    async def _handle(self, reader, writer):
        self.writers.append(writer)

        def send(obj):
            writer.write(json.dumps(obj).encode() + b"\n")

        while True:
            line = await reader.readline()
            if not line:
                return
            msg = json.loads(line)
            m, mid = msg["method"], msg["id"]
            self.methods.append(m)
            if m == "mining.configure":
                send({"id": mid, "result": {"version-rolling": True, "version-rolling.mask": "1fffe000"}, "error": None})
            elif m == "mining.subscribe":
                send({"id": mid, "result": [[["mining.notify", "s1"]], "abcd0001", 4], "error": None})
            elif m == "mining.authorize":
                send({"id": mid, "result": self.authorize, "error": None if self.authorize else [24, "bad user", None]})
                if self.authorize:
                    for note in self.after_auth:
                        send(note)
            elif m == "mining.extranonce.subscribe":
                send({"id": mid, "result": True, "error": None})
            elif m == "mining.submit":
                self.submits.append(msg["params"])
                r = self.submit_replies.pop(0) if self.submit_replies else True
                if r is True:
                    send({"id": mid, "result": True, "error": None})
                else:
                    send({"id": mid, "result": None, "error": [23, r, None]})
            await writer.drain()


def _creds():
    return Credentials(user="bc1qar0srrr7xfkvy5l643lydnw9re59gtzzwf5mdq.rig7", worker="rig7", version_rolling=True)


def run(coro):
    return asyncio.run(asyncio.wait_for(coro, 30))


def test_handshake_job_difficulty_and_submits():
    async def main():
        pool = ScriptedPool(after_auth=[{"id": None, "method": "mining.set_difficulty", "params": [2]},
                                        {"id": None, "method": "mining.notify", "params": NOTIFY}],
                            submit_replies=[True, "low difficulty share"])
        port = await pool.start()
        s = await V1Dialer().dial(f"stratum+tcp://127.0.0.1:{port}", _creds())
        job = await asyncio.wait_for(s.jobs.get(), 5)
        assert pool.methods[:3] == ["mining.configure", "mining.subscribe", "mining.authorize"]
        assert s.version_mask == BIP320_MASK and s.extranonce1 == bytes.fromhex("abcd0001")
        assert s.extranonce2_size == 4
        assert job.job_id == "1a" and job.prev_hash == bytes(range(32)) and job.nbits == 0x1D00FFFF
        assert job.extranonce1 == bytes.fromhex("abcd0001") and job.extranonce2_size == 4
        assert hash_to_int(job.target) == hash_to_int(target_from_difficulty(2.0))
        r1 = await s.submit(ShareSubmission(job_id="1a", nonce=0x1234, ntime=0x5F5E1000, version=job.version,
                                            extranonce2=bytes.fromhex("00000007"), worker="rig7"))
        r2 = await s.submit(ShareSubmission(job_id="1a", nonce=0x99, ntime=0x5F5E1001, version=job.version | 0x2000,
                                            extranonce2=bytes(4), worker="rig7"))
        assert r1.accepted and r1.difficulty == 2.0 and r1.latency_ms > 0
        assert not r2.accepted and r2.reason == "low difficulty share"
        assert pool.submits[0] == ["rig7", "1a", "00000007", "5f5e1000", "00001234"]
        assert pool.submits[1][5] == "00002000"   # BIP310: only the rolled bits, masked
        await s.close()
        await pool.stop()

    run(main())


def test_set_difficulty_reissues_the_active_job():
    async def main():
        pool = ScriptedPool(after_auth=[{"id": None, "method": "mining.notify", "params": NOTIFY},
                                        {"id": None, "method": "mining.set_difficulty", "params": [8]}])
        port = await pool.start()
        s = await V1Dialer().dial(f"stratum+tcp://127.0.0.1:{port}", _creds())
        first = await asyncio.wait_for(s.jobs.get(), 5)
        again = await asyncio.wait_for(s.jobs.get(), 5)
        assert again.job_id == first.job_id and not again.clean_jobs
        assert hash_to_int(again.target) == hash_to_int(target_from_difficulty(8.0))
        # the queued original is a different object and keeps its clean flag and the target it was issued with
        assert again is not first
        assert first.clean_jobs
        assert hash_to_int(first.target) == hash_to_int(target_from_difficulty(1.0))
        assert s.suggested_difficulty() == 8.0
        await s.close()
        await pool.stop()

    run(main())


def test_show_message_and_reconnect_is_not_followed():
    async def main():
        pool = ScriptedPool(after_auth=[{"id": None, "method": "client.show_message", "params": ["maintenance"]},
                                        {"id": None, "method": "client.reconnect",
                                         "params": ["evil.example", 3333, 5]}])
        port = await pool.start()
        s = await V1Dialer().dial(f"stratum+tcp://127.0.0.1:{port}", _creds())
        assert await asyncio.wait_for(s.notices.get(), 5) == "maintenance"
        for _ in range(100):
            if s.closed:
                break
            await asyncio.sleep(0.02)
        assert s.closed
        assert s.last_reconnect == {"host": "evil.example", "port": 3333, "wait": 5}
        assert s.remote_addr == "" or "evil" not in s.remote_addr
        await pool.stop()

    run(main())


def test_authorize_rejection_is_fatal():
    async def main():
        pool = ScriptedPool(authorize=False)
        port = await pool.start()
        with pytest.raises(FatalPoolError):
            await V1Dialer().dial(f"stratum+tcp://127.0.0.1:{port}", _creds())
        await pool.stop()

    run(main())


def test_oversized_line_terminates_the_session():
    async def main():
        big = {"id": None, "method": "client.show_message", "params": ["x" * (MAX_LINE_BYTES + 10)]}
        pool = ScriptedPool(after_auth=[big])
        port = await pool.start()
        s = await V1Dialer().dial(f"stratum+tcp://127.0.0.1:{port}", _creds())
        for _ in range(200):
            if s.closed:
                break
            await asyncio.sleep(0.02)
        assert s.closed and s.notices.empty()
        await pool.stop()

    run(main())
