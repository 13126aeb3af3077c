"""Append-only share journal + worker/vardiff persistence + payout accounting.

[NO REFERENCE CODE] v2 used PostgreSQL/SQLite (CHANGELOG.md:6650); SURVEY §5.4
recommends an append-only journal. SQLite (stdlib) in WAL mode: shares are
appended in batches from the event loop; worker difficulty survives restarts;
blocks found and their PPLNS / PROP payouts are recorded.
"""
from __future__ import annotations

import sqlite3
import threading
import time
from dataclasses import dataclass

SCHEMA = """
CREATE TABLE IF NOT EXISTS shares (
  id INTEGER PRIMARY KEY AUTOINCREMENT,
  ts REAL NOT NULL, worker TEXT NOT NULL, algo TEXT NOT NULL, job_id TEXT NOT NULL,
  difficulty REAL NOT NULL, accepted INTEGER NOT NULL, reason TEXT, hash TEXT,
  block INTEGER NOT NULL DEFAULT 0
);
CREATE INDEX IF NOT EXISTS shares_worker ON shares(worker);
CREATE TABLE IF NOT EXISTS workers (
  worker TEXT PRIMARY KEY, difficulty REAL NOT NULL, updated REAL NOT NULL
);
CREATE TABLE IF NOT EXISTS blocks (
  id INTEGER PRIMARY KEY AUTOINCREMENT, ts REAL NOT NULL, height INTEGER, hash TEXT, worker TEXT,
  reward INTEGER, scheme TEXT
);
CREATE TABLE IF NOT EXISTS payouts (
  block_id INTEGER NOT NULL, worker TEXT NOT NULL, amount INTEGER NOT NULL
);
"""


@dataclass
class ShareRow:
    ts: float
    worker: str
    algo: str
    job_id: str
    difficulty: float
    accepted: bool
    reason: str = ""
    hash: str = ""
    block: bool = False


class Journal:
    def __init__(self, path: str = ":memory:"):
        self.path = path
        self._db = sqlite3.connect(path, check_same_thread=False, isolation_level=None)
        if path != ":memory:":
            self._db.execute("PRAGMA journal_mode=WAL")
            self._db.execute("PRAGMA synchronous=NORMAL")
        self._db.executescript(SCHEMA)
        self._lock = threading.Lock()
        self._buf: list[ShareRow] = []

    def append(self, row: ShareRow) -> None:
        with self._lock:
            self._buf.append(row)
            if len(self._buf) >= 256:
                self._flush_locked()

    def flush(self) -> None:
        with self._lock:
            self._flush_locked()

    def _flush_locked(self) -> None:
        if not self._buf:
            return
        rows = [(r.ts, r.worker, r.algo, r.job_id, r.difficulty, int(r.accepted), r.reason, r.hash, int(r.block))
                for r in self._buf]
        self._buf.clear()
        self._db.execute("BEGIN")
        self._db.executemany("INSERT INTO shares(ts, worker, algo, job_id, difficulty, accepted, reason, hash, block)"
                             " VALUES (?,?,?,?,?,?,?,?,?)", rows)
        self._db.execute("COMMIT")

    def save_worker(self, worker: str, difficulty: float) -> None:
        with self._lock:
            self._db.execute("INSERT INTO workers(worker, difficulty, updated) VALUES(?,?,?) ON CONFLICT(worker) "
                             "DO UPDATE SET difficulty=excluded.difficulty, updated=excluded.updated",
                             (worker, difficulty, time.time()))

    def load_worker(self, worker: str) -> float | None:
        with self._lock:
            r = self._db.execute("SELECT difficulty FROM workers WHERE worker=?", (worker,)).fetchone()
        return r[0] if r else None

    def counts(self) -> dict:
        self.flush()
        with self._lock:
            acc = self._db.execute("SELECT COUNT(*), COALESCE(SUM(difficulty),0) FROM shares WHERE accepted=1"
                                   ).fetchone()
            rej = self._db.execute("SELECT COUNT(*) FROM shares WHERE accepted=0").fetchone()
            blk = self._db.execute("SELECT COUNT(*) FROM blocks").fetchone()
        return {"accepted": acc[0], "accepted_work": acc[1], "rejected": rej[0], "blocks": blk[0]}

    def pplns_window(self, n_shares: int) -> dict[str, float]:
        """Difficulty-weighted work per worker over the last n accepted shares."""
        self.flush()
        with self._lock:
            rows = self._db.execute(
                "SELECT worker, difficulty FROM shares WHERE accepted=1 ORDER BY id DESC LIMIT ?", (n_shares,)
            ).fetchall()
        work: dict[str, float] = {}
        for w, d in rows:
            work[w] = work.get(w, 0.0) + d
        return work

    def record_block(self, height: int, block_hash: str, worker: str, reward: int, scheme: str = "pplns",
                     window: int = 10_000) -> dict[str, int]:
        work = self.pplns_window(window) if scheme == "pplns" else {}
        if not work:
            work = {worker: 1.0}
        total = sum(work.values())
        payouts = {w: int(reward * v / total) for w, v in work.items()}
        with self._lock:
            cur = self._db.execute("INSERT INTO blocks(ts, height, hash, worker, reward, scheme) VALUES(?,?,?,?,?,?)",
                                   (time.time(), height, block_hash, worker, reward, scheme))
            bid = cur.lastrowid
            self._db.executemany("INSERT INTO payouts(block_id, worker, amount) VALUES(?,?,?)",
                                 [(bid, w, a) for w, a in payouts.items()])
        return payouts

    def worker_summary(self, limit: int = 100) -> list[dict]:
        """Per-worker totals from the journal (all time), busiest first: the /api/v1/workers payload."""
        self.flush()
        with self._lock:
            rows = self._db.execute(
                "SELECT s.worker, SUM(s.accepted), SUM(1 - s.accepted), COALESCE(SUM(CASE WHEN s.accepted=1 "
                "THEN s.difficulty END), 0), MAX(s.ts), SUM(s.block), w.difficulty FROM shares s LEFT JOIN workers w "
                "ON w.worker = s.worker GROUP BY s.worker ORDER BY 4 DESC LIMIT ?", (limit,)).fetchall()
        return [{"worker": w, "accepted": int(a or 0), "rejected": int(r or 0), "accepted_work": float(work),
                 "last_share": float(ts or 0.0), "blocks": int(b or 0), "saved_difficulty": d}
                for w, a, r, work, ts, b, d in rows]

    def recent_blocks(self, limit: int = 20) -> list[dict]:
        """Blocks found, newest first, each with its payout split: the /api/v1/blocks payload."""
        with self._lock:
            blocks = self._db.execute("SELECT id, ts, height, hash, worker, reward, scheme FROM blocks "
                                      "ORDER BY id DESC LIMIT ?", (limit,)).fetchall()
            out = []
            for bid, ts, height, h, worker, reward, scheme in blocks:
                pays = self._db.execute("SELECT worker, amount FROM payouts WHERE block_id=? ORDER BY amount DESC",
                                        (bid,)).fetchall()
                out.append({"height": height, "hash": h, "found_by": worker, "ts": ts, "reward": reward,
                            "scheme": scheme, "payouts": [{"worker": w, "amount": a} for w, a in pays]})
        return out

    def close(self) -> None:
        self.flush()
        self._db.close()
