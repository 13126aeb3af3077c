"""Structured logger with slog-style text / JSON output.

Parity: internal/logger/logger.go — ParseLevel (:75-86), New(Config) text|JSON
(:112-129), Discard (:133-138), Adapter() -> func(level, msg) used by the engine
(:143-156), context carriage (:167-184; here a contextvar), SetDefault (:219-224).

Text lines follow slog's TextHandler: ``time=... level=INFO msg="..." k=v``.
"""
from __future__ import annotations

import contextvars
import datetime as _dt
import json
import sys
import threading
from dataclasses import dataclass, field
from typing import Callable, TextIO

DEBUG, INFO, WARN, ERROR = -4, 0, 4, 8
_NAMES = {DEBUG: "DEBUG", INFO: "INFO", WARN: "WARN", ERROR: "ERROR"}


def parse_level(s: str) -> int:
    s = (s or "").strip().lower()
    return {"debug": DEBUG, "warn": WARN, "warning": WARN, "error": ERROR}.get(s, INFO)


def _quote(v: str) -> str:
    if v == "" or any(c in v for c in ' ="\\\n\t') or not v.isprintable():
        return json.dumps(v, ensure_ascii=False)
    return v


@dataclass
class Config:
    level: int = INFO
    format: str = "text"  # text | json
    writer: TextIO | None = None
    add_source: bool = False


@dataclass
class Logger:
    config: Config = field(default_factory=Config)
    attrs: dict = field(default_factory=dict)
    _lock: threading.Lock = field(default_factory=threading.Lock, repr=False)

    def enabled(self, level: int) -> bool:
        return level >= self.config.level

    def with_attrs(self, **kw) -> "Logger":
        return Logger(self.config, {**self.attrs, **kw}, self._lock)

    def log(self, level: int, msg: str, **kw) -> None:
        if not self.enabled(level):
            return
        w = self.config.writer or sys.stderr
        now = _dt.datetime.now().astimezone().isoformat(timespec="milliseconds")
        attrs = {**self.attrs, **kw}
        lvl = _NAMES.get(level, f"LEVEL{level}")
        if self.config.format == "json":
            line = json.dumps({"time": now, "level": lvl, "msg": msg, **attrs}, default=str, ensure_ascii=False)
        else:
            parts = [f"time={now}", f"level={lvl}", f"msg={_quote(msg)}"]
            parts += [f"{k}={_quote(str(v))}" for k, v in attrs.items()]
            line = " ".join(parts)
        with self._lock:
            try:
                w.write(line + "\n")
                w.flush()
            except (ValueError, OSError):
                pass

    def debug(self, msg: str, **kw) -> None:
        self.log(DEBUG, msg, **kw)

    def info(self, msg: str, **kw) -> None:
        self.log(INFO, msg, **kw)

    def warn(self, msg: str, **kw) -> None:
        self.log(WARN, msg, **kw)

    warning = warn

    def error(self, msg: str, **kw) -> None:
        self.log(ERROR, msg, **kw)

    def adapter(self) -> Callable[[str, str], None]:
        """func(level, msg) used by the engine, which does not import the logger."""

        def fn(level: str, msg: str) -> None:
            self.log(parse_level(level), msg)

        return fn


class _Discard:
    def write(self, s):
        return len(s)

    def flush(self):
        pass


def new(level: int = INFO, fmt: str = "text", writer: TextIO | None = None) -> Logger:
    return Logger(Config(level=level, format=fmt, writer=writer))


def discard() -> Logger:
    return Logger(Config(level=ERROR + 1, writer=_Discard()))


_default: Logger | None = None
_default_lock = threading.Lock()
_ctx: contextvars.ContextVar[Logger | None] = contextvars.ContextVar("otedama_logger", default=None)


def default() -> Logger:
    global _default
    with _default_lock:
        if _default is None:
            _default = new()
        return _default


def set_default(lg: Logger | None) -> None:
    global _default
    if lg is None:
        return
    with _default_lock:
        _default = lg


def into_context(lg: Logger | None) -> None:
    if lg is not None:
        _ctx.set(lg)


def from_context() -> Logger:
    return _ctx.get() or default()
