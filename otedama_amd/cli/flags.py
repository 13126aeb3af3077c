"""A small Go ``flag``-compatible parser (the reference CLI uses the stdlib
flag package: ``-name value``, ``--name=value``, boolean flags without a value,
``--`` ends flags, ``-h/--help`` -> ErrHelp; cmd/otedama/main.go:56-105)."""
from __future__ import annotations

from dataclasses import dataclass
from typing import TextIO


class FlagError(Exception):
    pass


class ErrHelp(Exception):
    pass


@dataclass
class _Flag:
    name: str
    kind: type
    default: object
    usage: str


class FlagSet:
    def __init__(self, name: str, out: TextIO | None = None):
        self.name = name
        self.out = out
        self._flags: dict[str, _Flag] = {}
        self.values: dict[str, object] = {}
        self.args: list[str] = []
        self.set_flags: set[str] = set()

    def string(self, name: str, default: str, usage: str) -> None:
        self._def(name, str, default, usage)

    def bool(self, name: str, default: bool, usage: str) -> None:
        self._def(name, bool, default, usage)

    def int(self, name: str, default: int, usage: str) -> None:
        self._def(name, int, default, usage)

    def float(self, name: str, default: float, usage: str) -> None:
        self._def(name, float, default, usage)

    def _def(self, name, kind, default, usage):
        self._flags[name] = _Flag(name, kind, default, usage)
        self.values[name] = default

    def __getitem__(self, name: str):
        return self.values[name]

    def usage(self) -> str:
        lines = [f"Usage of {self.name}:"]
        for name in sorted(self._flags):
            f = self._flags[name]
            tname = {str: " string", int: " int", float: " float", bool: ""}[f.kind]
            lines.append(f"  -{name}{tname}")
            d = f.default
            dflt = f" (default {d!r})" if (d not in ("", 0, 0.0, False) and d is not None) else ""
            lines.append(f"    \t{f.usage}{dflt}")
        return "\n".join(lines) + "\n"

    def _fail(self, msg: str) -> None:
        if self.out is not None:
            self.out.write(msg + "\n" + self.usage())
        raise FlagError(msg)

    def parse(self, args: list[str]) -> list[str]:
        i = 0
        while i < len(args):
            a = args[i]
            if a == "--":
                self.args = list(args[i + 1:])
                return self.args
            if not a.startswith("-") or a == "-":
                self.args = list(args[i:])
                return self.args
            name = a.lstrip("-")
            if a.startswith("---") or not name:
                self._fail(f"bad flag syntax: {a}")
            value = None
            if "=" in name:
                name, value = name.split("=", 1)
            if name in ("h", "help") and name not in self._flags:
                if self.out is not None:
                    self.out.write(self.usage())
                raise ErrHelp()
            f = self._flags.get(name)
            if f is None:
                self._fail(f"flag provided but not defined: -{name}")
            if f.kind is bool:
                if value is None:
                    self.values[name] = True
                else:
                    lv = value.lower()
                    if lv in ("1", "t", "true"):
                        self.values[name] = True
                    elif lv in ("0", "f", "false"):
                        self.values[name] = False
                    else:
                        self._fail(f"invalid boolean value {value!r} for -{name}")
            else:
                if value is None:
                    i += 1
                    if i >= len(args):
                        self._fail(f"flag needs an argument: -{name}")
                    value = args[i]
                try:
                    self.values[name] = f.kind(value)
                except ValueError:
                    self._fail(f"invalid value {value!r} for flag -{name}: parse error")
            self.set_flags.add(name)
            i += 1
        self.args = []
        return self.args


def has_help_flag(args: list[str]) -> bool:
    for a in args:
        if a in ("-h", "-help", "--help"):
            return True
        if a == "--":
            return False
    return False
