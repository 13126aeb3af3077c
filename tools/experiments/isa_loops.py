"""Static VALU histogram of a compiled gfx950 kernel per loop and per basic block, with dynamic counts from trip
counts (the X11 instruction-floor accounting in docs/KERNELS.md; tools/isa_mix.py prices the innermost loops' mix).

python tools/isa_loops.py <file.s> <kernel-substring> [--trips HDR=N ...] [--blocks]

Reads the assembly that ``hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S`` writes, splits the kernel into
basic blocks, and uses LLVM's loop comments (``=>This Inner Loop Header``, ``in Loop: Header=BBx_y``,
``Parent Loop``) to attribute every VALU instruction to its innermost loop. With ``--trips`` (trip count of each
loop header, per enclosing iteration) it also prints the dynamic VALU count per work item, the number to hold
against the SQ_INSTS_VALU / work-items counter. Instruction classes: alignbit (rotates), bitop3, xor, add, shift,
perm, mov, cndmask, other.
"""
from __future__ import annotations

import argparse
import collections
import json
import re
import sys

CLASSES = (("alignbit", ("v_alignbit",)), ("bitop3", ("v_bitop3",)), ("xor", ("v_xor",)),
           ("add", ("v_add", "v_sub", "v_mad", "v_lshl_add", "v_add3")),
           ("shift", ("v_lshl", "v_lshr", "v_ashr", "v_bfe", "v_bfi", "v_lshl_or")), ("perm", ("v_perm",)),
           ("mov", ("v_mov", "v_readfirstlane", "v_readlane", "v_writelane", "v_accvgpr")),
           ("cndmask", ("v_cndmask",)), ("logic", ("v_and", "v_or", "v_not")),
           ("dot", ("v_dot",)))


def klass(op: str) -> str:
    for name, prefixes in CLASSES:
        if op.startswith(prefixes):
            return name
    return "other"


def parse(path: str, kernel: str) -> dict:
    lines = open(path).read().splitlines()
    start = next((i for i, ln in enumerate(lines) if re.match(r"^_Z\S*:", ln) and kernel in ln.split(":")[0]), None)
    if start is None:
        raise SystemExit(f"kernel {kernel!r} not found in {path}")
    name = lines[start].split(":")[0]
    blocks: list[dict] = []
    cur = {"name": "entry", "loop": None, "valu": collections.Counter(), "header_of": None, "parent": None}
    blocks.append(cur)
    pending_comments = True
    for ln in lines[start + 1:]:
        if "s_endpgm" in ln and not ln.strip().startswith(";"):
            break
        m = re.match(r"^\.LBB(\d+_\d+):(.*)$", ln) or re.match(r"^; %bb\.(\d+):(.*)$", ln)
        if m:
            cur = {"name": f"BB{m.group(1)}", "loop": None, "valu": collections.Counter(), "header_of": None,
                   "parent": None}
            blocks.append(cur)
            pending_comments = True
            rest = m.group(2)
            _loop_comment(cur, rest)
            continue
        s = ln.strip()
        if s.startswith(";"):
            if pending_comments:
                _loop_comment(cur, s)
            continue
        pending_comments = False
        if s.startswith("v_"):
            cur["valu"][klass(s.split()[0])] += 1
    loops: dict[str, dict] = {}
    for b in blocks:
        if b["header_of"]:
            loops.setdefault(b["name"], {"parent": b["parent"], "valu": collections.Counter()})
    straight = collections.Counter()
    for b in blocks:
        hdr = b["name"] if b["header_of"] else b["loop"]
        if hdr:
            loops.setdefault(hdr, {"parent": None, "valu": collections.Counter()})["valu"].update(b["valu"])
        else:
            straight.update(b["valu"])
    return {"kernel": name, "straight": straight, "loops": loops, "blocks": blocks}


def _loop_comment(block: dict, text: str) -> None:
    m = re.search(r"in Loop: Header=(BB\d+_\d+)", text)
    if m:
        block["loop"] = m.group(1)
    if "Loop Header" in text:
        block["header_of"] = True
    m = re.search(r"Parent Loop (BB\d+_\d+)", text)
    if m:
        block["parent"] = m.group(1)


def dynamic(res: dict, trips: dict[str, int]) -> tuple[int, collections.Counter]:
    """VALU per work item: straight-line code once, each loop body x the product of its and its parents' trips."""
    def mult(hdr):
        k, h = 1, hdr
        while h:
            k *= trips.get(h, 1)
            h = res["loops"][h]["parent"]
        return k

    tot = collections.Counter(res["straight"])
    for hdr, lp in res["loops"].items():
        for c, n in lp["valu"].items():
            tot[c] += n * mult(hdr)
    return sum(tot.values()), tot


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("kernel")
    ap.add_argument("--trips", nargs="*", default=[], help="HDR=N, e.g. BB3_2=6")
    ap.add_argument("--blocks", action="store_true", help="list every basic block (VALU, v_mov, loop)")
    a = ap.parse_args()
    res = parse(a.asm, a.kernel)
    if a.blocks:
        for b in res["blocks"]:
            print(f"{b['name']:>10} loop={b['loop'] or ('header' if b['header_of'] else '-'):>8} "
                  f"valu={sum(b['valu'].values()):5d} mov={b['valu'].get('mov', 0):4d}")
    out = {"kernel": res["kernel"], "straight_valu": sum(res["straight"].values()),
           "loops": {h: {"parent": lp["parent"], "valu": sum(lp["valu"].values()), "mix": dict(lp["valu"])}
                     for h, lp in res["loops"].items()}}
    if a.trips:
        trips = {k: int(v) for k, v in (t.split("=") for t in a.trips)}
        n, mix = dynamic(res, trips)
        out["trips"] = trips
        out["dynamic_valu_per_item"] = n
        out["dynamic_mix"] = dict(mix)
    json.dump(out, sys.stdout)
    print()
    return 0


if __name__ == "__main__":
    sys.exit(main())
