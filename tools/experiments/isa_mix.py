"""Instruction mix of the innermost loops of each kernel in a hipcc -S listing, priced with the gfx950 VALU
issue costs measured by tools/bench_valu.hip (profiles/r1/valu_issue_rates.json).

Usage: python tools/isa_mix.py file.s [kernel-substring]
"""
import collections
import re
import sys

# wall cycles per wave64 instruction per SIMD at 8 waves/SIMD (bench_valu); "fast" VOP1/VOP2 and all-VGPR
# v_bitop3 issue every ~2 cycles, the rest of the VOP3 integer ops every ~4.
SLOW = ("v_alignbit", "v_alignbyte", "v_add3", "v_perm", "v_lshl_add", "v_lshl_or", "v_and_or", "v_or3",
        "v_bfe", "v_bfi", "v_mad", "v_dot", "v_lshrrev_b64", "v_lshlrev_b64", "v_lshl_add_u64", "v_mul_lo",
        "v_mul_hi", "v_readlane", "v_writelane")


def cost(op: str, line: str) -> float:
    if op.startswith("v_bitop3"):
        return 4.0 if re.search(r",\s*s\d+|,\s*0x|,\s*-?\d+\s", line.split("bitop3:")[0]) else 2.0
    if op.startswith(SLOW):
        return 4.0
    return 2.0


def main() -> None:
    path = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    fn, lines = None, []
    funcs = {}
    for raw in open(path):
        m = re.match(r"^(_Z\w+):", raw)
        if m:
            fn, lines = m.group(1), []
            funcs[fn] = lines
            continue
        if fn:
            lines.append(raw.rstrip())
    for fn, body in funcs.items():
        if want not in fn:
            continue
        labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
        loops = []
        for i, l in enumerate(body):
            m = re.match(r"\s*s_cbranch_\w+\s+(\.LBB\w+)|\s*s_branch\s+(\.LBB\w+)", l)
            if m:
                tgt = m.group(1) or m.group(2)
                if tgt in labels and labels[tgt] < i:
                    loops.append((labels[tgt], i))
        inner = [lp for lp in loops if not any(o != lp and lp[0] <= o[0] and o[1] <= lp[1] for o in loops)]
        for a, b in inner:
            mix = collections.Counter()
            cyc = 0.0
            n_valu = n_lds = 0
            for l in body[a:b + 1]:
                t = l.split()
                if not t or t[0].startswith((";", ".")):
                    continue
                op = t[0]
                if op.startswith("v_"):
                    mix[op] += 1
                    n_valu += 1
                    cyc += cost(op, l)
                elif op.startswith("ds_"):
                    n_lds += 1
                    mix[op] += 1
            if n_valu < 50:
                continue
            top = ", ".join(f"{k} {v}" for k, v in mix.most_common(10))
            print(f"{fn[:60]} loop@{a}: {n_valu} VALU, {n_lds} LDS, est {cyc:.0f} SIMD-cyc "
                  f"({cyc / n_valu:.2f}/instr)\n    {top}")


if __name__ == "__main__":
    main()
