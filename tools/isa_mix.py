"""VALU instruction mix of a kernel's innermost loops, weighted by measured gfx950 issue costs.

    python tools/isa_mix.py <file.s> <symbol-prefix>

Costs (SIMD cycles per wave64 instruction, all SIMDs busy, 8 waves/SIMD) are the
tools/valu_rates.hip measurements committed in profiles/r01_valu_rates.txt.
"""
import re
import sys

FAST = {"v_xor_b32", "v_add_u32", "v_and_b32", "v_or_b32", "v_bitop3_b32", "v_sub_u32", "v_mov_b32", "v_lshrrev_b32"}
COST_FAST, COST_SLOW = 2.85, 4.4


def op(line):
    t = line.strip().split()
    return t[0] if t and re.match(r"v_", t[0]) else None


def main():
    path, prefix = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(prefix))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    body = lines[start:end]
    # innermost loops: from a label line followed by 'Inner Loop Header' to its backward branch
    loops = []
    for i, l in enumerate(body):
        if "Inner Loop Header" in l:
            lab = body[i - 1].split(":")[0] if body[i - 1].startswith(".LBB") else None
            if lab is None:
                continue
            j = next((k for k in range(i, len(body)) if re.search(r"s_cbranch_\w+\s+" + re.escape(lab) + r"\b", body[k])), None)
            if j:
                loops.append((lab, body[i:j + 1]))
    for lab, blk in loops:
        ops = [o for o in (op(l) for l in blk) if o]
        fast = sum(1 for o in ops if o.split("_e")[0] in FAST or o.rsplit("_e", 1)[0] in FAST)
        slow = len(ops) - fast
        cyc = fast * COST_FAST + slow * COST_SLOW
        print(f"{lab}: VALU {len(ops)} (fast {fast}, slow {slow}) -> {cyc:.0f} issue cycles, "
              f"{cyc / max(len(ops), 1):.2f} per instruction")


if __name__ == "__main__":
    main()
