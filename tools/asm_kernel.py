"""Extract one kernel's ISA from a hipcc -save-temps .s and summarise instruction classes per loop.

    python tools/asm_kernel.py <file.s> <symbol-prefix> [--dump out.s]
"""
import re
import sys
from collections import Counter


def main():
    path, prefix = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(prefix) and l.split(":")[0].startswith(prefix))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    body = lines[start:end + 1]
    if "--dump" in sys.argv:
        open(sys.argv[sys.argv.index("--dump") + 1], "w").write("\n".join(body))
    insts = [l.strip().split()[0] for l in body if re.match(r"\s+[vs]_", l)]
    v = sum(1 for i in insts if i.startswith("v_"))
    s = sum(1 for i in insts if i.startswith("s_"))
    print(f"{body[0].split(':')[0]}: {len(body)} lines, VALU {v}, SALU {s}")
    # loops: label lines with 'Loop Header' comments -> count instructions until the backedge
    for i, l in enumerate(body):
        if "Loop Header" in l:
            lab = body[i - 2].split(":")[0] if body[i - 2].startswith(".LBB") else body[i].split(":")[0]
            print("  loop at", i, l.strip()[:80])
    print(Counter(i for i in insts if i.startswith("v_")).most_common(25))


if __name__ == "__main__":
    main()
