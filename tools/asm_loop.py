"""Instruction mix of the innermost loops of a kernel in a hipcc --save-temps .s file.
    python tools/asm_loop.py FILE.s KERNEL_SUBSTRING [N_LOOPS]
A loop = label .LBBx_y ... backward branch to it; prints the N loops with the most VALU ops."""
import collections
import re
import sys


def main():
    path, kname = sys.argv[1], sys.argv[2]
    nshow = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and kname in l)
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    body = lines[start:end + 1]
    labels = {l.split(":")[0]: i for i, l in enumerate(body) if l.startswith(".LBB")}
    loops = []
    for i, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)", l) or re.search(r"s_branch\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            seg = body[labels[m.group(1)]:i + 1]
            ops = [s.split()[0] for s in seg if s.strip() and not s.strip().startswith((";", ".")) and s.startswith("\t")]
            c = collections.Counter(ops)
            valu = sum(v for k, v in c.items() if k.startswith("v_"))
            inner = not any(re.search(r"s_c?branch\w*\s+(\.LBB\w+)", x) and
                            labels.get(re.search(r"s_c?branch\w*\s+(\.LBB\w+)", x).group(1), -1) > labels[m.group(1)]
                            and body.index(x) < i for x in seg[1:-1])
            if inner or "--all" in sys.argv:
                loops.append((valu, m.group(1), c, len(ops)))
    loops.sort(key=lambda x: -x[0])
    for valu, lab, c, n in loops[:nshow]:
        print(f"loop {lab}: {n} instrs, {valu} VALU")
        for k, v in c.most_common():
            print(f"  {v:4d} {k}")


if __name__ == "__main__":
    main()
