"""Static check of the gfx950 ISA: no s_barrier inside an exec-divergent loop.

A loop that is exited per lane (the latch clears finished lanes from exec:
`s_andn2_b64 exec, exec, ...` + `s_cbranch_execz <exit>`, or loops back with
`s_cbranch_execnz`) and that contains `s_barrier` lets a wave execute a
barrier for a subset of its lanes, which desynchronises the workgroup (a
hang).  Loops are recovered from the compiler's own annotations (`Loop
Header`, `in Loop: Header=`, `Child Loop`).
Usage: check_barrier_loops.py kernel.s   (exit status 1 on any hazard)
"""
import collections
import re
import sys


def functions(asm: str):
    for m in re.finditer(r"\n(_Z\w+):\s*(?:;[^\n]*)?\n", asm):
        end = asm.find(".Lfunc_end", m.end())
        yield m.group(1), asm[m.end():end].split("\n")


def blocks(lines):
    """[(label, [lines])] in layout order; the entry block is 'entry'."""
    out, cur, buf = [], "entry", []
    for l in lines:
        m = re.match(r"^\.?(LBB\w+):", l) or re.match(r"^; %bb\.(\d+):", l)
        if m:
            out.append((cur, buf))
            cur = m.group(1) if m.group(1).startswith("LBB") else f"bb{m.group(1)}"
            buf = [l]
        else:
            buf.append(l)
    out.append((cur, buf))
    return out


def hazards(lines):
    blks = blocks(lines)
    member = collections.defaultdict(set)   # header -> blocks
    children = collections.defaultdict(set)
    for name, body in blks:
        text = "\n".join(body[:40])
        for h in re.findall(r"in Loop: Header=(BB\w+)", text):
            member["L" + h].add(name)
        if "Loop Header" in text:
            member[name].add(name)
            for c in re.findall(r"Child Loop (BB\w+)", text):
                children[name].add("L" + c)

    def all_blocks(h, seen=None):
        seen = seen or set()
        if h in seen:
            return set()
        seen.add(h)
        s = set(member[h])
        for c in children[h]:
            s |= all_blocks(c, seen)
        return s

    body_of = dict(blks)
    out = []
    for h in list(member):
        bl = all_blocks(h)
        own = member[h]  # the loop's own blocks (not nested loops)
        divergent = False
        for b in own:
            code = body_of.get(b, [])
            for i, l in enumerate(code):
                if re.search(r"s_cbranch_execnz\s+\.(\w+)", l):
                    tgt = re.search(r"s_cbranch_execnz\s+\.(\w+)", l).group(1)
                    if tgt == h:
                        divergent = True
                m = re.search(r"s_cbranch_execz\s+\.(\w+)", l)
                if m and m.group(1) not in bl and any(
                        re.search(r"s_andn2_b64\s+exec,\s*exec", x) for x in code[max(0, i - 3):i]):
                    divergent = True
        has_barrier = any("s_barrier" in x for b in bl for x in body_of.get(b, []))
        if divergent and has_barrier:
            out.append(h)
    return out


def main(path):
    asm = open(path).read()
    bad = 0
    for name, lines in functions(asm):
        hz = hazards(lines)
        if hz:
            bad += 1
            print(f"HAZARD {name[:90]}: exec-divergent loops containing s_barrier: {hz[:6]}")
    print("checked", path, "hazardous kernels:", bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
