"""Compact map of one kernel's device asm: labels (with loop depth), vector
memory ops, scratch spills / reloads, s_waitcnt vmcnt, barriers and LDS
atomics, consecutive duplicates folded.  Shows where a kernel drains its
memory pipeline (a scratch reload or a dynamic-count loop forces
`s_waitcnt vmcnt(0)`, which also waits for every older store and load).

Usage: loopmap.py ASM_FILE NAME_SUBSTRING
"""
import re
import sys

KEEP = re.compile(r"^\s*(scratch_|global_|buffer_|s_waitcnt\s+vmcnt|s_barrier|ds_add|s_endpgm|"
                  r"s_branch|s_cbranch)")


def main(path, sub):
    lines = open(path).read().split("\n")
    start = None
    for i, ln in enumerate(lines):
        m = re.match(r"^(_Z\S+):", ln)
        if m and sub in m.group(1) and not ln.startswith("\t"):
            start = i
            print(m.group(1)[:100])
            break
    if start is None:
        sys.exit(f"no kernel matching {sub}")
    prev, n = None, 0
    out = []
    for ln in lines[start + 1:]:
        if re.match(r"^\s*\.Lfunc_end", ln):
            break
        lab = re.match(r"^(\.LBB\S+):.*?(Loop Header: Depth=\d+|Depth=\d+)?\s*$", ln)
        if lab:
            item = f"{lab.group(1)} {lab.group(2) or ''}"
        elif KEEP.match(ln):
            item = "    " + re.sub(r"\s+", " ", ln.strip())
            item = re.sub(r"v\[\d+:\d+\]|v\d+", "v", item)
            item = re.sub(r"s\[\d+:\d+\]", "s", item)
        else:
            continue
        if item == prev:
            n += 1
            continue
        if prev is not None:
            out.append(prev + (f"  x{n}" if n > 1 else ""))
        prev, n = item, 1
    if prev is not None:
        out.append(prev + (f"  x{n}" if n > 1 else ""))
    print("\n".join(out))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
