"""Static instruction mix of one kernel in a device asm file.

Usage: asm_mix.py ASM_FILE NAME_SUBSTRING [TOP]
"""
import collections
import re
import sys


def main(path, sub, top=40):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if l.endswith(":") and sub in l and not l.startswith((".", "\t")) and "@" not in l.split(":")[0]:
            start = i
            break
        if re.match(r"^\S+:\s*;\s*@", l) and sub in l:
            start = i
            break
    if start is None:
        sys.exit("kernel not found")
    ins = []
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        t = l.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        ins.append(t.split()[0])
    c = collections.Counter(ins)
    print("instructions", len(ins))
    for k, v in c.most_common(int(top)):
        print(f"  {k:32s}{v}")


if __name__ == "__main__":
    main(*sys.argv[1:])
