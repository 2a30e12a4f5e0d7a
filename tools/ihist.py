"""Instruction histogram of one kernel in a device asm file.

Usage: ihist.py ASM_FILE NAME_SUBSTRING [TOP]"""
import collections
import re
import sys


def main(path, sub, top=40):
    s = open(path).read()
    names = [n for n in re.findall(r"^(_Z\S+):", s, re.M) if sub in n]
    for name in names:
        i = s.index(name + ":")
        j = s.index(".Lfunc_end", i)
        lines = [l.strip() for l in s[i:j].split("\n")
                 if l.strip() and not l.strip().startswith((".", ";", "_"))]
        c = collections.Counter(l.split()[0] for l in lines)
        print(name[:90], len(lines))
        print("  " + ", ".join(f"{k} {v}" for k, v in c.most_common(int(top))))


if __name__ == "__main__":
    main(*sys.argv[1:])
