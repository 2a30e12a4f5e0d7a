"""Barrier context and instruction mix of one kernel in a device asm file.

Usage: isa_scan.py ASM_FILE KERNEL_SYMBOL_PREFIX
"""
import sys

s = open(sys.argv[1]).read().split("\n")
pre = sys.argv[2]
st = next(i for i, l in enumerate(s) if l.startswith(pre) and l.split(" ")[0].endswith(":"))
en = next(i for i in range(st, len(s)) if s[i].startswith(".Lfunc_end"))
body = [l.strip() for l in s[st:en]]
print(en - st, "lines")
for k, l in enumerate(body):
    if l.startswith("s_barrier"):
        print(k, " | ".join(body[max(0, k - 4):k + 1]))
cnt = {}
for l in body:
    t = l.split(" ")[0]
    if t.startswith(("v_", "s_", "ds_", "global_", "buffer_", "scratch_")):
        cnt[t] = cnt.get(t, 0) + 1
print(sorted(cnt.items(), key=lambda x: -x[1])[:40])
