"""Per-kernel summary of rocprofv3 SQ counter passes.

Usage: pmc_summary.py PASS_CSV [PASS_CSV ...]

Prints, per kernel, the per-launch average of every counter seen and the
wave-cycle split (SQ_WAIT_ANY = parked on s_waitcnt / barrier,
SQ_WAIT_INST_ANY = issue stall, SQ_ACTIVE_INST_ANY = issuing; the three are
disjoint and sum to about SQ_WAVE_CYCLES, MI355X_MICROARCH.md PMC slots).
"""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    m = re.search(r"dpg::(k_\w+)(<(?:dpg::)?(\w+))?", name)
    if not m:
        return name.split("(")[0][:60]
    base = m.group(1)
    if m.group(3) and base in ("k_scatter", "k_hist", "k_reduce_items", "k_bound_chunks", "k_bound_waves",
                               "k_bound_big"):
        return f"{base}<{m.group(3)}>"
    return base


def load(paths):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main(paths):
    agg = load(paths)
    for k in sorted(agg):
        if not k.startswith("k_"):
            continue
        c = {n: sum(v) / len(v) for n, v in agg[k].items()}
        print(f"== {k}")
        for n in sorted(c):
            print(f"   {n:24s} {c[n]:16.4g}")
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if n in c:
                    print(f"   {n + ' / WAVE_CYCLES':40s} {c[n] / wc:8.3f}")
        w = c.get("SQ_WAVES")
        if w:
            for n in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
                      "SQ_INSTS_VMEM_WR"):
                if n in c:
                    print(f"   {n + ' per wave':40s} {c[n] / w:10.1f}")
        if c.get("SQ_LDS_IDX_ACTIVE"):
            print(f"   {'LDS bank-conflict cycles / LDS active':40s} "
                  f"{c.get('SQ_LDS_BANK_CONFLICT', 0.0) / c['SQ_LDS_IDX_ACTIVE']:8.3f}")


if __name__ == "__main__":
    main(sys.argv[1:])
