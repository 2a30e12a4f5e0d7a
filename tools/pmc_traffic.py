"""HBM bytes per kernel launch from two rocprofv3 PMC passes.

Usage: pmc_traffic.py FETCH_CSV WRITE_CSV RECORDS OUT_JSON

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE
reports half the bytes of wide (16 B/lane) coalesced streaming reads
(MI355X_MICROARCH.md, HBM section), so it is doubled; WRITE_SIZE is taken as
is.  Infinity-Cache hits are counted by these counters, i.e. the figure is
"bytes leaving L2", an upper bound on HBM traffic.
"""
import collections
import csv
import json
import re
import sys


def short(name: str) -> str:
    # same naming as bench.py's dominant-kernel map: k_scatter<SrcSoAKey>, ...
    m = re.search(r"dpg::(k_\w+)(<(?:dpg::)?(\w+))?", name)
    if not m:
        return name.split("(")[0][:60]
    base = m.group(1)
    if m.group(3) and base in ("k_scatter", "k_hist", "k_reduce_items"):
        return f"{base}<{m.group(3)}>"
    return base


def per_kernel(path, counter):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = short(r["Kernel_Name"])
        agg[k][0] += 1
        agg[k][1] += float(r["Counter_Value"])
    return {k: (n, v / n * 1024.0) for k, (n, v) in agg.items()}


def main(fetch_csv, write_csv, records, out):
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    kernels, raw = {}, {}
    for k in sorted(set(f) | set(w)):
        if not k.startswith("k_"):
            continue
        fb = f.get(k, (0, 0.0))[1]
        wb = w.get(k, (0, 0.0))[1]
        kernels[k] = 2.0 * fb + wb
        raw[k] = {"fetch_size_bytes": fb, "write_size_bytes": wb,
                  "launches": max(f.get(k, (0,))[0], w.get(k, (0,))[0])}
    res = {"records": int(records), "correction": "2 x FETCH_SIZE + WRITE_SIZE (gfx950)",
           "kernels": kernels, "raw": raw,
           "bytes_per_step": sum(kernels.values())}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in sorted(kernels.items(), key=lambda x: -x[1]):
        print(f"{k:40s} {v / 1e9:8.2f} GB/launch  ({v / int(records):6.1f} B/record)")


if __name__ == "__main__":
    main(*sys.argv[1:5])
