"""HBM bytes per kernel launch from two rocprofv3 PMC passes.

Usage: pmc_traffic.py FETCH_CSV WRITE_CSV RECORDS OUT_JSON [CAL_FETCH_CSV CAL_WRITE_CSV CAL_JSON]

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch.  MI355X_MICROARCH.md:
FETCH_SIZE reports half the bytes of 16-B/lane coalesced streaming reads and
other widths are uncalibrated.  With the calibration passes
(tools/calib_fetch.hip: known byte counts read 8 B/lane, 16 B/lane, as random
8-B gathers, and written 8 B/lane) the factor bytes / FETCH_SIZE measured for
8-B/lane streaming loads -- the width every dpg kernel loads with -- is
applied (and the write factor likewise); without them the guide's 2x is used.
Infinity-Cache hits are counted by these counters, i.e. the figure is "bytes
leaving L2", an upper bound on HBM traffic.  The JSON records the library
hash, so bench.py reports it only for the build it was measured on.
"""
import collections
import csv
import hashlib
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
UNTIMED = ("k_pid_minmax",)


def short(name: str) -> str:
    # same naming as bench.py's dominant-kernel map: k_scatter<SrcSoAKey>, ...
    m = re.search(r"(?:dpg::)?(k_\w+)(<(?:dpg::)?(\w+))?", name)
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


def calibration(cf, cw, cj):
    """Factors true_bytes / counter_bytes per access form (per launch)."""
    known = json.load(open(cj))
    f = per_kernel(cf, "FETCH_SIZE")
    w = per_kernel(cw, "WRITE_SIZE")
    out = {"read8": known["read_bytes"] / f["k_read8"][1],
           "read16": known["read_bytes"] / f["k_read16"][1],
           "gather8_bytes_per_read": f["k_gather8"][1] / known["gather_reads"],
           "write8": known["write_bytes"] / w["k_write8"][1]}
    out["raw"] = {k: v[1] for k, v in list(f.items()) + [("k_write8:WRITE", w["k_write8"])]}
    return out


def lib_sha() -> str:
    with open(os.path.join(ROOT, "pipelinedp_amd", "lib", "libdpg.so"), "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def main(fetch_csv, write_csv, records, out, cal_f=None, cal_w=None, cal_j=None):
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    cal = calibration(cal_f, cal_w, cal_j) if cal_f else None
    rf = cal["read8"] if cal else 2.0
    wf = cal["write8"] if cal else 1.0
    kernels, raw = {}, {}
    for k in sorted(set(f) | set(w)):
        if not k.startswith("k_"):
            continue
        fb = f.get(k, (0, 0.0))[1]
        wb = w.get(k, (0, 0.0))[1]
        kernels[k] = rf * fb + wf * wb
        raw[k] = {"fetch_size_bytes": fb, "write_size_bytes": wb,
                  "launches": max(f.get(k, (0,))[0], w.get(k, (0,))[0])}
    # kernels of bench.py's untimed calls only: the privacy-id range pass
    # (kernels.pidrange_untimed in the bench line; the timed calls declare
    # the range) is not part of a step
    untimed = {k: v for k, v in kernels.items() if k in UNTIMED}
    res = {"records": int(records), "lib_sha256": lib_sha(),
           "correction": (f"{rf:.3f} x FETCH_SIZE + {wf:.3f} x WRITE_SIZE (factors measured "
                          f"on 8-B/lane streaming loads / stores, tools/calib_fetch.hip)"
                          if cal else "2 x FETCH_SIZE + WRITE_SIZE (guide's 16-B/lane rule)"),
           "calibration": cal, "kernels": kernels, "raw": raw,
           "untimed_kernels": sorted(untimed),
           "bytes_per_step": sum(v for k, v in kernels.items() if k not in UNTIMED)}
    json.dump(res, open(out, "w"), indent=1)
    if cal:
        print("calibration:", {k: round(v, 3) for k, v in cal.items() if k != "raw"})
    for k, v in sorted(kernels.items(), key=lambda x: -x[1]):
        print(f"{k:40s} {v / 1e9:8.2f} GB/launch  ({v / int(records):6.1f} B/record)")


if __name__ == "__main__":
    main(*sys.argv[1:])
