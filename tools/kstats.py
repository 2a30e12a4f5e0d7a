"""Print the top kernels of a rocprofv3 --stats CSV (name, calls, avg ms, %).

Usage: kstats.py KERNEL_STATS_CSV [N]
"""
import csv
import sys


def main(path, n="25"):
    for r in list(csv.DictReader(open(path)))[:int(n)]:
        print(f"{r['Name'][:80]:80s} {r['Calls']:>4} {float(r['AverageNs']) / 1e6:8.3f} ms "
              f"{float(r['Percentage']):6.2f} %")


if __name__ == "__main__":
    main(*sys.argv[1:])
