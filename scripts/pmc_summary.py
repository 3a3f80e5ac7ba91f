"""Summarise rocprofv3 --pmc counter CSVs: mean per dispatch, per kernel.
usage: python scripts/pmc_summary.py <csv>... [--match substr]"""
import collections
import csv
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
by_grid = "--by-grid" in sys.argv
match = None
if "--match" in sys.argv:
    match = sys.argv[sys.argv.index("--match") + 1]
    args.remove(match)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in args:
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"]
        if match and match not in k:
            continue
        key = k[:90] + (f"  grid={r.get('Grid_Size', r.get('Grid_Size_X', '?'))}" if by_grid else "")
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"    {c:28s} {sum(v) / len(v):12.4g}  (n={len(v)})")
