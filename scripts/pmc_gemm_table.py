"""GEMM PMC table from rocprofv3 --pmc CSVs: per (kernel, grid) -> calls,
GRBM_GUI_ACTIVE, MFMA busy, SQ_WAIT_ANY / wave cycles, LDS conflict share,
L2 hit.  MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GUI_ACTIVE / 8 XCDs x 256
CUs x 4 SIMDs).  usage: python scripts/pmc_gemm_table.py <csv>... [--match s]"""
import collections
import csv
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else None
if match:
    args.remove(match)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
names = {}
for p in args:
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"]
        if not any(s in k for s in ("gemm", "Cijk")) or (match and match not in k):
            continue
        key = (k[:70], r.get("Grid_Size", "?"))
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
print("| kernel | grid | GUI_ACTIVE (sum XCDs) | MFMA busy | SQ_WAIT_ANY / wave cycles | LDS conflict / LDS active | L2 hit |")
print("|---|---:|---:|---:|---:|---:|---:|")
for (k, g), d in sorted(agg.items(), key=lambda kv: -max(kv[1].get("GRBM_GUI_ACTIVE", [0]))):
    m = {c: sum(v) / len(v) for c, v in d.items()}
    gui = m.get("GRBM_GUI_ACTIVE", 0)
    busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1, gui / 8 * 1024)
    wait = m.get("SQ_WAIT_ANY", 0) / max(1, m.get("SQ_WAVE_CYCLES", 1))
    lds = m.get("SQ_LDS_BANK_CONFLICT", 0) / max(1, m.get("SQ_LDS_IDX_ACTIVE", 1))
    h, mi = m.get("TCC_HIT_sum", 0), m.get("TCC_MISS_sum", 0)
    l2 = h / max(1, h + mi)
    print(f"| `{k}` | {g} | {gui / 1e6:.3f} M | {busy:.1%} | {wait:.1%} | {lds:.1%} | {l2:.1%} |")
