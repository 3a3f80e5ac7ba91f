"""Per-kernel PMC summary from a rocprofv3 --pmc SQLite database (the default
output format): per kernel name -> dispatches, mean duration, shader clock
(GRBM_GUI_ACTIVE summed over the 8 XCDs / 8 / duration), MFMA busy
(SQ_VALU_MFMA_BUSY_CYCLES / (GUI_ACTIVE / 8 x 1024 SIMDs)), SQ_WAIT_ANY /
SQ_WAVE_CYCLES.  usage: python scripts/pmc_db_table.py <pmc_results.db> [--match s]"""
import collections
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else "gemm"
per = collections.defaultdict(lambda: collections.defaultdict(float))
meta = {}
for disp, name, cnt, val, dur in db.execute(
        "select dispatch_id, kernel_name, counter_name, value, duration from counters_collection"):
    if match not in name:
        continue
    per[disp][cnt] += val
    meta[disp] = (name, dur)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for disp, c in per.items():
    name, dur = meta[disp]
    for k, v in c.items():
        agg[name][k].append(v)
    agg[name]["_dur"].append(dur)
print("| kernel | dispatches | mean us | clock GHz | MFMA busy | SQ_WAIT_ANY / wave cycles |")
print("|---|---:|---:|---:|---:|---:|")
for name, d in agg.items():
    m = {k: sum(v) / len(v) for k, v in d.items()}
    dur = m["_dur"]
    gui = m.get("GRBM_GUI_ACTIVE", 0)
    clk = gui / 8 / dur if dur else 0
    busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(1, gui / 8 * 1024)
    wait = m.get("SQ_WAIT_ANY", 0) / max(1, m.get("SQ_WAVE_CYCLES", 1))
    print(f"| `{name[:60]}` | {len(d['_dur'])} | {dur / 1e3:.1f} | {clk:.2f} | {busy:.1%} | {wait:.1%} |")
