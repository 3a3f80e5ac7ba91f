"""Per-kernel PMC table for the round-5 preprocess / summarise kernel passes
(scripts/gpu_r5_kernel_pmc.sh): one row per (config, kernel) with the mean
per dispatch of each counter, merged over the four counter passes.

usage: python scripts/kpmc_table.py gpurun_out/r5_kpmc > table.md

Derived columns (MI355X: 8 XCDs, 256 CUs, 1024 SIMDs; the guide's rules):
  dur_us      mean End-Start of the dispatch in the WRITE_SIZE pass (one
              counter, least perturbed)
  clk_GHz     GRBM_GUI_ACTIVE / 8 / duration (reads high below ~0.3 ms)
  mfma_chip   SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024):
              fraction of the whole chip's matrix-core cycles
  lds_confl   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  MB          (FETCH_SIZE + WRITE_SIZE) KiB -> MB moved to/from L2/memory
  GB/s        MB / duration
"""
import collections
import csv
import os
import sys

PASSES = ("mfma", "lds", "fetch", "write")
SKIP = ("__amd_rocclr", "at::native::")


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("llmq::", "")
    return n


def load(root, cfg):
    cnt = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for p in PASSES:
        path = os.path.join(root, f"{cfg}_{p}", "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        per_disp = collections.defaultdict(lambda: collections.defaultdict(float))
        meta = {}
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"]
            if k.startswith(SKIP) or any(s in k for s in SKIP):
                continue
            d = r["Dispatch_Id"]
            per_disp[d][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[d] = (short(k), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), int(r["Grid_Size"]))
        for d, cs in per_disp.items():
            k, ns, grid = meta[d]
            key = (k, grid)
            for c, v in cs.items():
                cnt[key][c].append(v)
            if p == "write":
                dur[key].append(ns)
    return cnt, dur


def mean(xs):
    return sum(xs) / len(xs) if xs else float("nan")


def rows(root, cfg):
    cnt, dur = load(root, cfg)
    out = []
    for key, cs in cnt.items():
        m = {c: mean(v) for c, v in cs.items()}
        ns = mean(dur.get(key, []))
        gui = m.get("GRBM_GUI_ACTIVE", float("nan"))
        mfma = m.get("SQ_VALU_MFMA_BUSY_CYCLES", float("nan"))
        mb = (m.get("FETCH_SIZE", 0.0) + m.get("WRITE_SIZE", 0.0)) * 1024 / 1e6
        out.append(dict(
            kernel=key[0], grid=key[1], dur_us=ns / 1e3,
            clk_GHz=gui / 8 / ns if ns == ns and ns > 0 else float("nan"),
            waves=m.get("SQ_WAVES", float("nan")),
            mfma_chip=mfma / (gui / 8 * 1024) if gui == gui and gui > 0 else float("nan"),
            mfma_mops=m.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", float("nan")),
            lds_confl=(m.get("SQ_LDS_BANK_CONFLICT", 0.0) / m["SQ_LDS_IDX_ACTIVE"]
                       if m.get("SQ_LDS_IDX_ACTIVE") else 0.0),
            lds_insts=m.get("SQ_INSTS_LDS", float("nan")),
            fetch_MB=m.get("FETCH_SIZE", float("nan")) * 1024 / 1e6,
            write_MB=m.get("WRITE_SIZE", float("nan")) * 1024 / 1e6,
            GBps=mb / (ns / 1e3) * 1e3 if ns == ns and ns > 0 else float("nan"),
        ))
    out.sort(key=lambda r: -r["dur_us"] if r["dur_us"] == r["dur_us"] else 0)
    return out


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/r5_kpmc"
    cfgs = sorted({d.rsplit("_", 1)[0] for d in os.listdir(root)
                   if os.path.isdir(os.path.join(root, d)) and d.rsplit("_", 1)[-1] in PASSES},
                  key=lambda c: (c.rstrip("0123456789"), int("".join(ch for ch in c if ch.isdigit()) or 0)))
    cols = ["grid", "dur_us", "clk_GHz", "waves", "mfma_chip", "TFLOPs", "lds_confl", "fetch_MB", "write_MB",
            "GBps", "FLOP_per_B"]
    by_kernel = collections.defaultdict(list)
    for cfg in cfgs:
        for r in rows(root, cfg):
            fl = r["mfma_mops"] * 512 if r["mfma_mops"] == r["mfma_mops"] else 0.0   # 512 FLOP per MOPS unit
            mb = r["fetch_MB"] + r["write_MB"]
            r["TFLOPs"] = fl / (r["dur_us"] * 1e6) if fl else 0.0
            r["FLOP_per_B"] = fl / (mb * 1e6) if fl and mb else 0.0
            by_kernel[r["kernel"]].append((cfg, r))
    for k, rs in by_kernel.items():
        print(f"\n### `{k}`\n")
        print("| config | " + " | ".join(cols) + " |")
        print("|---" * (len(cols) + 1) + "|")
        for cfg, r in rs:
            vals = []
            for c in cols:
                v = r[c]
                if isinstance(v, float):
                    v = ("%.1f%%" % (100 * v)) if c in ("mfma_chip", "lds_confl") else (
                        "%.0f" % v if c == "waves" else "%.3g" % v if abs(v) < 100 else "%.0f" % v)
                vals.append(str(v))
            print(f"| {cfg} | " + " | ".join(vals) + " |")


if __name__ == "__main__":
    main()
