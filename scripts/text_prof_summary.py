"""Per-kernel mean time (us) of the preprocess chain from
`scripts/gpu_text_prof.sh <tag>` output: one line per batch size.

    python scripts/text_prof_summary.py gpurun_out/text_<tag>
"""
import csv
import os
import sys


def main(d: str) -> None:
    for b in sorted((int(x[1:]) for x in os.listdir(d) if x.startswith("b") and x[1:].isdigit())):
        path = None
        for root, _dirs, files in os.walk(os.path.join(d, f"b{b}")):
            for f in files:
                if f.endswith("kernel_stats.csv"):
                    path = os.path.join(root, f)
        if path is None:
            continue
        rows = list(csv.DictReader(open(path)))
        keep = [r for r in rows if r["Name"].startswith("llmq::") or "llmq::" in r["Name"]]
        parts = sorted(((r["Name"].split("(")[0].replace("void ", "").replace("llmq::", "").split("<")[0],
                         float(r["AverageNs"]) / 1e3) for r in keep), key=lambda x: -x[1])
        print(b, " ".join(f"{n}={t:.1f}us" for n, t in parts))


if __name__ == "__main__":
    main(sys.argv[1])
