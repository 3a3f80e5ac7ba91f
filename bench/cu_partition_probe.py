#!/usr/bin/env python3
"""CU partitions on one MI355X: which hardware units a CU-masked stream's
workgroups run on (``hipExtStreamCreateWithCUMask`` bit i -> XCC / SE / CU,
read back from the HW_ID / XCC_ID registers), and the copy bandwidth a
partition of n CUs reaches (the bound of a weight-streaming micro-forward
confined to it).  One JSON line per mask.

    python bench/cu_partition_probe.py
"""
from __future__ import annotations

import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _mask(bits, ncu):
    words = [0] * ((ncu + 31) // 32)
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    return words


def main() -> int:
    import numpy as np
    import torch

    from llm_message_queue_amd import _native
    k = _native.require_hipops()
    info = k.device_info(0)
    ncu = int(info["cus"])
    torch.cuda.set_device(0)
    src = torch.empty(1 << 31, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    masks = {
        "all": list(range(ncu)),
        "bits0_15": list(range(16)),
        "bits0_31": list(range(32)),
        "bits_mod16_0": list(range(0, ncu, 16)),
        "bits_mod32_0_1": [b for b in range(ncu) if b % 32 < 2],
        "bits_mod8_0": list(range(0, ncu, 8)),
        "bits_ge_224": list(range(224, ncu)),
        "bits_lt_224": list(range(224)),
        "bits_ge_240": list(range(240, ncu)),
    }
    for name, bits in masks.items():
        s = k.stream_with_cu_mask(_mask(bits, ncu))
        try:
            raw = np.asarray(k.hw_probe(8192, 20000, s), dtype=np.uint32).reshape(-1, 2)
            hw, xcc = raw[:, 0], raw[:, 1] & 0xF
            cu, sh, se = (hw >> 8) & 0xF, (hw >> 12) & 1, (hw >> 13) & 0x7
            units = set(zip(xcc.tolist(), se.tolist(), sh.tolist(), cu.tolist()))
            per_xcc = {int(x): len({u for u in units if u[0] == x}) for x in sorted(set(xcc.tolist()))}
            st = torch.cuda.ExternalStream(s)
            with torch.cuda.stream(st):
                for _ in range(2):
                    k.copy_bytes(dst.data_ptr(), src.data_ptr(), src.numel(), s)
                st.synchronize()
                t0 = time.perf_counter()
                n = 5
                for _ in range(n):
                    k.copy_bytes(dst.data_ptr(), src.data_ptr(), src.numel(), s)
                st.synchronize()
                dt = (time.perf_counter() - t0) / n
            print(json.dumps({"mask": name, "bits": len(bits), "distinct_units": len(units), "per_xcc": per_xcc,
                              "copy_gb_s": round(2 * src.numel() / dt / 1e9, 1)}), flush=True)
        finally:
            k.stream_destroy(s)
    return 0


if __name__ == "__main__":
    sys.exit(main())
