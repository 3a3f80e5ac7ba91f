"""CU partitions of one MI355X (``backend.micro_stream = partition``): the
serving steps and the realtime micro-forwards each get streams whose kernels
may only run on their own set of CUs (``hipExtStreamCreateWithCUMask``), so a
micro-forward never waits for a serving GEMM's workgroups to drain.

Mask layout, measured (``bench/cu_partition_probe.py`` ->
``profiles/r6_cu_partition_probe.jsonl``): mask bit i is a CU of XCD i mod 8
-- consecutive bits go round-robin over the eight XCDs -- so any contiguous
range of bits is balanced over the XCDs (bits 224-255: 4 CUs on every XCD).
The micro partition takes the top ``micro_cus`` bits, the serving steps the
rest; their GEMM wave plans use the smaller CU count (``ops.gemm.EFFECTIVE_CUS``).
Copy bandwidth of a partition (same probe): 16 CUs 0.86 TB/s, 32 CUs
1.45 TB/s, 224 CUs 4.15 TB/s, the chip 4.56 TB/s (read + write).
"""
from __future__ import annotations

from typing import Tuple


def mask_words(bits, ncu: int):
    words = [0] * ((ncu + 31) // 32)
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    return words


_STREAMS = {}


def partition_streams(device, micro_cus: int) -> Tuple[object, object, int]:
    """(serving stream, micro stream, serving CU count) on ``device``.

    The streams live for the process, one pair per (device, micro_cus),
    shared by every engine that asks: blocks of PyTorch's caching allocator
    stay associated with the stream that allocated them, so a tensor freed
    after its stream was destroyed would record an event on a dead stream
    (a segfault in the deallocation).  PyTorch never destroys its own pool
    streams for the same reason."""
    import torch
    from .. import _native
    k = _native.require_hipops()
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, int(micro_cus))
    got = _STREAMS.get(key)
    if got is not None:
        return got
    ncu = int(k.device_info(idx)["cus"])
    if micro_cus % 8 or not 8 <= micro_cus <= ncu // 2:
        raise ValueError(f"micro_cus must be a multiple of 8 (one per XCD) in [8, {ncu // 2}], not {micro_cus}")
    big = ncu - micro_cus
    with torch.cuda.device(idx):
        hs = k.stream_with_cu_mask(mask_words(range(big), ncu))
        hm = k.stream_with_cu_mask(mask_words(range(big, ncu), ncu))
    dev = torch.device("cuda", idx)
    got = _STREAMS[key] = (torch.cuda.ExternalStream(hs, device=dev), torch.cuda.ExternalStream(hm, device=dev), big)
    return got


def release_streams() -> None:
    """Destroy the process's partition streams -- only when no tensor
    allocated on them can be freed later: the caller dropped every engine
    and tensor first.  The GPU is drained and the allocator's cached blocks
    released before the streams go (a profiler's exit-time teardown then
    finds no live external stream)."""
    if not _STREAMS:
        return
    import gc

    import torch
    from .. import _native
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    k = _native.require_hipops()
    for big, micro, _n in list(_STREAMS.values()):
        for st in (big, micro):
            k.stream_destroy(st.cuda_stream)
    _STREAMS.clear()
