"""Fixed-width int32 rows the ranks exchange in every tick's all_to_all
(``parallel.comm``): request descriptors a router hands to another GPU,
completion / failure / abort records owed back to the origin router, KV
migration orders and cancels.  int64 fields travel as (lo, hi) int32 pairs.
The reference has no inter-service transport at all: its binaries do not
share queues."""
from __future__ import annotations

import numpy as np

# --------------------------------------------------------------------------- descriptors
K_DISPATCH, K_DONE, K_FAIL = 1, 2, 3     # K_FAIL: an evacuating backend hands a request back
K_MIGRATE = 4       # [kind, conv lo/hi, dest]: to a conversation's home GPU -- send its KV to dest this tick
# a backend aborted a request in flight: its processing deadline passed /
# its origin cancelled it (completion-record layout, owed like K_DONE)
K_TIMEOUT, K_CANCELLED = 5, 6
# K_FAIL's admitted field: the backend failed while running the request
# (the origin retries with backoff) / it never ran there (requeued as is)
FAIL_UNTOUCHED, FAIL_FAILED = 0, 1
K_CANCEL = 7        # [kind, handle lo/hi, origin]: origin -> the GPU running its request: abort it
# origin -> the GPU it dispatched a dialog turn to, one tick after the
# K_DISPATCH row: the dialog's real token history for a non-resident replay,
# HIST_SPAN tokens a row in the payload columns: [kind, handle lo/hi, origin,
# offset, ..., n (col 10), ..., history length (col 14), prefix length (col 15)];
# the payload is the compressed-context prefix (N5 salient tokens) then the history
K_HIST = 8
# completion records (K_DONE) carry the turn's generated token ids in the
# payload columns, their count in col 10 (dialog turns: the origin's history)
DESC_HDR = 17       # [kind, handle lo/hi, origin, tier, arrival lo/hi, enq lo/hi, gen, plen, flags, conv lo/hi,
#                    dialog history length, decision - enq (us), processing timeout (ms)];
#                    flags = (home GPU + 1) | KV_MIGRATE | DIALOG_TURN
KV_MIGRATE = 1 << 8     # descriptor flag: hold the turn until its KV arrives from the home GPU
DIALOG_TURN = 1 << 9    # descriptor flag: a conversation turn -- its generated ids go back with K_DONE


def conv_key(conversation_id: str) -> int:
    """63-bit key of a conversation id (KV residency / affinity)."""
    if not conversation_id:
        return -1
    import hashlib
    return int.from_bytes(hashlib.blake2b(conversation_id.encode(), digest_size=8).digest(), "little") >> 1


def _put64(buf: np.ndarray, col: int, vals) -> None:
    """Store int64 ``vals`` into int32 columns (col, col + 1) = (lo, hi) of
    ``buf`` [n][width] (little-endian: an int64 viewed as two int32s)."""
    buf[:, col:col + 2] = np.asarray(vals, dtype=np.int64).reshape(-1, 1).view(np.int32)


def _get64(buf: np.ndarray, col: int) -> np.ndarray:
    """int64 from int32 columns (col, col + 1) = (lo, hi) of ``buf`` [n][width]."""
    return np.ascontiguousarray(buf[:, col:col + 2]).view(np.int64).reshape(-1)
