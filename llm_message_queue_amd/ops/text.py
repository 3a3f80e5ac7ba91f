"""GPU preprocess pipeline: ``text_analyze`` (N1-N3) + ``embed_pool`` /
``classify_head`` (N4) HIP kernels, driven from PyTorch-ROCm.

One ``TextPipeline.run(contents, patterns)`` call does, on the current HIP
stream:
  1. pack the micro-batch's UTF-8 bytes + offsets into a pinned staging
     buffer and copy them to the device in one transfer;
  2. ``text_analyze`` -> per-message stats [B,16] + token hashes [B,L];
  3. ``scan_rows`` -> compacted token row offsets;
  4. ``embed_pool`` -> pooled [B,H] (bf16 MFMA GEMM over gathered rows);
  5. ``classify_head`` -> logits [B,8], predicted priority;
  6. one D2H copy of stats + predictions (one sync per micro-batch).
Pooled vectors and hashes stay on the device for context summarisation (N5).
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .. import _native
from ..preprocess import oracle

MAX_PATTERNS = 32
STAT_COLS = 16
ST_WORDS, ST_POS, ST_NEG, ST_QUESTION, ST_FLAGS, ST_NTOK, ST_SCORES = 0, 1, 2, 3, 4, 5, 8
ST_BEST_SLOT, ST_CODE = 6, 7          # kernel-side decisions (text_kernels.h)
FLAG_FOLD = 1
_SENT = ("neutral", "positive", "negative", "neutral")
_QS = ("false", "true")
_SENT_A = np.array(_SENT, dtype=object)
_QS_A = np.array(_QS, dtype=object)
SMALL_BATCH = 40                      # below: per-row Python beats numpy's fixed cost


def _has_border(b: bytes) -> bool:
    n = len(b)
    return any(b[:k] == b[n - k:] for k in range(1, n))


def gpu_eligible(p) -> bool:
    """Literal patterns the kernel matches exactly (see text_kernels.h)."""
    if not isinstance(p, oracle.LiteralPattern):
        return False
    if "�" in p.text or "\x00" in p.text:
        return False
    b = p.text.encode("utf-8")
    if not (1 <= len(b) <= 16):
        return False
    if p.ci:
        for ch in p.text:
            if ord(ch) >= 0x80 and (ch.lower() != ch or ch.upper() != ch):
                return False
            if ch in oracle.FOLD_SPECIAL:
                return False
    return True


@dataclass
class PackedPatterns:
    table: bytes
    slot_prio: List[int]                   # slot index -> priority value
    cpu_patterns: List[Tuple[int, object]]  # (slot, pattern) scored on the host
    version: int


def pack_patterns(patterns: Dict[int, list], version: int = 0) -> PackedPatterns:
    prios = sorted(patterns)
    if len(prios) > 8:
        raise ValueError("at most 8 distinct keyword priorities are supported")
    slot_of = {p: i for i, p in enumerate(prios)}
    text = np.zeros((MAX_PATTERNS, 4), dtype=np.uint32)
    mask = np.zeros((MAX_PATTERNS, 4), dtype=np.uint32)
    lens = np.zeros(MAX_PATTERNS, dtype=np.int32)
    slots = np.zeros(MAX_PATTERNS, dtype=np.int32)
    flags = np.zeros(MAX_PATTERNS, dtype=np.int32)
    n = 0
    cpu: List[Tuple[int, object]] = []
    for prio in prios:
        for p in patterns[prio]:
            if n >= MAX_PATTERNS or not gpu_eligible(p):
                cpu.append((slot_of[prio], p))
                continue
            raw = p.text.encode("utf-8")
            if p.ci:
                raw = bytes((c + 32) if 65 <= c <= 90 else c for c in raw)
            buf = raw.ljust(16, b"\x00")
            mbuf = (b"\xff" * len(raw)).ljust(16, b"\x00")
            text[n] = np.frombuffer(buf, dtype="<u4")
            mask[n] = np.frombuffer(mbuf, dtype="<u4")
            lens[n] = len(raw)
            slots[n] = slot_of[prio]
            flags[n] = (1 if p.ci else 0) | (2 if _has_border(raw) else 0)
            n += 1
    table = (text.tobytes() + mask.tobytes() + lens.tobytes() + slots.tobytes() + flags.tobytes()
             + np.int32(n).tobytes())
    return PackedPatterns(table, prios, cpu, version)


class ClassifierWeights:
    """Random-init weights of the hashed-token priority classifier (N4)."""

    def __init__(self, vocab: int = 65536, dim: int = 256, hidden: int = 1024, seed: int = 1234,
                 device="cuda"):
        import torch
        if vocab & (vocab - 1):
            raise ValueError("vocab_buckets must be a power of two")
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.vocab, self.dim, self.hidden = vocab, dim, hidden
        self.E = (torch.randn(vocab, dim, generator=g) * 0.5).to(torch.bfloat16).to(device)
        self.W1t = (torch.randn(hidden, dim, generator=g) / dim ** 0.5).to(torch.bfloat16).to(device)
        self.b1 = (torch.randn(hidden, generator=g) * 0.02).float().to(device)
        self.W2 = (torch.randn(hidden, 8, generator=g) / hidden ** 0.5).float().to(device).contiguous()
        self.b2 = torch.zeros(8, dtype=torch.float32, device=device)


def _utf8(c: str) -> bytes:
    try:
        return c.encode("utf-8")
    except UnicodeEncodeError:                         # lone surrogates -> U+FFFD (oracle.sanitize)
        return oracle.sanitize(c).encode("utf-8")


class TextResult:
    __slots__ = ("stats", "pred", "elapsed_ms", "has_classifier", "slot_prio", "extra_scores",
                 "pooled", "hashes", "L", "prompt_hashes")

    def __init__(self, stats, pred, elapsed_ms, has_classifier, slot_prio, extra_scores, pooled, hashes, L,
                 prompt_hashes=None):
        self.stats = stats
        self.pred = pred
        self.elapsed_ms = elapsed_ms
        self.has_classifier = has_classifier
        self.slot_prio = slot_prio
        self.extra_scores = extra_scores
        self.pooled = pooled      # device tensor [B, H] (or None)
        self.hashes = hashes      # device tensor [B, L] int32 view of uint32
        self.L = L
        self.prompt_hashes = prompt_hashes   # host [B, prompt_cap] uint32 (or None)

    def prompt_ids(self, j: int):
        n = min(int(self.stats[j, ST_NTOK]), self.prompt_hashes.shape[1])
        return self.prompt_hashes[j, :n]

    @property
    def word_count(self):
        return self.stats[:, ST_WORDS]

    @property
    def question(self):
        return self.stats[:, ST_QUESTION]

    @property
    def ntok(self):
        return self.stats[:, ST_NTOK]

    @property
    def fallback(self):
        return (self.stats[:, ST_FLAGS] & FLAG_FOLD) != 0

    @property
    def ml_priority(self):
        return self.pred

    def scores(self, j: int) -> Dict[int, int]:
        row = self.stats[j, ST_SCORES:ST_SCORES + 8]
        out = {p: int(row[s]) for s, p in enumerate(self.slot_prio)}
        if self.extra_scores is not None:
            for s, p in enumerate(self.slot_prio):
                out[p] += int(self.extra_scores[j, s])
        return out

    def decide(self, default_priority: int) -> Dict[str, list]:
        """Whole-batch decisions as Python lists (one numpy pass each):
        keyword priority = the oracle's ``pick_priority`` (highest strictly
        positive score, ties to the more urgent level -- slots are in
        ascending priority order, so argmax's first maximum is that level),
        sentiment, question string, fallback flag, token counts."""
        st = self.stats
        nslot = len(self.slot_prio)
        cap = self.prompt_hashes.shape[1] if self.prompt_hashes is not None else 1 << 30
        if self.extra_scores is None:
            # the kernel already picked the slot and coded sentiment / question / fold
            sp = self.slot_prio
            if len(st) <= SMALL_BATCH:
                rows = [(sp[r[6]] if r[6] >= 0 else default_priority, _SENT[r[7] & 3], _QS[(r[7] >> 2) & 1],
                         r[0], (r[7] & 8) != 0, r[5] if r[5] < cap else cap) for r in st[:, :8].tolist()]
                cols = [list(c) for c in zip(*rows)] if rows else [[] for _ in range(6)]
                return dict(zip(("priority", "sentiment", "question", "word_count", "fallback", "ntok"), cols))
            bs, code = st[:, ST_BEST_SLOT], st[:, ST_CODE]
            prio = (np.where(bs >= 0, np.asarray(sp, dtype=np.int64)[bs], default_priority) if nslot
                    else np.full(len(st), default_priority))
            return {"priority": prio.tolist(), "sentiment": _SENT_A[code & 3].tolist(),
                    "question": _QS_A[(code >> 2) & 1].tolist(), "word_count": st[:, ST_WORDS].tolist(),
                    "fallback": ((code & 8) != 0).tolist(), "ntok": np.minimum(st[:, ST_NTOK], cap).tolist()}
        out: Dict[str, list] = {}
        if nslot:
            sc = st[:, ST_SCORES:ST_SCORES + nslot].astype(np.int64)
            if self.extra_scores is not None:
                sc = sc + self.extra_scores[:, :nslot]
            best = sc.max(axis=1)
            prio = np.asarray(self.slot_prio, dtype=np.int64)[sc.argmax(axis=1)]
            out["priority"] = np.where(best > 0, prio, default_priority).tolist()
        else:
            out["priority"] = [default_priority] * len(st)
        pos, neg = st[:, ST_POS], st[:, ST_NEG]
        out["sentiment"] = np.where(pos > neg, "positive", np.where(neg > pos, "negative", "neutral")).tolist()
        out["question"] = np.where(st[:, ST_QUESTION] != 0, "true", "false").tolist()
        out["word_count"] = st[:, ST_WORDS].tolist()
        out["fallback"] = ((st[:, ST_FLAGS] & FLAG_FOLD) != 0).tolist()
        ntok = st[:, ST_NTOK]
        if self.prompt_hashes is not None:
            ntok = np.minimum(ntok, self.prompt_hashes.shape[1])
        out["ntok"] = ntok.tolist()
        return out

    def priority(self, j: int, default_priority: int) -> int:
        return oracle.pick_priority(self.scores(j), default_priority)

    def sentiment(self, j: int) -> str:
        pos, neg = self.stats[j, ST_POS], self.stats[j, ST_NEG]
        return "positive" if pos > neg else ("negative" if neg > pos else "neutral")


class TextPipeline:
    def __init__(self, cfg=None, device: str = "cuda"):
        import torch
        from ..utils.config import PreprocessorConfig
        self.torch = torch
        self.cfg = cfg or PreprocessorConfig()
        self.ops = _native.require_hipops()
        assert self.ops.PATTERN_TABLE_BYTES == 4 * (MAX_PATTERNS * 8 + MAX_PATTERNS * 3 + 1)
        self.device = torch.device(device)
        self.L = int(self.cfg.max_tokens)
        self.weights: Optional[ClassifierWeights] = None
        self._packed: Optional[PackedPatterns] = None
        self._dev_bytes = torch.empty(0, dtype=torch.uint8, device=self.device)
        self._pin = torch.empty(1 << 16, dtype=torch.uint8).pin_memory()
        self._pin_dev = self.ops.host_device_ptr(self._pin.data_ptr())
        self._rb = None                                               # pinned readback (host-mapped)
        self._rb_dev = 0
        self._ws = None                                               # reused device buffers (one-call path)
        # own HIGH-PRIORITY HIP stream: preprocess kernels run concurrently
        # with the backend forward on the default stream, and the hardware
        # scheduler dispatches their workgroups ahead of the forward's pending
        # GEMM workgroups -- otherwise every preprocess kernel queues behind a
        # full-chip GEMM and ingest latency grows with the backend's load
        self.stream = torch.cuda.Stream(device=self.device, priority=-1)
        self._sh = self.stream.cuda_stream
        self._ev = torch.cuda.Event()
        import threading
        self._inflight = threading.Lock()

    def _ensure_readback(self, n_int32: int) -> None:
        if self._rb is None or self._rb.numel() < n_int32:
            n = max(n_int32, 2 * (self._rb.numel() if self._rb is not None else 0), 1 << 14)
            self._rb = self.torch.empty(n, dtype=self.torch.int32).pin_memory()
            self._rb_dev = self.ops.host_device_ptr(self._rb.data_ptr())

    def _ensure_weights(self) -> ClassifierWeights:
        if self.weights is None:
            c = self.cfg
            # initialised on the preprocess stream (ordered before the kernels
            # that read them; see _workspace for the allocator's stream pools)
            with self.torch.cuda.stream(self.stream):
                self.weights = ClassifierWeights(c.vocab_buckets, c.embed_dim, c.hidden_dim, c.seed,
                                                 device=self.device)
        return self.weights

    def _patterns(self, patterns, version) -> PackedPatterns:
        if self._packed is None or self._packed.version != version or version < 0:
            self._packed = pack_patterns(patterns, version)
        return self._packed

    @staticmethod
    def pack(contents: Sequence[str]):
        """UTF-8 bytes + offsets for a batch (host side)."""
        n = len(contents)
        if all(c.isascii() for c in contents):        # the common case: one encode for the batch
            lens = np.fromiter(map(len, contents), dtype=np.int64, count=n)
            blob = "".join(contents).encode("ascii") + b"\x00" * 16
        else:
            enc = [_utf8(c) for c in contents]
            lens = np.fromiter(map(len, enc), dtype=np.int64, count=n)
            blob = b"".join(enc) + b"\x00" * 16
        offsets = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(lens, out=offsets[1:])
        return blob, offsets, lens

    def run(self, contents: Sequence[str], patterns: Dict[int, list], version: int = -1,
            classify: bool = True, keep_device: bool = False, prompt_cap: int = 0) -> TextResult:
        return self.collect(self.launch(contents, patterns, version, classify, keep_device, prompt_cap))

    def launch(self, contents: Sequence[str], patterns: Dict[int, list], version: int = -1,
               classify: bool = True, keep_device: bool = False, prompt_cap: int = 0):
        """Enqueue the whole chain (H2D, kernels, readback into host-mapped
        memory, event) and return at once; ``collect`` waits and decodes.  The
        staging and readback buffers are single-buffered: collect a launch
        before the next one (``ready`` tells whether ``collect`` would
        block)."""
        # one launch in flight per pipeline (single-buffered staging): a
        # second caller -- e.g. the HTTP micro-batcher thread next to the
        # serve loop -- waits here until the first batch is collected
        self._inflight.acquire()
        try:
            if not keep_device and contents:       # serve-loop path: explicit stream handle, no context switch
                return self._launch(contents, patterns, version, classify, False, prompt_cap)
            with self.torch.cuda.stream(self.stream):
                return self._launch(contents, patterns, version, classify, keep_device, prompt_cap)
        except BaseException:
            self._inflight.release()
            raise

    @staticmethod
    def ready(pend) -> bool:
        return pend["event"].query()

    def collect(self, pend) -> TextResult:
        try:
            pend["event"].synchronize()
        finally:
            self._inflight.release()
        B, cap, o_pred, o_ph = pend["B"], pend["cap"], pend["o_pred"], pend["o_ph"]
        rbn = self._rb.numpy()
        stats_h = rbn[:B * STAT_COLS].reshape(B, STAT_COLS).copy()
        pred_h = rbn[o_pred:o_pred + B].copy() if pend["pred"] is not None else None
        ph = rbn[o_ph:o_ph + B * cap].reshape(B, cap).view(np.uint32).copy() if cap else None
        extra = None
        pk, contents = pend["pk"], pend["contents"]
        if pk.cpu_patterns:
            extra = np.zeros((B, 8), dtype=np.int64)
            for j, c in enumerate(contents):
                for slot, p in pk.cpu_patterns:
                    extra[j, slot] += p.count(c)
        el = (time.perf_counter() - pend["t0"]) * 1e3
        keep = pend["keep_device"]
        return TextResult(stats_h, pred_h, el, pend["pred"] is not None, pk.slot_prio, extra,
                          pend["pooled"] if keep else None, pend["hashes"] if keep else None, self.L, ph)

    def _workspace(self, B: int, classify: bool):
        """Device buffers of the one-call path, grown geometrically and reused
        batch after batch (one batch is in flight per pipeline, see launch)."""
        torch = self.torch
        ws = self._ws
        H = self._ensure_weights().hidden if classify else 0
        if ws is None or ws["B"] < B or ws["H"] < H:
            n = max(B, 2 * ws["B"] if ws else 0, 256)
            h = max(H, ws["H"] if ws else 0)
            dev = self.device
            # allocated in the PREPROCESS stream's pool: the kernels that use
            # these buffers run there.  A block from the compute stream's pool
            # may have been freed by a forward that is still running on the
            # GPU (the caching allocator orders reuse on the allocating stream
            # only), and preprocess kernels writing into it corrupted that
            # forward's activations (token ids -> out-of-range embedding gather,
            # seen under a 5k req/s multi-rank HTTP load whose growing batches
            # re-grew this workspace mid-serving)
            with torch.cuda.stream(self.stream):
                ws = self._ws = self._alloc_ws(n, h, dev)
        return ws

    def _alloc_ws(self, n: int, h: int, dev):
        torch = self.torch
        return {
                "B": n, "H": h,
                "stats": torch.empty((n, STAT_COLS), dtype=torch.int32, device=dev),
                "hashes": torch.empty((n, self.L), dtype=torch.int32, device=dev),
                "row_off": torch.empty(n + 1, dtype=torch.int32, device=dev),
                "pooled": torch.empty((n, h), dtype=torch.float32, device=dev) if h else None,
                "logits": torch.empty((n, 8), dtype=torch.float32, device=dev),
                "pred": torch.empty(n, dtype=torch.int32, device=dev),
            }

    def _launch_one_call(self, t0, B, pk, lens, ob, total, classify, prompt_cap, stream, contents):
        """The serve loop's path: the whole chain is one native call
        (``_hipops.text_batch``) over reused buffers -- no per-batch tensor
        allocations, four launches instead of eleven."""
        ws = self._workspace(B, classify)
        L = self.L
        cap = min(prompt_cap, L) if prompt_cap > 0 else 0
        a16 = lambda n: (n + 3) & ~3
        o_pred = a16(B * STAT_COLS)
        o_ph = o_pred + (a16(B) if classify else 0)
        self._ensure_readback(o_ph + B * cap)
        w = self._ensure_weights() if classify else None
        rows_upper = int(np.minimum((lens + 1) // 2, L).sum()) if classify else 0
        self.ops.text_batch(self._pin_dev, self._dev_bytes.data_ptr(), total, ob, B, L, pk.table,
                            ws["stats"].data_ptr(), ws["hashes"].data_ptr(), bool(classify),
                            ws["row_off"].data_ptr(), rows_upper,
                            w.E.data_ptr() if w else 0, w.vocab if w else 1, w.W1t.data_ptr() if w else 0,
                            w.b1.data_ptr() if w else 0, w.hidden if w else 0,
                            ws["pooled"].data_ptr() if w else 0, w.W2.data_ptr() if w else 0,
                            w.b2.data_ptr() if w else 0, ws["logits"].data_ptr(), ws["pred"].data_ptr(),
                            cap, self._rb_dev, o_pred, o_ph, stream)
        ev = self._ev                       # reused: one batch is in flight per pipeline
        ev.record(self.stream)
        return {"event": ev, "B": B, "cap": cap, "o_pred": o_pred, "o_ph": o_ph,
                "pred": ws["pred"] if classify else None, "pk": pk, "contents": contents, "t0": t0,
                "keep_device": False, "pooled": None, "hashes": None}

    def _launch(self, contents, patterns, version, classify, keep_device, prompt_cap):
        torch = self.torch
        t0 = time.perf_counter()
        B = len(contents)
        pk = self._patterns(patterns, version)
        blob, offsets, lens = self.pack(contents)
        ob = len(blob) + (-len(blob)) % 8        # offsets 8-byte aligned after the bytes
        nb = ob + offsets.nbytes
        if self._pin.numel() < nb:
            self._pin = torch.empty(max(nb, 2 * self._pin.numel()), dtype=torch.uint8).pin_memory()
            self._pin_dev = self.ops.host_device_ptr(self._pin.data_ptr())
        pin = self._pin
        pnp = pin.numpy()
        pnp[:len(blob)] = np.frombuffer(blob, dtype=np.uint8)
        pnp[ob:ob + offsets.nbytes] = offsets.view(np.uint8)
        total = ob + offsets.nbytes
        if self._dev_bytes.numel() < total:
            with torch.cuda.stream(self.stream):          # (the preprocess stream's pool, see _workspace)
                self._dev_bytes = torch.empty(max(total, 2 * self._dev_bytes.numel()), dtype=torch.uint8,
                                              device=self.device)
        dev = self._dev_bytes
        # H2D with a copy kernel reading host-mapped pinned memory: the
        # runtime's async H2D path was measured to wait for the backend's
        # queued forward steps on the other stream (~60 ms per batch)
        if not keep_device and B:
            return self._launch_one_call(t0, B, pk, lens, ob, total, classify, prompt_cap, self._sh, contents)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        self.ops.copy_bytes(dev.data_ptr(), self._pin_dev, total, stream)
        L = self.L
        d_off = dev[ob:ob + offsets.nbytes].view(torch.int64)
        stats = torch.empty((B, STAT_COLS), dtype=torch.int32, device=self.device)
        # every reader stops at the message's token count: no zero-fill needed
        hashes = torch.empty((B, L), dtype=torch.int32, device=self.device)
        self.ops.text_analyze(dev.data_ptr(), d_off.data_ptr(), B, L, pk.table, stats.data_ptr(),
                              hashes.data_ptr(), stream)
        pooled = pred = None
        if classify and B:
            w = self._ensure_weights()
            row_off = torch.empty(B + 1, dtype=torch.int32, device=self.device)
            self.ops.scan_rows(stats.data_ptr() + 4 * ST_NTOK, STAT_COLS, B, row_off.data_ptr(), stream)
            # host bound on token rows: a token needs >= 1 byte plus a separator
            rows_upper = int(np.minimum((lens + 1) // 2, L).sum())
            pooled = torch.zeros((B, w.hidden), dtype=torch.float32, device=self.device)
            self.ops.embed_pool(hashes.data_ptr(), L, row_off.data_ptr(), B, rows_upper, w.E.data_ptr(),
                                w.vocab, w.W1t.data_ptr(), w.b1.data_ptr(), w.hidden, pooled.data_ptr(),
                                stream)
            logits = torch.empty((B, 8), dtype=torch.float32, device=self.device)
            pred = torch.empty(B, dtype=torch.int32, device=self.device)
            self.ops.classify_head(pooled.data_ptr(), B, w.hidden, w.W2.data_ptr(), w.b2.data_ptr(),
                                   logits.data_ptr(), pred.data_ptr(), stream)
        # Read back with a copy kernel into host-mapped pinned memory, then an
        # event on THIS stream (see the H2D note above).
        cap = min(prompt_cap, L) if prompt_cap > 0 and B else 0
        a16 = lambda n: (n + 3) & ~3                          # int32 count -> 16-B multiple
        o_pred = a16(B * STAT_COLS)
        o_ph = o_pred + (a16(B) if pred is not None else 0)
        need = o_ph + B * cap
        self._ensure_readback(need)
        rd = self._rb_dev
        self.ops.copy_bytes(rd, stats.data_ptr(), 4 * B * STAT_COLS, stream)
        if pred is not None:
            self.ops.copy_bytes(rd + 4 * o_pred, pred.data_ptr(), 4 * B, stream)
        if cap:
            hc = hashes[:, :cap].contiguous()
            self.ops.copy_bytes(rd + 4 * o_ph, hc.data_ptr(), 4 * B * cap, stream)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        # device tensors stay referenced by the pending record until collect
        return {"event": ev, "B": B, "cap": cap, "o_pred": o_pred, "o_ph": o_ph, "pred": pred, "pk": pk,
                "contents": contents, "t0": t0, "keep_device": keep_device, "pooled": pooled, "hashes": hashes,
                "stats": stats, "hc": hc if cap else None}


class CpuTextPipeline:
    """The text pipeline on the CPU (no GPU on the host): the ``_textcpu``
    module runs the same per-byte analysis as ``text_analyze_kernel`` over
    the same packed batch and pattern table, and returns the same stats rows
    and token hashes, so ``Preprocessor.end_batch`` decides priorities
    exactly as on the GPU path (fold-special messages still go to the
    oracle).  No classifier (the CPU oracle path has none either).  Same
    launch / ready / collect interface as :class:`TextPipeline`; ``launch``
    does the work."""

    def __init__(self, cfg=None):
        from ..utils.config import PreprocessorConfig
        self.cfg = cfg or PreprocessorConfig()
        self.L = int(self.cfg.max_tokens)
        self.mod = _native.textcpu()
        assert self.mod.PATTERN_TABLE_BYTES == 4 * (MAX_PATTERNS * 8 + MAX_PATTERNS * 3 + 1)
        self._packed: Optional[PackedPatterns] = None

    def _patterns(self, patterns, version) -> PackedPatterns:
        if self._packed is None or self._packed.version != version or version < 0:
            self._packed = pack_patterns(patterns, version)
        return self._packed

    def run(self, contents: Sequence[str], patterns: Dict[int, list], version: int = -1,
            classify: bool = False, keep_device: bool = False, prompt_cap: int = 0) -> TextResult:
        return self.collect(self.launch(contents, patterns, version, classify, keep_device, prompt_cap))

    def launch(self, contents: Sequence[str], patterns: Dict[int, list], version: int = -1,
               classify: bool = False, keep_device: bool = False, prompt_cap: int = 0):
        t0 = time.perf_counter()
        pk = self._patterns(patterns, version)
        blob, offsets, _lens = TextPipeline.pack(contents)
        B, L = len(contents), self.L
        stats = np.empty((B, STAT_COLS), dtype=np.int32)
        hashes = np.empty((B, L), dtype=np.uint32)
        self.mod.analyze(np.frombuffer(blob, dtype=np.uint8), offsets, B, L, pk.table, stats, hashes)
        extra = None
        if pk.cpu_patterns:
            extra = np.zeros((B, 8), dtype=np.int64)
            for j, c in enumerate(contents):
                for slot, pat in pk.cpu_patterns:
                    extra[j, slot] += pat.count(c)
        cap = min(prompt_cap, L) if prompt_cap > 0 else 0
        res = TextResult(stats, None, (time.perf_counter() - t0) * 1e3, False, pk.slot_prio, extra, None, None, L,
                         hashes[:, :cap] if cap else None)
        return {"result": res}

    @staticmethod
    def ready(pend) -> bool:
        return True

    def collect(self, pend) -> TextResult:
        return pend["result"]

