"""GPU backend engine: continuous batching over fixed batch slots (N12 + N9).

One engine per GPU process.  ``admit`` places dispatched requests into free
slots; ``launch`` enqueues ONE model forward over a token batch made of
  * one decode token for every slot that is generating, then
  * chunked-prefill tokens of admitted prompts, up to ``token_budget``;
and returns immediately.  The pipeline is fully asynchronous:
  * a decode token's id is the previous step's greedy output, which stays on
    the device -- the next step gathers it there (``index_select``), so the
    host never waits for token values;
  * completions are deterministic (greedy decode always yields a token), so
    a request's slot is freed at launch of its last step and can be re-admitted
    into the NEXT step (same-stream ordering keeps its KV rows safe);
  * at most ``max_inflight`` (2) steps are queued on the GPU; ``finish`` reaps
    finished steps (blocking only when the queue is full), so host work of the
    next tick overlaps the current forward and the GPU never idles between
    steps.
The slot census of every step is written by the ``slot_census`` kernel into
the node-shared load page (zero-copy for routers, N9).

Reference: the reference has no model backend -- its workers call a
``ProcessFunc`` (`internal/priorityqueue/worker.go:162-189`) that
`cmd/server/main.go:172-193` (`startWorkers`) stubs out; this engine is what a
dispatched request runs on instead.

Request cost model (README/bench): prompt = the message's tokens from the
GPU tokenizer (capped), generation = ``gen_tokens`` greedy tokens, all 32
layers of the stub, never skipped.
"""
from __future__ import annotations

import collections
import time
from dataclasses import dataclass
from typing import Deque, Dict, List, Optional, Sequence

import numpy as np
import torch

from ..models.llama_stub import LlamaConfig, LlamaStub


@dataclass
class Request:
    req_id: int
    prompt: np.ndarray            # int32 token ids
    gen_tokens: int
    tier: int = 2
    slot: int = -1
    prefilled: int = 0
    generated: int = 0
    admitted_ns: int = 0
    first_token_ns: int = 0
    done_ns: int = 0
    meta: object = None
    out_idx: int = -1             # row of the previous step's output holding my last token
    out_step: int = -1
    conv: int = -1                # conversation key: its KV stays resident in the slot between turns
    reused: int = 0               # context tokens served from the resident KV (not re-prefilled)
    history: Optional[np.ndarray] = None   # earlier dialog tokens, prefilled only if not resident
    # compressed context of an evicted window (N5 salient tokens), prepended
    # to a non-resident replay ahead of ``history``; never part of a resident KV
    prefix: Optional[np.ndarray] = None
    timeout_ns: int = 0           # processing timeout of this attempt (0: none); the deadline starts at admission
    deadline_ns: int = 0          # admitted_ns + timeout_ns (monotonic), set by ``admit``
    micro: bool = False           # served by the realtime micro-forwards (``realtime_mode="micro"``)
    aborted: bool = False         # this attempt was aborted (timeout / cancel / evacuation)
    # the greedy token ids this attempt generated, read back from the device
    # with the step that sampled them (set when the request completes)
    out_tokens: Optional[np.ndarray] = None
    # a conversation turn dispatched by another router: its ``out_tokens``
    # go back with the completion record even when ``conv`` is -1 (no KV
    # residency), so the origin's dialog history holds the real ids
    dialog: bool = False


@dataclass
class StepResult:
    tokens: int
    prefill_tokens: int
    decode_tokens: int
    completed: List[Request]
    first_tokens: List[Request]
    elapsed_ms: float


class _blas:
    """torch's library-GEMM backend for a block ("cublas" = rocBLAS on ROCm,
    "cublaslt" = hipBLASLt), restored after it (the serve loop is one thread)."""

    def __init__(self, lib: str):
        self.lib = lib

    def __enter__(self):
        self.prev = torch.backends.cuda.preferred_blas_library()
        torch.backends.cuda.preferred_blas_library(self.lib)
        return self

    def __exit__(self, *exc):
        torch.backends.cuda.preferred_blas_library(self.prev)
        return False


class _NullCtx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


class BackendHung(Exception):
    """A forward step has not completed on the GPU within the engine's
    ``step_timeout_s``.  Not a RuntimeError on purpose: a recoverable
    backend error (HIP error, OOM) evacuates this GPU and keeps serving, but
    a step that never completes leaves nothing to evacuate to -- the work
    queued behind it waits forever -- so the process must end (the serve
    loop treats it like ``PeerLost``) and the launcher restarts the job."""


@dataclass
class _Inflight:
    step: int
    event: object
    T: int
    n_pre: int
    n_dec: int
    completed: List[Request]
    firsts: List[Request]
    t0: float
    out: object                   # device tensor of sampled tokens (kept alive for the next gather)
    t0_ns: int = 0                # monotonic launch time (tracing)
    ev_start: object = None       # timing event before the forward (``time_steps``)
    micro: bool = False           # a realtime micro-forward (``_qm``), not a serving step
    samp_slots: object = None     # int64 [S]: the slot each sampled row belongs to
    gidx: object = None           # int64 [S]: which generated token of its request each row is
    host_out: object = None       # pinned int32 [>= S]: the sampled ids, copied back behind the forward


class BackendEngine:
    MICRO_GRAPH_BUCKETS = (8, 16, 32, 64)

    def __init__(self, model_cfg: LlamaConfig, slots: int = 256, max_ctx: int = 512,
                 token_budget: int = 2048, device="cuda", impl: str = "hip", seed: int = 0,
                 page=None, gpu_index: int = 0, max_inflight: int = 2, residual_in_gemm: bool = True,
                 split_qkv: bool = False, fused_mlp=None, fused_qkv=None, row_scale_norm: bool = True,
                 fused_head=None, fused_resid=None, prune_last: bool = True, step_timeout_s: float = 60.0,
                 realtime_step_tokens: int = 0, fused_rms=None, realtime_mode: str = "",
                 micro_slots: int = 96, micro_budget: int = 512, micro_inflight: int = 1,
                 micro_stream: str = "partition", micro_cus: int = 64, micro_gemm: str = "hip",
                 library_gemm: bool = False, micro_graph: bool = True):
        self.cfg = model_cfg
        # a queued forward older than this raises BackendHung (0 = wait forever)
        self.step_timeout_s = float(step_timeout_s)
        self.slots = slots
        self.max_ctx = max_ctx
        # every generating slot gets its decode token each step (the on-device
        # token gather reads the previous step's output only)
        self.token_budget = max(token_budget, slots)
        # How realtime requests (tier < fast_tiers) are served
        # (``backend.realtime_mode``; docs/performance.md "Realtime modes"):
        #   "off"   -- in the serving steps like everyone else (prefilled first);
        #   "cap"   -- the step cap (``backend.realtime_step_tokens``): while a
        #              realtime request is in the batch a step carries at most
        #              that many tokens (never fewer than its decode rows), so
        #              its 4 forwards finish sooner -- at the price of the
        #              smaller steps' GEMM efficiency for everyone in them
        #              (profiles/r5_step_budget_sweep_1gpu.jsonl);
        #   "micro" -- realtime micro-forwards: realtime requests take slots of
        #              a separate pool (``micro_slots``) that only small
        #              forwards over those slots touch, launched back to back
        #              on their own stream (``micro_stream``: "high" = a
        #              high-priority HIP stream next to the serving stream,
        #              "same" = the serving stream) while the big steps run.
        # An empty mode follows ``realtime_step_tokens`` (> 0: "cap").
        self.rt_step_tokens = int(realtime_step_tokens)
        mode = realtime_mode or ("cap" if self.rt_step_tokens > 0 else "off")
        if mode not in ("off", "cap", "micro"):
            raise ValueError(f"realtime_mode must be off / cap / micro, not {mode!r}")
        if mode != "cap":
            self.rt_step_tokens = 0
        self.realtime_mode = mode
        self.micro = mode == "micro"
        self.micro_slots = int(micro_slots) if self.micro else 0
        if self.micro and self.micro_slots < 1:
            raise ValueError("realtime_mode micro needs micro_slots >= 1")
        self.micro_budget = max(int(micro_budget), self.micro_slots + 1)
        self.micro_inflight = max(1, int(micro_inflight))
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        # decode-only micro-forwards (<= 64 rows) replay HIP graphs captured
        # at warm-up, one per row bucket (``MICRO_GRAPH_BUCKETS``): a
        # micro-forward is ~350 kernel launches the serve loop's host thread
        # would otherwise issue one by one between pumping arrivals.  The
        # padding rows of a bucket run on a scratch slot past the micro pool.
        self.micro_graph = bool(micro_graph) and self.micro and self.cuda and impl == "hip" \
            and micro_stream in ("high", "partition")
        self.scratch_slot = slots + self.micro_slots if self.micro_graph else -1
        # KV slots: serving pool, then the micro pool (+ the graphs' scratch slot)
        self.n_all = slots + self.micro_slots + (1 if self.micro_graph else 0)
        self.async_device = self.cuda          # forwards run asynchronously (a GPU stream)
        self.rt_stream = None
        self.main_stream = None          # (partition: the serving steps' CU-masked stream)
        self.micro_cus = 0
        if self.micro and micro_stream not in ("high", "same", "partition"):
            raise ValueError(f"micro_stream must be high / same / partition, not {micro_stream!r}")
        if self.micro and self.cuda and micro_stream == "high":
            self.rt_stream = torch.cuda.Stream(self.device, priority=torch.cuda.Stream.priority_range()[1])
        elif self.micro and self.cuda and micro_stream == "partition":
            # the chip split in two CU partitions: the micro-forwards own
            # ``micro_cus`` CUs, the serving steps the rest (their GEMM tile
            # plans size waves for that count), so neither waits for the
            # other's kernels to drain (docs/performance.md "Realtime modes")
            from .cu_partition import partition_streams
            self.micro_cus = int(micro_cus)
            self.main_stream, self.rt_stream, big_cus = partition_streams(self.device, self.micro_cus)
            from ..ops import gemm as _G
            _G.EFFECTIVE_CUS[self.device.index if self.device.index is not None else 0] = big_cus
            # serving steps of whole waves on the remaining CUs: 16 row tiles
            # per 256 CUs (4,096 tokens on the chip, 3,072 on 192 CUs --
            # profiles/r6_token_budget_sweep_1gpu.jsonl, r6_realtime_modes.md)
            self.token_budget = max(min(self.token_budget, 16 * big_cus), slots)
        self.micro_stream = micro_stream if self.micro else ""
        # the micro-forwards' GEMMs on a CU partition: "hip" = the hand-written
        # kernels (split-K small steps), "rocblas" = the library through
        # rocBLAS (classic, non-persistent kernels: safe on a CU mask, unlike
        # hipBLASLt's stream-K grids sized for the whole chip)
        if micro_gemm not in ("hip", "rocblas"):
            raise ValueError(f"micro_gemm must be hip / rocblas, not {micro_gemm!r}")
        self.micro_gemm = micro_gemm
        if self.micro_cus and micro_gemm == "rocblas":
            import os
            # rocBLAS may hand some GEMMs to hipBLASLt on gfx950: keep them classic
            os.environ.setdefault("ROCBLAS_USE_HIPBLASLT", "0")
        self.model = LlamaStub(model_cfg, self.n_all, max_ctx, device=self.device, impl=impl, seed=seed,
                               residual_in_gemm=residual_in_gemm, split_qkv=split_qkv, fused_mlp=fused_mlp,
                               fused_qkv=fused_qkv, row_scale_norm=row_scale_norm, fused_head=fused_head,
                               fused_resid=fused_resid, fused_rms=fused_rms, prune_last=prune_last,
                               library_gemm=library_gemm)
        self.impl = impl
        self.weight_bytes = self.model.weight_bytes()
        self.active: Dict[int, Request] = {}            # slot -> request
        self.free: List[int] = list(range(slots - 1, -1, -1))
        # the realtime micro pool: slots [slots, n_all), never in ``free`` /
        # ``conv_lru``, so no serving step ever reads or writes their KV rows
        # (the two streams never share a slot)
        self.free_micro: List[int] = list(range(slots + self.micro_slots - 1, slots - 1, -1))
        n_all = self.n_all
        # Conversation KV residency (BASELINE config 4): when a request of a
        # conversation completes, its slot keeps the KV of the dialog so far
        # (prompt + generated tokens except the last) and parks in an LRU;
        # the conversation's next turn is admitted into that slot and only
        # prefills its new tokens.  Parked slots count as free: they are
        # evicted (LRU) when no truly free slot is left.
        self.conv_lru: "collections.OrderedDict[int, int]" = collections.OrderedDict()
        self.s_conv = np.full(n_all, -1, dtype=np.int64)
        self.s_cached = np.zeros(n_all, dtype=np.int64)
        self.kv_reused_tokens = 0
        self.kv_evictions = 0
        self.kv_imported = 0
        self.kv_stale = 0                                   # parked copies found outdated at admission
        self.replay_tokens = 0                              # dialog tokens prefilled by non-resident replays
        self.replay_nonzero = 0                             # ... of which not the id 0 (placeholders were 0)
        self._importing: Dict[int, int] = {}                # slot -> conv: KV arriving (migration in flight)
        # per-slot host state (the batch builder is vectorised over these)
        self.s_prompt = np.zeros((n_all, max_ctx), dtype=np.int32)
        self.s_plen = np.zeros(n_all, dtype=np.int64)
        self.s_pref = np.zeros(n_all, dtype=np.int64)       # prompt tokens prefilled
        self.s_gen = np.zeros(n_all, dtype=np.int64)        # tokens generated
        self.s_gmax = np.zeros(n_all, dtype=np.int64)       # tokens to generate
        self.s_seq = np.zeros(n_all, dtype=np.int64)        # admission order
        self.s_out_idx = np.zeros(n_all, dtype=np.int64)    # row of my last token in the step output
        self.s_out_step = np.full(n_all, -2, dtype=np.int64)
        self.s_active = np.zeros(n_all, dtype=bool)
        self.s_tier = np.zeros(n_all, dtype=np.int64)
        self.s_micro = np.zeros(n_all, dtype=bool)
        self.s_micro[slots:] = True
        # host copy of every generated token id, per slot (written when the
        # step that sampled it is reaped; steps of one pool are reaped in
        # launch order, so a slot's next request never overwrites a row
        # before the previous one's completion copied it out)
        self.h_tokens = np.zeros((n_all, max_ctx), dtype=np.int32)
        # processing deadline per slot (monotonic ns, 0 = none): a request
        # still running past it is aborted by ``expire`` (the reference runs
        # every message under context.WithTimeout(msg.Timeout),
        # `internal/priorityqueue/worker.go:162-188`)
        self.s_deadline = np.zeros(n_all, dtype=np.int64)
        self.expired_total = 0
        self.cancelled_total = 0
        self._admit_seq = 0
        self._mean_plen = 16.0                              # EMA of admitted prompt lengths
        # realtime lane: requests of tiers < fast_tiers are prefilled ahead of
        # every other admitted prompt (their admission order key is shifted
        # below all others), and the dispatcher may admit them past the
        # step's prefill headroom (``lane_capacity``)
        self.fast_tiers = 1
        self.warmed_shapes = 0
        self.page = page
        self.gpu_index = gpu_index
        self.max_inflight = max(1, max_inflight)
        self.step_id = 0
        self.total_tokens = 0
        self.completed_total = 0
        self.completed_tokens = 0
        self.matmul_flops = 0                            # GEMM FLOPs of every launched forward (``_step_flops``)
        self._q: Deque[_Inflight] = collections.deque()
        self._reaped: List[_Inflight] = []               # reaped by launch(), not yet returned
        self._fence: List[object] = []                   # events of steps dropped by abort_all
        self.host_ns = np.zeros(3, dtype=np.int64)       # [batch build, wait for GPU, enqueue forward] host time
        self._prev_out = None                            # device int32 [n_samples] of the last launched step
        # pinned staging rings (a buffer is reused only after the step that
        # read it has finished: launch keeps <= max_inflight steps queued, so
        # step k reuses step k - ring's buffer only once that one was reaped)
        ring = max(2, self.max_inflight)
        self._pins = [self._alloc_pin(4 * (7 * self.token_budget + 2 * slots + 64)) for _ in range(ring)]
        # sampled token ids copied back behind each forward (read at reap)
        self._out_pins = [self._alloc_pin(4 * self.n_all).view(torch.int32) for _ in range(ring)]
        # realtime micro-forwards: their own queue, staging, token gather source
        self._qm: Deque[_Inflight] = collections.deque()
        self._reaped_m: List[_Inflight] = []
        self._prev_out_m = None
        self.micro_id = 0
        self.micro_steps = 0
        self.micro_gpu_ms = 0.0                          # device time of timed micro-forwards (``time_steps``)
        self.micro_timed = 0
        self._mg: Dict[int, tuple] = {}                  # bucket -> (graph, static inputs, token ids, output)
        self.micro_graph_steps = 0
        if self.micro:
            mr = self.micro_inflight + 1
            # a micro step's staging: tokens, pos, slot (3T), samples + decode
            # gather rows (<= 3T) and ~one 1-token tile per row (4T) -- sized
            # so it never grows (a grown pinned buffer frees the old one
            # behind the copies still queued from it)
            self._pins_m = [self._alloc_pin(4 * (11 * self.micro_budget + 2 * self.micro_slots + 64))
                            for _ in range(mr)]
            self._out_pins_m = [self._alloc_pin(4 * self.micro_slots).view(torch.int32) for _ in range(mr)]
        # segment-tiled MFMA attention on the HIP path (per-token otherwise)
        self.use_tiles = impl == "hip"
        self._state_pins = [self._alloc_pin(4 * slots) for _ in range(2)]
        self._slot_state_d = torch.zeros(slots, dtype=torch.int32, device=self.device)
        # fault injection: {"fail_launch": n} raises on the next
        # n launches (a HIP error / OOM), {"slow_ms": x} stalls every launch,
        # {"drop_heartbeat": True} stops the load-page census
        self.fault: Dict[str, float] = {}
        self.tracer = None          # utils.tracing.RequestTracer (backend step spans)
        # GPU execution time of every forward step (timing events around it;
        # the start event's timestamp is when the GPU reached the step, so the
        # difference is device time, not queueing): bench.py's lock-step
        # attribution (slowest vs mean GPU of a multi-rank job)
        self.time_steps = False
        self.gpu_step_ms = 0.0
        self.gpu_steps = 0
        self.gpu_step_max_ms = 0.0
        if self.cuda and page is not None and page.dev_ptr is None:
            page.register_device()
        if page is not None:
            page.set_health(True)
            page.write_host(0, slots, 0, 0)

    def _alloc_pin(self, nbytes: int) -> torch.Tensor:
        t = torch.empty(nbytes, dtype=torch.uint8)
        return t.pin_memory() if self.cuda else t

    # ------------------------------------------------------------------ admission
    def free_slots(self) -> int:
        return len(self.free) + len(self.conv_lru)

    def inflight(self) -> int:
        """Requests holding a slot (serving pool + realtime micro pool)."""
        return self.slots - self.free_slots() + self.micro_slots - len(self.free_micro)

    def _big_active(self) -> np.ndarray:
        return self.s_active & ~self.s_micro if self.micro else self.s_active

    def _take_slot(self) -> int:
        if self.free:
            return self.free.pop()
        conv, s = self.conv_lru.popitem(last=False)          # evict the least recently used context
        self.s_conv[s] = -1
        self.kv_evictions += 1
        return s

    def resident_context(self, conv: int) -> int:
        """Tokens of conversation ``conv`` resident in this engine's KV (0 if none)."""
        s = self.conv_lru.get(conv)
        return int(self.s_cached[s]) if s is not None else 0

    def admit_capacity(self) -> int:
        """How many new requests the NEXT step can take: free slots, bounded
        by the step's prefill headroom (token budget - decode tokens - prompt
        tokens already admitted but not yet prefilled) over the running mean
        prompt length.  The dispatcher admits at most this many, so requests
        that could not start prefilling next step wait in the priority queue
        (where tier order and aging apply), not in a FIFO inside the engine."""
        free = len(self.free) + len(self.conv_lru)
        if free == 0:
            return 0
        act = self._big_active()
        pending = int((self.s_plen[act] - self.s_pref[act]).sum())
        head = self.step_budget() - int(act.sum()) - pending
        if head <= 0:
            return 0
        # round UP: the last admitted prompt may spill into the following step
        # (chunked prefill), so a saturated step fills its token budget -- GEMM
        # cost is quantised in 256-row tiles, the tail rows are nearly free
        return min(free, max(1, -(-head // max(1, int(round(self._mean_plen))))))

    # ------------------------------------------------------------------ KV migration (N11)
    def export_kv(self, conv: int):
        """(slot, tokens) of conversation ``conv``'s parked KV, or (-1, 0)
        when it is not resident here (evicted, or a turn is in flight)."""
        s = self.conv_lru.get(conv)
        if s is None:
            return -1, 0
        return s, int(self.s_cached[s])

    def drop_parked(self, conv: int) -> None:
        """Forget a parked conversation (its KV moved to another GPU); the
        slot is free for the next admission (stream order keeps the pending
        pack copy ahead of any later write to it)."""
        s = self.conv_lru.pop(conv, None)
        if s is not None:
            self.s_conv[s] = -1
            self.s_cached[s] = 0
            self.free.insert(0, s)          # reused last (``free`` pops from the end)

    def import_kv(self, conv: int, tokens: int) -> int:
        """Park an incoming conversation's KV (``tokens`` positions) in a
        slot; returns the slot the caller unpacks into.  The conversation's
        turn is then admitted like any resident turn (prefills only its new
        tokens)."""
        self.drop_parked(conv)
        s = self._take_slot()
        self.s_conv[s] = conv
        self.s_cached[s] = int(tokens)
        self.conv_lru[conv] = s
        self.kv_imported += 1
        return s

    def reserve_import(self, conv: int, tokens: int = 0) -> int:
        """A slot for an incoming conversation's KV while the transfer is in
        flight on the migration stream: out of the free list and the LRU
        (so no admission can take it) until ``finish_import`` parks it."""
        self.drop_parked(conv)
        s = self._take_slot()
        self.s_conv[s] = -1
        self.s_cached[s] = int(tokens)
        self._importing[s] = conv
        return s

    def finish_import(self, conv: int, slot: int, tokens: int) -> None:
        """The KV landed in ``slot``: park it like a resident dialog (the
        conversation's held turn is admitted next and reuses it)."""
        if self._importing.pop(slot, None) is None:
            return                                          # aborted meanwhile (evacuation)
        old = self.conv_lru.pop(conv, None)
        if old is not None and old != slot:
            self.s_conv[old] = -1
            self.free.append(old)
        self.s_conv[slot] = conv
        self.s_cached[slot] = int(tokens)
        self.conv_lru[conv] = slot
        self.kv_imported += 1

    def resident_kv_tokens(self) -> int:
        """KV positions held in this GPU's cache right now: the context of
        every active request (prompt + generated so far) plus every parked
        dialog -- the live HBM occupancy of the KV pool (the pool itself is
        preallocated, so allocator figures never move)."""
        act = self.s_active
        n = int((self.s_plen[act] + self.s_gen[act]).sum())
        if self.conv_lru:
            n += int(self.s_cached[np.fromiter(self.conv_lru.values(), dtype=np.int64)].sum())
        return n + int(self.s_cached[list(self._importing)].sum()) if self._importing else n

    def kv_token_capacity(self) -> int:
        return self.slots * self.max_ctx

    def kv_bytes_per_token(self) -> int:
        c = self.cfg
        return c.layers * 2 * c.kv_heads * c.head_dim * 2          # K and V, bf16 (128 KiB for Llama-3-8B)

    def ready_tokens(self) -> int:
        """Tokens the next launch would run right now: one per decoding slot
        plus the pending prefill, capped at the token budget."""
        act = self._big_active()
        if not act.any():
            return 0
        plen, pref = self.s_plen[act], self.s_pref[act]
        return min(self.step_budget(), int((pref >= plen).sum()) + int((plen - pref).clip(min=0).sum()))

    def step_budget(self) -> int:
        """Tokens the next step may carry: ``token_budget``, or the realtime
        cap while a realtime-lane request is active (at least one more than
        the decode rows, which every step must carry)."""
        cap = self.rt_step_tokens
        if cap <= 0 or cap >= self.token_budget or not self.active:
            return self.token_budget
        act = self.s_active
        if not (act & (self.s_tier < self.fast_tiers)).any():
            return self.token_budget
        dec = int((self.s_pref[act] >= self.s_plen[act]).sum())
        return max(cap, dec + 1)

    def lane_capacity(self) -> int:
        """Slots a realtime request may take beyond ``admit_capacity``: every
        free (or parked) slot, plus the free micro-pool slots.  Its prefill
        goes first in the next step (or into the next micro-forward), so it
        starts computing there instead of waiting for headroom."""
        return len(self.free) + len(self.conv_lru) + len(self.free_micro)

    def _to_micro(self, r: Request) -> bool:
        """Serve ``r`` on the micro pool: a realtime request, a free micro
        slot, and no resident KV of its dialog in the serving pool (a
        resident turn stays where its context is)."""
        return (self.micro and 0 <= r.tier < self.fast_tiers and bool(self.free_micro)
                and not (r.conv >= 0 and r.conv in self.conv_lru))

    def admit(self, reqs: Sequence[Request]) -> List[Request]:
        now = time.monotonic_ns()
        out = []
        cap = self.max_ctx - 1
        for r in reqs:
            micro = self._to_micro(r)
            if not micro and not self.free and not self.conv_lru:
                if self.micro:
                    continue                                  # (a later realtime request may still fit)
                break
            if r.gen_tokens < 1:
                r.gen_tokens = 1
            plen = max(1, min(len(r.prompt), cap - r.gen_tokens + 1))
            r.prompt = np.asarray(r.prompt[:plen], dtype=np.int64) % self.cfg.vocab
            if len(r.prompt) == 0:
                r.prompt = np.zeros(1, dtype=np.int64)
            r.micro = micro
            r.aborted = False
            r.out_tokens = None
            base = 0
            s = self.conv_lru.pop(r.conv, None) if (r.conv >= 0 and not micro) else None
            if micro:
                # a micro-pool slot keeps no dialog KV: the turn replays its
                # history (``r.history``) and nothing is parked afterwards
                s = self.free_micro.pop()
            elif s is not None:
                base = int(self.s_cached[s])
                if r.history is not None and base < len(r.history):
                    # a stale copy: this GPU served an earlier turn, later turns
                    # ran elsewhere -- attending over it would drop them
                    base = 0
                    self.kv_stale += 1
                if base + len(r.prompt) + r.gen_tokens > cap + 1:
                    base = 0                                  # context window full: restart the dialog KV
            else:
                s = self._take_slot()
            if base == 0 and ((r.history is not None and len(r.history)) or (r.prefix is not None and len(r.prefix))):
                # not resident here: replay the dialog -- its compressed
                # context (if a window was evicted), then the most recent
                # history tokens that fit
                room = cap + 1 - r.gen_tokens - len(r.prompt)
                if room > 0:
                    pre = np.asarray(r.prefix if r.prefix is not None else (), dtype=np.int64)[:room // 4]
                    hist = np.asarray(r.history if r.history is not None else (), dtype=np.int64)
                    keep = room - len(pre)
                    h = hist[len(hist) - keep:] if 0 < keep < len(hist) else (hist if keep > 0 else hist[:0])
                    r.prompt = np.concatenate([pre % self.cfg.vocab, h % self.cfg.vocab, r.prompt])
                    self.replay_tokens += len(pre) + len(h)
                    self.replay_nonzero += int(np.count_nonzero(pre)) + int(np.count_nonzero(h))
            r.slot = s
            r.reused = base
            r.prefilled = 0
            r.generated = 0
            r.out_idx = r.out_step = -1
            r.admitted_ns = now
            r.deadline_ns = now + int(r.timeout_ns) if r.timeout_ns > 0 else 0
            self.s_deadline[s] = r.deadline_ns
            self.active[s] = r
            n = len(r.prompt)
            self.s_prompt[s, base:base + n] = r.prompt
            self.s_plen[s] = base + n
            self.s_pref[s] = base
            self.s_gen[s] = 0
            self.s_gmax[s] = r.gen_tokens
            # prefill order key: realtime-lane tiers sort before everything else
            self.s_seq[s] = self._admit_seq - (1 << 48 if 0 <= r.tier < self.fast_tiers else 0)
            self._admit_seq += 1
            self.s_active[s] = True
            self.s_tier[s] = r.tier
            self.s_conv[s] = -1 if micro else r.conv
            self.kv_reused_tokens += base
            if not micro:                                     # (the serving steps' headroom estimate)
                self._mean_plen += 0.01 * (n - self._mean_plen)
            out.append(r)
        return out

    # ------------------------------------------------------------------ abort (timeout / cancel)
    def _abort_slots(self, slots) -> List[Request]:
        """Take the active requests of ``slots`` out of the batch: their slots
        return to the free list for the NEXT launch.  Steps already queued on
        the GPU still compute their rows; a request admitted into the slot
        afterwards is prefilled by a later step on the same stream, so stream
        order keeps it from reading anything the aborted request wrote.  The
        aborted turn's KV is partial, so it is never parked for reuse."""
        out = []
        for s in slots:
            s = int(s)
            r = self.active.pop(s, None)
            if r is None:
                continue
            self.s_active[s] = False
            self.s_deadline[s] = 0
            self.s_conv[s] = -1
            self.s_cached[s] = 0
            # reused first (``_take_slot`` pops from the end)
            (self.free_micro if self.s_micro[s] else self.free).append(s)
            # steps still queued on the GPU list it among their first tokens:
            # their reap must not stamp an attempt that no longer exists
            r.aborted = True
            out.append(r)
        return out

    def expire(self, now_ns: Optional[int] = None) -> List[Request]:
        """Abort every active request whose processing deadline
        (``Request.timeout_ns`` after admission) has passed; returns them so
        the caller can retry or dead-letter them.  Requests whose last token
        is already launched completed at that launch and are not touched."""
        if not self.active:
            return []
        now = time.monotonic_ns() if now_ns is None else int(now_ns)
        d = self.s_deadline
        hit = np.flatnonzero(self.s_active & (d > 0) & (d < now))
        if not len(hit):
            return []
        out = self._abort_slots(hit)
        self.expired_total += len(out)
        return out

    def cancel(self, req_ids: Sequence[int]) -> List[Request]:
        """Abort the active requests with these ids (``DELETE
        /api/v1/messages/{id}`` on a request in flight); returns the ones
        found (a request that completed or was never admitted is not)."""
        want = {int(x) for x in req_ids}
        if not want or not self.active:
            return []
        out = self._abort_slots([s for s, r in self.active.items() if r.req_id in want])
        self.cancelled_total += len(out)
        return out

    # ------------------------------------------------------------------ step
    def _build(self, micro: bool = False):
        """Vectorised batch construction over the per-slot state arrays of
        one pool (the serving slots, or with ``micro`` the realtime micro
        pool): decode rows first (one token per generating slot, ids gathered
        on the device from the pool's previous step output), then chunked
        prefill in admission order up to the step's token budget.  Returns
        int32 arrays."""
        if self.micro:
            act = np.flatnonzero(self.s_active & (self.s_micro if micro else ~self.s_micro))
        else:
            act = np.flatnonzero(self.s_active)
        plen, pref = self.s_plen[act], self.s_pref[act]
        is_dec = pref >= plen
        dec = act[is_dec]
        D = len(dec)
        prev = (self.micro_id if micro else self.step_id) - 1
        if D and (self.s_out_step[dec] != prev).any():
            raise RuntimeError("decode token source is not the previous step")
        pre = act[~is_dec]
        if len(pre):
            pre = pre[np.argsort(self.s_seq[pre], kind="stable")]
        rem = self.s_plen[pre] - self.s_pref[pre]
        budget = (self.micro_budget if micro else self.step_budget()) - D
        before = np.cumsum(rem) - rem
        take = np.clip(budget - before, 0, rem)
        keep = take > 0
        pre, take = pre[keep], take[keep]
        n_pre = int(take.sum())
        T = D + n_pre
        a0 = self.s_pref[pre]
        # prefill token rows: slot pre[i] contributes prompt[a0:a0+take]
        start = D + np.cumsum(take) - take                   # first row of each chunk
        rep = np.repeat(np.arange(len(pre)), take)
        off = np.arange(n_pre) - (start[rep] - D) if n_pre else np.zeros(0, np.int64)
        p_slot = pre[rep]
        p_pos = a0[rep] + off
        toks = np.zeros(T, dtype=np.int32)
        pos = np.empty(T, dtype=np.int32)
        slot = np.empty(T, dtype=np.int32)
        d_pos = self.s_plen[dec] + self.s_gen[dec] - 1
        pos[:D] = d_pos
        slot[:D] = dec
        if n_pre:
            toks[D:] = self.s_prompt[p_slot, p_pos]
            pos[D:] = p_pos
            slot[D:] = p_slot
        fin = a0 + take >= self.s_plen[pre]                   # chunk completes the prompt
        samp = np.concatenate([np.arange(D), (start + take - 1)[fin]]).astype(np.int32)
        samp_slots = np.concatenate([dec, pre[fin]])
        dec_rows = np.arange(D, dtype=np.int32)
        dec_src = self.s_out_idx[dec].astype(np.int32)
        # attention tiles: decode rows are 1-token tiles; chunks cut at 16
        nt = (take + 15) // 16
        trep = np.repeat(np.arange(len(pre)), nt)
        toff = (np.arange(int(nt.sum())) - np.repeat(np.cumsum(nt) - nt, nt)) * 16
        tiles = np.empty((D + len(trep), 4), dtype=np.int32)
        tiles[:D, 0] = dec_rows
        tiles[:D, 1] = 1
        tiles[:D, 2] = dec
        tiles[:D, 3] = d_pos
        if len(trep):
            tiles[D:, 0] = start[trep] + toff
            tiles[D:, 1] = np.minimum(16, take[trep] - toff)
            tiles[D:, 2] = pre[trep]
            tiles[D:, 3] = a0[trep] + toff
        self.s_pref[pre] += take
        return toks, pos, slot, samp, samp_slots, dec_rows, dec_src, tiles, n_pre, D

    def warm_shapes(self, sizes: Optional[Sequence[int]] = None) -> int:
        """Run one throw-away forward at every token count a cold start can
        produce, before serving.

        A saturated warm-up only ever runs ~token_budget-token steps; the
        first SMALL step afterwards (a gateway going idle -> busy, or the first
        requests after start) used to pay the one-time GEMM kernel selection /
        code-object load of small-M shapes -- measured at ~135 ms for the
        first T = 1 forward of the 8B stub (``bench/cold_shapes.py``,
        ``profiles/r2_cold_shapes.md``) -- on live requests.  Every T in
        1..32 is run (lm_head rows = T), then a geometric ladder up to the
        token budget.  Must be called on an idle engine (uses scratch rows of
        free slots; nothing it writes is ever read by a request)."""
        if not self.cuda:
            return 0
        if self.active or self.conv_lru or self._q or self._qm:
            raise RuntimeError("warm_shapes needs an idle engine")
        if sizes is None:
            ladder, t = [], 48
            while t < self.token_budget:
                ladder.append(t)
                t = t * 3 // 2
            sizes = list(range(1, 33)) + ladder + [self.token_budget]
        dev = self.device
        n = 0
        with self.stream_ctx():
            for T in sizes:
                T = int(min(max(1, T), self.token_budget))
                r = torch.arange(T, device=dev, dtype=torch.int32)
                seg = min(16, self.max_ctx)
                slot = (r // seg) % self.slots
                pos = r % seg
                t0 = torch.arange(0, T, seg, device=dev, dtype=torch.int32)
                tiles = torch.stack([t0, torch.clamp(T - t0, max=seg), (t0 // seg) % self.slots,
                                     torch.zeros_like(t0)], 1).contiguous() if self.use_tiles else None
                samp = torch.arange(min(T, self.slots), device=dev, dtype=torch.long)
                self.model.forward(torch.zeros(T, dtype=torch.long, device=dev), pos.contiguous(),
                                   slot.contiguous(), samp, tiles=tiles, n_dec=0)
                n += 1
            if getattr(self.model, "prune_last", False) and hasattr(self.model, "warm_tail"):
                # the pruned last layer runs at the sampled-row count: a finer ladder
                tail, t = list(range(1, 33)), 32
                while t < self.token_budget:
                    t = max(t + 1, t * 9 // 8)
                    tail.append(min(t, self.token_budget))
                n += self.model.warm_tail(tail)
        if self.rt_stream is not None:
            # the micro-forwards' stream: its per-stream GEMM workspaces and
            # first launches there, on the micro pool's own slots
            torch.cuda.synchronize(dev)
            with torch.cuda.stream(self.rt_stream):
                T = 1
                while T <= self.micro_budget:
                    r = torch.arange(T, device=dev, dtype=torch.int32)
                    slot = (self.slots + r % self.micro_slots).to(torch.int32)
                    pos = (r // self.micro_slots).to(torch.int32)
                    tiles = torch.stack([r, torch.ones_like(r), slot, pos], 1).contiguous() \
                        if self.use_tiles else None
                    samp = torch.arange(min(T, self.micro_slots), device=dev, dtype=torch.long)
                    if self.micro_cus and self.micro_gemm == "rocblas":
                        with _blas("cublas"):
                            self.model.forward(torch.zeros(T, dtype=torch.long, device=dev), pos.contiguous(),
                                               slot.contiguous(), samp, tiles=tiles, n_dec=0)
                    else:
                        self.model.forward(torch.zeros(T, dtype=torch.long, device=dev), pos.contiguous(),
                                           slot.contiguous(), samp, tiles=tiles, n_dec=0,
                                           **({"small_cus": self.micro_cus} if self.micro_cus else {}))
                    n += 1
                    T *= 2
        if self.micro_graph:
            n += self._capture_micro_graphs()
        torch.cuda.synchronize(dev)
        self.warmed_shapes = n
        return n

    def _launch_micro_graph(self, Tb: int, t0: float, t_mono: int, pos, slot, samp_slots, dec_src) -> bool:
        """A decode-only micro-forward of D <= Tb rows as a replay of bucket
        Tb's graph: one staging copy, the decode-id gather from the previous
        micro-forward's output, the replay, the id copy back.  Rows D.. Tb
        stay on the scratch slot."""
        graph, g_in, g_tok, out = self._mg[Tb]
        D = len(pos)
        buf = np.empty(7 * Tb, dtype=np.int32)
        buf[:Tb] = 0
        buf[:D] = pos
        buf[Tb:2 * Tb] = self.scratch_slot
        buf[Tb:Tb + D] = slot
        til = buf[2 * Tb:6 * Tb].reshape(Tb, 4)
        til[:, 0] = np.arange(Tb)
        til[:, 1] = 1
        til[:, 2] = buf[Tb:2 * Tb]
        til[:, 3] = buf[:Tb]
        buf[6 * Tb:6 * Tb + D] = dec_src
        buf[6 * Tb + D:] = 0
        sid = self.micro_id
        k = sid % len(self._pins_m)
        pin = self._pins_m[k]
        pin.numpy()[:buf.nbytes] = buf.view(np.uint8)
        host_out = self._out_pins_m[k]
        prev = self._prev_out_m
        with torch.cuda.stream(self.rt_stream):
            g_in.copy_(pin[:buf.nbytes].view(torch.int32), non_blocking=True)
            g_tok[:D] = prev.index_select(0, g_in[6 * Tb:6 * Tb + D].long()).long()
            if D < Tb:
                g_tok[D:] = 0
            ev0 = self._start_event()
            te = time.perf_counter_ns()
            graph.replay()
            self.host_ns[2] += time.perf_counter_ns() - te
            host_out[:D].copy_(out[:D], non_blocking=True)
            ev = self._end_event(D, ev0 is not None)
        # the same deterministic bookkeeping as an eager micro-forward
        ss = samp_slots
        gidx = self.s_gen[ss].copy()
        self.s_gen[ss] += 1
        self.s_out_idx[ss] = np.arange(len(ss))
        self.s_out_step[ss] = sid
        g = self.s_gen[ss]
        firsts = [self.active[int(x)] for x in ss[g == 1]]
        done = ss[g >= self.s_gmax[ss]]
        completed = []
        for x in done.tolist():
            r = self.active.pop(x)
            r.prefilled = int(self.s_plen[x]) - r.reused
            r.generated = int(self.s_gen[x])
            completed.append(r)
            self.s_conv[x] = -1
            self.free_micro.append(x)
        self.s_active[done] = False
        f = _Inflight(sid, ev, D, 0, D, completed, firsts, t0, out, t_mono, ev0, micro=True,
                      samp_slots=ss, gidx=gidx, host_out=host_out)
        self._prev_out_m = out
        self._qm.append(f)
        self.micro_id += 1
        self.micro_steps += 1
        self.micro_graph_steps += 1
        self.total_tokens += D
        self.matmul_flops += self._step_flops(D, D)
        self.completed_total += len(completed)
        self.completed_tokens += sum(len(r.prompt) + r.gen_tokens - 1 for r in completed)
        return True

    def _micro_forward_kw(self) -> dict:
        return {"small_cus": self.micro_cus} if self.micro_cus else {}

    def _capture_micro_graphs(self) -> int:
        """Capture the decode-only micro-forward once per row bucket on the
        micro stream (after ``warm_shapes`` ran it eagerly: workspaces and
        first launches exist).  Static inputs per bucket: int32 [pos | slot |
        tiles (4 per row) | gather rows] and the int64 token ids; every row
        starts on the scratch slot at position 0, so a replay's padding rows
        write and read only that slot."""
        dev, rt = self.device, self.rt_stream
        pool = torch.cuda.graph_pool_handle()
        n = 0
        for Tb in self.MICRO_GRAPH_BUCKETS:
            if Tb > max(self.MICRO_GRAPH_BUCKETS[0], self.micro_slots):
                break
            g_in = torch.zeros(6 * Tb + Tb, dtype=torch.int32, device=dev)
            g_tok = torch.zeros(Tb, dtype=torch.long, device=dev)
            pos, slot = g_in[:Tb], g_in[Tb:2 * Tb]
            til = g_in[2 * Tb:6 * Tb].view(Tb, 4)
            slot.fill_(self.scratch_slot)
            til[:, 0] = torch.arange(Tb, device=dev, dtype=torch.int32)
            til[:, 1] = 1
            til[:, 2] = self.scratch_slot
            samp = torch.arange(Tb, device=dev, dtype=torch.long)
            kw = self._micro_forward_kw()
            torch.cuda.synchronize(dev)
            with torch.cuda.stream(rt):
                for _ in range(2):
                    self.model.forward(g_tok, pos, slot, samp, tiles=til, n_dec=Tb, **kw)
            torch.cuda.synchronize(dev)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, pool=pool, stream=rt, capture_error_mode="thread_local"):
                out = self.model.forward(g_tok, pos, slot, samp, tiles=til, n_dec=Tb, **kw)
            torch.cuda.synchronize(dev)
            self._mg[Tb] = (graph, g_in, g_tok, out)
            n += 1
        return n

    def inject(self, **fault) -> None:
        """Fault injection: ``fail_launch=n``, ``slow_ms=x``, ``drop_heartbeat=True``
        (0/False clears one)."""
        for k, v in fault.items():
            if k not in ("fail_launch", "slow_ms", "drop_heartbeat"):
                raise ValueError(f"unknown fault {k!r}")
            if v:
                self.fault[k] = v
            else:
                self.fault.pop(k, None)

    def fence(self, events) -> None:
        """Device events the next launch waits for (work that may still write
        slots this engine is about to reuse: evacuated steps, abandoned KV
        imports)."""
        self._fence.extend(e for e in events if e is not None)

    def abort_all(self) -> List[Request]:
        """Evacuate: drop every queued step and active request (slots are
        freed) and return the unfinished requests so the caller can re-route
        them.  Steps not yet reaped by ``finish`` count as unfinished (their
        completions were never reported): at-least-once.  Makes no GPU call,
        so it is safe after a device error; reap first if the GPU is fine."""
        steps = list(self._q) + self._reaped + list(self._qm) + self._reaped_m
        out = [r for f in steps for r in f.completed]
        out += list(self.active.values())
        for r in out:
            r.aborted = True
        # steps still queued on the GPU keep reading their pinned staging
        # buffers (the async H2D copy may not have run yet): the next launch
        # must not refill a buffer before they finish, so their events stay
        # as a fence (waited in launch; a dead device raises there instead)
        self._fence.extend(f.event for f in list(self._q) + list(self._qm) if f.event is not None)
        self._q.clear()
        self._reaped = []
        self._prev_out = None
        self._qm.clear()
        self._reaped_m = []
        self._prev_out_m = None
        self.active.clear()
        self.s_active[:] = False
        self.s_deadline[:] = 0
        self.conv_lru.clear()
        self._importing.clear()
        self.s_conv[:] = -1
        self.free = list(range(self.slots - 1, -1, -1))
        self.free_micro = list(range(self.slots + self.micro_slots - 1, self.slots - 1, -1))
        return out

    def launch(self, wait_cb=None) -> None:
        """Build the next token batch and enqueue its forward (async).

        If ``max_inflight`` steps are already queued, wait for the oldest;
        with ``wait_cb`` the wait polls the step's event and calls
        ``wait_cb()`` in between (the gateway keeps ingesting/dispatching
        while the GPU computes) instead of blocking."""
        if self.fault:
            if self.fault.get("fail_launch", 0) > 0:
                self.fault["fail_launch"] -= 1
                if self.fault["fail_launch"] <= 0:
                    del self.fault["fail_launch"]
                raise RuntimeError("HIP error: out of memory (injected fault)")
            if self.fault.get("slow_ms"):
                time.sleep(self.fault["slow_ms"] / 1e3)
        ts = time.perf_counter_ns()
        if self._fence:                                # steps dropped by abort_all still in flight
            for ev in self._fence:
                ev.synchronize()
            self._fence = []
        while len(self._q) >= self.max_inflight:       # bound the run-ahead (and staging reuse)
            if wait_cb is None:
                self._reaped.append(self._reap(block=True))  # handed to the next finish()
                continue
            f = self._reap(block=False)
            if f is not None:
                self._reaped.append(f)
                continue
            if self.micro:
                self.pump_micro()                      # realtime micro-forwards keep flowing meanwhile
            if not wait_cb():
                time.sleep(0.0002)
        self.host_ns[1] += time.perf_counter_ns() - ts
        self._launch_pool(False)

    def close(self) -> None:
        """Drain the GPU work of this engine.  The CU-partition streams
        (``micro_stream=partition``) are process-wide and stay alive
        (``cu_partition.partition_streams``): tensors this engine allocated
        on them may outlive it, and freeing one returns its block to the
        stream it was allocated on."""
        if self.cuda:
            torch.cuda.synchronize(self.device)

    def stream_ctx(self):
        """Context that makes the serving steps' stream current (a no-op
        unless the chip is CU-partitioned): anything else ordered with the
        serving steps -- KV imports, the slot census -- runs inside it."""
        return torch.cuda.stream(self.main_stream) if self.main_stream is not None else _NullCtx()

    def _launch_pool(self, micro: bool) -> bool:
        """Build one pool's next token batch and enqueue its forward: the
        serving step, or (``micro``) a realtime micro-forward on the micro
        stream.  False if the pool had no token to run."""
        t0 = time.perf_counter()
        tb = time.perf_counter_ns()
        t_mono = time.monotonic_ns()
        toks, pos, slot, samp, samp_slots, dec_rows, dec_src, tiles, n_pre, n_dec = self._build(micro)
        self.host_ns[0] += time.perf_counter_ns() - tb
        T = len(toks)
        if T == 0:
            return False
        dev = self.device
        S, D, NT = len(samp), len(dec_rows), len(tiles)
        if micro and self._mg and n_pre == 0 and D == T and self._prev_out_m is not None:
            Tb = next((b for b in self.MICRO_GRAPH_BUCKETS if b >= T and b in self._mg), 0)
            if Tb:
                return self._launch_micro_graph(Tb, t0, t_mono, pos, slot, samp_slots, dec_src)
        o_dec = 3 * T + S
        o_til = o_dec + 2 * D
        buf = np.empty(o_til + 4 * NT, dtype=np.int32)
        buf[:T] = toks
        buf[T:2 * T] = pos
        buf[2 * T:3 * T] = slot
        buf[3 * T:o_dec] = samp
        buf[o_dec:o_dec + D] = dec_rows
        buf[o_dec + D:o_til] = dec_src
        buf[o_til:] = tiles.reshape(-1)
        nbytes = buf.nbytes
        sid = self.micro_id if micro else self.step_id
        pins, outs = (self._pins_m, self._out_pins_m) if micro else (self._pins, self._out_pins)
        k = sid % len(pins)
        pin = pins[k]
        if pin.numel() < nbytes:
            pin = pins[k] = self._alloc_pin(2 * nbytes)
        pin.numpy()[:nbytes] = buf.view(np.uint8)
        host_out = outs[k]
        prev = self._prev_out_m if micro else self._prev_out
        stream = self.rt_stream if micro else self.main_stream
        ctx = torch.cuda.stream(stream) if stream is not None else _NullCtx()
        with ctx:
            d = pin[:nbytes].to(dev, non_blocking=True).view(torch.int32)
            tok_d = d[:T].long()
            if D:
                if prev is None:
                    raise RuntimeError("decode token without a previous step output")
                rows = d[o_dec:o_dec + D].long()
                src = d[o_dec + D:o_til].long()
                tok_d.index_copy_(0, rows, prev.index_select(0, src).long())
            til = d[o_til:].view(NT, 4) if self.use_tiles else None
            ev0 = self._start_event()
            te = time.perf_counter_ns()
            if micro and self.micro_cus and self.micro_gemm == "rocblas":
                with _blas("cublas"):
                    out = self.model.forward(tok_d, d[T:2 * T], d[2 * T:3 * T], d[3 * T:o_dec].long(), tiles=til,
                                             n_dec=D)
            else:
                out = self.model.forward(tok_d, d[T:2 * T], d[2 * T:3 * T], d[3 * T:o_dec].long(), tiles=til,
                                         n_dec=D,
                                         **({"small_cus": self.micro_cus} if micro and self.micro_cus else {}))
            self.host_ns[2] += time.perf_counter_ns() - te
            if not micro:
                self._census(T)
            # the sampled ids come back behind the forward (read at reap)
            host_out[:S].copy_(out, non_blocking=True)
            ev = self._end_event(T, ev0 is not None)
        # deterministic bookkeeping: every sampled slot gets one token
        ss = samp_slots
        gidx = self.s_gen[ss].copy()
        self.s_gen[ss] += 1
        self.s_out_idx[ss] = np.arange(len(ss))
        self.s_out_step[ss] = sid
        g = self.s_gen[ss]
        firsts = [self.active[int(x)] for x in ss[g == 1]]
        done = ss[g >= self.s_gmax[ss]]
        completed = []
        for x in done.tolist():
            r = self.active.pop(x)
            r.prefilled = int(self.s_plen[x]) - r.reused
            r.generated = int(self.s_gen[x])
            completed.append(r)
            if micro:
                self.s_conv[x] = -1
                self.free_micro.append(x)
            elif r.conv >= 0:
                # park the dialog KV: every position but the last sampled token
                self.s_cached[x] = self.s_plen[x] + self.s_gen[x] - 1
                old = self.conv_lru.pop(r.conv, None)
                if old is not None and old != x:           # a stale copy elsewhere: free it
                    self.s_conv[old] = -1
                    self.free.append(old)
                self.conv_lru[r.conv] = x
            else:
                self.s_conv[x] = -1
                self.free.append(x)
        self.s_active[done] = False
        f = _Inflight(sid, ev, T, n_pre, n_dec, completed, firsts, t0, out, t_mono, ev0, micro=micro,
                      samp_slots=ss, gidx=gidx, host_out=host_out)
        if micro:
            self._prev_out_m = out
            self._qm.append(f)
            self.micro_id += 1
            self.micro_steps += 1
        else:
            self._prev_out = out
            self._q.append(f)
            self.step_id += 1
        self.total_tokens += T
        self.matmul_flops += self._step_flops(T, S)
        self.completed_total += len(completed)
        self.completed_tokens += sum(len(r.prompt) + r.gen_tokens - 1 for r in completed)
        return True

    def _step_flops(self, T: int, S: int) -> int:
        """Matrix-multiply FLOPs of one forward of ``T`` tokens sampling ``S``
        rows: every layer's qkv / o / gate-up / down over every row (the last
        layer's o + MLP over the sampled rows only, with ``prune_last``) and
        the LM head over the sampled rows.  Attention (<= max_ctx keys per
        row, ~0.2 % at the serving shape) is not counted."""
        c = self.cfg
        d, hd = c.dim, c.head_dim
        qkv = d * (c.heads + 2 * c.kv_heads) * hd
        rest = c.heads * hd * d + 3 * d * c.ffn                 # o + gate/up + down
        last = S if getattr(self.model, "prune_last", False) else T
        return 2 * (T * (c.layers * qkv + (c.layers - 1) * rest) + last * rest + S * c.vocab * d)

    # ------------------------------------------------------------------ realtime micro-forwards
    def micro_pending(self) -> bool:
        """A micro-pool request still has tokens no launched micro-forward
        computes (prefill left, or generation not yet launched to the end)."""
        if not self.micro or len(self.free_micro) == self.micro_slots:
            return False
        act = self.s_active & self.s_micro
        return bool(act.any())

    def pump_micro(self) -> int:
        """Reap finished micro-forwards (their results go to the next
        ``finish`` / ``finish_micro``) and launch the next ones while the
        micro pool has work and fewer than ``micro_inflight`` are queued.
        Bookkeeping is deterministic (greedy decode always yields a token),
        so a realtime request's whole prefill + decode chain can be queued
        at once: each micro-forward gathers its decode ids on the device from
        the previous one.  Returns the number launched."""
        if not self.micro:
            return 0
        while self._qm:
            f = self._reap(block=False, micro=True)
            if f is None:
                break
            self._reaped_m.append(f)
        n = 0
        while len(self._qm) < self.micro_inflight and self.micro_pending():
            if not self._launch_pool(True):
                break
            n += 1
        return n

    def finish_micro(self) -> StepResult:
        """Results of the micro-forwards reaped so far (non-blocking)."""
        done, self._reaped_m = self._reaped_m, []
        return self._result(done)

    def _start_event(self):
        """Timing event before a forward (``time_steps``), or None."""
        if self.cuda and self.time_steps:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
            return ev0
        return None

    def _end_event(self, T: int, timing: bool):
        """Completion event of the forward just enqueued (None: the step ran
        synchronously on the host)."""
        if not self.cuda:
            return None
        ev = torch.cuda.Event(enable_timing=timing)
        ev.record()
        return ev

    def _check_hung(self, f: _Inflight) -> None:
        if self.step_timeout_s > 0 and f.t0_ns and \
                time.monotonic_ns() - f.t0_ns > self.step_timeout_s * 1e9:
            raise BackendHung(f"forward step {f.step} ({f.T} tokens) incomplete "
                              f"{(time.monotonic_ns() - f.t0_ns) / 1e9:.1f} s after launch")

    def _reap(self, block: bool, micro: bool = False) -> Optional[_Inflight]:
        q = self._qm if micro else self._q
        if not q:
            return None
        f = q[0]
        if f.event is not None:
            if block:
                if self.step_timeout_s > 0:
                    while not f.event.query():         # bounded: a hung GPU surfaces as BackendHung
                        self._check_hung(f)
                        time.sleep(0.0001)
                else:
                    f.event.synchronize()
            elif not f.event.query():
                self._check_hung(f)
                return None
        q.popleft()
        now = time.monotonic_ns()
        if f.ev_start is not None:
            ms = f.ev_start.elapsed_time(f.event)
            if micro:
                self.micro_gpu_ms += ms
                self.micro_timed += 1
            else:
                self.gpu_step_ms += ms
                self.gpu_steps += 1
                self.gpu_step_max_ms = max(self.gpu_step_max_ms, ms)
        if self.tracer is not None:
            self.tracer.step(f.step, f.t0_ns, now, f.T)
        if f.host_out is not None and f.samp_slots is not None and len(f.samp_slots):
            # the step's sampled ids (valid now: the copy ran before its event)
            ss = f.samp_slots
            ok = f.gidx < self.max_ctx
            self.h_tokens[ss[ok], f.gidx[ok]] = f.host_out.numpy()[:len(ss)][ok]
        for r in f.firsts:
            if not r.aborted:
                r.first_token_ns = now
        for r in f.completed:
            r.done_ns = now
            r.out_tokens = self.h_tokens[r.slot, :min(r.generated, self.max_ctx)].copy()
        if self.page is not None and not self.cuda and not self.fault.get("drop_heartbeat") and not micro:
            self.page.write_host(self.inflight(), self.free_slots(), f.T, f.step)
        return f

    def queued_steps(self) -> int:
        """Forward steps launched and not yet reaped (serving steps and
        realtime micro-forwards)."""
        return len(self._q) + len(self._qm)

    def poll_one(self) -> bool:
        """Reap the oldest queued step if the GPU finished it (non-blocking);
        its results are returned by the next ``finish``."""
        f = self._reap(block=False)
        if f is None:
            if self._qm:
                return self.pump_micro() > 0 or bool(self._reaped_m)
            return False
        self._reaped.append(f)
        return True

    @staticmethod
    def _result(done: List[_Inflight]) -> StepResult:
        comp = [r for f in done for r in f.completed]
        firsts = [r for f in done for r in f.firsts]
        return StepResult(sum(f.T for f in done), sum(f.n_pre for f in done), sum(f.n_dec for f in done),
                          comp, firsts, (time.perf_counter() - done[0].t0) * 1e3 if done else 0.0)

    def finish(self, block: bool = False) -> StepResult:
        """Reap finished steps (and micro-forwards).  Non-blocking unless
        ``block`` (then waits for every queued one)."""
        done: List[_Inflight] = self._reaped
        self._reaped = []
        while self._q:
            f = self._reap(block=block)
            if f is None:
                break
            done.append(f)
        if self.micro:
            while True:
                self.pump_micro()
                done.extend(self._reaped_m)
                self._reaped_m = []
                if not block or not (self._qm or self.micro_pending()):
                    break
                f = self._reap(block=True, micro=True)
                if f is not None:
                    done.append(f)
        return self._result(done)

    def step(self) -> StepResult:
        """Synchronous step: launch + wait."""
        self.launch()
        return self.finish(block=True)

    def sync(self) -> None:
        self.finish(block=True)

    # ------------------------------------------------------------------ N9 page
    def _census(self, tokens: int) -> None:
        if self.page is None or not self.cuda or self.page.dev_ptr is None or self.fault.get("drop_heartbeat"):
            return
        pin = self._state_pins[self.step_id % 2]
        st = pin.numpy().view(np.int32)
        st[:] = 0
        if self.active:
            a = np.fromiter(self.active.keys(), dtype=np.int64)
            st[a[a < self.slots]] = 1                      # (the serving pool's census)
        self._slot_state_d.copy_(pin.view(torch.int32), non_blocking=True)
        from .. import _native
        _native.require_hipops().slot_census(self._slot_state_d.data_ptr(), self.slots, int(tokens),
                                             int(self.step_id) & 0xFFFFFFFF, self.page.dev_ptr,
                                             torch.cuda.current_stream(self.device).cuda_stream)

    def drain(self, max_steps: int = 10000) -> List[Request]:
        out = []
        for _ in range(max_steps):
            if not self.active:
                break
            out.extend(self.step().completed)
        out.extend(self.finish(block=True).completed)
        return out
