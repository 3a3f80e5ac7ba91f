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


@dataclass
class StepResult:
    tokens: int
    prefill_tokens: int
    decode_tokens: int
    completed: List[Request]
    first_tokens: List[Request]
    elapsed_ms: float


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


class BackendEngine:
    def __init__(self, model_cfg: LlamaConfig, slots: int = 256, max_ctx: int = 512,
                 token_budget: int = 2048, device="cuda", impl: str = "hip", seed: int = 0,
                 page=None, gpu_index: int = 0, max_inflight: int = 2):
        self.cfg = model_cfg
        self.slots = slots
        self.max_ctx = max_ctx
        # every generating slot gets its decode token each step (the on-device
        # token gather reads the previous step's output only)
        self.token_budget = max(token_budget, slots)
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.model = LlamaStub(model_cfg, slots, max_ctx, device=self.device, impl=impl, seed=seed)
        self.impl = impl
        self.active: Dict[int, Request] = {}            # slot -> request
        self.free: List[int] = list(range(slots - 1, -1, -1))
        self.page = page
        self.gpu_index = gpu_index
        self.max_inflight = max(1, max_inflight)
        self.step_id = 0
        self.total_tokens = 0
        self.completed_total = 0
        self.completed_tokens = 0
        self._q: Deque[_Inflight] = collections.deque()
        self._reaped: List[_Inflight] = []               # reaped by launch(), not yet returned
        self._prev_out = None                            # device int32 [n_samples] of the last launched step
        # double-buffered pinned staging (a buffer is reused only after the
        # step that read it has finished: <= 2 steps in flight)
        self._pins = [self._alloc_pin(4 * (3 * token_budget + 2 * slots + 64)) for _ in range(2)]
        self._state_pins = [self._alloc_pin(4 * slots) for _ in range(2)]
        self._slot_state_d = torch.zeros(slots, dtype=torch.int32, device=self.device)
        # fault injection: {"fail_launch": n} raises on the next
        # n launches (a HIP error / OOM), {"slow_ms": x} stalls every launch,
        # {"drop_heartbeat": True} stops the load-page census
        self.fault: Dict[str, float] = {}
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
        return len(self.free)

    def inflight(self) -> int:
        return self.slots - len(self.free)

    def admit(self, reqs: Sequence[Request]) -> List[Request]:
        now = time.monotonic_ns()
        out = []
        cap = self.max_ctx - 1
        for r in reqs:
            if not self.free:
                break
            if r.gen_tokens < 1:
                r.gen_tokens = 1
            plen = max(1, min(len(r.prompt), cap - r.gen_tokens + 1))
            r.prompt = np.asarray(r.prompt[:plen], dtype=np.int64) % self.cfg.vocab
            if len(r.prompt) == 0:
                r.prompt = np.zeros(1, dtype=np.int64)
            r.slot = self.free.pop()
            r.prefilled = 0
            r.generated = 0
            r.out_idx = r.out_step = -1
            r.admitted_ns = now
            self.active[r.slot] = r
            out.append(r)
        return out

    # ------------------------------------------------------------------ step
    def _build(self):
        toks, pos, slot, samp, sample_reqs = [], [], [], [], []
        dec_rows, dec_src = [], []
        budget = self.token_budget
        n_dec = n_pre = 0
        # decode tokens first (in-flight generations keep their cadence);
        # their ids are gathered on the device from the previous output
        for s, r in self.active.items():
            if r.prefilled >= len(r.prompt):
                if r.out_step != self.step_id - 1:
                    raise RuntimeError("decode token source is not the previous step")
                ctx = len(r.prompt) + r.generated - 1
                dec_rows.append(len(toks))
                dec_src.append(r.out_idx)
                toks.append(0)
                pos.append(ctx)
                slot.append(s)
                samp.append(len(toks) - 1)
                sample_reqs.append(r)
                budget -= 1
                n_dec += 1
        # then chunked prefill in admission order
        for s, r in sorted(self.active.items(), key=lambda kv: kv[1].admitted_ns):
            if budget <= 0:
                break
            rem = len(r.prompt) - r.prefilled
            if rem <= 0:
                continue
            n = min(rem, budget)
            a = r.prefilled
            toks.extend(r.prompt[a:a + n].tolist())
            pos.extend(range(a, a + n))
            slot.extend([s] * n)
            r.prefilled += n
            budget -= n
            n_pre += n
            if r.prefilled >= len(r.prompt):
                samp.append(len(toks) - 1)
                sample_reqs.append(r)
        return toks, pos, slot, samp, sample_reqs, dec_rows, dec_src, n_pre, n_dec

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

    def abort_all(self) -> List[Request]:
        """Evacuate: drop every queued step and active request (slots are
        freed) and return the unfinished requests so the caller can re-route
        them.  Steps not yet reaped by ``finish`` count as unfinished (their
        completions were never reported): at-least-once.  Makes no GPU call,
        so it is safe after a device error; reap first if the GPU is fine."""
        out = [r for f in list(self._q) + self._reaped for r in f.completed]
        out += list(self.active.values())
        self._q.clear()
        self._reaped = []
        self._prev_out = None
        self.active.clear()
        self.free = list(range(self.slots - 1, -1, -1))
        return out

    def launch(self) -> None:
        """Build the next token batch and enqueue its forward (async)."""
        if self.fault:
            if self.fault.get("fail_launch", 0) > 0:
                self.fault["fail_launch"] -= 1
                if self.fault["fail_launch"] <= 0:
                    del self.fault["fail_launch"]
                raise RuntimeError("HIP error: out of memory (injected fault)")
            if self.fault.get("slow_ms"):
                time.sleep(self.fault["slow_ms"] / 1e3)
        while len(self._q) >= self.max_inflight:       # bound the run-ahead (and staging reuse)
            self._reaped.append(self._reap(block=True))  # handed to the next finish()
        t0 = time.perf_counter()
        toks, pos, slot, samp, sample_reqs, dec_rows, dec_src, n_pre, n_dec = self._build()
        T = len(toks)
        if T == 0:
            return
        dev = self.device
        S, D = len(samp), len(dec_rows)
        buf = np.empty(3 * T + S + 2 * D, dtype=np.int32)
        buf[:T] = toks
        buf[T:2 * T] = pos
        buf[2 * T:3 * T] = slot
        buf[3 * T:3 * T + S] = samp
        buf[3 * T + S:3 * T + S + D] = dec_rows
        buf[3 * T + S + D:] = dec_src
        nbytes = buf.nbytes
        pin = self._pins[self.step_id % 2]
        if pin.numel() < nbytes:
            pin = self._pins[self.step_id % 2] = self._alloc_pin(2 * nbytes)
        pin[:nbytes].numpy()[:] = buf.view(np.uint8)
        d = pin[:nbytes].to(dev, non_blocking=True).view(torch.int32)
        tok_d = d[:T].long()
        if D:
            if self._prev_out is None:
                raise RuntimeError("decode token without a previous step output")
            rows = d[3 * T + S:3 * T + S + D].long()
            src = d[3 * T + S + D:].long()
            tok_d.index_copy_(0, rows, self._prev_out.index_select(0, src).long())
        out = self.model.forward(tok_d, d[T:2 * T], d[2 * T:3 * T], d[3 * T:3 * T + S].long())
        self._census(T)
        ev = None
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record()
        # deterministic bookkeeping: every sampled request gets one token
        completed, firsts = [], []
        for i, r in enumerate(sample_reqs):
            r.generated += 1
            r.out_idx, r.out_step = i, self.step_id
            if r.generated == 1:
                firsts.append(r)
            if r.generated >= r.gen_tokens:
                completed.append(r)
        for r in completed:
            del self.active[r.slot]
            self.free.append(r.slot)
        self._prev_out = out
        self._q.append(_Inflight(self.step_id, ev, T, n_pre, n_dec, completed, firsts, t0, out))
        self.step_id += 1
        self.total_tokens += T
        self.completed_total += len(completed)
        self.completed_tokens += sum(len(r.prompt) + r.gen_tokens - 1 for r in completed)

    def _reap(self, block: bool) -> Optional[_Inflight]:
        if not self._q:
            return None
        f = self._q[0]
        if f.event is not None:
            if block:
                f.event.synchronize()
            elif not f.event.query():
                return None
        self._q.popleft()
        now = time.monotonic_ns()
        for r in f.firsts:
            r.first_token_ns = now
        for r in f.completed:
            r.done_ns = now
        if self.page is not None and not self.cuda and not self.fault.get("drop_heartbeat"):
            self.page.write_host(self.inflight(), self.free_slots(), f.T, f.step)
        return f

    def finish(self, block: bool = False) -> StepResult:
        """Reap finished steps.  Non-blocking unless ``block`` (then waits for
        every queued step)."""
        done: List[_Inflight] = self._reaped
        self._reaped = []
        while self._q:
            f = self._reap(block=block)
            if f is None:
                break
            done.append(f)
        comp = [r for f in done for r in f.completed]
        firsts = [r for f in done for r in f.firsts]
        return StepResult(sum(f.T for f in done), sum(f.n_pre for f in done), sum(f.n_dec for f in done),
                          comp, firsts, (time.perf_counter() - done[0].t0) * 1e3 if done else 0.0)

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
            st[np.fromiter(self.active.keys(), dtype=np.int64)] = 1
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
