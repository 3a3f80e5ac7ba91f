"""GPU backend engine: continuous batching over fixed batch slots (N12 + N9).

One engine per GPU process.  ``admit`` places dispatched requests into free
slots; ``step`` runs ONE model forward over a token batch made of
  * one decode token for every slot that is generating, then
  * chunked-prefill tokens of newly admitted prompts, up to ``token_budget``;
samples the next token for every slot whose chunk ended its prompt or that
decoded, retires requests that reached ``gen_tokens``, and publishes the
slot census to the node-shared load page (``slot_census`` kernel -> mapped
host page, read zero-copy by routers).

Request cost model (documented in README/bench): prompt = the message's
tokens from the GPU tokenizer (capped), generation = ``gen_tokens`` greedy
tokens.  This is real work on the full 32-layer stub, never skipped.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

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
    last_token: int = 0
    admitted_ns: int = 0
    first_token_ns: int = 0
    done_ns: int = 0
    meta: object = None


@dataclass
class StepResult:
    tokens: int
    prefill_tokens: int
    decode_tokens: int
    completed: List[Request]
    first_tokens: List[Request]
    elapsed_ms: float


class BackendEngine:
    def __init__(self, model_cfg: LlamaConfig, slots: int = 256, max_ctx: int = 512,
                 token_budget: int = 2048, device="cuda", impl: str = "hip", seed: int = 0,
                 page=None, gpu_index: int = 0):
        self.cfg = model_cfg
        self.slots = slots
        self.max_ctx = max_ctx
        self.token_budget = token_budget
        self.device = torch.device(device)
        self.model = LlamaStub(model_cfg, slots, max_ctx, device=self.device, impl=impl, seed=seed)
        self.impl = impl
        self.active: Dict[int, Request] = {}            # slot -> request
        self.free: List[int] = list(range(slots - 1, -1, -1))
        self.waiting: List[Request] = []                 # admitted, prefill not started/finished
        self.page = page
        self.gpu_index = gpu_index
        self.step_id = 0
        self._pending = None
        self.total_tokens = 0
        self.completed_tokens = 0
        self.completed_total = 0
        self._slot_state_h = torch.zeros(slots, dtype=torch.int32).pin_memory() if self.device.type == "cuda" \
            else torch.zeros(slots, dtype=torch.int32)
        self._slot_state_d = torch.zeros(slots, dtype=torch.int32, device=self.device)
        self._pin = torch.empty(4 * (token_budget * 4 + 16), dtype=torch.uint8)
        if self.device.type == "cuda":
            self._pin = self._pin.pin_memory()
            if page is not None and page.dev_ptr is None:
                page.register_device()
        if page is not None:
            page.set_health(True)
            self._publish(0)

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
            r.prompt = np.asarray(r.prompt[:plen], dtype=np.int32) % self.cfg.vocab
            if len(r.prompt) == 0:
                r.prompt = np.zeros(1, dtype=np.int32)
            r.slot = self.free.pop()
            r.prefilled = 0
            r.generated = 0
            r.admitted_ns = now
            self.active[r.slot] = r
            out.append(r)
        return out

    # ------------------------------------------------------------------ step
    def _build(self):
        toks, pos, slot, samp, sample_reqs = [], [], [], [], []
        budget = self.token_budget
        n_dec = n_pre = 0
        # decode tokens first (in-flight generations keep their cadence)
        for s, r in self.active.items():
            if r.prefilled >= len(r.prompt) and budget > 0:
                ctx = len(r.prompt) + r.generated - 1
                toks.append(r.last_token)
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
        return toks, pos, slot, samp, sample_reqs, n_pre, n_dec

    def step(self) -> StepResult:
        """Synchronous step: launch + finish."""
        self.launch()
        return self.finish()

    def launch(self) -> None:
        """Build the token batch and enqueue the forward on the current HIP
        stream WITHOUT waiting for it; ``finish`` collects the result.  The
        gateway overlaps its host work (ingest, preprocess on a side stream)
        with the forward between the two calls."""
        if self._pending is not None:
            raise RuntimeError("launch() called twice without finish()")
        t0 = time.perf_counter()
        toks, pos, slot, samp, sample_reqs, n_pre, n_dec = self._build()
        T = len(toks)
        nxt = None
        if T:
            dev = self.device
            S = len(samp)
            buf = np.empty(3 * T + S, dtype=np.int32)
            buf[:T] = toks
            buf[T:2 * T] = pos
            buf[2 * T:3 * T] = slot
            buf[3 * T:] = samp
            nbytes = buf.nbytes
            if self._pin.numel() < nbytes:
                self._pin = torch.empty(2 * nbytes, dtype=torch.uint8)
                if dev.type == "cuda":
                    self._pin = self._pin.pin_memory()
            self._pin[:nbytes].numpy()[:] = buf.view(np.uint8)
            d = self._pin[:nbytes].to(dev, non_blocking=True).view(torch.int32)
            tok_d = d[:T].long()
            pos_d, slot_d = d[T:2 * T], d[2 * T:3 * T]
            samp_d = d[3 * T:].long()
            nxt = self.model.forward(tok_d, pos_d, slot_d, samp_d)
            self.step_id += 1
            self._publish(T, device_side=True)
            if dev.type == "cuda":
                nxt_h = torch.empty(nxt.shape, dtype=nxt.dtype).pin_memory()
                nxt_h.copy_(nxt, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
            else:
                nxt_h, ev = nxt, None
            nxt = (nxt_h, ev)
        self._pending = (t0, T, n_pre, n_dec, sample_reqs, nxt)

    def finish(self) -> StepResult:
        if self._pending is None:
            return StepResult(0, 0, 0, [], [], 0.0)
        t0, T, n_pre, n_dec, sample_reqs, nxt = self._pending
        self._pending = None
        completed: List[Request] = []
        firsts: List[Request] = []
        if T:
            nxt_h, ev = nxt
            if ev is not None:
                ev.synchronize()
            nxt_h = nxt_h.numpy()
            now = time.monotonic_ns()
            for r, t in zip(sample_reqs, nxt_h):
                r.last_token = int(t)
                r.generated += 1
                if r.generated == 1:
                    r.first_token_ns = now
                    firsts.append(r)
                if r.generated >= r.gen_tokens:
                    r.done_ns = now
                    completed.append(r)
            for r in completed:
                del self.active[r.slot]
                self.free.append(r.slot)
            self.total_tokens += T
            self.completed_total += len(completed)
            self.completed_tokens += sum(len(r.prompt) + r.gen_tokens - 1 for r in completed)
            if completed:
                self._publish(T, device_side=False)
        return StepResult(T, n_pre, n_dec, completed, firsts, (time.perf_counter() - t0) * 1e3)

    # ------------------------------------------------------------------ N9 page
    def _publish(self, tokens: int, device_side: bool = False) -> None:
        if self.page is None:
            return
        if device_side and self.device.type == "cuda" and self.page.dev_ptr is not None:
            st = self._slot_state_h.numpy()
            st[:] = 0
            for s in self.active:
                st[s] = 1
            self._slot_state_d.copy_(self._slot_state_h, non_blocking=True)
            from .. import _native
            _native.require_hipops().slot_census(self._slot_state_d.data_ptr(), self.slots, int(tokens),
                                                 int(self.step_id) & 0xFFFFFFFF, self.page.dev_ptr,
                                                 torch.cuda.current_stream(self.device).cuda_stream)
        else:
            self.page.write_host(self.inflight(), self.free_slots(), tokens, self.step_id)

    def drain(self, max_steps: int = 10000) -> List[Request]:
        out = []
        for _ in range(max_steps):
            if not self.active:
                break
            out.extend(self.step().completed)
        return out
