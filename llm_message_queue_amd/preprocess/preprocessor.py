"""Preprocessor (component C10): content-based priority + analysis metadata.

Reference: `internal/preprocessor/preprocessor.go`.  ``process_message``
follows `:56-114` step by step (explicit non-normal priority respected and NOT
analysed; ``metadata.user_priority`` override; per-user default; keyword
scoring; content analysis; ``analyzed=true``; queue name = ``priority.String()``).

Two execution paths with identical results:
  * ``process_message`` / ``process_batch(..., use_gpu=False)``: the exact CPU
    oracle (`oracle.py`);
  * ``process_batch(..., use_gpu=True)``: one fused ``text_analyze`` HIP launch
    for the whole micro-batch (word count, sentiment, question, keyword
    scores, token hashes) followed by the MFMA embedding classifier
    (``embed_classify``).  Messages containing the three fold-special
    characters (U+017F, U+212A, U+0130) are flagged by the kernel and
    re-scored by the oracle, so GPU results are bit-identical to the oracle.

Thread-safety: user priorities and patterns are guarded by a lock (the
reference's map writes are unguarded).
"""
from __future__ import annotations

import json
import threading
import time
from typing import Any, Dict, List, Optional, Sequence

from ..models.message import (Message, PRIORITY_NORMAL, level_priority_from_name,
                              priority_name)
from . import oracle

_PNAME = {p: priority_name(p) for p in range(0, 6)}


class Preprocessor:
    def __init__(self, cfg=None, *, use_gpu: Optional[bool] = None, device: str = "cuda"):
        """``cfg`` is a ``PreprocessorConfig`` (or None for defaults)."""
        from ..utils.config import PreprocessorConfig
        self.cfg = cfg or PreprocessorConfig()
        self._lock = threading.RLock()
        self._patterns: Dict[int, list] = oracle.default_patterns()
        self._user_priorities: Dict[str, int] = {}
        self.default_priority = PRIORITY_NORMAL
        self.positive_words = list(oracle.POSITIVE_WORDS)
        self.negative_words = list(oracle.NEGATIVE_WORDS)
        self.question_words = list(oracle.QUESTION_WORDS)
        self._want_gpu = self.cfg.use_gpu if use_gpu is None else use_gpu
        self._device = device
        self._gpu = None           # lazily-built ops.text.TextPipeline
        self._cpu = None           # lazily-built ops.text.CpuTextPipeline (False: unavailable)
        self._pattern_version = 0
        # metadata["analysis"] (AnalyzeMessageContent as JSON, `api/handlers.go:
        # 181-191`) for every message of a batch: set where raw requests are
        # preprocessed away from the API handler that adds it otherwise (the
        # GPU ranks behind the C++ front door, when queue.enable_metrics)
        self.record_analysis = False
        self.stats = {"gpu_batches": 0, "gpu_messages": 0, "oracle_fallbacks": 0,
                      "cpu_messages": 0, "last_gpu_ms": 0.0}

    # ------------------------------------------------------------------ admin
    def set_user_priority(self, user_id: str, priority: int) -> None:
        with self._lock:
            self._user_priorities[user_id] = int(priority)

    def user_priorities(self) -> Dict[str, int]:
        with self._lock:
            return dict(self._user_priorities)

    def add_keyword_pattern(self, priority: int, pattern: str) -> None:
        """``AddKeywordPattern`` (`:176-184`): raises ``re.error`` on a bad regex."""
        compiled = oracle.compile_pattern(pattern)
        with self._lock:
            self._patterns.setdefault(int(priority), []).append(compiled)
            self._pattern_version += 1

    def remove_keyword_pattern(self, priority: int, pattern: str) -> bool:
        with self._lock:
            pats = self._patterns.get(int(priority), [])
            for i, p in enumerate(pats):
                if p.source == pattern:
                    del pats[i]
                    self._pattern_version += 1
                    return True
        return False

    def set_default_priority(self, priority: int) -> None:
        with self._lock:
            self.default_priority = int(priority)

    def get_keyword_patterns(self, priority: int) -> List[str]:
        with self._lock:
            return [p.source for p in self._patterns.get(int(priority), [])]

    def all_patterns(self) -> Dict[int, List[str]]:
        with self._lock:
            return {k: [p.source for p in v] for k, v in sorted(self._patterns.items())}

    def patterns_snapshot(self):
        with self._lock:
            return {k: list(v) for k, v in self._patterns.items()}, self._pattern_version

    def export_state(self) -> Dict[str, Any]:
        """The admin-settable state (keyword rules, per-user defaults, default
        priority) as plain data: what a multi-rank job copies from the rank
        that serves the admin API to every other rank (``load_state``)."""
        with self._lock:
            return {"patterns": [[int(k), [p.source for p in v]] for k, v in sorted(self._patterns.items())],
                    "user_priorities": dict(self._user_priorities),
                    "default_priority": int(self.default_priority)}

    def load_state(self, state: Dict[str, Any]) -> None:
        """Replace the admin-settable state with ``export_state()``'s output
        (all patterns compiled before anything changes: a bad pattern raises
        and leaves the current state in place)."""
        pats = {int(k): [oracle.compile_pattern(s) for s in srcs] for k, srcs in state["patterns"]}
        users = {str(u): int(p) for u, p in state["user_priorities"].items()}
        with self._lock:
            self._patterns = pats
            self._user_priorities = users
            self.default_priority = int(state["default_priority"])
            self._pattern_version += 1

    # ------------------------------------------------------------------ single message (CPU)
    def _resolve_priority_head(self, msg: Message) -> Optional[bool]:
        """Steps 1-3 of ProcessMessage that need no content analysis.
        Returns None if the message must be returned unchanged, True if the
        priority still needs content analysis, False if it was decided."""
        if msg.metadata is None:
            msg.metadata = {}
        if msg.priority != PRIORITY_NORMAL and msg.priority != 0:
            return None
        up = msg.metadata.get("user_priority")
        if isinstance(up, str):
            p = level_priority_from_name(up)
            if p is not None:
                msg.priority = p
                msg.metadata["priority_reason"] = "user_override"
            return False
        with self._lock:
            udef = self._user_priorities.get(msg.user_id)
        if udef is not None:
            msg.priority = udef
            msg.metadata["priority_reason"] = "user_default"
            return False
        return True

    def _head_fast(self, msg: Message, udefs) -> Optional[bool]:
        """``_resolve_priority_head`` against a per-batch snapshot of the user
        defaults (one lock per batch, not per message)."""
        md = msg.metadata
        if md is None:
            md = msg.metadata = {}
        if msg.priority != PRIORITY_NORMAL and msg.priority != 0:
            return None
        up = md.get("user_priority")
        if isinstance(up, str):
            p = level_priority_from_name(up)
            if p is not None:
                msg.priority = p
                md["priority_reason"] = "user_override"
            return False
        if udefs:
            udef = udefs.get(msg.user_id)
            if udef is not None:
                msg.priority = udef
                md["priority_reason"] = "user_default"
                return False
        return True

    def _finish(self, msg: Message, now_ns: int) -> None:
        msg.metadata["analyzed"] = True
        if not msg.queue_name:
            msg.queue_name = priority_name(msg.priority)
        if not msg.created_at:
            msg.created_at = now_ns
        msg.updated_at = now_ns

    def _analyze_priority_cpu(self, msg: Message) -> int:
        content = msg.content
        if content == "":
            ps = msg.metadata.get("priority")
            if isinstance(ps, str):
                p = level_priority_from_name(ps)
                if p is not None:
                    return p
            return self.default_priority
        pats, _ = self.patterns_snapshot()
        return oracle.pick_priority(oracle.keyword_scores(content, pats), self.default_priority)

    @staticmethod
    def _content_metadata(msg: Message, word_count: int, sentiment: str, question: bool) -> None:
        if msg.content == "":
            return
        msg.metadata["word_count"] = word_count
        msg.metadata["sentiment"] = sentiment
        msg.metadata["contains_question"] = "true" if question else "false"

    def process_message(self, msg: Message) -> Message:
        """``ProcessMessage`` (`preprocessor.go:56-114`) on the CPU oracle."""
        head = self._resolve_priority_head(msg)
        if head is None:
            return msg
        if head:
            original = msg.priority
            msg.priority = self._analyze_priority_cpu(msg)
            if msg.priority != original:
                msg.metadata["priority_reason"] = "content_keywords"
        if msg.content:
            wc, sent, q = oracle.content_analysis(msg.content)
            self._content_metadata(msg, wc, sent, q)
        self._finish(msg, time.time_ns())
        self.stats["cpu_messages"] += 1
        return msg

    def analyze_message_content(self, content: str) -> Dict[str, Any]:
        """``AnalyzeMessageContent`` (`:253-298`)."""
        wc, sent, q = oracle.content_analysis(content)
        return {"word_count": wc, "sentiment": sent, "is_question": q}

    @staticmethod
    def analysis_json(word_count: int, sentiment: str, is_question: bool) -> str:
        """``json.Marshal`` of AnalyzeMessageContent's map (keys sorted, as Go
        emits a map)."""
        return json.dumps({"is_question": bool(is_question), "sentiment": sentiment, "word_count": int(word_count)},
                          separators=(",", ":"))

    # ------------------------------------------------------------------ batch (GPU)
    def gpu_pipeline(self):
        """The HIP text pipeline, built on first use.  Raises if the HIP
        extension is missing on a GPU host (never a silent fallback)."""
        if self._gpu is None:
            from ..ops.text import TextPipeline
            self._gpu = TextPipeline(self.cfg, device=self._device)
        return self._gpu

    def cpu_pipeline(self):
        """The native CPU twin of the text kernel, or None (disabled by
        ``preprocessor.native_cpu`` or the module cannot be built/loaded --
        then the per-message oracle runs, with a warning once)."""
        if self._cpu is None:
            self._cpu = False
            if getattr(self.cfg, "native_cpu", True):
                try:
                    from ..ops.text import CpuTextPipeline
                    self._cpu = CpuTextPipeline(self.cfg)
                except Exception as e:              # no compiler / module on this host
                    import logging
                    logging.getLogger("preprocessor").warning("native CPU preprocess unavailable (%s); "
                                                              "using the Python oracle", e)
        return self._cpu or None

    def gpu_enabled(self) -> bool:
        if not self._want_gpu:
            return False
        try:
            import torch
            return torch.cuda.is_available()
        except Exception:
            return False

    def process_batch(self, msgs: Sequence[Message], use_gpu: Optional[bool] = None,
                      classify: Optional[bool] = None, prompt_cap: int = 0) -> Sequence[Message]:
        """Process a micro-batch.  Same results as ``process_message`` per
        message; on the GPU path one fused launch covers the whole batch."""
        use_gpu = self.gpu_enabled() if use_gpu is None else use_gpu
        if not use_gpu and msgs and self.cpu_pipeline() is not None:
            # the C++ twin of the GPU kernel, then the same batch decisions
            return self.end_batch(self.begin_batch(msgs, classify=False, prompt_cap=prompt_cap, cpu=True))
        if not use_gpu:
            for m in msgs:
                self.process_message(m)
                if prompt_cap:
                    m.prompt_ids = oracle.token_hashes(m.content, prompt_cap)
                if self.record_analysis:
                    a = self.analyze_message_content(m.content)
                    m.metadata["analysis"] = self.analysis_json(a["word_count"], a["sentiment"], a["is_question"])
            return msgs
        # Per-message Python is the ingest ceiling at tens of thousands of
        # requests/s, so everything the kernels return is decided for the
        # whole batch in numpy first (keyword priority argmax with the
        # oracle's tie-break, sentiment, question, fallback flags); the loop
        # below only stores the decided values.
        return self.end_batch(self.begin_batch(msgs, classify=classify, prompt_cap=prompt_cap))

    # ------------------------------------------------------------------ asynchronous batch (GPU)
    def begin_batch(self, msgs: Sequence[Message], classify: Optional[bool] = None, prompt_cap: int = 0,
                    cpu: bool = False):
        """Launch a micro-batch's GPU preprocess and return at once (the
        host does not wait for the kernels, which queue behind the backend's
        forward for CUs); ``end_batch`` applies the results.  One batch may be
        outstanding per preprocessor."""
        with self._lock:
            udefs = dict(self._user_priorities) if self._user_priorities else None
        heads = [self._head_fast(m, udefs) for m in msgs]
        # every message with content goes through the kernels: explicit-
        # priority messages are returned unanalysed (ProcessMessage's early
        # return) but the backend still needs their prompt token ids
        work = [i for i in range(len(msgs)) if msgs[i].content] if prompt_cap else \
            [i for i, h in enumerate(heads) if h is not None and msgs[i].content]
        pend = pipe = None
        if work:
            pipe = self.cpu_pipeline() if cpu else self.gpu_pipeline()
            pats, ver = self.patterns_snapshot()
            pend = pipe.launch([msgs[i].content for i in work], pats, ver,
                               classify=False if cpu else (self.cfg.classifier if classify is None else classify),
                               prompt_cap=prompt_cap)
        return {"msgs": msgs, "heads": heads, "work": work, "pend": pend, "prompt_cap": prompt_cap, "pipe": pipe,
                "cpu": cpu}

    def batch_ready(self, tok) -> bool:
        return tok["pend"] is None or tok["pipe"].ready(tok["pend"])

    def end_batch(self, tok) -> Sequence[Message]:
        msgs, heads, work, prompt_cap = tok["msgs"], tok["heads"], tok["work"], tok["prompt_cap"]
        now = time.time_ns()
        if work:
            res = tok["pipe"].collect(tok["pend"])
            if tok.get("cpu"):
                self.stats["cpu_native_batches"] = self.stats.get("cpu_native_batches", 0) + 1
                self.stats["cpu_native_messages"] = self.stats.get("cpu_native_messages", 0) + len(work)
            else:
                self.stats["gpu_batches"] += 1
                self.stats["gpu_messages"] += len(work)
                self.stats["last_gpu_ms"] = res.elapsed_ms
                self.stats["gpu_ms_total"] = self.stats.get("gpu_ms_total", 0.0) + res.elapsed_ms
            d = res.decide(self.default_priority)
            fb, kp, wc, sent, qs, ntok = d["fallback"], d["priority"], d["word_count"], d["sentiment"], \
                d["question"], d["ntok"]
            ml = res.ml_priority.tolist() if res.has_classifier else None
            use_ml = self.cfg.use_classifier_priority
            ph = res.prompt_hashes if prompt_cap else None
            for j, i in enumerate(work):
                m = msgs[i]
                if ph is not None:
                    m.prompt_ids = ph[j, :ntok[j]]
                if heads[i] is None:                 # explicit priority: tokens only
                    continue
                md = m.metadata
                if fb[j]:
                    # fold-special characters / non-literal patterns: oracle
                    self.stats["oracle_fallbacks"] += 1
                    if heads[i]:
                        original = m.priority
                        m.priority = self._analyze_priority_cpu(m)
                        if m.priority != original:
                            md["priority_reason"] = "content_keywords"
                    w, se, q = oracle.content_analysis(m.content)
                    md["word_count"] = w
                    md["sentiment"] = se
                    md["contains_question"] = "true" if q else "false"
                else:
                    if heads[i]:
                        p = kp[j]
                        if p != m.priority:
                            m.priority = p
                            md["priority_reason"] = "content_keywords"
                    md["word_count"] = wc[j]
                    md["sentiment"] = sent[j]
                    md["contains_question"] = qs[j]
                if ml is not None:
                    md["ml_priority"] = ml[j]
                    if use_ml and heads[i] and md.get("priority_reason") is None:
                        m.priority = ml[j]
                        md["priority_reason"] = "classifier"
                # _finish, inlined (analysed, queue name, timestamps)
                md["analyzed"] = True
                if not m.queue_name:
                    m.queue_name = _PNAME.get(m.priority) or priority_name(m.priority)
                if not m.created_at:
                    m.created_at = now
                m.updated_at = now
                heads[i] = None                     # finished
        if self.record_analysis:
            seen = {}
            if work:
                for j, i in enumerate(work):
                    if not fb[j]:
                        seen[i] = (wc[j], sent[j], qs[j] == "true")
            for i, m in enumerate(msgs):
                a = seen.get(i)
                if a is None:
                    w, se, q = oracle.content_analysis(m.content) if m.content else (0, "neutral", False)
                    a = (w, se, q)
                if m.metadata is None:
                    m.metadata = {}
                m.metadata["analysis"] = self.analysis_json(*a)
        # messages the kernels never saw: empty content (the oracle's
        # metadata-priority / default rule) and user-decided heads
        for i, h in enumerate(heads):
            if h is None:
                continue
            m = msgs[i]
            if h:
                original = m.priority
                m.priority = self._analyze_priority_cpu(m)
                if m.priority != original:
                    m.metadata["priority_reason"] = "content_keywords"
            self._finish(m, now)
        return msgs
