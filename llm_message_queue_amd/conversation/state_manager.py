"""Conversation StateManager (component C14).

Reference `internal/conversation/state_manager.go`:
  * ``get_conversation(id, user)`` is get-or-create (`:72-114`);
  * ``add_message`` appends, keeps the last ``max_context_length`` messages
    (`:117-147`) and persists;
  * per-user overflow beyond ``max_conversations`` archives the oldest
    (`:310-351`); cleanup removes TTL-expired, idle and long-completed
    conversations (`:354-403`); ``get_stats`` (`:406-422`).

Changes:
  * D20: persistence is write-behind -- a writer thread snapshots dirty
    conversations outside the manager lock (coalescing repeated updates);
  * D19: ``find_conversation`` (no create) backs ``GET /conversations/:id``
    so unknown ids are a 404; POST paths keep get-or-create;
  * the reference's race on ``LastActiveTime`` after RUnlock is gone;
  * N5: messages evicted by the context window are not dropped -- they are
    queued for the summarise-on-evict engine (GPU kernels) which folds them
    into ``conversation.summary_vec`` + ``summary_tokens``;
  * KV-residency hint: ``home_gpu`` records which backend holds the
    conversation's KV so the dispatcher can route it stickily.
"""
from __future__ import annotations

import threading
import time
import uuid
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from ..models.message import Conversation, ConversationNotFound, ConversationState, Message
from ..utils.logging import get_logger

DAY_NS = 24 * 3600 * 1_000_000_000


def message_tokens(m: Message) -> int:
    """Tokens a message adds to a context window: the preprocessor's
    ``word_count`` (GPU tokenizer, Go ``strings.Fields`` semantics) when it
    ran, else a whitespace split."""
    wc = m.metadata.get("word_count") if m.metadata else None
    if wc is not None:
        try:
            return int(wc)
        except (TypeError, ValueError):
            pass
    return len(m.content.split())


class StateManager:
    def __init__(self, *, conversation_ttl: int = DAY_NS, cleanup_interval: int = 60 * 1_000_000_000,
                 max_conversations: int = 1000, max_context_length: int = 4096,
                 max_idle_time: int = 30 * 60 * 1_000_000_000, persistence=None,
                 async_persistence: bool = True, summary_engine=None, summarise_on_evict: bool = True,
                 logger=None, max_context_tokens: int = 0):
        self.conversation_ttl = conversation_ttl
        self.cleanup_interval = cleanup_interval
        self.max_conversations = max_conversations
        self.max_context_length = max_context_length
        # token-aware window (SURVEY.md §5 long-context plan): besides the
        # reference's message-count cap, keep the window's token total (the
        # preprocessor's word_count, i.e. the GPU tokenizer's count) under
        # this budget by evicting the oldest messages (summarised, N5).  0 = off
        self.max_context_tokens = int(max_context_tokens)
        self._ctx_tokens: Dict[str, int] = {}
        self.max_idle_time = max_idle_time
        self.persistence = persistence
        self.async_persistence = async_persistence and persistence is not None
        self.summary_engine = summary_engine
        self.summarise_on_evict = summarise_on_evict
        self.logger = logger or get_logger("state_manager")
        self._convs: Dict[str, Conversation] = {}
        self._users: Dict[str, List[str]] = {}
        self._lock = threading.RLock()
        self._dirty: Dict[str, None] = {}
        self._dirty_cv = threading.Condition()
        self._evicted: Dict[str, List[str]] = {}   # conv id -> evicted contents awaiting summary
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self.persist_errors = 0

    @classmethod
    def from_config(cls, cfg, persistence=None, summary_engine=None, **kw) -> "StateManager":
        c = cfg.conversation
        return cls(conversation_ttl=cfg.queue.max_retention_period, cleanup_interval=cfg.queue.cleanup_interval,
                   max_conversations=c.max_conversations, max_context_length=c.max_context_length,
                   max_idle_time=c.max_idle_time, persistence=persistence, summary_engine=summary_engine,
                   summarise_on_evict=c.summarise_on_evict,
                   max_context_tokens=getattr(c, "max_context_tokens", 0), **kw)

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        if self._threads:
            return
        self._stop.clear()
        if self.cleanup_interval > 0:
            t = threading.Thread(target=self._cleanup_loop, name="conv-cleanup", daemon=True)
            t.start()
            self._threads.append(t)
        if self.async_persistence:
            t = threading.Thread(target=self._writer_loop, name="conv-writer", daemon=True)
            t.start()
            self._threads.append(t)

    def stop(self) -> None:
        self._stop.set()
        with self._dirty_cv:
            self._dirty_cv.notify_all()
        for t in self._threads:
            t.join(timeout=5)
        self._threads = []
        self.flush()

    # ------------------------------------------------------------------ persistence
    def _persist(self, conv: Conversation) -> None:
        if self.persistence is None:
            return
        if self.async_persistence and self._threads:
            with self._dirty_cv:
                self._dirty[conv.id] = None
                self._dirty_cv.notify()
            return
        self._save(conv)

    def _save(self, conv: Conversation) -> None:
        try:
            self.persistence.save_conversation(conv)
        except Exception as e:
            self.persist_errors += 1
            self.logger.error("Failed to persist conversation", conversation_id=conv.id, error=str(e))

    def _snapshot(self, cid: str) -> Optional[Conversation]:
        with self._lock:
            c = self._convs.get(cid)
            if c is None:
                return None
            d = c.to_dict()
            snap = Conversation.from_dict(d)
            snap.summary_vec = None if c.summary_vec is None else list(map(float, c.summary_vec))
            return snap

    def flush(self) -> int:
        """Write every dirty conversation now (writer thread or shutdown)."""
        with self._dirty_cv:
            ids, self._dirty = list(self._dirty), {}
        n = 0
        for cid in ids:
            snap = self._snapshot(cid)
            if snap is not None:
                self._save(snap)
                n += 1
        return n

    def _writer_loop(self) -> None:
        while not self._stop.is_set():
            with self._dirty_cv:
                if not self._dirty:
                    self._dirty_cv.wait(0.05)
            self.flush()

    # ------------------------------------------------------------------ CRUD
    def create_conversation(self, user_id: str, metadata: Optional[Dict[str, Any]] = None,
                            conversation_id: Optional[str] = None) -> Conversation:
        cid = conversation_id or str(uuid.uuid4())
        conv = Conversation(cid, user_id, metadata=dict(metadata or {}))
        with self._lock:
            self._convs[cid] = conv
            self._add_to_active_users(user_id, cid)
        self._persist(conv)
        return conv

    def get_conversation(self, conversation_id: str, user_id: str = "") -> Conversation:
        """Get-or-create (reference semantics)."""
        with self._lock:
            conv = self._convs.get(conversation_id)
            if conv is not None:
                conv.last_active_time = time.time_ns()
                return conv
        if self.persistence is not None:
            try:
                loaded = self.persistence.load_conversation(conversation_id)
            except Exception:
                loaded = None
            if loaded is not None:
                with self._lock:
                    self._convs.setdefault(conversation_id, loaded)
                    self._add_to_active_users(user_id or loaded.user_id, conversation_id)
                    return self._convs[conversation_id]
        conv = Conversation(conversation_id, user_id)
        with self._lock:
            existing = self._convs.setdefault(conversation_id, conv)
            if existing is conv:
                self._add_to_active_users(user_id, conversation_id)
        return existing

    def find_conversation(self, conversation_id: str) -> Optional[Conversation]:
        """Lookup without creating (memory, then persistence)."""
        with self._lock:
            conv = self._convs.get(conversation_id)
        if conv is not None:
            return conv
        if self.persistence is not None:
            try:
                loaded = self.persistence.load_conversation(conversation_id)
            except Exception:
                return None
            with self._lock:
                self._convs.setdefault(conversation_id, loaded)
                self._add_to_active_users(loaded.user_id, conversation_id)
                return self._convs[conversation_id]
        return None

    def add_message(self, conversation_id: str, message: Message) -> None:
        with self._lock:
            conv = self._convs.get(conversation_id)
            if conv is None:
                raise ConversationNotFound(conversation_id)
            conv.messages.append(message)
            conv.message_count += 1
            now = time.time_ns()
            conv.last_active_time = now
            conv.last_activity = now
            conv.updated_at = now
            excess = 0
            if self.max_context_length > 0 and len(conv.messages) > self.max_context_length:
                excess = len(conv.messages) - self.max_context_length
            if self.max_context_tokens > 0:
                # running total, cached per conversation OBJECT (a conversation
                # dropped by cleanup and re-created under the same id recounts)
                cached = self._ctx_tokens.get(conversation_id)
                tot = cached[1] if cached is not None and cached[0] is conv else None
                if tot is None:
                    tot = sum(message_tokens(m) for m in conv.messages[:-1])
                tot += message_tokens(message)
                tot -= sum(message_tokens(m) for m in conv.messages[:excess])
                # evict oldest while over budget (the newest message always stays)
                while tot > self.max_context_tokens and excess < len(conv.messages) - 1:
                    tot -= message_tokens(conv.messages[excess])
                    excess += 1
                self._ctx_tokens[conversation_id] = (conv, tot)
            if excess:
                evicted = conv.messages[:excess]
                conv.messages = conv.messages[excess:]
                if self.summarise_on_evict:
                    self._evicted.setdefault(conversation_id, []).extend(m.content for m in evicted)
        self._persist(conv)

    def context_tokens(self, conversation_id: str) -> int:
        """Token total of the conversation's current window."""
        with self._lock:
            conv = self._convs.get(conversation_id)
            if conv is None:
                raise ConversationNotFound(conversation_id)
            return sum(message_tokens(m) for m in conv.messages)

    def update_conversation_state(self, conversation_id: str, state: str) -> None:
        with self._lock:
            conv = self._convs.get(conversation_id)
            if conv is None:
                raise ConversationNotFound(conversation_id)
            conv.state = state
            conv.updated_at = time.time_ns()
            if state in (ConversationState.COMPLETED, ConversationState.ARCHIVED):
                conv.completed_at = time.time_ns()
        self._persist(conv)

    def all_conversations(self) -> List[Conversation]:
        """Snapshot of every in-memory conversation (``GET /conversations``
        without a user filter)."""
        with self._lock:
            return list(self._convs.values())

    def get_user_conversations(self, user_id: str) -> List[Conversation]:
        with self._lock:
            ids = list(self._users.get(user_id, []))
        if not ids and self.persistence is not None:
            ids = self.persistence.list_user_conversations(user_id)
        out = []
        for cid in ids:
            conv = self.find_conversation(cid)
            if conv is not None:
                out.append(conv)
        return out

    def delete_conversation(self, conversation_id: str) -> None:
        with self._lock:
            conv = self._convs.pop(conversation_id, None)
            if conv is None:
                raise ConversationNotFound(conversation_id)
            ids = self._users.get(conv.user_id)
            if ids is not None:
                self._users[conv.user_id] = [i for i in ids if i != conversation_id]
            self._evicted.pop(conversation_id, None)
            self._ctx_tokens.pop(conversation_id, None)
        with self._dirty_cv:
            self._dirty.pop(conversation_id, None)
        if self.persistence is not None:
            self.persistence.delete_conversation(conversation_id)

    def update_conversation_metadata(self, conversation_id: str, metadata: Dict[str, Any]) -> None:
        with self._lock:
            conv = self._convs.get(conversation_id)
            if conv is None:
                raise ConversationNotFound(conversation_id)
            conv.metadata.update(metadata or {})
            conv.updated_at = time.time_ns()
        self._persist(conv)

    def get_conversation_context(self, conversation_id: str, limit: int = 0) -> List[Message]:
        with self._lock:
            conv = self._convs.get(conversation_id)
            if conv is None:
                raise ConversationNotFound(conversation_id)
            msgs = list(conv.messages)
        if 0 < limit < len(msgs):
            return msgs[-limit:]
        return msgs

    def set_home_gpu(self, conversation_id: str, gpu: int) -> None:
        with self._lock:
            conv = self._convs.get(conversation_id)
            if conv is not None:
                conv.home_gpu = int(gpu)

    def home_gpu(self, conversation_id: str) -> int:
        with self._lock:
            conv = self._convs.get(conversation_id)
            return -1 if conv is None else conv.home_gpu

    def summary_tokens(self, conversation_id: str) -> List[int]:
        """The N5 salient tokens of the conversation's evicted window (empty
        while nothing was evicted): the gateway prepends them to a
        non-resident replay as the dialog's compressed context."""
        with self._lock:
            conv = self._convs.get(conversation_id)
            return [] if conv is None else list(conv.summary_tokens)

    # ------------------------------------------------------------------ user caps
    def _add_to_active_users(self, user_id: str, conversation_id: str) -> None:
        ids = self._users.setdefault(user_id, [])
        if conversation_id in ids:
            return
        ids.append(conversation_id)
        if self.max_conversations > 0 and len(ids) > self.max_conversations:
            excess = len(ids) - self.max_conversations
            oldest, self._users[user_id] = ids[:excess], ids[excess:]
            for oid in oldest:
                old = self._convs.get(oid)
                if old is not None:
                    old.state = ConversationState.ARCHIVED
                    old.completed_at = time.time_ns()
                    self._persist(old)

    # ------------------------------------------------------------------ N5
    def pending_evictions(self) -> int:
        with self._lock:
            return sum(len(v) for v in self._evicted.values())

    def summarise_pending(self, max_conversations: int = 4096) -> int:
        """Fold evicted messages into each conversation's summary (one batched
        GPU launch chain for all pending conversations)."""
        if self.summary_engine is None:
            return 0
        with self._lock:
            items: List[Tuple[str, List[str]]] = []
            for cid in list(self._evicted)[:max_conversations]:
                items.append((cid, self._evicted.pop(cid)))
            groups = []
            for cid, contents in items:
                conv = self._convs.get(cid)
                prev = None if conv is None or conv.summary_vec is None else np.asarray(conv.summary_vec)
                groups.append((prev, contents))
        if not items:
            return 0
        results = self.summary_engine.summarise(groups)
        with self._lock:
            for (cid, contents), (vec, sal) in zip(items, results):
                conv = self._convs.get(cid)
                if conv is None:
                    continue
                conv.summary_vec = vec
                # newest salient tokens first, then older ones still fitting in k
                k = getattr(self.summary_engine, "k", 8)
                fresh = [h for h, _ in sal]
                conv.summary_tokens = (fresh + [h for h in conv.summary_tokens if h not in fresh])[:k]
                conv.evicted_count += len(contents)
        for cid, _ in items:
            conv = self._convs.get(cid)
            if conv is not None:
                self._persist(conv)
        return len(items)

    # ------------------------------------------------------------------ cleanup / stats
    def cleanup_expired_conversations(self, now_ns: Optional[int] = None) -> int:
        now = time.time_ns() if now_ns is None else now_ns
        expired = []
        with self._lock:
            for cid, conv in self._convs.items():
                if self.conversation_ttl > 0 and now - conv.created_at > self.conversation_ttl:
                    expired.append(cid)
                elif self.max_idle_time > 0 and now - conv.last_active_time > self.max_idle_time:
                    expired.append(cid)
                elif conv.state in (ConversationState.COMPLETED, ConversationState.ARCHIVED) and \
                        conv.completed_at and conv.completed_at + DAY_NS < now:
                    expired.append(cid)
        for cid in expired:
            try:
                self.delete_conversation(cid)
            except ConversationNotFound:
                pass
        return len(expired)

    def _cleanup_loop(self) -> None:
        while not self._stop.wait(self.cleanup_interval / 1e9):
            self.cleanup_expired_conversations()
            try:
                self.summarise_pending()
            except Exception as e:
                self.logger.error("summarise failed", error=str(e))

    def get_stats(self) -> Dict[str, Any]:
        with self._lock:
            states: Dict[str, int] = {}
            for c in self._convs.values():
                states[c.state] = states.get(c.state, 0) + 1
            return {"total_conversations": len(self._convs), "total_users": len(self._users),
                    "conversation_states": states,
                    "pending_evictions": sum(len(v) for v in self._evicted.values())}
