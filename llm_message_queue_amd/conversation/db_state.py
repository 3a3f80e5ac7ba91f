"""DB-backed conversation state manager (component C16), unified onto SQLite.

Reference `internal/statemanager/manager.go` (used by the api-gateway and
queue-manager binaries): write-through relational store + two cache levels
(process map, then Redis ``conversation:<id>`` with 24 h TTL).  Conversation
ids are ``conv_<unixnano>`` (`:271-273`).  ``add_message`` inserts the
message, bumps ``message_count`` and appends completed contents to
``context`` (`:116-138`).

The relational store is Postgres (as in the reference, spoken over the wire
protocol by ``pgwire.PgConnection`` -- no driver package in this image) or
stdlib ``sqlite3`` for single-node deployments and tests; the statements
are written once, in the dialect both accept (``?`` placeholders converted
to ``$n`` for Postgres, ``INSERT ... ON CONFLICT (id) DO UPDATE`` upserts,
BIGINT nanosecond timestamps).  The optional Redis level is the RESP client
(``resp.RespClient``).  The reference's two Redis client majors (go-redis
v8 + v9, D25) collapse into one client.
"""
from __future__ import annotations

import json
import sqlite3
import threading
import time
from typing import Any, Dict, List, Optional

from ..models.message import Conversation, ConversationNotFound, Message, MessageStatus

_CONV_COLS = ("id", "user_id", "title", "context", "status", "state", "priority", "message_count",
              "last_activity", "last_active_time", "created_at", "updated_at", "completed_at", "metadata")


class _SQLiteDB:
    def __init__(self, path: str):
        self.db = sqlite3.connect(path, check_same_thread=False)

    def execute(self, sql: str, params=()) -> list:
        cur = self.db.execute(sql, tuple(params))
        rows = cur.fetchall()
        self.db.commit()
        return rows

    def close(self) -> None:
        self.db.close()


class _PostgresDB:
    def __init__(self, conn):
        self.conn = conn

    def execute(self, sql: str, params=()) -> list:
        from .pgwire import qmark_to_dollar
        return self.conn.execute(qmark_to_dollar(sql), tuple(params)).rows

    def close(self) -> None:
        self.conn.close()


_MSG_UPSERT = ("INSERT INTO messages VALUES (?,?,?,?,?) ON CONFLICT (id) DO UPDATE SET "
               "conversation_id = excluded.conversation_id, user_id = excluded.user_id, "
               "created_at = excluded.created_at, doc = excluded.doc")


class DBStateManager:
    def __init__(self, path: str = ":memory:", redis=None, redis_ttl_s: int = 24 * 3600, pg=None):
        """``pg``: a ``pgwire.PgConnection`` (or DSN string) -> Postgres;
        otherwise SQLite at ``path``."""
        if pg is not None:
            from .pgwire import PgConnection
            self.db = _PostgresDB(PgConnection.from_dsn(pg) if isinstance(pg, str) else pg)
        else:
            self.db = _SQLiteDB(path)
        self.redis = redis
        self.redis_ttl_s = redis_ttl_s
        self._lock = threading.RLock()
        self._cache: Dict[str, Conversation] = {}
        self._last_id = 0
        with self._lock:
            self.db.execute("CREATE TABLE IF NOT EXISTS conversations (id TEXT PRIMARY KEY, user_id TEXT, "
                            "title TEXT, context TEXT, status TEXT, state TEXT, priority BIGINT, "
                            "message_count BIGINT, last_activity BIGINT, last_active_time BIGINT, "
                            "created_at BIGINT, updated_at BIGINT, completed_at BIGINT, metadata TEXT)")
            self.db.execute("CREATE TABLE IF NOT EXISTS messages (id TEXT PRIMARY KEY, conversation_id TEXT, "
                            "user_id TEXT, created_at BIGINT, doc TEXT)")
            self.db.execute("CREATE INDEX IF NOT EXISTS msg_conv ON messages(conversation_id)")
            self.db.execute("CREATE INDEX IF NOT EXISTS conv_user ON conversations(user_id)")

    @classmethod
    def from_config(cls, cfg, redis=None) -> "DBStateManager":
        """``database.backend``: postgres -> the configured server; else SQLite."""
        if (cfg.database.backend or "").lower() == "postgres":
            from .persistence import postgres_dsn
            return cls(pg=postgres_dsn(cfg), redis=redis)
        return cls(cfg.database.sqlite_path, redis=redis)

    # ------------------------------------------------------------------ helpers
    def _gen_id(self) -> str:
        with self._lock:
            t = max(time.time_ns(), self._last_id + 1)
            self._last_id = t
        return f"conv_{t}"

    @staticmethod
    def _row_to_conv(row) -> Conversation:
        d = dict(zip(_CONV_COLS, row))
        c = Conversation(d["id"], d["user_id"] or "", created_at=d["created_at"] or 0,
                         state=d["state"] or "", metadata=json.loads(d["metadata"] or "{}"))
        c.title, c.context, c.status = d["title"] or "", d["context"] or "", d["status"] or ""
        c.priority, c.message_count = int(d["priority"] or 0), int(d["message_count"] or 0)
        c.last_activity, c.last_active_time = d["last_activity"] or 0, d["last_active_time"] or 0
        c.updated_at, c.completed_at = d["updated_at"] or 0, d["completed_at"] or 0
        return c

    def _redis_key(self, cid: str) -> str:
        return f"conversation:{cid}"

    def _cache_put(self, conv: Conversation) -> None:
        with self._lock:
            self._cache[conv.id] = conv
        if self.redis is not None:
            try:
                self.redis.set(self._redis_key(conv.id), json.dumps(conv.to_dict(False)).encode(), self.redis_ttl_s)
            except Exception:
                pass

    def _invalidate(self, cid: str) -> None:
        with self._lock:
            self._cache.pop(cid, None)
        if self.redis is not None:
            try:
                self.redis.delete(self._redis_key(cid))
            except Exception:
                pass

    # ------------------------------------------------------------------ API
    def create_conversation(self, user_id: str, title: str = "", priority: int = 0) -> Conversation:
        now = time.time_ns()
        conv = Conversation(self._gen_id(), user_id, created_at=now, state="")
        conv.title, conv.status, conv.priority = title, "active", int(priority)
        conv.last_activity = conv.updated_at = now
        with self._lock:
            self.db.execute(f"INSERT INTO conversations VALUES ({','.join('?' * len(_CONV_COLS))})",
                            (conv.id, user_id, title, "", "active", "", int(priority), 0, now, now, now, now, 0,
                             "{}"))
        self._cache_put(conv)
        return conv

    def get_conversation(self, conversation_id: str) -> Conversation:
        with self._lock:
            c = self._cache.get(conversation_id)
        if c is not None:
            return c
        if self.redis is not None:
            try:
                raw = self.redis.get(self._redis_key(conversation_id))
            except Exception:
                raw = None
            if raw:
                c = Conversation.from_dict(json.loads(raw))
                with self._lock:
                    self._cache[c.id] = c
                return c
        with self._lock:
            rows = self.db.execute(f"SELECT {','.join(_CONV_COLS)} FROM conversations WHERE id = ?",
                                   (conversation_id,))
        row = rows[0] if rows else None
        if row is None:
            raise ConversationNotFound(conversation_id)
        c = self._row_to_conv(row)
        self._cache_put(c)
        return c

    def update_conversation(self, conversation_id: str, updates: Dict[str, Any]) -> None:
        cols = [k for k in updates if k in _CONV_COLS and k != "id"]
        if cols:
            vals = [json.dumps(updates[k]) if k == "metadata" else updates[k] for k in cols]
            with self._lock:
                self.db.execute(f"UPDATE conversations SET {', '.join(c + ' = ?' for c in cols)} WHERE id = ?",
                                (*vals, conversation_id))
        self._invalidate(conversation_id)

    def add_message(self, conversation_id: str, message: Message) -> None:
        conv = self.get_conversation(conversation_id)
        message.conversation_id = conversation_id
        with self._lock:
            self.db.execute(_MSG_UPSERT,
                            (message.id, conversation_id, message.user_id, message.created_at or time.time_ns(),
                             json.dumps(message.to_dict())))
        now = time.time_ns()
        upd = {"message_count": conv.message_count + 1, "last_activity": now, "updated_at": now}
        if message.status == MessageStatus.COMPLETED:
            upd["context"] = conv.context + "\n" + message.content
        self.update_conversation(conversation_id, upd)

    def get_conversation_messages(self, conversation_id: str, limit: int = 100) -> List[Message]:
        with self._lock:
            rows = self.db.execute("SELECT doc FROM messages WHERE conversation_id = ? ORDER BY created_at DESC "
                                   "LIMIT ?", (conversation_id, int(limit)))
        return [Message.from_dict(json.loads(r[0])) for r in rows]

    def get_user_conversations(self, user_id: str, limit: int = 100) -> List[Conversation]:
        with self._lock:
            rows = self.db.execute(f"SELECT {','.join(_CONV_COLS)} FROM conversations WHERE user_id = ? "
                                   "ORDER BY last_activity DESC LIMIT ?", (user_id, int(limit)))
        return [self._row_to_conv(r) for r in rows]

    def archive_conversation(self, conversation_id: str) -> None:
        self.update_conversation(conversation_id, {"status": "archived", "updated_at": time.time_ns()})

    def delete_conversation(self, conversation_id: str) -> None:
        with self._lock:
            self.db.execute("DELETE FROM conversations WHERE id = ?", (conversation_id,))
        self._invalidate(conversation_id)

    def get_active_conversations(self, limit: int = 100) -> List[Conversation]:
        with self._lock:
            rows = self.db.execute(f"SELECT {','.join(_CONV_COLS)} FROM conversations WHERE status = 'active' "
                                   "ORDER BY last_activity DESC LIMIT ?", (int(limit),))
        return [self._row_to_conv(r) for r in rows]

    def update_conversation_priority(self, conversation_id: str, priority: int) -> None:
        self.update_conversation(conversation_id, {"priority": int(priority), "updated_at": time.time_ns()})

    def get_conversation_context(self, conversation_id: str) -> str:
        return self.get_conversation(conversation_id).context

    def update_message(self, message: Message) -> None:
        with self._lock:
            self.db.execute(_MSG_UPSERT,
                            (message.id, message.conversation_id, message.user_id,
                             message.created_at or time.time_ns(), json.dumps(message.to_dict())))

    def get_message(self, message_id: str) -> Optional[Message]:
        with self._lock:
            rows = self.db.execute("SELECT doc FROM messages WHERE id = ?", (message_id,))
        return Message.from_dict(json.loads(rows[0][0])) if rows else None

    def close(self) -> None:
        with self._lock:
            self.db.close()
