"""PersistenceStore implementations (component C15).

Reference `internal/conversation/persistence.go`:
  * ``RedisPersistenceStore``: key ``prefix+id`` -> conversation JSON with TTL,
    set ``prefix+"user:"+uid`` of ids (`:46-159`);
  * ``PostgresPersistenceStore``: ``ConversationModel{id,user_id,created_at,
    last_active_time,completed_at,state,messages(json),metadata(json)}``
    (`:162-320`).
Here: ``MemoryPersistenceStore`` (tests/dev), ``SQLitePersistenceStore``
(stdlib, same row schema as the Postgres model), ``RedisPersistenceStore`` over
our RESP client, and ``PostgresPersistenceStore`` which needs ``psycopg2``
(not in this image: constructing it raises a clear error -- parity unpinned).
"""
from __future__ import annotations

import json
import sqlite3
import threading
from typing import Dict, List, Optional

from ..models.message import Conversation, ConversationNotFound


class PersistenceStore:
    """`state_manager.go:28-33`."""

    def save_conversation(self, conv: Conversation) -> None:
        raise NotImplementedError

    def load_conversation(self, conversation_id: str) -> Conversation:
        raise NotImplementedError

    def list_user_conversations(self, user_id: str) -> List[str]:
        raise NotImplementedError

    def delete_conversation(self, conversation_id: str) -> None:
        raise NotImplementedError

    def close(self) -> None:
        pass


def _dump(conv: Conversation) -> bytes:
    d = conv.to_dict()
    if conv.summary_vec is not None:
        d["summary_vec"] = [float(x) for x in conv.summary_vec]
    return json.dumps(d).encode()


def _load(raw: bytes) -> Conversation:
    d = json.loads(raw)
    c = Conversation.from_dict(d)
    if "summary_vec" in d:
        c.summary_vec = d["summary_vec"]
    return c


class MemoryPersistenceStore(PersistenceStore):
    def __init__(self):
        self._data: Dict[str, bytes] = {}
        self._users: Dict[str, set] = {}
        self._lock = threading.Lock()
        self.saves = 0

    def save_conversation(self, conv):
        raw = _dump(conv)
        with self._lock:
            self._data[conv.id] = raw
            self._users.setdefault(conv.user_id, set()).add(conv.id)
            self.saves += 1

    def load_conversation(self, conversation_id):
        with self._lock:
            raw = self._data.get(conversation_id)
        if raw is None:
            raise ConversationNotFound(conversation_id)
        return _load(raw)

    def list_user_conversations(self, user_id):
        with self._lock:
            return sorted(self._users.get(user_id, ()))

    def delete_conversation(self, conversation_id):
        with self._lock:
            raw = self._data.pop(conversation_id, None)
            if raw is not None:
                uid = json.loads(raw).get("user_id", "")
                self._users.get(uid, set()).discard(conversation_id)


class SQLitePersistenceStore(PersistenceStore):
    """Rows of the reference's ``ConversationModel`` (`persistence.go:168-177`)."""

    def __init__(self, path: str = ":memory:"):
        self._db = sqlite3.connect(path, check_same_thread=False)
        self._lock = threading.Lock()
        with self._lock:
            self._db.execute(
                "CREATE TABLE IF NOT EXISTS conversations (id TEXT PRIMARY KEY, user_id TEXT, "
                "created_at TEXT, last_active_time TEXT, completed_at TEXT, state TEXT, "
                "messages BLOB, metadata BLOB, doc BLOB)")
            self._db.execute("CREATE INDEX IF NOT EXISTS conv_user ON conversations(user_id)")
            self._db.commit()

    def save_conversation(self, conv):
        doc = _dump(conv)
        d = json.loads(doc)
        with self._lock:
            self._db.execute(
                "INSERT OR REPLACE INTO conversations VALUES (?,?,?,?,?,?,?,?,?)",
                (conv.id, conv.user_id, d["created_at"], d["last_active_time"],
                 d["completed_at"] if conv.completed_at else None, conv.state,
                 json.dumps(d["messages"]).encode(), json.dumps(conv.metadata).encode(), doc))
            self._db.commit()

    def load_conversation(self, conversation_id):
        with self._lock:
            row = self._db.execute("SELECT doc FROM conversations WHERE id = ?", (conversation_id,)).fetchone()
        if row is None:
            raise ConversationNotFound(conversation_id)
        return _load(row[0])

    def list_user_conversations(self, user_id):
        with self._lock:
            rows = self._db.execute("SELECT id FROM conversations WHERE user_id = ? ORDER BY id",
                                    (user_id,)).fetchall()
        return [r[0] for r in rows]

    def delete_conversation(self, conversation_id):
        with self._lock:
            self._db.execute("DELETE FROM conversations WHERE id = ?", (conversation_id,))
            self._db.commit()

    def close(self):
        with self._lock:
            self._db.close()


class RedisPersistenceStore(PersistenceStore):
    """`persistence.go:24-159` over the RESP client."""

    def __init__(self, client, prefix: str = "conversation:", expiration_ns: int = 0):
        self.client = client
        self.prefix = prefix
        self.expiration_s = int(expiration_ns // 1_000_000_000)

    def save_conversation(self, conv):
        key = self.prefix + conv.id
        self.client.set(key, _dump(conv), self.expiration_s)
        ukey = self.prefix + "user:" + conv.user_id
        self.client.sadd(ukey, conv.id)
        if self.expiration_s > 0:
            self.client.expire(ukey, self.expiration_s)

    def load_conversation(self, conversation_id):
        raw = self.client.get(self.prefix + conversation_id)
        if raw is None:
            raise ConversationNotFound(conversation_id)
        return _load(raw)

    def list_user_conversations(self, user_id):
        return self.client.smembers(self.prefix + "user:" + user_id)

    def delete_conversation(self, conversation_id):
        key = self.prefix + conversation_id
        raw = self.client.get(key)
        self.client.delete(key)
        if raw is not None:
            uid = json.loads(raw).get("user_id", "")
            self.client.srem(self.prefix + "user:" + uid, conversation_id)


class PostgresPersistenceStore(PersistenceStore):
    """``PostgresPersistenceStore`` (`persistence.go:162-320`): one row per
    conversation with the reference's ``ConversationModel`` columns
    (`:168-177`), upserted on save.  Speaks the wire protocol itself
    (``pgwire.PgConnection``; no driver package in this image)."""

    def __init__(self, dsn_or_conn):
        from .pgwire import PgConnection
        self._conn = PgConnection.from_dsn(dsn_or_conn) if isinstance(dsn_or_conn, str) else dsn_or_conn
        self._conn.simple("CREATE TABLE IF NOT EXISTS conversation_models (id TEXT PRIMARY KEY, user_id TEXT, "
                          "created_at BIGINT, last_active_time BIGINT, completed_at BIGINT, state TEXT, "
                          "messages TEXT, metadata TEXT, doc TEXT);"
                          "CREATE INDEX IF NOT EXISTS conversation_models_user ON conversation_models (user_id)")

    def save_conversation(self, conv):
        doc = _dump(conv).decode()
        d = json.loads(doc)
        self._conn.execute(
            "INSERT INTO conversation_models VALUES ($1,$2,$3,$4,$5,$6,$7,$8,$9) ON CONFLICT (id) DO UPDATE "
            "SET last_active_time = excluded.last_active_time, completed_at = excluded.completed_at, "
            "state = excluded.state, messages = excluded.messages, metadata = excluded.metadata, doc = excluded.doc",
            (conv.id, conv.user_id, int(conv.created_at or 0), int(conv.last_active_time or 0),
             int(conv.completed_at) if conv.completed_at else None, conv.state,
             json.dumps(d.get("messages", [])), json.dumps(conv.metadata), doc))

    def load_conversation(self, conversation_id):
        row = self._conn.execute("SELECT doc FROM conversation_models WHERE id = $1", (conversation_id,)).fetchone()
        if row is None:
            raise ConversationNotFound(conversation_id)
        return _load(row[0].encode())

    def list_user_conversations(self, user_id):
        rows = self._conn.execute("SELECT id FROM conversation_models WHERE user_id = $1 ORDER BY id", (user_id,))
        return [r[0] for r in rows.rows]

    def delete_conversation(self, conversation_id):
        self._conn.execute("DELETE FROM conversation_models WHERE id = $1", (conversation_id,))

    def close(self):
        self._conn.close()


def postgres_dsn(cfg) -> str:
    p = cfg.database.postgres
    return f"host={p.host} port={p.port} user={p.user} password={p.password} dbname={p.dbname} sslmode={p.sslmode}"


def make_store(cfg) -> Optional[PersistenceStore]:
    """From ``Config.database`` (backend: memory|sqlite|redis|postgres|none)."""
    b = (cfg.database.backend or "memory").lower()
    if b in ("none", "off", ""):
        return None
    if b == "memory":
        return MemoryPersistenceStore()
    if b == "sqlite":
        return SQLitePersistenceStore(cfg.database.sqlite_path)
    if b == "redis":
        from .resp import RespClient
        r = cfg.database.redis
        return RedisPersistenceStore(RespClient(r.addr, r.password, r.db, pool_size=r.pool_size), "conversation:",
                                     cfg.queue.max_retention_period)
    if b == "postgres":
        return PostgresPersistenceStore(postgres_dsn(cfg))
    raise ValueError(f"unknown persistence backend {b!r}")
