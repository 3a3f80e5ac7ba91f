"""Minimal Redis RESP2 client (the ``redis`` Python package is not available
in this image).  Implements the commands the reference's persistence uses:
SET (with EX), GET, DEL, SADD, SREM, SMEMBERS, EXPIRE, PING, plus an
in-process ``MiniRedis`` server speaking the same protocol for tests.
Reference call sites: `internal/conversation/persistence.go:59-156`,
`internal/statemanager/manager.go:229-269`.
"""
from __future__ import annotations

import socket
import socketserver
import threading
import time
from typing import Dict, List, Optional, Set, Union

Reply = Union[None, int, bytes, str, list, Exception]


class RedisError(Exception):
    pass


def _encode(args) -> bytes:
    out = [b"*%d\r\n" % len(args)]
    for a in args:
        b = a if isinstance(a, (bytes, bytearray)) else str(a).encode()
        out.append(b"$%d\r\n%s\r\n" % (len(b), b))
    return b"".join(out)


class _Reader:
    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.buf = b""

    def _fill(self):
        chunk = self.sock.recv(65536)
        if not chunk:
            raise ConnectionError("redis connection closed")
        self.buf += chunk

    def line(self) -> bytes:
        while b"\r\n" not in self.buf:
            self._fill()
        ln, self.buf = self.buf.split(b"\r\n", 1)
        return ln

    def exact(self, n: int) -> bytes:
        while len(self.buf) < n + 2:
            self._fill()
        data, self.buf = self.buf[:n], self.buf[n + 2:]
        return data

    def reply(self) -> Reply:
        ln = self.line()
        t, rest = ln[:1], ln[1:]
        if t == b"+":
            return rest.decode()
        if t == b"-":
            return RedisError(rest.decode())
        if t == b":":
            return int(rest)
        if t == b"$":
            n = int(rest)
            return None if n < 0 else self.exact(n)
        if t == b"*":
            n = int(rest)
            return None if n < 0 else [self.reply() for _ in range(n)]
        raise RedisError(f"bad RESP type {t!r}")


class _Conn:
    """One RESP connection of a ``RespClient`` pool (connected lazily)."""

    def __init__(self, owner: "RespClient"):
        self.o = owner
        self.sock: Optional[socket.socket] = None
        self.reader: Optional[_Reader] = None

    def connect(self):
        o = self.o
        s = socket.create_connection((o.host, o.port), timeout=o.timeout)
        self.sock, self.reader = s, _Reader(s)
        if o.password:
            self.call_once("AUTH", o.password)
        if o.db:
            self.call_once("SELECT", o.db)

    def call_once(self, *args) -> Reply:
        self.sock.sendall(_encode(args))
        r = self.reader.reply()
        if isinstance(r, RedisError):
            raise r
        return r

    def close(self):
        if self.sock is not None:
            try:
                self.sock.close()
            except OSError:
                pass
        self.sock = self.reader = None


class RespClient:
    """Thread-safe RESP client over a pool of up to ``pool_size`` connections
    (``database.redis.pool_size``, the go-redis pool option the reference
    sets): each call borrows one, so concurrent callers -- the state
    manager's write-behind thread, API readers -- do not queue behind one
    socket.  Connections open on first use; the most recently returned is
    reused first, so the pool only grows to the concurrency it sees."""

    def __init__(self, addr: str = "localhost:6379", password: str = "", db: int = 0, timeout: float = 5.0,
                 pool_size: int = 1):
        import queue
        host, _, port = addr.rpartition(":")
        self.host, self.port = host or "localhost", int(port or 6379)
        self.password, self.db, self.timeout = password, db, timeout
        self.pool_size = max(1, int(pool_size))
        self._conns = [_Conn(self) for _ in range(self.pool_size)]
        self._free: "queue.LifoQueue[_Conn]" = queue.LifoQueue()
        for c in reversed(self._conns):
            self._free.put(c)

    def call(self, *args) -> Reply:
        c = self._free.get()
        try:
            for attempt in (0, 1):
                try:
                    if c.sock is None:
                        c.connect()
                    return c.call_once(*args)
                except (ConnectionError, OSError):
                    c.close()
                    if attempt:
                        raise
        finally:
            self._free.put(c)

    def connections(self) -> int:
        """Pool connections currently open."""
        return sum(c.sock is not None for c in self._conns)

    def close(self):
        """Close every idle connection (a busy one closes when its call
        returns it and the next call reconnects)."""
        held = []
        while True:
            try:
                held.append(self._free.get_nowait())
            except Exception:                 # queue.Empty
                break
        for c in held:
            c.close()
            self._free.put(c)

    # convenience wrappers
    def ping(self) -> bool:
        return self.call("PING") == "PONG"

    def set(self, key: str, value: bytes, ex_s: int = 0):
        return self.call("SET", key, value, "EX", int(ex_s)) if ex_s > 0 else self.call("SET", key, value)

    def get(self, key: str) -> Optional[bytes]:
        return self.call("GET", key)

    def delete(self, *keys) -> int:
        return self.call("DEL", *keys)

    def sadd(self, key: str, *members) -> int:
        return self.call("SADD", key, *members)

    def srem(self, key: str, *members) -> int:
        return self.call("SREM", key, *members)

    def smembers(self, key: str) -> List[str]:
        return sorted(m.decode() for m in (self.call("SMEMBERS", key) or []))

    def expire(self, key: str, s: int) -> int:
        return self.call("EXPIRE", key, int(s))


class MiniRedis:
    """Tiny threaded RESP server (strings + sets + TTL) for tests/dev."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0):
        self.kv: Dict[str, bytes] = {}
        self.sets: Dict[str, Set[bytes]] = {}
        self.ttl: Dict[str, float] = {}
        self.lock = threading.Lock()
        outer = self

        class H(socketserver.BaseRequestHandler):
            def handle(self):
                rd = _Reader(self.request)
                try:
                    while True:
                        cmd = rd.reply()
                        if not isinstance(cmd, list) or not cmd:
                            return
                        self.request.sendall(outer._exec([c if isinstance(c, bytes) else str(c).encode() for c in cmd]))
                except (ConnectionError, OSError):
                    return

        self.srv = socketserver.ThreadingTCPServer((host, port), H)
        self.srv.daemon_threads = True
        self.addr = f"{self.srv.server_address[0]}:{self.srv.server_address[1]}"
        self.th = threading.Thread(target=self.srv.serve_forever, daemon=True)
        self.th.start()

    def close(self):
        self.srv.shutdown()
        self.srv.server_close()

    def _alive(self, k: str) -> bool:
        t = self.ttl.get(k)
        if t is not None and time.monotonic() > t:
            self.kv.pop(k, None)
            self.sets.pop(k, None)
            self.ttl.pop(k, None)
            return False
        return k in self.kv or k in self.sets

    def _exec(self, cmd: List[bytes]) -> bytes:
        name = cmd[0].decode().upper()
        a = [c.decode() for c in cmd[1:2]]
        with self.lock:
            if name == "PING":
                return b"+PONG\r\n"
            if name in ("AUTH", "SELECT"):
                return b"+OK\r\n"
            k = a[0] if a else ""
            if name == "SET":
                self.kv[k] = cmd[2]
                self.ttl.pop(k, None)
                if len(cmd) >= 5 and cmd[3].upper() == b"EX":
                    self.ttl[k] = time.monotonic() + int(cmd[4])
                return b"+OK\r\n"
            if name == "GET":
                if not self._alive(k) or k not in self.kv:
                    return b"$-1\r\n"
                v = self.kv[k]
                return b"$%d\r\n%s\r\n" % (len(v), v)
            if name == "DEL":
                n = 0
                for key in cmd[1:]:
                    kk = key.decode()
                    if self._alive(kk):
                        n += 1
                    self.kv.pop(kk, None)
                    self.sets.pop(kk, None)
                    self.ttl.pop(kk, None)
                return b":%d\r\n" % n
            if name == "SADD":
                self._alive(k)
                s = self.sets.setdefault(k, set())
                before = len(s)
                s.update(cmd[2:])
                return b":%d\r\n" % (len(s) - before)
            if name == "SREM":
                s = self.sets.get(k, set())
                before = len(s)
                s.difference_update(cmd[2:])
                return b":%d\r\n" % (before - len(s))
            if name == "SMEMBERS":
                s = self.sets.get(k, set()) if self._alive(k) else set()
                return b"*%d\r\n" % len(s) + b"".join(b"$%d\r\n%s\r\n" % (len(m), m) for m in sorted(s))
            if name == "EXPIRE":
                if not self._alive(k):
                    return b":0\r\n"
                self.ttl[k] = time.monotonic() + int(cmd[2])
                return b":1\r\n"
        return b"-ERR unknown command\r\n"
