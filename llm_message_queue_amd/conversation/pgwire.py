"""Minimal PostgreSQL client (frontend/backend protocol v3) -- no driver
package is available in this image (``psycopg2``/``psycopg`` are absent),
and the reference's relational store is Postgres through GORM
(`internal/conversation/persistence.go:162-320`,
`internal/statemanager/manager.go:16-207`, `deployments/docker-compose.yml`).

Client (``PgConnection``):
  * startup + authentication: trust, cleartext, MD5 and SCRAM-SHA-256
    (RFC 5802 / 7677, the PostgreSQL >= 14 default);
  * ``execute(sql, params)``: the extended query protocol (Parse / Bind /
    Describe / Execute / Sync) with text-format parameters -- values are
    never spliced into SQL; ``$1..$n`` placeholders (``qmark_to_dollar``
    converts the ``?`` style the SQLite paths use);
  * ``simple(sql)``: the simple query protocol (DDL, several statements);
  * results are decoded from text format by type OID (int, float, bool,
    bytea, text / json / timestamps as str); errors raise ``PgError`` with
    the SQLSTATE.  One connection, serialised by a lock.

Test server (``MiniPostgres``): an in-process, threaded protocol-v3 server
that authenticates with SCRAM-SHA-256 or MD5 and executes the statements on
SQLite (``$n`` -> ``?n``; Postgres type names are accepted by SQLite's
type affinity, and ``INSERT ... ON CONFLICT ... DO UPDATE`` is common
syntax).  It lets the persistence and DB-state tests run the real wire path
on a CPU box, like ``resp.MiniRedis`` does for Redis.
"""
from __future__ import annotations

import base64
import hashlib
import hmac
import os
import re
import socket
import socketserver
import sqlite3
import struct
import threading
from typing import Any, Dict, List, Optional, Sequence, Tuple

PROTOCOL_V3 = 196608

# type OIDs used in RowDescription
OID_BOOL, OID_BYTEA, OID_INT8, OID_INT2, OID_INT4, OID_TEXT = 16, 17, 20, 21, 23, 25
OID_JSON, OID_FLOAT4, OID_FLOAT8, OID_VARCHAR, OID_JSONB = 114, 700, 701, 1043, 3802
_INT_OIDS = {OID_INT2, OID_INT4, OID_INT8, 26}
_FLOAT_OIDS = {OID_FLOAT4, OID_FLOAT8, 1700}


class PgError(Exception):
    def __init__(self, fields: Dict[str, str]):
        self.fields = fields
        self.sqlstate = fields.get("C", "")
        super().__init__(f"{fields.get('S', 'ERROR')} {self.sqlstate}: {fields.get('M', '')}")


def qmark_to_dollar(sql: str) -> str:
    """``?`` placeholders -> ``$1..$n`` (outside single-quoted literals)."""
    out, n, q = [], 0, False
    for ch in sql:
        if ch == "'":
            q = not q
        if ch == "?" and not q:
            n += 1
            out.append(f"${n}")
        else:
            out.append(ch)
    return "".join(out)


def _param_text(v: Any) -> Optional[bytes]:
    if v is None:
        return None
    if isinstance(v, bool):
        return b"true" if v else b"false"
    if isinstance(v, (bytes, bytearray, memoryview)):
        return b"\\x" + bytes(v).hex().encode()
    return str(v).encode()


def _decode(oid: int, raw: Optional[bytes]) -> Any:
    if raw is None:
        return None
    if oid in _INT_OIDS:
        return int(raw)
    if oid in _FLOAT_OIDS:
        return float(raw)
    if oid == OID_BOOL:
        return raw in (b"t", b"true", b"1")
    if oid == OID_BYTEA:
        return bytes.fromhex(raw[2:].decode()) if raw.startswith(b"\\x") else raw
    return raw.decode("utf-8")


class PgResult:
    def __init__(self, columns: List[str], rows: List[Tuple[Any, ...]], tag: str):
        self.columns, self.rows, self.tag = columns, rows, tag

    @property
    def rowcount(self) -> int:
        parts = self.tag.split()
        return int(parts[-1]) if parts and parts[-1].isdigit() else len(self.rows)

    def fetchone(self):
        return self.rows[0] if self.rows else None

    def fetchall(self):
        return list(self.rows)


# ---------------------------------------------------------------- SCRAM-SHA-256
def _hi(password: bytes, salt: bytes, iters: int) -> bytes:
    return hashlib.pbkdf2_hmac("sha256", password, salt, iters)


def _hmac(key: bytes, msg: bytes) -> bytes:
    return hmac.new(key, msg, hashlib.sha256).digest()


def _xor(a: bytes, b: bytes) -> bytes:
    return bytes(x ^ y for x, y in zip(a, b))


def _scram_attrs(s: str) -> Dict[str, str]:
    return dict(kv.split("=", 1) for kv in s.split(",") if "=" in kv)


class PgConnection:
    def __init__(self, host: str = "localhost", port: int = 5432, user: str = "postgres", password: str = "",
                 dbname: str = "postgres", timeout: float = 10.0, sslmode: str = "disable"):
        if sslmode not in ("disable", "allow", "prefer"):
            raise PgError({"M": f"sslmode={sslmode} needs TLS, which this client does not implement"})
        self.user, self.password, self.dbname = user, password, dbname
        self._sock = socket.create_connection((host, int(port)), timeout=timeout)
        self._sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._buf = b""
        self._lock = threading.Lock()
        self.params: Dict[str, str] = {}
        self.txn_status = "I"
        self._startup()

    @classmethod
    def from_dsn(cls, dsn: str) -> "PgConnection":
        kv = dict(p.split("=", 1) for p in dsn.split() if "=" in p)
        return cls(kv.get("host", "localhost"), int(kv.get("port", 5432)), kv.get("user", "postgres"),
                   kv.get("password", ""), kv.get("dbname", "postgres"), sslmode=kv.get("sslmode", "disable"))

    # ------------------------------------------------------------ framing
    def _send(self, typ: bytes, payload: bytes = b"") -> None:
        self._sock.sendall(typ + struct.pack("!I", len(payload) + 4) + payload)

    def _recv_exact(self, n: int) -> bytes:
        while len(self._buf) < n:
            chunk = self._sock.recv(max(65536, n - len(self._buf)))
            if not chunk:
                raise ConnectionError("postgres server closed the connection")
            self._buf += chunk
        out, self._buf = self._buf[:n], self._buf[n:]
        return out

    def _recv(self) -> Tuple[bytes, bytes]:
        hdr = self._recv_exact(5)
        typ, ln = hdr[:1], struct.unpack("!I", hdr[1:])[0]
        return typ, self._recv_exact(ln - 4)

    @staticmethod
    def _fields(payload: bytes) -> Dict[str, str]:
        out, i = {}, 0
        while i < len(payload) and payload[i] != 0:
            j = payload.index(b"\x00", i + 1)
            out[chr(payload[i])] = payload[i + 1:j].decode("utf-8", "replace")
            i = j + 1
        return out

    # ------------------------------------------------------------ startup / auth
    def _startup(self) -> None:
        body = struct.pack("!I", PROTOCOL_V3)
        for k, v in (("user", self.user), ("database", self.dbname), ("client_encoding", "UTF8")):
            body += k.encode() + b"\x00" + v.encode() + b"\x00"
        body += b"\x00"
        self._sock.sendall(struct.pack("!I", len(body) + 4) + body)
        scram = None
        while True:
            typ, p = self._recv()
            if typ == b"R":
                code = struct.unpack("!I", p[:4])[0]
                if code == 0:
                    continue
                if code == 3:                                   # cleartext
                    self._send(b"p", self.password.encode() + b"\x00")
                elif code == 5:                                 # md5
                    inner = hashlib.md5((self.password + self.user).encode()).hexdigest()
                    outer = hashlib.md5(inner.encode() + p[4:8]).hexdigest()
                    self._send(b"p", b"md5" + outer.encode() + b"\x00")
                elif code == 10:                                # SASL: mechanisms
                    mechs = [m for m in p[4:].split(b"\x00") if m]
                    if b"SCRAM-SHA-256" not in mechs:
                        raise PgError({"M": f"unsupported SASL mechanisms {mechs}"})
                    nonce = base64.b64encode(os.urandom(18)).decode()
                    first_bare = f"n=,r={nonce}"
                    msg = ("n,," + first_bare).encode()
                    self._send(b"p", b"SCRAM-SHA-256\x00" + struct.pack("!I", len(msg)) + msg)
                    scram = {"nonce": nonce, "first_bare": first_bare}
                elif code == 11:                                # SASL continue
                    srv_first = p[4:].decode()
                    a = _scram_attrs(srv_first)
                    if not a["r"].startswith(scram["nonce"]):
                        raise PgError({"M": "SCRAM nonce mismatch"})
                    salted = _hi(self.password.encode(), base64.b64decode(a["s"]), int(a["i"]))
                    client_key = _hmac(salted, b"Client Key")
                    final_wo = f"c=biws,r={a['r']}"
                    auth_msg = f"{scram['first_bare']},{srv_first},{final_wo}".encode()
                    proof = _xor(client_key, _hmac(hashlib.sha256(client_key).digest(), auth_msg))
                    scram["server_sig"] = _hmac(_hmac(salted, b"Server Key"), auth_msg)
                    self._send(b"p", f"{final_wo},p={base64.b64encode(proof).decode()}".encode())
                elif code == 12:                                # SASL final: verify the server
                    v = _scram_attrs(p[4:].decode()).get("v", "")
                    if not hmac.compare_digest(base64.b64decode(v), scram["server_sig"]):
                        raise PgError({"M": "SCRAM server signature mismatch"})
                else:
                    raise PgError({"M": f"unsupported authentication request {code}"})
            elif typ == b"S":
                k, v, _ = p.split(b"\x00", 2)
                self.params[k.decode()] = v.decode()
            elif typ == b"K":
                pass
            elif typ == b"E":
                raise PgError(self._fields(p))
            elif typ == b"N":
                pass
            elif typ == b"Z":
                self.txn_status = p[:1].decode()
                return

    # ------------------------------------------------------------ queries
    def _collect(self) -> List[PgResult]:
        """Read until ReadyForQuery; raise the first error after syncing."""
        results: List[PgResult] = []
        cols: List[Tuple[str, int]] = []
        rows: List[Tuple[Any, ...]] = []
        err = None
        while True:
            typ, p = self._recv()
            if typ == b"T":
                n = struct.unpack("!H", p[:2])[0]
                i, cols = 2, []
                for _ in range(n):
                    j = p.index(b"\x00", i)
                    name = p[i:j].decode()
                    oid = struct.unpack("!I", p[j + 7:j + 11])[0]
                    cols.append((name, oid))
                    i = j + 19
                rows = []
            elif typ == b"D":
                n = struct.unpack("!H", p[:2])[0]
                i, vals = 2, []
                for k in range(n):
                    ln = struct.unpack("!i", p[i:i + 4])[0]
                    i += 4
                    raw = None if ln < 0 else p[i:i + ln]
                    i += max(ln, 0)
                    vals.append(_decode(cols[k][1] if k < len(cols) else OID_TEXT, raw))
                rows.append(tuple(vals))
            elif typ == b"C":
                results.append(PgResult([c[0] for c in cols], rows, p[:-1].decode()))
                cols, rows = [], []
            elif typ == b"I":
                results.append(PgResult([], [], ""))
            elif typ == b"E":
                err = err or PgError(self._fields(p))
            elif typ == b"Z":
                self.txn_status = p[:1].decode()
                if err is not None:
                    raise err
                return results
            # '1' ParseComplete, '2' BindComplete, 'n' NoData, 'N' notice, 'S' param status, 's' suspended

    def execute(self, sql: str, params: Sequence[Any] = ()) -> PgResult:
        """One statement through the extended protocol, ``$n`` parameters."""
        q = sql.encode() + b"\x00"
        vals = [_param_text(v) for v in params]
        bind = b"\x00\x00" + struct.pack("!HH", 0, len(vals))     # portal "", stmt "", all-text params
        for v in vals:
            bind += struct.pack("!i", -1) if v is None else struct.pack("!i", len(v)) + v
        bind += struct.pack("!H", 0)                                 # all-text results
        with self._lock:
            self._sock.sendall(
                b"P" + struct.pack("!I", 4 + 1 + len(q) + 2) + b"\x00" + q + b"\x00\x00"
                + b"B" + struct.pack("!I", 4 + len(bind)) + bind
                + b"D" + struct.pack("!I", 4 + 2) + b"P\x00"
                + b"E" + struct.pack("!I", 4 + 5) + b"\x00" + struct.pack("!I", 0)
                + b"S" + struct.pack("!I", 4))
            res = self._collect()
        return res[-1] if res else PgResult([], [], "")

    def simple(self, sql: str) -> List[PgResult]:
        with self._lock:
            self._send(b"Q", sql.encode() + b"\x00")
            return self._collect()

    def close(self) -> None:
        try:
            with self._lock:
                self._send(b"X")
        except OSError:
            pass
        self._sock.close()


# ================================================================ test server
class MiniPostgres:
    """In-process PostgreSQL protocol-v3 server over SQLite (tests / demos).

    ``auth``: "scram" (SCRAM-SHA-256, default), "md5", "password" or "trust".
    One SQLite database shared by every connection (serialised)."""

    def __init__(self, host: str = "127.0.0.1", port: int = 0, user: str = "postgres",
                 password: str = "password", auth: str = "scram"):
        self.user, self.password, self.auth = user, password, auth
        self.db = sqlite3.connect(":memory:", check_same_thread=False)
        self.db_lock = threading.Lock()
        self.statements = 0
        outer = self

        class Handler(socketserver.BaseRequestHandler):
            def handle(self):
                try:
                    _Session(self.request, outer).run()
                except (ConnectionError, OSError, struct.error):
                    pass

        class Server(socketserver.ThreadingTCPServer):
            daemon_threads = True
            allow_reuse_address = True

        self._srv = Server((host, port), Handler)
        self.addr = "%s:%d" % self._srv.server_address
        self.host, self.port = self._srv.server_address
        self._t = threading.Thread(target=self._srv.serve_forever, daemon=True)
        self._t.start()

    def close(self) -> None:
        self._srv.shutdown()
        self._srv.server_close()
        self.db.close()


_DOLLAR = re.compile(r"\$(\d+)")


class _Session:
    def __init__(self, sock, srv: MiniPostgres):
        self.sock, self.srv = sock, srv
        self.buf = b""
        self.stmt: Optional[str] = None
        self.params: List[Any] = []
        self.result: Optional[Tuple[List[str], List[tuple], str]] = None
        self.failed = False

    def recv_exact(self, n):
        while len(self.buf) < n:
            c = self.sock.recv(65536)
            if not c:
                raise ConnectionError()
            self.buf += c
        out, self.buf = self.buf[:n], self.buf[n:]
        return out

    def send(self, typ: bytes, payload: bytes = b""):
        self.sock.sendall(typ + struct.pack("!I", len(payload) + 4) + payload)

    def error(self, code: str, msg: str):
        self.send(b"E", b"SERROR\x00C" + code.encode() + b"\x00M" + msg.encode() + b"\x00\x00")

    def auth(self) -> bool:
        s = self.srv
        if s.auth == "trust":
            return True
        if s.auth == "password":
            self.send(b"R", struct.pack("!I", 3))
            typ, p = self.recv_msg()
            return p[:-1].decode() == s.password
        if s.auth == "md5":
            salt = os.urandom(4)
            self.send(b"R", struct.pack("!I", 5) + salt)
            typ, p = self.recv_msg()
            inner = hashlib.md5((s.password + s.user).encode()).hexdigest()
            want = "md5" + hashlib.md5(inner.encode() + salt).hexdigest()
            return hmac.compare_digest(p[:-1].decode(), want)
        # SCRAM-SHA-256
        self.send(b"R", struct.pack("!I", 10) + b"SCRAM-SHA-256\x00\x00")
        typ, p = self.recv_msg()
        mech_end = p.index(b"\x00")
        ln = struct.unpack("!i", p[mech_end + 1:mech_end + 5])[0]
        client_first = p[mech_end + 5:mech_end + 5 + ln].decode()
        first_bare = client_first.split(",", 2)[2]
        cnonce = _scram_attrs(first_bare)["r"]
        salt, iters = os.urandom(16), 4096
        nonce = cnonce + base64.b64encode(os.urandom(18)).decode()
        srv_first = f"r={nonce},s={base64.b64encode(salt).decode()},i={iters}"
        self.send(b"R", struct.pack("!I", 11) + srv_first.encode())
        typ, p = self.recv_msg()
        final = p.decode()
        a = _scram_attrs(final)
        final_wo = final[:final.rindex(",p=")]
        salted = _hi(s.password.encode(), salt, iters)
        client_key = _hmac(salted, b"Client Key")
        stored = hashlib.sha256(client_key).digest()
        auth_msg = f"{first_bare},{srv_first},{final_wo}".encode()
        proof = base64.b64decode(a.get("p", ""))
        if a.get("r") != nonce or hashlib.sha256(_xor(proof, _hmac(stored, auth_msg))).digest() != stored:
            return False
        sig = base64.b64encode(_hmac(_hmac(salted, b"Server Key"), auth_msg)).decode()
        self.send(b"R", struct.pack("!I", 12) + f"v={sig}".encode())
        return True

    def recv_msg(self):
        hdr = self.recv_exact(5)
        return hdr[:1], self.recv_exact(struct.unpack("!I", hdr[1:])[0] - 4)

    def run(self):
        ln = struct.unpack("!I", self.recv_exact(4))[0]
        body = self.recv_exact(ln - 4)
        if struct.unpack("!I", body[:4])[0] == 80877103:       # SSLRequest -> not supported
            self.sock.sendall(b"N")
            ln = struct.unpack("!I", self.recv_exact(4))[0]
            body = self.recv_exact(ln - 4)
        kv = body[4:].split(b"\x00")
        opts = {kv[i].decode(): kv[i + 1].decode() for i in range(0, len(kv) - 1, 2) if kv[i]}
        if opts.get("user") != self.srv.user or not self.auth():
            self.error("28P01", f'password authentication failed for user "{opts.get("user")}"')
            return
        self.send(b"R", struct.pack("!I", 0))
        for k, v in (("server_version", "16.0 (llmq MiniPostgres)"), ("client_encoding", "UTF8")):
            self.send(b"S", k.encode() + b"\x00" + v.encode() + b"\x00")
        self.send(b"K", struct.pack("!II", os.getpid() & 0x7FFFFFFF, 0))
        self.send(b"Z", b"I")
        while True:
            typ, p = self.recv_msg()
            if typ == b"X":
                return
            if typ == b"Q":
                self.simple(p[:-1].decode())
            elif typ == b"P":
                if self.failed:
                    continue
                j = p.index(b"\x00")
                k = p.index(b"\x00", j + 1)
                self.stmt = p[j + 1:k].decode()
                self.send(b"1")
            elif typ == b"B":
                if self.failed:
                    continue
                i = p.index(b"\x00") + 1
                i = p.index(b"\x00", i) + 1
                nf = struct.unpack("!H", p[i:i + 2])[0]
                i += 2 + 2 * nf
                n = struct.unpack("!H", p[i:i + 2])[0]
                i += 2
                vals = []
                for _ in range(n):
                    ln = struct.unpack("!i", p[i:i + 4])[0]
                    i += 4
                    vals.append(None if ln < 0 else p[i:i + ln].decode())
                    i += max(ln, 0)
                self.params = vals
                self.send(b"2")
            elif typ == b"D":
                if self.failed:
                    continue
                self.result = self.run_sql(self.stmt or "", self.params)
                if self.result is None:
                    continue
                cols, rows, _tag = self.result
                if cols:
                    self.row_description(cols, rows)
                else:
                    self.send(b"n")
            elif typ == b"E":
                if self.failed or self.result is None:
                    continue
                cols, rows, tag = self.result
                for r in rows:
                    self.data_row(r)
                self.send(b"C", tag.encode() + b"\x00")
            elif typ == b"S":
                self.failed = False
                self.result = None
                self.send(b"Z", b"I")

    def simple(self, sql: str):
        for stmt in [s for s in sql.split(";") if s.strip()]:
            res = self.run_sql(stmt, [])
            if res is None:
                break
            cols, rows, tag = res
            if cols:
                self.row_description(cols, rows)
                for r in rows:
                    self.data_row(r)
            self.send(b"C", tag.encode() + b"\x00")
        self.failed = False
        self.send(b"Z", b"I")

    def run_sql(self, sql: str, params: List[Any]):
        s = _DOLLAR.sub(lambda m: "?" + m.group(1), sql)
        try:
            with self.srv.db_lock:
                cur = self.srv.db.execute(s, params)
                rows = cur.fetchall()
                cols = [d[0] for d in cur.description] if cur.description else []
                self.srv.db.commit()
                self.srv.statements += 1
        except sqlite3.IntegrityError as e:
            self.failed = True
            self.error("23505", str(e))
            return None
        except sqlite3.Error as e:
            self.failed = True
            self.error("42601", str(e))
            return None
        verb = s.strip().split(None, 1)[0].upper() if s.strip() else ""
        tag = {"SELECT": f"SELECT {len(rows)}", "INSERT": f"INSERT 0 {cur.rowcount}",
               "UPDATE": f"UPDATE {cur.rowcount}", "DELETE": f"DELETE {cur.rowcount}"}.get(verb, verb)
        return cols, rows, tag

    def row_description(self, cols, rows):
        body = struct.pack("!H", len(cols))
        for k, name in enumerate(cols):
            v = next((r[k] for r in rows if r[k] is not None), None)   # column type from its first value
            oid = (OID_BOOL if isinstance(v, bool) else OID_INT8 if isinstance(v, int) else
                   OID_FLOAT8 if isinstance(v, float) else OID_BYTEA if isinstance(v, bytes) else OID_TEXT)
            body += name.encode() + b"\x00" + struct.pack("!IHIhiH", 0, 0, oid, -1, -1, 0)
        self.send(b"T", body)

    def data_row(self, r):
        body = struct.pack("!H", len(r))
        for v in r:
            if v is None:
                body += struct.pack("!i", -1)
                continue
            b = (b"\\x" + v.hex().encode()) if isinstance(v, bytes) else str(v).encode()
            body += struct.pack("!i", len(b)) + b
        self.send(b"D", body)
