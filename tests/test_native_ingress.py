"""Native C++ HTTP ingress -> shared request ring -> dispatcher (preprocess,
queue, CPU workers) end to end, plus the ingress's HTTP/JSON edge cases."""
import json
import os
import socket
import time
import urllib.request

import pytest

from llm_message_queue_amd import _native
from llm_message_queue_amd.gateway.native_ingress import NativeIngress
from llm_message_queue_amd.gateway.shm_bridge import RingPair


def _post(port, body, raw=False):
    data = body if raw else json.dumps(body).encode()
    req = urllib.request.Request(f"http://127.0.0.1:{port}/api/v1/messages", data=data, method="POST",
                                 headers={"Content-Type": "application/json"})
    try:
        with urllib.request.urlopen(req, timeout=5) as r:
            return r.status, json.loads(r.read())
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read())


def test_lone_surrogate_in_another_field_does_not_poison_the_id():
    """a lone-surrogate escape in content must not make a
    later valid id fail (the flag was never reset); Python accepts this body."""
    scan = _native.ingress().scan_message
    r = scan(b'{"content":"bad \\ud800 escape","id":"abc-123","user_id":"u1"}')
    assert r[0] and r[1] == "abc-123" and r[3] == "u1", r
    assert not scan(b'{"id":"a\\ud800b"}')[0]          # the id itself still must be printable ASCII
    # conversation_id presence (front door routing to the conversation owner's ring)
    assert scan(b'{"content":"x","conversation_id":"c-1"}')[5]
    for v in (b'null', b'""', b'0', b'false'):
        assert not scan(b'{"content":"x","conversation_id":' + v + b'}')[5], v


def test_json_scanner():
    scan = _native.ingress().scan_message
    assert scan(b'{"content":"hi","priority":"urgent","id":"abc"}')[:4] == (True, "abc", 1, "")
    assert scan(b'{"content":"a\\"b","metadata":{"x":[1,{"y":null}]},"priority":4,"user_id":"u"}')[0:3:2] == (True, 4)
    assert scan(b'{}')[:4] == (True, "", 0, "")
    for bad in (b'', b'[1]', b'{"content":}', b'{"priority":"bogus"}', b'{"a":1,}', b'{"a":1} x', b'{"priority":9}',
                b'{"priority":-1}', b'{"priority":"5"}', b'{"priority":"-2"}', b'{"priority":" "}',
                b'{}\x00', b'{}\x80', b'{} x', b'{ }}'):
        assert not scan(bad)[0], bad


def test_priority_rule_matches_python_front_door():
    """Both front doors accept the same priorities and assign the same tier:
    the native scanner's value equals ``parse_priority`` (what the Python
    front door and the rank's decode use) and it rejects exactly what
    ``parse_priority`` rejects."""
    from hypothesis import given, settings, strategies as st
    from llm_message_queue_amd.models.message import PriorityParseError, parse_priority
    scan = _native.ingress().scan_message
    names = ["realtime", "urgent", "high", "normal", "medium", "low", "URGENT", " High\t", "\nlow ", "Medium",
             "0", "1", "4", "5", "-0", "-1", "+2", "+", "-", "", " ", "002", "0004", "00005", "1_0", "2.0", "1e0",
             " high", "high ", "٣", "Kow", "hi gh", "realtime!"]
    nums = [0, 1, 2, 3, 4, 5, -1, 9, 2.0, 2.5, -0.0, 1e300, 4.000001]

    def check(v):
        body = json.dumps({"content": "x", "priority": v}).encode()
        ok, _id, prio = scan(body)[:3]
        try:
            want = parse_priority(v, 0)
        except PriorityParseError:
            assert not ok, (v, prio)
            return
        assert ok and prio == want, (v, ok, prio, want)

    for v in names + nums:
        check(v)

    @settings(max_examples=300, deadline=None)
    @given(st.text(alphabet=st.sampled_from(list("0123456789+- \t\nLOWHIGHlowhighmediumurgent ")), max_size=9)
           | st.integers(-10, 10))
    def prop(v):
        check(v)
    prop()


def test_gateway_compat_reply():
    """``cli api-gateway --native``: the 202 also carries the reference
    api-gateway's ``message`` / ``id`` (cmd/api-gateway/main.go:113); the
    monolith front door's reply stays the reference server's shape."""
    name = f"pyt-compat-{os.getpid()}"
    ring = RingPair(name, 1 << 20, "create")
    ings = [NativeIngress(0, name, threads=1, host="127.0.0.1", gateway_compat=c) for c in (True, False)]
    try:
        ports = [i.start() for i in ings]
        code, r = _post(ports[0], {"content": "hi", "id": "cid-7"})
        assert code == 202 and r["message"] == "Message accepted" and r["id"] == "cid-7" == r["message_id"], r
        code, r = _post(ports[1], {"content": "hi"})
        assert code == 202 and "id" not in r and "message" not in r and len(r["message_id"]) == 36, r
    finally:
        for i in ings:
            i.stop()
        ring.close(unlink=True)


@pytest.fixture
def stack():
    from llm_message_queue_amd.gateway.app import GatewayApp
    from llm_message_queue_amd.utils.config import default_config
    cfg = default_config()
    cfg.queue.worker.process_interval = 5_000_000
    name = f"pyt-native-{os.getpid()}"
    ring = RingPair(name, 1 << 20, "create")
    disp = GatewayApp(cfg, use_gpu=False, simulate_ms=(1, 1, 1, 1), role="dispatcher", ring=ring)
    ing = NativeIngress(0, name, threads=2, host="127.0.0.1")
    port = ing.start()
    yield disp, ing, port
    ing.stop()
    disp.stop()
    ring.close(unlink=True)


def test_native_ingress_end_to_end(stack):
    disp, ing, port = stack
    ids = []
    for i in range(30):
        body = {"content": ("EMERGENCY now " if i % 5 == 0 else "hello ") + str(i), "user_id": f"u{i}"}
        if i % 7 == 0:
            body["priority"] = "low"
        code, r = _post(port, body)
        assert code == 202 and len(r["message_id"]) == 36, r
        ids.append(r["message_id"])
    code, r = _post(port, {"content": "mine", "id": "client-id-1"})
    assert code == 202 and r["message_id"] == "client-id-1"
    ids.append("client-id-1")
    t0 = time.time()
    while time.time() - t0 < 10 and not all((disp.messages.get(i) and disp.messages.get(i).status == "completed")
                                            for i in ids):
        time.sleep(0.02)
    got = [disp.messages.get(i) for i in ids]
    assert all(g is not None and g.status == "completed" for g in got)
    assert got[5].priority == 1 and got[5].metadata.get("analyzed")        # preprocessed in the dispatcher
    # the dispatcher records AnalyzeMessageContent like the API handler does (queue.enable_metrics)
    assert all(json.loads(g.metadata["analysis"]) == disp.preprocessor.analyze_message_content(g.content)
               for g in got)
    assert got[7].priority == 4 and got[0].arrival_ns > 0
    assert ing.stats()["accepted"] == 31


def test_native_ingress_http_edges(stack):
    _, ing, port = stack
    assert _post(port, b'{"content": "x",', raw=True)[0] == 400
    with urllib.request.urlopen(f"http://127.0.0.1:{port}/health", timeout=5) as r:
        assert r.status == 200 and json.loads(r.read())["status"] == "ok"
    try:
        urllib.request.urlopen(f"http://127.0.0.1:{port}/api/v1/queues/stats", timeout=5)
        assert False
    except urllib.error.HTTPError as e:
        assert e.code == 404
    # keep-alive + pipelining: two requests in one write, two responses in order
    b1 = json.dumps({"content": "one"}).encode()
    b2 = json.dumps({"content": "two", "priority": 2}).encode()
    req = b"".join(b"POST /api/v1/messages HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n%s" % (len(b), b)
                   for b in (b1, b2))
    s = socket.create_connection(("127.0.0.1", port))
    s.sendall(req)
    data = b""
    t0 = time.time()
    while data.count(b"HTTP/1.1 202") < 2 and time.time() - t0 < 5:
        data += s.recv(65536)
    s.close()
    assert data.count(b"HTTP/1.1 202") == 2 and b'"priority":2' in data


def _raw(port, payload, timeout=3.0):
    s = socket.create_connection(("127.0.0.1", port))
    s.settimeout(timeout)
    try:
        s.sendall(payload)
        data = b""
        while True:
            try:
                chunk = s.recv(65536)
            except (socket.timeout, ConnectionResetError):
                break
            if not chunk:
                break
            data += chunk
            if b"\r\n\r\n" in data:
                break
        return data
    finally:
        s.close()


def test_native_ingress_hostile_framing(stack):
    """Untrusted framing: absurd / non-numeric Content-Length, chunked bodies,
    oversized headers and random bytes get a clean error (or a close) and the
    server keeps serving."""
    _, ing, port = stack
    post = b"POST /api/v1/messages HTTP/1.1\r\nHost: x\r\n"
    assert b" 400 " in _raw(port, post + b"Content-Length: 18446744073709551615\r\n\r\n{}")
    assert b" 400 " in _raw(port, post + b"Content-Length: -5\r\n\r\n{}")
    assert b" 400 " in _raw(port, post + b"Content-Length: 12abc\r\n\r\n{}")
    assert b" 413 " in _raw(port, post + b"Content-Length: 999999999\r\n\r\n{}")
    assert b" 501 " in _raw(port, post + b"Transfer-Encoding: chunked\r\n\r\n2\r\n{}\r\n0\r\n\r\n")
    assert b" 431 " in _raw(port, post + b"X-Pad: " + b"a" * (70 << 10))
    import random
    rnd = random.Random(3)
    for _ in range(40):
        junk = bytes(rnd.getrandbits(8) for _ in range(rnd.randrange(1, 400)))
        if rnd.random() < 0.5:
            junk = post + junk + b"\r\n\r\n"
        _raw(port, junk, timeout=0.3)
    with urllib.request.urlopen(f"http://127.0.0.1:{port}/health", timeout=5) as r:
        assert r.status == 200
    code, r = _post(port, {"content": "still alive"})
    assert code == 202


def test_json_scanner_properties():
    """The native scanner on arbitrary bytes never faults, and accepts every
    well-formed JSON object whose reserved fields are absent."""
    from hypothesis import given, settings, strategies as st
    scan = _native.ingress().scan_message
    leaf = st.none() | st.booleans() | st.integers(-10**12, 10**12) | st.floats(allow_nan=False, allow_infinity=False) \
        | st.text(max_size=20)
    val = st.recursive(leaf, lambda c: st.lists(c, max_size=4) | st.dictionaries(st.text(max_size=8), c, max_size=4),
                       max_leaves=12)
    reserved = {"id", "priority", "user_id", "content", "metadata", "timeout", "max_retries", "retry_count",
                "created_at", "updated_at", "scheduled_at", "completed_at"}

    @settings(max_examples=300, deadline=None)
    @given(st.binary(max_size=200))
    def arbitrary(b):
        r = scan(b)
        assert isinstance(r, tuple) and r[0] in (True, False)

    @settings(max_examples=300, deadline=None)
    @given(st.dictionaries(st.text(max_size=8).filter(lambda k: k not in reserved), val, max_size=5), st.booleans())
    def wellformed(d, ascii_only):
        doc = json.dumps(d, ensure_ascii=ascii_only).encode()
        assert scan(doc)[0], d
        # every strict prefix of an object is malformed and must be refused
        for k in range(0, len(doc), max(1, len(doc) // 7)):
            assert not scan(doc[:k])[0], doc[:k]

    arbitrary()
    wellformed()


def test_native_ingress_expect_continue_and_half_close(stack):
    _, ing, port = stack
    body = json.dumps({"content": "x" * 2000}).encode()
    s = socket.create_connection(("127.0.0.1", port))
    s.settimeout(5)
    s.sendall(b"POST /api/v1/messages HTTP/1.1\r\nHost: x\r\nExpect: 100-continue\r\n"
              b"Content-Length: %d\r\n\r\n" % len(body))
    assert s.recv(4096).startswith(b"HTTP/1.1 100 Continue\r\n\r\n")
    s.sendall(body)
    data = b""
    while b"\r\n\r\n" not in data:
        data += s.recv(65536)
    assert data.startswith(b"HTTP/1.1 202")
    s.close()
    # a client that half-closes after its request still gets the answer
    s = socket.create_connection(("127.0.0.1", port))
    s.settimeout(5)
    b2 = json.dumps({"content": "bye"}).encode()
    s.sendall(b"POST /api/v1/messages HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n%s" % (len(b2), b2))
    s.shutdown(socket.SHUT_WR)
    data = b""
    while True:
        chunk = s.recv(65536)
        if not chunk:
            break
        data += chunk
    s.close()
    assert data.startswith(b"HTTP/1.1 202")


def test_native_ingress_1500_concurrent_keepalive_connections(stack):
    """The reference's "> 1,000 concurrent connections" target
    (docs/performance.md:11): 1500 open keep-alive connections, two requests
    each, every one answered 202 on its own connection."""
    import selectors
    _, ing, port = stack
    N = 1500
    body = json.dumps({"content": "conn test"}).encode()
    req = b"POST /api/v1/messages HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n%s" % (len(body), body)
    socks = []
    try:
        for _ in range(N):
            s = socket.create_connection(("127.0.0.1", port), timeout=10)
            socks.append(s)
        for rnd in range(2):
            for s in socks:
                s.sendall(req)
            sel = selectors.DefaultSelector()
            got = {}
            for s in socks:
                s.setblocking(False)
                sel.register(s, selectors.EVENT_READ)
                got[s] = b""
            done = 0
            t0 = time.time()
            while done < N and time.time() - t0 < 30:
                for key, _ in sel.select(timeout=1):
                    s = key.fileobj
                    got[s] += s.recv(4096)
                    if b"\r\n\r\n" in got[s] and got[s].count(b"}") >= 1:
                        sel.unregister(s)
                        done += 1
            sel.close()
            assert done == N, (rnd, done)
            assert all(g.startswith(b"HTTP/1.1 202") for g in got.values())
            for s in socks:
                s.setblocking(True)
        assert ing.stats()["accepted"] >= 2 * N
    finally:
        for s in socks:
            s.close()


_FD_CHILD = r'''
import os, resource, sys, json, time
sys.path.insert(0, sys.argv[1])
from llm_message_queue_amd.gateway.native_ingress import NativeIngress
from llm_message_queue_amd.gateway.shm_bridge import RingPair
name = f"pyt-fd-{os.getpid()}"
ring = RingPair(name, 1 << 20, "create")
ing = NativeIngress(0, name, threads=1, host="127.0.0.1")
port = ing.start()
soft, hard = resource.getrlimit(resource.RLIMIT_NOFILE)
used = len(os.listdir("/proc/self/fd"))
resource.setrlimit(resource.RLIMIT_NOFILE, (used + 40, hard))
print(port, flush=True)
sys.stdin.readline()
t0 = time.process_time()
time.sleep(1.0)
cpu = time.process_time() - t0
print(json.dumps({"refused": ing.stats()["refused_no_fd"], "cpu_s": cpu}), flush=True)
sys.stdin.readline()
ing.stop()
ring.close(unlink=True)
'''


def test_native_ingress_survives_descriptor_exhaustion():
    """Past RLIMIT_NOFILE the ingress refuses new connections (instead of its
    level-triggered listener spinning) and serves again once fds free up."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.Popen([sys.executable, "-c", _FD_CHILD, root], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                         text=True)
    try:
        port = int(p.stdout.readline())
        socks = []
        for _ in range(80):
            try:
                socks.append(socket.create_connection(("127.0.0.1", port), timeout=2))
            except OSError:
                pass
        time.sleep(0.3)
        p.stdin.write("\n")
        p.stdin.flush()
        st = json.loads(p.stdout.readline())
        assert st["refused"] > 0
        assert st["cpu_s"] < 0.5, st                   # no accept spin while exhausted
        for s in socks:
            s.close()
        time.sleep(0.3)
        with urllib.request.urlopen(f"http://127.0.0.1:{port}/health", timeout=5) as r:
            assert r.status == 200
    finally:
        try:
            p.stdin.write("\n")
            p.stdin.flush()
        except OSError:
            pass
        p.wait(timeout=20)


def test_native_ingress_reaps_idle_and_stalled_connections(stack):
    _, ing, port = stack
    ing.set_idle_timeout(0.4)
    idle = socket.create_connection(("127.0.0.1", port), timeout=5)
    stalled = socket.create_connection(("127.0.0.1", port), timeout=5)
    stalled.sendall(b"POST /api/v1/messages HTTP/1.1\r\nHost: x\r\nContent-Le")   # slowloris
    busy = socket.create_connection(("127.0.0.1", port), timeout=5)
    body = json.dumps({"content": "k"}).encode()
    req = b"POST /api/v1/messages HTTP/1.1\r\nHost: x\r\nContent-Length: %d\r\n\r\n%s" % (len(body), body)
    t0 = time.time()
    while time.time() - t0 < 1.5:                 # keeps talking: must survive
        busy.sendall(req)
        assert busy.recv(4096).startswith(b"HTTP/1.1 202")
        time.sleep(0.1)
    assert idle.recv(10) == b"" and stalled.recv(10) == b""          # closed by the server
    busy.sendall(req)
    assert busy.recv(4096).startswith(b"HTTP/1.1 202")
    assert ing.stats()["idle_closed"] >= 2
    for s in (idle, stalled, busy):
        s.close()


STRICT_BAD = [
    b'{"content":"x","n":1.2.3}', b'{"n":+1}', b'{"n":01}', b'{"n":1.}', b'{"n":.5}', b'{"n":1e}', b'{"n":-}',
    b'{"n":NaN}', b'{"n":Infinity}', b'{"c":"bad \\q escape"}', b'{"c":"\\u12G4"}', b'{"c":"\xff\xfe"}',
    b'{"c":"\xc0\xaf"}', b'{"c":"\xed\xa0\x80"}', b'{"metadata":5}', b'{"metadata":"x"}', b'{"metadata":[1]}',
    b'{"timeout":"abc"}', b'{"timeout":"5"}', b'{"timeout":true}', b'{"timeout":1e400}', b'{"max_retries":"x"}',
    b'{"retry_count":[1]}', b'{"created_at":"yesterday"}', b'{"created_at":"2024-02-30T00:00:00Z"}',
    b'{"id":"a\\"b"}', b'{"id":"a\\\\b"}', b'{"id":"\\u00e9"}', b'{"id":5}', b'{"user_id":"x\\ny"}',
    b'{"priority":""}', b'{"priority":2.5}', b'{"priority":"bogus"}',
]


def test_json_scanner_strict_refusals():
    """every body the dispatcher's json.loads / Message.from_dict
    would refuse is refused at the door (400), so a 202 is never followed by
    a silent drop; the reason is reported."""
    scan = _native.ingress().scan_message
    for bad in STRICT_BAD:
        r = scan(bad)
        assert not r[0] and r[4], bad
    ok = [b'{"timeout":"1m30s","max_retries":5,"retry_count":0,"metadata":null}',
          b'{"timeout":30000000000,"created_at":"2024-02-29T12:00:00.5+02:00","c":"\\u00e9\\ud83d\\ude00 \xc3\xa9"}',
          b'{"id":"abc-123_X.y","user_id":"u 1","priority":null,"timeout":null}']
    for good in ok:
        assert scan(good)[0], good


def test_scan_ok_implies_dispatcher_decodes():
    """Property: whenever the native scanner accepts a body, the dispatcher's
    decode (json.loads + Message.from_dict) succeeds on the same bytes."""
    from hypothesis import given, settings, strategies as st
    from llm_message_queue_amd.gateway.shm_bridge import decode_raw
    scan = _native.ingress().scan_message
    leaf = st.none() | st.booleans() | st.integers(-10**20, 10**20) | st.floats() | st.text(max_size=12)
    val = st.recursive(leaf, lambda c: st.lists(c, max_size=3) | st.dictionaries(st.text(max_size=6), c, max_size=3),
                       max_leaves=8)
    typed = st.sampled_from(["id", "user_id", "priority", "metadata", "timeout", "max_retries", "retry_count",
                             "created_at", "scheduled_at", "content", "conversation_id", "status"])
    special = st.sampled_from(["1m", "10ms", "1.5h", "abc", "", "0", "2024-01-31T10:00:00Z", "2023-02-29T00:00:00Z",
                               "urgent", "realtime", "4", " 3 ", "+2", "x\\y", "ok-id"])

    def record(body: bytes) -> bytes:
        return (123).to_bytes(8, "little", signed=True) + b"id-1".ljust(36, b"\0") + \
            len(body).to_bytes(4, "little") + body

    @settings(max_examples=400, deadline=None)
    @given(st.dictionaries(typed, val | special, max_size=6), st.booleans())
    def prop(d, ascii_only):
        try:
            body = json.dumps(d, ensure_ascii=ascii_only).encode("utf-8", "surrogatepass")
        except (ValueError, UnicodeEncodeError):
            return
        if scan(body)[0]:
            decode_raw(record(body))            # must not raise

    @settings(max_examples=400, deadline=None)
    @given(st.binary(max_size=120))
    def raw(b):
        if scan(b)[0]:
            decode_raw(record(b))

    prop()
    raw()


def test_undecodable_record_is_dead_lettered_not_dropped(stack):
    """A RAW ring record the dispatcher cannot decode (the scanner let it
    through) is accounted for: failed status, dead-letter queue, metric."""
    from llm_message_queue_amd.gateway.shm_bridge import TAG_RAW
    disp, ing, port = stack
    body = b'{"content": "x", "created_at": "not a time"}'
    rec = (5).to_bytes(8, "little", signed=True) + b"bad-rec-1".ljust(36, b"\0") + len(body).to_bytes(4, "little") + body
    disp.ring.requests.push_many([rec], TAG_RAW)
    t0 = time.time()
    while time.time() - t0 < 5 and disp.messages.get("bad-rec-1") is None:
        time.sleep(0.02)
    m = disp.messages.get("bad-rec-1")
    assert m is not None and m.status == "failed" and "undecodable" in m.metadata["error"]
    assert any(it.message.id == "bad-rec-1" for it in disp.factory.dead_letter_queue.get_all())


def test_slow_reader_does_not_spin_ingress_thread():
    """after a write hit EAGAIN the connection's EPOLLOUT interest
    must be dropped again once the output drained -- otherwise the ingress
    thread busy-polls the idle writable socket for the connection's life."""
    import resource
    name = f"pyt-spin-{os.getpid()}"
    ring = RingPair(name, 1 << 20, "create")
    ing = NativeIngress(0, name, threads=1, host="127.0.0.1")
    port = ing.start()
    try:
        s = socket.create_connection(("127.0.0.1", port))
        s.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 1 << 16)
        req = b"GET /health HTTP/1.1\r\nHost: x\r\n\r\n"
        n = 40000
        s.sendall(req * n)                      # pipelined; responses pile up unread
        time.sleep(0.5)                         # server hits EAGAIN with EPOLLOUT armed
        s.settimeout(10)
        seen, tail = 0, b""
        while seen < n:
            chunk = s.recv(1 << 20)
            if not chunk:
                break
            buf = tail + chunk
            seen += buf.count(b"HTTP/1.1 200")
            tail = buf[-11:]                    # a status line split across reads
            seen -= tail.count(b"HTTP/1.1 200")
        assert seen == n
        time.sleep(0.2)
        c0 = resource.getrusage(resource.RUSAGE_SELF)
        time.sleep(1.0)                         # idle keep-alive connection
        c1 = resource.getrusage(resource.RUSAGE_SELF)
        cpu = (c1.ru_utime - c0.ru_utime) + (c1.ru_stime - c0.ru_stime)
        assert cpu < 0.3, f"ingress burned {cpu:.2f} s CPU on an idle connection"
        s.close()
    finally:
        ing.stop()
        ring.close(unlink=True)


def test_front_door_proxy_is_async_ordered_and_reports_502():
    """The multi-GPU front door reverse-proxies every non-submit route to the
    API server.  The upstream round trip runs on a proxy worker, so a slow
    admin request does not stall other connections of the same epoll thread;
    pipelined requests on one connection are answered in order; an
    unreachable API server is a 502."""
    import http.server
    import socket
    import threading
    import time

    class Slow(http.server.BaseHTTPRequestHandler):
        def do_GET(self):
            if "slow" in self.path:
                time.sleep(1.0)
            body = json.dumps({"path": self.path, "xff": self.headers.get("X-Forwarded-For", "")}).encode()
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    up = http.server.ThreadingHTTPServer(("127.0.0.1", 0), Slow)
    threading.Thread(target=up.serve_forever, daemon=True).start()
    from llm_message_queue_amd.gateway.native_ingress import NativeIngress
    name = f"pytest-proxy-{os.getpid()}"
    ing = NativeIngress(0, name, threads=1, host="127.0.0.1", upstream=("127.0.0.1", up.server_address[1]))
    port = ing.start()
    try:
        res = {}

        def slow():
            t0 = time.time()
            with urllib.request.urlopen(f"http://127.0.0.1:{port}/api/v1/queues/slow", timeout=10) as r:
                res["slow"] = (r.status, json.loads(r.read()), time.time() - t0)

        th = threading.Thread(target=slow)
        th.start()
        time.sleep(0.2)                               # the slow request is with the API server now
        t0 = time.time()
        st, body = _post(port, {"content": "hello", "id": "fast-1"})
        fast_s = time.time() - t0
        th.join()
        assert st == 202 and body["message_id"] == "fast-1"
        assert fast_s < 0.5, fast_s                   # not stuck behind the 1 s upstream answer
        assert res["slow"][0] == 200 and res["slow"][1]["path"] == "/api/v1/queues/slow"
        assert res["slow"][1]["xff"] == "127.0.0.1" and res["slow"][2] >= 0.9
        # pipelining: a proxied request then a native one on ONE connection -> answers in order
        s = socket.create_connection(("127.0.0.1", port), timeout=10)
        body = b'{"content":"x","id":"pipe-2"}'
        s.sendall(b"GET /slow-first HTTP/1.1\r\nHost: x\r\n\r\n"
                  b"POST /api/v1/messages HTTP/1.1\r\nHost: x\r\nContent-Type: application/json\r\n"
                  b"Content-Length: " + str(len(body)).encode() + b"\r\n\r\n" + body)
        data = b""
        t0 = time.time()
        while data.count(b"HTTP/1.") < 2 and time.time() - t0 < 10:
            data += s.recv(65536)
        s.close()
        first, second = data.index(b"/slow-first"), data.index(b"pipe-2")
        assert first < second and data.count(b" 200 OK") == 1 and data.count(b"HTTP/1.1 202") == 1
        st_ = ing.stats()
        assert st_["proxied"] == 2 and st_["proxy_errors"] == 0
    finally:
        ing.stop()
        up.shutdown()
    # an API server that is gone: 502
    dead = socket.socket()
    dead.bind(("127.0.0.1", 0))
    dead_port = dead.getsockname()[1]
    dead.close()
    ing = NativeIngress(0, name, threads=1, host="127.0.0.1", upstream=("127.0.0.1", dead_port))
    port = ing.start()
    try:
        try:
            urllib.request.urlopen(f"http://127.0.0.1:{port}/api/v1/queues/stats", timeout=10)
            assert False, "expected 502"
        except urllib.error.HTTPError as e:
            assert e.code == 502
        assert ing.stats()["proxy_errors"] == 1
    finally:
        ing.stop()
        from llm_message_queue_amd import _native
        _native.shmring().ShmRing(f"llmq-{name}-req", 1 << 20, "open").unlink()
