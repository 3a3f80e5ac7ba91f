"""Job-owned shared-memory segments and fatal stalls.

``torch.distributed.run`` with a static rendezvous gives every launch the run
id ``"none"``, and a ``--max-restarts`` restart keeps the run id, so segment
names built from the run id alone let a new job (or restart incarnation)
re-attach a dead one's rings.  ``cli serve`` now names every segment with a
per-incarnation token (run id + restart count + a nonce rank 0 broadcasts),
creates them on rank 0 stamped with a generation, attaches on the others
after a barrier (refusing any other generation), and drops the names once
every process has mapped them.  A stall that lasts is fatal.
Reference: `cmd/server/main.go:100-118` (process lifecycle)."""
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
import urllib.error
import urllib.request

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _req(method, url, body=None, timeout=10):
    data = json.dumps(body).encode() if body is not None else None
    req = urllib.request.Request(url, data=data, method=method, headers={"Content-Type": "application/json"})
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:
            return r.status, json.loads(r.read() or b"{}")
    except urllib.error.HTTPError as e:
        return e.code, json.loads(e.read() or b"{}")


def _shm_names():
    try:
        return set(os.listdir("/dev/shm"))
    except FileNotFoundError:
        return set()


class Server:
    """A ``cli serve`` process (optionally under torchrun) whose stdout JSON
    events are collected by a reader thread."""

    def __init__(self, args, env_extra=None, torchrun=0, mport=0, restarts=0, standalone=False, gpu=False):
        self.port = _port()
        env = dict(os.environ, LLMQ_LOGGING__LEVEL="warning", OMP_NUM_THREADS="1", **(env_extra or {}))
        mode = ["--model", "tiny"] if gpu else ["--cpu-ranks"]     # gpu: every rank on the visible GPU(s)
        cmd = [sys.executable, "-m", "llm_message_queue_amd.cli", "serve"] + mode + ["--port", str(self.port),
               "--host", "127.0.0.1"] + list(args)
        if torchrun:
            # static rendezvous (run id "none", as the round-4 HTTP runs), or
            # --standalone: the c10d rendezvous deployments use, whose restart
            # rounds re-rendezvous (gloo under a static one can read the dead
            # incarnation's addresses from the store on restart)
            rdzv = (["--standalone", "--local-addr=127.0.0.1"] if standalone else
                    ["--master-addr=127.0.0.1", f"--master-port={mport or _port()}"])
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={torchrun}"] \
                + rdzv + [f"--max-restarts={restarts}"] + cmd[1:]
        self.proc = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                     text=True, start_new_session=True)
        self.events, self.err = [], []
        self._cv = threading.Condition()
        threading.Thread(target=self._read, args=(self.proc.stdout, True), daemon=True).start()
        threading.Thread(target=self._read, args=(self.proc.stderr, False), daemon=True).start()
        self.base = f"http://127.0.0.1:{self.port}"

    def _read(self, f, out):
        for line in f:
            if not out:
                self.err.append(line)
                continue
            if line.startswith("{"):
                try:
                    ev = json.loads(line)
                except ValueError:
                    continue
                with self._cv:
                    self.events.append(ev)
                    self._cv.notify_all()

    def wait_for(self, pred, timeout=180):
        deadline = time.time() + timeout
        with self._cv:
            while time.time() < deadline:
                got = [e for e in self.events if pred(e)]
                if got:
                    return got
                if self.proc.poll() is not None:
                    break
                self._cv.wait(0.5)
        tail = "".join(self.err[-120:])
        raise AssertionError(f"server event not seen (rc={self.proc.poll()}); stderr tail:\n{tail}")

    def ranks(self, n, restart=0, timeout=180):
        def pred(e):
            return e.get("event") == "rank" and e.get("restart", 0) == restart
        deadline = time.time() + timeout
        while True:
            got = self.wait_for(pred, max(1, deadline - time.time()))
            if len({e["rank"] for e in got}) >= n or time.time() > deadline:
                return sorted(got, key=lambda e: e["rank"])
            time.sleep(0.2)

    def post_all(self, n, tag):
        ids = []
        for i in range(n):
            st, r = _req("POST", self.base + "/api/v1/messages", {"content": f"job test {tag} {i}", "user_id": f"u{i}"})
            assert st == 202, r
            ids.append(r["message_id"])
        return ids

    def wait_completed(self, ids, timeout=120):
        deadline = time.time() + timeout
        done = set()
        while time.time() < deadline and len(done) < len(ids):
            for mid in ids:
                if mid not in done:
                    st, m = _req("GET", self.base + f"/api/v1/messages/{mid}")
                    if st == 200 and m.get("status") == "completed":
                        done.add(mid)
            time.sleep(0.2)
        return len(done)

    def stop(self, sig=signal.SIGTERM):
        # torchrun's workers run in sessions of their own: signal them by pid
        # too (a SIGKILL of the launcher alone would leave them running)
        pids = {int(e["pid"]) for e in self.events if e.get("event") == "rank" and "pid" in e}
        if sig == signal.SIGKILL:
            for pid in pids:
                try:
                    os.kill(pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
        try:
            os.killpg(self.proc.pid, sig)
            self.proc.wait(timeout=60)
        except Exception:
            try:
                os.killpg(self.proc.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            self.proc.wait(timeout=10)
        deadline = time.time() + 30
        for pid in pids:                               # nothing of the job outlives the test
            while time.time() < deadline:
                try:
                    os.kill(pid, 0)
                except ProcessLookupError:
                    break
                time.sleep(0.2)
            else:
                try:
                    os.kill(pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass


def test_ring_generation_refuses_a_stale_segment():
    """``ShmRing`` generation: "create" stamps it; "attach" and "open" refuse
    a segment of another generation, so a restarted incarnation can never
    drain a dead one's records or inherit its balanced-share ledger."""
    from llm_message_queue_amd import _native
    R = _native.shmring().ShmRing
    name = f"llmq-gentest-{os.getpid()}"
    old = R(name, 1 << 16, "create", 11)
    try:
        assert old.push(b"left over by a dead incarnation", 3)
        assert old.generation == 11 and old.creator_pid == os.getpid()
        with pytest.raises(RuntimeError, match="stale"):
            R(name, 0, "attach", 22)
        with pytest.raises(RuntimeError, match="stale"):
            R(name, 1 << 16, "open", 22)
        assert R(name, 0, "attach", 11).size() == 1          # the right generation attaches
        assert R(name, 0, "attach", 0).size() == 1           # gen 0: no check (split deployment)
        new = R(name, 1 << 16, "create", 22)                 # a new incarnation replaces it
        assert new.generation == 22 and new.size() == 0
        assert R(name, 0, "attach", 22).size() == 0
    finally:
        R(name, 1 << 12, "open", 0).unlink()


def test_job_token_unique_per_incarnation(monkeypatch):
    """Every launch (even under the same static rendezvous) and every restart
    gets its own token; all ranks of one job share rank 0's nonce."""
    from llm_message_queue_amd.parallel.comm import FakeComm, job_token
    monkeypatch.setenv("TORCHELASTIC_RUN_ID", "none")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    t1, g1 = job_token()
    t2, g2 = job_token()
    assert t1 != t2 and g1 != g2 and t1.startswith("none.0.") and g1 > 0
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    assert job_token()[0].startswith("none.1.")
    comms = FakeComm.make(3, timeout_s=10)
    out = [None] * 3

    def run(r):
        out[r] = job_token(comms[r])
    ths = [threading.Thread(target=run, args=(r,)) for r in range(3)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(10)
    assert out[0] == out[1] == out[2] and out[0][0].startswith("none.1.")


def test_sigkilled_job_leaves_nothing_and_next_job_completes_every_request():
    """SIGKILL a one-rank ``cli serve`` with requests in flight, then start a
    two-rank job under the same static rendezvous (run id "none", same master
    port): the killed job left no segment in /dev/shm, the new job's token
    differs, a stale ring under the round-4 naming is never drained, and
    every request of the new job completes (the round-4 stalls followed a
    one-rank run in the same call)."""
    from llm_message_queue_amd import _native
    before = _shm_names()
    mport = _port()
    a = Server([], torchrun=1, mport=mport)
    try:
        ra = a.ranks(1)
        a.wait_for(lambda e: e.get("event") == "listening")
        tok_a = ra[0]["job"]
        assert tok_a.startswith("none.0.")
        assert any(tok_a in n for n in _shm_names() - before) is False   # names dropped once mapped
        a.post_all(60, "a")
    finally:
        a.stop(signal.SIGKILL)
    leaked = [n for n in _shm_names() - before if tok_a in n]
    assert leaked == [], leaked
    assert a.proc.poll() is not None
    # a stale ring under the round-4 name (run id only) with a leftover record
    R = _native.shmring().ShmRing
    stale = R("llmq-default-none-req", 1 << 16, "open", 0)
    stale.push(b"\x00" * 48, 3)
    try:
        b = Server([], torchrun=2, mport=mport)
        try:
            rb = b.ranks(2)
            b.wait_for(lambda e: e.get("event") == "listening")
            assert rb[0]["job"] == rb[1]["job"] != tok_a
            ids = b.post_all(40, "b")
            assert b.wait_completed(ids) == len(ids)
            assert stale.size() == 1                         # never drained by the new job
        finally:
            b.stop()
    finally:
        stale.unlink()
    assert not [n for n in _shm_names() - before if rb[0]["job"] in n]


def _restart_after_peer_lost(standalone, gpu=False):
    env = {"LLMQ_SERVER__FAULT_INJECTION": "true", "LLMQ_COLLECTIVE_TIMEOUT_S": "4",
           "LLMQ_SERVER__STALL_FATAL_AFTER": "0", "LLMQ_FATAL_EXIT_GRACE_S": "5"}
    s = Server([], env_extra=env, torchrun=2, restarts=1, standalone=standalone, gpu=gpu)
    try:
        r0 = s.ranks(2, restart=0)
        s.wait_for(lambda e: e.get("event") == "listening")
        st, r = _req("POST", s.base + "/api/v1/admin/faults", {"slow_ms": 20000})
        assert st == 200 and r["faults"] == {"slow_ms": 20000}, r
        s.post_all(5, "x")
        r1 = s.ranks(2, restart=1, timeout=240)
        run0, rs0, n0 = r0[0]["job"].split(".")
        run1, rs1, n1 = r1[0]["job"].split(".")
        assert r1[0]["job"] == r1[1]["job"] and (rs0, rs1) == ("0", "1") and n1 != n0
        fatal = [e for e in s.events if e.get("event") == "fatal"]
        assert fatal and any("control" in e["error"] or "did not reach" in e["error"] or "rank" in e["error"]
                             for e in fatal), fatal
        deadline = time.time() + 60
        while time.time() < deadline:                       # the new rank 0's front door is up
            try:
                if _req("GET", s.base + "/health", timeout=2)[0] == 200:
                    break
            except OSError:
                pass
            time.sleep(0.5)
        ids = s.post_all(30, "y")
        assert s.wait_completed(ids) == len(ids)
    finally:
        s.stop()


@pytest.mark.parametrize("standalone", [True, False])
def test_restart_after_peer_lost_gets_a_fresh_incarnation(standalone):
    """``torchrun --max-restarts 1``: rank 0's backend stalls (injected), so
    rank 1 loses its peer at the control-plane collective (``PeerLost``) and
    exits non-zero; torchrun restarts the group.  The new incarnation has its
    own token (restart count 1, new nonce) -- it does not see the old rings --
    and serves every request."""
    _restart_after_peer_lost(standalone)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_restart_after_peer_lost_on_gpu():
    """The same restart with GPU backends: two ranks of ``cli serve --model
    tiny`` on the box's GPU (time-sharing it; the data plane falls back to
    gloo when ranks share a device), the stalled HIP engine, PeerLost, a
    torchrun restart, and the new incarnation serving every request on the
    GPU."""
    _restart_after_peer_lost(True, gpu=True)


def test_forced_stall_reports_503_then_exits_nonzero():
    """A serve loop that stops ticking while requests wait: ``/health``
    answers 503 (the C++ front door's too) from ``server.stall_dump_after``
    on, and at ``server.stall_fatal_after`` the process exits with status 3
    so a launcher replaces it -- it no longer looks alive forever."""
    env = {"LLMQ_SERVER__FAULT_INJECTION": "true", "LLMQ_SERVER__STALL_DUMP_AFTER": "1s",
           "LLMQ_SERVER__STALL_FATAL_AFTER": "5s", "LLMQ_FATAL_EXIT_GRACE_S": "5"}
    s = Server([], env_extra=env)
    try:
        s.wait_for(lambda e: e.get("event") == "listening")
        assert _req("GET", s.base + "/health")[0] == 200
        st, r = _req("POST", s.base + "/api/v1/admin/faults", {"slow_ms": 60000})
        assert st == 200, r
        s.post_all(3, "stall")
        t0 = time.time()
        code = None
        while time.time() - t0 < 20:
            st, body = _req("GET", s.base + "/health", timeout=3)
            if st == 503:
                code = st
                break
            time.sleep(0.2)
        assert code == 503 and "stalled" in body.get("reason", ""), body
        rc = s.proc.wait(timeout=40)
        assert rc == 3, (rc, "".join(s.err[-30:]))
        assert any(e.get("event") == "fatal" and "stall_fatal_after" in e["error"] for e in s.events)
    finally:
        if s.proc.poll() is None:
            s.stop(signal.SIGKILL)


def test_fault_injection_is_off_by_default():
    from fastapi.testclient import TestClient
    from llm_message_queue_amd.api.server import create_app
    from llm_message_queue_amd.gateway.app import GatewayApp
    from llm_message_queue_amd.utils.config import default_config
    cfg = default_config()
    cfg.queue.enable_metrics = False
    app = GatewayApp(cfg, use_gpu=False, start=False)
    try:
        c = TestClient(create_app(app))
        assert c.post("/api/v1/admin/faults", json={"slow_ms": 5}).status_code == 403
        cfg.server.fault_injection = True
        assert c.post("/api/v1/admin/faults", json={"slow_ms": 5}).status_code == 409   # no backend here
    finally:
        app.stop()


def test_ranks_exit_when_their_launcher_dies():
    """torchrun's workers run in sessions of their own, so SIGKILLing the
    launcher used to leave the ranks serving (holding GPU and port) forever;
    a rank now notices its launcher is gone and stops."""
    s = Server([], torchrun=2)
    try:
        rk = s.ranks(2)
        s.wait_for(lambda e: e.get("event") == "listening")
        os.killpg(s.proc.pid, signal.SIGKILL)              # the launcher only
        s.proc.wait(timeout=10)
        deadline = time.time() + 40
        alive = {int(e["pid"]) for e in rk}
        while alive and time.time() < deadline:
            for pid in list(alive):
                try:
                    os.kill(pid, 0)
                except ProcessLookupError:
                    alive.discard(pid)
            time.sleep(0.3)
        assert not alive, f"ranks {alive} outlived their launcher"
    finally:
        s.stop(signal.SIGKILL)
