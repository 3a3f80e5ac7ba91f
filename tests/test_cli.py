"""The command line (reference binaries C18-C21) as real processes: the CPU
monolith over HTTP, config validation, and the autoscaler against it."""
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _get(url):
    with urllib.request.urlopen(url, timeout=5) as r:
        return json.loads(r.read())


def test_validate_config():
    r = subprocess.run([sys.executable, "-m", "llm_message_queue_amd.cli", "validate-config", "--config",
                        os.path.join(ROOT, "configs")], capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert r.returncode == 0 and json.loads(r.stdout.strip().splitlines()[-1])["valid"]
    r = subprocess.run([sys.executable, "-m", "llm_message_queue_amd.cli", "validate-config", "--config",
                        "/nonexistent/dir"], capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert r.returncode == 1


def test_serve_monolith_and_scheduler():
    port, gport = _port(), _port()
    env = dict(os.environ, LLMQ_LOGGING__LEVEL="warning", LLMQ_QUEUE__WORKER__PROCESS_INTERVAL="5ms")
    srv = subprocess.Popen([sys.executable, "-m", "llm_message_queue_amd.cli", "serve", "--no-gpu", "--port",
                            str(port), "--host", "127.0.0.1", "--grpc-port", str(gport)], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                           stderr=subprocess.DEVNULL, text=True, start_new_session=True)
    base = f"http://127.0.0.1:{port}"
    try:
        t0 = time.time()
        while time.time() - t0 < 120:
            try:
                if _get(base + "/health")["status"] == "ok":
                    break
            except Exception:
                time.sleep(0.2)
        body = json.dumps({"content": "EMERGENCY: disk full", "user_id": "cli"}).encode()
        req = urllib.request.Request(base + "/api/v1/messages", data=body, method="POST",
                                     headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=5) as r:
            assert r.status == 202
            mid = json.loads(r.read())["message_id"]
        t0 = time.time()
        while time.time() - t0 < 10 and _get(base + f"/api/v1/messages/{mid}")["status"] != "completed":
            time.sleep(0.05)
        m = _get(base + f"/api/v1/messages/{mid}")
        assert m["status"] == "completed" and m["priority"] == 1
        # the same gateway over gRPC (--grpc-port)
        from llm_message_queue_amd.api.grpc_server import GrpcClient
        g = GrpcClient(f"127.0.0.1:{gport}")
        t0 = time.time()
        while True:
            try:
                assert g.get_message(mid, timeout=2).status == "completed"
                break
            except Exception:
                if time.time() - t0 > 30:
                    raise
                time.sleep(0.2)
        r = g.submit("hello over grpc", user_id="cli")
        assert [x.status for x in g.watch(r.message_id, timeout_ms=10_000)][-1] == "completed"
        g.close()
        # the autoscaler binary against the live gateway: one scheduling round
        sch = subprocess.run([sys.executable, "-m", "llm_message_queue_amd.cli", "scheduler", "--gateway", base,
                              "--iterations", "1"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
        assert sch.returncode == 0 and "error" not in json.loads(sch.stdout.strip().splitlines()[-1])
    finally:
        os.killpg(srv.pid, signal.SIGTERM)
        srv.wait(timeout=30)
    assert srv.returncode == 0
