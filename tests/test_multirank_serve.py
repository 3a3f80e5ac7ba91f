"""The multi-GPU `cli serve` front door as real processes (VERDICT r2 missing
#2 / next #3), rehearsed on the CPU: ``torch.distributed.run`` starts 2 ranks
of ``cli serve --cpu-ranks`` (tiny reference-op engines, gloo data plane,
shared-memory control plane).  Rank 0's C++ front door takes
``POST /api/v1/messages`` into the ring BOTH ranks drain, routes
conversation turns to rank 0, and reverse-proxies every other route to rank
0's API server, which answers status queries for messages either rank
popped.  Reference: one process serves every route
(`cmd/server/main.go:100-106`, `api/handlers.go:160-219`)."""
import json
import os
import signal
import socket
import subprocess
import sys
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


def test_two_rank_serve_native_front_door():
    port, mport, gport = _port(), _port(), _port()
    env = dict(os.environ, LLMQ_LOGGING__LEVEL="warning", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={mport}", "-m", "llm_message_queue_amd.cli", "serve",
           "--cpu-ranks", "--port", str(port), "--host", "127.0.0.1", "--grpc-port", str(gport)]
    srv = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                           start_new_session=True)
    base = f"http://127.0.0.1:{port}"
    try:
        ev = None
        t0 = time.time()
        while time.time() - t0 < 180:
            line = srv.stdout.readline()
            if not line:
                if srv.poll() is not None:
                    break
                continue
            if line.startswith("{") and '"listening"' in line:
                ev = json.loads(line)
                break
        assert ev is not None, srv.stderr.read()[-3000:] if srv.poll() is not None else "no listening line"
        assert ev["front_door"] == "native" and ev["world"] == 2 and ev["port"] == port
        assert ev["api_port"] != port
        # health on the native path, a proxied GET on the API server behind it
        assert _req("GET", base + "/health")[0] == 200
        st, body = _req("GET", base + "/api/v1/queues/stats")
        assert st == 200 and "dispatch" in body
        # a conversation (proxied POST) and a turn of it through the hot path
        st, conv = _req("POST", base + "/api/v1/conversations", {"user_id": "u1"})
        assert st == 201
        cid = conv["conversation_id"]
        # admin changes on rank 0's API reach the preprocessor of EVERY rank
        # (each preprocesses what it pops): a keyword rule and a user default
        st, r = _req("POST", base + "/api/v1/admin/preprocessor/rules", {"pattern": "(?i)zebra", "priority": 1})
        assert st == 201, r
        st, r = _req("POST", base + "/api/v1/admin/preprocessor/user-priorities", {"user_id": "u3", "priority": "low"})
        assert st == 200, r
        ids = []
        for burst in range(6):
            for i in range(10):
                st, r = _req("POST", base + "/api/v1/messages",
                             {"content": f"please summarise the Zebra report {burst}-{i}", "user_id": f"u{i}"})
                assert st == 202, r
                ids.append(r["message_id"])
            time.sleep(0.05)
        st, r = _req("POST", base + "/api/v1/messages",
                     {"content": "what did we decide?", "user_id": "u1", "conversation_id": cid})
        assert st == 202
        turn = r["message_id"]
        # every message completes and is addressable through rank 0's API,
        # whichever rank popped it
        deadline = time.time() + 120
        done = {}
        while time.time() < deadline and len(done) < len(ids) + 1:
            for mid in ids + [turn]:
                if mid in done:
                    continue
                st, m = _req("GET", base + f"/api/v1/messages/{mid}")
                if st == 200 and m["status"] == "completed":
                    done[mid] = m
            time.sleep(0.2)
        assert len(done) == len(ids) + 1, f"{len(done)} of {len(ids) + 1} completed"
        ranks = {m["metadata"].get("ingest_rank") for m in done.values()}
        assert ranks == {0, 1}, ranks                        # ingest spread over both ranks
        # ... evenly: the ring threads drain with the balanced share (ADVICE
        # r4: nothing end to end pinned the split).  The 60 plain messages come
        # through the shared ring; the turn through rank 0's conversation ring
        n_by = [sum(1 for mid in ids if done[mid]["metadata"].get("ingest_rank") == r) for r in (0, 1)]
        assert max(n_by) <= 1.5 * min(n_by) + 8, n_by
        for mid in ids:                                      # ... and both applied the admin rules
            m = done[mid]
            want = (4, "user_default") if m["user_id"] == "u3" else (1, "content_keywords")
            assert (m["priority"], m["metadata"].get("priority_reason")) == want, m
        assert done[turn]["metadata"]["ingest_rank"] == 0    # conversation turns go to rank 0
        st, c = _req("GET", base + f"/api/v1/conversations/{cid}")
        assert st == 200 and any(m["id"] == turn for m in c.get("messages", [])), c
        # list spans both ranks
        st, lst = _req("GET", base + "/api/v1/messages?limit=200")
        assert st == 200 and lst["total"] >= len(ids) + 1
        assert _req("GET", base + "/api/v1/messages/does-not-exist")[0] == 404
        # one Prometheus scrape covers every rank (a `rank` label per sample)
        with urllib.request.urlopen(base + "/metrics", timeout=10) as resp:
            prom = resp.read().decode()
        from prometheus_client.parser import text_string_to_metric_families
        fams = {f.name: f for f in text_string_to_metric_families(prom)}
        done_by_rank = {}
        for smp in fams["llm_queue_messages_completed"].samples:
            if smp.name.endswith("_total"):
                done_by_rank[smp.labels["rank"]] = done_by_rank.get(smp.labels["rank"], 0) + smp.value
        assert set(done_by_rank) == {"0", "1"} and sum(done_by_rank.values()) >= len(ids), done_by_rank
        # gRPC on rank 0 sees the whole job too: a message rank 1 popped, and
        # tier counters summed over both ranks
        from llm_message_queue_amd.api.grpc_server import GrpcClient
        gcli = GrpcClient(f"127.0.0.1:{gport}")
        try:
            on_rank1 = next(mid for mid, m in done.items() if m["metadata"].get("ingest_rank") == 1)
            info = gcli.get_message(on_rank1)
            assert info.id == on_rank1 and info.status == "completed"
            st_rep = gcli.queue_stats()
            assert sum(t.completed for t in st_rep.tiers) >= len(ids)
        finally:
            gcli.close()
        # dead letters live on the rank that popped the request: the admin
        # routes on rank 0 list / remove / requeue them job-wide
        exp = []
        for burst in range(4):
            for i in range(10):
                st, r = _req("POST", base + "/api/v1/messages", {"content": f"late {burst}-{i}", "timeout": "1us"})
                assert st == 202, r
                exp.append(r["message_id"])
            time.sleep(0.05)
        deadline = time.time() + 60
        items = []
        while time.time() < deadline:
            st, d = _req("GET", base + "/api/v1/admin/dead-letter")
            items = [it for it in d["items"] if it["message"]["id"] in exp]
            if len(items) == len(exp):
                break
            time.sleep(0.2)
        assert len(items) == len(exp), f"{len(items)} of {len(exp)} dead-lettered"
        assert {it["rank"] for it in items} == {0, 1}
        on1 = [it["message"]["id"] for it in items if it["rank"] == 1]
        st, qs = _req("GET", base + "/api/v1/queues/status")
        assert st == 200 and qs["job"]["dead_letter"] >= len(exp)
        # every rank's serve-loop profile (host ms per tick, collective wait,
        # stage breakdown) rides in the job stats
        st, js = _req("GET", base + "/api/v1/queues/stats")
        prof = js["job"]["profile_by_rank"]
        assert sorted(int(r) for r in prof) == [0, 1], prof
        for p_ in prof.values():
            assert p_["ticks"] > 0 and "launch" in p_["host_ms_per_tick"] and "p99_ms" in p_["collective"]
            assert set(p_["latency_breakdown"]) >= {"ingress", "queue", "handoff", "admitted_by_path"}
        assert _req("DELETE", base + f"/api/v1/admin/queues/dead_letter/{on1[0]}")[0] == 200
        assert _req("DELETE", base + f"/api/v1/admin/queues/dead_letter/{on1[0]}")[0] == 404
        assert _req("POST", base + f"/api/v1/admin/dead-letter/requeue/{on1[1]}")[0] == 200
        assert _req("POST", base + "/api/v1/admin/dead-letter/requeue/nope")[0] == 404
        st, r = _req("POST", base + "/api/v1/admin/dead-letter/requeue-all")
        assert st == 200 and r["count"] >= len(exp) - 3, r
    finally:
        try:
            os.killpg(srv.pid, signal.SIGTERM)
            srv.wait(timeout=60)
        except Exception:
            os.killpg(srv.pid, signal.SIGKILL)
            srv.wait(timeout=10)


@pytest.mark.gpu
def test_two_rank_serve_front_door_on_gpu():
    """The same topology with GPU engines (tiny Llama-shaped model on the HIP
    kernels, both ranks on the one MI355X of the box -- gloo between them):
    HTTP POSTs through the C++ front door complete on the GPU backends and
    every message is addressable from rank 0's API."""
    port, mport = _port(), _port()
    env = dict(os.environ, LLMQ_LOGGING__LEVEL="warning", LLMQ_GPU__SLOTS_PER_GPU="64",
               LLMQ_BACKEND__TOKEN_BUDGET="512")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={mport}", "-m", "llm_message_queue_amd.cli", "serve",
           "--model", "tiny", "--port", str(port), "--host", "127.0.0.1"]
    srv = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           start_new_session=True)
    base = f"http://127.0.0.1:{port}"
    try:
        ev = None
        t0 = time.time()
        while time.time() - t0 < 240:
            line = srv.stdout.readline()
            if not line:
                if srv.poll() is not None:
                    break
                continue
            if line.startswith("{") and '"listening"' in line:
                ev = json.loads(line)
                break
        assert ev is not None and ev["gpu"] and ev["front_door"] == "native", "server did not come up"
        # a keyword rule added at run time is re-packed into EVERY rank's GPU
        # text-kernel pattern table (each rank preprocesses what it pops)
        st, r = _req("POST", base + "/api/v1/admin/preprocessor/rules", {"pattern": "(?i)zebra", "priority": 4})
        assert st == 201, r
        ids = []
        for i in range(40):
            st, r = _req("POST", base + "/api/v1/messages", {"content": f"zebra zebra: check node {i}",
                                                             "user_id": f"g{i % 5}"})
            assert st == 202, r
            ids.append(r["message_id"])
        deadline = time.time() + 120
        done = {}
        while time.time() < deadline and len(done) < len(ids):
            for mid in ids:
                if mid not in done:
                    st, m = _req("GET", base + f"/api/v1/messages/{mid}")
                    if st == 200 and m["status"] == "completed":
                        done[mid] = m
            time.sleep(0.1)
        assert len(done) == len(ids), f"{len(done)} of {len(ids)} completed"
        assert all((m["priority"], m["metadata"].get("priority_reason")) == (4, "content_keywords")
                   for m in done.values()), [m["priority"] for m in done.values()]
        st, stats = _req("GET", base + "/api/v1/queues/stats")
        assert st == 200 and stats["job"]["ranks"] == [0, 1]
        assert stats["job"]["dispatch"]["completed"] >= len(ids)
    finally:
        try:
            os.killpg(srv.pid, signal.SIGTERM)
            srv.wait(timeout=60)
        except Exception:
            os.killpg(srv.pid, signal.SIGKILL)
            srv.wait(timeout=10)


def test_single_rank_serve_native_front_door():
    """``cli serve`` without a launcher (one backend) is fronted by the C++
    ingress too: POST /api/v1/messages never touches the Python ASGI stack
    (~2k req/s), every other route is proxied to the API server behind it."""
    port = _port()
    env = dict(os.environ, LLMQ_LOGGING__LEVEL="warning", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    cmd = [sys.executable, "-m", "llm_message_queue_amd.cli", "serve", "--cpu-ranks", "--port", str(port),
           "--host", "127.0.0.1"]
    srv = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                           start_new_session=True)
    base = f"http://127.0.0.1:{port}"
    try:
        ev = None
        t0 = time.time()
        while time.time() - t0 < 120:
            line = srv.stdout.readline()
            if not line:
                if srv.poll() is not None:
                    break
                continue
            if line.startswith("{") and '"listening"' in line:
                ev = json.loads(line)
                break
        assert ev is not None, srv.stderr.read()[-3000:] if srv.poll() is not None else "no listening line"
        assert ev["front_door"] == "native" and ev["world"] == 1 and ev["port"] == port and ev["api_port"] != port
        st, conv = _req("POST", base + "/api/v1/conversations", {"user_id": "solo"})
        assert st == 201
        ids = []
        for i in range(30):
            st, r = _req("POST", base + "/api/v1/messages", {"content": f"urgent: ping {i}", "user_id": f"u{i % 3}"})
            assert st == 202, r
            ids.append(r["message_id"])
        st, r = _req("POST", base + "/api/v1/messages", {"content": "and then?", "user_id": "solo",
                                                         "conversation_id": conv["conversation_id"]})
        assert st == 202
        ids.append(r["message_id"])
        deadline = time.time() + 60
        done = set()
        while time.time() < deadline and len(done) < len(ids):
            for mid in ids:
                if mid not in done:
                    st, m = _req("GET", base + f"/api/v1/messages/{mid}")
                    if st == 200 and m["status"] == "completed":
                        done.add(mid)
            time.sleep(0.1)
        assert len(done) == len(ids)
        st, c = _req("GET", base + f"/api/v1/conversations/{conv['conversation_id']}")
        assert st == 200 and any(m["id"] == ids[-1] for m in c.get("messages", []))
    finally:
        try:
            os.killpg(srv.pid, signal.SIGTERM)
            srv.wait(timeout=60)
        except Exception:
            os.killpg(srv.pid, signal.SIGKILL)
            srv.wait(timeout=10)


def _wait_listening(proc, timeout=180):
    t0 = time.time()
    while time.time() - t0 < timeout:
        line = proc.stdout.readline()
        if not line:
            if proc.poll() is not None:
                return None
            continue
        if line.startswith("{") and '"listening"' in line:
            return json.loads(line)
    return None


def test_split_deployment_two_queue_manager_ranks():
    """The documented split deployment (docs/deployment.md): ``queue-manager``
    under torchrun (here 2 CPU ranks) drains ONE shared request ring that an
    ``api-gateway`` process fills; every rank pushes status events back
    through the event ring, so the gateway that accepted a message reports it
    completed whichever rank served it."""
    ring = f"splittest{os.getpid()}"
    qport, gport, mport = _port(), _port(), _port()
    env = dict(os.environ, LLMQ_LOGGING__LEVEL="warning", OMP_NUM_THREADS="1")
    qm = subprocess.Popen([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                           "--master-addr=127.0.0.1", f"--master-port={mport}", "-m", "llm_message_queue_amd.cli",
                           "queue-manager", "--cpu-ranks", "--ring", ring, "--port", str(qport), "--host",
                           "127.0.0.1"], cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                          text=True, start_new_session=True)
    gw = None
    try:
        ev = _wait_listening(qm)
        assert ev is not None and ev["world"] == 2, qm.stderr.read()[-3000:] if qm.poll() is not None else ev
        gw = subprocess.Popen([sys.executable, "-m", "llm_message_queue_amd.cli", "api-gateway", "--no-gpu",
                               "--ring", ring, "--port", str(gport), "--host", "127.0.0.1"], cwd=ROOT, env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
        assert _wait_listening(gw) is not None, gw.stderr.read()[-3000:] if gw.poll() is not None else "no gw"
        base = f"http://127.0.0.1:{gport}"
        ids = []
        for i in range(40):
            st, r = _req("POST", base + "/api/v1/messages", {"content": f"please check item {i}", "user_id": f"s{i}"})
            assert st == 202, r
            # the reference api-gateway's reply fields ride along (cmd/api-gateway/main.go:113)
            assert r["message"] == "Message accepted" and r["id"] == r["message_id"], r
            ids.append(r["message_id"])
        deadline = time.time() + 90
        done = set()
        while time.time() < deadline and len(done) < len(ids):
            for mid in ids:
                if mid not in done:
                    st, m = _req("GET", base + f"/api/v1/messages/{mid}")
                    if st == 200 and m["status"] == "completed":
                        done.add(mid)
            time.sleep(0.2)
        assert len(done) == len(ids), f"{len(done)} of {len(ids)} completed"
        st, stats = _req("GET", f"http://127.0.0.1:{qport}/api/v1/queues/stats")
        assert st == 200 and stats["dispatch"]["completed"] > 0       # rank 0's own share
        # ... and rank 0's API sees the whole queue-manager job through the peer channel
        assert stats["job"]["ranks"] == [0, 1] and stats["job"]["dispatch"]["completed"] >= len(ids), stats["job"]
    finally:
        for p in (gw, qm):
            if p is None:
                continue
            try:
                os.killpg(p.pid, signal.SIGTERM)
                p.wait(timeout=60)
            except Exception:
                os.killpg(p.pid, signal.SIGKILL)
                p.wait(timeout=10)
