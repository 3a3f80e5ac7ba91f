"""HTTP-level load test of the REST API (the reference's doc-only k6 / Go
load tests, `docs/performance.md:1039-1155`: p99 < 500 ms, error rate < 10%;
>= 900 RPS of a 1,000 RPS target with 100 workers).

Open-loop Poisson arrivals of ``POST /api/v1/messages`` (4-tier content mix)
from ``--procs`` client processes, each an aiohttp event loop.  Either starts
the server itself (``--spawn serve|split``) or targets ``--url``.

    python bench/http_load.py --spawn serve --rate 2000 --duration 10
    python bench/http_load.py --spawn split --ingress 4 --rate 8000 --duration 10
    python bench/http_load.py --url http://127.0.0.1:8080 --rate 1000
"""
from __future__ import annotations

import argparse
import asyncio
import json
import multiprocessing as mp
import os
import random
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BODIES = [
    {"content": "EMERGENCY: the payment service is down right now", "user_id": "rt"},
    {"content": "urgent: please review the deploy before noon", "user_id": "hi"},
    {"content": "can you summarise the meeting notes for the team?", "user_id": "n"},
    {"content": "background batch job report", "user_id": "lo", "priority": "low"},
]
MIX = [0.1, 0.3, 0.4, 0.2]


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


async def _client(urls, rate, duration, seed, out):
    import aiohttp
    rng = random.Random(seed)
    lat, codes = [], {}
    conn = aiohttp.TCPConnector(limit=0)
    async with aiohttp.ClientSession(connector=conn) as sess:
        tasks = []

        async def one(body, url):
            t0 = time.perf_counter()
            try:
                async with sess.post(url + "/api/v1/messages", json=body) as r:
                    await r.read()
                    codes[r.status] = codes.get(r.status, 0) + 1
            except Exception:
                codes["err"] = codes.get("err", 0) + 1
            lat.append(time.perf_counter() - t0)

        t_end = time.perf_counter() + duration
        t_next = time.perf_counter()
        k = 0
        while True:
            now = time.perf_counter()
            if now >= t_end:
                break
            while t_next <= now:
                body = dict(rng.choices(BODIES, MIX)[0])
                tasks.append(asyncio.ensure_future(one(body, urls[k % len(urls)])))
                k += 1
                t_next += rng.expovariate(rate)
            await asyncio.sleep(max(0.0, min(t_next - time.perf_counter(), 0.01)))
        if tasks:
            await asyncio.wait(tasks, timeout=30)
    out.put({"sent": k, "codes": codes, "lat": lat})


def _client_proc(urls, rate, duration, seed, out):
    asyncio.run(_client(urls, rate, duration, seed, out))


def _wait_up(url, timeout=120.0):
    import urllib.request
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            with urllib.request.urlopen(url + "/health", timeout=1) as r:
                if r.status == 200:
                    return True
        except Exception:
            time.sleep(0.2)
    return False


def _bench_config_file(slots: int = 1536) -> str:
    """configs/config.yaml plus the serving settings bench.py measures."""
    import yaml
    with open(os.path.join(ROOT, "configs", "config.yaml")) as fh:
        c = yaml.safe_load(fh)
    for lv, ms in zip(sorted(c["queue"]["levels"], key=lambda x: x["priority"]), (50, 100, 150, 200)):
        lv["max_concurrent"] = slots * 8
        lv["max_wait_time"] = f"{ms}ms"
    c.setdefault("gpu", {})["slots_per_gpu"] = slots
    c.setdefault("backend", {}).update({"token_budget": 4096, "max_ctx": 512, "prompt_tokens": 32, "gen_tokens": 4})
    c.setdefault("logging", {})["level"] = "warning"
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"llmq_bench_config_{os.getpid()}.yaml")
    with open(path, "w") as fh:
        yaml.safe_dump(c, fh)
    return path


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--url", default="")
    ap.add_argument("--spawn", choices=["", "serve", "split", "native", "multirank"], default="",
                    help="multirank: torch.distributed.run --nproc-per-node RANKS cli serve (C++ front door on "
                         "rank 0, every rank drains the shared ring; --gpu: ranks wrap onto the visible GPUs)")
    ap.add_argument("--ranks", type=int, default=2, help="multirank: serving ranks")
    ap.add_argument("--sim-gpu", default="",
                    help="multirank on CPU: per-rank relative GPU speeds (each rank a SimEngine at the serving "
                         "config) -- the front door at the 8-GPU request rate without GPUs")
    ap.add_argument("--server-log", default="", help="file for the spawned server's stdout+stderr")
    ap.add_argument("--slots", type=int, default=1536, help="--bench-config: batch slots per rank")
    ap.add_argument("--threads", type=int, default=4, help="native ingress threads")
    ap.add_argument("--ingress", type=int, default=2, help="api-gateway processes (split)")
    ap.add_argument("--gpu", action="store_true", help="spawned server uses the GPU")
    ap.add_argument("--rate", type=float, default=1000.0, help="offered requests/s (total)")
    ap.add_argument("--duration", type=float, default=10.0)
    ap.add_argument("--procs", type=int, default=2, help="client processes (python client) / threads (native)")
    ap.add_argument("--client", choices=["python", "native"], default="python",
                    help="native = csrc/tools/http_bench.cpp (open-loop, keep-alive, no coordinated omission)")
    ap.add_argument("--conns", type=int, default=16, help="native client: connections per thread")
    ap.add_argument("--rss-every", type=float, default=10.0,
                    help="seconds between server RSS samples over the measured run (native client)")
    ap.add_argument("--warmup", type=float, default=0.0,
                    help="seconds of load before the measured window (the dispatcher's latency window is reset "
                         "after it)")
    ap.add_argument("--workload", action="store_true",
                    help="native client sends bench.py's synthetic 4-tier workload (gateway/workload.py) instead "
                         "of four fixed bodies")
    ap.add_argument("--admin-churn", type=float, default=0.0,
                    help="every this many seconds of the measured run: add + remove a keyword rule (copied to "
                         "every rank), scrape /metrics, list dead letters, read /queues/status; reports their "
                         "latencies and errors")
    ap.add_argument("--cancel-churn", type=float, default=0.0,
                    help="per second during the measured run: POST a message through the front door, wait 0-60 ms "
                         "(it may be in the ring, a rank's inbox, its tier queue or on a GPU by then) and DELETE it; "
                         "reports the DELETE outcomes and the job's request accounting after the drain")
    ap.add_argument("--dialog-frac", type=float, default=0.0,
                    help="--workload: this fraction of the bodies are turns of --dialog-convs conversations "
                         "(conversation_id set: KV residency, affinity, history replay / migration across ranks)")
    ap.add_argument("--dialog-convs", type=int, default=2000)
    ap.add_argument("--timeout-frac", type=float, default=0.0,
                    help="--workload: this fraction of the bodies carry a short processing timeout "
                         "(--timeout-val, Go duration) and max_retries 2: in-flight timeouts, retry backoff "
                         "in the DelayedQueue, dead-lettering")
    ap.add_argument("--timeout-val", default="150ms")
    ap.add_argument("--fault-cycle", type=float, default=0.0,
                    help="every this many seconds of the measured run: inject a failed launch into rank 0's GPU "
                         "backend (it evacuates; its requests re-route to the other ranks), then half a cycle "
                         "later set its endpoint healthy again (the spawned server runs with fault injection on)")
    ap.add_argument("--bench-config", action="store_true",
                    help="spawned GPU dispatcher runs bench.py's serving config (1536 slots, 4096-token steps, "
                         "32-token prompts, 4 generated tokens, tier caps = slots, aging 50/100/150/200 ms)")
    a = ap.parse_args()
    procs, urls = [], []
    slog = open(a.server_log, "w") if a.server_log else subprocess.DEVNULL
    api_url = ""
    env = dict(os.environ, PYTHONUNBUFFERED="1", LLMQ_LOGGING__LEVEL="warning", LLMQ_SERVER__MODE="release",
               LLMQ_QUEUE__WORKER__MAX_CONCURRENT="512", LLMQ_QUEUE__WORKER__MAX_BATCH_SIZE="256",
               LLMQ_QUEUE__WORKER__PROCESS_INTERVAL="5ms")
    if a.fault_cycle > 0:
        env["LLMQ_SERVER__FAULT_INJECTION"] = "true"
    gpu = [] if a.gpu else ["--no-gpu"]
    cfg_args = []
    if a.bench_config:
        cfg_args = ["--config", _bench_config_file(a.slots)]
    try:
        if a.spawn == "serve":
            port = _port()
            procs.append(subprocess.Popen([sys.executable, "-m", "llm_message_queue_amd.cli", "serve", "--port",
                                           str(port), "--host", "127.0.0.1"] + gpu, cwd=ROOT, env=env,
                                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                                          start_new_session=True))
            urls = [f"http://127.0.0.1:{port}"]
        elif a.spawn == "split":
            ring = f"httpload{os.getpid()}"
            procs.append(subprocess.Popen([sys.executable, "-m", "llm_message_queue_amd.cli", "queue-manager",
                                           "--ring", ring, "--port", str(_port())] + gpu, cwd=ROOT, env=env,
                                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                                          start_new_session=True))
            for _ in range(a.ingress):
                port = _port()
                procs.append(subprocess.Popen([sys.executable, "-m", "llm_message_queue_amd.cli", "api-gateway",
                                               "--ring", ring, "--port", str(port), "--host", "127.0.0.1",
                                               "--no-gpu"], cwd=ROOT, env=env, stdout=subprocess.DEVNULL,
                                              stderr=subprocess.DEVNULL, start_new_session=True))
                urls.append(f"http://127.0.0.1:{port}")
        elif a.spawn == "native":
            ring = f"httpload{os.getpid()}"
            api_port = _port()
            api_url = f"http://127.0.0.1:{api_port}"
            procs.append(subprocess.Popen([sys.executable, "-m", "llm_message_queue_amd.cli", "queue-manager",
                                           "--ring", ring, "--port", str(api_port), "--host", "127.0.0.1"]
                                          + gpu + cfg_args,
                                          cwd=ROOT, env=env,
                                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                                          start_new_session=True))
            port = _port()
            procs.append(subprocess.Popen([sys.executable, "-m", "llm_message_queue_amd.cli", "api-gateway",
                                           "--native", "--ring", ring, "--port", str(port), "--host", "127.0.0.1",
                                           "--ingress-threads", str(a.threads)], cwd=ROOT, env=env,
                                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                                          start_new_session=True))
            urls = [f"http://127.0.0.1:{port}"]
        elif a.spawn == "multirank":
            port = _port()
            procs.append(subprocess.Popen([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                                           f"--nproc-per-node={a.ranks}", "--master-addr=127.0.0.1",
                                           f"--master-port={_port()}", "-m", "llm_message_queue_amd.cli", "serve",
                                           "--port", str(port), "--host", "127.0.0.1", "--ingress-threads",
                                           str(a.threads)] + ([] if a.gpu else ["--cpu-ranks"])
                                          + (["--sim-gpu", a.sim_gpu] if a.sim_gpu and not a.gpu else []) + cfg_args,
                                          cwd=ROOT, env=env, stdout=slog, stderr=subprocess.STDOUT,
                                          start_new_session=True))
            urls = [f"http://127.0.0.1:{port}"]
            api_url = urls[0]                    # every other route is proxied by the front door
        else:
            urls = [a.url or "http://127.0.0.1:8080"]
        for u in urls + ([api_url] if api_url else []):
            if not _wait_up(u, timeout=300):
                raise SystemExit(f"server {u} did not come up")
        if a.client == "native":
            exe = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"llmq_http_bench_{os.getpid()}")
            subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", os.path.join(ROOT, "csrc", "tools", "http_bench.cpp"),
                            "-o", exe], check=True)
            host, port = urls[0].split("//")[1].split(":")
            import threading
            import urllib.request
            extra = []
            if a.workload:
                from llm_message_queue_amd.gateway.workload import Workload
                bpath = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"llmq_bodies_{os.getpid()}.jsonl")
                import random
                rnd = random.Random(3)
                with open(bpath, "w") as fh:
                    for m in Workload(seed=7).make(int(a.rate * (a.duration + a.warmup)) + 1000):
                        b = {"content": m.content, "user_id": m.user_id}
                        if m.priority:
                            b["priority"] = m.priority
                        if a.dialog_frac > 0 and rnd.random() < a.dialog_frac:
                            c = rnd.randrange(a.dialog_convs)
                            b["conversation_id"] = f"conv-{c}"
                            b["user_id"] = f"du{c}"
                        if a.timeout_frac > 0 and rnd.random() < a.timeout_frac:
                            b["timeout"] = a.timeout_val
                            b["max_retries"] = 2
                        fh.write(json.dumps(b) + "\n")
                extra = [bpath]
            if a.warmup > 0:
                subprocess.run([exe, host, port, str(a.rate), str(a.warmup), str(a.procs), str(a.conns)] + extra,
                               capture_output=True, text=True, timeout=a.warmup + 60)
            # the measured window: the load keeps running while the
            # dispatcher's latency histograms restart (reset ~1 s in)
            if api_url and a.warmup > 0:
                def _reset():
                    time.sleep(1.0)
                    req = urllib.request.Request(api_url + "/api/v1/admin/stats/reset", method="POST", data=b"")
                    urllib.request.urlopen(req, timeout=10).read()
                threading.Thread(target=_reset, daemon=True).start()
            churn = {"calls": 0, "errors": 0, "ms": []}
            churn_stop = threading.Event()

            def _churn():
                k = 0
                while not churn_stop.wait(a.admin_churn):
                    k += 1
                    calls = [("POST", "/api/v1/admin/preprocessor/rules", {"pattern": f"(?i)churn{k}", "priority": 2}),
                             ("GET", "/metrics", None), ("GET", "/api/v1/admin/dead-letter?limit=10", None),
                             ("GET", "/api/v1/queues/status", None),
                             ("DELETE", "/api/v1/admin/preprocessor/rules", {"pattern": f"(?i)churn{k}", "priority": 2})]
                    for method, path, body in calls:
                        t0 = time.perf_counter()
                        try:
                            req = urllib.request.Request(api_url + path, method=method,
                                                         data=json.dumps(body).encode() if body else None,
                                                         headers={"Content-Type": "application/json"})
                            urllib.request.urlopen(req, timeout=10).read()
                        except Exception:                      # noqa: BLE001 -- counted
                            churn["errors"] += 1
                        churn["calls"] += 1
                        churn["ms"].append((time.perf_counter() - t0) * 1e3)
            if a.admin_churn > 0 and api_url:
                threading.Thread(target=_churn, daemon=True).start()
            cancels = {"posted": 0, "post_errors": 0, "deleted": 0, "dequeued": 0, "cancelled": 0,
                       "already_done": 0, "not_found": 0, "errors": 0}

            def _cancel_churn():
                import random
                rnd = random.Random(11)
                period = 1.0 / a.cancel_churn
                nxt = time.monotonic()
                k = 0
                while not churn_stop.is_set():
                    nxt += period
                    k += 1
                    try:
                        req = urllib.request.Request(urls[0] + "/api/v1/messages", method="POST",
                                                     data=json.dumps({"content": f"cancel me {k}", "user_id": "cc",
                                                                      "priority": 1 + k % 4}).encode(),
                                                     headers={"Content-Type": "application/json"})
                        mid = json.loads(urllib.request.urlopen(req, timeout=10).read())["message_id"]
                        cancels["posted"] += 1
                    except Exception:                      # noqa: BLE001 -- counted
                        cancels["post_errors"] += 1
                        continue
                    time.sleep(rnd.uniform(0.0, 0.06))
                    try:
                        req = urllib.request.Request(urls[0] + f"/api/v1/messages/{mid}", method="DELETE")
                        d = json.loads(urllib.request.urlopen(req, timeout=10).read())
                        cancels["deleted"] += 1
                        if d.get("dequeued"):
                            cancels["dequeued"] += 1
                        elif d.get("cancelled"):
                            cancels["cancelled"] += 1
                        else:
                            cancels["already_done"] += 1
                    except urllib.error.HTTPError as e:
                        cancels["not_found" if e.code == 404 else "errors"] += 1
                    except Exception:                      # noqa: BLE001 -- counted
                        cancels["errors"] += 1
                    time.sleep(max(0.0, nxt - time.monotonic()))
            if a.cancel_churn > 0:
                import urllib.error
                threading.Thread(target=_cancel_churn, daemon=True).start()
            faults = {"injected": 0, "restored": 0, "errors": 0}

            def _fault_cycle():
                def call(method, path, body):
                    req = urllib.request.Request(api_url + path, method=method, data=json.dumps(body).encode(),
                                                 headers={"Content-Type": "application/json"})
                    urllib.request.urlopen(req, timeout=10).read()
                while not churn_stop.wait(a.fault_cycle / 2):
                    try:
                        call("POST", "/api/v1/admin/faults", {"fail_launch": 1})
                        faults["injected"] += 1
                    except Exception:                      # noqa: BLE001 -- counted
                        faults["errors"] += 1
                    if churn_stop.wait(a.fault_cycle / 2):
                        break
                    try:
                        call("PUT", "/api/v1/endpoints/gpu0/status", {"status": "healthy"})
                        faults["restored"] += 1
                    except Exception:                      # noqa: BLE001 -- counted
                        faults["errors"] += 1
            if a.fault_cycle > 0 and api_url:
                threading.Thread(target=_fault_cycle, daemon=True).start()
            # server memory over the measured run (every spawned process and
            # its children): a leak shows up as a growing series; a progress
            # line on stderr every sample keeps long soaks visibly alive
            rss = []
            rss_stop = threading.Event()

            def _rss():
                import psutil
                t0 = time.monotonic()
                while True:
                    tot = 0
                    for p0 in procs:
                        try:
                            pp = psutil.Process(p0.pid)
                            for q in [pp] + pp.children(recursive=True):
                                tot += q.memory_info().rss
                        except psutil.Error:
                            pass
                    rss.append((round(time.monotonic() - t0, 1), round(tot / 2**20, 1)))
                    print(f"[http_load] t={rss[-1][0]}s server rss {rss[-1][1]} MiB", file=sys.stderr, flush=True)
                    if rss_stop.wait(a.rss_every):
                        return
            if procs:
                threading.Thread(target=_rss, daemon=True).start()
            r = subprocess.run([exe, host, port, str(a.rate), str(a.duration), str(a.procs), str(a.conns)] + extra,
                               capture_output=True, text=True, timeout=a.duration + 60)
            churn_stop.set()
            rss_stop.set()
            st_end = None
            if api_url:                         # latency window closes with the load (before the drain)
                with urllib.request.urlopen(api_url + "/api/v1/queues/stats", timeout=10) as rr:
                    st_end = json.loads(rr.read())
            os.unlink(exe)
            out = json.loads(r.stdout.strip().splitlines()[-1])
            if api_url:
                time.sleep(2.0)
                with urllib.request.urlopen(api_url + "/api/v1/queues/stats", timeout=10) as rr:
                    st = json.loads(rr.read())
                t_drain = time.monotonic()
                while a.cancel_churn > 0 and time.monotonic() - t_drain < 60:
                    dd = (st.get("job") or st).get("dispatch") or {}
                    ended = sum(int(dd.get(k, 0)) for k in ("completed", "cancelled", "expired", "retry_exhausted",
                                                            "rejected"))
                    if int(dd.get("submitted", 0)) - ended - cancels["dequeued"] <= 0:
                        break                    # drained: every accepted request has ended
                    time.sleep(1.0)
                    with urllib.request.urlopen(api_url + "/api/v1/queues/stats", timeout=10) as rr:
                        st = json.loads(rr.read())
                if "job" in st:                  # multi-rank: every rank's counters and histograms
                    st, st_end = st["job"], st_end["job"]
                    out["ranks"] = st.get("ranks")
                    out["accepted_by_rank"] = st.get("accepted_by_rank")
                    out["front_door"] = st.get("front_door")
                    out["missing_ranks"] = st.get("missing_ranks")
                    out["profile_by_rank"] = st_end.get("profile_by_rank")
                out["dispatcher"] = {"dispatch": st.get("dispatch"), "latency": st_end.get("latency"),
                                     "latency_e2e": st_end.get("latency_e2e"),
                                     "note": "latency: HTTP arrival (native ingress clock) -> GPU slot admission; "
                                             "latency_e2e: -> last generated token; window = the measured run"}
            out["mode"] = a.spawn or "url"
            if rss:
                out["server_rss_mib"] = {"every_s": a.rss_every, "first": rss[0][1], "last": rss[-1][1],
                                         "max": max(v for _t, v in rss), "series": rss}
            if a.fault_cycle > 0:
                out["fault_cycle"] = dict(faults, every_s=a.fault_cycle)
            if a.cancel_churn > 0:
                out["cancel_churn"] = dict(cancels, per_s=a.cancel_churn)
                dsp = (out.get("dispatcher") or {}).get("dispatch") or {}
                if dsp:
                    # every accepted request ends exactly once: completed, cancelled
                    # (in flight / in backoff / held), shed at its deadline, dead-lettered,
                    # or taken out of its tier queue by a DELETE (client-side "dequeued")
                    ended = sum(int(dsp.get(k, 0)) for k in ("completed", "cancelled", "expired",
                                                             "retry_exhausted", "rejected"))
                    out["cancel_churn"]["accounting"] = {
                        "submitted": int(dsp.get("submitted", 0)), "ended": ended,
                        "dequeued_by_delete": cancels["dequeued"],
                        "unaccounted": int(dsp.get("submitted", 0)) - ended - cancels["dequeued"]}
            if a.admin_churn > 0 and churn["ms"]:
                ms = sorted(churn["ms"])
                out["admin_churn"] = {"every_s": a.admin_churn, "calls": churn["calls"], "errors": churn["errors"],
                                      "p50_ms": round(ms[len(ms) // 2], 2), "max_ms": round(ms[-1], 2)}
            print(json.dumps(out))
            return
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        cs = [ctx.Process(target=_client_proc, args=(urls, a.rate / a.procs, a.duration, 17 + i, q))
              for i in range(a.procs)]
        t0 = time.perf_counter()
        for c in cs:
            c.start()
        res = [q.get(timeout=a.duration + 90) for _ in cs]
        wall = time.perf_counter() - t0
        for c in cs:
            c.join(timeout=10)
        lat = sorted(x for r in res for x in r["lat"])
        codes = {}
        for r in res:
            for k, v in r["codes"].items():
                codes[str(k)] = codes.get(str(k), 0) + v
        sent = sum(r["sent"] for r in res)
        dispatcher = None
        if api_url:                              # what the GPU/CPU dispatcher behind the ring did
            import urllib.request
            time.sleep(2.0)
            with urllib.request.urlopen(api_url + "/api/v1/queues/stats", timeout=10) as r:
                st = json.loads(r.read())
            dispatcher = {"dispatch": st.get("dispatch"), "latency": st.get("latency"), "rings": st.get("rings")}
        ok = codes.get("202", 0)
        pct = lambda q_: lat[min(len(lat) - 1, int(q_ * len(lat)))] * 1e3 if lat else 0.0   # noqa: E731
        print(json.dumps({"mode": a.spawn or "url", "ingress_procs": len(urls), "offered_rps": a.rate,
                          "sent": sent, "accepted_rps": round(ok / a.duration, 1),
                          "error_rate": round(1 - ok / max(1, sent), 4), "codes": codes,
                          "p50_ms": round(pct(0.5), 2), "p99_ms": round(pct(0.99), 2),
                          "wall_s": round(wall, 1), "dispatcher": dispatcher}))
    finally:
        for p in procs:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)


if __name__ == "__main__":
    main()
