"""bench.py driver contract, rehearsed on CPU: the multi-rank control flow
(torch.distributed.run, one process per rank, fixed tick counts so every rank
issues the same collectives, max-over-ranks timing, one JSON line from rank 0)
with gloo and a tiny model (``--cpu-dry-run``; never a measurement)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(args, timeout=240):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(args, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def test_bench_single_rank_dry_run():
    d = _run([sys.executable, "bench.py", "--cpu-dry-run", "--steps", "4", "--warmup", "2",
              "--gateway-only-s", "0.3", "--gateway-only-rate", "300"])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 2 and d["scaling"] == "weak"
    assert "DRY RUN" in d["data"] and d["value"] >= 0 and "gateway_only" in d
    # the timed window starts in steady state: untimed serving ticks at the
    # offered rate ran first (the driver's 20-step window used to
    # start from the empty system the calibration drain left)
    assert d["steady_ticks"] >= 60
    # the reported window's rate = min(dispatched, arrived) per second: never
    # above the rate the offered load actually arrived at; value is that rate
    # when the window held the operating point and 0 otherwise (SLO search)
    # (the reported window: the best attempt that held the SLO, else the last)
    att = d["slo_search"]["attempts"]
    w = next((t for t in att if t["met"] and t["util"] == d["config"]["util"]), att[-1])["value"]
    assert w <= d["dispatch_rate_in_window"] + 1e-6
    assert w <= d["arrival_rate_in_window"] + 1e-6
    assert abs(w - min(d["dispatch_rate_in_window"], d["arrival_rate_in_window"])) < 0.02
    assert d["value"] == (w if d["p99_target_met"] else 0.0)
    lb = d["latency_breakdown"]
    assert set(lb) >= {"ingress", "inbox", "preprocess", "queue", "handoff", "admitted_by_path"}
    assert sum(sum(v) for v in lb["admitted_by_path"].values()) > 0
    # what one request is: its shape and the GEMM FLOP rate vs peak
    rs = d["request_shape"]
    assert rs["gen_tokens"] == 4 and 1 <= rs["mean_prompt_tokens"] <= rs["prompt_cap"]
    assert abs(rs["tokens_per_request"] - (rs["mean_prompt_tokens"] + 3)) < 0.02
    assert 0 <= d["mfma_peak_fraction"] < 1 and d["backend_matmul_tflops"] >= 0
    assert d["config"]["seq_len_is"] == "max_ctx" and d["config"]["max_ctx"] == d["config"]["seq_len"]
    assert d["realtime_mode"] == d["config"]["realtime_mode"] == "off"
    assert d["data_plane"] == "none"


def test_bench_realtime_micro_mode_dry_run():
    d = _run([sys.executable, "bench.py", "--cpu-dry-run", "--steps", "4", "--warmup", "2", "--gateway-only-s", "0",
              "--realtime-mode", "micro", "--micro-slots", "4"])
    assert d["realtime_mode"] == "micro" and d["config"]["micro"]["slots"] == 4
    assert d["micro_forwards"]["count"] >= 0 and d["requests_accounted"]["lost"] == 0


def _preflight_run(fault):
    env = dict(os.environ, OMP_NUM_THREADS="1", LLMQ_RCCL_PREFLIGHT_S="3")
    if fault:
        env["LLMQ_RCCL_PREFLIGHT_FAULT"] = fault
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
                        "--cpu-dry-run", "--data-backend", "nccl", "--steps", "4", "--warmup", "2",
                        "--gateway-only-s", "0", "--slo-climb", ""],
                       cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert r.returncode == 0, r.stderr[-3000:]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0]), r.stderr


def test_rccl_preflight_hang_falls_back_to_gloo_data_plane():
    """an RCCL data plane whose preflight hangs (or
    fails) must not cost the run its headline -- every rank agrees on the
    gloo fallback, the job serves, and the JSON says so."""
    d, err = _preflight_run("hang")
    assert d["data_plane"] == "gloo-fallback" and d["comm"]["data_backend"] == "gloo-fallback"
    pf = d["comm"]["preflight"]
    assert not pf["ok_all_ranks"] and "hang" in pf["error"] and pf["wall_ms"] >= 2900
    assert d["comm"]["rccl_world"] == 0
    assert d["requests_accounted"]["completed"] > 0 and "falls back to gloo" in err


def test_rccl_preflight_failure_falls_back_to_gloo_data_plane():
    d, _err = _preflight_run("fail")
    assert d["data_plane"] == "gloo-fallback"
    assert "injected" in d["comm"]["preflight"]["error"]
    assert d["requests_accounted"]["completed"] > 0


def test_bench_four_ranks_torchrun_dry_run():
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
              "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "4",
              "--cpu-dry-run", "--steps", "5", "--warmup", "2", "--gateway-only-s", "0.5",
              "--gateway-only-rate", "200"])
    assert d["n_gpus"] == 4 and d["config"]["parallelism"] == "dp4"
    # 4 CPU ranks of a tiny model on a shared host: whether a util holds the
    # SLO is timing noise here, so pin the contract, not the outcome -- every
    # attempt served requests, and value is the best attempt that held the
    # target or 0 with the reason stated
    slo = d["slo_search"]
    assert all(a["value"] > 0 for a in slo["attempts"])
    met = [a["value"] for a in slo["attempts"] if a["met"]]
    assert d["value"] == (max(met) if met else 0.0)
    assert met or "reason" in slo
    # the secondary null-backend phase runs multi-rank too (the driver's 8-GPU run does it)
    assert d["gateway_only"]["requests_per_s"] > 0


def _rank0_ingress(world, mode="rank0"):
    # --tick-ms: with the shared-memory control plane a tiny-model CPU tick
    # takes ~1 ms, so 14 unpaced ticks would see almost no Poisson arrivals
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
              "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", str(world),
              "--cpu-dry-run", "--steps", "6", "--warmup", "2", "--steady-ticks", "8", "--gateway-only-s", "0",
              "--ingress", mode, "--lb", "round_robin", "--tick-ms", "20", "--rate", "200"], timeout=420)
    assert d["n_gpus"] == world and d["config"]["ingress"] == mode
    acc = d["requests_accounted"]
    assert acc["offered"] > 0 and acc["lost"] == 0 and acc["completed"] > 0, acc
    return d


def test_bench_rank0_ingress_world4_dry_run():
    """One front door for the job: a feeder process writes the raw records
    into ONE shared ring (the `cli serve` topology) and every rank drains
    it, so every rank preprocesses a share (GPU 0 used
    to preprocess the whole job's traffic).  The ring is pull-based: the
    shares follow each rank's pump cadence, the planner balances dispatch."""
    d = _rank0_ingress(4)
    ing = d["lockstep"]["ingested_by_rank"]
    assert len(ing) == 4 and min(ing) > 0, ing
    # (every rank took part over the whole attempt too; the even split of the
    # balanced share needs consumers that poll continuously -- cli serve's
    # ring threads -- and is pinned in test_multirank_serve.py, while these
    # dry-run pumps poll once per 20 ms tick)
    tot = d["lockstep"]["ingested_total_by_rank"]
    assert d["config"]["door_share"] == "fair" and min(tot) > 0, tot


def test_bench_rank0_funnel_world4_dry_run():
    """The r2 form (A/B): rank 0 preprocesses everything; the planner then
    spreads the dispatches."""
    d = _rank0_ingress(4, "rank0-funnel")
    ing = d["lockstep"]["ingested_by_rank"]
    assert ing[0] > 0 and ing[1:] == [0, 0, 0], ing
    assert d["remote_dispatched"] > 0


def test_bench_rank0_ingress_world8_dry_run():
    d = _rank0_ingress(8)
    assert sum(v > 0 for v in d["lockstep"]["ingested_by_rank"]) >= 6


def test_bench_self_launches_without_torchrun():
    """``bench.py --gpus 4`` with no launcher starts 4 ranks itself (a child
    torch.distributed.run) instead of silently running one."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--cpu-dry-run", "--steps", "4", "--warmup", "2",
                        "--gateway-only-s", "0"], cwd=ROOT, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["comm"]["world"] == 4
    assert d["comm"]["data_backend"] == "gloo" and len(d["comm"]["devices"]) == 4
    assert d["comm"]["allreduce"]["busbw_GBps"] > 0
    ls = d["lockstep"]
    assert len(ls["collective_wait_ms_p50_by_rank"]) == 4 and len(ls["gpu_steps_by_rank"]) == 4
    assert d["requests_accounted"]["lost"] == 0


def test_bench_refuses_world_mismatch():
    """A launcher that started a different number of ranks than --gpus makes
    bench.py exit non-zero instead of reporting n_gpus for the wrong count."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--cpu-dry-run"], cwd=ROOT,
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert "WORLD_SIZE=2" in r.stderr


def test_bench_sim_gpu_two_ranks_extra_steps():
    """``--sim-gpu``: each rank's backend is a SimEngine at the serving config
    (1536 slots, 4096-token steps, 8B step clock).  With rank 1 simulated 30 %
    slower, rank 0 takes extra local steps instead of idling for rank 1's
    pace, and every request is accounted for."""
    d = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
              "--cpu-dry-run", "--sim-gpu", "1,0.7", "--steps", "40", "--warmup", "2", "--gateway-only-s", "0"],
             timeout=420)
    assert d["config"]["sim_gpu"] == "1,0.7" and d["config"]["extra_steps"]
    assert d["config"]["global_batch"] == 2 * 1536 and d["config"]["token_budget"] == 4096
    ls = d["lockstep"]
    assert ls["extra_steps_by_rank"][0] > ls["extra_steps_by_rank"][1]
    assert ls["gpu_steps_by_rank"][0] > ls["gpu_steps_by_rank"][1]
    assert d["requests_accounted"]["lost"] == 0 and d["value"] > 0


def test_bench_slo_search_backs_off_to_a_met_operating_point():
    """the headline is req/s AT the SLO.  A window that
    misses it (forced here by a test-only hook for every util above 0.95) is
    re-served in the same process at the next lower utilisation, and the
    value reported is that window's rate; the first attempt is listed."""
    d = _run([sys.executable, "bench.py", "--cpu-dry-run", "--sim-gpu", "1", "--steps", "20", "--warmup", "2",
              "--gateway-only-s", "0", "--test-miss-above-util", "0.95"], timeout=420)
    s = d["slo_search"]
    assert s["util_tried"][0] == 0.98 and s["attempts"][0]["met"] is False
    # 0.95 is the first util the hook lets through; on a loaded host (the
    # suite under xdist) the sim can genuinely miss there too and the search
    # goes on down -- either way the value is the first met attempt's
    u = s["value_util"]
    assert d["p99_target_met"] and u <= 0.95 and u == d["config"]["util"]
    assert s["attempts"][-1]["met"] and not any(t["met"] for t in s["attempts"][:-1])
    assert d["value"] == s["attempts"][-1]["value"] > 0
    assert abs(d["offered_rate_per_gpu"] - u * d["calibrated_capacity_per_gpu"]) < 1.0
    assert d["requests_accounted"]["lost"] == 0


def test_bench_slo_search_climbs_while_the_slo_holds():
    """the search climbs too.  The first window (0.98)
    holds the SLO, so 1.0, 1.02, ... are served while it keeps holding (the
    test hook makes every util above 1.01 miss); the headline is the best
    window that held it, and every attempt is listed."""
    d = _run([sys.executable, "bench.py", "--cpu-dry-run", "--sim-gpu", "1", "--steps", "20", "--warmup", "2",
              "--gateway-only-s", "0", "--test-miss-above-util", "1.01"], timeout=420)
    s = d["slo_search"]
    met = [t for t in s["attempts"] if t["met"]]
    if not s["attempts"][0]["met"]:                 # a loaded host missed at 0.98: the back-off path ran
        assert s["util_tried"][1] < 0.98
        return
    assert s["util_tried"][:3] == [0.98, 1.0, 1.02] and s["attempts"][2]["met"] is False
    assert len(s["util_tried"]) == 3                # stopped at the first miss above the knee
    best = max(met, key=lambda t: t["value"])
    assert d["value"] == best["value"] > 0 and s["value_util"] == best["util"] == d["config"]["util"]
    assert d["p99_target_met"] and s["search_s"] > 0 and d["requests_accounted"]["lost"] == 0


def test_overload_bench_multirank_sheds_low_tiers_parks_and_unparks():
    """BASELINE config 5 across ranks: at 1.5x the
    job's capacity realtime and high are served in full and the rest is shed
    to the dead-letter queue at its deadline, nothing lost; a drop to 0.1x
    parks a GPU through rank 0's resource scheduler and the return of the
    overload (queued demand no active GPU has room for) unparks it."""
    d = _run([sys.executable, "bench/overload_bench.py", "--gpus", "2", "--cpu-dry-run", "--sim-gpu", "1",
              "--seconds", "3", "--policies", "fifo", "--autoscale", "1.5:2,0.1:3,1.5:3",
              "--scale-cooldown-s", "0.5"], timeout=420)
    r = d["policies"]["fifo"]
    assert r["expired_to_dlq_by_tier"][0] == 0 and r["expired_to_dlq_by_tier"][1] == 0
    assert r["served_by_tier"][0] > 0 and r["served_by_tier"][1] > 0
    assert r["expired"] > 0 and r["dlq_added"] == r["expired"]
    assert r["requests_accounted"]["lost"] == 0
    steps = d["autoscale"]["steps"]
    assert any(e["action"] == "scale_down" for e in steps[1]["scale_events"]) and steps[1]["parked_at_end"]
    assert any(e["action"] == "scale_up" for e in steps[2]["scale_events"]) and steps[2]["parked_at_end"] == []
    assert d["autoscale"]["requests_accounted"]["lost"] == 0


def test_dialog_bench_multirank_reports_per_rank_kv_counts():
    """BASELINE config 4 across ranks: conversations
    entering at rank 0 are homed over the job's GPUs; with KV residency every
    turn after the first prefills only its new tokens, replay re-prefills the
    dialog; per-rank counts are reported and every turn completes."""
    d = _run([sys.executable, "bench/dialog_bench.py", "--gpus", "2", "--cpu-dry-run", "--sim-gpu", "1",
              "--convs", "64", "--turns", "3", "--ingress", "rank0"], timeout=420)
    res, rep = d["modes"]["residency"], d["modes"]["replay"]
    for m in (res, rep):
        assert m["turns_completed"] == m["turns_offered"] == 2 * 64 * 3
        assert len(m["by_rank"]["kv_migrated"]) == 2 and len(m["by_rank"]["turns_completed"]) == 2
    assert res["kv_reused_tokens"] > 0 and rep["kv_reused_tokens"] == 0
    assert res["forward_tokens_per_turn"] < rep["forward_tokens_per_turn"]
    assert res["remote_sent"] > 0                     # rank 0's turns run on both GPUs
    assert rep["kv_migrated"] == 0 and rep["kv_migrate_replays"] == 0
