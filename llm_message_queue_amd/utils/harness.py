"""Shared scaffolding of the multi-GPU benchmarks (``bench.py``,
``bench/overload_bench.py``, ``bench/dialog_bench.py``): starting N ranks
when no launcher did, the evidence of what a job ran on, and the per-rank
lock-step report.  One process per GPU, ``torch.distributed`` for the data
plane (RCCL on MI355X), the node-local shared-memory control plane for the
per-tick collectives."""
from __future__ import annotations

import os
import sys
import time

import numpy as np


def comm_evidence(comm, dev, world: int, dry: bool, binding: dict = None) -> dict:
    """Proof of what the job ran on, gathered from every rank: data-plane
    backend, per-rank HIP device index and PCI address (distinct unless the
    ranks were wrapped onto fewer GPUs), each rank's host CPU binding
    (``parallel.placement``: NUMA node and cores of its GPU's socket), and
    one timed all_reduce on the data plane (64 MiB on RCCL; 8 MiB on the CPU
    rehearsal's gloo)."""
    import torch
    from ..parallel.comm import gpus_oversubscribed
    ev = {"world": world, "control_plane": "solo" if world == 1 else str(getattr(comm, "backend", "?")),
          "data_backend": "none", "oversubscribed": False}
    if binding is not None:
        from ..parallel.placement import parse_cpulist
        cpus = parse_cpulist(str(binding.get("cpus") or ""))
        row = np.array([int(binding.get("numa_node", -1)), len(cpus), cpus[0] if cpus else -1,
                        cpus[-1] if cpus else -1, int(binding.get("bound_threads", 0))], dtype=np.int64)
        g = comm.all_gather_i64(row)
        ev["cpu_binding"] = {"mode": binding.get("mode"), "source": binding.get("source", ""),
                             "rank0_cpus": binding.get("cpus", ""),
                             "by_rank": [{"rank": r, "numa_node": int(x[0]), "ncpus": int(x[1]),
                                          "first_cpu": int(x[2]), "last_cpu": int(x[3]),
                                          "threads_bound": int(x[4])} for r, x in enumerate(g.tolist())]}
    if dev.type == "cuda":
        p = torch.cuda.get_device_properties(dev)
        mine = [int(dev.index), int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id)]
    else:
        mine = [-1, -1, -1, -1]
    rows = comm.all_gather_i64(np.array(mine, dtype=np.int64))
    ev["devices"] = [{"rank": r, "hip_device": int(x[0]),
                      "pci": "%04x:%02x:%02x" % (x[1], x[2], x[3]) if x[0] >= 0 else "cpu"}
                     for r, x in enumerate(rows.tolist())]
    if dev.type == "cuda":
        ev["device_name"] = torch.cuda.get_device_name(dev)
        ev["distinct_devices"] = len({tuple(x[1:]) for x in rows.tolist()})
    if world == 1:
        return ev
    import torch.distributed as dist
    inner = getattr(comm, "data", comm)
    group = getattr(inner, "data_group", None)
    ev["data_backend"] = getattr(comm, "data_backend", None) or dist.get_backend(group)
    if getattr(comm, "preflight", None) is not None:
        ev["preflight"] = comm.preflight
        ev["rccl_world"] = int(comm.preflight.get("rccl_world", 0)) if ev["data_backend"] == "nccl" else 0
    ev["oversubscribed"] = bool(gpus_oversubscribed()) if not dry else False
    if dev.type == "cuda":
        ev["one_gpu_per_rank"] = ev["distinct_devices"] == world
        if not ev["oversubscribed"] and not ev["one_gpu_per_rank"]:
            print(f"bench: WARNING ranks share GPUs without oversubscription: {ev['devices']}", file=sys.stderr)
    nbytes = (64 << 20) if ev["data_backend"] == "nccl" else (8 << 20)
    tdev = dev if ev["data_backend"] == "nccl" else torch.device("cpu")
    try:
        x = torch.ones(nbytes // 4, dtype=torch.float32, device=tdev)
        for _ in range(2):
            dist.all_reduce(x, group=group)
        iters = 5
        if tdev.type == "cuda":
            torch.cuda.synchronize(tdev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(x, group=group)
        if tdev.type == "cuda":
            torch.cuda.synchronize(tdev)
        dt = (time.perf_counter() - t0) / iters
        err = 0.0
    except Exception as e:      # noqa: BLE001 -- the serving path's control plane does not use this group
        print(f"bench: data-plane all_reduce failed: {e!r}", file=sys.stderr)
        dt, err = 0.0, 1.0
    # every rank reaches this gather (on the control plane), so a rank whose
    # collective raised cannot leave the others waiting on a later one
    dt, failed = comm.max_f64(dt), comm.max_f64(err) > 0
    if failed:
        ev["allreduce"] = {"bytes": nbytes, "backend": ev["data_backend"], "error": "all_reduce failed (see stderr)"}
        return ev
    alg = nbytes / dt / 1e9
    ev["allreduce"] = {"bytes": nbytes, "backend": ev["data_backend"], "ms": round(dt * 1e3, 3),
                       "algbw_GBps": round(alg, 2), "busbw_GBps": round(alg * 2 * (world - 1) / world, 2)}
    return ev


def lockstep_report(gw, engine, comm, elapsed: float) -> dict:
    """Where a multi-rank tick's time goes, per rank: control-plane wait
    (collectives: the exchange plus waiting for the slowest peer) and GPU
    execution time of the forward steps (timing events)."""
    ls = gw.lockstep_stats(reset=True)
    gms = engine.gpu_step_ms
    nst = max(1, engine.gpu_steps)
    mine = np.array([int(ls["p50_ms"] * 1e4), int(ls["max_ms"] * 1e4), int(ls["mean_ms"] * 1e4),
                     int(gms / nst * 1e4), int(engine.gpu_step_max_ms * 1e4), int(gms * 1e4), engine.gpu_steps],
                    dtype=np.int64)
    g = comm.all_gather_i64(mine).astype(np.float64)
    step_mean = g[:, 3] / 1e4
    busy = g[:, 5] / 1e4 / max(1e-9, elapsed * 1e3)
    return {"collective_wait_ms_p50_by_rank": [round(v, 3) for v in (g[:, 0] / 1e4).tolist()],
            "collective_wait_ms_max_by_rank": [round(v, 3) for v in (g[:, 1] / 1e4).tolist()],
            "collective_wait_ms_mean_by_rank": [round(v, 3) for v in (g[:, 2] / 1e4).tolist()],
            "gpu_step_ms_mean_by_rank": [round(v, 3) for v in step_mean.tolist()],
            "gpu_step_ms_max_by_rank": [round(v, 3) for v in (g[:, 4] / 1e4).tolist()],
            "gpu_busy_frac_by_rank": [round(v, 4) for v in busy.tolist()],
            "gpu_steps_by_rank": [int(v) for v in g[:, 6].tolist()],
            "slowest_over_mean_gpu_step": round(float(step_mean.max() / max(1e-9, step_mean.mean())), 4)}


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def self_launch(a, argv, script: str) -> int:
    """``bench.py --gpus N`` (N > 1) started without a launcher: run the
    same command under ``torch.distributed.run`` (one rank per GPU, N ranks)
    as a CHILD process and return its exit code.  Nothing here touches the
    GPU (no HIP call before the child starts; never exec).  Rank 0's JSON
    line reaches our stdout because the child inherits it."""
    import subprocess
    args = list(sys.argv[1:] if argv is None else argv)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(script)] + args
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    print(f"bench: --gpus {a.gpus} without a launcher; starting {a.gpus} ranks under torch.distributed.run",
          file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)
