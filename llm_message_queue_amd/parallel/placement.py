"""GPU-local host placement: bind each rank's process (every thread of it,
and the helper processes it starts) to the CPU cores of the socket its GPU
hangs off.

An 8-GPU MI355X node has two sockets with four GPUs behind each.  A rank's
host work per tick is real -- kernel enqueue (~3.7 ms), dispatch (~2 ms),
the shared-memory spin-waits of the control plane, reads of the host-mapped
slot page the GPU writes -- and every one of those touches memory or a PCIe
path local to ONE socket.  ``--pin-cpu`` used to pin rank r to core r, which
puts every rank on socket 0.  Here the kernel's own topology decides:

  * ``/sys/bus/pci/devices/<dddd:bb:dd.f>/local_cpulist`` of the rank's GPU
    (its PCI address from the HIP device properties);
  * intersected with the CPUs this process may use (cgroup cpuset);
  * split evenly, by physical core (SMT siblings stay together,
    ``/sys/devices/system/cpu/cpuN/topology/thread_siblings_list``), among
    the local ranks whose GPUs share that cpulist, in local-rank order -- so
    four ranks on one socket do not contend for the same cores.

The reference has no multi-GPU path; its deployment notes
size the node only (`docs/deployment.md:14-24`).
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional, Sequence, Set


def parse_cpulist(text: str) -> List[int]:
    """Linux cpulist ("0-3,8,10-11") -> sorted CPU ids."""
    out: Set[int] = set()
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.update(range(int(a), int(b) + 1))
        else:
            out.add(int(part))
    return sorted(out)


def format_cpulist(cpus: Iterable[int]) -> str:
    """Sorted CPU ids -> compact cpulist ("0-3,8")."""
    xs = sorted(set(int(c) for c in cpus))
    out, i = [], 0
    while i < len(xs):
        j = i
        while j + 1 < len(xs) and xs[j + 1] == xs[j] + 1:
            j += 1
        out.append(str(xs[i]) if i == j else f"{xs[i]}-{xs[j]}")
        i = j + 1
    return ",".join(out)


def pci_address(domain: int, bus: int, device: int, function: int = 0) -> str:
    return "%04x:%02x:%02x.%x" % (domain, bus, device, function)


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def gpu_local_cpus(pci: str, sysfs: str = "/sys") -> Optional[List[int]]:
    """CPUs local to the PCI device (its socket / NUMA node), or None."""
    txt = _read(os.path.join(sysfs, "bus", "pci", "devices", pci, "local_cpulist"))
    if not txt:
        return None
    cpus = parse_cpulist(txt)
    return cpus or None


def gpu_numa_node(pci: str, sysfs: str = "/sys") -> int:
    txt = _read(os.path.join(sysfs, "bus", "pci", "devices", pci, "numa_node"))
    try:
        return int(txt) if txt is not None else -1
    except ValueError:
        return -1


def physical_cores(cpus: Sequence[int], sysfs: str = "/sys") -> List[List[int]]:
    """``cpus`` grouped by physical core (SMT siblings together), cores in
    ascending order of their first CPU.  A CPU without topology information
    is a core of its own."""
    allowed = set(cpus)
    seen: Set[int] = set()
    groups: List[List[int]] = []
    for c in sorted(allowed):
        if c in seen:
            continue
        txt = _read(os.path.join(sysfs, "devices", "system", "cpu", f"cpu{c}", "topology", "thread_siblings_list"))
        sib = [x for x in parse_cpulist(txt) if x in allowed] if txt else [c]
        if c not in sib:
            sib = [c]
        seen.update(sib)
        groups.append(sorted(sib))
    return groups


def plan_binding(local_rank: int, rank_pci: Sequence[str], allowed: Iterable[int],
                 sysfs: str = "/sys") -> Dict[str, object]:
    """The CPU set of local rank ``local_rank`` given every local rank's GPU
    PCI address (``rank_pci[i]`` = local rank i's GPU).  Ranks whose GPUs
    share a cpulist split its physical cores evenly in local-rank order (the
    first ``n % k`` ranks take one more).  ``cpus`` is empty when the
    topology is unknown or leaves this process no CPU (then nothing is
    bound)."""
    allowed = set(int(c) for c in allowed)
    pci = rank_pci[local_rank]
    local = gpu_local_cpus(pci, sysfs)
    plan: Dict[str, object] = {"pci": pci, "numa_node": gpu_numa_node(pci, sysfs), "cpus": [],
                               "source": "sysfs local_cpulist"}
    if local is None:
        plan["source"] = "unknown (no local_cpulist)"
        return plan
    mine = [c for c in local if c in allowed]
    if not mine:
        plan["source"] = "local_cpulist outside this process's cpuset"
        return plan
    key = tuple(local)
    peers = [i for i, p in enumerate(rank_pci) if tuple(gpu_local_cpus(p, sysfs) or ()) == key]
    k, idx = len(peers), peers.index(local_rank)
    cores = physical_cores(mine, sysfs)
    if len(cores) >= k:
        base, extra = divmod(len(cores), k)
        lo = idx * base + min(idx, extra)
        hi = lo + base + (1 if idx < extra else 0)
        sel = [c for g in cores[lo:hi] for c in g]
    else:                                           # fewer cores than ranks: share the socket's cores
        sel = mine
    plan.update(cpus=sorted(sel), shared_with=peers, cores=len(cores))
    return plan


def process_threads(pid: int = 0) -> List[int]:
    """Thread ids of a process (``/proc/<pid>/task``)."""
    d = f"/proc/{pid or os.getpid()}/task"
    try:
        return [int(t) for t in os.listdir(d)]
    except OSError:
        return [pid or os.getpid()]


def apply_binding(cpus: Sequence[int], pids: Sequence[int] = (0,)) -> int:
    """Bind every thread of each process in ``pids`` (0 = this one) to
    ``cpus``; threads started later inherit it from their creator.  Returns
    the number of threads bound (0: nothing to do / not permitted)."""
    if not cpus or not hasattr(os, "sched_setaffinity"):
        return 0
    cs = set(int(c) for c in cpus)
    n = 0
    for pid in pids:
        for tid in process_threads(pid):
            try:
                os.sched_setaffinity(tid, cs)
                n += 1
            except OSError:
                pass
    return n


def torch_rank_pci(local_world: int) -> List[str]:
    """PCI address of every local rank's GPU (the rank -> HIP device map of
    ``parallel.comm.local_device_index``), from the HIP device properties."""
    import torch
    from .comm import _DEVICES
    n = torch.cuda.device_count()
    out = []
    for lr in range(local_world):
        dev = _DEVICES[lr % len(_DEVICES)] if _DEVICES else (lr % n if n else 0)
        p = torch.cuda.get_device_properties(dev)
        out.append(pci_address(int(p.pci_domain_id), int(p.pci_bus_id), int(p.pci_device_id)))
    return out


MIN_AUTO_CPUS = 4


def bind_rank(mode: str = "auto", extra_pids: Sequence[int] = (), sysfs: str = "/sys",
              world: Optional[int] = None) -> Dict[str, object]:
    """Bind this rank (and ``extra_pids``, e.g. its front-door feeder) to its
    GPU's local cores.  ``mode``: "gpu" always; "auto" only when the job has
    more than one rank (a one-GPU run is left as launched); "core" the old
    rank -> core r pinning; "off" nothing.  Returns the plan (recorded in the
    bench JSON's ``comm`` block)."""
    world = int(os.environ.get("WORLD_SIZE", "1")) if world is None else world
    local_rank = int(os.environ.get("LOCAL_RANK", os.environ.get("RANK", "0")))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if mode == "off" or (mode == "auto" and world <= 1) or not hasattr(os, "sched_getaffinity"):
        return {"mode": mode, "cpus": "", "bound_threads": 0}
    allowed = sorted(os.sched_getaffinity(0))
    if mode == "core":
        cpus = [allowed[local_rank % len(allowed)]]
        plan: Dict[str, object] = {"source": "rank -> core"}
    else:
        try:
            import torch
            if not torch.cuda.is_available():
                return {"mode": mode, "cpus": "", "bound_threads": 0, "source": "no GPU"}
            plan = plan_binding(local_rank, torch_rank_pci(local_world), allowed, sysfs)
        except Exception as e:                 # noqa: BLE001 -- placement is an optimisation, never fatal
            return {"mode": mode, "cpus": "", "bound_threads": 0, "source": f"error: {e}"}
        cpus = list(plan.get("cpus") or [])
        if mode == "auto" and 0 < len(cpus) < MIN_AUTO_CPUS:
            # a rank's serve loop, ring / ingest / peer threads and the
            # preprocess host work need a few cores: a cpuset that leaves it
            # fewer is better shared than split (explicit "gpu" still binds)
            plan = dict(plan, source=f"{plan.get('source')}: only {len(cpus)} CPUs for this rank, left unbound")
            cpus = []
    n = apply_binding(cpus, [0] + [int(p) for p in extra_pids]) if cpus else 0
    out = dict(plan, mode=mode, cpus=format_cpulist(cpus), bound_threads=n)
    return out
