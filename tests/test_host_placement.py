"""GPU-local host placement against a fake sysfs tree:
two sockets, eight GPUs, SMT siblings -- each rank gets its own physical cores
on its GPU's socket, never socket 0 for everyone (the old ``--pin-cpu``)."""
import os

from llm_message_queue_amd.parallel.placement import (apply_binding, format_cpulist, parse_cpulist,
                                                      physical_cores, plan_binding)

PCI = [f"0000:{b:02x}:00.0" for b in (0x05, 0x15, 0x25, 0x35, 0x85, 0x95, 0xa5, 0xb5)]


def _fake_sysfs(root):
    # socket 0: cores 0-15 (+ SMT siblings 32-47); socket 1: cores 16-31 (+ 48-63)
    for i, p in enumerate(PCI):
        d = os.path.join(root, "bus", "pci", "devices", p)
        os.makedirs(d)
        with open(os.path.join(d, "local_cpulist"), "w") as f:
            f.write("0-15,32-47\n" if i < 4 else "16-31,48-63\n")
        with open(os.path.join(d, "numa_node"), "w") as f:
            f.write("0\n" if i < 4 else "1\n")
    for c in range(64):
        d = os.path.join(root, "devices", "system", "cpu", f"cpu{c}", "topology")
        os.makedirs(d)
        core = c % 32
        with open(os.path.join(d, "thread_siblings_list"), "w") as f:
            f.write(f"{core},{core + 32}\n")
    return root


def test_cpulist_roundtrip():
    assert parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert format_cpulist([11, 0, 1, 2, 3, 8, 10]) == "0-3,8,10-11"
    assert parse_cpulist("") == []


def test_eight_gpus_two_sockets_each_rank_its_own_local_cores(tmp_path):
    root = _fake_sysfs(str(tmp_path))
    allowed = range(64)
    plans = [plan_binding(r, PCI, allowed, root) for r in range(8)]
    for r, p in enumerate(plans):
        sock = 0 if r < 4 else 1
        k = r % 4
        cores = list(range(16 * sock + 4 * k, 16 * sock + 4 * k + 4))
        assert p["cpus"] == sorted(cores + [c + 32 for c in cores]), (r, p)
        assert p["numa_node"] == sock and p["shared_with"] == list(range(4 * sock, 4 * sock + 4))
    # disjoint, and together exactly the node's CPUs
    allc = [c for p in plans for c in p["cpus"]]
    assert len(allc) == len(set(allc)) == 64


def test_cpuset_restricted_and_uneven_split(tmp_path):
    root = _fake_sysfs(str(tmp_path))
    # a container allowed 6 physical cores of socket 1 (no siblings): 4 ranks share them 2/2/1/1
    allowed = [16, 17, 18, 19, 20, 21]
    plans = [plan_binding(r, PCI, allowed, root) for r in range(4, 8)]
    assert [p["cpus"] for p in plans] == [[16, 17], [18, 19], [20], [21]]
    # nothing of the GPU's socket allowed: no binding, reason recorded
    p = plan_binding(0, PCI, allowed, root)
    assert p["cpus"] == [] and "outside" in p["source"]
    # unknown topology (no sysfs entry): no binding
    assert plan_binding(0, ["0000:ff:00.0"], range(8), root)["cpus"] == []


def test_physical_cores_keep_siblings_together(tmp_path):
    root = _fake_sysfs(str(tmp_path))
    assert physical_cores([0, 32, 1, 33, 5], root) == [[0, 32], [1, 33], [5]]


def test_apply_binding_binds_every_thread_of_this_process():
    import threading
    if not hasattr(os, "sched_setaffinity"):
        return
    before = os.sched_getaffinity(0)
    one = {min(before)}
    ev = threading.Event()
    th = threading.Thread(target=ev.wait, daemon=True)
    th.start()
    try:
        n = apply_binding(sorted(one))
        assert n >= 2 and os.sched_getaffinity(0) == one
        assert os.sched_getaffinity(th.native_id) == one       # an already running thread too
    finally:
        apply_binding(sorted(before))
        ev.set()
    assert os.sched_getaffinity(0) == before
