"""Per-rank host resources: CPU affinity on the GPU's NUMA node and a thread budget per rank.

The reference sizes every worker explicitly -- ``--num-executors``, ``--executor-cores 1`` and
``--executor-memory`` (/root/reference/ml_ops.sh:57,108), 62 executors x 12 cores
(/root/reference/dns_pre_lda.scala:1-2).  Here the workers are the N ranks of one node (one per GPU,
torchrun): without a budget each would size its native pools (ingest, formatters, the C++ engine) for
the whole host, N x oversubscribed, and float over sockets away from its GPU.

``bind_rank`` (called by parallel/dist.init_from_env) gives each rank:

- the CPUs of its GPU's NUMA node (sysfs ``/sys/bus/pci/devices/<pci id>/local_cpulist`` from the
  device's PCI domain / bus / device ids), split evenly between the local ranks whose GPUs sit on that
  node (by local rank order), intersected with the CPUs the process may use;
- without GPU topology (CPU ranks, gloo rehearsals, a sysfs that reports no node): the host's CPUs
  cut into LOCAL_WORLD_SIZE contiguous slices, slice ``local_rank``;
- planned over the host's CPUs (cgroup cpuset), then intersected with the process's affinity, so a
  child of a bound rank that binds again keeps its parent's set;
- ``torch.set_num_threads`` to that CPU count (at most its share of the cgroup's CPU quota).

``cpu_budget()`` is what every pool sizes itself from (knobs.threads): the bound set's size, or the
allowed CPUs divided by LOCAL_WORLD_SIZE when nothing was bound.  An explicit ONI_THREADS wins and
turns the binding off (the operator sizes the host).
"""
from __future__ import annotations

import os
from typing import Callable, List, Optional, Sequence

_BOUND: Optional[List[int]] = None   # the CPU set bind_rank applied (None: not bound)


def local_world() -> int:
    return max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))


def allowed_cpus() -> List[int]:
    try:
        return sorted(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return list(range(os.cpu_count() or 1))


def host_cpus() -> List[int]:
    """The CPUs this host (its cgroup cpuset) gives the job -- not the calling process's affinity, which an
    earlier bind_rank (a parent rank of this process: bench.py's cold ml_ops child) may already have
    narrowed, so planning over it is idempotent: a child re-binding gets its parent's set."""
    for p in ("/sys/fs/cgroup/cpuset.cpus.effective", "/sys/fs/cgroup/cpuset/cpuset.effective_cpus",
              "/sys/fs/cgroup/cpuset/cpuset.cpus"):
        try:
            with open(p) as f:
                cpus = parse_cpulist(f.read())
            if cpus:
                return cpus
        except (OSError, ValueError):
            pass
    return list(range(os.cpu_count() or 1))


def quota_cpus() -> Optional[float]:
    """CPUs the cgroup's CFS quota allows (cgroup v2 cpu.max, v1 cpu.cfs_quota_us / cpu.cfs_period_us), or
    None without a quota.  A container can see every CPU of the host in its cpuset and still run on a
    fraction of them (the GPU boxes: the whole machine visible, a 16-CPU share)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = float(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = float(f.read())
        return None if q <= 0 or per <= 0 else q / per
    except (OSError, ValueError):
        return None


def cpu_budget() -> int:
    """Host threads this rank's pools may use: its bound CPUs (else the allowed CPUs / LOCAL_WORLD_SIZE),
    at most its share of the cgroup's CPU quota."""
    n = len(_BOUND) if _BOUND is not None else len(allowed_cpus()) // local_world()
    q = quota_cpus()
    if q is not None:
        n = min(n, int(q // local_world()))
    return max(1, n)


def parse_cpulist(text: str) -> List[int]:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11]."""
    out = []
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        a, _, b = part.partition("-")
        out.extend(range(int(a), int(b or a) + 1))
    return out


def pci_path(domain: int, bus: int, device: int, root: str = "/sys/bus/pci/devices") -> str:
    return os.path.join(root, f"{domain:04x}:{bus:02x}:{device:02x}.0")


def gpu_node_cpus(props, root: str = "/sys/bus/pci/devices"):
    """(NUMA node, its CPU list) of a GPU from its device properties (pci_domain_id / pci_bus_id /
    pci_device_id); (None, []) when sysfs does not say."""
    try:
        p = pci_path(int(props.pci_domain_id), int(props.pci_bus_id), int(props.pci_device_id), root)
        with open(os.path.join(p, "numa_node")) as f:
            node = int(f.read().strip())
        with open(os.path.join(p, "local_cpulist")) as f:
            cpus = parse_cpulist(f.read())
    except (OSError, ValueError, AttributeError):
        return None, []
    return (node if node >= 0 else None), cpus


def plan_cpus(local_rank: int, nlocal: int, allowed: Sequence[int],
              node_cpus_of: Optional[Callable[[int], tuple]] = None) -> List[int]:
    """The CPU set of local rank ``local_rank`` of ``nlocal``: its GPU node's allowed CPUs, split evenly
    between the ranks on that node; else slice ``local_rank`` of ``allowed`` cut into ``nlocal``.
    ``node_cpus_of(r)`` -> (node, cpus) of local rank r's GPU (gpu_node_cpus)."""
    allowed = sorted(set(allowed))
    nlocal = max(1, nlocal)
    if node_cpus_of is not None:
        nodes = [node_cpus_of(r) for r in range(nlocal)]
        node, cpus = nodes[local_rank]
        mine = sorted(set(cpus) & set(allowed))
        if node is not None and mine:
            peers = [r for r in range(nlocal) if nodes[r][0] == node]
            k, i = len(peers), peers.index(local_rank)
            if len(mine) >= k:
                return mine[i * len(mine) // k:(i + 1) * len(mine) // k]
            return mine
    if len(allowed) < nlocal:
        return allowed
    return allowed[local_rank * len(allowed) // nlocal:(local_rank + 1) * len(allowed) // nlocal]


def bind_rank(local_rank: int, device=None) -> List[int]:
    """Pin this process to its planned CPU set and size torch's intra-op pool to it (best effort:
    a refused sched_setaffinity leaves the process as it was and only the budget applies)."""
    global _BOUND
    nlocal = local_world()
    if nlocal <= 1 and _BOUND is None:
        return allowed_cpus()                # one rank: the whole host, nothing to divide
    node_of = None
    if device is not None and getattr(device, "type", "") == "cuda":
        import torch
        n = torch.cuda.device_count()
        if n >= nlocal:
            node_of = lambda r: gpu_node_cpus(torch.cuda.get_device_properties(r))   # noqa: E731
    allowed = allowed_cpus()
    cpus = [c for c in plan_cpus(local_rank, nlocal, host_cpus(), node_of) if c in set(allowed)] or allowed
    try:
        os.sched_setaffinity(0, cpus)
    except (AttributeError, OSError):
        pass
    _BOUND = list(cpus)
    from ..ops import native
    native.apply_thread_budget()             # the native pools' default, if the module is loaded
    try:
        import torch
        torch.set_num_threads(cpu_budget())
    except Exception:  # noqa: BLE001 -- torch's pool may already be running; the budget still applies
        pass
    return _BOUND


def reset() -> None:
    """Forget the bound set (tests)."""
    global _BOUND
    _BOUND = None
