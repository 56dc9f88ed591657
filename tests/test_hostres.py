"""Per-rank host resources (utils/hostres.py): CPU sets on the GPU's NUMA node, thread budgets per rank
(reference: one core per executor, /root/reference/ml_ops.sh:57,108)."""
import os
import subprocess
import sys
from types import SimpleNamespace

from oni_ml_amd.utils import hostres

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parse_cpulist():
    assert hostres.parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert hostres.parse_cpulist("") == []


def test_plan_splits_node_cpus_between_its_ranks():
    allowed = list(range(32))
    # 8 GPUs on 2 NUMA nodes (4 each), 16 CPUs per node
    nodes = {r: (r // 4, list(range(16 * (r // 4), 16 * (r // 4) + 16))) for r in range(8)}
    sets = [hostres.plan_cpus(r, 8, allowed, nodes.__getitem__) for r in range(8)]
    assert sets[0] == [0, 1, 2, 3] and sets[5] == [20, 21, 22, 23]
    flat = sorted(c for s in sets for c in s)
    assert flat == allowed                                   # disjoint, covering
    for r, s in enumerate(sets):
        assert set(s) <= set(nodes[r][1])                    # on the GPU's own node
    # a restricted allowed set: only the node's allowed CPUs are used
    sets = [hostres.plan_cpus(r, 8, range(0, 32, 2), nodes.__getitem__) for r in range(8)]
    assert sets[0] == [0, 2] and all(len(s) == 2 for s in sets)


def test_plan_without_topology_slices_allowed():
    sets = [hostres.plan_cpus(r, 8, range(64), None) for r in range(8)]
    assert sets[2] == list(range(16, 24)) and sorted(c for s in sets for c in s) == list(range(64))
    # a node the sysfs does not report (-1) falls back to the slices
    none = lambda r: (None, [])                               # noqa: E731
    assert hostres.plan_cpus(3, 4, range(8), none) == [6, 7]
    # more ranks than CPUs: every rank keeps the allowed set
    assert hostres.plan_cpus(5, 16, range(8), None) == list(range(8))


def test_gpu_node_cpus_from_sysfs(tmp_path):
    d = tmp_path / "0000:c1:00.0"
    d.mkdir()
    (d / "numa_node").write_text("1\n")
    (d / "local_cpulist").write_text("48-95,144-191\n")
    props = SimpleNamespace(pci_domain_id=0, pci_bus_id=0xC1, pci_device_id=0)
    node, cpus = hostres.gpu_node_cpus(props, root=str(tmp_path))
    assert node == 1 and cpus[:2] == [48, 49] and len(cpus) == 96
    assert hostres.gpu_node_cpus(SimpleNamespace(pci_domain_id=0, pci_bus_id=1, pci_device_id=0),
                                 root=str(tmp_path)) == (None, [])


def test_local_world_8_pools_and_affinity():
    """LOCAL_WORLD_SIZE=8 on this host: every rank's affinity mask is its own slice, and the pools it
    sizes (knobs.threads, torch's intra-op pool, RunConfig.threads) fit the slice."""
    code = """
import os, json, torch
from oni_ml_amd import knobs, config
from oni_ml_amd.parallel import dist as D
ctx = D.init_from_env()
cfg = config.resolve('20160122', 'flow', conf_path=None)
print(json.dumps(dict(aff=sorted(os.sched_getaffinity(0)), t16=knobs.threads(16), t8=knobs.threads(8),
                      torch=torch.get_num_threads(), cfg=cfg.threads)))
"""
    import json
    allowed = hostres.host_cpus()
    assert set(allowed) == set(os.sched_getaffinity(0))          # this container: no narrower mask
    n = 8
    got = []
    for r in range(n):
        env = dict(os.environ, PYTHONPATH=ROOT, LOCAL_WORLD_SIZE=str(n), LOCAL_RANK=str(r), WORLD_SIZE="1", RANK="0")
        env.pop("ONI_THREADS", None)
        out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True,
                             timeout=300)
        assert out.returncode == 0, out.stderr[-2000:]
        got.append(json.loads(out.stdout.strip().splitlines()[-1]))
    want = [hostres.plan_cpus(r, n, allowed, None) for r in range(n)]
    for r in range(n):
        k = len(want[r])
        assert got[r]["aff"] == want[r]
        assert got[r]["t16"] == min(16, k) and got[r]["t8"] == min(8, k) and got[r]["cfg"] == min(8, k)
        assert got[r]["torch"] == k
    if len(allowed) >= n:
        assert sorted(c for g in got for c in g["aff"]) == allowed     # disjoint slices of the host
    # a child of a bound rank binding again (bench.py's cold ml_ops child) keeps the parent's set
    child = f"""
import os, subprocess, sys
from oni_ml_amd.utils import hostres
hostres.bind_rank(5)
print(subprocess.run([sys.executable, '-c', {code!r}], capture_output=True, text=True, check=True).stdout)
"""
    env = dict(os.environ, PYTHONPATH=ROOT, LOCAL_WORLD_SIZE=str(n), LOCAL_RANK="5")
    env.pop("ONI_THREADS", None)
    out = subprocess.run([sys.executable, "-c", child], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert json.loads(out.stdout.strip().splitlines()[-1])["aff"] == want[5]
    # an explicit ONI_THREADS leaves the mask and sizes the pools
    env = dict(os.environ, PYTHONPATH=ROOT, LOCAL_WORLD_SIZE=str(n), LOCAL_RANK="1", ONI_THREADS="3")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    g = json.loads(out.stdout.strip().splitlines()[-1])
    assert g["aff"] == allowed and g["t16"] == 3 and g["cfg"] == 3


def test_cpu_quota_caps_the_budget(monkeypatch):
    """A cgroup CPU quota smaller than the visible CPUs (the GPU boxes) caps every rank's share."""
    monkeypatch.setattr(hostres, "quota_cpus", lambda: 16.0)
    monkeypatch.setattr(hostres, "allowed_cpus", lambda: list(range(192)))
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setattr(hostres, "_BOUND", None)
    assert hostres.cpu_budget() == 2
    monkeypatch.setattr(hostres, "_BOUND", list(range(24)))
    assert hostres.cpu_budget() == 2
    monkeypatch.setattr(hostres, "quota_cpus", lambda: None)
    assert hostres.cpu_budget() == 24
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    monkeypatch.setattr(hostres, "_BOUND", None)
    monkeypatch.setattr(hostres, "quota_cpus", lambda: 16.0)
    assert hostres.cpu_budget() == 16


def test_background_writers_share_one_thread_pool(tmp_path):
    """Native calls on background writer threads (ops/native.background_thread_budget) draw their worker
    threads from one process-wide pool of budget - WRITER_RESERVE tokens; every token comes back, and the
    files are the same as a foreground write's."""
    import threading
    import numpy as np
    from oni_ml_amd.io import ldac
    from oni_ml_amd.ops import native
    L = native.lib()
    native.apply_thread_budget()
    free0 = L.background_pool_free()
    assert free0 >= 1
    g = np.random.default_rng(0).random((20000, 24))
    ldac.save_gamma(str(tmp_path / "fg.gamma"), g)
    errs = []

    def writer(i):
        try:
            native.background_thread_budget(2)
            ldac.save_gamma(str(tmp_path / f"bg{i}.gamma"), g)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=writer, args=(i,)) for i in range(3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs and L.background_pool_free() == free0
    ref = (tmp_path / "fg.gamma").read_bytes()
    assert all((tmp_path / f"bg{i}.gamma").read_bytes() == ref for i in range(3))
