"""NUMA placement (include/nxec.h, nexoedge_amd/csrc/nxec_numa.cpp): GPU ->
PCI numa_node -> node cpulist -> thread affinity, on a fake sysfs tree
(NXEC_SYSFS_ROOT).  CPU only; the binding itself runs in a child process so
the test runner's own affinity is never touched."""
import os
import subprocess
import sys

import pytest

from nexoedge_amd import _lib, nxec

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def fake_sysfs(tmp_path, nodes, devices):
    """nodes: {node: cpulist text}; devices: {bus id: numa_node text}"""
    for node, cpulist in nodes.items():
        d = tmp_path / "sys" / "devices" / "system" / "node" / f"node{node}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpulist + "\n")
    for bus, nd in devices.items():
        d = tmp_path / "sys" / "bus" / "pci" / "devices" / bus
        d.mkdir(parents=True)
        (d / "numa_node").write_text(nd + "\n")
    return str(tmp_path)


@pytest.fixture
def sysfs(tmp_path, monkeypatch):
    cpus = sorted(os.sched_getaffinity(0))
    half = len(cpus) // 2 or 1
    lst = lambda cs: ",".join(str(c) for c in cs)  # noqa: E731
    root = fake_sysfs(tmp_path, {0: "0-3,8-11", 1: "4-7,12-15", 2: lst(cpus[:half]), 3: lst(cpus[half:]) or lst(cpus),
                                 5: "9999"},
                      {"0000:05:00.0": "0", "0000:c1:00.0": "1", "0000:11:00.0": "-1", "0000:22:00.0": "2",
                       "0000:33:00.0": "3", "0000:44:00.0": "5"})
    monkeypatch.setenv("NXEC_SYSFS_ROOT", root)
    return root, cpus[:half], cpus[half:] or cpus


def test_gpu_to_node_mapping(sysfs):
    assert nxec.pci_numa_node("0000:05:00.0") == 0
    assert nxec.pci_numa_node("0000:C1:00.0") == 1  # hipDeviceGetPCIBusId may print upper-case hex
    assert nxec.pci_numa_node("0000:11:00.0") == -1  # sysfs: unknown
    assert nxec.pci_numa_node("0000:99:00.0") == -1  # no such device


def test_node_to_cpus(sysfs):
    assert nxec.numa_node_cpus(0) == [0, 1, 2, 3, 8, 9, 10, 11]
    assert nxec.numa_node_cpus(1) == [4, 5, 6, 7, 12, 13, 14, 15]
    with pytest.raises(nxec.NxecError):
        nxec.numa_node_cpus(7)


CHILD = r"""
import os, sys
sys.path.insert(0, {root!r})
from nexoedge_amd import nxec
before = sorted(os.sched_getaffinity(0))
node = nxec.bind_thread_pci(sys.argv[1])
print(node, ",".join(map(str, sorted(os.sched_getaffinity(0)))), ",".join(map(str, before)))
"""


def _bind(sysfs_root, bus):
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT), bus], capture_output=True, text=True,
                       env=dict(os.environ, NXEC_SYSFS_ROOT=sysfs_root), timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    node, after, before = r.stdout.split()
    return int(node), [int(x) for x in after.split(",")], [int(x) for x in before.split(",")]


def test_bind_to_the_gpus_node(sysfs):
    root, lo, hi = sysfs
    node, after, before = _bind(root, "0000:22:00.0")
    assert node == 2 and after == lo
    node, after, _ = _bind(root, "0000:33:00.0")
    assert node == 3 and after == hi


def test_bind_leaves_affinity_alone_when_unknown_or_disjoint(sysfs):
    root, _, _ = sysfs
    for bus in ("0000:11:00.0", "0000:99:00.0", "0000:44:00.0"):  # unknown node, no device, CPUs outside the mask
        node, after, before = _bind(root, bus)
        assert node == -1 and after == before


def test_bench_records_a_node_per_rank():
    """bench.py binds each rank before it allocates anything and reports the
    node of every rank (numa_node_per_rank); the dry run exercises the gather."""
    from nexoedge_amd.dist import RankGroup

    g = RankGroup()
    assert g.gather(3) == [3.0]
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert "bind_thread_numa(dev)" in src and src.index("bind_thread_numa(dev)") < src.index("ctx = nxec.Context(dev)")
    assert _lib.lib.nxec_bind_thread_to_device(0, None) in (_lib.NXEC_OK, _lib.NXEC_ERR_NODEV, _lib.NXEC_ERR_HIP)
