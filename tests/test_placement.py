"""NUMA placement of the replicas (VERDICT r03 next #4a) against a fake sysfs tree:
an 8-GPU node, 2 sockets x 64 cores, 4 GPUs per socket (the MI355X platform shape)."""
from __future__ import annotations

import os

import pytest

from smsgate_amd.parallel.placement import format_cpulist, gpu_topology, parse_cpulist, plan


def _fake_node(root, gpus=8, per_socket=4, cores=64):
    kfd = root / "class/kfd/kfd/topology/nodes"
    # KFD lists the CPU sockets first (no SIMDs), then the GPUs
    for n in range(2):
        d = kfd / str(n)
        d.mkdir(parents=True)
        (d / "properties").write_text(f"cpu_cores_count {cores}\nsimd_count 0\nlocation_id 0\ndomain 0\n")
    for g in range(gpus):
        d = kfd / str(2 + g)
        d.mkdir(parents=True)
        bus = 0x05 + 0x10 * g
        (d / "properties").write_text(f"cpu_cores_count 0\nsimd_count 1024\nlocation_id {bus << 8}\ndomain 0\n"
                                      "gfx_target_version 90500\n")
        pci = root / "bus/pci/devices" / f"0000:{bus:02x}:00.0"
        pci.mkdir(parents=True)
        sock = g // per_socket
        (pci / "numa_node").write_text(f"{sock}\n")
        (pci / "local_cpulist").write_text(f"{sock * cores}-{sock * cores + cores - 1}\n")
    return str(root)


def test_cpulist_roundtrip():
    assert parse_cpulist("0-3,8,10-11\n") == [0, 1, 2, 3, 8, 10, 11]
    assert format_cpulist([11, 0, 1, 2, 3, 8, 10]) == "0-3,8,10-11"


def test_topology_in_hip_order(tmp_path):
    root = _fake_node(tmp_path)
    g = gpu_topology(root, env={}, allowed=range(128))
    assert [x.index for x in g] == list(range(8)) and [x.kfd_node for x in g] == list(range(2, 10))
    assert g[0].bdf == "0000:05:00.0" and g[5].numa_node == 1 and g[5].cpus[0] == 64
    vis = gpu_topology(root, env={"HIP_VISIBLE_DEVICES": "4,5"}, allowed=range(128))
    assert [(x.index, x.bdf) for x in vis] == [(0, "0000:45:00.0"), (1, "0000:55:00.0")]


def test_eight_rank_plan_is_numa_local_and_disjoint(tmp_path):
    root = _fake_node(tmp_path)
    plans = [plan(r, 8, broker_cores=2, sysfs=root, env={}, allowed=range(128)) for r in range(8)]
    used = set()
    for r, p in enumerate(plans):
        sock = r // 4
        node = set(range(sock * 64, sock * 64 + 64))
        mine = set(p.rank_cpus) | set(p.worker_cpus)
        assert p.numa_node == sock and mine <= node  # every process of the replica on its GPU's socket
        assert len(p.rank_cpus) >= 2 and len(p.worker_cpus) >= 8
        assert not (mine & used)  # replicas never share a core
        used |= mine
    assert plans[0].broker_cpus == [62, 63] and not (set(plans[0].broker_cpus) & used)
    assert all(not p.broker_cpus for p in plans[1:]) and plans[4].ranks_on_numa == 4


def test_plan_without_topology_is_none(tmp_path):
    assert plan(0, 1, sysfs=str(tmp_path), env={}) is None


def test_apply_pins_this_process(tmp_path):
    root = _fake_node(tmp_path, gpus=1, per_socket=1, cores=len(os.sched_getaffinity(0)))
    allowed = sorted(os.sched_getaffinity(0))
    p = plan(0, 1, broker_cores=0, sysfs=root, env={}, allowed=allowed)
    before = os.sched_getaffinity(0)
    try:
        p.apply(rank_pid=0)
        assert os.sched_getaffinity(0) == set(p.rank_cpus)
    finally:
        os.sched_setaffinity(0, before)
    assert p.describe()["rank_cpus"] == format_cpulist(p.rank_cpus)


@pytest.mark.parametrize("world", [1, 2, 4])
def test_partial_node(tmp_path, world):
    root = _fake_node(tmp_path)
    ps = [plan(r, world, sysfs=root, env={}, allowed=range(128)) for r in range(world)]
    assert all(p is not None and p.numa_node == 0 for p in ps)
    assert all(len(p.rank_cpus) >= 2 for p in ps)
    assert not set.intersection(*(set(p.rank_cpus) | set(p.worker_cpus) for p in ps)) if world > 1 else True
