"""CPU placement of a replica: pin each GPU's rank process and parser workers to the
cores of that GPU's NUMA node, and the node's brokers to a reserved set.

Each MI355X hangs off one socket / NUMA node.  A replica's host work -- the rank
process feeding the GPU (engine launches, IPC with its parser processes) and its
parser processes (bus I/O, tokenisation, post-processing) -- crosses the socket
interconnect on every message when the scheduler places it on the far socket, and
8 ranks x (1 + K) processes left unpinned migrate freely.  The reference runs one
container per service and leaves placement to Docker (docker-compose.yml:81-104);
here the layout is computed from the kernel's own topology:

* GPUs in HIP order = KFD topology nodes with SIMDs
  (``/sys/class/kfd/kfd/topology/nodes/*/properties``: ``simd_count``,
  ``location_id`` = bus << 8 | dev << 3 | fn, ``domain``), filtered by
  ``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` when they are indices;
* each GPU's NUMA node and local CPUs from its PCI device
  (``/sys/bus/pci/devices/<dddd:bb:dd.f>/numa_node``, ``local_cpulist``),
  intersected with this process's allowed CPUs;
* the ranks whose GPUs share a NUMA node split its cores into equal contiguous
  slices; in each slice the first quarter (at least 2 cores) runs the rank process
  and the rest the parser workers; local rank 0's node gives up ``broker_cores``
  cores (its last ones) to the node's brokers first.

:func:`plan` returns a :class:`Placement` (or None when the topology is not
readable, e.g. no GPU driver); :meth:`Placement.apply` sets the affinities.
``tests/test_placement.py`` runs it against a fake sysfs tree of an 8-GPU,
2-socket node.
"""
from __future__ import annotations

import os
from dataclasses import asdict, dataclass, field
from pathlib import Path
from typing import Dict, Iterable, List, Optional, Sequence

__all__ = ["GpuInfo", "Placement", "gpu_topology", "plan", "parse_cpulist", "format_cpulist"]


@dataclass
class GpuInfo:
    index: int  # HIP device ordinal
    kfd_node: int
    bdf: str
    numa_node: int
    cpus: List[int]


@dataclass
class Placement:
    local_rank: int
    numa_node: int
    gpu_bdf: str
    rank_cpus: List[int]
    worker_cpus: List[int]
    broker_cpus: List[int] = field(default_factory=list)
    ranks_on_numa: int = 1

    def apply(self, rank_pid: int = 0, worker_pids: Iterable[int] = (), broker_pids: Iterable[int] = ()) -> None:
        """Pin the processes (0 = this one).  A process that already exited is skipped."""
        for pids, cpus in ((worker_pids, self.worker_cpus or self.rank_cpus), (broker_pids, self.broker_cpus)):
            if not cpus:
                continue
            for pid in pids:
                try:
                    os.sched_setaffinity(pid, cpus)
                except ProcessLookupError:
                    pass
        if self.rank_cpus:
            os.sched_setaffinity(rank_pid, self.rank_cpus)

    def describe(self) -> Dict[str, object]:
        d = asdict(self)
        for k in ("rank_cpus", "worker_cpus", "broker_cpus"):
            d[k] = format_cpulist(d[k])
        return d


def parse_cpulist(text: str) -> List[int]:
    """``"0-3,8,10-11"`` -> ``[0, 1, 2, 3, 8, 10, 11]``."""
    out: List[int] = []
    for part in text.strip().split(","):
        part = part.strip()
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-", 1)
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def format_cpulist(cpus: Sequence[int]) -> str:
    cpus = sorted(set(cpus))
    out, i = [], 0
    while i < len(cpus):
        j = i
        while j + 1 < len(cpus) and cpus[j + 1] == cpus[j] + 1:
            j += 1
        out.append(str(cpus[i]) if i == j else f"{cpus[i]}-{cpus[j]}")
        i = j + 1
    return ",".join(out)


def _props(path: Path) -> Dict[str, int]:
    out: Dict[str, int] = {}
    for line in path.read_text().splitlines():
        parts = line.split()
        if len(parts) == 2:
            try:
                out[parts[0]] = int(parts[1])
            except ValueError:
                pass
    return out


def _visible(env: Dict[str, str]) -> Optional[List[int]]:
    for k in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(k)
        if v:
            try:
                return [int(x) for x in v.split(",") if x.strip()]
            except ValueError:
                return None  # UUIDs: no index mapping from sysfs; treat every GPU as visible
    return None


def gpu_topology(sysfs: str = "/sys", env: Optional[Dict[str, str]] = None,
                 allowed: Optional[Sequence[int]] = None) -> List[GpuInfo]:
    """GPUs in HIP device order with their NUMA node and (allowed) local CPUs."""
    env = dict(os.environ) if env is None else env
    root = Path(sysfs) / "class/kfd/kfd/topology/nodes"
    if not root.is_dir():
        return []
    allowed_set = set(allowed) if allowed is not None else set(os.sched_getaffinity(0))
    nodes = sorted((int(p.name), p) for p in root.iterdir() if p.name.isdigit())
    gpus: List[GpuInfo] = []
    for nid, p in nodes:
        try:
            pr = _props(p / "properties")
        except OSError:
            continue
        if pr.get("simd_count", 0) <= 0:
            continue
        loc = pr.get("location_id", 0)
        bdf = f"{pr.get('domain', 0):04x}:{(loc >> 8) & 0xFF:02x}:{(loc >> 3) & 0x1F:02x}.{loc & 0x7:x}"
        dev = Path(sysfs) / "bus/pci/devices" / bdf
        try:
            numa = int((dev / "numa_node").read_text().strip())
        except (OSError, ValueError):
            numa = -1
        try:
            cpus = [c for c in parse_cpulist((dev / "local_cpulist").read_text()) if c in allowed_set]
        except OSError:
            cpus = sorted(allowed_set)
        gpus.append(GpuInfo(len(gpus), nid, bdf, max(numa, 0), cpus or sorted(allowed_set)))
    vis = _visible(env)
    if vis is not None:
        gpus = [g for g in gpus if g.index in vis]
        for i, g in enumerate(gpus):
            g.index = i
    return gpus


def plan(local_rank: int, local_world: int, broker_cores: int = 2, sysfs: str = "/sys",
         env: Optional[Dict[str, str]] = None, allowed: Optional[Sequence[int]] = None) -> Optional[Placement]:
    """Placement of ``local_rank`` (one rank per GPU, ranks 0..local_world-1 on
    GPUs 0..local_world-1).  None when the GPU topology is unreadable."""
    gpus = gpu_topology(sysfs, env, allowed)
    if local_rank >= len(gpus) or local_world > len(gpus):
        return None
    mine = gpus[local_rank]
    peers = [g for g in gpus[:local_world] if g.numa_node == mine.numa_node]
    cores = list(mine.cpus)
    brokers: List[int] = []
    if broker_cores > 0 and gpus[0].numa_node == mine.numa_node and len(cores) > broker_cores + len(peers):
        brokers = cores[-broker_cores:]
        cores = cores[:-broker_cores]
    slot = [g.index for g in peers].index(mine.index)
    per = max(1, len(cores) // len(peers))
    chunk = cores[slot * per:(slot + 1) * per] if len(cores) >= len(peers) else cores
    # the rank process is multi-threaded (the launch loop, torch's pool, the HIP runtime's
    # threads: ~1.8 cores busy at the r03 rate): a quarter of the slice, at least 2 cores
    nr = min(len(chunk), max(2, len(chunk) // 4))
    rank_cpus = chunk[:nr]
    worker_cpus = chunk[nr:] or chunk
    return Placement(local_rank, mine.numa_node, mine.bdf, rank_cpus, worker_cpus,
                     brokers if local_rank == 0 else [], len(peers))
