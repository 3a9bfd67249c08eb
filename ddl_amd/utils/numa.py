"""NUMA placement: keep a rank's producers, its pinned arena and its GPU on one socket.

The pinned arena's pages are first touched (and pinned) by this rank's
processes, so binding the consumer -- and, by inheritance, the producers it
spawns -- to the CPUs of the GPU's NUMA node places the DMA source next to the
GPU's PCIe root complex (no inter-socket hop on the H2D path; matters when 8
ranks stream ~50 GB/s each out of host memory).

The GPU's node is found from sysfs *without initialising HIP* (producers must be
spawned before the GPU is touched): the KFD topology lists GPU nodes in HIP
enumeration order with their DRM render minor; the render node's PCI device
gives ``numa_node``. Disable with ``DDL_NUMA_BIND=0``.
"""

from __future__ import annotations

import glob
import os

from .logging import logger

_KFD = "/sys/class/kfd/kfd/topology/nodes"


def _props(path: str) -> dict[str, int]:
    out: dict[str, int] = {}
    try:
        with open(path) as f:
            for line in f:
                parts = line.split()
                if len(parts) == 2:
                    try:
                        out[parts[0]] = int(parts[1])
                    except ValueError:
                        pass
    except OSError:
        pass
    return out


def _accessible(minor: int) -> bool:
    p = f"/dev/dri/renderD{minor}"
    try:
        fd = os.open(p, os.O_RDWR | os.O_CLOEXEC)
    except OSError:
        return False
    os.close(fd)
    return True


def visible_gpu_render_minors() -> list[int]:
    nodes = []
    for d in glob.glob(os.path.join(_KFD, "*")):
        try:
            nid = int(os.path.basename(d))
        except ValueError:
            continue
        pr = _props(os.path.join(d, "properties"))
        if pr.get("simd_count", 0) > 0 and "drm_render_minor" in pr:
            nodes.append((nid, pr["drm_render_minor"]))
    minors = [m for _, m in sorted(nodes) if _accessible(m)]
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v:
            try:
                sel = [int(x) for x in v.split(",") if x.strip()]
            except ValueError:
                return []  # UUID selectors: cannot map safely
            minors = [minors[i] for i in sel if 0 <= i < len(minors)]
    return minors


def gpu_numa_node(local_index: int) -> int | None:
    minors = visible_gpu_render_minors()
    if not 0 <= local_index < len(minors):
        return None
    try:
        with open(f"/sys/class/drm/renderD{minors[local_index]}/device/numa_node") as f:
            node = int(f.read().strip())
    except (OSError, ValueError):
        return None
    return node if node >= 0 else None


def node_cpus(node: int) -> set[int]:
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            spec = f.read().strip()
    except OSError:
        return set()
    cpus: set[int] = set()
    for part in spec.split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return cpus


def rank_cpu_slice(local_index: int, local_world: int, allowed: set[int] | None = None) -> tuple[int | None, set[int]]:
    """(node, CPUs) of this local rank: its GPU's NUMA node's allowed CPUs, split into equal contiguous
    slices among the local ranks whose GPUs sit on that node (in local-rank order), so the ranks of one
    socket do not compete for the same cores. Falls back to the whole node (one rank on it, or fewer
    CPUs than ranks) and to the allowed set when the GPU's node is unknown."""
    allowed = set(os.sched_getaffinity(0)) if allowed is None else set(allowed)
    node = gpu_numa_node(local_index)
    if node is None:
        return None, allowed
    cpus = sorted(node_cpus(node) & allowed)
    if not cpus:
        return node, allowed
    peers = [i for i in range(max(1, local_world)) if i == local_index or gpu_numa_node(i) == node]
    k, i = len(peers), peers.index(local_index)
    if k <= 1 or len(cpus) < k:
        return node, set(cpus)
    per = len(cpus) // k
    return node, set(cpus[i * per:(i + 1) * per])


def split_consumer_producers(cpus: set[int], n_producers: int, consumer_cpus: int = 4) -> tuple[set[int], set[int]]:
    """Split a rank's CPUs between its consumer (main thread, native stager / retire threads, RCCL and
    gloo helpers) and its producer processes (user hooks, native gather pools): the consumer keeps the
    first ``consumer_cpus``, the producers share the rest. Only when there are enough CPUs for both
    (at least ``consumer_cpus + 2 * n_producers``); otherwise both get all of them."""
    c = sorted(cpus)
    if n_producers < 1 or len(c) < consumer_cpus + 2 * n_producers:
        return set(c), set(c)
    return set(c[:consumer_cpus]), set(c[consumer_cpus:])


def bind_to_gpu_numa(local_index: int, local_world: int = 1) -> int | None:
    """Restrict this process's CPU affinity to its share of its GPU's NUMA node (``rank_cpu_slice``);
    return the node (or None). ``DDL_NUMA_BIND=0`` disables it, ``DDL_CPU_PARTITION=0`` keeps the whole
    node instead of a per-rank slice."""
    if os.environ.get("DDL_NUMA_BIND", "1") == "0":
        return None
    allowed = os.sched_getaffinity(0)
    if os.environ.get("DDL_CPU_PARTITION", "1") == "0":
        local_world = 1
    node, cpus = rank_cpu_slice(local_index, local_world, allowed)
    if node is None:
        return None
    if not cpus or cpus == allowed:
        return node
    os.sched_setaffinity(0, cpus)
    logger.debug("bound to NUMA node %d (%d CPUs) for GPU %d", node, len(cpus), local_index)
    return node


def partition_after_spawn(producer_pids: list[int], n_producers: int) -> dict | None:
    """After the producers are spawned (they inherited this rank's CPU slice): move the producers off the
    first CPUs of the slice (``split_consumer_producers``), which stay free for the consumer's loader
    threads (native stager / retire, RCCL proxy, gloo). The consumer process itself keeps the WHOLE
    slice: it is the user's training process, and narrowing it would also confine the user's main thread,
    torch's intra-op pool and any workers it spawns later. Returns the layout, or None when not
    partitioned. ``DDL_CPU_PARTITION=0`` disables it."""
    if os.environ.get("DDL_CPU_PARTITION", "1") == "0" or not producer_pids:
        return None
    mine = os.sched_getaffinity(0)
    cons, prod = split_consumer_producers(mine, n_producers)
    if cons == prod:
        return None
    for pid in producer_pids:
        try:
            os.sched_setaffinity(pid, prod)
        except OSError:
            return None
    logger.info("CPU layout: consumer process keeps %d CPUs (%d kept free of producers), %d producers on %d CPUs",
                len(mine), len(cons), len(producer_pids), len(prod))
    return {"consumer_cpus": sorted(mine), "consumer_reserved_cpus": sorted(cons), "producer_cpus": sorted(prod)}
