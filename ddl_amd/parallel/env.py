"""Topology / process-environment bootstrap (reference ddl/ddl_env.py:12-97).

The reference derives its layout from ``mpirun`` ranks: contiguous blocks of
``size/n_instances`` ranks per GPU, four communicator splits, and an
``Abort(1)`` when the sizes do not divide (reference ddl/ddl_env.py:12-97).

Here one process per MI355X is the DP rank (torchrun / srun task); its
producers are child processes, so there is nothing to split. The rank math
comes from the environment (torchrun ``RANK/WORLD_SIZE/LOCAL_RANK/
LOCAL_WORLD_SIZE``, falling back to SLURM ``SLURM_PROCID/SLURM_NTASKS/
SLURM_LOCALID``), the DP group is a torch.distributed group -- RCCL (backend
"nccl") on GPUs, gloo on CPU -- plus a gloo *control* group for host-side
metadata, and the node-locality check of the reference's
``Split_type(COMM_TYPE_SHARED)`` becomes a hostname all-gather.
"""

from __future__ import annotations

import os
import socket
from datetime import timedelta

from ..exceptions import TopologyError
from ..types import DDLEnv
from ..utils.logging import logger

DEFAULT_PRODUCERS = 3  # the reference's CI layout: mpirun -np 4 = 1 consumer + 3 producers


def _int_env(*names: str, default: int | None = None) -> int | None:
    for n in names:
        v = os.environ.get(n)
        if v not in (None, ""):
            try:
                return int(v.split("(")[0].split(",")[0])
            except ValueError:
                raise TopologyError(v, f"environment variable {n}={v!r} is not an integer") from None
    return default


def read_env(n_producers: int | None = None) -> DDLEnv:
    """Compute the rank layout from the environment (no GPU, no communication)."""
    rank = _int_env("RANK", "SLURM_PROCID", default=0)
    world = _int_env("WORLD_SIZE", "SLURM_NTASKS", default=1)
    local_rank = _int_env("LOCAL_RANK", "SLURM_LOCALID", default=0)
    local_world = _int_env("LOCAL_WORLD_SIZE", "SLURM_NTASKS_PER_NODE", default=None)
    if local_world is None:
        local_world = world if _int_env("SLURM_NNODES", default=1) == 1 else 1
    assert rank is not None and world is not None and local_rank is not None
    if world < 1 or not 0 <= rank < world:
        raise TopologyError((rank, world), f"invalid rank {rank} for world size {world}")
    if not 0 <= local_rank < max(local_world, 1):
        raise TopologyError((local_rank, local_world), f"invalid local rank {local_rank} of {local_world}")
    if world % max(local_world, 1) != 0:
        raise TopologyError((world, local_world),
                            f"world size {world} is not a multiple of the ranks per node {local_world}")
    if n_producers is None:
        n_producers = _int_env("DDL_PRODUCERS_PER_RANK", default=DEFAULT_PRODUCERS)
    assert n_producers is not None
    if n_producers < 0:
        raise TopologyError(n_producers, "number of producers must be >= 0")
    return DDLEnv(
        rank=rank,
        world_size=world,
        local_rank=local_rank,
        local_world_size=local_world,
        node_rank=rank // max(local_world, 1),
        n_producers=n_producers,
        # DDL_HOSTNAME overrides the node identity (containers with unreliable hostnames, and the
        # multi-node rehearsal tests that run several "nodes" on one box)
        hostname=os.environ.get("DDL_HOSTNAME") or socket.gethostname(),
    )


_VISIBILITY_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL")


def rehearsal() -> bool:
    """``DDL_REHEARSAL=1``: this multi-rank run is a rehearsal (several ranks on one GPU over gloo, or ranks
    on the CPU), not a measurement of N GPUs. Without it a layout that shares a device is refused
    (:func:`check_device_count`, :func:`check_node_locality`) and ``bench.py`` exits non-zero at N > 1 unless
    the DP group is RCCL over N distinct GPUs."""
    return os.environ.get("DDL_REHEARSAL", "0") == "1"


def check_device_count(env: DDLEnv, n_dev: int) -> None:
    """Raise ``TopologyError`` when this node has more ranks than visible GPUs: ``local_rank % n_dev`` would
    wrap and put two ranks on one device silently (gloo runs that way; RCCL fails later with "Duplicate GPU").

    With a ``*_VISIBLE_DEVICES`` mask (per-task GPU isolation, e.g. SLURM ``--gpus-per-task``) every rank
    legitimately sees fewer devices than the node has ranks; the PCI-bus-ID all-gather of
    :func:`check_node_locality` then catches a shared device instead."""
    if env.local_world_size <= n_dev or rehearsal():
        return
    if n_dev >= 1 and any(os.environ.get(v) for v in _VISIBILITY_VARS):
        return
    raise TopologyError((env.local_world_size, n_dev),
                        f"{env.local_world_size} ranks on host {env.hostname} but only {n_dev} visible GPU(s): ranks "
                        "would share a device. One rank per GPU; set DDL_REHEARSAL=1 for a deliberate rehearsal")


def device_identity(device: str | None) -> dict:
    """PCI location and UUID of ``device`` (``{}`` on the CPU): the key that tells two GPUs apart even when
    per-task visibility masks make every rank call its GPU ``cuda:0``."""
    if not device or not str(device).startswith("cuda"):
        return {}
    import torch

    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    p = torch.cuda.get_device_properties(idx)
    bus = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
    uuid = str(getattr(p, "uuid", "") or "")
    return {"device_index": idx, "pci_bus_id": bus, "uuid": uuid, "name": p.name,
            "arch": getattr(p, "gcnArchName", "")}


_CLAIMED: dict = {}  # PCI bus ID -> fd of the held lock (kept open for the life of the process)


def claim_device(env: DDLEnv) -> None:
    """Take this job's exclusive claim on the rank's GPU before any group exists: a non-blocking ``flock`` on
    a per-job, per-PCI-bus-ID file in the node's temp directory. A second rank of the same job that lands on
    the same GPU (a wrapped index, a visibility mask handing every task the same device) gets a
    ``TopologyError`` naming the holder, instead of RCCL's "Duplicate GPU" deep inside the first collective or
    gloo's silent sharing. The kernel drops the lock when the process exits. Skipped under
    ``DDL_REHEARSAL=1``."""
    import fcntl
    import tempfile
    import zlib

    if rehearsal():
        return
    bus = device_identity(env.device).get("pci_bus_id")
    if not bus or bus in _CLAIMED:
        return
    job = f"{os.environ.get('MASTER_ADDR', '')}:{os.environ.get('MASTER_PORT', '')}"
    path = os.path.join(tempfile.gettempdir(),
                        f"ddl_amd_gpu_{bus.replace(':', '_')}_{zlib.crc32(job.encode()):08x}.lock")
    try:
        fd = os.open(path, os.O_CREAT | os.O_RDWR, 0o666)
    except OSError as e:  # no writable temp directory: the PCI-bus-ID all-gather still checks (after the groups)
        logger.warning("cannot claim GPU %s (%s): relying on the bus-ID all-gather", bus, e)
        return
    try:
        fcntl.flock(fd, fcntl.LOCK_EX | fcntl.LOCK_NB)
    except OSError:
        holder = os.pread(fd, 64, 0).decode(errors="replace").strip()
        os.close(fd)
        raise TopologyError((env.rank, bus, holder),
                            f"rank {env.rank} and {holder or 'another rank'} of this job share a device (GPU at PCI "
                            f"{bus}): one rank per GPU; set DDL_REHEARSAL=1 for a deliberate rehearsal") from None
    os.ftruncate(fd, 0)
    os.pwrite(fd, f"rank {env.rank} (pid {os.getpid()})".encode(), 0)
    _CLAIMED[bus] = fd


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def init_distributed(env: DDLEnv, backend: str | None = None, timeout_s: float = 600.0,
                     device: str | None = None) -> DDLEnv:
    """Create the DP (RCCL or gloo) group and a gloo control group; set the device.

    ``backend`` defaults to ``$DDL_BACKEND``, else RCCL ("nccl") on a GPU and gloo on
    the CPU; at world size 1 no group is built unless a backend is named.
    ``timeout_s`` is both groups' collective timeout (``start(timeout_s=)`` passes its own through).
    ``device="cpu"`` (or ``$DDL_DEVICE=cpu``) keeps the rank off the GPU even
    when one is visible (CPU rehearsals of multi-rank runs). Touches the GPU
    otherwise: call it only after producer workers have been spawned.
    """
    import torch
    import torch.distributed as dist

    device = device or os.environ.get("DDL_DEVICE") or None
    use_gpu = device != "cpu" and torch.cuda.is_available()
    if use_gpu:
        n_dev = torch.cuda.device_count()
        check_device_count(env, n_dev)
        dev_index = env.local_rank % max(n_dev, 1)
        torch.cuda.set_device(dev_index)
        env.device = f"cuda:{dev_index}"
        if env.world_size > 1:
            claim_device(env)
    else:
        env.device = "cpu"
    backend = backend or os.environ.get("DDL_BACKEND") or None
    if env.world_size == 1 and backend is None:
        env.backend = None  # no process group: nothing to exchange with
        return env
    # an explicit backend at world size 1 builds a 1-rank group, so the collective path (the
    # global-shuffle exchange over RCCL) can be exercised and timed on a single GPU
    backend = backend or ("nccl" if use_gpu else "gloo")
    env.backend = backend
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        # a 1-rank group has no peers to agree on a port with: take a free one (a fixed 29500 collides with
        # any other job on the host); larger worlds keep torch's conventional default
        os.environ["MASTER_PORT"] = str(_free_port()) if env.world_size == 1 else "29500"
    if not dist.is_initialized():
        kwargs = dict(backend=backend, rank=env.rank, world_size=env.world_size, timeout=timedelta(seconds=timeout_s))
        if backend == "nccl":
            kwargs["device_id"] = torch.device(env.device)
        dist.init_process_group(**kwargs)
    env.process_group = dist.group.WORLD
    env.control_group = (dist.new_group(backend="gloo", timeout=timedelta(seconds=timeout_s)) if backend != "gloo"
                         else dist.group.WORLD)
    check_node_locality(env)
    return env


def init_mpi_error_handling(env: DDLEnv, n_instances: int) -> None:
    """Reference ``init_mpi_error_handling(comm_global, n_instances)`` (ddl/ddl_env.py:12-30).

    The reference warns on a single rank and ``Abort(1)``s the whole MPI job when
    the rank count is not a multiple of ``n_instances``. Here a rank is a GPU, so
    the check is ``world_size % n_instances``, and it raises ``TopologyError``
    (the launcher tears the job down) instead of aborting.
    """
    if env.world_size < 2 and env.rank == 0:
        logger.warning("Using only a single rank!")
    if n_instances < 1 or env.world_size % n_instances != 0:
        raise TopologyError((env.world_size, n_instances),
                            f"number of ranks ({env.world_size}) must be a multiple of {n_instances}")


def init_mpi(n_instances: int | None = None, n_producers: int | None = None, backend: str | None = None) -> DDLEnv:
    """Reference entry point ``init_mpi(n_instances)`` (ddl/ddl_env.py:33-97).

    The reference splits ``mpirun``'s ranks into per-GPU groups of one consumer
    and P producers. Here the ranks ARE the GPUs (one process each; producers
    are child processes spawned by ``start`` / ``distributed_dataloader``), so
    ``n_instances`` must equal the world size, and the reference's ``Abort(1)``
    on a rank count that does not divide (ddl/ddl_env.py:25-30) becomes a
    ``TopologyError``. Returns the environment with the DP groups created.
    """
    env = read_env(n_producers)
    if n_instances is not None and n_instances != env.world_size:
        raise TopologyError((n_instances, env.world_size),
                            f"n_instances={n_instances} GPUs but the job has {env.world_size} ranks "
                            "(one rank per GPU)")
    return init_distributed(env, backend)


def check_node_locality(env: DDLEnv) -> None:
    """Hostname all-gather: ranks sharing a host must be exactly its local ranks.

    The reference raises ``DoesNotMatchError`` when a GPU group spans nodes
    (reference ddl/ddl_env.py:72-73).
    """
    import torch.distributed as dist

    if env.world_size == 1 or env.control_group is None:
        return
    ident = device_identity(env.device)
    infos: list = [None] * env.world_size
    dist.all_gather_object(infos, (env.hostname, env.local_rank, env.local_world_size,
                                   ident.get("pci_bus_id"), ident.get("uuid")), group=env.control_group)
    mine = [i for i in infos if i[0] == env.hostname]
    local_ranks = sorted(i[1] for i in mine)
    if local_ranks != list(range(len(mine))) or len(mine) != env.local_world_size:
        raise TopologyError(infos, f"ranks on host {env.hostname} have local ranks {local_ranks}, "
                                   f"expected 0..{env.local_world_size - 1}")
    # one GPU per rank: no two ranks of a host on the same PCI device (a wrapped device index, or a
    # visibility mask that hands every task the same GPU)
    buses = [i[3] for i in mine if i[3] is not None]
    if len(set(buses)) != len(buses) and not rehearsal():
        raise TopologyError(infos, f"ranks on host {env.hostname} share GPUs (PCI bus IDs {buses}); one rank per "
                                   "GPU, or DDL_REHEARSAL=1 for a deliberate rehearsal")
    logger.debug("node locality ok: %s", infos)


def destroy_distributed() -> None:
    import torch.distributed as dist

    if dist.is_initialized():
        try:
            dist.destroy_process_group()
        except Exception:  # pragma: no cover - best effort at teardown
            pass
