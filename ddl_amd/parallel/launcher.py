"""Launcher / role dispatcher: ``@distributed_dataloader`` (reference ddl/ddl_env.py:100-128).

Reference: every MPI rank enters the decorator; local rank 0 of each GPU
group runs the user function, the other local ranks become ``DataPusher``s,
and kwargs given to the user function are dropped (reference
ddl/ddl_env.py:115-116).

Here one process per GPU (torchrun / srun task) enters the decorator; it
spawns its ``P`` producer workers as child processes (``spawn`` start method,
*before* anything touches the GPU), then creates the DP process groups (RCCL
on GPUs), then calls ``func(*args, env, conn, **kwargs)`` (kwargs forwarded).
On exit the producers are shut down and joined, and all ranks meet at a final
barrier (reference ddl/ddl_env.py:126).
"""

from __future__ import annotations

import contextlib
import functools
import multiprocessing as mp
import os
from typing import Any, Callable, Iterator

from ..connection import DEFAULT_TIMEOUT_S, Connection
from ..types import DDLEnv
from ..utils.logging import configure, logger
from .abort import DEFAULT_PEER_TIMEOUT_S, DeathWatch, JobWatchdog, abort_on_exception
from .env import destroy_distributed, init_distributed, read_env


def spawn_producers(env: DDLEnv, timeout_s: float = DEFAULT_TIMEOUT_S, env_overrides: dict | None = None,
                    mode: str | None = None) -> Connection:
    """Start ``env.n_producers`` producer workers; return the consumer Connection.

    ``mode`` (default ``$DDL_PRODUCER_MODE`` or ``"process"``): ``"process"``
    spawns one host process per producer (the production layout: user hooks
    run truly in parallel, a crash is contained); ``"thread"`` runs them as
    threads of the consumer (debugging, and profiling under ``rocprofv3``,
    whose preloaded library may initialise the GPU before ``main`` -- a
    process spawned after that would be forked from a GPU-initialised parent).
    """
    import threading

    from ..datapusher import producer_main

    mode = mode or os.environ.get("DDL_PRODUCER_MODE", "process")
    if mode not in ("process", "thread"):
        raise ValueError(f"producer mode must be 'process' or 'thread', got {mode!r}")
    ctx = mp.get_context("spawn")
    pipes, procs = [], []
    for i in range(env.n_producers):
        parent, child = ctx.Pipe(duplex=True)
        args = (child, i, os.getpid(), env.rank, env.world_size, timeout_s, env_overrides)
        if mode == "process":
            proc = ctx.Process(target=producer_main, name=f"ddl-producer-{env.rank}.{i}", args=args, daemon=True)
            proc.start()
            child.close()
        else:
            proc = threading.Thread(target=producer_main, name=f"ddl-producer-{env.rank}.{i}", args=args,
                                    kwargs={"in_thread": True}, daemon=True)
            proc.start()
        pipes.append(parent)
        procs.append(proc)
    logger.debug("spawned %d producers: %s", len(procs), [getattr(p, "pid", None) for p in procs])
    return Connection(pipes, procs, timeout_s=timeout_s, rank=env.rank)


@contextlib.contextmanager
def start(n_producers: int | None = None, init_dist: bool = True, backend: str | None = None,
          timeout_s: float = DEFAULT_TIMEOUT_S, env_overrides: dict | None = None,
          device: str | None = None, abort_on_error: bool = True,
          peer_timeout_s: float = DEFAULT_PEER_TIMEOUT_S,
          spare_connections: int = 0,
          producer_mode: str | None = None) -> Iterator[tuple[DDLEnv, Connection | None]]:
    """Context-manager form of the launcher: ``with start() as (env, conn): ...``.

    ``timeout_s`` bounds every wait: the shm hand-offs with the producers AND the process groups'
    collectives (``init_distributed``). With ``abort_on_error`` (default) and more than one rank, a
    failure on any rank ends the whole job, as the reference's ``Abort(1)`` does
    (``/root/reference/ddl/ddl_env.py:25-30``): the failing rank publishes the error and exits 1, its
    peers exit ``PEER_ABORT_EXIT`` within a fraction of a second; a rank that is killed or crashes ends the
    job as fast (its death watch reports it), and a stopped or frozen rank after ``peer_timeout_s`` without
    a heartbeat (``parallel/abort.py``).

    ``spare_connections``: that many more independent sets of ``n_producers`` producers, spawned with the
    first (the rank's CPU slice is then split over all of them at once), as ``conn.spares``: one per later
    ``DistributedDataLoader`` of the same program (an evaluation loader after the training loader, a second
    order). A producer set serves one loader; an unused spare
    shuts down cleanly at exit.

    ``producer_mode``: ``"process"`` or ``"thread"`` (``spawn_producers``; default ``$DDL_PRODUCER_MODE``).
    """
    configure()
    env = read_env(n_producers)
    from ..utils.numa import bind_to_gpu_numa, partition_after_spawn

    # before spawning: the producers inherit the rank's CPU slice of its GPU's NUMA node
    node = bind_to_gpu_numa(env.local_rank, env.local_world_size)
    conn = spawn_producers(env, timeout_s, env_overrides, producer_mode) if env.n_producers > 0 else None
    spares = [spawn_producers(env, timeout_s, env_overrides, producer_mode)
              for _ in range(int(spare_connections))] if conn is not None else []
    if conn is not None:
        conn.spares = spares
    if conn is not None and node is not None:  # a GPU host: split the slice between consumer and producers
        every = [conn, *spares]
        pids = [p for c in every for p in c.producer_pids if p and p != os.getpid()]  # thread mode: none
        layout = partition_after_spawn(pids, len(pids)) if len(pids) == env.n_producers * len(every) else None
        for c in every:
            c.cpu_layout = layout
    # the death reporter is a process too: spawned before anything touches the GPU
    death_watch = DeathWatch.spawn(env.rank) if abort_on_error and init_dist and env.world_size > 1 else None

    def stop_helpers() -> None:
        """Job abort (this rank failed, or a peer did): the producers stop now, the death watch stands down
        (the abort is published already; this exit is no silent death)."""
        if death_watch is not None:
            death_watch.disarm()
        if conn is not None:
            for c in (conn, *spares):
                c.kill()

    created_pg = False
    watchdog = None
    try:
        if init_dist:
            import torch.distributed as dist

            was = dist.is_available() and dist.is_initialized()
            init_distributed(env, backend, timeout_s=timeout_s, device=device)
            created_pg = not was and dist.is_initialized()  # a named backend builds a group at world size 1 too
            if abort_on_error and env.world_size > 1 and env.control_group is not None:
                watchdog = JobWatchdog(env.rank, env.world_size, peer_timeout_s=peer_timeout_s,
                                       on_abort=stop_helpers, death_watch=death_watch).start()
        yield env, conn
    except BaseException as e:
        if watchdog is not None and not (isinstance(e, SystemExit) and e.code in (None, 0)):
            abort_on_exception(watchdog, e, cleanup=stop_helpers)
        raise
    finally:
        if watchdog is not None:
            watchdog.finishing()
        if death_watch is not None:  # a clean shutdown from here on (a raise already published its abort)
            death_watch.done()
        for c in spares:
            c.finalize()
        if conn is not None:
            conn.finalize()
        if created_pg:
            import torch.distributed as dist

            try:
                dist.barrier(group=env.control_group)
            except Exception as e:  # pragma: no cover
                logger.warning("final barrier failed: %s", e)
            if watchdog is not None:
                watchdog.stop()
            destroy_distributed()
        elif watchdog is not None:
            watchdog.stop()


def distributed_dataloader(func: Callable | None = None, *, n_producers: int | None = None, init_dist: bool = True,
                           backend: str | None = None, timeout_s: float = DEFAULT_TIMEOUT_S,
                           abort_on_error: bool = True, peer_timeout_s: float = DEFAULT_PEER_TIMEOUT_S):
    """Decorator: run ``func(*args, env, conn, **kwargs)`` as this rank's consumer with its producers.

    Usable bare (``@distributed_dataloader``) or with options
    (``@distributed_dataloader(n_producers=4)``). The number of producers per
    rank defaults to ``$DDL_PRODUCERS_PER_RANK`` or 3. ``timeout_s``, ``abort_on_error`` and
    ``peer_timeout_s``: as for ``start``.
    """

    def deco(f: Callable) -> Callable:
        @functools.wraps(f)
        def wrapper(*args: Any, **kwargs: Any) -> Any:
            with start(n_producers, init_dist, backend, timeout_s, abort_on_error=abort_on_error,
                       peer_timeout_s=peer_timeout_s) as (env, conn):
                return f(*args, env, conn, **kwargs)

        return wrapper

    if func is not None:
        return deco(func)
    return deco
