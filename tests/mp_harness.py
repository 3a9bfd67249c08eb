"""Run a function on W torch.distributed ranks (gloo, 127.0.0.1) as separate processes.

Each rank process is non-daemonic so it can spawn its own producer workers
(the production layout). Results come back through a Queue; a rank that
raises reports its traceback and the harness re-raises it in the test.
"""

import multiprocessing as mp
import os
import socket
import traceback


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(fn, rank, world, port, q, args, env, nodes=1):
    # CPU multi-rank tests: several ranks on one box must not share (or fight over) a GPU
    os.environ["DDL_DEVICE"] = "cpu"
    per_node = world // nodes
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank % per_node),
                       "LOCAL_WORLD_SIZE": str(per_node), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    if nodes > 1:  # rehearse a multi-node job: each block of ranks claims its own host
        os.environ["DDL_HOSTNAME"] = f"rehearsal-node{rank // per_node}"
    os.environ.update(env)  # explicit overrides win
    try:
        q.put((rank, "ok", fn(rank, world, *args)))
    except BaseException:
        q.put((rank, "err", traceback.format_exc()))


def run_ranks(fn, world: int, *args, timeout: float = 180.0, env: dict | None = None, nodes: int = 1):
    if world % nodes:
        raise ValueError("world must be a multiple of nodes")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_rank_main, args=(fn, r, world, port, q, args, env or {}, nodes))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world):
            rank, status, payload = q.get(timeout=timeout)
            if status == "err":
                raise AssertionError(f"rank {rank} failed:\n{payload}")
            results[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
                p.join()
    return [results[r] for r in range(world)]
