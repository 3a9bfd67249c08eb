"""One rank of the job-abort tests (``test_job_abort.py``): a loop of control-group all-reduces inside
``ddl_amd.start``; ``--stop-rank`` SIGSTOPs itself mid-loop (a silent hang: sockets open, no heartbeat),
``--raise-rank`` raises mid-loop; ``--kill-rank`` SIGKILLs itself mid-loop while the others compute (no
collective in flight: only the library can notice the death); ``--gil-hold-rank`` holds the GIL in one C call
for ``--gil-hold-s`` seconds mid-loop (alive and healthy, but no Python thread of it can run).
``--gpu-loader``: the loop is a device loader's epoch instead (H2D staging, exchange collectives every window,
gfx950 kernels), for the GPU version of the kill test."""

import argparse
import os
import signal
import time

import torch
import torch.distributed as dist

import ddl_amd


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--stop-rank", type=int, default=-1)
    ap.add_argument("--raise-rank", type=int, default=-1)
    ap.add_argument("--kill-rank", type=int, default=-1)
    ap.add_argument("--gil-hold-rank", type=int, default=-1)
    ap.add_argument("--gil-hold-s", type=int, default=8)
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--peer-timeout", type=float, default=3.0)
    ap.add_argument("--timeout", type=float, default=600.0, help="start(timeout_s=): shm waits + process groups")
    ap.add_argument("--no-abort", action="store_true", help="start(abort_on_error=False): no watchdog")
    ap.add_argument("--gpu-loader", action="store_true")
    args = ap.parse_args()
    if args.gpu_loader:
        return gpu_loader(args)
    with ddl_amd.start(n_producers=1, peer_timeout_s=args.peer_timeout, timeout_s=args.timeout,
                       abort_on_error=not args.no_abort) as (env, conn):
        t = torch.ones(1)
        for i in range(args.iters):
            if i == 10 and env.rank == args.stop_rank:
                os.kill(os.getpid(), signal.SIGSTOP)
            if i == 10 and env.rank == args.gil_hold_rank:
                import ctypes

                ctypes.PyDLL(None).sleep(args.gil_hold_s)  # a PyDLL call keeps the GIL for its whole duration
            if i == 10 and env.rank == args.raise_rank:
                raise RuntimeError("abort_rank: injected failure")
            if i == 10 and args.kill_rank >= 0:
                if env.rank == args.kill_rank:
                    os.kill(os.getpid(), signal.SIGKILL)
                time.sleep(120)  # "compute": no collective that could notice the dead peer
            dist.all_reduce(t, group=env.control_group)
            time.sleep(0.02)
    print(f"rank {env.rank} done", flush=True)


def gpu_loader(args) -> None:
    from ddl_amd import Marker
    from tests.helpers import IdProducer

    with ddl_amd.start(n_producers=2, peer_timeout_s=args.peer_timeout, timeout_s=args.timeout) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(64, 6), 16, conn, 1000, 0.5, "alltoall", env=env,
                                           device=torch.device(env.device),
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           staging=ddl_amd.StagingSpec(prefetch_depth=2),
                                           order=ddl_amd.OrderSpec(seed=1))
        n = 0
        for epoch in range(1000):
            for a, _ in dl:
                n += 1
                if n == 40 and env.rank == args.kill_rank:
                    print(f"rank {env.rank} killing itself mid-epoch on {a.device}", flush=True)
                    os.kill(os.getpid(), signal.SIGKILL)
                dl.mark(Marker.END_OF_BATCH)
            dl.mark(Marker.END_OF_EPOCH)
        dl.close()
    print(f"rank {env.rank} done", flush=True)


if __name__ == "__main__":
    main()
