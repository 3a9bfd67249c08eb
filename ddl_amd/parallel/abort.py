"""Job-wide failure propagation: the ``MPI_Abort`` of a torch.distributed job.

In the reference a fatal error ``Abort(1)``s every rank (``/root/reference/ddl/ddl_env.py:25-30``) and
mpirun tears the whole job down when one rank dies. A torch.distributed job has neither: a rank that
raises mid-epoch leaves its peers blocked inside the next exchange all-to-all or DDP all-reduce until
the process-group timeout, and a rank that is SIGKILLed leaves them there too.

``JobWatchdog`` closes that gap with one daemon thread per rank and a side channel that does not go
through the (possibly blocked) collectives: a client of the job's rendezvous ``TCPStore``
(``MASTER_ADDR:MASTER_PORT``, under a per-job prefix).

* **Raise -> abort.** ``start()`` catches an exception escaping the user's code on any rank, publishes
  ``abort = "rank r: <error>"`` in the store, prints the traceback and exits the process with status 1
  (the failing rank never waits in the final barrier or in ``torch.cuda.synchronize`` behind a
  collective its peers will never join).
* **Abort -> exit.** Every other rank's watchdog sees the key within ``poll_s``, logs it, stops its
  producer workers and exits with ``PEER_ABORT_EXIT`` (``os._exit``: the main thread may be blocked in
  a collective that will never complete).
* **Death.** Each rank has a ``DeathWatch``: a small child process, spawned before the rank touches the
  GPU, that holds one end of a pipe to the rank. When the rank dies without a clean shutdown (SIGKILL,
  OOM kill, a crash in native code) the pipe reaches EOF and the child publishes the abort at once, so
  the peers exit within ``poll_s`` -- not after ``peer_timeout_s``. It needs no GIL and no heartbeat.
* **Frozen rank.** Each rank's heartbeat counter is bumped by its watchdog thread AND by its death watch,
  which bumps only while the rank exists and is not stopped (``/proc``: SIGSTOP, a debugger, a frozen
  cgroup). Rank r watches rank ``(r + 1) % W`` only (O(W) store traffic). A counter that has not moved for
  ``peer_timeout_s`` (a stopped or frozen process, a lost node) makes the watcher publish the abort for
  it. An unreachable store (its host rank died) is an abort too.
* **Hung rank.** The death watch relays its beats only while the rank's watchdog thread keeps sending it
  liveness tokens (one per poll). A healthy rank holding the GIL in one long C call stops the tokens but
  keeps beating through the death watch for ``hang_timeout_s`` (default 5 x ``peer_timeout_s``, at least
  300 s), so it is not mistaken for a dead one; a rank that holds the GIL longer -- deadlocked or hung --
  stops beating and is aborted then, before the collective timeout (``timeout_s``, 600 s) would end it.
  A rank blocked in a collective with the GIL released keeps beating: its peers are blocked in the same
  collective, which the collective timeout bounds.
* **Clean exit.** ``stop()`` marks the rank done (watchers of a finished rank stop checking it) before
  the final barrier, so a slow rank is never mistaken for a dead one once its neighbour finished.

The process-group timeout itself is ``start(timeout_s=)`` (``parallel/env.init_distributed``); the
watchdog makes the typical failure end the job in about ``poll_s`` instead of that timeout.
"""

from __future__ import annotations

import os
import sys
import threading
import time
import traceback
from datetime import timedelta
from typing import Any, Callable

from ..utils.logging import logger

PEER_ABORT_EXIT = 75  # exit status of a rank torn down because ANOTHER rank failed
# A rank is declared dead when its heartbeat has not moved for this long. With a death watch (the default
# process-mode launch) the heartbeat needs no GIL: a rank holding it in one long C call still beats. Without
# one (thread-mode producers, no MASTER_ADDR / MASTER_PORT) only the Python thread beats, and a rank holding
# the GIL longer than this counts as hung; raise it (``start(peer_timeout_s=)``,
# ``distributed_dataloader(peer_timeout_s=)``) for such workloads.
DEFAULT_PEER_TIMEOUT_S = 60.0


def default_hang_timeout_s(peer_timeout_s: float) -> float:
    """How long a rank's death watch keeps beating for it without a liveness token from its watchdog thread."""
    return max(300.0, 5.0 * float(peer_timeout_s))


def _job_key() -> str:
    return os.environ.get("TORCHELASTIC_RUN_ID") or os.environ.get("MASTER_PORT", "0")


def _store_client(prefix: str, timeout_s: float):
    """A private client of the rendezvous TCPStore (never shares a socket with the collectives'
    bootstrap); the default group's store when the job was not rendezvoused over MASTER_ADDR/PORT."""
    import torch.distributed as dist

    try:
        host = os.environ["MASTER_ADDR"]
        port = int(os.environ["MASTER_PORT"])
        store = dist.TCPStore(host, port, is_master=False, timeout=timedelta(seconds=timeout_s),
                              wait_for_workers=False)
    except Exception as first:
        # a job not rendezvoused over MASTER_ADDR / MASTER_PORT: the default group's store (private torch API)
        try:
            from torch.distributed.distributed_c10d import _get_default_store

            store = _get_default_store()
        except Exception as e:
            raise RuntimeError("JobWatchdog needs a store for its side channel: no TCPStore at MASTER_ADDR:"
                               f"MASTER_PORT ({first}) and no default process-group store ({e}); pass "
                               "abort_on_error=False to run without the job-wide abort") from e
    return dist.PrefixStore(prefix, store)


def _linger_if_store_host(rank: int, poll_s: float) -> None:
    """Rank 0 hosts the rendezvous TCPStore under a plain launch (torchrun's agent hosts it otherwise): its exit
    takes the store down, and a peer that polls after that sees "store unreachable" instead of the abort's
    reason. Stay up for two polls first, so every peer reads the reason."""
    if rank == 0 and not os.environ.get("TORCHELASTIC_RUN_ID"):
        time.sleep(2 * poll_s + 0.5)


class JobWatchdog:
    """One per rank; see the module docstring. ``on_abort`` runs (best effort) before the exit."""

    def __init__(self, rank: int, world_size: int, *, peer_timeout_s: float = DEFAULT_PEER_TIMEOUT_S,
                 poll_s: float = 0.25, on_abort: Callable[[], None] | None = None, store: Any = None,
                 job_key: str | None = None, exit_fn: Callable[[int], None] | None = None,
                 death_watch: "DeathWatch | None" = None, hang_timeout_s: float | None = None):
        self.rank, self.world = int(rank), int(world_size)
        self.death_watch = death_watch  # beats for this rank too (alive and not stopped), GIL or not
        self.peer_timeout_s = float(peer_timeout_s)
        self.hang_timeout_s = float(hang_timeout_s if hang_timeout_s is not None
                                    else default_hang_timeout_s(peer_timeout_s))
        self.poll_s = float(poll_s)
        self.on_abort = on_abort
        self._exit = exit_fn or os._exit
        key = job_key or _job_key()
        self._store = store if store is not None else _store_client(f"ddl_amd/abort/{key}/", 30.0)
        self._stop = threading.Event()
        self._thread: threading.Thread | None = None
        self.aborted: str | None = None  # the abort message this rank acted on (tests, exit_fn overrides)
        self._beat = 0
        self._done = False

    # ------------------------------------------------------------------ store keys
    def _hb(self, r: int) -> str:
        return f"hb/{r}"

    def start(self) -> "JobWatchdog":
        self._store.set(self._hb(self.rank), "0")
        if self.death_watch is not None:
            self.death_watch.beat(self.poll_s, self.hang_timeout_s)
        self._thread = threading.Thread(target=self._run, name=f"ddl-watchdog-{self.rank}", daemon=True)
        self._thread.start()
        return self

    def abort(self, reason: str) -> None:
        """Publish a job-wide abort (the first reason wins: ``compare_set`` on an absent key)."""
        msg = f"rank {self.rank}: {reason}"[:2000]
        try:
            self._store.compare_set("abort", "", msg)
        except Exception as e:  # the store is gone: the peers' watchdogs will see that too
            logger.error("could not publish the abort (%s); peers will detect the store loss", e)

    def finishing(self) -> None:
        """This rank's work is done: watchers of this rank stop watching it (a rank that finished
        first is not 'dead'), but this rank keeps acting on aborts -- a peer can still fail while
        this one waits in the final barrier."""
        if self.death_watch is not None:
            self.death_watch.finishing()  # its beats stop; its last write is "done" too (after any beat in flight)
        try:
            self._store.set(self._hb(self.rank), "done")
        except Exception:  # pragma: no cover - the thread reports a lost store
            pass
        self._done = True

    def stop(self) -> None:
        """After the final barrier: no more checks."""
        if not self._done:
            self.finishing()
        self._stop.set()
        if self._thread is not None:
            self._thread.join(2 * self.poll_s + 1.0)

    # ------------------------------------------------------------------ thread
    def _fire(self, msg: str) -> None:
        if self._stop.is_set():
            return
        self.aborted = msg
        sys.stdout.flush()
        print(f"ddl_amd: rank {self.rank}: job aborted ({msg}); exiting with {PEER_ABORT_EXIT}",
              file=sys.stderr, flush=True)
        if self.on_abort is not None:
            try:
                self.on_abort()
            except Exception:  # pragma: no cover - best effort
                pass
        _linger_if_store_host(self.rank, self.poll_s)
        self._exit(PEER_ABORT_EXIT)

    def _run(self) -> None:
        target = (self.rank + 1) % self.world
        watch = target != self.rank
        last_val, last_change = None, time.monotonic()
        while not self._stop.wait(self.poll_s):
            try:
                if not self._done:
                    self._beat += 1
                    self._store.set(self._hb(self.rank), str(self._beat))
                    if self.death_watch is not None:
                        self.death_watch.alive()  # the token the death watch needs to keep beating for us
                if self._store.check(["abort"]):
                    msg = self._store.get("abort").decode(errors="replace")
                    if msg:
                        return self._fire(msg)
                if watch:
                    v = self._store.get(self._hb(target)) if self._store.check([self._hb(target)]) else b""
                    if v == b"done":
                        watch = False
                    elif v != last_val:
                        last_val, last_change = v, time.monotonic()
                    elif time.monotonic() - last_change > self.peer_timeout_s:
                        msg = (f"no heartbeat from rank {target} for {self.peer_timeout_s:.0f}s "
                               "(stopped, frozen or lost)")
                        self.abort(msg)
                        return self._fire(f"rank {self.rank}: {msg}")
            except Exception as e:  # store unreachable: its host rank (or the agent) is gone
                # ... or the job just ended cleanly and the store's host exited first: give stop() a
                # moment to arrive after the final barrier before calling it a failure
                if self._stop.wait(4 * self.poll_s + 1.0):
                    return
                return self._fire(f"rendezvous store unreachable ({type(e).__name__}: {e})")


def _process_stopped(pid: int) -> bool:
    """Is ``pid`` stopped (SIGSTOP, a debugger, a frozen cgroup)? Linux /proc; False where unknown."""
    try:
        with open(f"/proc/{pid}/stat") as f:
            state = f.read().rsplit(")", 1)[1].split()[0]
        if state in ("T", "t"):
            return True
        with open(f"/proc/{pid}/cgroup") as f:  # cgroup v2 freezer: the tasks are in "S" state, the cgroup frozen
            rel = f.read().strip().split("::", 1)[-1]
        with open(f"/sys/fs/cgroup{rel}/cgroup.events") as f:
            return "frozen 1" in f.read()
    except (OSError, IndexError):
        return False


def _death_watch_main(pipe, parent_pid: int, rank: int, job_key: str, host: str, port: int) -> None:
    """Body of a rank's ``DeathWatch`` child. Messages from the rank: ``("beat", period_s, hang_s)`` -- keep the
    rank's heartbeat going from here (while the rank exists, is not stopped, and sent a liveness token within
    ``hang_s``), ``"alive"`` -- a liveness token from the rank's watchdog thread, ``"finishing"`` -- mark it
    done and stop, ``"done"`` -- a clean shutdown, exit. EOF (or a new parent) = the rank died: publish the
    job-wide abort under the watchdogs' prefix."""
    os.environ["HIP_VISIBLE_DEVICES"] = "-1"  # never touches a GPU
    import torch.distributed as dist  # now, not at the rank's death: the report must not wait for an import

    prefix, hb = f"ddl_amd/abort/{job_key}/", f"hb/{rank}"
    store, period, beat = None, 1.0, 0
    hang_s, last_alive = float("inf"), time.monotonic()
    while True:
        try:
            if pipe.poll(period):
                msg = pipe.recv()
                if msg == "done":
                    return
                if msg == "alive":
                    last_alive = time.monotonic()
                elif msg == "finishing":
                    if store is not None:
                        store.set(hb, "done")
                    store = None
                elif isinstance(msg, tuple) and msg[0] == "beat":
                    period = float(msg[1])
                    hang_s = float(msg[2]) if len(msg) > 2 else float("inf")
                    last_alive = time.monotonic()
                    store = dist.PrefixStore(prefix, dist.TCPStore(host, port, is_master=False,
                                                                   timeout=timedelta(seconds=30),
                                                                   wait_for_workers=False))
            elif os.getppid() != parent_pid:
                break
            if (store is not None and not _process_stopped(parent_pid)
                    and time.monotonic() - last_alive <= hang_s):
                beat += 1
                store.set(hb, f"w{beat}")
        except (EOFError, OSError):
            break
        except Exception:  # the store is gone: the peers' watchdogs report that loss; keep watching for a death
            store = None
    msg = f"rank {rank}: process {parent_pid} died without a clean shutdown (killed or crashed)"
    print(f"ddl_amd: {msg}; aborting the job", file=sys.stderr, flush=True)
    try:
        # short: when the store's host is gone too, the peers' watchdogs see that loss themselves
        store = dist.TCPStore(host, port, is_master=False, timeout=timedelta(seconds=5), wait_for_workers=False)
        dist.PrefixStore(prefix, store).compare_set("abort", "", msg[:2000])
    except Exception:  # the store died with the rank that hosted it: the peers' watchdogs see the loss
        pass


class DeathWatch:
    """The death reporter -- and heartbeat -- of one rank (see the module docstring). ``spawn`` when the rank
    starts (``start()`` does, with the producers); ``done()`` on a clean shutdown."""

    def __init__(self, proc, pipe):
        self.proc, self._pipe = proc, pipe
        self._lock = threading.Lock()  # the watchdog thread and the main thread both send

    @classmethod
    def spawn(cls, rank: int) -> "DeathWatch | None":
        import multiprocessing as mp

        if os.environ.get("DDL_PRODUCER_MODE", "process") == "thread":
            # thread-mode producers mean "spawn no process" (under rocprofv3 the GPU may be initialised before
            # main): the heartbeat alone covers deaths then
            return None
        host, port = os.environ.get("MASTER_ADDR"), os.environ.get("MASTER_PORT")
        if not host or not port:
            logger.debug("no MASTER_ADDR / MASTER_PORT: no death watch (the heartbeat still covers deaths)")
            return None
        ctx = mp.get_context("spawn")
        reader, writer = ctx.Pipe(duplex=False)
        proc = ctx.Process(target=_death_watch_main, name=f"ddl-deathwatch-{rank}", daemon=True,
                           args=(reader, os.getpid(), rank, _job_key(), host, int(port)))
        proc.start()
        reader.close()  # the child reads; this process keeps the only write end: EOF when it dies
        return cls(proc, writer)

    def _send(self, msg, close: bool = False) -> bool:
        with self._lock:
            if self._pipe is None:
                return False
            try:
                self._pipe.send(msg)
                if close:
                    self._pipe.close()
                    self._pipe = None
                return True
            except (BrokenPipeError, OSError):
                return False

    def beat(self, period_s: float, hang_timeout_s: float = float("inf")) -> bool:
        """Heartbeat this rank from the child from now on (the rendezvous store is up), as long as a liveness
        token (``alive``) arrived within ``hang_timeout_s``."""
        return self._send(("beat", float(period_s), float(hang_timeout_s)))

    def alive(self) -> bool:
        """A liveness token: this rank's Python threads still run (sent by the watchdog thread every poll)."""
        return self._send("alive")

    def finishing(self) -> bool:
        return self._send("finishing")

    def disarm(self) -> None:
        """This rank is leaving on purpose (a clean shutdown, or an abort it already published or acted on):
        the child exits without reporting a death. Does not wait for it."""
        self._send("done", close=True)

    def done(self) -> None:
        self.disarm()
        self.proc.join(5.0)
        if self.proc.is_alive():
            self.proc.kill()


def abort_on_exception(watchdog: JobWatchdog | None, exc: BaseException, cleanup: Callable[[], None] | None = None,
                       exit_fn: Callable[[int], None] | None = None) -> None:
    """The failing rank's side: publish, report, clean up what is safe, exit(1) without waiting on peers."""
    reason = f"{type(exc).__name__}: {exc}"
    if watchdog is not None:
        watchdog._stop.set()  # its own abort key must not make it exit with the peer status
        watchdog.abort(reason)
    traceback.print_exception(type(exc), exc, exc.__traceback__, file=sys.stderr)
    print(f"ddl_amd: rank {getattr(watchdog, 'rank', '?')} failed ({reason}); aborting the job",
          file=sys.stderr, flush=True)
    if cleanup is not None:
        try:
            cleanup()
        except Exception:  # pragma: no cover - best effort
            pass
    _linger_if_store_host(getattr(watchdog, "rank", -1), getattr(watchdog, "poll_s", 0.25))
    (exit_fn or os._exit)(1)
