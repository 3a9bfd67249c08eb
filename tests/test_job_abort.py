"""Job-wide failure propagation (``ddl_amd/parallel/abort.py``): one rank's failure ends every rank
fast, as the reference's ``Abort(1)`` does (``/root/reference/ddl/ddl_env.py:25-30``), instead of
leaving the peers blocked in the exchange / DDP collectives until the process-group timeout.

Each multi-process test launches the ranks as plain processes (torchrun-style env, no agent that
would kill the siblings for us), so the only thing that can end the peers is the library itself; the
torchrun and ``bench.py --gpus N`` self-launch lines are covered too.
"""

import os
import signal
import subprocess
import sys
import time

import pytest

from ddl_amd.parallel.abort import PEER_ABORT_EXIT, JobWatchdog
from tests.mp_harness import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = [os.path.join(REPO, "bench.py"), "--steps", "40", "--warmup", "2", "--window", "64", "--batch", "16",
         "--idle-steps", "3", "--model-dim", "64", "--model-depth", "1", "--order", "window"]
PG_TIMEOUT_S = 600  # what the peers would otherwise wait for


def _base_env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(PYTHONPATH=REPO, DDL_DEVICE="cpu", DDL_REHEARSAL="1", **kw)  # CPU ranks: a labelled rehearsal
    return env


def _launch_plain(world: int, argv: list[str], env: dict) -> list[subprocess.Popen]:
    port = str(free_port())
    procs = []
    for r in range(world):
        e = dict(env, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        # own session per rank: _kill_all ends the rank's helpers too (producers, death watch), which hold
        # its output pipes
        procs.append(subprocess.Popen([sys.executable, *argv], env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True, start_new_session=True))
    return procs


def _wait_all(procs, timeout_s: float) -> tuple[list[int | None], float]:
    t0 = time.monotonic()
    while time.monotonic() - t0 < timeout_s and any(p.poll() is None for p in procs):
        time.sleep(0.1)
    codes = [p.poll() for p in procs]
    return codes, time.monotonic() - t0


def _communicate(p):
    """The rank's (stdout, stderr) once it has exited; a helper of the rank still holding its pipes after 30 s
    (on a loaded host, a death watch still importing) is killed with the rank's session."""
    try:
        return p.communicate(timeout=30)
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        return p.communicate(timeout=30)


def _kill_all(procs):
    for p in procs:
        if p.poll() is None:
            p.kill()
        _communicate(p)


# ---------------------------------------------------------------- in-process unit tests
def _pair(peer_timeout_s=60.0):
    import torch.distributed as dist

    store = dist.HashStore()
    fired = {}

    def mk(r):
        return JobWatchdog(r, 2, peer_timeout_s=peer_timeout_s, poll_s=0.05, store=dist.PrefixStore("t/", store),
                           exit_fn=lambda code, r=r: fired.setdefault(r, code))

    return mk(0), mk(1), fired


def _until(cond, s=5.0):
    t0 = time.monotonic()
    while not cond() and time.monotonic() - t0 < s:
        time.sleep(0.02)
    return cond()


def test_watchdog_abort_reaches_peer():
    a, b, fired = _pair()
    a.start(), b.start()
    try:
        b.abort("boom")
        assert _until(lambda: 0 in fired and 1 in fired)
        assert fired == {0: PEER_ABORT_EXIT, 1: PEER_ABORT_EXIT}
        assert "rank 1: boom" in a.aborted
    finally:
        a.stop(), b.stop()


def test_watchdog_declares_silent_peer_dead():
    a, b, fired = _pair(peer_timeout_s=0.5)
    b._store.set("hb/1", "0")  # rank 1 registered, then never beats again (SIGKILL / hang with the GIL held)
    a.start()
    try:
        assert _until(lambda: 0 in fired)
        assert "no heartbeat from rank 1" in a.aborted
        assert b._store.get("abort").startswith(b"rank 0:")  # published for the others
    finally:
        a.stop()


def test_watchdog_finished_peer_is_not_dead():
    a, b, fired = _pair(peer_timeout_s=0.3)
    a.start(), b.start()
    b.stop()  # rank 1 finished first and left
    time.sleep(1.0)
    assert fired == {}
    a.stop()


def test_watchdog_store_loss_is_an_abort():
    """The rendezvous store's host died (its rank, or the agent): every store call fails; after a grace period
    (a clean job end could have raced the final barrier) the watchdog exits with the peer-abort status."""
    import torch.distributed as dist

    class Dying:
        def __init__(self):
            self.inner, self.dead = dist.PrefixStore("t/", dist.HashStore()), False

        def __getattr__(self, name):
            fn = getattr(self.inner, name)

            def call(*a, **kw):
                if self.dead:
                    raise RuntimeError("Connection reset by peer")
                return fn(*a, **kw)

            return call

    store, fired = Dying(), {}
    w = JobWatchdog(0, 2, poll_s=0.05, store=store, exit_fn=lambda code: fired.setdefault(0, code))
    w.start()
    try:
        time.sleep(0.2)
        assert fired == {}
        store.dead = True
        assert _until(lambda: 0 in fired, 5.0)
        assert fired[0] == PEER_ABORT_EXIT and "store unreachable" in w.aborted
    finally:
        w.stop()


# ---------------------------------------------------------------- multi-process
@pytest.mark.timeout(200)
def test_process_stopped_reads_the_state():
    """The death watch beats only for a rank that is not stopped: /proc state T after SIGSTOP, not after SIGCONT;
    a process that is gone is not 'stopped' (its death is the pipe's EOF)."""
    from ddl_amd.parallel.abort import _process_stopped

    p = subprocess.Popen([sys.executable, "-c", "import time; time.sleep(60)"])
    try:
        assert not _process_stopped(p.pid)
        os.kill(p.pid, signal.SIGSTOP)
        t0 = time.monotonic()
        while not _process_stopped(p.pid) and time.monotonic() - t0 < 5:
            time.sleep(0.01)
        assert _process_stopped(p.pid)
        os.kill(p.pid, signal.SIGCONT)
        t0 = time.monotonic()
        while _process_stopped(p.pid) and time.monotonic() - t0 < 5:
            time.sleep(0.01)
        assert not _process_stopped(p.pid)
    finally:
        p.kill()
        p.wait()
    assert not _process_stopped(p.pid)


def test_raise_in_window_aborts_every_rank_plain_launch():
    """gloo W=4, exchange on: rank 2 raises when its cursor enters window 3. Rank 2 exits 1, every
    other rank exits PEER_ABORT_EXIT within seconds (not the 600 s process-group timeout)."""
    procs = _launch_plain(4, BENCH + ["--gpus", "4"], _base_env(DDL_FAULT_RANK="2:3"))
    try:
        codes, took = _wait_all(procs, 150)
        errs = [_communicate(p)[1] for p in procs]
    finally:
        _kill_all(procs)
    assert codes[2] == 1, errs[2][-2000:]
    assert "injected fault in rank 2 at window 3" in errs[2]
    for r in (0, 1, 3):
        # the watchdog's abort, or -- when gloo notices rank 2's closed sockets first -- the peer's own
        # collective error, which aborts the job the same way
        assert codes[r] in (PEER_ABORT_EXIT, 1), (r, codes, errs[r][-2000:])
        assert ("job aborted (rank 2: RuntimeError: injected fault" in errs[r]
                or "aborting the job" in errs[r]), errs[r][-2000:]
    assert PEER_ABORT_EXIT in codes
    assert took < 120 < PG_TIMEOUT_S


@pytest.mark.timeout(200)
@pytest.mark.parametrize("launch", ["torchrun", "self"])
def test_raise_in_window_fails_the_job(launch):
    """The same fault under the driver's torchrun line and under ``bench.py --gpus 4``'s self-launch:
    the job exits non-zero well inside the process-group timeout and prints no JSON line."""
    env = _base_env(DDL_FAULT_RANK="2:3")
    args = BENCH + ["--gpus", "4"]
    if launch == "torchrun":
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), *args]
    else:
        cmd = [sys.executable, *args]
    t0 = time.monotonic()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=env)
    took = time.monotonic() - t0
    assert r.returncode != 0
    assert "injected fault in rank 2 at window 3" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert took < 150


@pytest.mark.timeout(200)
def test_silent_hang_detected_by_heartbeat():
    """Rank 1 SIGSTOPs itself (sockets stay open, so gloo never errors; the peers block in an
    all-reduce): its watcher sees no heartbeat for peer_timeout_s = 3 s and aborts the job."""
    script = os.path.join(REPO, "tests", "abort_rank.py")
    procs = _launch_plain(3, [script, "--stop-rank", "1", "--peer-timeout", "3"], _base_env())
    try:
        t0 = time.monotonic()
        while time.monotonic() - t0 < 150 and (procs[0].poll() is None or procs[2].poll() is None):
            time.sleep(0.1)
        codes = [p.poll() for p in procs]
    finally:
        if procs[1].poll() is None:
            os.kill(procs[1].pid, signal.SIGCONT)
        _kill_all(procs)
    assert codes[0] == PEER_ABORT_EXIT and codes[2] == PEER_ABORT_EXIT, codes
    assert codes[1] is None  # still stopped when the others had gone


@pytest.mark.timeout(200)
def test_killed_rank_ends_the_job_at_once():
    """Rank 1 is SIGKILLed while the others compute (no collective in flight, so no socket error can
    tell them): its death watch sees the pipe to the dead rank close and publishes the abort, and the
    peers exit PEER_ABORT_EXIT within seconds -- long before the 60 s heartbeat timeout."""
    script = os.path.join(REPO, "tests", "abort_rank.py")
    procs = _launch_plain(3, [script, "--kill-rank", "1", "--peer-timeout", "60"], _base_env())
    try:
        codes, took = _wait_all(procs, 150)
        errs = [_communicate(p)[1] for p in procs]
    finally:
        _kill_all(procs)
    assert codes[1] == -signal.SIGKILL, codes
    assert codes[0] == PEER_ABORT_EXIT and codes[2] == PEER_ABORT_EXIT, (codes, errs[0][-1500:])
    assert "died without a clean shutdown" in errs[0] and "died without a clean shutdown" in errs[2]
    # the peers' own death watches stand down when they exit on the abort: no second, false death report
    assert "rank 0: process" not in errs[0] and "rank 2: process" not in errs[2]
    assert took < 30 < 60


@pytest.mark.timeout(200)
def test_gil_holding_rank_is_not_declared_dead():
    """Rank 1 holds the GIL for 8 s in one C call, with peer_timeout_s = 3 s: its Python threads cannot run,
    but it is alive -- the heartbeat comes from its death-watch process (which checks that the rank exists
    and is not stopped), so the job is not aborted and every rank finishes."""
    script = os.path.join(REPO, "tests", "abort_rank.py")
    procs = _launch_plain(3, [script, "--gil-hold-rank", "1", "--gil-hold-s", "8", "--iters", "40",
                              "--peer-timeout", "3"], _base_env())
    try:
        codes, _ = _wait_all(procs, 150)
        outs = [_communicate(p) for p in procs]
    finally:
        _kill_all(procs)
    assert codes == [0, 0, 0], (codes, [o[1][-1500:] for o in outs])
    assert all(f"rank {r} done" in outs[r][0] for r in range(3))


@pytest.mark.timeout(200)
def test_clean_run_exits_zero_with_watchdog():
    """No fault: every rank finishes, the watchdog never fires (ranks finish at different times)."""
    script = os.path.join(REPO, "tests", "abort_rank.py")
    procs = _launch_plain(3, [script, "--iters", "60", "--peer-timeout", "2"], _base_env())
    try:
        codes, _ = _wait_all(procs, 150)
        outs = [_communicate(p) for p in procs]
    finally:
        _kill_all(procs)
    assert codes == [0, 0, 0], [o[1][-1500:] for o in outs]


@pytest.mark.timeout(200)
def test_start_timeout_reaches_the_process_group():
    """``start(timeout_s=)`` is the collectives' timeout too (it used to stop at the shm waits, the
    groups kept a hard-coded 600 s): without the watchdog, a peer that stops answering makes the
    others' all-reduce fail after ~timeout_s."""
    script = os.path.join(REPO, "tests", "abort_rank.py")
    procs = _launch_plain(3, [script, "--stop-rank", "1", "--no-abort", "--timeout", "6"], _base_env())
    try:
        t0 = time.monotonic()
        while time.monotonic() - t0 < 150 and (procs[0].poll() is None or procs[2].poll() is None):
            time.sleep(0.1)
        took = time.monotonic() - t0
        codes = [p.poll() for p in procs]
    finally:
        if procs[1].poll() is None:
            os.kill(procs[1].pid, signal.SIGCONT)
        _kill_all(procs)
    assert codes[0] not in (None, 0, PEER_ABORT_EXIT) and codes[2] not in (None, 0, PEER_ABORT_EXIT), codes
    assert took < 90  # start-up + ~6 s, far from the 600 s default


@pytest.mark.timeout(120)
def test_death_watch_beats_only_while_liveness_tokens_arrive(monkeypatch):
    """The death watch keeps a rank's heartbeat going while its Python threads cannot run (a long C call holding
    the GIL) -- but only for hang_timeout_s after the last liveness token: a rank hung for longer stops beating,
    so its watcher aborts the job before the collective timeout would."""
    import time
    from datetime import timedelta

    import torch.distributed as dist

    from ddl_amd.parallel.abort import DeathWatch, _job_key
    from tests.mp_harness import free_port

    port = free_port()
    master = dist.TCPStore("127.0.0.1", port, is_master=True, timeout=timedelta(seconds=30), wait_for_workers=False)
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(port))
    monkeypatch.delenv("DDL_PRODUCER_MODE", raising=False)
    store = dist.PrefixStore(f"ddl_amd/abort/{_job_key()}/", master)
    dw = DeathWatch.spawn(7)
    assert dw is not None
    try:
        def hb():
            return store.get("hb/7") if store.check(["hb/7"]) else b""

        def moving(seconds: float, tokens: bool) -> bool:
            t_end, seen = time.monotonic() + seconds, {hb()}
            while time.monotonic() < t_end:
                if tokens:
                    dw.alive()
                time.sleep(0.05)
                seen.add(hb())
            return len(seen) > 2

        assert dw.beat(0.05, 1.0)
        t0 = time.monotonic()
        while hb() == b"" and time.monotonic() - t0 < 60:  # the child imports torch first
            dw.alive()
            time.sleep(0.05)
        assert moving(1.5, tokens=True)        # tokens arrive: the death watch beats
        time.sleep(1.5)                          # no token for longer than hang_timeout_s ...
        assert not moving(1.0, tokens=False)    # ... the beats stop: the rank counts as hung
        assert moving(1.5, tokens=True)         # tokens again: beating again
    finally:
        dw.done()
