"""Direct-DMA staging on the card: bit-exact batches and bounded waits.

Window copies go straight onto SDMA engines through ROCr (``csrc/kernels/stager.cpp``); every consumer of a
window waits for its copy's completion signal on the host. These tests hold the delivered batches to the
PRODUCER'S BYTES (``ops.ref_gather_rows`` over the window the producer wrote, in the window's Feistel
order), which is the reference's batch semantics -- a slice of the producer's window
(``/root/reference/ddl/mpi_dataloader.py:179-198``) -- plus the device shuffle; and they check that a copy that
never lands fails the loader within its timeout instead of hanging it (the reference's consumer blocks in
``Recv`` forever, ``/root/reference/ddl/connection.py:154``).
"""

import time

import pytest
import torch

import ddl_amd
from ddl_amd import Marker, ops
from ddl_amd.dataloader import window_perm_key
from ddl_amd.permutation import FeistelPermutation
from tests.helpers import IdProducer

pytestmark = pytest.mark.gpu

N, WIDTH, B, P, SEED = 64, 8, 16, 2, 3


def _dispatch(name: str):
    """StagingSpec.native_dispatch for a test's dispatch id ("python": the Python path)."""
    return False if name == "python" else name


def producer_window(p: int, rnd: int) -> torch.Tensor:
    """The window producer ``p`` writes in round ``rnd`` (IdProducer._write, rank 0), int32 [N, WIDTH]."""
    t = torch.empty(N, WIDTH, dtype=torch.int32)
    prod = IdProducer(N, WIDTH)
    prod.rank_global, prod.producer_index = 0, p
    prod._write(t, rnd)
    return t


def expected_batch(w: int, local: int) -> torch.Tensor:
    p, rnd = w % P, w // P  # round-robin schedule, one slot per producer
    perm = FeistelPermutation(N, SEED, window_perm_key(p, rnd))
    return ops.ref_gather_rows(producer_window(p, rnd), perm=perm, base=local * B, n_rows=B)


@pytest.fixture(params=[True, False], ids=["direct_dma", "hip_streams"])
def direct(request, monkeypatch):
    """Both staging paths: window copies straight onto SDMA engines through ROCr, and the HIP copy-stream
    fallback (what runs whenever ROCr refuses direct DMA)."""
    from ddl_amd import staging

    monkeypatch.setattr(staging, "DIRECT_DMA", request.param)
    return request.param


@pytest.mark.parametrize("dispatch", ["lookahead", "inline", "python"])
@pytest.mark.parametrize("slow", [False, True])
def test_direct_dma_batches_equal_the_producers_bytes(dispatch, slow, direct):
    """Every batch, fast or slow consumer (the ring refills a 2-buffer ring many times), through the native
    engine and the Python dispatch path, on direct DMA and on the HIP copy-stream fallback, equals the
    producer's window rows in the window's order, bitwise."""
    with ddl_amd.start(n_producers=P) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(N, WIDTH), B, conn, 8, env=env, device=torch.device("cuda"),
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           staging=ddl_amd.StagingSpec(prefetch_depth=2,
                                                                       native_dispatch=_dispatch(dispatch)),
                                           order=ddl_amd.OrderSpec(shuffle="device", seed=SEED))
        st = dl.stats()
        assert st["direct_dma"] is direct, st.get("direct_dma_reason")
        w = 0
        for e in range(8):
            for i in range(len(dl)):
                a, b = dl[i]
                got = torch.cat([a, b], 1).cpu()
                assert torch.equal(got, expected_batch(w, i)), (w, i)
                if slow:
                    time.sleep(0.003)
                dl.mark(Marker.END_OF_BATCH)
            w += 1
            if e < 7:
                dl.mark(Marker.END_OF_EPOCH)
        dl._stager.settle()
        st = dl.stats()
        assert st["bytes_landed"] == st["bytes_h2d"] == 8 * N * WIDTH * 4
        dl.close()


@pytest.mark.parametrize("dispatch", ["lookahead", "python"])
def test_stuck_copy_raises_within_the_timeout_and_close_returns(dispatch):
    """A window copy whose completion signal never drops (fault injection: armed one too high, what a hung
    SDMA engine looks like) fails the consumer with DDLTimeoutError naming the window and the engine within
    the loader's timeout, and close() returns promptly -- no wait anywhere is unbounded."""
    from ddl_amd.exceptions import DDLTimeoutError

    timeout_s = 3.0
    with ddl_amd.start(n_producers=P) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(N, WIDTH), B, conn, 8, env=env, device=torch.device("cuda"),
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           staging=ddl_amd.StagingSpec(prefetch_depth=2,
                                                                       timeout_s=timeout_s,
                                               native_dispatch=_dispatch(dispatch)),
                                           order=ddl_amd.OrderSpec(shuffle="device", seed=SEED))
        if not dl._stager.direct_dma:
            pytest.skip(f"no direct DMA here: {dl.stats()['direct_dma_reason']}")
        dl._stager._native.inject_stuck_copy(3)  # windows 0 and 1 fill the 2-buffer ring; 3 is not staged yet
        t0 = time.monotonic()
        with pytest.raises(DDLTimeoutError) as ei:
            for e in range(8):
                for i in range(len(dl)):
                    if e == 2 and i == 0:
                        t0 = time.monotonic()  # window 3's copy is enqueued from here on (window 1 released)
                    dl[i]
                    dl.mark(Marker.END_OF_BATCH)
                dl.mark(Marker.END_OF_EPOCH)
        waited = time.monotonic() - t0
        msg = str(ei.value)
        assert "window 3" in msg and "SDMA engine" in msg and "did not complete" in msg, msg
        assert waited < timeout_s + 5.0, waited
        t1 = time.monotonic()
        dl.close()
        assert time.monotonic() - t1 < 15.0


@pytest.mark.parametrize("dispatch", ["lookahead", "python"])
def test_consumer_times_out_first_and_pending_copies_are_quarantined(dispatch):
    """The consumer's wait on a stuck copy times out BEFORE the retire thread's (which is given 30 s more):
    the retire thread then gives up on that copy too, and every copy still queued -- the stuck one and the
    ones behind it -- is quarantined: its completion signal is never destroyed, and close() keeps the HBM
    ring and the pinned arena allocated (an engine that recovers later writes into live memory, not into
    freed or reused memory). close() still returns promptly."""
    from ddl_amd import staging
    from ddl_amd.exceptions import DDLTimeoutError

    timeout_s = 2.0
    with ddl_amd.start(n_producers=P) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(N, WIDTH), B, conn, 8, env=env, device=torch.device("cuda"),
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           staging=ddl_amd.StagingSpec(prefetch_depth=2,
                                                                       timeout_s=timeout_s,
                                               native_dispatch=_dispatch(dispatch)),
                                           order=ddl_amd.OrderSpec(shuffle="device", seed=SEED))
        st = dl._stager
        if not st.direct_dma:
            pytest.skip(f"no direct DMA here: {dl.stats()['direct_dma_reason']}")
        st._native.inject_slow_retire(30000)
        st._native.inject_stuck_copy(3)
        ring = [b.data_ptr() for b in st.buffers]
        n_q = len(staging._QUARANTINE)
        t0 = time.monotonic()
        with pytest.raises(DDLTimeoutError) as ei:
            for e in range(8):
                for i in range(len(dl)):
                    dl[i]
                    dl.mark(Marker.END_OF_BATCH)
                dl.mark(Marker.END_OF_EPOCH)
        assert "window 3" in str(ei.value)
        assert time.monotonic() - t0 < 4 * timeout_s + 5.0  # the consumer's own timeout, not the retire's 32 s
        deadline = time.monotonic() + 5.0
        while not st.poisoned and time.monotonic() < deadline:  # the retire thread sees the stuck flag
            time.sleep(0.01)
        assert st.poisoned and st._native.leaked_signals >= 1
        t1 = time.monotonic()
        dl.close()
        assert time.monotonic() - t1 < 15.0
        assert len(staging._QUARANTINE) == n_q + 1
        kept, arena, _ = staging._QUARANTINE[-1]
        assert [b.data_ptr() for b in kept] == ring and arena is conn.arena
        assert getattr(conn, "_quarantined", False)


def test_direct_dma_copy_timing_is_off_unless_asked():
    """ROCr's async-copy profiling is process-wide: a loader turns it on only with copy_timing=True, and its
    stager turns it off again when it is done with it (reference counted)."""
    with ddl_amd.start(n_producers=P) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(N, WIDTH), B, conn, 2, env=env, device=torch.device("cuda"),
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           staging=ddl_amd.StagingSpec(prefetch_depth=2))
        st = dl._stager
        assert not st.copy_timing
        st.copy_timing = True
        assert st.copy_timing
        st.copy_timing = False
        assert not st.copy_timing
        for _ in dl:
            dl.mark(Marker.END_OF_BATCH)
        dl.mark(Marker.END_OF_EPOCH)
        dl.close()


def test_close_interrupts_a_pending_free_event_wait(direct):
    """The stager waits for a ring buffer's free event (recorded behind the consumer's reads) by polling, so
    close() ends that wait at once even while the consumer's stream is still busy: here a ~3 s spin kernel sits
    on the batch stream in front of the last batch kernel of window 0, and so in front of window 0's free
    event, while the stager wants buffer 0 back for window 2. Same on the HIP copy-stream fallback (its
    free-event wait is polled on the host too)."""
    from ddl_amd.utils import streams

    with ddl_amd.start(n_producers=P) as (env, conn):
        # calibrate the spin kernel (its clock is the shader clock): cycles per second
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        torch.cuda._sleep(int(1e8))
        e1.record()
        e1.synchronize()
        cycles_per_s = 1e8 / max(1e-4, e0.elapsed_time(e1) / 1e3)
        dl = ddl_amd.DistributedDataLoader(
            IdProducer(N, WIDTH), B, conn, 8, env=env, device=torch.device("cuda"),
            order=ddl_amd.OrderSpec(shuffle="device", seed=SEED), output=ddl_amd.OutputSpec(copy_batches=True),
            staging=ddl_amd.StagingSpec(prefetch_depth=2, native_dispatch=False))
        assert dl._stager.direct_dma is direct and dl._stager._native.free_on_host
        bs, n = dl._batch_stream, len(dl)
        assert n == 4
        for i in range(n):
            if i == n - 2:  # batch n-1 (the window's last kernel) is enqueued when batch n-2 is fetched
                with streams.on_stream(bs):
                    torch.cuda._sleep(int(3.0 * cycles_per_s))
            dl[i]
            dl.mark(Marker.END_OF_BATCH)  # the last mark releases window 0 with its (pending) free event
        time.sleep(0.3)  # the stager is now waiting for that free event (window 2 needs buffer 0)
        assert not bs.query(), "the spin kernel finished too early for this test"
        assert dl._stager.windows_staged == 2  # window 2's copy is held by the pending free event
        t0 = time.monotonic()
        dl._stager._native.close()
        assert time.monotonic() - t0 < 1.0
        assert not bs.query()  # the wait was interrupted, not satisfied
        dl.close()


@pytest.mark.timeout(300)
def test_long_run_reanchors_and_flags_trimmed_copy_logs():
    """Past 4096 retires the stager re-anchors its device clock (off its lock), and past the 16,384 copies its
    logs keep, an interval or window that starts before the oldest kept record says so (``truncated`` /
    ``complete=False``) instead of undercounting; a recent interval still counts exactly."""
    from ddl_amd import _native

    rt = _native.runtime()
    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    n_win = 20000
    with ddl_amd.start(n_producers=P) as (env, conn):
        e0 = ev()
        e0.record()
        t0_ns = rt.now_ns()
        dl = ddl_amd.DistributedDataLoader(IdProducer(64, 64), 64, conn, n_win, env=env, device=torch.device("cuda"),
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           staging=ddl_amd.StagingSpec(prefetch_depth=4, copy_timing=True))
        em = None
        for e in range(n_win):
            if e == n_win - 200:
                torch.cuda.synchronize()
                em = ev()
                em.record()
            dl[0]
            dl.mark(Marker.END_OF_BATCH)
            if e + 1 < n_win:
                dl.mark(Marker.END_OF_EPOCH)
        torch.cuda.synchronize()
        e1 = ev()
        e1.record()
        e1.synchronize()
        st = dl._stager
        st.settle()
        assert st._native.reanchors >= 3, st._native.reanchors
        whole = st.bytes_in_interval(e0, e1)
        assert not whole["ok"] and whole["truncated"]
        recent = st.bytes_in_interval(em, e1)
        assert recent["ok"] and not recent["truncated"] and recent["bytes"] > 0
        assert recent["bytes"] <= 200 * 64 * 64 * 4 + 1e-6
        _, _, complete = st._native.copies_between(t0_ns, rt.now_ns())
        assert not complete
        dl.close()
