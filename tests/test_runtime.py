"""Native host runtime: shm arena, slot state machine, futex waits, liveness, host gather.

Replaces the reference's MPI windows + tag-7 handshake (reference
ddl/connection.py:88-187); tested across real processes (SURVEY §4.4 level 1).
"""

import multiprocessing as mp
import multiprocessing.connection
import os
import threading
import time
import uuid

import numpy as np
import pytest

from ddl_amd import _native

rt = _native.runtime()


def _name():
    return f"/ddl_amd.t.{os.getpid()}.{uuid.uuid4().hex[:6]}"


@pytest.fixture
def arena():
    a = rt.Arena.create(_name(), [1000, 5 << 20, 3], 2)
    a.unlink()
    yield a


def test_layout_alignment_and_capacity(arena):
    assert arena.n_producers == 3 and arena.n_slots == 2
    seen = set()
    for p in range(3):
        for s in range(2):
            addr = arena.slot_address(p, s)
            assert (addr - arena.base_address) % rt.DATA_ALIGN == 0
            assert arena.get_state(p, s) == rt.EMPTY
            seen.add(addr)
    assert len(seen) == 6
    assert arena.slot_capacity(1, 0) == 5 << 20
    # regions do not overlap
    addrs = sorted((arena.slot_address(p, s), arena.slot_capacity(p, s)) for p in range(3) for s in range(2))
    for (a0, c0), (a1, _) in zip(addrs, addrs[1:]):
        assert a0 + c0 <= a1


def test_attach_shares_memory_and_metadata():
    name = _name()
    a = rt.Arena.create(name, [4096], 1)
    b = rt.Arena.attach(name)
    a.unlink()
    va = np.frombuffer(a.slot_view(0, 0), dtype=np.uint8)
    vb = np.frombuffer(b.slot_view(0, 0), dtype=np.uint8)
    va[:] = 42
    assert (vb == 42).all()
    b.publish(0, 0, seq=7, used_bytes=100, epoch=3, tags=[5, -6])
    info = a.slot_info(0, 0)
    assert (info["state"], info["seq"], info["used_bytes"], info["epoch"]) == (rt.READY, 7, 100, 3)
    assert info["tag"][:2] == [5, -6]
    assert a.attached() == 1


def test_attach_missing_or_bad():
    with pytest.raises(RuntimeError):
        rt.Arena.attach("/ddl_amd.does.not.exist")
    with pytest.raises(ValueError):
        rt.Arena.create(_name(), [], 1)
    with pytest.raises(ValueError):
        rt.Arena.create(_name(), [10], 0)


def test_publish_overflow_rejected(arena):
    with pytest.raises(IndexError):
        arena.publish(0, 0, 1, 2000)


def test_wait_timeout_is_bounded(arena):
    t0 = time.monotonic()
    rc = arena.wait_state(0, 0, rt.READY, 150)
    dt = time.monotonic() - t0
    assert rc == rt.WaitResult.TIMEOUT
    assert 0.1 < dt < 2.0


def test_wait_wakes_on_publish_from_other_thread(arena):
    res = {}

    def waiter():
        t0 = time.monotonic()
        res["rc"] = arena.wait_state(1, 1, rt.READY, 10_000)
        res["dt"] = time.monotonic() - t0

    th = threading.Thread(target=waiter)
    th.start()
    time.sleep(0.1)
    arena.publish(1, 1, 1, 10)
    th.join(5)
    assert res["rc"] == rt.WaitResult.OK
    assert res["dt"] < 1.0


def test_shutdown_wakes_blocked_waiter(arena):
    res = {}

    def waiter():
        res["rc"] = arena.wait_state(0, 1, rt.READY, -1)

    th = threading.Thread(target=waiter)
    th.start()
    time.sleep(0.1)
    t0 = time.monotonic()
    arena.request_shutdown()
    th.join(5)
    assert not th.is_alive()
    assert res["rc"] == rt.WaitResult.SHUTDOWN
    assert time.monotonic() - t0 < 1.0
    assert arena.shutdown_requested()


def test_failed_producer_reported(arena):
    arena.mark_failed(2)
    assert arena.failed_producer() == 2
    assert arena.wait_state(2, 0, rt.READY, 5000, 0, 2) == rt.WaitResult.PEER_FAILED


def _exit_child(code):
    os._exit(code)


def test_dead_peer_detected_even_as_zombie(arena):
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_exit_child, args=(3,))
    p.start()
    # The sentinel becomes readable when the child exits, without reaping it: the child is
    # a zombie from here on (a spawn child can take seconds to start on a loaded host).
    assert mp.connection.wait([p.sentinel], timeout=60)
    t0 = time.monotonic()
    rc = arena.wait_state(0, 0, rt.READY, 10_000, p.pid, -1)
    assert rc == rt.WaitResult.PEER_DEAD
    assert time.monotonic() - t0 < 2.0
    p.join()
    assert not rt.pid_alive(p.pid)
    assert rt.pid_alive(os.getpid())


def test_cas_state(arena):
    assert arena.cas_state(0, 0, rt.EMPTY, rt.HELD)
    assert not arena.cas_state(0, 0, rt.EMPTY, rt.READY)
    assert arena.get_state(0, 0) == rt.HELD


def _producer_proc(name, rounds):
    a = rt.Arena.attach(name)
    a.set_producer_pid(0, os.getpid())
    for r in range(rounds):
        s = r % a.n_slots
        assert a.wait_state(0, s, rt.EMPTY, 20_000) == rt.WaitResult.OK
        v = np.frombuffer(a.slot_view(0, s), dtype=np.int64)
        v[:] = r
        a.publish(0, s, r, v.nbytes, 0, [r * 3])
        a.heartbeat(0, 1, 1)
    a.set_producer_status(0, rt.STATUS_DONE)


@pytest.mark.parametrize("n_slots", [1, 3])
def test_cross_process_ping_pong(n_slots):
    name = _name()
    a = rt.Arena.create(name, [8 * 1024], n_slots)
    rounds = 300
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_producer_proc, args=(name, rounds))
    p.start()
    try:
        for r in range(rounds):
            s = r % n_slots
            assert a.wait_state(0, s, rt.READY, 20_000, p.pid, 0) == rt.WaitResult.OK
            info = a.slot_info(0, s)
            assert info["seq"] == r and info["tag"][0] == r * 3
            v = np.frombuffer(a.slot_view(0, s), dtype=np.int64)
            assert (v == r).all()
            a.set_state(0, s, rt.EMPTY)
        p.join(20)
        assert p.exitcode == 0
        assert a.producer_info(0)["rounds"] == rounds
        assert a.producer_info(0)["status"] == rt.STATUS_DONE
    finally:
        a.unlink()
        if p.is_alive():
            p.kill()


@pytest.mark.parametrize("row_bytes", [1, 7, 36, 4096, 301056])
@pytest.mark.parametrize("threads", [1, 4])
def test_host_gather_rows(row_bytes, threads):
    n = 200 if row_bytes < 100_000 else 20
    src = np.random.default_rng(0).integers(0, 255, size=(n, row_bytes), dtype=np.uint8)
    idx = np.random.default_rng(1).integers(0, n, size=57).astype(np.int64)
    dst = np.zeros((57, row_bytes), dtype=np.uint8)
    rt.gather_rows(dst.ctypes.data, src.ctypes.data, row_bytes, idx, n, threads)
    assert np.array_equal(dst, src[idx])


def test_host_gather_bounds_checked():
    src = np.zeros((4, 8), np.uint8)
    dst = np.zeros((1, 8), np.uint8)
    with pytest.raises(IndexError):
        rt.gather_rows(dst.ctypes.data, src.ctypes.data, 8, np.array([4], np.int64), 4, 1)
    with pytest.raises(IndexError):
        rt.gather_rows(dst.ctypes.data, src.ctypes.data, 8, np.array([-1], np.int64), 4, 1)


def test_parallel_copy():
    src = np.random.default_rng(0).integers(0, 255, size=(30 << 20) + 13, dtype=np.uint8)
    dst = np.zeros_like(src)
    rt.parallel_copy(dst.ctypes.data, src.ctypes.data, src.nbytes, 4)
    assert np.array_equal(src, dst)


@pytest.mark.parametrize("dtype,widths", [(np.float32, (3, 5, 1)), (np.uint8, (1, 7)), (np.int64, (4,))])
@pytest.mark.parametrize("threads", [1, 4])
def test_host_pack_columns(dtype, widths, threads):
    import torch

    from ddl_amd import ops

    n = 70_001
    rng = np.random.default_rng(3)
    groups = [torch.from_numpy((rng.random((n, w)) * 100).astype(dtype)) for w in widths]
    out = ops.pack_columns(groups, host_threads=threads)
    assert torch.equal(out, torch.cat(groups, dim=1))
    # identity slice with an offset + a permuted (reference-path) pack
    part = ops.pack_columns(groups, base=123, n_rows=1000)
    assert torch.equal(part, torch.cat(groups, dim=1)[123:1123])
    idx = torch.from_numpy(rng.permutation(n)[:500].astype(np.int64))
    assert torch.equal(ops.pack_columns(groups, idx), torch.cat(groups, dim=1)[idx])
