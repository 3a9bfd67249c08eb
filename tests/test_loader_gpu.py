"""End-to-end loader on one MI355X: producers -> pinned shm -> H2D stager -> gfx950 kernels."""

import numpy as np
import pytest
import torch

import ddl_amd
from ddl_amd import Marker
from ddl_amd.dataloader import window_perm_key
from ddl_amd.specs import from_flat
from ddl_amd.permutation import FeistelPermutation
from tests.helpers import IdProducer

pytestmark = pytest.mark.gpu


def _run(n_producers=3, n=64, bs=16, epochs=6, shuffle="device", n_slots=1, depth=2, out_dtype=None):
    seen = []
    with ddl_amd.start(n_producers=n_producers) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IdProducer(n, 8), bs, conn, epochs, env=env,
                                           output=ddl_amd.OutputSpec(dtype=out_dtype),
                                           staging=ddl_amd.StagingSpec(n_slots=n_slots, prefetch_depth=depth),
                                           order=ddl_amd.OrderSpec(shuffle=shuffle, seed=11))
        assert dl.device.type == "cuda"
        for e in range(epochs):
            rows = []
            for i, (a, b) in enumerate(dl):
                assert a.is_cuda and a.shape == (bs, 2) and b.shape == (bs, 6)
                rows.append(torch.cat([a, b], 1).cpu())
                dl.mark(Marker.END_OF_BATCH)
            dl.mark(Marker.END_OF_EPOCH)
            seen.append(torch.cat(rows))
        st = dl.stats()
    return seen, st


def test_gpu_epochs_exactly_once_and_round_robin():
    seen, st = _run()
    assert st["windows_staged"] == 6
    for e, rows in enumerate(seen):
        assert rows.shape == (64, 8)
        assert sorted(rows[:, 2].tolist()) == list(range(64))  # every sample exactly once
        assert set(rows[:, 1].tolist()) == {e % 3}              # round-robin over producers
        assert set(rows[:, 3].tolist()) == {e // 3}             # producer round
        assert torch.equal(rows[:, 4], rows[:, 2] * 7 + 4)      # row content intact


def test_gpu_device_shuffle_matches_feistel_and_is_deterministic():
    seen1, _ = _run(epochs=3)
    seen2, _ = _run(epochs=3)
    for e in range(3):
        assert torch.equal(seen1[e], seen2[e])
        p = e % 3
        perm = FeistelPermutation(64, 11, window_perm_key(p, e // 3)).full()
        assert np.array_equal(seen1[e][:, 2].numpy(), perm)


def test_gpu_no_shuffle_zero_copy_order():
    seen, _ = _run(shuffle="none", epochs=2, n_slots=2, depth=3)
    for rows in seen:
        assert rows[:, 2].tolist() == list(range(64))


def test_gpu_multi_slot_deep_prefetch():
    seen, st = _run(n_producers=2, n_slots=3, depth=4, epochs=9)
    for e, rows in enumerate(seen):
        assert set(rows[:, 1].tolist()) == {e % 2}
        assert set(rows[:, 3].tolist()) == {e // 2}


def test_gpu_indexed_mode_world_size_invariant_order():
    import numpy as np

    from ddl_amd.models import IndexedProducer, SharedArraySource
    from ddl_amd.permutation import EpochOrder

    n, gb = 2000, 128
    data = torch.stack([torch.arange(n), torch.arange(n) * 3], 1)
    src = SharedArraySource.create(f"ddl_amd_gsrc_{np.random.randint(1 << 30)}", data)
    try:
        with ddl_amd.start(n_producers=3) as (env, conn):
            dl = ddl_amd.DistributedDataLoader(IndexedProducer(src, gb), gb, conn, 2, env=env, auto_mark=True,
                                               order=ddl_amd.OrderSpec(mode="indexed", seed=9))
            order = EpochOrder(n, gb, 9)
            for e in range(2):
                got = torch.cat([b[0][:, 0].cpu() for b in dl]).numpy()
                assert np.array_equal(got, order.perm(e).full()[: order.batches_per_epoch * gb])
    finally:
        src.close()


def test_gpu_file_source_indexed_and_resident(tmp_path):
    from ddl_amd.models import FileRowsSource, IndexedProducer
    from ddl_amd.permutation import EpochOrder
    from ddl_amd.resident import ResidentGlobalLoader

    n, gb = 3000, 128
    arr = np.random.default_rng(0).integers(0, 255, size=(n, 3, 8, 8), dtype=np.uint8)
    path = tmp_path / "imgs.npy"
    np.save(path, arr)
    src = FileRowsSource.from_npy(str(path), direct=True)
    order = EpochOrder(n, gb, 5)
    ref = arr[order.perm(0).full()[: order.batches_per_epoch * gb]]
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IndexedProducer(src, gb), gb, conn, 1, env=env, auto_mark=True,
                                           order=ddl_amd.OrderSpec(mode="indexed", seed=5))
        got = torch.cat([b[0].cpu() for b in dl]).numpy()
    assert np.array_equal(got.reshape(ref.shape), ref)
    res = ResidentGlobalLoader(src, gb, seed=5, n_epochs=1, chunk_bytes=64 << 10)
    assert res.shard.is_cuda
    got = torch.cat([b.cpu() for b in res]).numpy()
    assert np.array_equal(got, ref)
    res.close()


def test_gpu_uint8_normalised_and_hwc_collate():
    from ddl_amd.models.producers import ImageWindowProducer

    mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(ImageWindowProducer(32, (3, 24, 24), "uint8", refill="none"), 8, conn, 2,
                                           env=env,
                                           output=ddl_amd.OutputSpec(dtype=torch.bfloat16, normalize={"mean": mean,
                                                                     "std": std}),
                                           order=ddl_amd.OrderSpec(shuffle="none"))
        (x,) = dl[0]
        _, win = dl.arys[0][0]
        ref = ((win[:8].float() / 255 - torch.tensor(mean).view(1, 3, 1, 1)) / torch.tensor(std).view(1, 3, 1, 1))
        torch.testing.assert_close(x.float().cpu(), ref, rtol=1e-2, atol=1e-2)
        for i in range(len(dl)):
            dl.mark(Marker.END_OF_BATCH)
        dl.mark(Marker.END_OF_EPOCH)
        for i in range(len(dl)):
            dl.mark(Marker.END_OF_BATCH)
        dl.mark(Marker.END_OF_EPOCH)
    with ddl_amd.start(n_producers=1) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(ImageWindowProducer(16, (20, 20, 3), "uint8", refill="none"), 4, conn, 1,
                                           env=env,
                                           output=ddl_amd.OutputSpec(normalize={"mean": mean, "std": std,
                                                                     "layout": "hwc"}))
        (x,) = dl[1]
        _, win = dl.arys[0][0]
        ref = ((win[4:8].float() / 255 - torch.tensor(mean)) / torch.tensor(std)).permute(0, 3, 1, 2)
        assert x.shape == (4, 3, 20, 20)
        torch.testing.assert_close(x.float().cpu(), ref, rtol=1e-2, atol=1e-2)
        for i in range(len(dl)):
            dl.mark(Marker.END_OF_BATCH)
        dl.mark(Marker.END_OF_EPOCH)


def test_gpu_resume_mid_window_is_exact():
    def run(n_batches, resume=None):
        rows, sd = [], None
        with ddl_amd.start(n_producers=3) as (env, conn):
            dl = ddl_amd.DistributedDataLoader(IdProducer(64, 8), 16, conn, 3, env=env, auto_mark=True,
                                               resume_state=resume, output=ddl_amd.OutputSpec(copy_batches=True),
                                               order=ddl_amd.OrderSpec(shuffle="device", seed=5))
            assert dl.device.type == "cuda"
            done = 0
            while dl.epoch < 3 and done < n_batches:
                for b in dl:
                    rows.append(torch.cat(b, 1).cpu())
                    done += 1
                    if done == n_batches:
                        sd = dl.state_dict()
                        break
            dl.close()
        return rows, sd

    head, sd = run(7)
    assert sd["epoch"] == 1 and sd["batch"] == 3
    tail, _ = run(10 ** 9, resume=sd)
    full, _ = run(10 ** 9)
    assert len(head) + len(tail) == len(full) == 12
    for a, b in zip(head + tail, full):
        assert torch.equal(a, b)


@pytest.mark.parametrize("fault,exc", [("1:1:exit", "PeerDeathError"), ("0:1:raise", "PeerDeathError"),
                                       ("0:1:hang", "DDLTimeoutError")])
def test_gpu_native_stager_surfaces_producer_faults(monkeypatch, fault, exc):
    """The native stager thread reports a dead / failing / hung producer to the consumer as a typed error."""
    from ddl_amd import exceptions

    monkeypatch.setenv("DDL_FAULT_PRODUCER", fault)
    with pytest.raises(getattr(exceptions, exc)):
        with ddl_amd.start(n_producers=2, timeout_s=4) as (env, conn):
            dl = ddl_amd.DistributedDataLoader(IdProducer(8, 4), 4, conn, 10, env=env,
                                               order=ddl_amd.OrderSpec(shuffle="device"))
            assert dl._stager is not None
            for _ in range(10):
                for _b in dl:
                    dl.mark(Marker.END_OF_BATCH)
                dl.mark(Marker.END_OF_EPOCH)


def test_gpu_augment_random_resized_crop_in_loader():
    from ddl_amd.models.producers import ImageWindowProducer

    mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]

    def run():
        outs = []
        with ddl_amd.start(n_producers=2) as (env, conn):
            dl = ddl_amd.DistributedDataLoader(ImageWindowProducer(32, (3, 64, 80), "uint8", refill="none"), 8, conn,
                                               2, env=env,
                                               output=ddl_amd.OutputSpec(normalize={"mean": mean, "std": std},
                                                                         copy_batches=True, augment={"size": (32, 32),
                                                                         "scale": (0.2, 1.0), "flip_p": 0.5}),
                                               order=ddl_amd.OrderSpec(shuffle="device", seed=3))
            for _ in range(2):
                for (x,) in dl:
                    assert x.shape == (8, 3, 32, 32) and x.dtype == torch.bfloat16 and x.is_cuda
                    outs.append(x.float().cpu())
                    dl.mark(Marker.END_OF_BATCH)
                dl.mark(Marker.END_OF_EPOCH)
        return outs

    a, b = run(), run()
    assert len(a) == 8
    for x, y in zip(a, b):
        assert torch.equal(x, y)  # deterministic for a seed
    lo, hi = (0 - max(mean)) / min(std), (1 - min(mean)) / min(std)
    assert all(float(x.min()) >= lo - 0.05 and float(x.max()) <= hi + 0.05 for x in a)
    assert not torch.equal(a[0], a[4])  # epoch 2 revisits window 0 with new crops


def test_gpu_exception_unwinds_cleanly_with_native_stager():
    """A user exception mid-epoch (loader never closed): leaving start() stops the native stager
    before the arena is unpinned, and does not hang behind a slow producer."""
    import time

    t0 = time.monotonic()
    with pytest.raises(KeyError):
        with ddl_amd.start(n_producers=2) as (env, conn):
            dl = ddl_amd.DistributedDataLoader(IdProducer(64, 8, delay_s=2.0), 16, conn, 5, env=env,
                                               staging=ddl_amd.StagingSpec(n_slots=2, prefetch_depth=2),
                                               order=ddl_amd.OrderSpec(shuffle="device"))
            next(iter(dl))
            raise KeyError("user error")
    assert time.monotonic() - t0 < 30
    assert dl._stager._closed


def test_gpu_resident_augment_matches_direct_crop():
    """ResidentGlobalLoader(augment=...) crops every epoch's global order out of the HBM shard,
    keyed by (seed, epoch, sample id): identical to cropping the dataset directly."""
    from ddl_amd import ops
    from ddl_amd.batching import _mix
    from ddl_amd.models import SharedArraySource
    from ddl_amd.resident import ResidentGlobalLoader

    n, gb = 96, 16
    data = (torch.rand((n, 3, 40, 52)) * 255).to(torch.uint8)
    src = SharedArraySource.create(f"ddl_amd_resaug_{np.random.randint(1 << 30)}", data)
    norm = {"mean": [0.485, 0.456, 0.406], "std": [0.229, 0.224, 0.225]}
    try:
        with ddl_amd.start(n_producers=0) as (env, _):
            dl = ResidentGlobalLoader(src, gb, env, seed=4, n_epochs=2, out_dtype=torch.bfloat16, normalize=norm,
                                      augment={"size": (32, 32), "flip_p": 0.5})
            full = data.cuda()
            for e in range(2):
                perm = dl.order.perm(e)
                for g, b in enumerate(dl):
                    assert b.shape == (gb, 3, 32, 32) and b.dtype == torch.bfloat16
                    ref = ops.random_resized_crop(full, perm=perm, base=g * gb, n_rows=gb, size=(32, 32),
                                                  seed=_mix(4, e), **norm)
                    assert torch.equal(b, ref), (e, g)
            dl.close()
    finally:
        src.close()


def _collect(native, make, epochs=4, partial=None, **kw):
    """Batches of `epochs` epochs (optionally stopping epoch e after `partial[e]` batches), as CPU tensors."""
    out = []
    with ddl_amd.start(n_producers=3) as (env, conn):
        prod, bs = make()
        dl = ddl_amd.DistributedDataLoader(prod, bs, conn, epochs, env=env,
                                           **from_flat(dict(kw, native_dispatch=native)))
        for e in range(epochs):
            for i in range(len(dl)):
                if partial and i >= partial.get(e, 10 ** 9):
                    break
                b = dl[i]
                out.append(torch.cat([t.reshape(t.shape[0], -1).float() for t in b], 1).cpu())
                dl.mark(Marker.END_OF_BATCH)
            dl.mark(Marker.END_OF_EPOCH)
        st = dl.stats()
    return out, st


@pytest.mark.parametrize("case", ["split_i32", "gather_cast_bf16", "images_u8_norm", "images_bf16_noshuffle_copy",
                                  "images_u8_hwc_norm", "images_u8_augment"])
def test_native_dispatch_matches_python_path(case):
    """The native batch engine (csrc/kernels/engine.cpp) delivers bit-identical batches to the Python
    dispatch path -- same Feistel order per window visit, same kernels -- including partial epochs
    (windows skipped unread) and lookahead across window boundaries."""
    from ddl_amd.models.producers import ImageWindowProducer

    kw = dict(shuffle="device", seed=5)
    if case == "split_i32":
        make, kw = (lambda: (IdProducer(64, 8), 16)), dict(kw, contiguous=True)
    elif case == "gather_cast_bf16":
        make, kw = (lambda: (IdProducer(48, 2, dtype="float32"), 8)), dict(kw, out_dtype=torch.bfloat16)
    elif case == "images_u8_norm":
        make = lambda: (ImageWindowProducer(32, (3, 16, 16), "uint8", seed=3), 8)  # noqa: E731
        kw = dict(kw, out_dtype=torch.bfloat16, normalize={"mean": [0.5, 0.4, 0.3], "std": [0.2, 0.25, 0.3]})
    elif case == "images_u8_augment":  # RandomResizedCrop + flip + normalise on the device (engine kind 4)
        make = lambda: (ImageWindowProducer(32, (3, 20, 24), "uint8", seed=3), 8)  # noqa: E731
        kw = dict(kw, out_dtype=torch.bfloat16, normalize={"mean": [0.5, 0.4, 0.3], "std": [0.2, 0.25, 0.3]},
                  augment={"size": (16, 16), "scale": (0.3, 1.0), "flip_p": 0.5})
    elif case == "images_u8_hwc_norm":  # decoded-JPEG layout: HWC uint8 -> normalised CHW bf16 (engine kind 3)
        make = lambda: (ImageWindowProducer(32, (16, 16, 3), "uint8", seed=3), 8)  # noqa: E731
        kw = dict(kw, out_dtype=torch.bfloat16,
                  normalize={"mean": [0.5, 0.4, 0.3], "std": [0.2, 0.25, 0.3], "layout": "hwc"})
    else:
        make = lambda: (ImageWindowProducer(32, (3, 16, 16), "bfloat16", seed=3), 8)  # noqa: E731
        kw = dict(shuffle="none", copy_batches=True)
    partial = {1: 2, 2: 0}
    ref, st_ref = _collect(False, make, partial=partial, **kw)
    assert st_ref.get("native_dispatch") is None
    for mode in ("inline", "lookahead", "window"):
        nat, st = _collect(mode, make, partial=partial, **kw)
        # whole-window launches need contiguous slots: a gather whose batch is not a multiple of 256 bytes
        # (gather_cast_bf16: 32 B) falls back to inline
        # (augment: one launch per batch, never whole-window)
        expect = "inline" if (mode == "window" and case in ("gather_cast_bf16", "images_u8_augment")) else mode
        assert st["native_dispatch"]["batches"] == len(nat) and st["native_dispatch"]["mode"] == expect
        assert len(nat) == len(ref) > 0
        for a, b in zip(nat, ref):
            assert torch.equal(a, b)


def test_native_dispatch_held_batches_stay_valid():
    """Engine output slots are never reused: batches kept across many later batches keep their values."""
    from ddl_amd.models.producers import ImageWindowProducer

    with ddl_amd.start(n_producers=3) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(ImageWindowProducer(32, (3, 16, 16), "bfloat16", seed=3), 8, conn, 30,
                                           env=env, order=ddl_amd.OrderSpec(shuffle="device", seed=2))
        held, snap = [], []
        for e in range(30):
            for i in range(len(dl)):
                (x,) = dl[i]
                if e % 7 == 0:
                    held.append(x)
                    snap.append(x.cpu().clone())
                dl.mark(Marker.END_OF_BATCH)
            dl.mark(Marker.END_OF_EPOCH)
        torch.cuda.synchronize()
        assert dl.stats()["native_dispatch"]["batches"] == 30 * 4
    for x, s in zip(held, snap):
        assert torch.equal(x.cpu(), s)


def test_window_dispatch_batches_on_other_streams():
    """Whole-window mode builds a window's batches at its first get on that stream; a later batch of the
    window consumed on another stream is ordered behind that launch (event + wait), values unchanged."""
    make = lambda: (IdProducer(64, 8), 16)  # noqa: E731
    kw = dict(shuffle="device", seed=5, contiguous=True)
    ref, _ = _collect(False, make, epochs=2, **kw)
    side = [torch.cuda.Stream() for _ in range(2)]
    out = []
    with ddl_amd.start(n_producers=3) as (env, conn):
        prod, bs = make()
        dl = ddl_amd.DistributedDataLoader(prod, bs, conn, 2, env=env,
                                           **from_flat(dict(kw, native_dispatch="window")))
        for e in range(2):
            for i in range(len(dl)):
                with torch.cuda.stream(side[i % 2]):
                    b = dl[i]
                    out.append(torch.cat([t.reshape(t.shape[0], -1).float() for t in b], 1).cpu())
                dl.mark(Marker.END_OF_BATCH)
            dl.mark(Marker.END_OF_EPOCH)
        assert dl.stats()["native_dispatch"]["mode"] == "window"
    assert len(out) == len(ref) > 0
    for a, b in zip(out, ref):
        assert torch.equal(a, b)


def test_inline_dispatch_window_read_on_two_streams_is_not_overwritten():
    """Inline mode: the batches of one window are launched on two streams; the window's FIRST batch goes
    to a stream held back by a long GEMM chain, the later ones to the default stream. The window's ring
    buffer goes back to the stager (depth 1: the next copy lands in the SAME buffer) only behind BOTH
    streams' reads, so the delayed batch still sees its own window."""
    make = lambda: (IdProducer(64, 8), 16)  # noqa: E731
    kw = dict(shuffle="device", seed=3, contiguous=True, prefetch_depth=1)
    ref, _ = _collect(False, make, epochs=3, **kw)
    slow = torch.cuda.Stream()
    a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    out = []
    with ddl_amd.start(n_producers=3) as (env, conn):
        prod, bs = make()
        dl = ddl_amd.DistributedDataLoader(prod, bs, conn, 3, env=env,
                                           **from_flat(dict(kw, native_dispatch="inline")))
        for e in range(3):
            held = []
            for i in range(len(dl)):
                if i == 0:  # the window's first batch, on a stream busy for tens of ms
                    with torch.cuda.stream(slow):
                        for _ in range(60):
                            a = a @ a * 1e-3
                        held.append(dl[i])
                else:
                    held.append(dl[i])
                dl.mark(Marker.END_OF_BATCH)
            dl.mark(Marker.END_OF_EPOCH)
            torch.cuda.synchronize()
            out += [torch.cat([t.reshape(t.shape[0], -1).float() for t in b], 1).cpu() for b in held]
        assert dl.stats()["native_dispatch"]["mode"] == "inline"
    assert len(out) == len(ref) > 0
    for x, y in zip(out, ref):
        assert torch.equal(x, y)


def test_stager_counts_the_copies_of_a_time_window():
    """copies_between(t0, t1): the H2D copies enqueued inside [t0, t1] and complete -- what bench.py counts
    as the timed region's own H2D work. Over the whole run it is every copy; over an empty window, none."""
    from ddl_amd import _native

    rt = _native.runtime()
    with ddl_amd.start(n_producers=3) as (env, conn):
        t0 = rt.now_ns()
        dl = ddl_amd.DistributedDataLoader(IdProducer(64, 8), 16, conn, 4, env=env,
                                           output=ddl_amd.OutputSpec(copy_batches=True),
                                           order=ddl_amd.OrderSpec(shuffle="device", seed=2))
        st = dl._stager
        for e in range(4):  # every window of the run: nothing is left to stage afterwards
            for i in range(len(dl)):
                dl[i]
                dl.mark(Marker.END_OF_BATCH)
            if e < 3:
                dl.mark(Marker.END_OF_EPOCH)
        torch.cuda.synchronize()
        t1 = rt.now_ns()
        n, b, complete = st._native.copies_between(t0, t1)
        assert complete and n == st.windows_staged == 4 and b == st.bytes_h2d == n * 64 * 8 * 4
        assert st._native.copies_between(t1 + 1, t1 + 2) == (0, 0, True)
        dl.close()


@pytest.mark.parametrize("anchor_every", [None, 3])
def test_stager_bytes_in_interval_is_pro_rata_and_additive(anchor_every):
    """bytes_in_interval(e0, e1): the H2D bytes that crossed PCIe between two timing events, from the
    device times of every copy (bench.py's landed count). An interval around the whole run holds every byte;
    splitting it at an event in the middle splits the bytes exactly (pro rata per copy, nothing lost or
    counted twice); an interval after the run holds none. With the device clock re-anchored every 3 retires
    (instead of every 4096) the same holds across the re-anchors."""
    from ddl_amd.models.producers import ImageWindowProducer

    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    with ddl_amd.start(n_producers=2) as (env, conn):
        e0 = ev()
        e0.record()
        dl = ddl_amd.DistributedDataLoader(ImageWindowProducer(64, (3, 64, 64), "bfloat16", refill="stamp"), 32, conn,
                                           6, env=env, device=torch.device("cuda"),
                                           output=ddl_amd.OutputSpec(dtype=torch.bfloat16),
                                           staging=ddl_amd.StagingSpec(prefetch_depth=2, copy_timing=True),
                                           order=ddl_amd.OrderSpec(shuffle="device"))
        st = dl._stager
        assert st.copy_timing
        if anchor_every:
            st._native.set_anchor_every(anchor_every)
        n_batches = 0
        em = None
        for e in range(6):
            for i in range(len(dl)):
                dl[i]
                dl.mark(Marker.END_OF_BATCH)
                n_batches += 1
                if n_batches == 5:
                    em = ev()
                    em.record()
            if e < 5:
                dl.mark(Marker.END_OF_EPOCH)
        torch.cuda.synchronize()
        e1 = ev()
        e1.record()
        e1.synchronize()
        whole = st.bytes_in_interval(e0, e1)
        first, second = st.bytes_in_interval(e0, em), st.bytes_in_interval(em, e1)
        assert whole["ok"] and first["ok"] and second["ok"]
        total = st.bytes_h2d
        assert total == st.windows_staged * 64 * 3 * 64 * 64 * 2 > 0
        assert abs(whole["bytes"] - total) <= 1e-6 * total and whole["copies"] == st.windows_staged
        assert 0 < first["bytes"] < total and abs(first["bytes"] + second["bytes"] - total) <= 1e-6 * total
        assert abs(first["windows"] + second["windows"] - st.windows_staged) < 1e-6
        e2, e3 = ev(), ev()
        e2.record()
        e3.record()
        after = st.bytes_in_interval(e2, e3)
        assert after["ok"] and after["bytes"] == 0.0 and after["copies"] == 0
        if anchor_every:
            assert st._native.reanchors >= 2
        dl.close()


def test_untimed_direct_copies_make_the_interval_unusable():
    """Direct-DMA copy times come from a process-wide ROCr switch that is off unless a loader asks for it
    (copy_timing): without it an interval that the copies overlap reports ok=False (untimed), never a
    silent zero; after the run, an interval no copy overlaps is fine."""
    from ddl_amd.models.producers import ImageWindowProducer

    ev = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
    with ddl_amd.start(n_producers=2) as (env, conn):
        e0 = ev()
        e0.record()
        dl = ddl_amd.DistributedDataLoader(ImageWindowProducer(64, (3, 32, 32), "bfloat16", refill="stamp"), 32, conn,
                                           3, env=env, device=torch.device("cuda"),
                                           output=ddl_amd.OutputSpec(dtype=torch.bfloat16),
                                           staging=ddl_amd.StagingSpec(prefetch_depth=2),
                                           order=ddl_amd.OrderSpec(shuffle="device"))
        st = dl._stager
        if not st.direct_dma:
            pytest.skip(f"no direct DMA here: {st.stats()['direct_dma_reason']}")
        assert not st.copy_timing
        for e in range(3):
            for i in range(len(dl)):
                dl[i]
                dl.mark(Marker.END_OF_BATCH)
            if e < 2:
                dl.mark(Marker.END_OF_EPOCH)
        torch.cuda.synchronize()
        e1 = ev()
        e1.record()
        e1.synchronize()
        r = st.bytes_in_interval(e0, e1)
        assert not r["ok"] and r["untimed"]
        st.settle()  # the retire thread has seen every copy land (an untimed copy's end is when it saw it)
        e2, e3 = ev(), ev()
        e2.record()
        e3.record()
        assert st.bytes_in_interval(e2, e3)["ok"]
        dl.close()


@pytest.mark.parametrize("mode", ["inline", "lookahead", "window"])
def test_native_dispatch_refetch_after_last_batch(mode):
    """Early hand-back (a window's ring buffer goes back to the stager when its LAST batch is launched)
    must not let a later fetch read a buffer that is being refilled: re-fetching a batch already fetched
    in the window returns the same batch (checksum unchanged, even after the next windows were staged
    over the buffer), and fetching a never-fetched batch after the last one raises DDLError in the
    per-batch modes (the whole-window mode built every batch at the first get)."""
    from ddl_amd import ops
    from ddl_amd.exceptions import DDLError
    from ddl_amd.models.producers import ImageWindowProducer

    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(ImageWindowProducer(32, (3, 16, 16), "bfloat16", seed=3), 8, conn, 4,
                                           env=env,
                                           staging=ddl_amd.StagingSpec(native_dispatch=mode, prefetch_depth=2),
                                           order=ddl_amd.OrderSpec(shuffle="device", seed=2))
        assert len(dl) == 4
        first = [ops.checksum(dl[i][0]).item() for i in range(4)]  # batch 3 is the last: window handed back
        torch.cuda.synchronize()
        import time

        time.sleep(0.5)  # the stager is free to refill the buffer with a later window now
        again = ops.checksum(dl[2][0]).item()
        assert again == first[2]
        for i in range(4):
            dl.mark(Marker.END_OF_BATCH)
        dl.mark(Marker.END_OF_EPOCH)
        # epoch 1: skip batch 1, fetch the last one, then the skipped one
        dl[0], dl[3]
        if mode == "window":
            dl[1]  # built with the window at its first get
        else:
            with pytest.raises(DDLError, match="out of order"):
                dl[1]
        dl.close()
