"""Producer-free zero-copy loader: gfx950 gather straight from pinned, device-mapped host memory."""

import numpy as np
import pytest
import torch

from ddl_amd.permutation import EpochOrder
from ddl_amd.zerocopy import ZeroCopyLoader


def _src(n=600, shape=(2,)):
    return torch.stack([torch.arange(n), torch.arange(n) * 3], 1).to(torch.int64)


def test_zerocopy_cpu_order_and_resume():
    src = _src()
    dl = ZeroCopyLoader(src, 40, seed=4, n_epochs=2, device="cpu")
    order = EpochOrder(600, 40, 4)
    out = [torch.cat([b[:, 0] for b in dl]).numpy() for _ in range(2)]
    for e in range(2):
        assert np.array_equal(out[e], order.perm(e).full()[: order.batches_per_epoch * 40])
    dl2 = ZeroCopyLoader(src, 40, seed=4, n_epochs=2, device="cpu")
    it = iter(dl2)
    for _ in range(3):
        next(it)
    sd = dl2.state_dict()
    assert sd["global_batch_cursor"] == 3
    dl3 = ZeroCopyLoader(src, 40, seed=4, n_epochs=2, device="cpu", resume_state=sd)
    rest = torch.cat([b[:, 0] for b in dl3]).numpy()
    assert np.array_equal(rest, order.perm(0).full()[3 * 40: order.batches_per_epoch * 40])


@pytest.mark.gpu
@pytest.mark.parametrize("max_blocks,prep_streams", [(0, 1), (4, 1), (64, 1), (16, 2)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.uint8])
def test_zerocopy_gpu_matches_reference(max_blocks, prep_streams, dtype):
    n, shape = 512, (3, 32, 32)
    src = (torch.rand((n, *shape)) * 255).to(dtype)
    norm = {"mean": [0.5, 0.4, 0.3], "std": [0.2, 0.2, 0.2]} if dtype == torch.uint8 else None
    dl = ZeroCopyLoader(src, 64, seed=1, n_epochs=1, out_dtype=torch.bfloat16, normalize=norm, max_blocks=max_blocks,
                        depth=3, prep_streams=prep_streams)
    order = EpochOrder(n, 64, 1)
    got = torch.cat([b.float().cpu() for b in dl])
    idx = torch.from_numpy(order.perm(0).full()[: order.batches_per_epoch * 64])
    ref = src[idx].float()
    if norm:
        m = torch.tensor(norm["mean"]).view(1, 3, 1, 1)
        s = torch.tensor(norm["std"]).view(1, 3, 1, 1)
        ref = (ref / 255 - m) / s
    torch.testing.assert_close(got, ref.to(torch.bfloat16).float(), rtol=1e-2, atol=2e-2)
    assert dl.stats()["prefault_s"] > 0  # every page of the mapped source was touched once before batch 0
    dl.close()


@pytest.mark.gpu
@pytest.mark.parametrize("handoff", ["host", "device"])
def test_zerocopy_handoff_modes_deliver_the_same_bytes_behind_a_busy_stream(handoff):
    """Host hand-off (the default: the host waits for the gather's event, the consumer's stream gets no barrier)
    and device hand-off deliver the same batches, bitwise -- also when the consumer's stream is busy with a long
    kernel while the gathers run ahead, and the consumer reads each batch right after it is handed over. The rows
    are large enough for the deep-tile PCIe gather, on a grid of 8 workgroups."""
    # 76,800 B rows: the deep-tile host gather (64 KB per workgroup tile) with a partial second tile per row
    n, shape = 512, (3, 128, 100)
    src = (torch.rand((n, *shape)) * 100).to(torch.bfloat16)
    dl = ZeroCopyLoader(src, 64, seed=2, n_epochs=1, depth=3, handoff=handoff, max_blocks=8)
    order = EpochOrder(n, 64, 2)
    idx = torch.from_numpy(order.perm(0).full()[: order.batches_per_epoch * 64]).view(-1, 64)
    outs = []
    for g, b in enumerate(dl):
        if g % 4 == 0:
            torch.cuda._sleep(2_000_000)  # the consumer's stream is busy; later gathers finish first
        outs.append(b.clone())  # read on the consumer's stream, right away
    assert torch.equal(torch.cat(outs).cpu(), src[idx.reshape(-1)])
    st = dl.stats()
    assert st["handoff"] == handoff and (st["host_waits"] == 0 or handoff == "host")
    dl.close()


@pytest.mark.gpu
@pytest.mark.parametrize("prep_streams", [1, 2])
def test_batches_carved_from_blocks_stay_intact(prep_streams):
    """Batches are carved from multi-batch blocks and the consumer's stream is recorded once per block: a batch
    the consumer holds is never overwritten by later gathers, and a dropped block is reused only after the
    consumer's reads -- here the consumer's stream is busy before every read, so the gathers run far ahead."""
    n, shape = 1024, (3, 32, 32)
    src = (torch.rand((n, *shape)) * 100).to(torch.bfloat16)
    dl = ZeroCopyLoader(src, 64, seed=3, n_epochs=3, depth=3, prep_streams=prep_streams)
    dl.block_bytes = 3 * 64 * 3 * 32 * 32 * 2  # 3 batches per block: many blocks, each reused many times
    order = EpochOrder(n, 64, 3)
    outs, held, blocks = [], [], 0
    for e in range(3):
        idx = torch.from_numpy(order.perm(e).full()[: order.batches_per_epoch * 64]).view(-1, 64)
        for g, b in enumerate(dl):
            assert b._base is not None and b._base.numel() == 3 * b.numel()
            blocks += b.data_ptr() == b._base.data_ptr()
            torch.cuda._sleep(300_000)  # the consumer reads late
            outs.append((b.clone(), idx[g]))
            if g % 4 == 0:
                held.append((b, idx[g]))  # kept to the end: its block must never be handed out again
    assert blocks >= len(outs) // 3
    for got, i in outs + held:
        assert torch.equal(got.cpu(), src[i])
    dl.close()


@pytest.mark.gpu
def test_touch_pages_reads_every_page():
    """touch_pages: one 4 B read per page; the per-block xor of the words lands in the sink (the loads are real)."""
    from ddl_amd import _native

    page, n_pages = 4096, 1000
    host = torch.zeros(n_pages * page // 4, dtype=torch.int32).pin_memory()
    host.view(n_pages, page // 4)[:, 0] = torch.arange(1, n_pages + 1, dtype=torch.int32)
    hip = _native.hip()
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    hip.touch_pages(hip.host_device_pointer(host.data_ptr()), host.numel() * 4, page, sink.data_ptr(), 1,
                    torch.cuda.current_stream().cuda_stream)
    want = 0
    for i in range(1, n_pages + 1):
        want ^= i
    assert int(sink.item()) == want
