"""Token family (BASELINE config 4): ragged windows, pad / pack collate, exactly-once sequences."""

import numpy as np
import pytest
import torch

import ddl_amd
from ddl_amd.specs import from_flat
from ddl_amd import ops
from ddl_amd.models.tokens import SharedTokenSource, TokenBatchProducer, expected_tokens
from ddl_amd.permutation import EpochOrder


@pytest.fixture
def corpus():
    src = SharedTokenSource.synthetic(f"ddl_amd_tok_{np.random.randint(1 << 30)}", 200, 5, 300, seed=3)
    yield src
    src.close()


@pytest.fixture(params=["int32", "uint16"])
def wire_corpus(request):
    """The corpus with int32 tokens, and with uint16 tokens (2 B per token on the wire, widened on the
    device); vocab 65536 so the top ids (sign bit of an int16) are exercised."""
    src = SharedTokenSource.synthetic(f"ddl_amd_tok_{np.random.randint(1 << 30)}", 200, 5, 300, seed=3,
                                      vocab=65536, token_dtype=request.param)
    assert src.token_bytes == (2 if request.param == "uint16" else 4)
    yield src
    src.close()


def _check_pad(batch, source, idx, seq_len):
    ids, mask, pos = batch["input_ids"].cpu(), batch["attention_mask"].cpu(), batch["position_ids"].cpu()
    for r, seq in enumerate(expected_tokens(source, idx)):
        n = min(len(seq), seq_len)
        assert torch.equal(ids[r, :n], torch.from_numpy(seq[:n]))
        assert mask[r, :n].all() and not mask[r, n:].any()
        assert torch.equal(pos[r, :n], torch.arange(n))


@pytest.mark.parametrize("k", [1, 5])
@pytest.mark.parametrize("mode", ["pad", "pack"])
def test_token_batches_cpu(wire_corpus, mode, k, monkeypatch):
    """k=5 asks for 5 batches per window: 12 batches per epoch -> 4 (the largest divisor <= 5)."""
    monkeypatch.setenv("DDL_DEVICE", "cpu")  # host collate path, even on a GPU box
    seq_len, gb = 256, 16
    order = EpochOrder(wire_corpus.n, gb, 4)
    with ddl_amd.start(n_producers=2) as (env, conn):
        prod = TokenBatchProducer(wire_corpus, gb, seq_len, mode, batches_per_window=k)
        dl = ddl_amd.DistributedDataLoader(prod, gb, conn, 2, env=env, auto_mark=True,
                                           output=ddl_amd.OutputSpec(collate="tokens"),
                                           order=ddl_amd.OrderSpec(mode="indexed", seed=4))
        assert dl.batches_per_window == [1 if k == 1 else 4] * 2
        assert len(dl) == order.batches_per_epoch
        for e in range(2):
            for g, batch in enumerate(dl):
                idx = order.indices(e, g)
                if mode == "pad":
                    assert batch["input_ids"].shape == (gb, seq_len)
                    _check_pad(batch, wire_corpus, idx, seq_len)
                else:
                    m = batch["attention_mask"].bool()
                    flat = batch["input_ids"][m]
                    ref = np.concatenate(expected_tokens(wire_corpus, idx))
                    assert np.array_equal(flat.numpy(), ref)  # every token exactly once, in order
                    assert batch["input_ids"].shape[1] == seq_len
                    cu = batch["cu_seqlens"]
                    assert int(cu[-1]) == len(ref) == batch["n_tokens"] == int(batch["attention_mask"].sum())


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 4])
@pytest.mark.parametrize("mode", ["pad", "pack"])
def test_token_batches_gpu(wire_corpus, mode, k):
    seq_len, gb = 256, 16
    order = EpochOrder(wire_corpus.n, gb, 4)
    with ddl_amd.start(n_producers=2) as (env, conn):
        prod = TokenBatchProducer(wire_corpus, gb, seq_len, mode, batches_per_window=k)
        dl = ddl_amd.DistributedDataLoader(prod, gb, conn, 1, env=env, auto_mark=True,
                                           output=ddl_amd.OutputSpec(collate="tokens"),
                                           order=ddl_amd.OrderSpec(mode="indexed", seed=4))
        held = None
        for g, batch in enumerate(dl):
            assert batch["input_ids"].is_cuda
            idx = order.indices(0, g)
            if mode == "pad":
                _check_pad(batch, wire_corpus, idx, seq_len)
            else:
                m = batch["attention_mask"].bool().cpu()
                flat = batch["input_ids"].cpu()[m]
                assert np.array_equal(flat.numpy(), np.concatenate(expected_tokens(wire_corpus, idx)))
                if held is None:
                    lens = [len(x) for x in expected_tokens(wire_corpus, idx)]
                    held = (batch["cu_seqlens"], ops.pack_plan(np.concatenate([[0], np.cumsum(lens)]), seq_len)[2])
        if held is not None:  # cu_seqlens is owned: still intact after the staging buffers were reused
            assert held[0].dtype == torch.int32
            assert np.array_equal(held[0].cpu().numpy(), held[1])


@pytest.mark.parametrize("seq_len", [4096, 100, 7])
def test_native_pack_plan_matches_reference(seq_len):
    from ddl_amd import ops

    rng = np.random.default_rng(seq_len)
    for n in (0, 1, 5, 64):
        lens = rng.integers(0, 3 * seq_len, size=n)
        offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        got = ops.pack_plan(offs, seq_len)
        ref = ops.ref_pack_plan(offs, seq_len)
        for a, b in zip(got, ref):
            assert np.array_equal(a, b), (n, a, b)


def _doubling_plan(offs, S):
    """numpy mirror of the device planner (tokens.hip pack_plan_kernel): segments by a scan, the greedy jump
    by a search over segment starts, the rows as the orbit of segment 0 by pointer doubling."""
    lens = np.diff(offs)
    c = np.where(lens > 0, -(-lens // S), 0)
    first = np.concatenate([[0], np.cumsum(c)])[:-1]
    n_seg = int(c.sum())
    so = np.empty(n_seg + 1, np.int64)
    for i in np.nonzero(c)[0]:
        so[first[i]:first[i] + c[i]] = offs[i] + S * np.arange(c[i])
    so[n_seg] = offs[-1] if n_seg else 0
    J = np.append(np.searchsorted(so, so[:n_seg] + S, side="right") - 1, n_seg)
    P = np.array([0])
    while P[-1] < n_seg:  # P[len + i] = jump^len(P[i]); jump^len -> jump^(2 len)
        P = np.concatenate([P, J[P]])
        J = J[J]
    P = P[: np.argmax(P == n_seg) + 1]
    return so[P[:-1]], so[P[1:]], so


@pytest.mark.parametrize("seq_len", [4096, 100, 7, 1])
def test_pointer_doubling_plan_equals_the_sequential_plan(seq_len):
    """The device planner's algorithm (checked here in numpy; the kernel itself in test_kernels_gpu.py)."""
    rng = np.random.default_rng(11 + seq_len)
    for n in (0, 1, 2, 5, 64, 333):
        for hi in (2, seq_len + 1, 3 * seq_len):
            lens = rng.integers(0, hi, size=n)
            offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
            got = _doubling_plan(offs, seq_len)
            ref = ops.ref_pack_plan(offs, seq_len)
            for a, b in zip(got, ref):
                assert np.array_equal(a, b), (n, hi, a, b)
            n_segs, n_rows = ops.pack_capacity(n, int(offs[-1]), seq_len)
            assert len(ref[0]) <= n_rows and len(ref[2]) - 1 <= n_segs


def test_sixteen_bit_tokens_widen_in_the_host_references():
    ids = np.array([0, 1, 32767, 32768, 65535, 7], np.uint16)
    t16 = torch.from_numpy(ids.view(np.int16))
    offs = torch.tensor([0, 2, 6], dtype=torch.int64)
    out, mask, _ = ops.ref_pad_tokens(t16, offs, 5)
    assert out[1, :4].tolist() == [32767, 32768, 65535, 7]
    rs, re_, so = ops.ref_pack_plan(offs.numpy(), 8)
    packed = ops.ref_pack_tokens(t16, rs, re_, so, 8)[0]
    assert packed[0, :6].tolist() == ids.astype(np.int64).tolist()


def test_token_source_dtype_choice():
    ok = SharedTokenSource.create(f"ddl_amd_tokdt_{np.random.randint(1 << 30)}", np.array([1, 65535]),
                                  np.array([0, 2]), "auto")
    wide = SharedTokenSource.create(f"ddl_amd_tokdt_{np.random.randint(1 << 30)}", np.array([1, 70000]),
                                    np.array([0, 2]), "auto")
    try:
        assert ok.token_bytes == 2 and wide.token_bytes == 4
        assert [x.tolist() for x in expected_tokens(ok, [0])] == [[1, 65535]]
        with pytest.raises(ValueError):
            SharedTokenSource.create("ddl_amd_never", np.array([70000]), np.array([0, 1]), "uint16")
    finally:
        ok.close()
        wide.close()


def test_pack_tokens_device_host_reference_shapes():
    """CPU form of pack_tokens_device: fixed capacity rows, counts, padding rows after the plan's."""
    offs = np.array([0, 10, 10, 60, 61, 100], np.int64)
    toks = torch.arange(100, dtype=torch.int32)
    r = ops.pack_tokens_device(toks, torch.from_numpy(offs), 16, pad_id=9)
    rs, re_, so = ops.ref_pack_plan(offs, 16)
    assert r["counts"].tolist() == [len(rs), len(so) - 1]
    assert r["input_ids"].shape == (ops.pack_capacity(5, 100, 16)[1], 16)
    assert torch.equal(r["input_ids"][r["attention_mask"].bool()], toks)
    assert bool((r["input_ids"][len(rs):] == 9).all()) and bool((r["segment_ids"][len(rs):] == -1).all())


def test_native_gather_ragged():
    from ddl_amd import _native

    rng = np.random.default_rng(0)
    lens = rng.integers(0, 5000, size=300)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    toks = rng.integers(0, 1 << 30, size=int(offs[-1]), dtype=np.int32)
    idx = rng.permutation(300)[:77]
    cap = int(lens[idx].sum())
    dst = np.zeros(cap, np.int32)
    dofs = np.zeros(78, np.int64)
    rt = _native.runtime()
    n = rt.gather_ragged(dst.ctypes.data, dofs.ctypes.data, toks.ctypes.data, offs.ctypes.data, 300, idx, 4, cap, 3)
    assert n == cap
    ref = np.concatenate([toks[offs[i]:offs[i + 1]] for i in idx])
    assert np.array_equal(dst, ref) and np.array_equal(dofs[1:], np.cumsum(lens[idx]))
    with pytest.raises(ValueError):  # std::length_error -> capacity
        rt.gather_ragged(dst.ctypes.data, dofs.ctypes.data, toks.ctypes.data, offs.ctypes.data, 300, idx, 4, cap - 1, 3)
    with pytest.raises(IndexError):
        rt.gather_ragged(dst.ctypes.data, dofs.ctypes.data, toks.ctypes.data, offs.ctypes.data, 300, [300], 4, cap, 1)


def test_token_train_step_on_collated_pack_batch():
    """The config-4 idle-% consumer trains on a collated pack batch; padding is ignored in the loss."""
    from ddl_amd.models.trainstep import TokenTrainStep

    S = 64
    toks = torch.arange(1, 151, dtype=torch.int32)
    ids, mask, pos, seg = ops.ref_pack_tokens(toks, np.array([0, 64, 128]), np.array([64, 128, 150]),
                                              np.array([0, 40, 100, 150]), S, 0)
    step = TokenTrainStep("cpu", seq_len=S, dim=16, depth=1, n_out=32, dtype=torch.float32, vocab=200)
    batch = {"input_ids": ids, "attention_mask": mask, "position_ids": pos}
    l0 = float(step(batch))
    for _ in range(20):
        l1 = float(step(batch))
    assert np.isfinite(l0) and l1 < l0  # it learns: the step really runs fwd + bwd + update


def test_ffd_order_rows_equal_bins_and_beat_in_order():
    from ddl_amd.models.tokens import ffd_order

    rng = np.random.default_rng(3)
    tot_ffd = tot_in = 0
    for _ in range(100):
        S = int(rng.choice([7, 100, 4096]))
        lens = rng.integers(1, 2 * S, size=int(rng.integers(1, 70)))
        order, n_rows = ffd_order(lens, S)
        assert sorted(order.tolist()) == list(range(len(lens)))
        offs = np.concatenate([[0], np.cumsum(lens[order])])
        assert len(ops.pack_plan(offs, S)[0]) == n_rows  # in-order packing of that order breaks at bin ends
        tot_ffd += n_rows
        tot_in += len(ops.pack_plan(np.concatenate([[0], np.cumsum(lens)]), S)[0])
    assert tot_ffd < tot_in  # fewer rows overall (FFD can lose on a rare adversarial batch)


def test_ffd_order_native_matches_numpy_reference():
    """The native C++ ffd_order (arena.cpp) equals its NumPy reference, empty and exact-multiple lengths included."""
    from ddl_amd.models.tokens import ffd_order, ffd_order_py

    rng = np.random.default_rng(11)
    for _ in range(200):
        S = int(rng.choice([1, 5, 64, 4096]))
        lens = rng.integers(0, 3 * S + 1, size=int(rng.integers(0, 90)))
        if len(lens) and rng.random() < 0.3:
            lens[rng.integers(0, len(lens))] = 2 * S  # only full chunks
        o_nat, r_nat = ffd_order(lens, S)
        o_py, r_py = ffd_order_py(lens, S)
        assert r_nat == r_py and o_nat.tolist() == o_py.tolist()
        assert sorted(o_nat.tolist()) == list(range(len(lens)))
    with pytest.raises(ValueError):
        ffd_order(np.array([3]), 0)


def test_token_batches_ffd_pack_order(corpus, monkeypatch):
    """pack_order="ffd": the same sequences per batch, in first-fit-decreasing order when that packs into
    fewer rows than the batch's own order (else the batch's order) -- so never more rows, batch by batch."""
    from ddl_amd.models.tokens import ffd_order, in_order_rows

    monkeypatch.setenv("DDL_DEVICE", "cpu")
    seq_len, gb = 256, 16
    order = EpochOrder(corpus.n, gb, 4)
    rows = {}
    for po in ("in_order", "ffd"):
        with ddl_amd.start(n_producers=2) as (env, conn):
            dl = ddl_amd.DistributedDataLoader(TokenBatchProducer(corpus, gb, seq_len, "pack", pack_order=po), gb,
                                               conn, 1, env=env, auto_mark=True,
                                               output=ddl_amd.OutputSpec(collate="tokens"),
                                               order=ddl_amd.OrderSpec(mode="indexed", seed=4))
            rows[po] = 0
            for g, batch in enumerate(dl):
                seqs = expected_tokens(corpus, order.indices(0, g))
                lens = np.array([len(x) for x in seqs])
                n_in = in_order_rows(lens, seq_len)
                if po == "ffd":
                    o, n_ffd = ffd_order(lens, seq_len)
                    if n_ffd < n_in:
                        seqs = [seqs[i] for i in o]
                flat = batch["input_ids"][batch["attention_mask"].bool()].numpy()
                assert np.array_equal(flat, np.concatenate(seqs))  # every token once, in the packing order
                assert batch["input_ids"].shape[0] <= n_in
                rows[po] += batch["input_ids"].shape[0]
    assert rows["ffd"] <= rows["in_order"]


def test_ffd_never_packs_into_more_rows():
    """FFD is a heuristic: S=10, lengths [5,3,2,4,3,3] pack in order into 2 rows, FFD needs 3.
    The producer keeps the batch's own order then."""
    from ddl_amd.models.tokens import ffd_order, ffd_order_py, in_order_rows

    lens = np.array([5, 3, 2, 4, 3, 3])
    assert in_order_rows(lens, 10) == 2 == len(ops.pack_plan(np.concatenate([[0], np.cumsum(lens)]), 10)[0])
    assert ffd_order(lens, 10)[1] == 3 == ffd_order_py(lens, 10)[1]
    from ddl_amd.models.tokens import in_order_rows_py

    rng = np.random.default_rng(5)
    for _ in range(200):  # in_order_rows (native) == its Python reference == the native planner's row count
        S = int(rng.choice([1, 7, 100]))
        ln = rng.integers(0, 3 * S + 1, size=int(rng.integers(0, 40)))
        assert in_order_rows(ln, S) == in_order_rows_py(ln, S) == \
            len(ops.pack_plan(np.concatenate([[0], np.cumsum(ln)]), S)[0])


def test_ffd_requires_pack_mode(corpus):
    with pytest.raises(ValueError, match="pack_order"):
        TokenBatchProducer(corpus, 16, 256, "pad", pack_order="ffd")


def _attention(x, causal=True):
    """softmax(x x^T / sqrt(d)) x for one sequence [L, d] (q = k = v = x), fp32."""
    s = x @ x.T / x.shape[1] ** 0.5
    if causal:
        s = s.masked_fill(torch.triu(torch.ones_like(s, dtype=torch.bool), 1), float("-inf"))
    return torch.softmax(s, dim=-1) @ x


def _varlen_attention(x, cu):
    """Reference varlen attention over a packed stream [T, d]: block-diagonal causal attention
    between cu_seqlens boundaries (the flash-attn varlen semantics, in plain PyTorch)."""
    T = x.shape[0]
    seg = torch.bucketize(torch.arange(T), cu[1:].long(), right=True)
    s = x @ x.T / x.shape[1] ** 0.5
    allowed = (seg[:, None] == seg[None, :]) & ~torch.triu(torch.ones(T, T, dtype=torch.bool), 1)
    return torch.softmax(s.masked_fill(~allowed, float("-inf")), dim=-1) @ x


def test_cu_seqlens_drive_varlen_attention(corpus, monkeypatch):
    """Pack mode: int32 cu_seqlens over input_ids[attention_mask.bool()] drive a varlen attention that
    equals attention computed per segment (seq_len chunks of each sequence) -- over-long sequences
    included (max_len 300 > seq_len 128); max_seqlen is the longest segment."""
    monkeypatch.setenv("DDL_DEVICE", "cpu")
    seq_len, gb = 128, 8
    order = EpochOrder(corpus.n, gb, 4)
    emb = torch.randn(50257, 16, generator=torch.Generator().manual_seed(0))
    with ddl_amd.start(n_producers=1) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(TokenBatchProducer(corpus, gb, seq_len, "pack"), gb, conn, 1, env=env,
                                           auto_mark=True, output=ddl_amd.OutputSpec(collate="tokens"),
                                           order=ddl_amd.OrderSpec(mode="indexed", seed=4))
        for g, batch in enumerate(dl):
            if g == 3:
                break
            cu = batch["cu_seqlens"]
            assert cu.dtype == torch.int32
            stream = batch["input_ids"][batch["attention_mask"].bool()].long()
            segs = [c for s in expected_tokens(corpus, order.indices(0, g))
                    for c in (s[i:i + seq_len] for i in range(0, len(s), seq_len)) if len(c)]
            assert cu.tolist() == np.concatenate([[0], np.cumsum([len(c) for c in segs])]).tolist()
            assert batch["max_seqlen"] == max(len(c) for c in segs)
            got = _varlen_attention(emb[stream], cu)
            want = torch.cat([_attention(emb[torch.from_numpy(c.astype(np.int64))]) for c in segs])
            torch.testing.assert_close(got, want, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("bpw", [1, 4])
@pytest.mark.parametrize("mode", ["pad", "pack"])
def test_token_native_dispatch_matches_python_path(corpus, mode, bpw):
    """Native batch engine (kind 2: pad/pack kernel straight from the staged window) == the Python collate,
    also for k-batch windows (per-sub-batch header + token run from the stager's host copy of the meta)."""
    seq_len, gb = 256, 16

    def run(native):
        out = []
        with ddl_amd.start(n_producers=2) as (env, conn):
            dl = ddl_amd.DistributedDataLoader(TokenBatchProducer(corpus, gb, seq_len, mode, batches_per_window=bpw),
                                               gb, conn, 2, env=env, auto_mark=True,
                                               output=ddl_amd.OutputSpec(collate="tokens"),
                                               staging=ddl_amd.StagingSpec(native_dispatch=native),
                                               order=ddl_amd.OrderSpec(mode="indexed", seed=4))
            for _ in range(2):
                for b in dl:
                    out.append({k: (v.cpu().clone() if isinstance(v, torch.Tensor) else v) for k, v in b.items()})
            st = dl.stats()
        return out, st

    ref, st_ref = run(False)
    assert "native_dispatch" not in st_ref
    for native in ("inline", "lookahead", "window"):
        nat, st = run(native)
        # window: one multi-batch pad/pack launch per window (k > 1); a 1-batch window falls back to inline
        expect = "inline" if (native == "window" and bpw == 1) else native
        assert st["native_dispatch"]["batches"] == len(nat) and st["native_dispatch"]["mode"] == expect
        assert len(nat) == len(ref) > 0
        for a, b in zip(nat, ref):
            assert a.keys() == b.keys()
            for k in a:
                if isinstance(a[k], torch.Tensor):
                    assert a[k].dtype == b[k].dtype and torch.equal(a[k], b[k]), k
                else:
                    assert a[k] == b[k], k


@pytest.mark.parametrize("live", [False, True])
def test_multi_batch_window_resume_mid_window(corpus, live, monkeypatch):
    """Indexed checkpoint of a k-batch-window loader: the cursor counts global batches; resume lands
    mid-window (window 1, sub-batch 2) and continues with exactly the next global batch."""
    monkeypatch.setenv("DDL_DEVICE", "cpu")
    seq_len, gb, k = 256, 16, 4
    order = EpochOrder(corpus.n, gb, 4)

    def make(conn, env, sd=None):
        return ddl_amd.DistributedDataLoader(TokenBatchProducer(corpus, gb, seq_len, "pad", batches_per_window=k), gb,
                                             conn, 2, env=env, auto_mark=True, resume_state=sd,
                                             output=ddl_amd.OutputSpec(collate="tokens"),
                                             order=ddl_amd.OrderSpec(mode="indexed", seed=4))

    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = make(conn, env)
        it = iter(dl)
        for _ in range(6):
            next(it)
        sd = dl.state_dict()
        assert sd["global_batch_cursor"] == 6 and sd["batches_per_window"] == k
        assert sd["batches_per_epoch"] == order.batches_per_epoch
        if live:
            next(it)
            next(it)
            dl.load_state_dict(sd)
            got = [b for _, b in zip(range(3), iter(dl))]
        else:
            dl.close()
    if not live:
        with ddl_amd.start(n_producers=2) as (env, conn):
            dl = make(conn, env, sd)
            got = [b for _, b in zip(range(3), iter(dl))]
            dl.close()
    for j, b in enumerate(got):
        _check_pad(b, corpus, order.indices(0, 6 + j), seq_len)


def _check_fixed_against_exact(fixed, exact, max_rows, seq_len, pad_id=0):
    n = exact["input_ids"].shape[0]
    assert fixed["n_rows"] == n and fixed["input_ids"].shape == (max_rows, seq_len)
    for k in ("input_ids", "attention_mask", "position_ids", "segment_ids"):
        assert fixed[k].dtype == exact[k].dtype and torch.equal(fixed[k][:n].cpu(), exact[k].cpu()), k
    pad = {"input_ids": pad_id, "attention_mask": 0, "position_ids": 0, "segment_ids": -1}
    for k, v in pad.items():
        assert bool((fixed[k][n:].cpu() == v).all()), k
    assert torch.equal(fixed["cu_seqlens"].cpu(), exact["cu_seqlens"].cpu())
    assert fixed["n_tokens"] == exact["n_tokens"] and fixed["max_seqlen"] == exact["max_seqlen"]


def _token_run(corpus, gb, seq_len, k, epochs=1, **kw):
    out = []
    with ddl_amd.start(n_producers=2) as (env, conn):
        dl = ddl_amd.DistributedDataLoader(TokenBatchProducer(corpus, gb, seq_len, "pack", batches_per_window=k), gb,
                                           conn, epochs, env=env, auto_mark=True,
                                           **from_flat(dict(kw, collate="tokens"), mode="indexed", seed=4))
        for _ in range(epochs):
            for b in dl:
                out.append({x: (v.cpu().clone() if isinstance(v, torch.Tensor) else v) for x, v in b.items()})
        st = dl.stats()
        layout = dl.metadata_from_producer[0].extra["token_layout"]
    return out, st, layout


def test_fixed_token_rows_cpu(corpus, monkeypatch):
    """token_rows="fixed": every packed batch has the layout's max rows; the packed rows equal the exact
    batch and the rest are padding (static shapes for graph-captured steps)."""
    monkeypatch.setenv("DDL_DEVICE", "cpu")
    from ddl_amd.models.tokens import TokenWindowLayout

    exact, _, _ = _token_run(corpus, 16, 256, 4)
    fixed, _, lay = _token_run(corpus, 16, 256, 4, token_rows="fixed")
    max_rows = TokenWindowLayout(**lay).max_segments
    assert len(exact) == len(fixed) > 0
    for f, e in zip(fixed, exact):
        _check_fixed_against_exact(f, e, max_rows, 256)


@pytest.mark.gpu
def test_fixed_token_rows_gpu_native_and_python():
    """Fixed-row packed batches from the native engine (inline and whole-window) == the Python collate
    == the exact batches padded."""
    from ddl_amd.models.tokens import TokenWindowLayout

    src = SharedTokenSource.synthetic(f"ddl_amd_tokfix_{np.random.randint(1 << 30)}", 200, 5, 300, seed=3)
    try:
        exact, _, _ = _token_run(src, 16, 256, 4, native_dispatch=False)
        ref, _, lay = _token_run(src, 16, 256, 4, native_dispatch=False, token_rows="fixed")
        max_rows = TokenWindowLayout(**lay).max_segments
        for f, e in zip(ref, exact):
            _check_fixed_against_exact(f, e, max_rows, 256)
        for native in ("inline", "window"):
            nat, st, _ = _token_run(src, 16, 256, 4, native_dispatch=native, token_rows="fixed")
            assert st["native_dispatch"]["mode"] == native and len(nat) == len(ref)
            for a, b in zip(nat, ref):
                assert a.keys() == b.keys()
                for x in a:
                    if isinstance(a[x], torch.Tensor):
                        assert torch.equal(a[x], b[x]), (native, x)
                    else:
                        assert a[x] == b[x], (native, x)
    finally:
        src.close()


def test_view_cache_entries_of_a_dropped_ring_are_forgotten():
    """The collate view cache holds views of staging buffers; closing a stager (live seek / close)
    drops that ring's entries so the cache does not keep its memory alive."""
    from ddl_amd.models import tokens as tk

    lay = tk.TokenWindowLayout(batch=4, seq_len=16, max_len=20, k=2)
    a = torch.zeros(lay.nbytes, dtype=torch.uint8)
    b = torch.zeros(lay.nbytes, dtype=torch.uint8)
    for sub in range(2):
        tk._cached_views(a, lay, sub)
        tk._cached_views(b, lay, sub)
    assert tk.drop_cached_views([a.data_ptr()]) == 2
    assert not any(k[0] == a.data_ptr() for k in tk._VIEW_CACHE)
    assert sum(1 for k in tk._VIEW_CACHE if k[0] == b.data_ptr()) == 2
    tk.drop_cached_views([b.data_ptr()])
