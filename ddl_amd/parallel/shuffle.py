"""Cross-GPU global shuffle (reference ddl/shuffle.py).

Reference: the k-th producers of all GPUs swap ``fraction x nData`` rows per
window iteration with ``Sendrecv_replace`` -- first half to ``send_to``,
second half to ``recv_from``, partners from a seeded derangement without
2-cycles (reference ddl/shuffle.py:32-108). It never runs: the callback
dispatcher only calls ``callbacks[0]`` (reference ddl/utils.py:22).

Here the exchange really runs, on the consumer side, on the window *after* it
has been staged into HBM, on the prefetch stream, over RCCL/xGMI:

1. a per-window exchange permutation ``Px = Feistel(n, seed', window)`` picks
   the ``n_ex`` rows to trade (``Px(0..n_ex-1)``: a uniformly random subset,
   identical formula on every rank, nothing communicated);
2. the ``gather_rows`` HIP kernel packs them contiguously (Px evaluated
   inline, no index table);
3. ``all_to_all_single`` on the DP process group (RCCL) -- the same group,
   ncclComm and stream as the trainer's DDP all-reduce, so every collective of
   the rank has one device-side order (``parallel/order.py``): an
   8-GPU MI355X node is fully connected by xGMI, and an all-to-all drives all 7
   links of every GPU at once, where the reference's 2-partner exchange
   drives 2 (SURVEY §5 "MI355X-native communication design");
   ``exchange_method="sendrecv_replace"`` keeps the reference's 2-partner
   pattern (grouped ``isend``/``irecv``);
4. ``scatter_rows`` puts the received rows back at the same positions.

Deterministic: partners and rows depend only on (seed, window index).
"""

from __future__ import annotations

import math

import numpy as np
import torch

from .. import ops
from ..ops import _dtypes
from ..permutation import FeistelPermutation
from ..types import DDLEnv
from ..utils.logging import logger
from .order import check_group, issue, loader_group

_EXCHANGE_SALT = 0x5EED_C0DE


def derangement_partners(n: int, rank: int, rng: np.random.Generator, max_tries: int = 1000) -> tuple[int, int]:
    """(send_to, recv_from) of ``rank`` under a random permutation with no fixed
    points and no 2-cycles (reference semantics, ddl/shuffle.py:32-79)."""
    if n == 1:
        return 0, 0
    if n == 2:
        return (1, 1) if rank == 0 else (0, 0)
    idx = np.arange(n)
    for _ in range(max_tries):
        col = rng.permutation(n)
        if np.any(col == idx):
            continue
        if np.any(col[col] == idx):  # 2-cycle: send_to == recv_from for someone
            continue
        send_to = int(col[rank])
        recv_from = int(np.nonzero(col == rank)[0][0])
        return send_to, recv_from
    raise RuntimeError(f"no valid communication pattern after {max_tries} tries")


class GlobalShuffler:
    """Base: owns the loader process group and the row-selection permutation."""

    def __init__(self, env: DDLEnv, fraction: float, n_rows: int, sample_shape: tuple[int, ...], dtype: torch.dtype,
                 seed: int, device: torch.device, group=None):
        import torch.distributed as dist

        self.env = env
        self.world = env.world_size
        self.rank = env.rank
        self.fraction = fraction
        self.n_rows = n_rows
        self.sample_shape = tuple(sample_shape)
        self.dtype = dtype
        self.seed = seed
        self.device = torch.device(device)
        # the DP group itself: one communicator (and one RCCL stream) for loader and trainer
        # collectives, so their device order is the consumer thread's issue order (parallel/order.py)
        self.group = group if group is not None else loader_group(env)
        check_group(env, self.group, f"{type(self).__name__}")
        if env.control_group is not None:
            # every rank must trade the same number of rows: agree on the smallest window
            t = torch.tensor([n_rows], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=env.control_group)
            n_rows = self.n_rows = int(t.item())
        self.row_elems = int(math.prod(self.sample_shape)) if self.sample_shape else 1
        self.n_exchange = self._n_exchange()
        self.calls = 0
        self.bytes_sent = 0
        self.host_s = 0.0
        self._timing: list = []  # (start, end) device events of the exchanges, resolved by stats()
        self._device_ms = 0.0
        if self.device.type == "cuda" and self.world > 1 and self.n_exchange > 0:
            self.warm_up()

    def warm_up(self) -> None:
        """Run this method's transfer pattern once on scratch buffers of the exchange's size, at
        construction (every rank builds its loader at the same point of the program): RCCL sets up its
        peer connections and buffers on the first transfer to each peer, which would otherwise land on
        the first windows of the run."""
        issue(self.env, self.group, "loader.exchange_warmup")
        n = self.n_exchange * self.row_elems * _dtypes.itemsize(self.dtype)
        send = torch.zeros(n, dtype=torch.uint8, device=self.device)
        recv = torch.empty_like(send)
        self._transfer(send, recv, 0)
        torch.cuda.current_stream(self.device).synchronize()

    def _transfer(self, send: torch.Tensor, recv: torch.Tensor, window: int) -> None:  # pragma: no cover
        raise NotImplementedError

    def _n_exchange(self) -> int:
        return int(self.n_rows * self.fraction)

    def rows_perm(self, window: int) -> FeistelPermutation:
        return FeistelPermutation(self.n_rows, self.seed ^ _EXCHANGE_SALT, window)

    def _rows(self, win_bytes: torch.Tensor) -> torch.Tensor:
        return win_bytes.view(self.dtype).view((-1,) + self.sample_shape)[: self.n_rows]

    def __call__(self, win_bytes: torch.Tensor, window: int, info: dict | None = None) -> None:
        import time

        if self.n_exchange == 0:
            return
        issue(self.env, self.group, "loader.exchange", window)
        t0 = time.perf_counter()
        ev = None
        if self.device.type == "cuda":
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        self.global_shuffle(win_bytes, window)
        if ev is not None:
            ev[1].record()
            self._timing.append(ev)
            if len(self._timing) > 64:
                self._resolve(block=False)
        self.host_s += time.perf_counter() - t0

    def _resolve(self, block: bool = True) -> None:
        """Fold finished exchanges' device time into the total. ``block=False`` (the hot path) only takes
        the ones that already retired, oldest first: never a host wait on an exchange still in flight."""
        while self._timing:
            a, b = self._timing[0]
            if block:
                b.synchronize()
            elif not b.query():
                break
            self._device_ms += a.elapsed_time(b)
            self._timing.pop(0)

    def stats(self) -> dict:
        """Exchange counters: calls, bytes sent to peers, host issue time, device time (ms)."""
        self._resolve()
        return {"exchange_calls": self.calls, "rccl_bytes": self.bytes_sent,
                "exchange_ms": round(self._device_ms, 3), "exchange_host_s": round(self.host_s, 4)}

    def global_shuffle(self, win_bytes: torch.Tensor, window: int) -> None:
        """Trade this window's ``n_exchange`` rows selected by ``rows_perm(window)``: gather them into a
        contiguous send buffer, run the method's ``_transfer`` on the DP group, scatter the received rows
        back into the same positions (all on the current stream: the stager's post-copy stream)."""
        n_ex = self.n_exchange
        if n_ex == 0:
            return
        rows = self._rows(win_bytes)
        px = self.rows_perm(window)
        send = ops.gather_rows(rows, perm=px, base=0, n_rows=n_ex)
        recv = torch.empty_like(send)
        self._transfer(send.view(-1).view(torch.uint8), recv.view(-1).view(torch.uint8), window)
        idx = ops.feistel_indices(px, 0, n_ex, device=rows.device)
        ops.scatter_rows(rows, recv, idx)
        self.calls += 1
        self.bytes_sent += self._peer_bytes(send.numel() * send.element_size())

    def _peer_bytes(self, n: int) -> int:
        return n


class AllToAllGlobalShuffler(GlobalShuffler):
    """Fraction-exchange as one all-to-all over every peer (all xGMI links)."""

    def _n_exchange(self) -> int:
        n = int(self.n_rows * self.fraction)
        return n // self.world * self.world

    def _peer_bytes(self, n: int) -> int:
        return n * (self.world - 1) // self.world  # the chunk for self stays

    def _transfer(self, send: torch.Tensor, recv: torch.Tensor, window: int) -> None:
        import torch.distributed as dist

        dist.all_to_all_single(recv, send, group=self.group)


class SendRecvReplaceGlobalShuffler(GlobalShuffler):
    """Reference pattern: half the rows to ``send_to``, half to ``recv_from`` (ddl/shuffle.py:82-108)."""

    def _n_exchange(self) -> int:
        return int(self.n_rows * self.fraction) // 2 * 2

    def partners(self, window: int) -> tuple[int, int]:
        rng = np.random.default_rng([self.seed & 0xFFFFFFFF, window])
        return derangement_partners(self.world, self.rank, rng)

    def _calculate_comm_partner(self, window: int = 0) -> tuple[int, int]:
        """Reference name (ddl/shuffle.py:32-79). The reference draws one pattern per
        producer from a seed shared by the k-th producers; here it is drawn per
        window from (seed, window), identical on every rank, nothing communicated."""
        return self.partners(window)

    def _transfer(self, send: torch.Tensor, recv: torch.Tensor, window: int) -> None:
        """First half of the rows to ``send_to`` / from ``recv_from``, second half the other way round
        (reference ddl/shuffle.py:95-108), as one batch of point-to-point ops on the DP group."""
        import torch.distributed as dist

        half = send.numel() // 2
        send_to, recv_from = self.partners(window)
        p2p = [
            dist.P2POp(dist.isend, send[:half], send_to, group=self.group),
            dist.P2POp(dist.irecv, recv[:half], recv_from, group=self.group),
            dist.P2POp(dist.isend, send[half:], recv_from, group=self.group),
            dist.P2POp(dist.irecv, recv[half:], send_to, group=self.group),
        ]
        for req in dist.batch_isend_irecv(p2p):
            req.wait()


_METHODS = {
    "alltoall": AllToAllGlobalShuffler,
    "all_to_all": AllToAllGlobalShuffler,
    "sendrecv_replace": SendRecvReplaceGlobalShuffler,
}


def make_exchange(env: DDLEnv, method: str, fraction: float, n_rows: int, sample_shape, dtype, seed: int, device,
                  shuffle: str = "none") -> GlobalShuffler:
    try:
        cls = _METHODS[method]
    except KeyError:
        raise NotImplementedError(
            f"exchange method {method!r} is not implemented; one of {sorted(_METHODS)}") from None
    dtype = _dtypes.to_torch_dtype(dtype)
    sh = cls(env, fraction, n_rows, tuple(sample_shape), dtype, seed, device)
    logger.debug("global shuffle: %s, %d rows/window", cls.__name__, sh.n_exchange)
    return sh
