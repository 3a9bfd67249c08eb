"""Fixed-cost synthetic train steps used to measure GPU idle % behind the loader.

``PatchMLP`` is a ViT-shaped GEMM model (patch embedding + pre-norm MLP
blocks + mean pool + classifier) so its cost is hipBLASLt GEMMs -- no MIOpen
convolution tuning on first use -- and scales with ``dim``/``depth``. A step
is forward + backward + SGD update in bf16 on the compute stream.
"""

from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class PatchMLP(nn.Module):
    def __init__(self, in_ch: int = 3, image: int = 224, patch: int = 16, dim: int = 384, depth: int = 4,
                 mlp_ratio: int = 4, n_classes: int = 1000):
        super().__init__()
        self.patch = patch
        self.embed = nn.Linear(in_ch * patch * patch, dim)
        self.blocks = nn.ModuleList(
            nn.Sequential(nn.LayerNorm(dim), nn.Linear(dim, dim * mlp_ratio), nn.GELU(),
                          nn.Linear(dim * mlp_ratio, dim))
            for _ in range(depth))
        self.norm = nn.LayerNorm(dim)
        self.head = nn.Linear(dim, n_classes)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        b, c, h, w = x.shape
        p = self.patch
        x = x.reshape(b, c, h // p, p, w // p, p).permute(0, 2, 4, 1, 3, 5).reshape(b, (h // p) * (w // p), c * p * p)
        x = self.embed(x)
        for blk in self.blocks:
            x = x + blk(x)
        return self.head(self.norm(x).mean(dim=1))


class TrainStep:
    """forward + backward + SGD on one [B, 3, H, W] batch (labels synthetic).

    With a ``process_group`` of more than one rank the model is wrapped in
    ``DistributedDataParallel``: the gradient all-reduce (RCCL over xGMI on
    GPUs) runs in buckets overlapped with backward, as in real DP training.
    One bucket per ~the whole model (``bucket_cap_mb``) keeps it to a few large
    collectives, which is what a per-link-bound xGMI ring wants.
    """

    def __init__(self, device, dim: int = 384, depth: int = 4, lr: float = 1e-3, dtype=torch.bfloat16,
                 process_group=None, bucket_cap_mb: float = 16.0):
        torch.manual_seed(0)  # identical init on every rank (DDP also broadcasts rank 0's weights)
        self.model = PatchMLP(dim=dim, depth=depth).to(device=device, dtype=dtype)
        self.ddp = False
        if process_group is not None:
            import torch.distributed as dist

            if dist.get_world_size(process_group) > 1:
                dev = torch.device(device)
                self.model = nn.parallel.DistributedDataParallel(
                    self.model, device_ids=[dev.index] if dev.type == "cuda" else None,
                    process_group=process_group, bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True)
                self.ddp = True
                from ..parallel.order import LEDGER, ddp_ledger_hook

                if LEDGER.enabled:  # record each bucket all-reduce at issue (collective-order check)
                    self.model.register_comm_hook(None, ddp_ledger_hook(process_group))
        self.opt = torch.optim.SGD(self.model.parameters(), lr=lr)
        self.device = device
        self.dtype = dtype

    def __call__(self, images: torch.Tensor) -> torch.Tensor:
        x = images.to(self.dtype)
        labels = torch.zeros(x.shape[0], dtype=torch.long, device=x.device)
        loss = F.cross_entropy(self.model(x).float(), labels)
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        self.opt.step()
        return loss.detach()


class TokenMLP(nn.Module):
    """Token-model stand-in for config 4: token + position embeddings, pre-norm MLP blocks over every
    position (masked padding), a small per-token head. GEMM cost scales with rows x seq_len x dim."""

    def __init__(self, vocab: int = 50257, seq_len: int = 4096, dim: int = 256, depth: int = 2, mlp_ratio: int = 4,
                 n_out: int = 256):
        super().__init__()
        self.tok = nn.Embedding(vocab, dim)
        self.pos = nn.Embedding(seq_len, dim)
        self.blocks = nn.ModuleList(
            nn.Sequential(nn.LayerNorm(dim), nn.Linear(dim, dim * mlp_ratio), nn.GELU(),
                          nn.Linear(dim * mlp_ratio, dim))
            for _ in range(depth))
        self.norm = nn.LayerNorm(dim)
        self.head = nn.Linear(dim, n_out)

    def forward(self, ids: torch.Tensor, pos: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        x = self.tok(ids.long()) + self.pos(pos.long())
        x = x * mask.unsqueeze(-1).to(x.dtype)
        for blk in self.blocks:
            x = x + blk(x)
        return self.head(self.norm(x))


class TokenTrainStep:
    """forward + backward + SGD on one collated token batch (``input_ids``, ``position_ids``,
    ``attention_mask``); the target is the next token id folded into ``n_out`` classes, padding ignored."""

    def __init__(self, device, seq_len: int = 4096, dim: int = 256, depth: int = 2, n_out: int = 256,
                 lr: float = 1e-3, dtype=torch.bfloat16, vocab: int = 50257):
        torch.manual_seed(0)
        self.model = TokenMLP(vocab, seq_len, dim, depth, n_out=n_out).to(device=device, dtype=dtype)
        self.opt = torch.optim.SGD(self.model.parameters(), lr=lr)
        self.n_out = n_out

    def __call__(self, batch: dict) -> torch.Tensor:
        ids, pos, mask = batch["input_ids"], batch["position_ids"], batch["attention_mask"]
        logits = self.model(ids, pos, mask)
        target = torch.roll(ids, -1, dims=1).long() % self.n_out
        target = target.masked_fill(mask == 0, -100)
        loss = F.cross_entropy(logits.float().flatten(0, 1), target.flatten(), ignore_index=-100)
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        self.opt.step()
        return loss.detach()


class CalibratedStep:
    """A consumer step of a chosen GPU duration: read the whole batch, then a chain of bf16 GEMMs.

    Used to place the training step's rate at a chosen multiple of the loader's feed rate
    (``benchmarks/bench_idle_sweep.py``), so GPU idle % is measured where the loader is the
    bottleneck, not only behind a model far slower than the feed. The batch is read by the
    streaming checksum kernel (every byte, one launch); the GEMM chain (``m x k @ k x k``,
    hipBLASLt) is sized by timing it on this GPU: ``reps = round((step_ms - read_ms) / gemm_ms)`` whole
    GEMMs plus one GEMM over the first ``tail_rows`` rows (multiples of 256) for the remainder, so the
    step time is tunable to ~1% instead of one GEMM's ~10%. ``tune`` re-sizes the chain from a busy time
    measured in the real loop (clocks and memory traffic there differ from the isolated timing).
    """

    def __init__(self, device, step_ms: float, m: int | None = None, k: int = 4096, dtype=torch.bfloat16,
                 min_reps: int = 8, read_keys: tuple | None = None):
        from .. import ops

        self.device = torch.device(device)
        self.read_keys = read_keys  # dict batches: read only these entries (None: every tensor)
        self.step_ms = float(step_ms)
        g = torch.Generator(device="cpu").manual_seed(0)
        self.w = (torch.randn(k, k, generator=g) / k ** 0.5).to(self.device, dtype)
        if m is None:  # rows of the GEMM: at least `min_reps` GEMMs per step, so the step time is finely tunable
            probe = torch.empty(4096, k, dtype=dtype, device=self.device)
            t4k = self._time(lambda: torch.mm(probe, self.w))
            m = int(min(8192, max(256, 4096 * (self.step_ms / min_reps) / t4k)) // 256 * 256)
            del probe
        self.a = (torch.randn(m, k, generator=g) / k ** 0.5).to(self.device, dtype)
        self.out = torch.empty(m, k, dtype=dtype, device=self.device)
        self.acc = ops.ChecksumAccumulator(self.device)
        self.gemm_ms = self._time(lambda: torch.mm(self.a, self.w, out=self.out))
        self.reps = 0
        self.tail_rows = 0
        self.read_ms = 0.0

    def _time(self, fn, reps: int = 20) -> float:
        fn()
        torch.cuda.synchronize(self.device)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        return s.elapsed_time(e) / reps

    def calibrate(self, batch) -> "CalibratedStep":
        """Time the batch read on a real batch and size the GEMM chain to fill the step."""
        self.read_ms = self._time(lambda: self._read(batch))
        self._size(self.gemm_ms)
        return self

    def _size(self, gemm_ms: float) -> None:
        m = self.a.shape[0]
        plan = getattr(self, "plan_ms", self.step_ms)
        work = max(0.0, plan - self.read_ms) / max(gemm_ms, 1e-6)  # in whole GEMMs
        self.reps = int(work)
        self.tail_rows = min(m, int(round((work - self.reps) * m / 256)) * 256)
        if self.tail_rows == m:
            self.reps, self.tail_rows = self.reps + 1, 0

    def tune(self, busy_ms_per_step: float) -> "CalibratedStep":
        """Re-size the GEMM chain from the busy time per step measured in the real loop."""
        units = self.reps + self.tail_rows / self.a.shape[0]
        if units > 0 and busy_ms_per_step > self.read_ms:
            self.gemm_ms = (busy_ms_per_step - self.read_ms) / units
            self._size(self.gemm_ms)
        return self

    def correct(self, busy_ms_per_step: float) -> "CalibratedStep":
        """Multiplicative correction: the step measured ``busy_ms_per_step`` against its ``step_ms`` target, so
        plan the chain for ``plan x target / measured`` (the GEMMs' time in the loop is not exactly linear in
        their count -- the tail GEMM, clocks, the loader's traffic -- so re-sizing from a per-GEMM time alone
        can settle off target)."""
        if busy_ms_per_step > 0:
            self.plan_ms = getattr(self, "plan_ms", self.step_ms) * self.step_ms / busy_ms_per_step
            self._size(self.gemm_ms)
        return self

    def _read(self, batch) -> None:
        if isinstance(batch, dict):
            tensors = batch.values() if self.read_keys is None else (batch[k] for k in self.read_keys)
        else:
            tensors = batch if isinstance(batch, (tuple, list)) else (batch,)
        for t in tensors:
            if isinstance(t, torch.Tensor) and t.is_cuda:
                self.acc.add(t)

    @property
    def planned_ms(self) -> float:
        return self.read_ms + (self.reps + self.tail_rows / self.a.shape[0]) * self.gemm_ms

    def __call__(self, batch) -> None:
        self._read(batch)
        for _ in range(self.reps):
            torch.mm(self.a, self.w, out=self.out)
        if self.tail_rows:
            torch.mm(self.a[:self.tail_rows], self.w, out=self.out[:self.tail_rows])
