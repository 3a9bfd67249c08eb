"""Order verification of indexed windows (``DDL_VERIFY_ORDER`` / ``OrderSpec(verify=True)``).

SURVEY §5 race detection: a producer/consumer cursor disagreement, a stale or reused slot, or a wrong resume
position must raise instead of silently training on the wrong samples. ``IndexedProducer`` publishes
(epoch, global batch, digest of the sample ids) in the slot tags of each window; the consumer recomputes them
from its own cursor and ``EpochOrder``.
"""

from __future__ import annotations


class OrderVerifyMixin:
    def _setup_verify(self, verify_order: bool | None, md, rank, world) -> None:
        """``verify_order`` (default ``$DDL_VERIFY_ORDER=1``): check every window of the indexed order
        against the epoch order before its batches are used. ``IndexedProducer`` publishes (epoch,
        global batch, digest of the sample ids) in the slot tags of each window; the consumer recomputes
        them from its own cursor and ``EpochOrder``, so a producer/consumer cursor disagreement, a stale
        or reused slot, or a wrong resume position raises ``DataIntegrityError`` instead of silently
        training on the wrong samples (race detection). Costs one host-side Feistel
        evaluation of the local batch and a hash per window."""
        import os

        self._verify = None
        self.verified_windows = 0
        want = verify_order if verify_order is not None else os.environ.get("DDL_VERIFY_ORDER") == "1"
        if not want:
            return
        ex = md[0].extra if md else {}
        ok = (self.mode == "indexed" and self.collate is None and "order_seed" in ex
              and "windows_per_epoch" not in ex)  # one global batch per window (IndexedProducer)
        if not ok:
            if verify_order:
                raise ValueError("verify_order needs mode='indexed' windows from IndexedProducer")
            return
        from .permutation import EpochOrder

        self._verify = EpochOrder(int(ex["n_samples"]), int(ex["global_batch"]), int(ex["order_seed"]),
                                  bool(ex.get("order_drop_last", True)), bool(ex.get("order_shuffle", True)))
        self._verify_rank = (int(rank or 0), int(world or 1))

    def _verify_window(self, w: int, tags) -> None:
        from .exceptions import DataIntegrityError
        from .permutation import ids_digest

        epoch, g = divmod(int(w), self.windows_per_epoch)
        ids = self._verify.indices(epoch, g, *self._verify_rank)
        want = (epoch, g, ids_digest(ids))
        got = tuple(int(x) for x in tuple(tags)[:3])
        if got != want:
            raise DataIntegrityError(
                f"window {w}: the epoch order expects (epoch {epoch}, global batch {g}, ids digest {want[2]:#x}); "
                f"the producer published (epoch {got[0] if got else None}, global batch "
                f"{got[1] if len(got) > 1 else None}, ids digest {got[2] if len(got) > 2 else 0:#x})")
        self.verified_windows += 1
