"""Checkpoint / resume of ``DistributedDataLoader``: the epoch / sample-index cursor.

The reference has no checkpointing; its only resumable state is the consumer's ``epoch`` / ``batch`` /
``target_rank`` (``/root/reference/ddl/mpi_dataloader.py:119-121``) plus producer RNG states. Here the
cursor is the north star's epoch/sample-index format: ``kind="indexed"`` (world-size-invariant order)
stores ``(seed, epoch, global_batch_cursor, global_sample_cursor)`` plus the order's geometry and resumes
at ANY world size; ``kind="window"`` stores the producer-window schedule's cursor. ``set_epoch`` and
``load_state_dict`` on a running loader are live seeks: producers repositioned, staging restarted.
"""

from __future__ import annotations

import torch

from .exceptions import ShapeMismatchError
from .permutation import batch_cursor
from .utils.logging import for_all_methods, with_logging
from .utils.tracing import trace_range

STATE_VERSION = 1


@for_all_methods(with_logging)
class CheckpointMixin:
    """``set_epoch`` / ``state_dict`` / ``load_state_dict`` of ``DistributedDataLoader``."""

    def set_epoch(self, epoch: int) -> None:
        """torch-style ``sampler.set_epoch``: position the loader at the START of ``epoch``.

        A no-op when the cursor is already there (the usual ``for e in range(n): dl.set_epoch(e)``
        loop); otherwise a live seek (producers repositioned, staging restarted), so batches and
        their order are exactly those of ``epoch`` in an uninterrupted run. Called mid-epoch for
        the current epoch, it restarts that epoch.
        """
        epoch = int(epoch)
        if epoch == self.epoch and self.epoch_batch == 0 and not self._pending:
            return
        if not 0 <= epoch < self.n_epochs:
            raise ValueError(f"epoch {epoch} outside [0, {self.n_epochs})")
        if self.connection is None or self.connection.n_producers == 0:
            self.epoch = epoch
            return
        if self.mode == "indexed" or self.mode == "split_along_epoch" or self.mode == "do_not_split_along_epoch":
            w = epoch * self.windows_per_epoch
            self._seek(window=w, window_in_epoch=0, epoch=epoch, batch=0, epoch_batch=0)

    def state_dict(self) -> dict:
        """Checkpointable cursor. A batch already handed out by the auto-marking
        iterator counts as consumed (resume continues with the next one).

        ``kind="indexed"`` (world-size-invariant order): ``(seed, epoch,
        global_batch_cursor)`` + the order's geometry -- resumable at ANY world
        size with the same global batch. ``kind="window"``: epoch / window /
        batch cursor of the producer-window schedule (same layout required).
        """
        consumed = self.epoch_batch + (1 if self._pending else 0)
        base = {
            "version": STATE_VERSION,
            "seed": self.seed,
            "epoch": self.epoch,
            "batch_size": self.batch_size,
            "world_size": self.env.world_size if self.env else self.n_instances,
            "dtype": str(self.out_dtype or getattr(self, "window_dtype", torch.float32)).replace("torch.", ""),
            "shuffle": self.shuffle,
            "fraction_exchange": self.fraction_exchange,
        }
        if self.mode == "indexed":
            extra = self.metadata_from_producer[0].extra if self.metadata_from_producer else {}
            k = self.batches_per_window[0] if self.batches_per_window else 1
            base.update({
                "kind": "indexed",
                "global_batch_cursor": consumed,
                # the same position in samples of the epoch order (the epoch/sample-index format)
                "global_sample_cursor": consumed * int(extra.get("global_batch") or 0),
                "batches_per_epoch": self.windows_per_epoch * k,
                "batches_per_window": k,
                "global_batch": extra.get("global_batch"),
                "n_samples": extra.get("n_samples"),
                "order_seed": extra.get("order_seed"),
                "drop_last": extra.get("order_drop_last"),
            })
            return base
        base.update({
            "kind": "window",
            "mode": self.mode,
            "window": self.window,
            "window_in_epoch": self.window_in_epoch,
            "batch": self.batch + (1 if self._pending else 0),
            "epoch_batch": consumed,
            "n_producers": self.connection.n_producers if self.connection else 0,
            "n_slots": self.n_slots,
        })
        return base

    def _apply_state(self, sd: dict) -> None:
        if sd.get("version") != STATE_VERSION:
            raise ValueError(f"unsupported loader state version {sd.get('version')}")
        self.epoch = int(sd["epoch"])
        if sd.get("seed") is not None:
            self.seed = int(sd["seed"])
        if sd.get("kind") == "indexed":
            bpe = int(sd["batches_per_epoch"])
            k = int(sd.get("batches_per_window", 1))  # global batches per window (token windows)
            cur = batch_cursor(sd, sd.get("global_batch"))
            if cur >= bpe:
                self.epoch, cur = self.epoch + 1, 0
            self.window = self.epoch * (bpe // k) + cur // k
            self.window_in_epoch = cur // k
            self.epoch_batch = cur
            self.batch = cur % k
            self._resume_check = sd
            return
        # exact resume, also mid-window: the producers restart at this window's round
        # (deterministic content per round) and the cursor skips its consumed batches
        self._resume_window_sd = sd
        self.window = int(sd["window"])
        self.window_in_epoch = int(sd["window_in_epoch"])
        self.batch = int(sd.get("batch", 0))
        self.epoch_batch = int(sd.get("epoch_batch", 0))

    def load_state_dict(self, sd: dict) -> None:
        """Restore a ``state_dict()`` on a LIVE loader (torch ``DataLoader``/``StatefulDataLoader`` style).

        The staging ring is drained, the producers are repositioned to the checkpointed rounds
        (``Connection.seek_producers``) and the cursor is rebuilt, so the next batch is exactly
        the one an uninterrupted run would deliver after the checkpoint -- also mid-window, and
        for ``kind="indexed"`` at a different world size (same global batch). Every rank of a
        multi-rank job must call it at the same point (its exchange collectives restart from the
        checkpointed window). Equivalent to constructing with ``resume_state=sd``.
        """
        if self._finalized:
            raise RuntimeError("load_state_dict on a finished loader: construct a new one with resume_state=")
        saved = (self.epoch, self.seed, self.window, self.window_in_epoch, self.batch, self.epoch_batch)
        self._apply_state(sd)
        try:
            if self.connection is not None and self.connection.n_producers:
                self._check_resume_layout(self.connection.n_producers)
                if self.mode == "indexed":
                    self._check_indexed_resume()
        except Exception:
            (self.epoch, self.seed, self.window, self.window_in_epoch, self.batch, self.epoch_batch) = saved
            raise
        if self.connection is None or self.connection.n_producers == 0:
            return
        self._seek(self.window, self.window_in_epoch, self.epoch, self.batch, self.epoch_batch)

    def _check_resume_layout(self, n_producers: int) -> None:
        """Window-kind checkpoints name producer rounds: the producer count must match (the slot
        count may change -- content is a function of (producer, round), not of the slot)."""
        sd = getattr(self, "_resume_window_sd", None)
        if sd is None:
            return
        if int(sd.get("n_producers", n_producers)) != n_producers:
            raise ShapeMismatchError((sd.get("n_producers"), n_producers),
                                     f"window-kind checkpoint of {sd.get('n_producers')} producers cannot resume "
                                     f"with {n_producers}: windows are (producer, round) pairs; use mode='indexed' "
                                     "for a layout-independent order")
        if sd.get("mode", self.mode) != self.mode:
            raise ShapeMismatchError((sd.get("mode"), self.mode), "checkpoint window mode differs")

    def _check_indexed_resume(self) -> None:
        chk = getattr(self, "_resume_check", None)
        if chk is None or not self.metadata_from_producer:
            return
        ex = self.metadata_from_producer[0].extra
        dl_ck, dl_now = chk.get("drop_last"), ex.get("order_drop_last")
        if dl_ck is not None and dl_now is not None and bool(dl_ck) != bool(dl_now):
            raise ShapeMismatchError(("drop_last", dl_ck, dl_now),
                                     f"checkpoint was saved with drop_last={bool(dl_ck)}, this loader has "
                                     f"drop_last={bool(dl_now)} (the epoch has a different number of batches; "
                                     "note ddl_amd.DataLoader's default is drop_last=False since round 3)")
        for key in ("global_batch", "n_samples", "order_seed"):
            if chk.get(key) is not None and ex.get(key) is not None and chk[key] != ex[key]:
                raise ShapeMismatchError((key, chk[key], ex[key]),
                                         f"checkpoint {key}={chk[key]} does not match the producers' {ex[key]}")
        k = self.batches_per_window[0]
        if int(chk["batches_per_epoch"]) != self.windows_per_epoch * k:
            raise ShapeMismatchError(chk, "checkpoint batches_per_epoch does not match")
        if int(chk.get("batches_per_window", 1)) != k:
            raise ShapeMismatchError((chk.get("batches_per_window", 1), k),
                                     "checkpoint batches_per_window differs from the producers' (the window "
                                     "cursor would not map to the same global batches)")

    def _seek(self, window: int, window_in_epoch: int, epoch: int, batch: int, epoch_batch: int) -> None:
        """Live reposition: drain staging, move the producers, rebuild the cursor and the stager."""
        if epoch >= self.n_epochs:
            raise ValueError(f"cannot seek to epoch {epoch} of a {self.n_epochs}-epoch loader")
        P = self.connection.n_producers
        with trace_range("ddl.consumer.seek"):
            # 1. stop every reader of the slots / ring buffers
            if self._batch_stream is not None:
                self._lookahead.clear()
                self._win_done.clear()
                self._batch_stream.synchronize()
            if self._stager is not None:
                self._stager.close()  # joins the native thread; copies and their slot hand-backs retire
                self._drop_engine()
            elif self._host_window is not None:
                self._host_window = None  # seek_producers resets every slot, this one included
            self._cur = None
            self._pending = False
            # 2. cursor
            self.window, self.window_in_epoch, self.epoch = int(window), int(window_in_epoch), int(epoch)
            self.batch, self.epoch_batch = int(batch), int(epoch_batch)
            self.target_rank = self.window % P + 1
            # 3. producers continue at the rounds of the new window schedule
            self.connection.seek_producers([self._first_round(p, P, self.window) for p in range(P)])
            # 4. a fresh staging ring starting at the new window
            self.total_windows = self.n_epochs * self.windows_per_epoch - self.window
            if self._stager is not None:
                from .staging import WindowStager

                old = self._stager
                self.connection.remove_finalizer(old.close)
                self._stager = WindowStager(self.connection, self.n_slots, self.total_windows, self.prefetch_depth,
                                            self.device, old.max_window_bytes, post_copy=self._exchange_fn,
                                            timeout_s=self.timeout_s, first_window=self.window,
                                            meta_bytes=old.meta_bytes, copy_timing=old.copy_timing)
                self.connection.add_finalizer(self._stager.close)
                self.metrics.bytes_h2d += old.bytes_h2d
                del old
                if self._batch_stream is not None:
                    self._make_engine()
            self._update_len()
            if self.batch == 0:
                self._begin_window()
