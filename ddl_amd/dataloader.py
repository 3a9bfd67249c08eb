"""Consumer: ``DistributedDataLoader`` (reference ddl/mpi_dataloader.py:31-249).

Drop-in API of the reference -- constructor arguments, ``len()`` = batches of
the current epoch, ``__getitem__`` returning a tuple of column-group tensors,
``mark(Marker.END_OF_BATCH / END_OF_EPOCH)`` driving the window state machine,
round-robin over the producers' windows, shutdown after ``n_epochs`` -- on the
MI355X-native data path:

    producer windows (pinned shm arena)
      --hipMemcpyAsync, prefetch stream, depth-2 HBM ring (staging.py)-->
    HBM window  --global-shuffle exchange over RCCL/xGMI (parallel/shuffle.py)-->
    per-batch fused gfx950 kernel on the compute stream: Feistel permutation
    gather + dtype cast + per-channel normalise / HWC->CHW collate / contiguous
    column split (ops/) --> device tensors.

On a CPU-only host the batches are zero-copy views of the shm windows, as in
the reference (reference ddl/mpi_dataloader.py:190-196).

Additions over the reference: ``__iter__`` (optionally auto-marking, i.e. a
torch DataLoader drop-in), ``set_epoch``, ``state_dict``/``load_state_dict``
(epoch/window/batch cursor + seed), device output dtype/normalisation, the
device-side permutation, prefetch depth, bounded waits with typed errors.

Window schedule: window ``w`` (0, 1, 2, ... over the whole run) comes from
producer ``w % P``, which fills its rounds into slots ``round % n_slots``, so
window ``w`` is producer round ``w // P`` in slot ``(w // P) % n_slots``.
An epoch is ``windows_per_epoch`` consecutive windows: 1 (reference default
"do_not_split_along_epoch", ddl/mpi_dataloader.py:149-157), P
("split_along_epoch") or the producer-announced count (indexed producers,
where one window is one global batch).
"""

from __future__ import annotations

import collections
import math
import os
import time
from abc import ABC, abstractmethod
from typing import Any, Iterator

import torch

from . import ops
from .checkpoint import CheckpointMixin
from .connection import Connection
from .engine_dispatch import NativeDispatchMixin
from .datasetwrapper import ProducerFunctionSkeleton
from .exceptions import ShapeMismatchError
from .ops import _dtypes
from .permutation import FeistelPermutation
from .types import DDLEnv, Marker, MetaData_Consumer_To_Producer, MetaData_Producer_To_Consumer
from .utils.logging import for_all_methods, with_logging
from .utils import streams
from .utils.tracing import LoaderMetrics, trace_range

_FAULT_RANK = bool(os.environ.get("DDL_FAULT_RANK"))  # test hook (utils/faults.py)
MODES = ("do_not_split_along_epoch", "split_along_epoch", "window", "indexed")


def _mix(a: int, b: int) -> int:
    """64-bit mix of two ints (splitmix64 finaliser over a*phi + b)."""
    z = (int(a) * 0x9E3779B97F4A7C15 + int(b) + 0x632BE59BD9B4E019) & ((1 << 64) - 1)
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & ((1 << 64) - 1)
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & ((1 << 64) - 1)
    return z ^ (z >> 31)


def window_perm_key(producer: int, round_: int) -> int:
    """Key of the device permutation of one window visit (producer ``p``, round ``seq``): a 64-bit
    mix of both, so every (producer, round) pair has its own order at any producer count."""
    return _mix(producer, round_) & ((1 << 63) - 1)


class DistributedDataloaderABC(ABC):
    """The reference's abstract consumer interface (ddl/mpi_dataloader.py:31-103).

    ``_start_access_epoch`` / ``_end_access_epoch`` take / hand back the
    current producer window, ``_advance_to_next_producer`` moves the cursor to
    the next window of the round-robin, ``mark`` drives the state machine.
    """

    @abstractmethod
    def __len__(self) -> int: ...

    @abstractmethod
    def __getitem__(self, index: int): ...

    @abstractmethod
    def _advance_to_next_producer(self) -> None: ...

    @abstractmethod
    def _finalize(self) -> None: ...

    @abstractmethod
    def _start_access_epoch(self, target_rank: int = 0) -> None: ...

    @abstractmethod
    def _end_access_epoch(self, target_rank: int = 0) -> None: ...

    @abstractmethod
    def _can_continue(self) -> bool: ...

    @abstractmethod
    def mark(self, mark: Marker) -> None: ...


@for_all_methods(with_logging, exclude=["__getitem__", "__len__", "__iter__", "mark", "_on_batch_end",
                                        "_window", "_batch_from_window", "_schedule", "_engine_batch",
                                        "_engine_provide", "_release_window", "_advance_window",
                                        "_advance_to_next_producer", "_begin_window", "_update_len",
                                        "_end_access_epoch", "_device_batch", "_enqueue_batch"])
class DistributedDataLoader(NativeDispatchMixin, CheckpointMixin, DistributedDataloaderABC):
    def __init__(
        self,
        producer_function: ProducerFunctionSkeleton,
        batch_size: int,
        connection: Connection | None,
        n_epochs: int,
        fraction_exchange: float = 0.0,
        exchange_method: str = "alltoall",
        instance_idx: int = 0,
        n_instances: int = 1,
        *,
        device: str | torch.device | None = None,
        out_dtype: Any = None,
        shuffle: str = "none",
        seed: int = 0,
        n_slots: int | None = None,
        prefetch_depth: int = 4,
        mode: str = "window",
        normalize: dict | None = None,
        augment: dict | None = None,
        contiguous: bool = False,
        env: DDLEnv | None = None,
        auto_mark: bool = False,
        resume_state: dict | None = None,
        timeout_s: float | None = None,
        host_threads: int = 4,
        debug_checksum: bool = False,
        copy_batches: bool | None = None,
        collate: str | None = None,
        pad_id: int = 0,
        native_dispatch: bool | str = True,
        token_rows: str = "exact",
        verify_order: bool | None = None,
        max_ahead: int | None = None,
        copy_timing: bool = False,
    ):
        if mode not in MODES:
            raise ValueError(f"unknown mode {mode!r}; one of {MODES}")
        if shuffle not in ("none", "device"):
            raise ValueError("shuffle must be 'none' or 'device'")
        self.batch_size = int(batch_size)
        self.connection = connection
        self.n_epochs = int(n_epochs)
        self.fraction_exchange = float(fraction_exchange)
        self.exchange_method = exchange_method
        self.instance_idx = instance_idx
        self.n_instances = n_instances
        self.shuffle = shuffle
        self.seed = int(seed)
        # default: what the producer asks for (ProducerFunctionSkeleton.preferred_slots, 1 unless its rounds
        # rewrite the whole window)
        self.n_slots = int(n_slots if n_slots is not None else getattr(producer_function, "preferred_slots", 1))
        self.prefetch_depth = int(prefetch_depth)
        self.mode = "do_not_split_along_epoch" if mode == "window" else mode
        self.normalize = normalize
        # on-device RandomResizedCrop + flip (GPU only): {"size": (224, 224), "scale": (0.08, 1.0),
        # "ratio": (3/4, 4/3), "flip_p": 0.5, "layout": "chw" | "hwc"}; normalize's mean/std apply after it
        aug_keys = {"size", "scale", "ratio", "flip_p", "layout"}
        if augment is not None and not set(augment) <= aug_keys:
            raise ValueError(f"unknown augment keys {sorted(set(augment) - aug_keys)}")
        self.augment = augment
        self.contiguous = contiguous
        self.env = env
        self.auto_mark = auto_mark
        # Zero-copy views alias the window and die when it is released (reference
        # semantics, ddl/mpi_dataloader.py:193). With auto_mark the caller does not
        # control the release, so batches are owned copies by default.
        self.copy_batches = auto_mark if copy_batches is None else bool(copy_batches)
        if collate not in (None, "tokens"):
            raise ValueError("collate must be None or 'tokens'")
        self.collate = collate
        self.pad_id = pad_id
        # collate="tokens", pack mode: "exact" -> [packed rows, S] per batch; "fixed" -> every batch has the
        # window layout's max rows (padding rows past the packed ones): static shapes, and no per-batch
        # slicing of four [R, S] outputs on the host (~2 us per tensor view)
        if token_rows not in ("exact", "fixed"):
            raise ValueError("token_rows must be 'exact' or 'fixed'")
        self.token_rows = token_rows
        self.debug_checksum = debug_checksum
        # device times of every window copy from the first one (WindowStager.copy_timing: bytes_in_interval and
        # copy_summary need them; direct DMA takes them from a process-wide ROCr switch, so off by default)
        self.copy_timing = bool(copy_timing)
        self.metrics = LoaderMetrics()
        self.timeout_s = timeout_s if timeout_s is not None else (connection.timeout_s if connection else 600.0)
        self._timeout_ms = int(self.timeout_s * 1000)
        self.checksums: list[int] = []
        self._pending = False

        # cursor
        self.epoch = 0
        self.batch = 0          # batches consumed in the current window
        self.epoch_batch = 0    # batches consumed in the current epoch
        self.window = 0         # global window index
        self.window_in_epoch = 0
        if resume_state is not None:
            self._apply_state(resume_state)
        self.target_rank = 1    # reference-compatible: producer of the current window, 1-based

        if device is None:
            if env is not None and env.device:
                device = env.device
            else:
                device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        if self.augment is not None and self.device.type != "cuda":
            raise ValueError("augment= runs on the GPU (device-side crop boxes); this loader is on the CPU")
        self.out_dtype = _dtypes.to_torch_dtype(out_dtype) if out_dtype is not None else None

        self._finalized = False
        self._stager = None
        self._batch_stream = None
        self._lookahead: dict = {}
        self._verify = None  # verify_order's EpochOrder (_setup_verify)
        self.verified_windows = 0
        self._win_done: dict = {}  # window -> event after its last batch kernel (Python dispatch path)
        self._host_window: int | None = None  # host path: window currently held
        self._cur = None                      # device path: StagedWindow of the current window
        # True / "auto": native engine, inline (batch kernel on the caller's stream at get time) for batches
        # under 16 MB -- "window" (one kernel builds all of a window's batches at its first get) when a
        # window holds several small gather/split batches -- and lookahead (one batch ahead on the batch
        # stream) above 16 MB; False: the Python dispatch path
        if native_dispatch not in (True, False, "auto", "inline", "lookahead", "window"):
            raise ValueError("native_dispatch must be a bool or 'auto' / 'inline' / 'lookahead' / 'window'")
        self.native_dispatch = "auto" if native_dispatch is True else native_dispatch
        self._engine = None                   # native per-batch dispatch (csrc/kernels/engine.cpp)
        self._fields = None                   # MapDatasetSource rows: (fields, kind) to unpack batches into
        # Run-ahead bound (GPU device path): a host that never synchronises with its step (no .item(), no
        # host-side metric) would otherwise take batches as fast as the copies land, however far behind the
        # GPU's compute is, keeping the link and both copy engines saturated and a growing number of
        # batches alive in HBM. Every `_ahead_every` batches an event goes on the consumer's stream, and
        # fetching batch i waits (on the host) for the event of batch i - max_ahead: the copies then follow
        # the step's pace when the step is the bottleneck. 0 disables. (Default 16; off with the
        # global-shuffle exchange, see _setup_exchange.)
        ma = 16 if max_ahead is None else int(max_ahead)
        if ma < 0:
            raise ValueError("max_ahead must be >= 0")
        self.max_ahead = ma
        # an event every max_ahead / 4 batches (one per batch raised the GPU idle behind a slow step from
        # 0.12% to 0.17-0.18%: archive/profiles/r4_eleventh); a small ring of them is reused
        self._ahead_every = max(1, ma // 4)
        self._ahead_ring: list = []
        # (batch count, event on the consumer's stream)
        self._ahead_q = collections.deque() if self.device.type == "cuda" and ma > 0 else None
        self._ahead_n = 0
        self.ahead_waits = 0

        if connection is None or connection.n_producers == 0:
            # Reference behaviour for a single-rank run: nothing to iterate (ddl/mpi_dataloader.py:173-174).
            self._len = 0
            self.metadata_from_producer = []
            return

        P = connection.n_producers
        self._n_prod = P
        self._check_resume_layout(P)
        rounds0 = [self._first_round(p, P, self.window) for p in range(P)]
        base_meta = MetaData_Consumer_To_Producer(
            producer_function=producer_function,
            global_shuffle_fraction_exchange=self.fraction_exchange,
            global_shuffle_exchange_method=exchange_method,
            batch_size=self.batch_size,
            rank=env.rank if env else instance_idx,
            world_size=env.world_size if env else n_instances,
            n_slots=self.n_slots,
            seed=self.seed,
            host_threads=host_threads,
        )
        # per-producer start round (resume mid-run)
        import copy

        for i, pipe in enumerate(connection.pipes):
            m = copy.copy(base_meta)
            m.producer_index, m.n_producers, m.start_round = i, P, rounds0[i]
            pipe.send("meta", m)
        self.metadata_from_producer: list[MetaData_Producer_To_Consumer] = connection.recv_metadata_as_consumer()
        md = self.metadata_from_producer
        self.splits = [tuple(x.splits) for x in md]
        self.batches_per_window = [int(x.batches_per_window) for x in md]
        self.shapes = [tuple(x.shape) for x in md]
        self.dtypes = [_dtypes.to_torch_dtype(x.dtype) for x in md]
        if len(set(self.splits)) != 1 or len({s[1:] for s in self.shapes}) != 1 or len(set(self.dtypes)) != 1:
            raise ShapeMismatchError(md, "producers disagree on sample shape / splits / dtype")
        if self.mode == "indexed":
            # a window may hold k consecutive global batches (token windows: batches_per_window=k)
            wpe = {int(x.extra.get("windows_per_epoch", x.extra.get("batches_per_epoch", 0))) for x in md}
            if len(wpe) != 1 or 0 in wpe:
                raise ShapeMismatchError(md, "indexed producers must announce one batches_per_epoch")
            self.windows_per_epoch = wpe.pop()
            if len(set(self.batches_per_window)) != 1:
                raise ShapeMismatchError(md, "indexed producers must agree on batches per window")
            self._check_indexed_resume()
        elif self.mode == "split_along_epoch":
            self.windows_per_epoch = P
        else:
            self.windows_per_epoch = 1
        self._setup_verify(verify_order, md, env.rank if env else instance_idx, env.world_size if env else n_instances)
        self.sample_shape = self.shapes[0][1:]
        self.window_dtype = self.dtypes[0]
        # MapDatasetSource rows: batches come back in the dataset's sample structure (typed views)
        ex0 = md[0].extra if md else {}
        self._fields = (ex0.get("fields"), ex0.get("fields_kind")) if ex0.get("fields") else None
        if self._fields is not None and (self.window_dtype != torch.uint8 or len(self.sample_shape) != 1
                                         or self.normalize is not None or self.augment is not None
                                         or self.out_dtype not in (None, torch.uint8)):
            raise ValueError("dataset-field rows are raw bytes: no normalize / augment / out_dtype")

        views = connection.init_windows(self.shapes, self.dtypes, self.n_slots,
                                        pin=self.device.type == "cuda")
        self.arys = views  # reference name: zero-copy window views
        connection.Barrier()
        self.total_windows = self.n_epochs * self.windows_per_epoch - self.window
        self._setup_exchange()
        if self.device.type == "cuda":
            from .staging import WindowStager

            max_bytes = max(math.prod(s) * _dtypes.itemsize(d) for s, d in zip(self.shapes, self.dtypes))
            meta_bytes = max(int(x.extra.get("meta_bytes", 0)) for x in md)
            self._stager = WindowStager(connection, self.n_slots, self.total_windows, self.prefetch_depth,
                                        self.device, max_bytes, post_copy=self._exchange_fn,
                                        timeout_s=self.timeout_s, first_window=self.window, meta_bytes=meta_bytes,
                                        copy_timing=self.copy_timing)
            connection.add_finalizer(self._stager.close)  # stop the native thread before the arena is unpinned
            if self._produces_copy():
                self._batch_stream = streams.batch_stream(self.device)
                self._make_engine()
        self._update_len()


    # --------------------------------------------------------------- schedule
    def _schedule(self, w: int) -> tuple[int, int]:
        P = self.connection.n_producers
        return w % P, (w // P) % self.n_slots

    @staticmethod
    def _first_round(p: int, P: int, first_window: int = 0) -> int:
        """Number of windows of producer ``p`` before ``first_window`` (= its first round on resume)."""
        return max(0, -(-(first_window - p) // P))

    def _update_len(self) -> None:
        if self.mode == "do_not_split_along_epoch":
            p, _ = self._schedule(self.window)
            self._len = self.batches_per_window[p]
        else:
            first = self.window - self.window_in_epoch
            self._len = sum(self.batches_per_window[self._schedule(first + k)[0]]
                            for k in range(self.windows_per_epoch))

    def __len__(self) -> int:
        return self._len

    # --------------------------------------------------------------- exchange
    def _setup_exchange(self) -> None:
        self._exchange_fn = None
        world = self.env.world_size if self.env else 1
        if self.fraction_exchange <= 0 or self.env is None or self.env.process_group is None:
            return
        if world <= 1 and self.env.backend is None:
            return  # single rank without a process group: nothing to exchange with
        from .parallel.shuffle import make_exchange

        n_min = min(x.nData for x in self.metadata_from_producer)
        self._exchange_fn = make_exchange(self.env, self.exchange_method, self.fraction_exchange, n_min,
                                          self.sample_shape, self.window_dtype, self.seed,
                                          device=self.device, shuffle=self.shuffle)
        # no host-side run-ahead wait with the exchange on: the event it would wait for sits on the
        # compute stream behind collectives that wait on peer ranks, and the host must never block on
        # another rank's progress (the same rule as the device hand-off below). The exchange itself
        # bounds the run-ahead: window w + 2 is not exchanged before every rank has posted it.
        self._ahead_q = None

    # ----------------------------------------------------------------- verification
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

    # ----------------------------------------------------------------- access
    def _ensure_posted(self, w: int) -> None:
        """Issue the exchange collectives of windows ``w`` and ``w + 1`` (in order; no-ops when already
        issued). Called when the cursor enters window ``w`` -- a fixed point of the batch schedule, so
        every rank issues the same collectives in the same order (parallel/order.py) -- one window
        ahead, so window ``w + 1``'s exchange overlaps the consumption of ``w`` and the lookahead can
        build ``w + 1``'s first batch before the consumer gets there."""
        st = self._stager
        st.post(w)
        st.post(w + 1)

    def _window(self):
        """Make the current window available (device: staged; host: acquired)."""
        if self._engine is not None:
            if self._exchange_fn is not None:
                self._ensure_posted(self.window)
            if self._eng_window != self.window:
                rc, prod = self._engine.acquire(self.window, self._timeout_ms)
                if rc != 0:
                    self._engine_raise(-(10 + rc), prod, f"staging window {self.window}")
                self._eng_window = self.window
                self._eng_given.clear()
                self._eng_spare.clear()
                self.metrics.windows += 1
            return None
        if self._stager is not None:
            if self._cur is None or self._cur.index != self.window:
                t0 = time.perf_counter()
                if self._exchange_fn is not None:
                    self._ensure_posted(self.window)
                with trace_range("ddl.consumer.wait_window"):
                    self._cur = self._stager.get(self.window)
                self.metrics.consumer_wait_s += time.perf_counter() - t0
                self.metrics.windows += 1
                if self._verify is not None:
                    self._verify_window(self.window, self._cur.tags)
            return self._cur
        if self._host_window != self.window:
            p, s = self._schedule(self.window)
            t0 = time.perf_counter()
            info = self.connection.acquire(p, s, self.timeout_s)
            self.metrics.consumer_wait_s += time.perf_counter() - t0
            self.metrics.windows += 1
            if self._exchange_fn is not None:
                _, t = self.arys[p][s]
                self._exchange_fn(t.view(-1).view(torch.uint8), self.window, info)
            self._host_window = self.window
            self._host_seq = int(info["seq"])
            self._host_tags = tuple(info["tag"])
            if self._verify is not None:
                self._verify_window(self.window, self._host_tags)
            if self.collate == "tokens":  # per-sub-batch sizes live at the head of the window
                _, t = self.arys[p][s]
                nb = int(self.metadata_from_producer[p].extra.get("meta_bytes", 0))
                self._host_meta = tuple(t.reshape(-1).view(torch.uint8)[:nb].view(torch.int64).tolist())
        return None

    def _pace(self) -> None:
        """The run-ahead bound (``max_ahead``): one event per ``_ahead_every`` batches on the consumer's
        current stream; wait on the host for the one ``max_ahead`` batches back."""
        n = self._ahead_n
        self._ahead_n = n + 1
        q = self._ahead_q
        while q and q[0][0] <= n - self.max_ahead:
            ev = q.popleft()[1]
            if not ev.query():
                self.ahead_waits += 1
                ev.synchronize()
        if n % self._ahead_every == 0:
            ring, k = self._ahead_ring, n // self._ahead_every
            size = self.max_ahead // self._ahead_every + 2  # an event is re-recorded only after it left the queue
            if len(ring) < size:
                ring.append(torch.cuda.Event())
            ev = ring[k % size] if len(ring) == size else ring[-1]
            ev.record(torch.cuda.current_stream(self.device))
            q.append((n, ev))

    def __getitem__(self, idx: int):
        if self._ahead_q is not None:
            self._pace()
        eng = self._engine
        if eng is not None and 0 <= idx < self._len:  # native dispatch: the lean path
            bpw = self.batches_per_window[self.window % self._n_prod]
            local = idx - self.epoch_batch + self.batch
            if 0 <= local < bpw:
                out = self._engine_batch(local, bpw)
                self.metrics.on_batch(self.batch_size)
                if self.debug_checksum:
                    first = out["input_ids"] if isinstance(out, dict) else out[0]
                    self.checksums.append(int(ops.checksum(first).item()))
                return out if self._fields is None else self._unpack(out)
        if idx < 0:
            raise ValueError(f"negative batch index {idx}")
        if idx >= self._len:
            raise IndexError(idx)
        # map the epoch-level index to the current window
        p, s = self._schedule(self.window)
        bpw = self.batches_per_window[p]
        first_in_window = self.epoch_batch - self.batch
        local = idx - first_in_window
        if not 0 <= local < bpw:
            raise IndexError(f"batch {idx} is not in the current window (sequential access only across windows)")
        if self._engine is not None:
            out = self._engine_batch(local, bpw)
            self.metrics.on_batch(self.batch_size)
            if self.debug_checksum:
                first = out["input_ids"] if isinstance(out, dict) else out[0]
                self.checksums.append(int(ops.checksum(first).item()))
            return out if self._fields is None else self._unpack(out)
        sw = self._window()
        if self._batch_stream is not None:
            out = self._device_batch(sw, p, s, local, bpw)
        else:
            out = self._batch_from_window(sw, p, s, local)
        self.metrics.on_batch(self.batch_size)
        if self.debug_checksum:
            self.checksums.append(int(ops.checksum(out[0] if isinstance(out, tuple) else out).item()))
        return out if self._fields is None else self._unpack(out)

    def _unpack(self, out):
        from .models.datasets import unpack_fields

        rows = out[0] if isinstance(out, (tuple, list)) else out
        return unpack_fields(rows, *self._fields)

    # ---------------------------------------------------------- batch stream
    def _produces_copy(self) -> bool:
        """True when a batch is built by a kernel (not a zero-copy view of the window)."""
        return (self.shuffle == "device" or self.out_dtype not in (None, self.window_dtype) or self.augment is not None
                or self.normalize is not None or self.copy_batches or self.contiguous or self.collate is not None)

    def _enqueue_batch(self, sw, p: int, s: int, local: int):
        """Build batch ``local`` of window ``sw`` on the batch stream; returns (outputs, ready event)."""
        bs = self._batch_stream
        self._stager.wait_ready(sw, bs)
        with streams.on_stream(bs):
            out = self._batch_from_window(sw, p, s, local)
            ev = torch.cuda.Event()
            ev.record(bs)
        if local + 1 == self.batches_per_window[p]:
            # the window's free event: right after its last batch kernel, NOT at release time behind the
            # next window's lookahead kernel (which waits for that window's copy: the copy after it would
            # then wait for a copy plus a gather)
            self._win_done[sw.index] = ev
        return out, ev

    def _device_batch(self, sw, p: int, s: int, local: int, bpw: int):
        """Batch kernels run on their own stream one batch ahead of the consumer:
        batch l+1's gather overlaps the training step on batch l, and the compute
        stream only waits on an event (no host sync)."""
        hit = self._lookahead.pop((self.window, local), None)
        out, ev = hit if hit is not None else self._enqueue_batch(sw, p, s, local)
        cur = streams.current(self.device.index)
        cur.wait_event(ev)
        for t in (out.values() if isinstance(out, dict) else out):
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(cur)
        if local + 1 < bpw:
            if (self.window, local + 1) not in self._lookahead:
                self._lookahead[(self.window, local + 1)] = self._enqueue_batch(sw, p, s, local + 1)
        elif self.window_in_epoch + 1 < self.windows_per_epoch or self.epoch + 1 < self.n_epochs:
            # last batch of this window: start the next window's first batch if it is already in HBM
            nxt = self._stager.peek(self.window + 1)
            if nxt is not None and (self.window + 1, 0) not in self._lookahead:
                np_, ns = self._schedule(self.window + 1)
                self._lookahead[(self.window + 1, 0)] = self._enqueue_batch(nxt, np_, ns, 0)
        return out

    def _perm_for(self, p: int, seq: int) -> FeistelPermutation | None:
        if self.shuffle != "device":
            return None
        # key = (seed, producer, round): every window visit gets a fresh order.
        return FeistelPermutation(self.metadata_from_producer[p].nData, self.seed, window_perm_key(p, seq))

    def _batch_from_window(self, sw, p: int, s: int, local: int):
        B = self.batch_size
        n_data = self.shapes[p][0]
        wdt = self.window_dtype
        if sw is None:  # host path: zero-copy views of the shm window
            _, win = self.arys[p][s]
            seq, tags = self._host_seq, self._host_tags
            meta = getattr(self, "_host_meta", ())
        else:
            win = sw.data.view(wdt).view((n_data,) + self.sample_shape) if self.collate is None else sw.data
            seq, tags, meta = sw.seq, sw.tags, sw.meta
        if self.collate == "tokens":
            from .models.tokens import TokenWindowLayout, collate_token_window

            ex = self.metadata_from_producer[p].extra
            with trace_range("ddl.consumer.tokens"):
                return collate_token_window(win.reshape(-1), TokenWindowLayout(**ex["token_layout"]),
                                            ex["token_mode"], meta, self.pad_id, sub=local,
                                            fixed_rows=self.token_rows == "fixed")
        perm = self._perm_for(p, seq)
        out_dtype = self.out_dtype or (torch.float32 if self.normalize is not None else wdt)
        if self.augment is not None:
            aug, norm = self.augment, self.normalize or {}
            # crop randomness keyed by (seed, epoch OF THIS WINDOW) and the row's identity (producer, round, row);
            # the window's epoch, not the cursor's: a lookahead batch of the next window is built a step early
            w = sw.index if sw is not None else self.window
            epoch = self.epoch + (w - (self.window - self.window_in_epoch)) // self.windows_per_epoch
            return (ops.random_resized_crop(
                win, perm=perm, base=local * B, n_rows=B, size=aug.get("size", (224, 224)),
                scale=aug.get("scale", (0.08, 1.0)), ratio=aug.get("ratio", (3.0 / 4.0, 4.0 / 3.0)),
                flip_p=aug.get("flip_p", 0.5), seed=_mix(self.seed, epoch),
                sample_base=_mix(p, seq) & ~0xFFFFFFFF & ((1 << 63) - 1), layout=aug.get("layout", "chw"),
                out_dtype=self.out_dtype or torch.bfloat16, mean=norm.get("mean"), std=norm.get("std")),)
        splits = list(self.splits[p])
        norm = self.normalize
        with trace_range("ddl.consumer.batch"):
            if norm is not None and norm.get("layout", "chw") == "hwc":
                x = ops.collate_hwc_to_chw(win, perm=perm, base=local * B, n_rows=B, out_dtype=out_dtype,
                                           mean=norm.get("mean"), std=norm.get("std"))
                return (x,)
            if (self.contiguous or self.copy_batches) and len(splits) > 1 and len(self.sample_shape) == 1 \
                    and norm is None:
                return ops.split_columns(win, splits, perm=perm, base=local * B, n_rows=B, out_dtype=out_dtype)
            if perm is None and out_dtype == wdt and norm is None and not self.copy_batches:
                x = win[local * B:(local + 1) * B]  # zero-copy view (reference semantics)
            else:
                kw = {}
                if norm is not None:
                    plane = int(math.prod(self.sample_shape[1:])) if len(self.sample_shape) > 1 else 1
                    c = self.sample_shape[0] if len(self.sample_shape) > 1 else len(norm.get("mean", [0]))
                    sc, bi = ops.norm_affine(c, norm.get("mean"), norm.get("std"), norm.get("scale"),
                                             norm.get("bias"), ops.pixel_max(wdt))
                    kw = dict(scale=sc, bias=bi, plane=plane)
                x = ops.gather_rows(win, perm=perm, base=local * B, n_rows=B, out_dtype=out_dtype, **kw)
        if len(splits) == 1:
            return (x,)
        parts = torch.split(x.reshape(B, -1), splits, dim=1)
        if self.contiguous or self.copy_batches:  # normalised tabular rows: own each column group
            return tuple(t.contiguous() for t in parts)
        return parts

    def __iter__(self) -> Iterator:
        n = self._len
        start = self.epoch_batch  # 0 at an epoch start; the resumed cursor after load_state_dict
        for i in range(start, n):
            item = self[i]
            self._pending = self.auto_mark  # yielded, not yet marked: counts as consumed in state_dict
            yield item
            self._pending = False
            if self.auto_mark:
                self.mark(Marker.END_OF_BATCH)
        if self.auto_mark:
            self.mark(Marker.END_OF_EPOCH)

    # ---------------------------------------------------------- state machine
    def mark(self, mark: Marker) -> None:
        if mark == Marker.END_OF_BATCH:
            self._on_batch_end()
        elif mark == Marker.END_OF_EPOCH:
            self._on_epoch_end()
        else:
            raise ValueError(f"Unknown mark {mark}")

    def _release_window(self) -> None:
        if self._engine is not None:
            rc = self._engine.release(self.window)
            if rc != 0:
                self._engine_raise(rc, -1, f"releasing window {self.window}")
            if self._exchange_fn is not None:
                self._stager.forget(self.window)  # the Python face's record of the posted window
            if self._eng_window == self.window:
                self._eng_window = None
                self._eng_given.clear()
                self._eng_spare.clear()
            return
        if self._stager is not None:
            stream = None
            if self._batch_stream is not None:
                # only the batch kernels read the window (the consumer gets copies made on the batch
                # stream), so the free event goes on the batch stream, behind them: no cross-stream
                # wait, and the compute stream never waits on a lookahead gather
                for key in [k for k in self._lookahead if k[0] <= self.window]:
                    del self._lookahead[key]
                stream = self._batch_stream
                done = self._win_done.pop(self.window, None)
                for key in [k for k in self._win_done if k < self.window]:
                    del self._win_done[key]
                if done is not None and self._stager.post_copy is None:
                    self._stager.release(self.window, event=done)
                    self._cur = None
                    return
                sw = self._cur
                if sw is not None and sw.index == self.window:
                    # a window no batch was built from (skipped at a partial epoch end) can still have
                    # its exchange running on the post-copy stream: the free event must follow it too
                    self._stager.wait_ready(sw, stream)
            self._stager.release(self.window, stream)
            self._cur = None
        elif self._host_window == self.window:
            p, s = self._schedule(self.window)
            self.connection.release(p, s)
            self._host_window = None

    # reference protocol names (ddl/mpi_dataloader.py:200-218): the same state machine
    def _start_access_epoch(self, target_rank: int = 0) -> None:
        """Take the current window (staged in HBM, or the shm slot on the host path)."""
        if self.connection is not None and self.connection.n_producers and not self._finalized:
            self._window()

    def _end_access_epoch(self, target_rank: int = 0) -> None:
        """Hand the current window back to its producer."""
        if self.connection is not None and self.connection.n_producers:
            self._release_window()

    def _advance_to_next_producer(self) -> None:
        """Move the cursor to the next window of the producer round-robin."""
        self.window += 1
        self.window_in_epoch += 1
        self.batch = 0
        self.target_rank = self.window % self.connection.n_producers + 1
        if self.mode == "do_not_split_along_epoch":
            self._update_len()

    def _advance_window(self) -> None:
        self._end_access_epoch()
        self._advance_to_next_producer()
        self._begin_window()

    def _begin_window(self) -> None:
        """The cursor moved to a new window: issue its exchange collective now (consumer thread,
        fixed point of the schedule, parallel/order.py) and start gathering its first batch."""
        if _FAULT_RANK:
            from .utils.faults import maybe_fail_rank

            maybe_fail_rank(self.env.rank if self.env else 0, self.window)
        st = self._stager
        if st is None or st.post_copy is None or self._finalized:
            return
        self._ensure_posted(self.window)
        if self._engine is None and self._batch_stream is not None and (self.window, 0) not in self._lookahead:
            sw = st.peek(self.window)
            if sw is not None:
                p, s = self._schedule(self.window)
                self._lookahead[(self.window, 0)] = self._enqueue_batch(sw, p, s, 0)

    def _on_batch_end(self) -> None:
        if self._finalized:
            return
        self.batch += 1
        self.epoch_batch += 1
        p, _ = self._schedule(self.window)
        if self.batch >= self.batches_per_window[p]:
            if self.window_in_epoch + 1 < self.windows_per_epoch:
                self._advance_window()
            else:
                # last window of the epoch: hand it back now (the reference releases at
                # the window's last END_OF_BATCH too, ddl/mpi_dataloader.py:223-227)
                self._release_window()

    def _on_epoch_end(self) -> None:
        if self._finalized or self.connection is None or self.connection.n_producers == 0:
            self.epoch += 1
            return
        self._release_window()
        last = self.epoch + 1 >= self.n_epochs
        # a partial epoch still consumes its remaining windows, in order, so the
        # producers' round-robin stays aligned (skipped entirely when finishing)
        while self.window_in_epoch + 1 < self.windows_per_epoch:
            self.window += 1
            self.window_in_epoch += 1
            if not last:
                self._window()
                self._release_window()
        self.window += 1
        self.window_in_epoch = 0
        self.batch = 0
        self.epoch_batch = 0
        self.epoch += 1
        self.target_rank = self.window % self.connection.n_producers + 1
        if self.epoch >= self.n_epochs:
            self._finalize()
        else:
            self._update_len()
            self._begin_window()

    def _can_continue(self) -> bool:
        return self.epoch < self.n_epochs


    # --------------------------------------------------------------- teardown
    def _finalize(self) -> None:
        if self._finalized:
            return
        self._finalized = True
        if self._batch_stream is not None:
            self._lookahead.clear()
            self._win_done.clear()
            self._batch_stream.synchronize()
        if self.connection is not None:
            self.connection.shutdown_operation()
        if self._stager is not None:
            self.metrics.bytes_h2d += self._stager.bytes_h2d
            self._stager.close()
        self._drop_engine()
        if self.connection is not None:
            self.connection.finalize()

    def _drop_engine(self) -> None:
        if self._engine is not None:
            self.metrics.consumer_wait_s += self._engine.wait_s
            done = getattr(self, "_native_done", {"batches": 0, "lookahead_hits": 0})
            self._native_done = {"batches": done["batches"] + int(self._engine.batches),
                                 "lookahead_hits": done["lookahead_hits"] + int(self._engine.lookahead_hits)}
            self._engine.reset()
            self._engine = None
            self._eng_slots.clear()

    def close(self) -> None:
        self._finalize()

    def stats(self) -> dict:
        d = self.metrics.as_dict()
        done = getattr(self, "_native_done", None)
        if self._engine is not None or done is not None:
            nd = dict(done or {"batches": 0, "lookahead_hits": 0})
            if self._engine is not None:
                d["consumer_wait_s"] += self._engine.wait_s
                nd["batches"] += int(self._engine.batches)
                nd["lookahead_hits"] += int(self._engine.lookahead_hits)
                g, la, rec, sw = self._engine.timing_ns
                n = max(1, int(self._engine.batches))
                nd["compute_waits"] = int(self._engine.compute_waits)
                nd["ready_host_waits"] = int(self._engine.ready_host_waits)
                wait_ns = self._engine.wait_s * 1e9
                nd["host_us_per_batch"] = {"get": round(g / n / 1e3, 2),
                                           "get_excl_staging_wait": round(max(0.0, g - wait_ns) / n / 1e3, 2),
                                           "kernel_launch": round(la / n / 1e3, 2),
                                           "event_record": round(rec / n / 1e3, 2),
                                           "stream_wait": round(sw / n / 1e3, 2)}
            nd["mode"] = getattr(self, "_eng_mode", None)
            if self._engine is not None:
                nd["handoff"] = "host" if self._engine.host_handoff else "device"
            d["native_dispatch"] = nd
        if self._stager is not None:
            d.update(self._stager.stats())
        if self.connection is not None:
            d["producers"] = self.connection.producer_stats()
        if getattr(self, "_verify", None) is not None:
            d["verified_windows"] = self.verified_windows
        if getattr(self, "_ahead_q", None) is not None:
            d["run_ahead"] = {"max_ahead": self.max_ahead, "host_waits": self.ahead_waits}
        return d

    def __del__(self):  # pragma: no cover - best effort
        try:
            if not getattr(self, "_finalized", True):
                self._finalize()
        except Exception:
            pass
