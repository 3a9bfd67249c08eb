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
from .batching import WindowBatchMixin, window_perm_key
from .checkpoint import CheckpointMixin
from .connection import Connection
from .engine_dispatch import NativeDispatchMixin
from .datasetwrapper import ProducerFunctionSkeleton
from .exceptions import ShapeMismatchError
from .ops import _dtypes
from .specs import MODES, OrderSpec, OutputSpec, StagingSpec, resolve
from .types import DDLEnv, Marker, MetaData_Consumer_To_Producer, MetaData_Producer_To_Consumer
from .utils.logging import with_logging
from .utils import streams
from .utils.tracing import LoaderMetrics, trace_range
from .verify import OrderVerifyMixin

_FAULT_RANK = bool(os.environ.get("DDL_FAULT_RANK"))  # test hook (utils/faults.py)
__all__ = ["DistributedDataLoader", "DistributedDataloaderABC", "MODES", "window_perm_key"]


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


class DistributedDataLoader(WindowBatchMixin, OrderVerifyMixin, NativeDispatchMixin, CheckpointMixin,
                            DistributedDataloaderABC):
    """The reference's eight arguments (reference ddl/mpi_dataloader.py:108-118), then the rank environment,
    the device, the three option records of ``specs.py`` (``output=OutputSpec(...)``,
    ``staging=StagingSpec(...)``, ``order=OrderSpec(...)``), ``auto_mark`` (iteration marks the batches:
    a torch DataLoader drop-in) and ``resume_state`` (a ``state_dict()``). The flat keywords of earlier
    releases (``out_dtype=``, ``seed=``, ``prefetch_depth=`` ...) are deprecated aliases of the records'
    fields."""

    @with_logging
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
        env: DDLEnv | None = None,
        device: str | torch.device | None = None,
        output: OutputSpec | None = None,
        staging: StagingSpec | None = None,
        order: OrderSpec | None = None,
        auto_mark: bool = False,
        resume_state: dict | None = None,
        debug_checksum: bool = False,
        **legacy: Any,
    ):
        out, stg, odr = resolve(output, staging, order, legacy)
        self.output_spec, self.staging_spec, self.order_spec = out, stg, odr
        self.batch_size = int(batch_size)
        self.connection = connection
        self.n_epochs = int(n_epochs)
        self.fraction_exchange = float(fraction_exchange)
        self.exchange_method = exchange_method
        self.instance_idx = instance_idx
        self.n_instances = n_instances
        self.shuffle = odr.shuffle
        self.seed = int(odr.seed)
        # default: what the producer asks for (ProducerFunctionSkeleton.preferred_slots, 1 unless its rounds
        # rewrite the whole window)
        n_slots = stg.n_slots
        self.n_slots = int(n_slots if n_slots is not None else getattr(producer_function, "preferred_slots", 1))
        self.prefetch_depth = int(stg.prefetch_depth)
        self.mode = "do_not_split_along_epoch" if odr.mode == "window" else odr.mode
        self.normalize = out.normalize
        self.augment = out.augment  # on-device RandomResizedCrop + flip (GPU only); normalize applies after it
        self.contiguous = out.contiguous
        self.env = env
        self.auto_mark = auto_mark
        # Zero-copy views alias the window and die when it is released (reference
        # semantics, ddl/mpi_dataloader.py:193). With auto_mark the caller does not
        # control the release, so batches are owned copies by default.
        self.copy_batches = auto_mark if out.copy_batches is None else bool(out.copy_batches)
        self.collate = out.collate
        self.pad_id = out.pad_id
        # collate="tokens", pack mode: "exact" -> [packed rows, S] per batch; "fixed" -> every batch has the
        # window layout's max rows (padding rows past the packed ones): static shapes, and no per-batch
        # slicing of four [R, S] outputs on the host (~2 us per tensor view)
        self.token_rows = out.token_rows
        self.debug_checksum = debug_checksum
        # device times of every window copy from the first one (WindowStager.copy_timing: bytes_in_interval and
        # copy_summary need them; direct DMA takes them from a process-wide ROCr switch, so off by default)
        self.copy_timing = bool(stg.copy_timing)
        timeout_s, host_threads, out_dtype = stg.timeout_s, stg.host_threads, out.dtype
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
        self.native_dispatch = "auto" if stg.native_dispatch is True else stg.native_dispatch
        self._engine = None                   # native per-batch dispatch (csrc/kernels/engine.cpp)
        self._fields = None                   # MapDatasetSource rows: (fields, kind) to unpack batches into
        # Run-ahead bound (GPU device path): a host that never synchronises with its step (no .item(), no
        # host-side metric) would otherwise take batches as fast as the copies land, however far behind the
        # GPU's compute is, keeping the link and both copy engines saturated and a growing number of
        # batches alive in HBM. Every `_ahead_every` batches an event goes on the consumer's stream, and
        # fetching batch i waits (on the host) for the event of batch i - max_ahead: the copies then follow
        # the step's pace when the step is the bottleneck. 0 disables. (Default 16; off with the
        # global-shuffle exchange, see _setup_exchange.)
        ma = 16 if stg.max_ahead is None else int(stg.max_ahead)
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
        self._setup_verify(odr.verify, md, env.rank if env else instance_idx, env.world_size if env else n_instances)
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
    @with_logging
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
    @with_logging
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

    @with_logging
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
    @with_logging
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

    @with_logging
    def _drop_engine(self) -> None:
        if self._engine is not None:
            self.metrics.consumer_wait_s += self._engine.wait_s
            done = getattr(self, "_native_done", {"batches": 0, "lookahead_hits": 0})
            self._native_done = {"batches": done["batches"] + int(self._engine.batches),
                                 "lookahead_hits": done["lookahead_hits"] + int(self._engine.lookahead_hits)}
            self._engine.reset()
            self._engine = None
            self._eng_slots.clear()

    @with_logging
    def close(self) -> None:
        self._finalize()

    def stats(self) -> dict:
        d = self.metrics.as_dict()
        self._native_stats(d)
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
