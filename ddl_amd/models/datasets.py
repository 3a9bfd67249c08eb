"""Synthetic datasets and shared sample sources ("model families" of a data loader).

* ``PointWiseData`` / ``DummyDataset``: the reference harness's tabular
  point-cloud data with min-max / standard normalisation (reference
  tests/run_ddl.py:20-104), used by the reference-parity tests and configs.
* ``SyntheticImages``: ImageNet-shape samples (BASELINE configs 2/3/5).
* ``SyntheticTokens``: ragged token sequences (BASELINE config 4).
* ``SharedArraySource``: a node-wide dataset in POSIX shared memory, created
  once and mapped by every producer of every rank on the node; picklable by
  name. Producers gather samples out of it with the native multi-threaded
  gather (``_ddl_runtime.gather_rows``).
* ``NpyMemmapSource``: an ``.npy`` file mapped read-only (page cache shared).
* ``MapDatasetSource``: any map-style ``torch.utils.data.Dataset`` (the ``ddl_amd.DataLoader``
  drop-in); producers call ``ds[i]`` and pack each sample's fields into one byte row with a single
  native ``copy_spans`` call per batch (GIL released).
"""

from __future__ import annotations

import math
import os
from multiprocessing import shared_memory

import numpy as np
import torch

from ..ops import _dtypes


class PointWiseData:
    """Column groups [parameter | x | u | (sample weight)] (reference tests/run_ddl.py:20-77).

    REFERENCE-PARITY FIXTURE: this class and ``DummyDataset`` deliberately reproduce
    the reference harness's dataset (names, properties, normalisation and slice
    arithmetic) so the CI workload (BASELINE config 1, ``examples/run_ddl.py``)
    matches it sample for sample. It is test-fixture code, not loader logic."""

    def __init__(self, parameter_data, x_data, u_data, sample_weight=None):
        parts = [parameter_data, x_data, u_data] + ([sample_weight] if sample_weight is not None else [])
        self.data_raw = np.hstack(parts)
        self.data = None
        self.sample_weight = None
        self.n_p = parameter_data.shape[-1]
        self.n_x = x_data.shape[-1]
        self.n_o = u_data.shape[-1]

    @property
    def parameter(self):
        return self.data[:, : self.n_p]

    @property
    def x(self):
        return self.data[:, self.n_p : self.n_p + self.n_x]

    @property
    def u(self):
        return self.data[:, self.n_p + self.n_x : self.n_p + self.n_x + self.n_o]

    @staticmethod
    def standard_normalize(raw, area_weighted=False):
        mean = raw.mean(axis=0)
        std = raw.std(axis=0)
        if area_weighted:
            mean[-1] = 0.0
            std[-1] = np.mean(raw[:, -1])
            out = (raw - mean) / std
            return out[:, :-1], mean, std, out[:, -1]
        return (raw - mean) / std, mean, std

    @staticmethod
    def minmax_normalize(raw, n_para, n_x, n_target, area_weighted=False):
        mean = raw.mean(axis=0)
        std = raw.std(axis=0)
        lo, hi = raw.min(axis=0), raw.max(axis=0)
        k = n_para + n_x
        mean[:k] = 0.5 * (lo[:k] + hi[:k])
        std[:k] = 0.5 * (hi[:k] - lo[:k])
        std[k:k + n_target] = np.abs(raw[:, k:k + n_target]).max(axis=0)
        if area_weighted:
            mean[-1] = 0.0
            std[-1] = np.mean(raw[:, -1])
            out = (raw - mean) / std
            return out[:, :-1], mean, std, out[:, -1]
        return (raw - mean) / std, mean, std


class DummyDataset(PointWiseData):
    """Random (n x 10) f32 table split into groups (1, 2, 5, weight) (reference tests/run_ddl.py:80-104)."""

    ROWS_PER_TIMESTEP = 10052

    def __init__(self, nTimesteps: int, idx: int, n_instances: int, seed: int | None = None):  # noqa: N803
        n_data = nTimesteps * self.ROWS_PER_TIMESTEP
        start = -(idx + 1) * n_data // n_instances - 1
        end = -idx * n_data // n_instances - 1
        rng = np.random.default_rng(seed)
        data = rng.random((end - start, 10), dtype=np.float32)
        super().__init__(data[:, [0]], data[:, [2, 3]], data[:, [4, 5, 6, 7, 8]], data[:, [-1]])
        self.data, self.mean, self.std, self.sample_weight = self.minmax_normalize(
            self.data_raw, n_para=self.n_p, n_x=self.n_x, n_target=self.n_o, area_weighted=True)


def synthetic_images(n: int, shape=(3, 224, 224), dtype=torch.bfloat16, seed: int = 0, start: int = 0) -> torch.Tensor:
    """Deterministic synthetic images: sample i depends only on (seed, start + i)."""
    g = torch.Generator().manual_seed(seed * 1_000_003 + start)
    if dtype == torch.uint8:
        return torch.randint(0, 256, (n, *shape), generator=g, dtype=torch.uint8)
    return torch.rand((n, *shape), generator=g, dtype=torch.float32).to(dtype)


class SharedArraySource:
    """A node-wide [N, *sample_shape] array in POSIX shm (created once, mapped by name)."""

    def __init__(self, name: str, n: int, sample_shape: tuple[int, ...], dtype, create: bool = False):
        self.name = name.lstrip("/")
        self.n = int(n)
        self.sample_shape = tuple(sample_shape)
        self.dtype = _dtypes.to_torch_dtype(dtype)
        self.row_bytes = int(math.prod(self.sample_shape)) * _dtypes.itemsize(self.dtype)
        self._shm: shared_memory.SharedMemory | None = None
        self._owner = create
        if create:
            self._shm = shared_memory.SharedMemory(name=self.name, create=True, size=max(1, self.n * self.row_bytes))

    @classmethod
    def create(cls, name: str, data: torch.Tensor) -> "SharedArraySource":
        src = cls(name, data.shape[0], tuple(data.shape[1:]), data.dtype, create=True)
        src.tensor().copy_(data)
        return src

    def __getstate__(self):
        return {"name": self.name, "n": self.n, "sample_shape": self.sample_shape, "dtype": self.dtype}

    def __setstate__(self, st):
        self.__init__(st["name"], st["n"], st["sample_shape"], st["dtype"], create=False)

    def _map(self) -> shared_memory.SharedMemory:
        if self._shm is None:
            # attach without registering with the resource tracker (python < 3.13 has no
            # track=False): only the creator owns -- and unlinks -- the segment
            from multiprocessing import resource_tracker

            orig = resource_tracker.register
            resource_tracker.register = lambda *a, **k: None
            try:
                self._shm = shared_memory.SharedMemory(name=self.name, create=False)
            finally:
                resource_tracker.register = orig
        return self._shm

    @property
    def address(self) -> int:
        import ctypes

        buf = self._map().buf
        return ctypes.addressof(ctypes.c_char.from_buffer(buf))

    def tensor(self) -> torch.Tensor:
        shm = self._map()
        t = torch.frombuffer(shm.buf, dtype=torch.uint8, count=self.n * self.row_bytes)
        return t.view(self.dtype).view((self.n,) + self.sample_shape)

    def gather(self, indices: np.ndarray, dst_address: int, n_threads: int = 4) -> None:
        from .. import _native

        _native.runtime().gather_rows(dst_address, self.address, self.row_bytes,
                                      np.ascontiguousarray(indices, dtype=np.int64), self.n, n_threads)

    def bind_to_node(self, node: int, strict: bool = False) -> int:
        """Place the segment's pages on NUMA ``node`` (mbind of the shared object: pages already
        faulted in migrate, later faults by ANY process allocate there). 0 or -errno."""
        from .. import _native

        return int(_native.runtime().bind_memory_to_node(self.address, self.n * self.row_bytes, int(node), strict))

    def page_nodes(self, max_pages: int = 64) -> list[int]:
        """NUMA node of pages sampled evenly over the segment (for reports / tests)."""
        from .. import _native

        return list(_native.runtime().memory_nodes(self.address, self.n * self.row_bytes, max_pages))

    def close(self, unlink: bool | None = None) -> None:
        if self._shm is None:
            return
        unlink = self._owner if unlink is None else unlink
        try:
            self._shm.close()
        except BufferError:
            pass
        if unlink:
            try:
                self._shm.unlink()
            except FileNotFoundError:
                pass
        self._shm = None


def numa_local_source(base_name: str, n: int, sample_shape, dtype, env, fill=None):
    """One replica of a node-shared array per NUMA node that hosts a GPU of this node's ranks.

    The reference keeps each GPU group's data in node-local shared memory (its MPI shared windows,
    reference ddl/ddl_env.py:58-73, ddl/connection.py:88-139). A single node-wide segment read
    by every GPU (the zero-copy gather, ``zerocopy.py``) would make the GPUs of the other socket
    read across the inter-socket link. Here the ranks whose GPUs sit on the same NUMA node share
    one replica ``{base_name}_numa{node}``: its lowest local rank creates it, binds it to the node
    (``bind_to_node``, before any page is touched) and fills it with ``fill(tensor)``; the others
    attach after a barrier on ``env.control_group``. Returns ``(source, node, created)``; the
    caller closes the source (the creator unlinks) after every rank of the node is done with it.
    Collective: every rank of the job calls it (the barrier is on the control group).
    """
    import torch.distributed as dist

    from ..utils.numa import gpu_numa_node

    lw = max(1, int(getattr(env, "local_world_size", 1) or 1))
    lr = int(getattr(env, "local_rank", 0) or 0)
    nodes = [gpu_numa_node(i) for i in range(lw)]
    node = nodes[lr] if lr < len(nodes) else None
    tag = "any" if node is None else str(node)
    creator = nodes.index(node) == lr
    src = SharedArraySource(f"{base_name}_numa{tag}", n, sample_shape, dtype, create=creator)
    try:
        if creator:
            if node is not None:
                src.bind_to_node(node)
            if fill is not None:
                fill(src.tensor())
        if getattr(env, "world_size", 1) > 1 and dist.is_initialized():
            dist.barrier(group=env.control_group)
    except BaseException:
        src.close()
        raise
    return src, node, creator


class NpyMemmapSource:
    """Read-only memory-mapped ``.npy`` dataset [N, ...] (page cache shared across processes)."""

    def __init__(self, path: str):
        self.path = os.path.abspath(path)
        arr = np.load(self.path, mmap_mode="r")
        self.n = arr.shape[0]
        self.sample_shape = tuple(arr.shape[1:])
        self.dtype = _dtypes.to_torch_dtype(arr.dtype)
        self.row_bytes = int(math.prod(self.sample_shape)) * arr.dtype.itemsize
        self._arr = None

    def __getstate__(self):
        return {"path": self.path}

    def __setstate__(self, st):
        self.__init__(st["path"])

    def _a(self) -> np.ndarray:
        if self._arr is None:
            self._arr = np.load(self.path, mmap_mode="r")
        return self._arr

    @property
    def address(self) -> int:
        a = self._a()
        if not a.flags["C_CONTIGUOUS"]:  # pragma: no cover
            raise ValueError("memmap must be C-contiguous")
        return int(a.ctypes.data)

    def gather(self, indices: np.ndarray, dst_address: int, n_threads: int = 4) -> None:
        from .. import _native

        _native.runtime().gather_rows(dst_address, self.address, self.row_bytes,
                                      np.ascontiguousarray(indices, np.int64), self.n, n_threads)


class FileRowsSource:
    """File-backed dataset [N, *sample_shape] read with native coalesced ``pread``.

    For datasets larger than host RAM, or when 8 ranks x P producers should not
    thrash a node's page cache: producers pull exactly the rows of their next
    batch from disk into the pinned slot (``gather``), with ``direct=True``
    bypassing the page cache (O_DIRECT; falls back to buffered reads on
    filesystems that refuse it, e.g. tmpfs). The reference keeps each
    producer's whole shard in memory (tests/run_ddl.py:80-104).

    ``from_npy`` parses an ``.npy`` header (no pickles: object dtypes are
    refused) and reads the C-order payload in place.
    """

    def __init__(self, path: str, sample_shape, dtype, n: int | None = None, offset: int = 0, direct: bool = False):
        self.path = os.path.abspath(path)
        self.sample_shape = tuple(int(d) for d in sample_shape)
        self.dtype = _dtypes.to_torch_dtype(dtype)
        self.offset = int(offset)
        self.direct = bool(direct)
        self.row_bytes = int(math.prod(self.sample_shape)) * _dtypes.itemsize(self.dtype)
        size = os.path.getsize(self.path)
        avail = (size - self.offset) // self.row_bytes if self.row_bytes else 0
        self.n = int(avail if n is None else n)
        if self.n > avail:
            raise ValueError(f"{path}: {self.n} rows of {self.row_bytes} B do not fit in {size - self.offset} B")
        self._f = None

    @classmethod
    def from_npy(cls, path: str, direct: bool = False) -> FileRowsSource:
        from numpy.lib import format as npf

        with open(path, "rb") as fh:
            version = npf.read_magic(fh)
            read_header = npf.read_array_header_1_0 if version == (1, 0) else npf.read_array_header_2_0
            shape, fortran, dtype = read_header(fh)  # parses the header literal only; never unpickles
            offset = fh.tell()
        if fortran or dtype.hasobject or len(shape) < 1:
            raise ValueError(f"{path}: need a C-order, non-object array with a leading sample axis")
        return cls(path, shape[1:], dtype, n=shape[0], offset=offset, direct=direct)

    def __getstate__(self):
        st = dict(self.__dict__)
        st["_f"] = None  # reopened lazily in the producer
        return st

    def _file(self):
        if self._f is None or self._f.closed:
            from .. import _native

            self._f = _native.runtime().RowsFile(self.path, self.direct)
        return self._f

    def gather(self, indices: np.ndarray, dst_address: int, n_threads: int = 4) -> None:
        idx = np.ascontiguousarray(indices, np.int64)
        if idx.size and (idx.min() < 0 or idx.max() >= self.n):
            raise IndexError(f"row index out of range [0, {self.n})")
        self._file().read_rows(self.offset, self.row_bytes, idx, dst_address, self.direct, n_threads)

    def read_range(self, row0: int, n_rows: int, dst_address: int, n_threads: int = 4) -> None:
        self.gather(np.arange(row0, row0 + n_rows, dtype=np.int64), dst_address, n_threads)

    def close(self) -> None:
        if self._f is not None:
            self._f.close()
            self._f = None


class SyntheticTokens:
    """Deterministic ragged token sequences: sequence i has length in [min_len, max_len]."""

    def __init__(self, n: int, min_len: int = 128, max_len: int = 4096, vocab: int = 50257, seed: int = 0):
        self.n, self.min_len, self.max_len, self.vocab, self.seed = n, min_len, max_len, vocab, seed
        rng = np.random.default_rng(seed)
        self.lengths = rng.integers(min_len, max_len + 1, size=n).astype(np.int64)
        self.offsets = np.concatenate([[0], np.cumsum(self.lengths)]).astype(np.int64)

    def sequence(self, i: int) -> np.ndarray:
        rng = np.random.default_rng([self.seed, i])
        return rng.integers(0, self.vocab, size=int(self.lengths[i]), dtype=np.int32)

    def batch(self, indices) -> tuple[np.ndarray, np.ndarray]:
        seqs = [self.sequence(int(i)) for i in indices]
        offs = np.concatenate([[0], np.cumsum([len(s) for s in seqs])]).astype(np.int64)
        return (np.concatenate(seqs) if seqs else np.zeros(0, np.int32)), offs


class MapDatasetSource:
    """Any map-style dataset (``len(ds)``, ``ds[i]`` -- a ``torch.utils.data.Dataset``) as a row source
    for ``IndexedProducer``: the drop-in path for existing Dataset code.

    A sample is a tensor / ndarray / number, or a flat tuple, list or dict of them, with the same
    shapes and dtypes for every index (probed on ``ds[0]``). Each sample is packed into one byte row:
    field k at a 16-byte aligned offset. The loader turns a batch of rows back into the sample's
    structure with zero-copy typed views (``DistributedDataLoader`` does it by itself when the
    producers announce ``fields``): a tuple / dict / tensor of ``[B, *shape]`` tensors, like torch's
    ``default_collate``.

    Producers call ``ds[i]`` for their share of each global batch (``EpochOrder``: the world-size-
    invariant order, checkpointable by global batch), on ``n_threads`` threads per producer; the
    dataset object is pickled to every producer process, as with torch DataLoader workers.
    """

    ALIGN = 16

    def __init__(self, dataset, name: str | None = None):
        self.dataset = dataset
        self.n = len(dataset)
        if self.n < 1:
            raise ValueError("MapDatasetSource: empty dataset")
        self.name = name or type(dataset).__name__
        self.kind, fields = self._describe(dataset[0])
        off, self.fields = 0, []
        for key, shape, dt, nbytes in fields:
            self.fields.append((key, tuple(shape), dt, off, nbytes))
            off += -(-nbytes // self.ALIGN) * self.ALIGN
        self.row_bytes = max(self.ALIGN, off)
        self.sample_shape = (self.row_bytes,)
        self.dtype = torch.uint8
        self._torch_dtypes = None

    # sample structure ---------------------------------------------------------------------------
    @staticmethod
    def _leaf(v):
        """(shape, dtype name, bytes as a flat uint8 ndarray) of one field value."""
        if isinstance(v, torch.Tensor):
            t = v.detach().cpu().contiguous()
            return tuple(t.shape), str(t.dtype).replace("torch.", ""), t.view(-1).view(torch.uint8).numpy()
        if isinstance(v, (bool, np.bool_)):
            a = np.asarray(v, dtype=np.bool_)
        elif isinstance(v, int):
            a = np.asarray(v, dtype=np.int64)
        elif isinstance(v, float):
            a = np.asarray(v, dtype=np.float64)
        elif isinstance(v, (np.ndarray, np.generic)):
            a = np.asarray(v)  # (np.ascontiguousarray would turn a 0-d scalar into shape (1,))
            if not a.flags.c_contiguous:
                a = a.copy()
        else:
            raise TypeError(f"MapDatasetSource: unsupported field type {type(v).__name__} (tensor, ndarray or number)")
        if a.dtype == object:
            raise TypeError("MapDatasetSource: object arrays are not fixed-size")
        return tuple(a.shape), str(a.dtype), a.reshape(-1).view(np.uint8)

    def _items(self, sample):
        if isinstance(sample, dict):
            return "dict", list(sample.items())
        if isinstance(sample, (tuple, list)):
            return "tuple", list(enumerate(sample))
        return "tensor", [(0, sample)]

    def _describe(self, sample):
        kind, items = self._items(sample)
        fields = []
        for key, v in items:
            if isinstance(v, (dict, tuple, list)):
                raise TypeError("MapDatasetSource: nested samples are not supported; flatten them")
            shape, dt, raw = self._leaf(v)
            _field_dtype(dt)  # a dtype the loader can view
            fields.append((key, shape, dt, int(raw.nbytes)))
        return kind, fields

    # producer side --------------------------------------------------------------------------------
    def _spans(self, i: int, dst_row: int, spans: tuple[list, list, list, list]) -> None:
        """Call ``ds[i]``, check it against sample 0, and append one (dst, src, bytes) copy span per field;
        the source buffers are kept alive in ``spans[0]`` until the copies have run."""
        keep, dsts, srcs, sizes = spans
        kind, items = self._items(self.dataset[i])
        if len(items) != len(self.fields):
            raise ValueError(f"MapDatasetSource: sample {i} has {len(items)} fields, sample 0 has {len(self.fields)}")
        tdts = self._torch_dtypes
        if tdts is None:  # per-field torch dtypes (None: not a torch dtype name), for the fast tensor check
            tdts = self._torch_dtypes = [getattr(torch, dt, None) for _, _, dt, _, _ in self.fields]
        for (key, v), (key0, shape, dt, off, nbytes), tdt in zip(items, self.fields, tdts):
            if type(v) is torch.Tensor and v.dtype is tdt and key == key0 and v.shape == shape \
                    and v.device.type == "cpu" and v.is_contiguous():
                buf, ptr = v, v.data_ptr()  # the common case: a contiguous CPU tensor, checked without strings
            else:
                if isinstance(v, torch.Tensor):
                    t = v.detach()
                    if t.device.type != "cpu" or not t.is_contiguous():
                        t = t.cpu().contiguous()
                    s_, d, ptr, buf = tuple(t.shape), str(t.dtype).replace("torch.", ""), t.data_ptr(), t
                else:
                    s_, d, buf = self._leaf(v)
                    ptr = buf.ctypes.data
                if key != key0 or s_ != shape or d != dt:
                    raise ValueError(f"MapDatasetSource: sample {i} field {key!r} is {d}{list(s_)}, "
                                     f"sample 0 has {dt}{list(shape)}")
            if nbytes == 0:  # empty field: nothing to copy (its data pointer may be null)
                continue
            keep.append(buf)
            dsts.append(dst_row + off)
            srcs.append(ptr)
            sizes.append(nbytes)

    def gather(self, indices: np.ndarray, dst_address: int, n_threads: int = 4) -> None:
        """Rows for ``indices`` into the pinned slot at ``dst_address``. ``ds[i]`` runs in this thread
        (Python threads only contended for the GIL: 53 -> 68-79 us per 150 KB sample at 2-4 threads),
        then every field's bytes move in one native ``copy_spans`` call on the runtime's ``n_threads``
        worker pool without the GIL. Copying each field from Python instead (a torch / numpy copy per
        field) cost 85 us per sample on the build host."""
        from .. import _native

        idx = np.asarray(indices, dtype=np.int64)
        if len(idx) == 0:
            return
        ids = idx.tolist()
        rb = self.row_bytes
        parts = [([], [], [], [])]
        for j, i in enumerate(ids):
            self._spans(i, dst_address + j * rb, parts[0])
        dsts = np.fromiter((d for p in parts for d in p[1]), dtype=np.uint64)
        srcs = np.fromiter((x for p in parts for x in p[2]), dtype=np.uint64)
        sizes = np.fromiter((z for p in parts for z in p[3]), dtype=np.uint64)
        _native.runtime().copy_spans(dsts, srcs, sizes, max(1, n_threads))
        del parts  # the source buffers may go now


def _field_dtype(name: str) -> torch.dtype:
    dt = getattr(torch, name, None)
    if not isinstance(dt, torch.dtype):
        raise TypeError(f"MapDatasetSource: dtype {name!r} has no torch equivalent")
    return dt


def unpack_fields(rows: torch.Tensor, fields, kind: str):
    """Typed zero-copy views of a batch of packed rows [B, row_bytes] (``MapDatasetSource`` layout):
    a tensor, a tuple or a dict of ``[B, *shape]`` tensors, following the dataset's sample structure."""
    B = rows.shape[0]
    out = []
    for key, shape, dt, off, nbytes in fields:
        tdt = _field_dtype(dt)
        v = rows[:, off:off + nbytes]
        if tdt != torch.uint8:
            v = v.view(tdt)
        out.append((key, v.view((B,) + tuple(shape))))
    if kind == "tensor":
        return out[0][1]
    if kind == "dict":
        return {k: v for k, v in out}
    return tuple(v for _, v in out)
