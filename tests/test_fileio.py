"""Native file row reader (csrc/runtime/fileio.cpp) and FileRowsSource."""

import os

import numpy as np
import pytest
import torch

from ddl_amd import _native
from ddl_amd.models import FileRowsSource


@pytest.fixture
def npy(tmp_path):
    rng = np.random.default_rng(0)
    arr = rng.integers(0, 1 << 30, size=(3001, 37), dtype=np.int32)  # 148 B rows: unaligned to 4 KiB
    path = tmp_path / "rows.npy"
    np.save(path, arr)
    return path, arr


@pytest.mark.parametrize("direct", [False, True])
@pytest.mark.parametrize("threads", [1, 4])
def test_read_rows_random_sorted_duplicates(npy, direct, threads):
    path, arr = npy
    src = FileRowsSource.from_npy(str(path), direct=direct)
    assert (src.n, src.sample_shape, src.dtype) == (3001, (37,), torch.int32)
    rng = np.random.default_rng(1)
    for idx in (rng.permutation(3001)[:777], np.arange(100, 2900), np.array([5, 5, 6, 7, 7, 3000, 0]),
                np.arange(3001)[::-1].copy()):
        out = np.empty((len(idx), 37), np.int32)
        src.gather(idx, out.ctypes.data, threads)
        assert np.array_equal(out, arr[idx])
    src.close()


def test_direct_io_on_a_real_filesystem(tmp_path):
    # tmp_path may be tmpfs (O_DIRECT refused -> buffered fallback); also try the repo's filesystem
    d = os.path.join(os.path.dirname(__file__), "..", "build")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"direct_{os.getpid()}.bin")
    data = np.random.default_rng(2).integers(0, 255, size=(513, 4099), dtype=np.uint8)
    data.tofile(path)
    try:
        src = FileRowsSource(path, (4099,), "uint8", direct=True)
        idx = np.random.default_rng(3).permutation(513)
        out = np.empty_like(data)
        src.gather(idx, out.ctypes.data, 3)
        assert np.array_equal(out, data[idx])
        src.read_range(10, 20, out.ctypes.data, 2)
        assert np.array_equal(out[:20], data[10:30])
        src.close()
    finally:
        os.unlink(path)


def test_bounds_and_header_checks(npy, tmp_path):
    path, arr = npy
    src = FileRowsSource.from_npy(str(path))
    out = np.empty((1, 37), np.int32)
    with pytest.raises(IndexError):
        src.gather(np.array([3001]), out.ctypes.data)
    f = _native.runtime().RowsFile(str(path))
    with pytest.raises(IndexError):  # std::out_of_range: past EOF at the native layer
        f.read_rows(0, 148, np.array([10 ** 9]), out.ctypes.data)
    f.close()
    with pytest.raises(ValueError):
        FileRowsSource(str(path), (37,), "int32", n=10 ** 6)
    obj = tmp_path / "obj.npy"
    np.save(obj, np.array([{"a": 1}], dtype=object), allow_pickle=True)
    with pytest.raises(ValueError):
        FileRowsSource.from_npy(str(obj))


def test_file_source_indexed_loader(npy):
    import ddl_amd
    from ddl_amd.models import IndexedProducer
    from ddl_amd.permutation import EpochOrder

    path, arr = npy
    src = FileRowsSource.from_npy(str(path))
    with ddl_amd.start(n_producers=2, device="cpu") as (env, conn):
        dl = ddl_amd.DistributedDataLoader(IndexedProducer(src, 100, seed=4), 100, conn, 2, env=env, auto_mark=True,
                                           order=ddl_amd.OrderSpec(mode="indexed"))
        got = [torch.cat([b[0].cpu() for b in dl]).numpy() for _ in range(2)]
    for e in range(2):
        ref = EpochOrder(3001, 100, 4).perm(e).full()[:3000]
        assert np.array_equal(got[e].reshape(-1, 37), arr[ref])


def test_file_source_resident_loader(npy):
    from ddl_amd.permutation import EpochOrder
    from ddl_amd.resident import ResidentGlobalLoader

    path, arr = npy
    src = FileRowsSource.from_npy(str(path))
    dl = ResidentGlobalLoader(src, 64, seed=9, n_epochs=1, chunk_bytes=4096, device="cpu")
    got = torch.cat([b.clone() for b in dl]).numpy()
    ref = EpochOrder(3001, 64, 9).perm(0).full()[: len(got)]
    assert np.array_equal(got, arr[ref])
