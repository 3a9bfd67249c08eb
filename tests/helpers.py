"""Producer functions used by the tests (importable by spawned producer workers)."""

import numpy as np
import torch

from ddl_amd import DataProducerOnInitReturn, ProducerFunctionSkeleton


class IdProducer(ProducerFunctionSkeleton):
    """int32 window [n, width]: row i = [rank, producer, i, round, i*7+1, ...]."""

    def __init__(self, n=64, width=8, dtype="int32", delay_s=0.0):
        super().__init__()
        self.n, self.width, self.dtype, self.delay_s = n, width, dtype, delay_s

    def on_init(self, *args, **kwargs):
        super().on_init(*args, **kwargs)
        splits = (2, self.width - 2) if self.width > 2 else (self.width,)
        return DataProducerOnInitReturn(self.n, self.width, (self.n, self.width), splits, self.dtype)

    def post_init(self, *args, **kwargs):
        super().post_init(*args, **kwargs)
        self._write(self.my_tensor, 0)

    def _write(self, t, rnd):
        i = torch.arange(self.n, dtype=torch.int64)
        cols = [torch.full_like(i, self.rank_global or 0), torch.full_like(i, self.producer_index or 0), i,
                torch.full_like(i, rnd)]
        while len(cols) < self.width:
            cols.append(i * 7 + len(cols))
        t.copy_(torch.stack(cols[: self.width], 1).to(t.dtype))

    def execute_function(self, *args, **kwargs):
        if self.delay_s:
            import time

            time.sleep(self.delay_s)
        self._write(kwargs["my_tensor"], int(kwargs["round"]))


class FailingProducer(IdProducer):
    def on_init(self, *args, **kwargs):
        raise ValueError("boom in on_init")


class AtexitProducer(IdProducer):
    """IdProducer whose worker registers an atexit handler that writes ``path`` (the quick producer exit
    must still run it) and keeps a file open, written but not flushed (released with the producer object)."""

    def __init__(self, path, **kw):
        super().__init__(**kw)
        self.path = path

    def on_init(self, *args, **kwargs):
        import atexit

        ret = super().on_init(*args, **kwargs)
        idx = kwargs.get("producer_index", 0)
        atexit.register(lambda: open(f"{self.path}.atexit{idx}", "w").write("ran"))
        self._log = open(f"{self.path}.log{idx}", "w")
        self._log.write("buffered")  # flushed only when the file object is released
        return ret
