#!/usr/bin/env python3
"""Pure-Python share of the consumer's per-batch host cost: the native-dispatch path (``dl[i]`` +
``mark``) with the BatchEngine replaced by a stub that returns instantly (no HIP calls). Subtracting
this from ``tools/loader_host_cost.py``'s thread CPU time leaves the engine + HIP share. Runs on
the CPU (thread producers); on the GPU box it measures that host's Python speed.
"""
import collections, time, os, sys
os.environ["DDL_DEVICE"]="cpu"; os.environ["DDL_PRODUCER_MODE"]="thread"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import ddl_amd
from ddl_amd import Marker
from ddl_amd.models import PointwiseProducer
from ddl_amd.utils import streams

class Stub:
    def __init__(s): s.n=0; s.slots_left=10**9; s.inline=True
    def get(s,w,local,bpw,nxt,handle,t):
        s.n+=1; return (s.n-1,-1,(0,0,0,0))
    def release(s,w): return 0
    def acquire(s,w,t): return (0,-1)
    def provide(s,p): pass
with ddl_amd.start(n_producers=3) as (env, conn):
    dl = ddl_amd.DistributedDataLoader(PointwiseProducer(n_timesteps=10, host_shuffle=False), 4096, conn, 10**6, env=env, seed=1)
    torch._C._cuda_getCurrentStream = lambda i: 1
    class FakeStream:
        cuda_stream=0
    streams.current = lambda i: FakeStream()
    blk = torch.empty(1)
    class Blk:
        def record_stream(self, s): pass
    b = Blk()
    N=200000
    dl._engine = Stub(); dl._eng_slots = collections.deque((i, (blk,), b) for i in range(N+10))
    dl._eng_budget=0; dl._eng_streams={}; dl._eng_rec=(None,None); dl._eng_window=None; dl._eng_tokens=None
    dl._engine_provide = lambda: None
    def batches():
        while True:
            for i in range(len(dl)):
                yield dl[i]
                dl.mark(Marker.END_OF_BATCH)
            dl.mark(Marker.END_OF_EPOCH)
    it = batches()
    import cProfile, pstats
    for _ in range(1000): next(it)
    c0=time.thread_time()
    for _ in range(N - 30000): next(it)
    c1=time.thread_time()
    print('{"python_us_per_batch": %.3f}' % (1e6*(c1-c0)/(N - 30000)), flush=True)
    pr=cProfile.Profile(); pr.enable()
    for _ in range(20000): next(it)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(15)
    sys.stdout.flush()
    dl._engine=None
    os._exit(0)
