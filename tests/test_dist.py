"""Multi-process (gloo, world_size 2, CPU) test of the N>1 path's host logic: S range sharding
(hwbloomradixjoin_amd.shard_range, used by bench.py), R replication and the count reduction.
Each rank joins (R, its S shard) with the oracle standing in for its GPU; the reduced counts must
equal the single-process counts (and the reference golden)."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
GOLD = json.load(open(os.path.join(HERE, "golden", "survey_counts.json")))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    import hwbloomradixjoin_amd as hw
    from oracle import pyoracle as orc
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = GOLD["F3_grid"]
    R = hw.generate_host(g["r"], 2, g["r"], g["r"], 1.0, 1, 2)  # replicated
    lo, hi = hw.shard_range(g["s"], rank, world)
    S = hw.generate_host(g["s"], 2, 2**31 - 1, g["r"], g["q"], 2, 2)[lo:hi]  # this rank's shard
    res, filt, _ = orc.bpro(R, S, 2, 1, g["m"], 1, 1024)
    t = torch.tensor([filt, res, hi - lo], dtype=torch.int64)
    dist.all_reduce(t)
    q.put((rank, [int(x) for x in t.tolist()]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_counts_reduce_to_golden(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    g = GOLD["F3_grid"]
    for _, (filt, res, n) in outs:
        assert n == g["s"]
        assert (filt, res) == (g["rows"]["1024"][0], g["results"])


def test_shard_range_covers_exactly():
    import sys
    sys.path.insert(0, ROOT)
    import hwbloomradixjoin_amd as hw
    for n in (0, 1, 7, 1024000000, 1024000001):
        for world in (1, 2, 3, 4, 8):
            spans = [hw.shard_range(n, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def _xchg_worker(rank, world, port, q):
    """The partitioned join's exchange callbacks (pjoin.TorchExchange, include/hwbrj.h
    hwbrj_exchange_t) over gloo on CPU buffers, called through the C function pointers the
    library calls."""
    import ctypes
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from hwbloomradixjoin_amd import pjoin
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = pjoin.TorchExchange("cpu")
    c = x._c
    W, n = world, 3
    # alltoall_u64: block j of rank r's send goes to rank j
    send = (ctypes.c_uint64 * (W * n))(*[1000 * rank + 10 * j + i for j in range(W) for i in range(n)])
    recv = (ctypes.c_uint64 * (W * n))()
    assert c.alltoall_u64(None, send, recv, n) == 0
    a2a = list(recv)
    # alltoallv: rank r sends (j + 1) * (r + 1) bytes of value 16 r + j to rank j (consecutive blocks)
    sb = [(j + 1) * (rank + 1) for j in range(W)]
    so = [sum(sb[:j]) for j in range(W)]
    rb = [(rank + 1) * (j + 1) for j in range(W)]
    ro = [sum(rb[:j]) for j in range(W)]
    ps = c.buffer(None, 1, sum(sb))
    pr = c.buffer(None, 2, sum(rb))
    assert ps and pr
    payload = bytes(b for j in range(W) for b in [16 * rank + j] * sb[j])
    ctypes.memmove(ps, payload, len(payload))
    U = ctypes.c_uint64 * W
    assert c.alltoallv(None, 1, U(*so), U(*sb), 2, U(*ro), U(*rb)) == 0
    got = ctypes.string_at(pr, sum(rb))
    # allgather in place: rank r's slice [r nb, (r + 1) nb) of slot 3, nb bytes each
    nb = 8
    pg = c.buffer(None, 3, W * nb)
    ctypes.memmove(pg + rank * nb, bytes([100 + rank] * nb), nb)
    assert c.allgather(None, 3, nb) == 0
    gat = ctypes.string_at(pg, W * nb)
    q.put((rank, a2a, got, gat, x.error))
    dist.destroy_process_group()


def test_partitioned_exchange_callbacks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_xchg_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict((o[0], o[1:]) for o in [q.get(timeout=300) for _ in range(world)])
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    n = 3
    for r in range(world):
        a2a, got, gat, err = outs[r]
        assert err is None
        assert a2a == [1000 * j + 10 * r + i for j in range(world) for i in range(n)]
        assert got == bytes(b for j in range(world) for b in [16 * j + r] * ((r + 1) * (j + 1)))
        assert gat == bytes(b for j in range(world) for b in [100 + j] * 8)
