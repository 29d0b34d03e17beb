"""Multi-rank logic on CPU (gloo, world size 2): tile sharding and the per-barcode count
all-reduce (and the optional barcode-adjacency all-reduce) produce the same global counts as
one process over all tiles."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _tile_barcodes(t, R):
    rng = np.random.default_rng(1000 + t)
    return rng.integers(0, R, rng.integers(50, 200)).astype(np.int32)


def _worker(rank, world, port, ntiles, R, out):
    import torch.distributed as dist

    from hiprfish_image_analysis_amd import pipeline as P
    import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    local = np.zeros(R, np.int64)
    for t in P.shard(ntiles, rank, world):
        local += O.barcode_counts(_tile_barcodes(t, R), R)
    c = torch.from_numpy(local)
    P.allreduce_counts(c)
    # the optional adjacency exchange: each tile's (R', R') int64 matrix summed over ranks
    adj = torch.from_numpy(sum((_tile_adjacency(t) for t in P.shard(ntiles, rank, world)), np.zeros((31, 31), np.int64)))
    P.allreduce_adjacency(adj)
    out[rank] = (c.numpy().copy(), adj.numpy().copy())
    dist.destroy_process_group()


def _tile_adjacency(t):
    rng = np.random.default_rng(2000 + t)
    a = rng.integers(0, 5, (31, 31)).astype(np.int64)
    return a + a.T


def test_sharded_counts_allreduce_gloo():
    import multiprocessing as mp
    import sys
    ctx = mp.get_context("spawn")
    R, ntiles, world = 1023, 7, 2
    port = _free_port()
    mgr = ctx.Manager()
    out = mgr.dict()
    procs = [ctx.Process(target=_run, args=(r, world, port, ntiles, R, out, sys.path)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    import oracle as O
    ref = sum(O.barcode_counts(_tile_barcodes(t, R), R) for t in range(ntiles))
    ref_adj = sum(_tile_adjacency(t) for t in range(ntiles))
    for r in range(world):
        assert np.array_equal(out[r][0], ref)
        assert np.array_equal(out[r][1], ref_adj)


def _run(rank, world, port, ntiles, R, out, path):
    import sys
    sys.path[:] = path
    _worker(rank, world, port, ntiles, R, out)


def test_shard_covers_all_tiles():
    from hiprfish_image_analysis_amd import pipeline as P
    for world in (1, 2, 3, 8):
        got = sorted(t for r in range(world) for t in P.shard(20, r, world))
        assert got == list(range(20))
