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


def test_bench_self_launch(monkeypatch):
    """`bench.py --gpus N` without a torch.distributed environment starts torch.distributed.run
    with N ranks as a child process (no exec, nothing on the GPU first) and exits with its
    status; the driver's own torchrun form (WORLD_SIZE set) does not re-launch."""
    import sys as _sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    _sys.path.insert(0, repo)
    import bench

    cmd = bench.launch_cmd(8, ["--gpus", "8", "--steps", "5"], 12345)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    i = cmd.index("--nproc-per-node")
    assert cmd[i + 1] == "8" and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"] and cmd[-5].endswith("bench.py")
    calls = []
    monkeypatch.setattr(bench, "_self_launch", lambda n: calls.append(n) or 3)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(_sys, "argv", ["bench.py", "--gpus", "2", "--steps", "1"])
    with pytest.raises(SystemExit) as ex:
        bench.main()
    assert ex.value.code == 3 and calls == [2]
