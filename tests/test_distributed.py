"""Multi-rank path on CPU (gloo, world_size 2): shard coverage and the max/sum reductions that
bench.py uses for the whole-job number. No GPU and no data-path collective involved."""
import os
import socket

import pytest
import torch.multiprocessing as mp

import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    g = shard.Group()
    lo, hi = shard.shard_range(n_total, world, rank)
    g.barrier()
    mx = g.max(float(rank + 1) * 1.5)
    sm = g.sum(float(hi - lo))
    q.put((rank, lo, hi, mx, sm))
    g.close()


@pytest.mark.parametrize("world,n_total", [(2, 4096), (2, 1_048_577), (3, 10)])
def test_gloo_shards_and_reductions(world, n_total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    covered = []
    for rank, lo, hi, mx, sm in res:
        covered.extend(range(lo, hi))
        assert mx == world * 1.5
        assert sm == n_total
    assert covered == list(range(n_total))


def test_shard_range_edge_cases():
    assert shard.shard_range(0, 4, 2) == (0, 0)
    assert shard.shard_range(5, 8, 7) == (5, 5)
    assert [shard.shard_range(8, 8, r) for r in range(8)] == [(r, r + 1) for r in range(8)]
