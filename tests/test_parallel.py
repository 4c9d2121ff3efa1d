"""Multi-process sharding + AUDC gather on CPU (gloo, world size 2): the same helpers the
multi-GPU bench uses over RCCL.  Per-graph AUDC comes from the oracle's reference-shaped
rollout of small graphs, so the gathered list must equal a single-process run."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from mdcommunity_amd import gmm, parallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _graphs(n_graphs):
    return [(40,) + gmm.er_pair(40, seed1=2 * i + 1, seed2=2 * i + 2) for i in range(n_graphs)]


def _audc_of(graph):
    import torch
    torch.set_num_threads(1)
    from oracle import refenv, refmodel
    from mdcommunity_amd import engine
    w = refmodel.RefWeights.load(engine.DEFAULT_UNIT)
    n, e0, e1 = graph
    g = refenv.RefGraph(n, e0, e1)
    if g.max_rank <= 1:
        return 0.0, 0
    score, seq, _, _ = refenv.rollout(w, g)
    return score, len(seq)


def _worker(rank, world, port, n_graphs, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    graphs = _graphs(n_graphs)
    lo, hi = parallel.shard(n_graphs, rank, world)
    res = [_audc_of(graphs[i]) for i in range(lo, hi)]
    audc, rem = parallel.gather_results(dist, [a for a, _ in res], [r for _, r in res])
    tot = parallel.sum_over_ranks(dist, sum(r for _, r in res))
    mx = parallel.max_over_ranks(dist, float(rank))
    if rank == 0:
        q.put((audc, rem, tot, mx))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_covers_everything_once():
    for n in (0, 1, 5, 7, 512, 4096):
        for world in (1, 2, 3, 8):
            blocks = [parallel.shard(n, r, world) for r in range(world)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(b[1] == c[0] for b, c in zip(blocks, blocks[1:]))
            sizes = [b[1] - b[0] for b in blocks]
            assert max(sizes) - min(sizes) <= 1


@pytest.mark.timeout(300)
def test_gloo_world2_gather_equals_single_process():
    n_graphs = 5  # uneven split: 3 + 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_graphs, q)) for r in range(2)]
    for p in procs:
        p.start()
    audc, rem, tot, mx = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    ref = [_audc_of(g) for g in _graphs(n_graphs)]
    assert audc == [a for a, _ in ref]  # bit-identical float64
    assert rem == [r for _, r in ref]
    assert tot == sum(rem)
    assert mx == 1.0
