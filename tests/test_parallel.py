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


def _bench(*extra):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--cpu-dry-run", "--n", "40", "--steps", "1",
           "--warmup", "0", "--batch-steps", "1", "--degree-steps", "0", "--no-cpu-baseline", "--real-steps", "0"] + list(extra)
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    out = subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=240, env=env).stdout
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.timeout(300)
def test_bench_launcher_world2_gathers_like_one_process():
    """`bench.py --gpus 2` (no torchrun) launches two rank processes itself; they shard the
    batch seeds, gather per-graph AUDC and removal counts and take the max time over ranks —
    through the bench's own launcher, rank body, shard and gather code (gloo + the host stub
    engine in place of the device).  The gathered lists must equal a one-process run."""
    two = _bench("--gpus", "2", "--batch-graphs", "3", "--c5-graphs", "5")
    one = _bench("--gpus", "1", "--batch-graphs", "6", "--c5-graphs", "5")
    assert two["n_gpus"] == 2 and two["rccl_world"] == 2 and two["backend"] == "gloo"
    assert one["n_gpus"] == 1 and one["rccl_world"] == 1
    b2, b1 = two["batch"], one["batch"]
    assert b2["graphs"] == 6 and b2["graphs_rank0"] == 3
    assert b2["audc_all"] == b1["audc_all"] and b2["removals_all"] == b1["removals_all"]
    assert b2["removals_per_step"] == sum(b1["removals_all"])
    # weak scaling of the headline: each rank runs its own replica, and the line says so
    assert two["config"]["removals_per_step"] == 2 * one["config"]["removals_per_step"]
    assert two["scaling"] == "weak" and "replica" in two["value_note"] and "c5" in two["value_note"]
    # C5 (configs[4]) is strong-scaled: the same graphs at both world sizes, split over the ranks
    c2, c1 = two["c5"], one["c5"]
    assert c2["scaling"] == c1["scaling"] == "strong"
    assert c2["graphs"] == c1["graphs"] == 5 and c2["graphs_rank0"] == 3 and c1["graphs_rank0"] == 5
    assert c2["gather_complete"] and c1["gather_complete"]
    assert c2["audc_all"] == c1["audc_all"] and c2["removals_all"] == c1["removals_all"]
    assert c2["removals_per_step"] == c1["removals_per_step"]
    assert two["dist_check"] == {"backend": "gloo", "world": 2, "gather_ok": True}


@pytest.mark.timeout(300)
def test_batch_cpu_baseline_pool():
    """The batch CPU baseline's process pool (P x 1-thread oracle rollouts over the batch's
    first seeds) runs and reports what it sampled."""
    import bench
    cb = bench.cpu_baseline_batch(60, 2, graphs_per_proc=1)
    assert cb["cores"] == 2 and cb["kind"] == "port" and cb["value"] > 0
    assert "2 GMM N=60 graphs" in cb["sample"]


@pytest.mark.timeout(300)
def test_bench_launcher_fails_fast_when_a_rank_dies():
    """A rank that dies must not leave the others blocked in a collective until the driver's time
    limit: the launcher polls every rank, stops the siblings on the first non-zero exit and
    returns that status (rank 1 exits with 3 right after init; rank 0 would wait at its first
    barrier for the process group's 600 s timeout)."""
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--cpu-dry-run", "--gpus", "2", "--fail-rank", "1",
           "--n", "40", "--steps", "1", "--warmup", "0", "--batch-graphs", "2", "--c5-graphs", "0",
           "--degree-steps", "0", "--no-cpu-baseline", "--real-steps", "0"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    t0 = time.time()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    dt = time.time() - t0
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert "rank 1 exited with status 3" in r.stderr
    assert dt < 120, dt
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_available_cpus_and_roofline():
    import numpy as np
    import bench
    n, how = bench.available_cpus()
    assert 1 <= n <= (os.cpu_count() or n) and "affinity" in how
    # per-prediction max of the two roofs, bound = the dominating roof
    F = np.array([157.3e12 * 1e-6, 157.3e12 * 4e-6])   # 1 us, 4 us of MFMA time
    B = np.array([8e12 * 3e-6, 8e12 * 1e-6])           # 3 us, 1 us of HBM time
    rl = bench.roofline(F, B, kernel_ms_per_step=0.014, launches_per_step=1, traffic=None)
    assert abs(rl["roofline_ms_per_step"] - 0.007) < 1e-12
    assert abs(rl["roofline_time_frac"] - 0.5) < 1e-9
    assert rl["bound"] == "mfma" and rl["unit"] == "TFLOP/s"   # 4 us of MFMA-bound terms vs 3 us HBM
    assert abs(rl["frac"] - 5e-6 / 14e-6) < 1e-9 and abs(rl["hbm_frac"] - 4e-6 / 14e-6) < 1e-9
    assert rl["predictions_hbm_bound"] == 1 and rl["predictions_mfma_bound"] == 1
