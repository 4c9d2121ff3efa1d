#!/usr/bin/env python3
"""Benchmark of the MultiDismantler inference rollout on MI355X (BASELINE.json metric:
node-removals/sec (whole node) + AUDC match, 2-layer synthetic N=1000).

A "step" is one complete rollout (MvcEnv.s0 + GetSol loop until terminal) of the workload's
graphs, inputs already resident in HBM.  Default workload (BASELINE configs[1]): one
2-layer GMM graph, N=1000, generator seed 0 (mdcommunity_amd.gmm reproduces the reference's
U/GMM.py graph for that seed), unit-cost checkpoint g0.5 iter 100000.  With --gpus N each
rank (one process per GPU) runs its own replica (weak scaling); ``--workload batch``
shards independent graphs over ranks and gathers their AUDC to rank 0 over RCCL.

Prints one JSON line (rank 0) with the roofline of the rollout kernel and the CPU baseline
(the oracle, a reference-shaped restatement, timed on this host's cores).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "node-removals/sec (whole node) + AUDC match, 2-layer synthetic N=1000"
PEAK_FP32_TFLOPS = 157.3   # MI355X FP32 matrix (= vector) peak, MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E peak


def step_flops(n, m0, m1, g=1):
    """Algorithmic FLOPs of one removal step: node-update GEMMs, neighbour
    sums, virtual-node and graph-head work; reference redundancies not counted."""
    return 225600.0 * n + 384.0 * (m0 + m1) + 250000.0 * g


def step_bytes(n, m0, m1):
    """Algorithmic HBM bytes of one removal step."""
    return 1568.0 * (m0 + m1) + 3628.0 * n + 24.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=["single", "batch"], default="single")
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--graphs-per-rank", type=int, default=256)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-seconds", type=float, default=12.0)
    return ap.parse_args()


def cpu_baseline(edges, n, seconds):
    """The oracle (reference-shaped CPU restatement: Python featurisation + torch-CPU
    forward + networkx MCC each step) timed on this host, whole rollouts until ~seconds."""
    import torch
    from oracle import refenv, refmodel
    from mdcommunity_amd import engine
    threads = min(16, os.cpu_count() or 1)  # the reference sets 16 (U/MultiDismantler_torch.py:108)
    torch.set_num_threads(threads)
    w = refmodel.RefWeights.load(engine.DEFAULT_UNIT)
    g = refenv.RefGraph(n, edges[0], edges[1])
    removals, t0, runs, score = 0, time.time(), 0, None
    while True:
        score, seq, _, _ = refenv.rollout(w, g)
        removals += len(seq)
        runs += 1
        if time.time() - t0 >= seconds:
            break
    dt = time.time() - t0
    return dict(value=removals / dt, unit="removals/s", cores=threads, kind="port",
                sample=f"{runs} full oracle rollout(s) of the bench graph (N={n}, {len(seq)} removals each), "
                       f"{dt:.1f} s, torch threads {threads}, {os.cpu_count()} host CPUs visible",
                audc=score)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dist = tdist

    from mdcommunity_amd import _lib, engine, gmm

    weights = engine.load_weights(engine.DEFAULT_UNIT)
    eng = _lib.Engine(weights, device=local if world > 1 else 0)
    if args.workload == "single":
        seeds = [args.seed]
    else:
        seeds = [rank * args.graphs_per_rank + i for i in range(args.graphs_per_rank)]
    graphs = [(args.n,) + gmm.gmm_pair(args.n, seed=s) for s in seeds]
    eng.load_graphs(graphs)

    def one_step():
        mr = eng.reset()
        outs = eng.rollout()
        ms, launches = eng.last_timing()
        return mr, outs, ms, launches

    for _ in range(max(0, args.warmup)):
        one_step()

    def sync():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    sync()
    t0 = time.perf_counter()
    kernel_ms, launches, removals = 0.0, 0, 0
    last = None
    for _ in range(args.steps):
        mr, outs, ms, nl = one_step()
        kernel_ms += ms
        launches += nl
        removals += sum(len(o[0]) for o in outs)
        last = (mr, outs)
    sync()
    elapsed = time.perf_counter() - t0

    # roofline accounting from the device's own per-prediction trace
    flops = 0.0
    nbytes = 0.0
    for gidx in range(len(graphs)):
        tr = eng.trace(gidx)
        for n_t, a0, a1 in zip(tr["n_live"], tr["m0"], tr["m1"]):
            flops += step_flops(float(n_t), float(a0), float(a1))
            nbytes += step_bytes(float(n_t), float(a0), float(a1))
    mr, outs = last
    audc = []
    for (n, _, _), m, (seq, ranks) in zip(graphs, mr, outs):
        s = 0.0
        for r in ranks:
            s += -1 * (-float(r) / (int(m) * float(n)))
        audc.append(s)

    tot_removals = removals
    max_elapsed = elapsed
    all_audc = audc
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        max_elapsed = float(t.item())
        r = torch.tensor([removals], dtype=torch.int64, device="cuda")
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        tot_removals = int(r.item())
        a = torch.tensor(audc, dtype=torch.float64, device="cuda")
        gathered = [torch.zeros_like(a) for _ in range(world)]
        dist.all_gather(gathered, a)  # per-graph AUDC scalars to every rank (RCCL over xGMI)
        all_audc = [float(x) for g in gathered for x in g.tolist()]

    if rank == 0:
        golden = None
        gpath = os.path.join(ROOT, "tests", "golden", f"rollout_gmm1000_s{args.seed}.npz")
        if args.workload == "single" and args.n == 1000 and os.path.exists(gpath):
            z = np.load(gpath)
            golden = dict(audc=float(z["score"]), seq=z["seq"].tolist())
        per_launch_ms = kernel_ms / max(1, launches)
        achieved_tflops = flops / args.steps / (kernel_ms / args.steps * 1e-3) / 1e12 if kernel_ms > 0 else 0.0
        traffic = None
        tfile = os.path.join(ROOT, "profiles", "traffic_r01.json")
        if os.path.exists(tfile):
            with open(tfile) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        line = {
            "metric": METRIC,
            "value": tot_removals / max_elapsed,
            "unit": "removals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": max_elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (GMM generator = reference U/GMM.py streams)",
            "config": {
                "workload": ("single 2-layer GMM graph N=%d seed %d, full rollout per step" % (args.n, args.seed))
                if args.workload == "single" else
                ("%d 2-layer GMM graphs N=%d per GPU, sharded by seed, full rollouts per step"
                 % (args.graphs_per_rank, args.n)),
                "graphs_per_gpu": len(graphs),
                "n_nodes": args.n,
                "removals_per_step": tot_removals / args.steps,
                "parallelism": "replicas" if args.workload == "single" else "graph-sharded dp%d" % world,
                "checkpoint": "U/models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt",
            },
            "audc": all_audc[0] if len(all_audc) == 1 else float(np.mean(all_audc)),
            "audc_match": (abs(all_audc[0] - golden["audc"]) == 0.0) if golden else None,
            "seq_match": (outs[0][0].tolist() == golden["seq"]) if golden else None,
            "kernel_ms_per_step": kernel_ms / args.steps,
            "launches_per_step": launches / args.steps,
            "roofline": {
                "bound": "mfma",
                "achieved": achieved_tflops,
                "peak": PEAK_FP32_TFLOPS,
                "unit": "TFLOP/s",
                "frac": achieved_tflops / PEAK_FP32_TFLOPS,
                "traffic": traffic,
                "algorithmic_bytes_per_launch": nbytes / args.steps / max(1e-9, launches / args.steps),
                "algorithmic_flops_per_launch": flops / args.steps / max(1e-9, launches / args.steps),
                "kernel_ms_per_launch": per_launch_ms,
                "hbm_frac": (nbytes / args.steps / (kernel_ms / args.steps * 1e-3) / 1e9) / PEAK_HBM_GBS
                if kernel_ms > 0 else 0.0,
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(graphs[0][1:], args.n, args.cpu_sample_seconds)
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
