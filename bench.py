#!/usr/bin/env python3
"""Benchmark of the MultiDismantler inference rollout on MI355X (BASELINE.json metric:
node-removals/sec (whole node) + AUDC match, 2-layer synthetic N=1000).

A "step" is one complete rollout (MvcEnv.s0 + the GetSol loop until terminal) of the
workload's graphs, inputs already resident in HBM.  The headline workload (BASELINE configs[1])
is one 2-layer GMM graph, N=1000, generator seed 0 (mdcommunity_amd.gmm reproduces the
reference's U/GMM.py graph for that seed), unit-cost checkpoint g0.5 iter 100000; with
--gpus N every rank (one process per GPU) runs its own replica (weak scaling).

The same run also measures the batched path (configs[2]: 256 graphs N=1000 per GPU, seeds
sharded contiguously over ranks, per-graph AUDC gathered over RCCL) as the "batch" object.

Prints one JSON line (rank 0) with the roofline of the rollout kernel (HIP-event device time
of every launch in the timed region, algorithmic flops / bytes from the device's own
per-prediction trace) and the CPU baseline (the oracle, a reference-shaped
restatement, timed on this host's cores on a bounded sample).
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
PEAK_FP32_TFLOPS = 157.3   # MI355X dense FP32 matrix peak (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E peak
CKPT = "U/models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt"


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
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--batch-graphs", type=int, default=256, help="graphs per GPU of the batch object (0: skip)")
    ap.add_argument("--batch-steps", type=int, default=2)
    ap.add_argument("--degree-steps", type=int, default=3, help="timed degree-cost rollouts (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-per-step", action="store_true", help="skip the per-step-protocol comparison rollouts")
    ap.add_argument("--cpu-sample-seconds", type=float, default=12.0)
    return ap.parse_args()


def cpu_baseline(edges, n, seconds):
    """The oracle (reference-shaped CPU restatement: Python featurisation + torch-CPU
    forward + networkx MCC each step) timed on this host: whole rollouts of the bench graph
    until `seconds` have passed."""
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


def audc_of(ranks, max_rank, n):
    s = 0.0
    for r in ranks:
        s += -1 * (-float(r) / (int(max_rank) * float(n)))  # U/mvc_env.py:86,133-137
    return s


def run_steps(eng, steps):
    """`steps` timed rollouts (reset = MvcEnv.s0 in md_env_kernel, then the device rollout
    loop in md_rollout_kernel).  Returns the HIP-event device time and launch count of the
    rollout kernel, the same for the s0 launches, removals and the last outputs."""
    kernel_ms, launches, removals, s0_ms = 0.0, 0, 0, 0.0
    last = None
    for _ in range(steps):
        mr = eng.reset()
        ms, _ = eng.last_timing()
        s0_ms += ms
        outs = eng.rollout()
        ms, nl = eng.last_timing()
        kernel_ms += ms
        launches += nl
        removals += sum(len(o[0]) for o in outs)
        last = (mr, outs)
    return kernel_ms, launches, removals, last, s0_ms


def trace_work(eng, n_graphs):
    flops, nbytes, preds = 0.0, 0.0, 0
    for gidx in range(n_graphs):
        tr = eng.trace(gidx)
        for n_t, a0, a1 in zip(tr["n_live"], tr["m0"], tr["m1"]):
            flops += step_flops(float(n_t), float(a0), float(a1))
            nbytes += step_bytes(float(n_t), float(a0), float(a1))
            preds += 1
    return flops, nbytes, preds


def roofline(flops_per_step, bytes_per_step, kernel_ms_per_step, launches_per_step, traffic):
    t = kernel_ms_per_step * 1e-3
    achieved = flops_per_step / t / 1e12 if t > 0 else 0.0
    return {
        "bound": "mfma",
        "achieved": achieved,
        "peak": PEAK_FP32_TFLOPS,
        "unit": "TFLOP/s",
        "frac": achieved / PEAK_FP32_TFLOPS,
        "traffic": traffic,
        "algorithmic_flops_per_launch": flops_per_step / max(1e-9, launches_per_step),
        "algorithmic_bytes_per_launch": bytes_per_step / max(1e-9, launches_per_step),
        "kernel_ms_per_launch": kernel_ms_per_step / max(1e-9, launches_per_step),
        "hbm_achieved_GBs": bytes_per_step / t / 1e9 if t > 0 else 0.0,
        "hbm_frac": (bytes_per_step / t / 1e9) / PEAK_HBM_GBS if t > 0 else 0.0,
    }


def degree_object(args, edges):
    """Degree-cost rollouts (D/MultiDismantler_torch.py GetSol, D/mvc_env.py reward) of the
    seed-`seed` GMM graph: removals/s over `degree_steps` timed rollouts, the weighted score with the
    reference's expression, and the match against the reference's own run of this graph
    (tests/golden/rollout_deg_gmm1000_s0.npz, made by tests/golden/make_golden_degree.py)."""
    from mdcommunity_amd import _lib, engine, graph as mgraph
    # the D/ variant's own GMM generator (D/GMM.py, unlike U/GMM.py) made the reference's graph
    # for this seed; its edges are the fixture
    gpath = os.path.join(ROOT, "tests", "golden", "rollout_deg_gmm1000_s%d.npz" % args.seed)
    z = np.load(gpath) if args.n == 1000 and os.path.exists(gpath) else None
    if z is not None:
        edges = (z["edges0"], z["edges1"])
    g = mgraph.Graph_test.from_edges(args.n, edges[0], edges[1])
    mgraph.ensure_degree_weights(g)
    eng = _lib.Engine(engine.load_weights(engine.DEFAULT_DEGREE), cost_mode=_lib.MD_COST_DEGREE)
    eng.load_graphs([(args.n,) + edges], node_w=mgraph.node_weight_array([g]))
    run_steps(eng, 1)
    t0 = time.perf_counter()
    kms, nl, rem, last, _ = run_steps(eng, args.degree_steps)
    dt = time.perf_counter() - t0
    mr, outs = last
    seq, ranks = outs[0]
    eng.close()
    tw0, tw1 = sum(g.weights[0].values()), sum(g.weights[1].values())
    score = 0.0
    for a, r in zip(seq.tolist(), ranks.tolist()):  # D/mvc_env.py:127-134
        score += -1 * (-int(r) / int(mr[0]) * (g.weights[0][int(a)] / tw0 + g.weights[1][int(a)] / tw1) / 2.0)
    out = {"workload": "degree-cost rollout, 2-layer GMM graph N=%d seed %d (%s), checkpoint D/models/"
                       "nrange_30_50_iter_100000.ckpt" % (args.n, args.seed, "D/GMM.py, fixture" if z is not None
                                                          else "U/GMM.py"),
           "value": rem / dt, "unit": "removals/s", "steps": args.degree_steps,
           "ms_per_step": dt / args.degree_steps * 1e3, "kernel_ms_per_step": kms / args.degree_steps,
           "removals_per_step": rem / args.degree_steps, "score": score}
    if z is not None:
        amb = np.flatnonzero((z["step_stats"][:, 3] > 1) | (z["step_gap"] < 1e-6))
        k = int(amb[0]) if amb.size else len(z["seq"])
        out.update(score_match=abs(score - float(z["score"])) <= 1e-12 * max(1.0, abs(float(z["score"]))),
                   seq_match=seq.tolist()[:k] == z["seq"].tolist()[:k], seq_checked_steps=k,
                   reference_cpu_seconds_per_rollout=float(z["ref_seconds"]))
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    dev = None
    if world > 1:
        import torch
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        dist = tdist
        dev = "cuda"

    from mdcommunity_amd import _lib, engine, gmm, parallel

    weights = engine.load_weights(engine.DEFAULT_UNIT)
    eng = _lib.Engine(weights, device=local if world > 1 else 0)
    edges = gmm.gmm_pair(args.n, seed=args.seed)
    eng.load_graphs([(args.n,) + edges])

    def sync():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    # ---------------- headline: single graph rollouts (configs[1]); --steps 0 skips it (profiling
    # the batch object alone)
    kernel_ms, launches, removals, elapsed, s0_ms = 0.0, 0, 0, 1e-9, 0.0
    flops = nbytes = 0.0
    preds, audc, seq = 0, None, np.zeros(0, np.int32)
    if args.steps > 0:
        run_steps(eng, max(0, args.warmup))
        sync()
        t0 = time.perf_counter()
        kernel_ms, launches, removals, last, s0_ms = run_steps(eng, args.steps)
        sync()
        elapsed = time.perf_counter() - t0
        flops, nbytes, preds = trace_work(eng, 1)
        mr, outs = last
        seq, ranks = outs[0]
        audc = audc_of(ranks, mr[0], args.n)
    # host-buffer-inclusive rate (edge lists uploaded over PCIe by md_load_graphs, sequences
    # read back): reported beside `value`, never as it (Measurement)
    pcie_rate = None
    if args.steps > 0:
        tp = time.perf_counter()
        prem = 0
        for _ in range(3):
            eng.load_graphs([(args.n,) + edges])
            eng.reset()
            prem += sum(len(o[0]) for o in eng.rollout())
        pcie_rate = prem / (time.perf_counter() - tp)
    # the same rollouts with the K2 end-game shortcut off (every removal step runs its forward
    # pass and, on a tie, its own host hand-shake; MD_VARIANT bit 2048): reported beside `value`
    per_step_rate = per_step_same = None
    if args.steps > 0 and not args.no_per_step:
        old_v = os.environ.get("MD_VARIANT")
        os.environ["MD_VARIANT"] = str(int(old_v or "0") | 2048)
        try:
            peng = _lib.Engine(weights, device=local if world > 1 else 0)
        finally:
            if old_v is None:
                del os.environ["MD_VARIANT"]
            else:
                os.environ["MD_VARIANT"] = old_v
        peng.load_graphs([(args.n,) + edges])
        run_steps(peng, 1)
        tp = time.perf_counter()
        _, _, prem, plast, _ = run_steps(peng, args.steps)
        per_step_rate = prem / (time.perf_counter() - tp)
        per_step_same = plast[1][0][0].tolist() == seq.tolist()
        peng.close()
    tot_removals, max_elapsed = removals, elapsed
    if dist is not None:
        max_elapsed = parallel.max_over_ranks(dist, elapsed, dev)
        tot_removals = parallel.sum_over_ranks(dist, removals, dev)

    # ---------------- batch object (configs[2] per GPU; configs[4] shape across ranks)
    batch = None
    if args.batch_graphs > 0:
        total = args.batch_graphs * world
        lo, hi = parallel.shard(total, rank, world)
        bgraphs = [(args.n,) + gmm.gmm_pair(args.n, seed=s) for s in range(lo, hi)]
        beng = _lib.Engine(weights, device=local if world > 1 else 0)
        beng.load_graphs(bgraphs)
        run_steps(beng, 1)
        sync()
        tb = time.perf_counter()
        bk_ms, bl, brem, blast, _ = run_steps(beng, args.batch_steps)
        sync()
        belapsed = time.perf_counter() - tb
        bflops, bbytes, _ = trace_work(beng, len(bgraphs))
        bmr, bouts = blast
        baudc = [audc_of(r, m, n) for (n, _, _), m, (_, r) in zip(bgraphs, bmr, bouts)]
        brem_per_graph = [len(s) for s, _ in bouts]
        if dist is not None:
            baudc, brem_per_graph = parallel.gather_results(dist, baudc, brem_per_graph, dev)  # RCCL over xGMI
            belapsed = parallel.max_over_ranks(dist, belapsed, dev)
            brem = parallel.sum_over_ranks(dist, brem, dev)
        beng.close()
        batch = {
            "workload": "%d 2-layer GMM graphs N=%d (seeds 0..%d, %d per GPU), full rollouts per step"
                        % (total, args.n, total - 1, args.batch_graphs),
            "value": brem / belapsed,
            "unit": "removals/s",
            "steps": args.batch_steps,
            "ms_per_step": belapsed / args.batch_steps * 1e3,
            "removals_per_step": brem / args.batch_steps,
            "audc_mean": float(np.mean(baudc)),
            "graphs": len(baudc),
            "roofline": roofline(bflops, bbytes, bk_ms / args.batch_steps, bl / args.batch_steps, None),
        }

    # ---------------- degree-cost variant (configs[3] shape: the D/ agent on a synthetic N=1000
    # multiplex, the GMM seed-0 graph; real testReal inputs are absent), single graph, rank 0
    degree = None
    if rank == 0 and args.degree_steps > 0:
        degree = degree_object(args, edges)

    if rank == 0:
        golden = None
        gpath = os.path.join(ROOT, "tests", "golden", f"rollout_gmm1000_s{args.seed}.npz")
        if args.n == 1000 and os.path.exists(gpath):
            z = np.load(gpath)
            amb = np.flatnonzero((z["step_stats"][:, 3] > 1) | (z["step_gap"] < 1e-6))
            # the reference's own pick is a tie / near-tie from step k on (tests/test_gpu_parity.py)
            k = int(amb[0]) if amb.size else len(z["seq"])
            golden = dict(audc=float(z["score"]), seq=z["seq"].tolist(), k=k)
        traffic = None
        tfile = os.path.join(ROOT, "profiles", "traffic_r01.json")
        if os.path.exists(tfile):
            with open(tfile) as f:
                tj = json.load(f)
            traffic = tj.get("hbm_bytes_per_launch")
            # measured HBM bytes per md_queue_kernel launch of the 256-graph batch (PMC passes)
            if batch is not None and args.batch_graphs == 256 and "batch" in tj:
                batch["roofline"]["traffic"] = tj["batch"].get("hbm_bytes_per_launch")
        line = {
            "metric": METRIC,
            "value": tot_removals / max_elapsed,
            "unit": "removals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": max_elapsed / max(1, args.steps) * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (GMM generator = reference U/GMM.py streams; random seed graphs)",
            "config": {
                "workload": "single 2-layer GMM graph N=%d seed %d, unit cost, full rollout per step "
                            "(one replica per GPU)" % (args.n, args.seed),
                "n_nodes": args.n,
                "removals_per_step": tot_removals / max(1, args.steps),
                "parallelism": "replicas x%d" % world,
                "checkpoint": CKPT,
            },
            "audc": audc,
            "audc_match": (audc == golden["audc"]) if golden and audc is not None else None,
            "seq_match": (seq.tolist()[:golden["k"]] == golden["seq"][:golden["k"]]) if golden and audc is not None else None,
            "seq_checked_steps": golden["k"] if golden else None,
            "seq_full_match": (seq.tolist() == golden["seq"]) if golden and audc is not None else None,
            "kernel_ms_per_step": kernel_ms / max(1, args.steps),
            "s0_kernel_ms_per_step": s0_ms / max(1, args.steps),
            "launches_per_step": launches / max(1, args.steps),
            "predictions_per_step": preds,
            "pcie_inclusive_value": pcie_rate,
            # K2 end-game picks run in one hand-shake; the same rollouts with one
            # forward pass per removal step, same sequence checked:
            "per_step_protocol_value": per_step_rate,
            "per_step_protocol_same_sequence": per_step_same,
            "roofline": roofline(flops, nbytes, kernel_ms / max(1, args.steps), launches / max(1, args.steps), traffic),
            "batch": batch,
            "degree": degree,
        }
        if world == 1 and not args.no_cpu_baseline and args.steps > 0:
            cb = cpu_baseline(edges, args.n, args.cpu_sample_seconds)
            line["cpu_baseline"] = cb
            line["vs_cpu_baseline"] = line["value"] / cb["value"]
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
