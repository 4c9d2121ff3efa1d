#!/usr/bin/env python3
"""Benchmark of the MultiDismantler inference rollout on MI355X (BASELINE.json metric:
node-removals/sec (whole node) + AUDC match, 2-layer synthetic N=1000).

A "step" is one complete rollout (MvcEnv.s0 + the GetSol loop until terminal) of the
workload's graphs, inputs already resident in HBM.  The headline workload (BASELINE configs[1])
is one 2-layer GMM graph, N=1000, generator seed 0 (mdcommunity_amd.gmm reproduces the
reference's U/GMM.py graph for that seed), unit-cost checkpoint g0.5 iter 100000; with
--gpus N every rank (one process per GPU) runs its own replica (weak scaling).

The same run also measures the batched path (configs[2]: 256 graphs N=1000 per GPU, seeds
sharded contiguously over ranks, per-graph AUDC gathered over RCCL: configs[4]'s shape at
--gpus 8 --batch-graphs 512) as the "batch" object.

Ranks: under torchrun (WORLD_SIZE set) this process is one rank.  Otherwise `--gpus N` (N > 1)
makes this process a launcher: it spawns N rank processes of this script (RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_* set, one GPU each) before anything touches a GPU, relays rank 0's JSON
line and exits with the worst rank's status.  `--cpu-dry-run` runs the same launcher / rank /
shard / gather code on the CPU (gloo, a host stub in place of the device engine): the plumbing
check of tests/test_parallel.py.

Prints one JSON line (rank 0) with the roofline of the rollout kernel (HIP-event device time
of every launch in the timed region, algorithmic flops / bytes from the device's own
per-prediction trace) and the CPU baseline (the oracle, a reference-shaped
restatement, timed on this host's cores on a bounded sample).
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "node-removals/sec (whole node) + AUDC match, 2-layer synthetic N=1000"
PEAK_FP32_TFLOPS = 157.3   # MI355X dense FP32 matrix peak (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E peak
CKPT = "U/models/g0.5_TORCH-Model_GMM_30_50/nrange_30_50_iter_100000.ckpt"
# sources whose hash ties a committed PMC traffic file to the kernels that ran
KERNEL_SOURCES = ["mdcommunity_amd/csrc/md_kernels.hip", "mdcommunity_amd/csrc/md_env.h",
                  "mdcommunity_amd/csrc/md_common.h", "mdcommunity_amd/csrc/md_abi.cpp"]
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")


def step_flops(n, m0, m1, g=1):
    """Algorithmic FLOPs of one removal step: node-update GEMMs, neighbour
    sums, virtual-node and graph-head work; reference redundancies not counted."""
    return 225600.0 * n + 384.0 * (m0 + m1) + 250000.0 * g


def step_bytes(n, m0, m1):
    """Algorithmic HBM bytes of one removal step."""
    return 1568.0 * (m0 + m1) + 3628.0 * n + 24.0


def kernel_src_hash():
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--batch-graphs", type=int, default=256, help="graphs per GPU of the batch object (0: skip)")
    ap.add_argument("--batch-steps", type=int, default=2)
    ap.add_argument("--degree-steps", type=int, default=3, help="timed degree-cost rollouts (0: skip)")
    ap.add_argument("--real-steps", type=int, default=1, help="timed rollouts of the testReal-sized object (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-per-step", action="store_true", help="skip the per-step-protocol comparison rollouts")
    ap.add_argument("--cpu-sample-seconds", type=float, default=12.0)
    ap.add_argument("--batch-cpu-procs", type=int, default=16,
                    help="processes of the batch CPU baseline (1 torch thread each; capped by the CPUs available)")
    ap.add_argument("--cpu-dry-run", action="store_true",
                    help="launcher/rank/gather plumbing on the CPU: gloo backend, host stub engine, no GPU")
    ap.add_argument("--rehearse-shared-gpu", action="store_true",
                    help="N > 1 ranks on fewer GPUs (rank r on GPU r mod the visible count, gloo for the "
                         "collectives): the multi-rank path with the real engine on a one-GPU box; not a "
                         "scaling measurement (the line says so)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ launcher (no GPU calls here)
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args, argv):
    """Spawn `args.gpus` rank processes of this script (one per GPU), relay rank 0's output.
    The launcher itself never touches a GPU; each rank is a fresh interpreter."""
    world = args.gpus
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out, _ = procs[0].communicate()
    codes = [procs[0].returncode] + [p.wait() for p in procs[1:]]
    sys.stdout.write(out.decode())
    sys.stdout.flush()
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


# ------------------------------------------------------------------ host stub engine (--cpu-dry-run)
class DryEngine:
    """Stand-in for mdcommunity_amd._lib.Engine in --cpu-dry-run: same methods, host-only,
    trivially cheap.  It removes nodes in descending total degree (ties: lower id) until no edge
    is left and reports the remaining non-isolated node count as the LMCC trace: deterministic
    per graph, so a sharded run must gather exactly the single-process results.  It is not the
    rollout algorithm; it only drives the bench's rank / shard / gather code."""

    def __init__(self, *a, **k):
        self.graphs = []

    def load_graphs(self, graphs, node_w=None):
        self.graphs = list(graphs)

    def reset(self):
        return np.asarray([max(1, len(np.unique(np.concatenate([e0.reshape(-1), e1.reshape(-1)]))))
                           for _, e0, e1 in self.graphs], np.int32)

    def _one(self, n, e0, e1):
        deg = np.bincount(np.concatenate([e0.reshape(-1), e1.reshape(-1)]), minlength=n)
        order = np.lexsort((np.arange(n), -deg))
        alive = [set(map(tuple, e0.tolist())), set(map(tuple, e1.tolist()))]
        seq, ranks = [], []
        for v in order:
            if not alive[0] and not alive[1]:
                break
            for s in alive:
                s.difference_update([e for e in s if v in e])
            left = {x for s in alive for e in s for x in e}
            seq.append(int(v))
            ranks.append(len(left))
        return np.asarray(seq, np.int32), np.asarray(ranks, np.int32)

    def rollout(self, step=1):
        self._outs = [self._one(*g) for g in self.graphs]
        return self._outs

    def last_timing(self):
        return 0.0, 1

    def trace(self, g):
        k = len(self._outs[g][0])
        z = np.zeros(k, np.int32)
        return dict(n_live=z, m0=z, m1=z)

    def close(self):
        pass


# ------------------------------------------------------------------ CPU baselines (oracle)
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


def _oracle_rollout_seed(job):
    """Pool worker of the batch CPU baseline: one oracle rollout of GMM graph `seed` on one
    torch thread (the graph is generated in the worker, outside the timed region)."""
    n, seed = job
    import torch
    torch.set_num_threads(1)
    from oracle import refenv, refmodel
    from mdcommunity_amd import engine, gmm
    w = refmodel.RefWeights.load(engine.DEFAULT_UNIT)
    e0, e1 = gmm.gmm_pair(n, seed=seed)
    g = refenv.RefGraph(n, e0, e1)
    t0 = time.time()
    score, seq, _, _ = refenv.rollout(w, g) if g.max_rank > 1 else (0.0, [], [], [])
    return seed, len(seq), time.time() - t0, score


def cpu_baseline_batch(n, procs_wanted, graphs_per_proc=2):
    """BASELINE.md §3 / SURVEY.md §8(d): the batch workload on the CPU as P independent
    1-thread oracle processes (embarrassingly parallel over graphs), on a bounded sample of the
    batch's seeds (the first P * graphs_per_proc).  Rate = sample removals / pool wall time."""
    import multiprocessing as mp
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    P = max(1, min(procs_wanted, avail))
    jobs = [(n, s) for s in range(P * graphs_per_proc)]
    ctx = mp.get_context("spawn")  # fresh interpreters: nothing of this GPU process is inherited
    with ctx.Pool(P) as pool:
        pool.map(_oracle_rollout_seed, [(64, 0)] * P)  # import torch / networkx in every worker
        t0 = time.time()
        res = pool.map(_oracle_rollout_seed, jobs, chunksize=1)
        dt = time.time() - t0
    rem = sum(r[1] for r in res)
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    return dict(value=rem / dt, unit="removals/s", cores=P, kind="port",
                sample=f"{len(jobs)} GMM N={n} graphs (batch seeds 0..{len(jobs) - 1}), {rem} removals, one full "
                       f"oracle rollout each on a pool of {P} processes x 1 torch thread, {dt:.1f} s wall; "
                       f"{avail} CPUs available to this process, {os.cpu_count()} visible; {cpu_model}",
                audc=[r[3] for r in sorted(res)][:3])


# ------------------------------------------------------------------ measurement helpers
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


def load_traffic():
    """Measured HBM bytes per launch (PMC passes, scripts/rocprof_summary.py), used only when
    the file was made from the kernel sources that are built now (hash of KERNEL_SOURCES)."""
    if not os.path.exists(TRAFFIC_FILE):
        return None, "absent"
    with open(TRAFFIC_FILE) as f:
        tj = json.load(f)
    if tj.get("src_hash") != kernel_src_hash():
        return None, f"stale (made from sources {tj.get('src_hash')}, built {kernel_src_hash()})"
    return tj, "measured by " + str(tj.get("source", "rocprofv3 PMC passes"))


def golden_checks(seq_by_seed, audc_by_seed):
    """Seeds with reference goldens: AUDC bit-exact against the reference's, sequence equal to
    the certified GPU sequence (tests/test_certificates.py)."""
    out = {}
    for s, (seq, audc) in enumerate(zip(seq_by_seed, audc_by_seed)):
        gp = os.path.join(ROOT, "tests", "golden", f"rollout_gmm1000_s{s}.npz")
        cp = os.path.join(ROOT, "tests", "golden", f"cert_gmm1000_s{s}.npz")
        if seq is None or not os.path.exists(gp) or not os.path.exists(cp):
            continue
        with np.load(gp) as z, np.load(cp) as c:
            out[str(s)] = dict(audc_match=audc == float(z["score"]),
                               certified_seq_match=seq.tolist() == c["gpu_seq"].tolist())
    return out


def degree_object(args, edges, make_engine):
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
    eng = make_engine(engine.load_weights(engine.DEFAULT_DEGREE), cost_mode=_lib.MD_COST_DEGREE)
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
    cp = os.path.join(ROOT, "tests", "golden", "cert_deg_gmm1000_s%d.npz" % args.seed)
    if z is not None:
        out.update(score_match=score == float(z["score"]),
                   reference_cpu_seconds_per_rollout=float(z["ref_seconds"]))
        if os.path.exists(cp):
            with np.load(cp) as c:
                out["certified_seq_match"] = seq.tolist() == c["gpu_seq"].tolist()
    return out


def real_scale_object(args, make_engine, tmpdir):
    """configs[3] at the reference's real sizes: the testReal harness's rollout of an
    N = 18 000 two-layer multiplex shaped like homo_genetic_multiplex (mdcommunity_amd.synth;
    the real files are absent), read by the drop-in reader, environment in HBM: degree cost
    with stepRatio 0 and unit cost with stepRatio 0.01 (180 removals per prediction through the
    host hand-shake).  Timed like `value` (inputs resident in HBM)."""
    from mdcommunity_amd import _lib, agent, engine, graph as mgraph, synth
    n = 18000
    path = os.path.join(tmpdir, "real_like_multiplex.edges")
    synth.write_real_like(path, n, seed=0)
    a = agent.MultiDismantler.__new__(agent.MultiDismantler)
    _, gl = agent.MultiDismantler.read_multiplex(a, path, n)
    e0, e1 = np.asarray(gl[0], np.int32), np.asarray(gl[1], np.int32)
    g = mgraph.Graph_test.from_edges(n, e0, e1)
    mgraph.ensure_degree_weights(g)
    out = {"workload": "testReal-shaped 2-layer multiplex N=%d (mdcommunity_amd.synth seed 0: heavy-tailed, "
                       "%d / %d edges, hubs ~1100), HBM environment" % (n, len(e0), len(e1))}
    for key, cost, ckpt, step in (("degree_step1", _lib.MD_COST_DEGREE, engine.DEFAULT_DEGREE, 1),
                                  ("unit_step_ratio_0.01", _lib.MD_COST_UNIT, engine.DEFAULT_UNIT_REAL,
                                   max(int(0.01 * n), 1))):
        eng = make_engine(engine.load_weights(ckpt), cost_mode=cost)
        eng.load_graphs([(n, e0, e1)], node_w=mgraph.node_weight_array([g]) if cost == _lib.MD_COST_DEGREE else None)
        eng.reset()
        eng.rollout(step=step)  # warm
        t0 = time.perf_counter()
        kms = 0.0
        rem = 0
        for _ in range(max(1, args.real_steps)):
            mr = eng.reset()
            seq, ranks = eng.rollout(step=step)[0]
            kms += eng.last_timing()[0]
            rem += len(seq)
        dt = time.perf_counter() - t0
        eng.close()
        k = max(1, args.real_steps)
        out[key] = {"value": rem / dt, "unit": "removals/s", "removals_per_rollout": rem // k, "step": step,
                    "ms_per_rollout": dt / k * 1e3, "kernel_ms_per_rollout": kms / k, "max_rank": int(mr[0]),
                    "audc": audc_of(ranks, mr[0], n) if cost == _lib.MD_COST_UNIT else None}
    out["reference_note"] = ("the reference's committed homo_genetic_multiplex run (N=18222, unit cost, stepRatio 0): "
                             "2081 removals in 1582.6 s (results/unitcost/MultiDismantler_real/StepRatio_0.0000)")
    return out


# ------------------------------------------------------------------ one rank
def rank_main(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    dev = None
    backend = None
    if world > 1:
        import torch.distributed as tdist
        if args.cpu_dry_run or args.rehearse_shared_gpu:
            backend = "gloo"
            tdist.init_process_group("gloo")
        else:
            import torch
            backend = "nccl"  # RCCL over xGMI on ROCm
            torch.cuda.set_device(local)
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
            dev = "cuda"
        dist = tdist

    from mdcommunity_amd import engine, gmm, gmm_gpu, parallel

    if args.cpu_dry_run:
        def make_engine(weights, cost_mode=0):
            return DryEngine()
    else:
        from mdcommunity_amd import _lib

        if args.rehearse_shared_gpu:
            import torch
            ndev = max(1, torch.cuda.device_count())  # counts devices without initialising one
            gpu = local % ndev
        else:
            gpu = local if world > 1 else 0

        def make_engine(weights, cost_mode=_lib.MD_COST_UNIT):
            return _lib.Engine(weights, device=gpu, cost_mode=cost_mode)

    weights = engine.load_weights(engine.DEFAULT_UNIT)
    eng = make_engine(weights)
    edges = gmm.gmm_pair(args.n, seed=args.seed)
    eng.load_graphs([(args.n,) + edges])

    def sync():
        if dist is not None:
            dist.barrier()
            if dev is not None:
                import torch
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
    if args.steps > 0 and not args.cpu_dry_run:
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
    if args.steps > 0 and not args.no_per_step and not args.cpu_dry_run:
        old_v = os.environ.get("MD_VARIANT")
        os.environ["MD_VARIANT"] = str(int(old_v or "0") | 2048)
        try:
            peng = make_engine(weights)
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
        if args.cpu_dry_run:
            bgraphs = [(args.n,) + gmm.gmm_pair(args.n, seed=s) for s in range(lo, hi)]
        else:
            # the reference's GMM streams, pair loop on the device (gmm_gpu exact mode: the same
            # graphs as gmm.gmm_pair, outside the timed region)
            bgraphs = [(args.n,) + e for e in gmm_gpu.gmm_pairs(args.n, range(lo, hi), exact=True, device=gpu)]
        beng = make_engine(weights)
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
        # reference goldens exist for seeds 0-2 (all on rank 0: contiguous shards)
        gold = golden_checks([bouts[s - lo][0] if lo <= s < hi else None for s in range(3)],
                             [baudc[s - lo] if lo <= s < hi else None for s in range(3)]) if args.n == 1000 else {}
        local_graphs = len(bgraphs)
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
            "graphs_rank0": local_graphs,
            "removals_gathered": int(sum(brem_per_graph)),
            "golden": gold,
            # per batch step: the queue launch and its tail launch (MD_QPARK) together -- the
            # algorithmic work and the measured traffic of the whole batch rollout
            "roofline": roofline(bflops, bbytes, bk_ms / args.batch_steps, 1, None),
        }
        batch["roofline"]["per"] = "batch step (queue launch + tail launch)"
        batch["roofline"]["launches_per_step"] = bl / args.batch_steps
        if rank == 0 and args.cpu_dry_run:
            batch["audc_all"] = baudc
            batch["removals_all"] = brem_per_graph

    # ---------------- degree-cost variant (configs[3] shape: the D/ agent on a synthetic N=1000
    # multiplex, the GMM seed-0 graph; real testReal inputs are absent), single graph, rank 0
    degree = None
    if rank == 0 and args.degree_steps > 0 and not args.cpu_dry_run:
        degree = degree_object(args, edges, make_engine)
    real = None
    if rank == 0 and args.real_steps > 0 and not args.cpu_dry_run:
        import tempfile
        with tempfile.TemporaryDirectory() as td:
            real = real_scale_object(args, make_engine, td)

    if rank == 0:
        golden = None
        gpath = os.path.join(ROOT, "tests", "golden", f"rollout_gmm1000_s{args.seed}.npz")
        cpath = os.path.join(ROOT, "tests", "golden", f"cert_gmm1000_s{args.seed}.npz")
        if args.n == 1000 and os.path.exists(gpath) and os.path.exists(cpath):
            with np.load(gpath) as z, np.load(cpath) as c:
                golden = dict(audc=float(z["score"]), seq=z["seq"].tolist(), cert=c["gpu_seq"].tolist(),
                              prefix=int(c["prefix"]))
        traffic, traffic_note = load_traffic()
        if batch is not None and traffic is not None and args.batch_graphs == 256 and "batch" in traffic:
            tb = traffic["batch"]
            q, tail = tb.get("hbm_bytes_per_launch"), tb.get("tail_hbm_bytes_per_launch")
            extra = batch["roofline"]["launches_per_step"] - 1.0
            if q is not None and (extra < 0.5 or tail is not None):
                batch["roofline"]["traffic"] = q + (extra * tail if extra >= 0.5 else 0.0)
            batch["roofline"]["mfma_busy"] = tb.get("mfma_busy")
        have = golden is not None and audc is not None
        k = 0
        if have:
            while k < min(len(seq), len(golden["seq"])) and seq[k] == golden["seq"][k]:
                k += 1
        rl = roofline(flops, nbytes, kernel_ms / max(1, args.steps), launches / max(1, args.steps),
                      traffic.get("hbm_bytes_per_launch") if traffic else None)
        rl["traffic_note"] = traffic_note
        if traffic:
            rl["mfma_busy"] = traffic.get("mfma_busy")
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
            "rccl_world": dist.get_world_size() if dist is not None else 1,
            "backend": backend,
            # ranks sharing GPUs (--rehearse-shared-gpu): plumbing rehearsal, the value is not a
            # scaling figure
            "rehearsal_shared_gpu": bool(args.rehearse_shared_gpu),
            "audc": audc,
            "audc_match": (audc == golden["audc"]) if have else None,
            # equal to the reference's sequence up to its pinned divergence step (an exact tie or a
            # few-ulp gap of the reference), certified beyond it (tests/test_certificates.py)
            "seq_prefix_match": (k == golden["prefix"]) if have else None,
            "seq_certified_match": (seq.tolist() == golden["cert"]) if have else None,
            "kernel_ms_per_step": kernel_ms / max(1, args.steps),
            "s0_kernel_ms_per_step": s0_ms / max(1, args.steps),
            "launches_per_step": launches / max(1, args.steps),
            "predictions_per_step": preds,
            "pcie_inclusive_value": pcie_rate,
            # K2 end-game picks run in one hand-shake; the same rollouts with one
            # forward pass per removal step, same sequence checked:
            "per_step_protocol_value": per_step_rate,
            "per_step_protocol_same_sequence": per_step_same,
            "roofline": rl,
            "batch": batch,
            "degree": degree,
            "real_scale": real,
            "kernel_src_hash": kernel_src_hash(),
        }
        line["cpu_baseline"] = None
        if world == 1 and not args.no_cpu_baseline and args.steps > 0 and not args.cpu_dry_run:
            cb = cpu_baseline(edges, args.n, args.cpu_sample_seconds)
            line["cpu_baseline"] = cb
            line["vs_cpu_baseline"] = line["value"] / cb["value"]
            if batch is not None and args.batch_cpu_procs > 0:
                bcb = cpu_baseline_batch(args.n, args.batch_cpu_procs)
                batch["cpu_baseline"] = bcb
                batch["vs_cpu_baseline"] = batch["value"] / bcb["value"]
        print(json.dumps(line), flush=True)
    eng.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, argv)
    rank_main(args)
    return 0


if __name__ == "__main__":
    sys.exit(main())
