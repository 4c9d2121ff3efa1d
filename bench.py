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
                  "mdcommunity_amd/csrc/md_common.h", "mdcommunity_amd/csrc/md_abi.cpp",
                  "mdcommunity_amd/csrc/md_wave.h"]
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
    ap.add_argument("--real-cases", default="degree,unit",
                    help="cases of the testReal-sized object: degree (step 1), unit (stepRatio 0.01)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-per-step", action="store_true", help="skip the per-step-protocol comparison rollouts")
    ap.add_argument("--cpu-sample-seconds", type=float, default=12.0)
    ap.add_argument("--batch-cpu-procs", type=int, default=0,
                    help="processes of the batch CPU baseline (1 torch thread each); 0: the CPUs available to "
                         "this job (available_cpus())")
    ap.add_argument("--c5-graphs", type=int, default=4096,
                    help="graphs of the C5 object (BASELINE configs[4]), strong-scaled: the same graphs at every "
                         "world size, split contiguously over the ranks (0: skip)")
    ap.add_argument("--c5-steps", type=int, default=1)
    ap.add_argument("--c5-shard-graphs", type=int, default=512,
                    help="world size 1: also time one rank's C5 shard at 8 GPUs (4096 / 8 graphs) alone; 0: skip")
    ap.add_argument("--rccl", action="store_true",
                    help="initialise torch.distributed over RCCL (backend nccl) even at world size 1, so the "
                         "collectives of the multi-GPU path run on the GPU")
    ap.add_argument("--dist-timeout", type=float, default=600.0, help="seconds before a collective gives up")
    ap.add_argument("--launch-timeout", type=float, default=0.0,
                    help="launcher: stop every rank after this many seconds (0: no limit)")
    ap.add_argument("--fail-rank", type=int, default=-1, help=argparse.SUPPRESS)  # tests: this rank exits with 3
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
    The launcher itself never touches a GPU; each rank is a fresh interpreter.

    Fail-fast: every rank is polled; the first rank to exit non-zero (or the --launch-timeout
    deadline) terminates the other ranks -- a rank blocked in a collective with a dead peer
    would otherwise wait until the driver's time limit -- and its status is returned."""
    import tempfile
    world = args.gpus
    port = _free_port()
    procs = []
    out_f = tempfile.TemporaryFile()
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=out_f if r == 0 else subprocess.DEVNULL))
    deadline = time.time() + args.launch_timeout if args.launch_timeout > 0 else None
    status = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            r, status = bad[0]
            sys.stderr.write(f"bench launcher: rank {r} exited with status {status}; stopping the other ranks\n")
            break
        if all(c == 0 for c in codes):
            break
        if deadline is not None and time.time() > deadline:
            status = 124
            sys.stderr.write(f"bench launcher: ranks still running after {args.launch_timeout:.0f} s; stopping them\n")
            break
        time.sleep(0.1)
    if status != 0:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_end = time.time() + 10
        for p in procs:
            try:
                p.wait(max(0.1, t_end - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    out_f.seek(0)
    sys.stdout.write(out_f.read().decode())
    sys.stdout.flush()
    return status


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

    def reset_deferred(self):
        pass

    def max_rank(self):
        return self.reset()

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


def available_cpus():
    """(CPUs this job may use, how that was decided): the scheduler affinity mask, capped by a
    cgroup CPU quota (cgroup v2 cpu.max / v1 cfs_quota) and by the host share the environment
    states (OMP_NUM_THREADS) when set -- on a shared GPU box that share, not os.cpu_count(), is
    what the job owns."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        try:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
                q = float(f.read())
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                per = float(f.read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    n = aff if quota is None else max(1, min(aff, int(quota)))
    # a host whose CPUs are shared between jobs states the job's share in OMP_NUM_THREADS (the
    # GPU box sets it to the per-GPU share and asks that worker pools be sized to it)
    share = os.environ.get("OMP_NUM_THREADS", "")
    share = int(share) if share.isdigit() and int(share) > 0 else None
    if share is not None:
        n = min(n, share)
    how = (f"affinity {aff}, cgroup quota {'none' if quota is None else f'{quota:g}'}, OMP_NUM_THREADS share "
           f"{share if share is not None else 'unset'}, os.cpu_count {os.cpu_count()}")
    return n, how


def cpu_baseline_batch(n, procs_wanted=0, graphs_per_proc=8):
    """BASELINE.md §3 / SURVEY.md §8(d): the batch workload on the CPU as P independent
    1-thread oracle processes (embarrassingly parallel over graphs), P = the CPUs available to
    this job (available_cpus) unless `procs_wanted` > 0, on a bounded sample of the batch's
    seeds (the first P * graphs_per_proc, i.e. at least P graphs).  Rate = sample removals / pool
    wall time (each job also builds its graph, ~20 ms against seconds of rollout)."""
    import multiprocessing as mp
    avail, how = available_cpus()
    P = max(1, avail if procs_wanted <= 0 else min(procs_wanted, avail))
    jobs = [(n, s) for s in range(P * graphs_per_proc)]
    ctx = mp.get_context("spawn")  # fresh interpreters: nothing of this GPU process is inherited
    with ctx.Pool(P) as pool:
        pool.map(_oracle_rollout_seed, [(64, 0)] * P, chunksize=1)  # import torch / networkx in every worker
        t0 = time.time()
        res = pool.map(_oracle_rollout_seed, jobs, chunksize=1)
        dt = time.time() - t0
    rem = sum(r[1] for r in res)
    busy = sum(r[2] for r in res)
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")), "")
    except OSError:
        pass
    per_core = rem / busy if busy > 0 else 0.0
    return dict(value=rem / dt, unit="removals/s", cores=P, kind="port",
                per_core_value=per_core,
                # what the same per-core rate would give on every CPU the host shows (not measured:
                # the job owns only `cores` of them)
                full_host_extrapolated_value=per_core * (os.cpu_count() or P),
                sample=f"{len(jobs)} GMM N={n} graphs (batch seeds 0..{len(jobs) - 1}), {rem} removals, one full "
                       f"oracle rollout each on a pool of {P} processes x 1 torch thread, {dt:.1f} s wall; "
                       f"CPUs: {how}; {cpu_model}",
                audc=[r[3] for r in sorted(res)][:3])


# ------------------------------------------------------------------ measurement helpers
def audc_of(ranks, max_rank, n):
    s = 0.0
    for r in ranks:
        s += -1 * (-float(r) / (int(max_rank) * float(n)))  # U/mvc_env.py:86,133-137
    return s


def run_steps(eng, steps):
    """`steps` timed rollouts: the state reset with MvcEnv.s0's prune deferred into the rollout
    launch (md_reset_deferred: the launch's first environment step runs s0), then the device
    rollout loop in md_rollout_kernel / md_queue_kernel.  Returns the HIP-event device time and
    launch count of the rollout launches (s0 included), 0 for separate s0 launches (none),
    removals and the last outputs (max_rank read after the rollout)."""
    kernel_ms, launches, removals, s0_ms = 0.0, 0, 0, 0.0
    last = None
    for _ in range(steps):
        eng.reset_deferred()
        outs = eng.rollout()
        ms, nl = eng.last_timing()
        kernel_ms += ms
        launches += nl
        removals += sum(len(o[0]) for o in outs)
        last = (eng.max_rank(), outs)
    return kernel_ms, launches, removals, last, s0_ms


def trace_work(eng, n_graphs):
    """Per-prediction algorithmic flops and bytes of the last rollout of each
    graph, from the device's own trace (live nodes and residual edges at each prediction)."""
    fl, by = [], []
    for gidx in range(n_graphs):
        tr = eng.trace(gidx)
        for n_t, a0, a1 in zip(tr["n_live"], tr["m0"], tr["m1"]):
            fl.append(step_flops(float(n_t), float(a0), float(a1)))
            by.append(step_bytes(float(n_t), float(a0), float(a1)))
    return np.asarray(fl, np.float64), np.asarray(by, np.float64)


def roofline(F, B, kernel_ms_per_step, launches_per_step, traffic):
    """The kernel's roofline per SURVEY.md §8(d): each prediction t is bound by the larger of
    F_t / FP32-MFMA peak and B_t / HBM peak; the roofline time of a bench step is the sum of
    those, and `bound` names the roof whose terms dominate that sum.  `achieved` / `frac` are
    the algorithmic rate of that roof (bytes/s or flop/s over the measured kernel time);
    `roofline_time_frac` = Σ_t max(F_t/Pf, B_t/Pb) / kernel time; both roofs' fractions are
    reported beside it."""
    t = kernel_ms_per_step * 1e-3
    F = np.asarray(F, np.float64)
    B = np.asarray(B, np.float64)
    tf = F / (PEAK_FP32_TFLOPS * 1e12)
    tb = B / (PEAK_HBM_GBS * 1e9)
    hbm_terms = float(tb[tb >= tf].sum())
    mfma_terms = float(tf[tf > tb].sum())
    t_roof = float(np.maximum(tf, tb).sum())
    Fs, Bs = float(F.sum()), float(B.sum())
    mfma_frac = Fs / t / (PEAK_FP32_TFLOPS * 1e12) if t > 0 else 0.0
    hbm_frac = Bs / t / (PEAK_HBM_GBS * 1e9) if t > 0 else 0.0
    if hbm_terms >= mfma_terms:
        bound, achieved, peak, unit = "hbm", (Bs / t / 1e9 if t > 0 else 0.0), PEAK_HBM_GBS, "GB/s"
    else:
        bound, achieved, peak, unit = "mfma", (Fs / t / 1e12 if t > 0 else 0.0), PEAK_FP32_TFLOPS, "TFLOP/s"
    per = max(1e-9, launches_per_step)
    # one unit throughout: the bench step (== one launch for single-graph rollouts); the
    # per-launch averages follow for the rocprof comparison
    return {
        "bound": bound,
        "achieved": achieved,
        "peak": peak,
        "unit": unit,
        "frac": achieved / peak,
        "traffic": traffic,
        "roofline_time_frac": t_roof / t if t > 0 else 0.0,
        "mfma_frac": mfma_frac,
        "hbm_frac": hbm_frac,
        "mfma_achieved_TFLOPs": Fs / t / 1e12 if t > 0 else 0.0,
        "hbm_achieved_GBs": Bs / t / 1e9 if t > 0 else 0.0,
        "predictions_hbm_bound": int((tb >= tf).sum()),
        "predictions_mfma_bound": int((tf > tb).sum()),
        "roofline_ms_per_step": t_roof * 1e3,
        "per": "bench step",
        "algorithmic_flops_per_step": Fs,
        "algorithmic_bytes_per_step": Bs,
        "kernel_ms_per_step": kernel_ms_per_step,
        "traffic_over_algorithmic_bytes": (traffic / Bs) if (traffic is not None and Bs > 0) else None,
        "launches_per_step": launches_per_step,
        "algorithmic_flops_per_launch": Fs / per,
        "algorithmic_bytes_per_launch": Bs / per,
        "kernel_ms_per_launch": kernel_ms_per_step / per,
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


def apply_traffic(rl, tw, launches_per_step=1.0):
    """Measured HBM traffic of one workload of traffic.json (`tw`: its main kernel's bytes per
    launch, and for queue launches the tail launch's) as bytes per bench step, beside the
    algorithmic bytes of the same step."""
    if not tw:
        return rl
    q, tail = tw.get("hbm_bytes_per_launch"), tw.get("tail_hbm_bytes_per_launch")
    extra = launches_per_step - 1.0
    if q is not None and (extra < 0.5 or tail is not None):
        rl["traffic"] = q + (extra * tail if extra >= 0.5 else 0.0)
        b = rl.get("algorithmic_bytes_per_step") or 0.0
        rl["traffic_over_algorithmic_bytes"] = rl["traffic"] / b if b > 0 else None
    if tw.get("mfma_busy") is not None:
        rl["mfma_busy"] = tw.get("mfma_busy")
    return rl


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
    F, B = trace_work(eng, 1)
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
    traffic, tnote = load_traffic()
    out["roofline"] = apply_traffic(roofline(F, B, kms / args.degree_steps, nl / args.degree_steps, None),
                                    (traffic or {}).get("degree"), nl / args.degree_steps)
    out["roofline"]["traffic_note"] = tnote
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
    traffic, tnote = load_traffic()
    cases = [c.strip() for c in args.real_cases.split(",") if c.strip()]
    for key, cost, ckpt, step, tkey in (("degree_step1", _lib.MD_COST_DEGREE, engine.DEFAULT_DEGREE, 1, "real_degree"),
                                        ("unit_step_ratio_0.01", _lib.MD_COST_UNIT, engine.DEFAULT_UNIT_REAL,
                                         max(int(0.01 * n), 1), "real_unit")):
        if tkey.split("_")[1] not in cases:
            continue
        eng = make_engine(engine.load_weights(ckpt), cost_mode=cost)
        eng.load_graphs([(n, e0, e1)], node_w=mgraph.node_weight_array([g]) if cost == _lib.MD_COST_DEGREE else None)
        eng.reset()
        eng.rollout(step=step)  # warm
        t0 = time.perf_counter()
        kms = 0.0
        rem = 0
        nl = 0
        for _ in range(max(1, args.real_steps)):
            mr = eng.reset()
            seq, ranks = eng.rollout(step=step)[0]
            kms += eng.last_timing()[0]
            nl += eng.last_timing()[1]
            rem += len(seq)
        dt = time.perf_counter() - t0
        F, B = trace_work(eng, 1)
        eng.close()
        k = max(1, args.real_steps)
        out[key] = {"value": rem / dt, "unit": "removals/s", "removals_per_rollout": rem // k, "step": step,
                    "ms_per_rollout": dt / k * 1e3, "kernel_ms_per_rollout": kms / k, "max_rank": int(mr[0]),
                    "predictions_per_rollout": int(len(F)),
                    "audc": audc_of(ranks, mr[0], n) if cost == _lib.MD_COST_UNIT else None}
        # one bench step = one rollout (MvcEnv.s0 by md_reset's own launch, outside the rollout
        # launch and its roofline)
        out[key]["roofline"] = apply_traffic(roofline(F, B, kms / k, nl / k, None), (traffic or {}).get(tkey), nl / k)
        out[key]["roofline"]["traffic_note"] = tnote
    out["reference_note"] = ("the reference's committed homo_genetic_multiplex run (N=18222, unit cost, stepRatio 0): "
                             "2081 removals in 1582.6 s (results/unitcost/MultiDismantler_real/StepRatio_0.0000)")
    return out


# ------------------------------------------------------------------ one rank
def _init_dist(args, world, local):
    """torch.distributed for this rank: RCCL (backend "nccl") with one GPU per rank, gloo for
    the CPU dry run and the shared-GPU rehearsal.  `--rccl` initialises RCCL at world size 1 as
    well (the multi-GPU collectives then run on one GPU).  Returns (dist, device, backend)."""
    import datetime
    if world == 1 and not args.rccl:
        return None, None, None
    import torch.distributed as tdist
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        os.environ["MASTER_PORT"] = str(_free_port())
    os.environ.setdefault("RANK", "0")
    os.environ.setdefault("WORLD_SIZE", str(world))
    timeout = datetime.timedelta(seconds=args.dist_timeout)
    if args.cpu_dry_run or args.rehearse_shared_gpu:
        tdist.init_process_group("gloo", timeout=timeout)
        return tdist, None, "gloo"
    import torch
    torch.cuda.set_device(local)
    tdist.init_process_group("nccl", timeout=timeout, device_id=torch.device("cuda", local))  # RCCL over xGMI
    return tdist, "cuda", "nccl"


def _graph_source(args, gpu):
    """Seed -> (n, edges0, edges1) of the reference's GMM generator, cached per process: the
    device generator in exact mode (gmm_gpu: numpy/random streams on the host, pair loop on the
    GPU; the same graphs as gmm.gmm_pair), or gmm.gmm_pair in the CPU dry run."""
    from mdcommunity_amd import gmm, gmm_gpu
    cache = {}

    def get(seeds):
        seeds = list(seeds)
        need = [s for s in seeds if s not in cache]
        if need:
            if args.cpu_dry_run:
                made = [gmm.gmm_pair(args.n, seed=s) for s in need]
            else:
                made = gmm_gpu.gmm_pairs(args.n, need, exact=True, device=gpu)
            for s, e in zip(need, made):
                cache[s] = (args.n,) + tuple(e)
        return [cache[s] for s in seeds]
    return get


def many_graph_object(args, name, graphs, lo, steps, rank, world, dist, dev, make_engine, weights, sync,
                      parallel):
    """Whole rollouts of this rank's block of graphs (seeds lo..), `steps` timed bench steps after
    one warm-up; per-graph AUDC and removal counts gathered over the ranks (RCCL all-gather);
    rate = removals of all ranks / max rank time.  The roofline is per bench step (every launch
    of the step: queue launches and their tail launches)."""
    eng = make_engine(weights)
    eng.load_graphs(graphs)
    run_steps(eng, 1)
    sync()
    tb = time.perf_counter()
    k_ms, nl, rem, last, _ = run_steps(eng, steps)
    sync()
    elapsed = time.perf_counter() - tb
    F, B = trace_work(eng, len(graphs))
    mr, outs = last
    audc = [audc_of(r, m, n) for (n, _, _), m, (_, r) in zip(graphs, mr, outs)]
    rem_per_graph = [len(sq) for sq, _ in outs]
    gold = golden_checks([outs[s - lo][0] if lo <= s < lo + len(graphs) else None for s in range(3)],
                         [audc[s - lo] if lo <= s < lo + len(graphs) else None for s in range(3)]) \
        if args.n == 1000 else {}
    local_graphs = len(graphs)
    local_value = rem / elapsed
    if dist is not None:
        audc, rem_per_graph = parallel.gather_results(dist, audc, rem_per_graph, dev)  # RCCL over xGMI
        elapsed = parallel.max_over_ranks(dist, elapsed, dev)
        rem = parallel.sum_over_ranks(dist, rem, dev)
    eng.close()
    out = {
        "value": rem / elapsed,
        "unit": "removals/s",
        "steps": steps,
        "ms_per_step": elapsed / steps * 1e3,
        "removals_per_step": rem / steps,
        "audc_mean": float(np.mean(audc)) if audc else None,
        "graphs": len(audc),
        "graphs_rank0": local_graphs,
        "rank0_value": local_value,
        "removals_gathered": int(sum(rem_per_graph)),
        "golden": gold,
        "roofline": roofline(F, B, k_ms / steps, nl / steps, None),
    }
    out["roofline"]["per"] = "bench step (every launch of the step: queue launches + tail launches)"
    out["roofline"]["launches_per_step"] = nl / steps
    return out, audc, rem_per_graph


def rank_main(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rehearse_shared_gpu and world > 1:
        # ranks sharing one GPU: persistent kernels with grid barriers must all be resident at
        # once, so each rank takes only its share of the CUs and no speculative workgroups
        import torch
        ndev = max(1, torch.cuda.device_count())  # counts devices without initialising one
        per_gpu = -(-world // ndev)
        os.environ["MD_MAX_CUS"] = str(256 // per_gpu)
        os.environ["MD_SPEC"] = "0"
    dist, dev, backend = _init_dist(args, world, local)
    if args.fail_rank == rank:
        sys.stderr.write(f"rank {rank}: exiting with status 3 (--fail-rank)\n")
        os._exit(3)

    from mdcommunity_amd import engine, gmm, parallel

    if args.cpu_dry_run:
        gpu = None

        def make_engine(weights, cost_mode=0):
            return DryEngine()
    else:
        from mdcommunity_amd import _lib

        if args.rehearse_shared_gpu:
            import torch
            gpu = local % max(1, torch.cuda.device_count())
        else:
            gpu = local if world > 1 else 0

        def make_engine(weights, cost_mode=_lib.MD_COST_UNIT):
            return _lib.Engine(weights, device=gpu, cost_mode=cost_mode)

    graphs_of = _graph_source(args, gpu)
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
    F = B = np.zeros(0)
    audc, seq = None, np.zeros(0, np.int32)
    if args.steps > 0:
        run_steps(eng, max(0, args.warmup))
        sync()
        t0 = time.perf_counter()
        kernel_ms, launches, removals, last, s0_ms = run_steps(eng, args.steps)
        sync()
        elapsed = time.perf_counter() - t0
        F, B = trace_work(eng, 1)
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

    # ---------------- batch object (configs[2]: batch_graphs per GPU, weak-scaled over ranks)
    batch = None
    if args.batch_graphs > 0:
        total = args.batch_graphs * world
        lo, hi = parallel.shard(total, rank, world)
        batch, baudc, brem = many_graph_object(args, "batch", graphs_of(range(lo, hi)), lo, args.batch_steps, rank,
                                               world, dist, dev, make_engine, weights, sync, parallel)
        batch = dict({"workload": "%d 2-layer GMM graphs N=%d (seeds 0..%d, %d per GPU), full rollouts per step"
                                  % (total, args.n, total - 1, args.batch_graphs)}, **batch)
        batch["scaling"] = "weak"
        if rank == 0 and args.cpu_dry_run:
            batch["audc_all"] = baudc
            batch["removals_all"] = brem

    # ---------------- C5 object (configs[4]): the same c5_graphs graphs at every world size,
    # split contiguously over the ranks (strong scaling); one RCCL all-gather of AUDC + counts
    c5 = None
    if args.c5_graphs > 0:
        lo, hi = parallel.shard(args.c5_graphs, rank, world)
        c5, caudc, crem = many_graph_object(args, "c5", graphs_of(range(lo, hi)), lo, args.c5_steps, rank, world,
                                            dist, dev, make_engine, weights, sync, parallel)
        c5 = dict({"workload": "%d 2-layer GMM graphs N=%d (seeds 0..%d) split over %d GPU(s), %d on rank 0, full "
                               "rollouts per step" % (args.c5_graphs, args.n, args.c5_graphs - 1, world, hi - lo)},
                  **c5)
        c5["scaling"] = "strong"
        c5["gather_complete"] = c5["graphs"] == args.c5_graphs
        if world == 1 and 0 < args.c5_shard_graphs < args.c5_graphs:
            # one rank's shard at 8 GPUs (the first 512 seeds) on this GPU alone: 8 x its rate over
            # the 4096-graph rate predicts the 1 -> 8 strong-scaling ratio of `c5` (the shards'
            # rollout lengths differ a little: seeds are independent draws of one generator)
            sh, _, _ = many_graph_object(args, "c5_shard", graphs_of(range(0, args.c5_shard_graphs)), 0,
                                         max(1, args.c5_steps), rank, world, None, dev, make_engine, weights, sync,
                                         parallel)
            c5["rank_shard_at_8"] = {
                "graphs": args.c5_shard_graphs, "value": sh["value"], "ms_per_step": sh["ms_per_step"],
                "removals_per_step": sh["removals_per_step"], "launches_per_step": sh["roofline"]["launches_per_step"],
                "per_gpu_rate_vs_c5": sh["value"] / c5["value"],
                "predicted_8_gpu_ratio": (args.c5_graphs / args.c5_shard_graphs) * sh["value"] / c5["value"]
                * (c5["removals_per_step"] / (sh["removals_per_step"] * args.c5_graphs / args.c5_shard_graphs)),
                "note": "predicted ratio = (4096-graph time on 1 GPU) / (the 512-graph shard's time on 1 GPU)"}
        if rank == 0 and args.cpu_dry_run:
            c5["audc_all"] = caudc
            c5["removals_all"] = crem

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

    # the collectives themselves, checked: a gather of known per-rank data must come back whole
    dist_check = None
    if dist is not None:
        blk = parallel.shard(64, rank, world)
        ga, gr = parallel.gather_results(dist, [float(i) + 0.5 for i in range(*blk)], list(range(*blk)), dev)
        dist_check = dict(backend=backend, world=dist.get_world_size(),
                          gather_ok=ga == [float(i) + 0.5 for i in range(64)] and gr == list(range(64)))

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
            apply_traffic(batch["roofline"], traffic["batch"], batch["roofline"]["launches_per_step"])
            batch["roofline"]["traffic_note"] = traffic_note
        if c5 is not None and traffic is not None and args.c5_graphs == 4096 and world == 1 and "c5" in traffic:
            apply_traffic(c5["roofline"], traffic["c5"], c5["roofline"]["launches_per_step"])
            c5["roofline"]["traffic_note"] = traffic_note
        have = golden is not None and audc is not None
        k = 0
        if have:
            while k < min(len(seq), len(golden["seq"])) and seq[k] == golden["seq"][k]:
                k += 1
        rl = roofline(F, B, kernel_ms / max(1, args.steps), launches / max(1, args.steps),
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
            "value_note": "replica weak scaling: each rank rolls out its own copy of the headline graph (a "
                          "single-graph rollout does not shard); the strong-scaled north_star figure is "
                          "c5.value (4096 graphs split over the ranks), its 8-GPU prediction "
                          "c5.rank_shard_at_8.predicted_8_gpu_ratio",
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
            "dist_check": dist_check,
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
            "s0": "MvcEnv.s0's prune runs as the rollout launch's first environment step (md_reset_deferred)",
            "launches_per_step": launches / max(1, args.steps),
            "predictions_per_step": int(len(F)),
            "pcie_inclusive_value": pcie_rate,
            # K2 end-game picks run in one hand-shake; the same rollouts with one
            # forward pass per removal step, same sequence checked:
            "per_step_protocol_value": per_step_rate,
            "per_step_protocol_same_sequence": per_step_same,
            "roofline": rl,
            "batch": batch,
            "c5": c5,
            "degree": degree,
            "real_scale": real,
            "kernel_src_hash": kernel_src_hash(),
        }
        line["cpu_baseline"] = None
        if world == 1 and not args.no_cpu_baseline and args.steps > 0 and not args.cpu_dry_run:
            cb = cpu_baseline(edges, args.n, args.cpu_sample_seconds)
            line["cpu_baseline"] = cb
            line["vs_cpu_baseline"] = line["value"] / cb["value"]
            if batch is not None and args.batch_cpu_procs >= 0:
                bcb = cpu_baseline_batch(args.n, args.batch_cpu_procs)
                batch["cpu_baseline"] = bcb
                batch["vs_cpu_baseline"] = batch["value"] / bcb["value"]
                if c5 is not None:
                    c5["vs_cpu_baseline"] = c5["value"] / bcb["value"]
                    c5["cpu_baseline_note"] = "the batch object's CPU pool (same per-graph work, same generator)"
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
