"""GPU correctness of the batched configurations at full size (BASELINE.json configs[2] and the
per-GPU slice of configs[4]): 256 and 512 two-layer GMM graphs N=1000 (generator seeds 0..255 /
0..511, mdcommunity_amd.gmm = the reference's U/GMM.py streams) rolled out in one md_wq_kernel
launch (one work item per wave, work queue, admission limit, asynchronous tie hand-shakes, K2
end-games) whose tail continues in md_queue_kernel and the lock-step kernel — the launches behind
bench.py's `batch` object.

Every graph's (removal sequence, LMCC trace) must equal its own single-graph rollout
(md_rollout_kernel, dedicated mode), and seeds 0-2 must reproduce the certified sequences and
the reference's bit-exact AUDC (tests/test_certificates.py), as must the seeds of
tests/golden/batch_certs.npz (the longest rollouts among 3..511 and C5 seeds up to 4095, each
certified against the reference itself by tests/golden/make_batch_certs.py).  Per-graph semantics are
single-graph semantics: the reference's Predict batching quirk is not
replicated.
"""
import numpy as np
import pytest

from conftest import load_golden
from test_certificates import PINNED_PREFIX, load_cert
from mdcommunity_amd import _lib, engine, gmm

pytestmark = pytest.mark.gpu

N = 1000


def audc(ranks, max_rank, n):
    s = 0.0
    for r in ranks:
        s += -1 * (-float(r) / (max_rank * float(n)))  # U/mvc_env.py:86,133-137
    return s


@pytest.fixture(scope="module")
def graphs():
    return [(N,) + gmm.gmm_pair(N, seed=s) for s in range(512)]


@pytest.fixture(scope="module")
def weights():
    return engine.load_weights(engine.DEFAULT_UNIT)


@pytest.fixture(scope="module")
def single(graphs, weights):
    """Single-graph rollouts (dedicated mode, one launch per graph) of every seed."""
    eng = _lib.Engine(weights)
    out = []
    for g in graphs:
        eng.load_graphs([g])
        mr = int(eng.reset()[0])
        seq, ranks = eng.rollout()[0]
        out.append((mr, seq.copy(), ranks.copy()))
    eng.close()
    return out


def batch_rollout(weights, graphs):
    eng = _lib.Engine(weights)
    eng.load_graphs(graphs)
    mr = eng.reset().copy()
    outs = eng.rollout()
    _, launches = eng.last_timing()
    eng.close()
    return mr, outs, launches


def check_against_single(mr, outs, single, lo):
    bad = []
    for i, ((seq, ranks), m) in enumerate(zip(outs, mr)):
        smr, sseq, sranks = single[lo + i]
        if int(m) != smr or seq.tolist() != sseq.tolist() or ranks.tolist() != sranks.tolist():
            bad.append(lo + i)
    assert not bad, f"{len(bad)} graphs differ from their single-graph rollout, seeds {bad[:10]}"


def check_goldens(mr, outs):
    for s in range(3):
        name = f"gmm1000_s{s}"
        z, c = load_golden(name), load_cert(name)
        seq, ranks = outs[s]
        assert int(mr[s]) == int(z["max_rank"])
        assert seq.tolist() == c["gpu_seq"].tolist(), name
        k = 0
        while k < min(len(seq), len(z["seq"])) and seq[k] == z["seq"][k]:
            k += 1
        assert k == PINNED_PREFIX[name]
        assert ranks.tolist() == c["ref_ranks_along"].tolist()
        assert audc(ranks, int(mr[s]), N) == float(z["score"])  # bit-exact


def check_batch_certs(mr, outs, lo=0):
    """Seeds beyond 0-2 pinned to the REFERENCE (tests/golden/make_batch_certs.py: the longest
    rollouts of seeds 3..511 and C5 seeds above 511): the batch's sequence is the certified one,
    its LMCC trace is the reference's along it, its AUDC the reference's bit for bit (also the
    reference's own rollout's), every pick inside the reference's near-tie band.  Returns the
    seeds checked."""
    import os
    from conftest import GOLDEN
    with np.load(os.path.join(GOLDEN, "batch_certs.npz")) as z:
        c = {k: z[k] for k in z.files}
    done = []
    for s in c["seeds"].tolist():
        if not lo <= s < lo + len(outs):
            continue
        seq, ranks = outs[s - lo]
        assert int(mr[s - lo]) == int(c[f"s{s}_max_rank"]), s
        assert seq.tolist() == c[f"s{s}_gpu_seq"].tolist(), s
        assert ranks.tolist() == c[f"s{s}_ref_ranks_along"].tolist(), s
        a = audc(ranks, int(mr[s - lo]), N)
        assert a == float(c[f"s{s}_ref_score_along"]) == float(c[f"s{s}_ref_score"]), s  # bit-exact
        assert float(np.max(c[f"s{s}_margin"])) <= 2e-5, s
        done.append(s)
    return done


@pytest.mark.timeout(240)
def test_c3_256_graphs_one_queue_launch_and_tail(graphs, weights, single):
    """configs[2]: 256 graphs in one queue-mode launch (its last <= 8 running graphs continue
    in one lock-step launch, MD_QPARK) == 256 single-graph rollouts."""
    mr, outs, launches = batch_rollout(weights, graphs[:256])
    # the wave-item launch, its last MD_WQPARK running graphs in one per-workgroup queue launch,
    # whose last MD_QPARK continue in one lock-step launch -- fewer when the graphs a launch would
    # park all end (typically by a K2 end-game) at the environment step that would park them,
    # which depends on the order the workgroups reach them
    assert launches in (1, 2, 3)
    assert sum(len(s) for s, _ in outs) > 256 * 20
    check_against_single(mr, outs, single, 0)
    check_goldens(mr, outs)
    assert len(check_batch_certs(mr, outs)) >= 2  # the C3 tail's longest rollouts (seeds 24, 178)


@pytest.mark.timeout(240)
def test_c5_slice_512_graphs_one_queue_launch_and_tail(graphs, weights, single):
    """configs[4]'s per-GPU slice: 512 graphs (G_CAP) in one queue launch and its lock-step
    tail launch == single-graph rollouts."""
    mr, outs, launches = batch_rollout(weights, graphs)
    assert launches in (1, 2, 3)  # (see the C3 test)
    check_against_single(mr, outs, single, 0)
    check_goldens(mr, outs)
    assert len(check_batch_certs(mr, outs)) >= 6


@pytest.mark.timeout(240)
def test_shard_blocks_equal_whole(graphs, weights, single):
    """A contiguous shard (what rank 1 of 2 owns of the 512-graph C5 slice) rolled out alone
    gives the same per-graph results as inside the whole batch: no cross-graph coupling."""
    from mdcommunity_amd import parallel
    lo, hi = parallel.shard(512, 1, 2)
    mr, outs, _ = batch_rollout(weights, graphs[lo:hi])
    check_against_single(mr, outs, single, lo)


@pytest.mark.timeout(240)
def test_tail_handoff_off_same_rollouts(graphs, weights, monkeypatch):
    """MD_QPARK=0 (the whole batch in one queue launch) gives the same rollouts as the default
    hand-off of the last running graphs to the lock-step kernel."""
    monkeypatch.setenv("MD_QPARK", "0")
    mr0, outs0, launches0 = batch_rollout(weights, graphs[:64])
    monkeypatch.setenv("MD_QPARK", "16")
    mr1, outs1, launches1 = batch_rollout(weights, graphs[:64])
    assert launches0 == 1 and launches1 == 2
    assert np.array_equal(mr0, mr1)
    for a, b in zip(outs0, outs1):
        assert a[0].tolist() == b[0].tolist() and a[1].tolist() == b[1].tolist()


@pytest.mark.timeout(240)
def test_multi_node_steps_batch_tail_handoff(graphs, weights, monkeypatch):
    """step > 1 (every prediction through the host selection, several removals per step) on a
    queue-mode batch: the graphs handed to the lock-step kernel at the tail (MD_QPARK) keep
    their rollouts -- same as MD_QPARK=0 and as each graph's own single-graph rollout."""
    sel = graphs[:24]

    def run(park, batch):
        monkeypatch.setenv("MD_QPARK", park)
        eng = _lib.Engine(weights)
        try:
            outs = []
            for gs in ([sel] if batch else [[g] for g in sel]):
                eng.load_graphs(gs)
                eng.reset()
                outs += [(s.tolist(), r.tolist()) for s, r in eng.rollout(step=3)]
            return outs, eng.last_timing()[1]
        finally:
            eng.close()

    parked, launches = run("16", True)
    whole, _ = run("0", True)
    single, _ = run("0", False)
    assert launches >= 2
    assert parked == whole == single


@pytest.mark.timeout(300)
def test_c5_4096_graphs_one_queue_launch(weights, graphs):
    """configs[4] at one GPU: all 4096 graphs (seeds 0..4095, the reference's GMM streams made by
    the device generator in exact mode) in ONE queue launch of QG_CAP graphs (+ its lock-step
    tail launch) -- per graph the same rollouts as 512-graph launches of the same graphs (seeds
    0..511 of which test_c5_slice_512 checks against single-graph rollouts), goldens for 0-2."""
    from mdcommunity_amd import gmm_gpu
    big = [(N,) + tuple(e) for e in gmm_gpu.gmm_pairs(N, range(4096), exact=True, device=0)]
    for s in range(0, 4096, 997):  # the device generator reproduces the host's graphs
        e0, e1 = gmm.gmm_pair(N, seed=s)
        assert np.array_equal(big[s][1], e0) and np.array_equal(big[s][2], e1)
    mr, outs, launches = batch_rollout(weights, big)
    # (+ md_queue_kernel and lock-step tail launches when graphs were parked: with 4096 graphs
    # the last ones often end through their K2 end-game hand-shakes before any is parked; how
    # many launches run depends on the order the workgroups reach them, as in the C3 test)
    assert launches in (1, 2, 3)
    check_goldens(mr, outs)
    assert len(check_batch_certs(mr, outs)) >= 10  # (and the C5 seeds above 511)
    bad = []
    for lo in range(0, 4096, 512):
        cmr, couts, _ = batch_rollout(weights, big[lo:lo + 512])
        for i, ((seq, ranks), m) in enumerate(zip(couts, cmr)):
            o = outs[lo + i]
            if int(m) != int(mr[lo + i]) or seq.tolist() != o[0].tolist() or ranks.tolist() != o[1].tolist():
                bad.append(lo + i)
    assert not bad, f"{len(bad)} graphs differ between the 4096-graph launch and 512-graph launches: {bad[:10]}"


@pytest.mark.timeout(240)
def test_c3_endgame_one_pass_apply_same_states(monkeypatch, graphs, weights):
    """The K2 end-game answers of a wave-item launch (asynchronous hand-shakes; the graph's state
    is staged into the workgroup's LDS for the one-pass apply, md_kernels.hip eg_apply) against
    the per-action loop (MD_EG_APPLY=0): the same rollouts and the same final states (covered
    set, removed edges per layer, counters) for all 256 graphs."""
    def run(apply):
        monkeypatch.setenv("MD_EG_APPLY", apply)
        eng = _lib.Engine(weights)
        try:
            eng.load_graphs(graphs[:256])
            mr = eng.reset().copy()
            outs = [(s.tolist(), r.tolist()) for s, r in eng.rollout()]
            states = []
            for g in range(256):
                cov, r0, r1, cnt = eng.get_state(g)
                states.append((cov.tobytes(), r0.tobytes(), r1.tobytes(), cnt.tolist()))
            return mr.tolist(), outs, states
        finally:
            eng.close()

    one, each = run("1"), run("0")
    assert one[0] == each[0]
    bad = [g for g in range(256) if one[1][g] != each[1][g] or one[2][g] != each[2][g]]
    assert not bad, f"{len(bad)} graphs differ, seeds {bad[:10]}"
