"""GPU parity: libmdroll.so (gfx950) against the golden vectors of the reference and the
oracle.  Bars (north_star): LMCC sizes and AUDC bit-exact, Q within 1e-5 (absolute) at every
prediction of the reference's rollout, removal sequences equal to the reference's up to a
pinned step where the reference itself is ambiguous (exact tie / few-ulp gap) and certified
beyond it (tests/test_certificates.py)."""
import numpy as np
import pytest

from conftest import GOLDEN, load_golden
from test_certificates import PINNED_PREFIX, load_cert
from mdcommunity_amd import _lib, engine

pytestmark = pytest.mark.gpu

Q_TOL = 1e-5          # north_star: Q-values match within 1e-5
MASK = -(2147483647 / 2)
ALL = ["er100", "gmm200_s7", "er300_dense", "gmm1000_s0", "gmm1000_s1", "gmm1000_s2", "er1000"]


@pytest.fixture(scope="module")
def eng():
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
    yield e
    e.close()


def audc(ranks, max_rank, n):
    s = 0.0
    for r in ranks:
        s += -1 * (-float(r) / (max_rank * float(n)))  # U/mvc_env.py:86,133-137
    return s


@pytest.mark.parametrize("name", ALL)
def test_s0_and_cascade_replay_exact(eng, name):
    """MvcEnv.s0 max_rank and the LMCC after every golden removal are bit-exact."""
    z = load_golden(name)
    n = int(z["n_nodes"])
    eng.load_graphs([(n, z["edges0"], z["edges1"])])
    assert int(eng.reset()[0]) == int(z["max_rank"])
    ranks = []
    for a in z["seq"]:
        lm, term = eng.step(np.array([a], np.int32))
        ranks.append(int(lm[0]))
    assert ranks == z["ranks"].tolist()
    assert bool(term[0])
    _, r0, r1, cnt = eng.get_state(0)
    assert int(r0.sum()) == int(z["removed0"]) and int(r1.sum()) == int(z["removed1"])
    assert cnt[5] == 1


@pytest.mark.parametrize("name", ALL)
def test_q_rows_within_tolerance(eng, name):
    """Q at every prediction of the reference's rollout within 1e-5 of the reference's row."""
    z = load_golden(name)
    n = int(z["n_nodes"])
    eng.load_graphs([(n, z["edges0"], z["edges1"])])
    eng.reset()
    steps = set(int(t) for t in z["q_steps"])
    worst = 0.0
    for t in range(max(steps) + 1):
        if t in steps:
            q, am, nt, gap = eng.predict()
            ref = z["q_rows"][list(z["q_steps"]).index(t)]
            live = ref != MASK
            assert np.array_equal(np.isfinite(q), live), f"live set differs at step {t}"
            d = np.abs(q[live].astype(np.float64) - ref[live])
            worst = max(worst, float(d.max()) if d.size else 0.0)
        eng.step(np.array([z["seq"][t]], np.int32))
    assert worst < Q_TOL, worst


@pytest.mark.parametrize("name", ALL)
def test_rollout_sequence_and_audc(eng, name):
    """The whole GPU sequence is certified against the reference (tests/test_certificates.py):
    it equals the pinned certified sequence, it matches the reference's own sequence up to the
    pinned divergence step, every later pick lies in the reference's near-tie set at that state
    at the GPU's own measured |dQ| there, the LMCC trace equals the reference's along it and
    the AUDC is bit-exact."""
    z, c = load_golden(name), load_cert(name)
    n = int(z["n_nodes"])
    eng.load_graphs([(n, z["edges0"], z["edges1"])])
    mr = int(eng.reset()[0])
    seq, ranks = eng.rollout()[0]
    k = 0
    while k < min(len(seq), len(z["seq"])) and seq[k] == z["seq"][k]:
        k += 1
    assert k == PINNED_PREFIX[name], f"divergence step moved: {k} (pinned {PINNED_PREFIX[name]})"
    assert seq.tolist() == c["gpu_seq"].tolist(), "sequence differs from the certified one"
    assert ranks.tolist() == c["ref_ranks_along"].tolist()
    assert audc(ranks, mr, n) == float(z["score"])  # AUDC bit-exact
    # teacher-forced along its own sequence: |dQ| against the reference's rows at every state,
    # and each pick within the reference's near-tie set at that |dQ|
    eng.reset()
    for t, a in enumerate(seq):
        q = eng.predict()[0].astype(np.float64)
        ref = c["ref_q_along"][t].astype(np.float64)
        live = ~np.isnan(ref)
        assert np.array_equal(np.isfinite(q), live), t
        dq = float(np.max(np.abs(q[live] - ref[live])))
        assert dq < Q_TOL, (t, dq)
        assert np.nanmax(ref) - ref[a] <= dq, (t, np.nanmax(ref) - ref[a], dq)
        eng.step(np.array([a], np.int32))


def test_er100_fully_identical(eng):
    z = load_golden("er100")
    eng.load_graphs([(100, z["edges0"], z["edges1"])])
    eng.reset()
    seq, ranks = eng.rollout()[0]
    assert seq.tolist() == z["seq"].tolist() and ranks.tolist() == z["ranks"].tolist()


def test_mcc_cases_exact(eng):
    """Device MCC on random (graph, covered) states == reference Mcc.MCC results."""
    zc = np.load(f"{GOLDEN}/mcc_cases.npz")
    for i in range(int(zc["n_cases"])):
        n = int(zc[f"c{i}_n"])
        e0, e1 = zc[f"c{i}_e0"].reshape(-1, 2), zc[f"c{i}_e1"].reshape(-1, 2)
        cov = zc[f"c{i}_covered"]
        eng.load_graphs([(n, e0, e1)])
        mr = int(eng.reset()[0])
        if cov.size == 0:
            assert mr == int(zc[f"c{i}_rank"])
            _, r0, r1, _ = eng.get_state(0)
        else:
            c = np.zeros(n, np.uint8)
            c[cov[:-1]] = 1
            eng.set_state(0, c, np.zeros(len(e0), np.uint8), np.zeros(len(e1), np.uint8))
            lm, _ = eng.step(np.array([cov[-1]], np.int32))
            assert int(lm[0]) == int(zc[f"c{i}_rank"]), i
            _, r0, r1, _ = eng.get_state(0)
        assert np.array_equal(r0.astype(np.uint8), zc[f"c{i}_r0"]), i
        assert np.array_equal(r1.astype(np.uint8), zc[f"c{i}_r1"]), i


def test_grid_size_and_batching_do_not_change_results(eng):
    """Results are independent of the grid size and of batching (tile-order reductions)."""
    names = ["gmm1000_s1", "er300_dense", "gmm200_s7"]
    zs = [load_golden(nm) for nm in names]
    graphs = [(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in zs]
    ref = []
    for gsz in (0, 1, 7):
        eng.set_team_size(gsz)
        eng.load_graphs(graphs)
        eng.reset()
        out = [(s.tolist(), r.tolist()) for s, r in eng.rollout()]
        if not ref:
            ref = out
        assert out == ref, f"grid size {gsz} changed the rollouts"
    eng.set_team_size(0)
    for g, r in zip(graphs, ref):
        eng.load_graphs([g])
        eng.reset()
        s1, r1 = eng.rollout()[0]
        assert (s1.tolist(), r1.tolist()) == r


def test_errors_are_reported(eng):
    z = load_golden("er100")
    eng.load_graphs([(100, z["edges0"], z["edges1"])])
    eng.reset()
    a = int(z["seq"][0])
    eng.step(np.array([a], np.int32))
    with pytest.raises(_lib.MDError):
        eng.step(np.array([a], np.int32))  # covering a covered node (U/mvc_env.py:77 assert)
    with pytest.raises(_lib.MDError):
        eng.load_graphs([(3, np.array([[0, 0]]), np.array([[0, 1]]))])  # self-loop


def test_shared_mode_batch_matches_dedicated(eng, monkeypatch):
    """A launch of more than 16 graphs runs through the device work queue, and with MD_VARIANT
    bit 32 in the lock-step shared mode (every workgroup steps graphs, then tiles: the path of
    batches whose graphs exceed the queue's tile field); both equal the dedicated-workgroup path
    of single graphs."""
    names = ["gmm200_s7", "er100", "er300_dense"]
    zs = [load_golden(nm) for nm in names]
    graphs = [(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in zs]
    single = []
    for g in graphs:
        eng.load_graphs([g])
        eng.reset()
        s, r = eng.rollout()[0]
        single.append((s.tolist(), r.tolist()))
    batch = [graphs[i % 3] for i in range(18)]
    eng.load_graphs(batch)
    eng.reset()
    out = eng.rollout()
    for i, (s, r) in enumerate(out):
        assert (s.tolist(), r.tolist()) == single[i % 3], i
    monkeypatch.setenv("MD_VARIANT", "32")
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
    try:
        e.load_graphs(batch)
        e.reset()
        out = e.rollout()
        for i, (s, r) in enumerate(out):
            assert (s.tolist(), r.tolist()) == single[i % 3], ("lock-step shared", i)
    finally:
        e.close()


def test_host_handshake_modes_same_rollouts(monkeypatch):
    """MD_HOST_HANDSHAKE=0 (a tie ends the launch; the host selects and relaunches) gives the
    rollouts of the in-kernel hand-shake: single graphs with ties and end-games, and a 18-graph
    queue-mode batch."""
    names = ["gmm1000_s0", "gmm1000_s1", "er300_dense"]
    graphs = [(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in map(load_golden, names)]
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("MD_HOST_HANDSHAKE", mode)
        e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
        try:
            res = []
            for g in graphs:
                e.load_graphs([g])
                e.reset()
                res += [(s.tolist(), r.tolist()) for s, r in e.rollout()]
            e.load_graphs([graphs[i % 3] for i in range(18)])
            e.reset()
            res += [(s.tolist(), r.tolist()) for s, r in e.rollout()]
            out[mode] = res
        finally:
            e.close()
    assert out["0"] == out["1"]


def test_first_request_same_rollouts(monkeypatch):
    """MD_FIRST_REQ=0 (no speculative request at a rollout's first environment step) gives the
    rollouts of the default degree-ranked first request (single graphs, dataflow and barrier
    modes)."""
    names = ["gmm1000_s0", "gmm200_s7", "er300_dense"]
    graphs = [(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in map(load_golden, names)]
    out = {}
    for fr in ("1", "0"):
        for df in ("1", "0"):
            monkeypatch.setenv("MD_FIRST_REQ", fr)
            monkeypatch.setenv("MD_DF", df)
            e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
            try:
                res = []
                for g in graphs:
                    e.load_graphs([g])
                    for _ in range(2):
                        e.reset_deferred()
                        res += [(s.tolist(), r.tolist()) for s, r in e.rollout()]
                out[(fr, df)] = res
            finally:
                e.close()
    base = out[("1", "1")]
    for k, v in out.items():
        assert v == base, k


@pytest.mark.parametrize("admit,tpi", [(1, 2), (4, 1), (4, 3), (64, 2)])
def test_queue_admission_limit_matches_single(monkeypatch, admit, tpi):
    """Queue mode starts only `admit` graphs and admits the next one whenever a graph stops
    (MD_VARIANT bits 16+ set the limit), and runs `tpi` tiles per work item (bits 9-10):
    every rollout equals its single-graph rollout."""
    names = ["gmm200_s7", "er100", "er300_dense"]
    graphs = [(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in map(load_golden, names)]
    ref = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
    single = []
    try:
        for g in graphs:
            ref.load_graphs([g])
            ref.reset()
            s, r = ref.rollout()[0]
            single.append((s.tolist(), r.tolist()))
    finally:
        ref.close()
    monkeypatch.setenv("MD_VARIANT", str((admit << 16) | (tpi << 9)))
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
    try:
        e.load_graphs([graphs[i % 3] for i in range(18)])
        e.reset()
        out = e.rollout()
        for i, (s, r) in enumerate(out):
            assert (s.tolist(), r.tolist()) == single[i % 3], i
    finally:
        e.close()


def test_global_memory_environment_mode(monkeypatch):
    """Graphs too large for one workgroup's LDS run the environment step on HBM scratch
    (EnvView<true>); MD_VARIANT=64 forces that mode for small graphs: same results."""
    monkeypatch.setenv("MD_VARIANT", "64")
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
    try:
        for name in ("er100", "gmm200_s7", "er300_dense"):
            z = load_golden(name)
            n = int(z["n_nodes"])
            e.load_graphs([(n, z["edges0"], z["edges1"])])
            assert int(e.reset()[0]) == int(z["max_rank"])
            seq, ranks = e.rollout()[0]
            assert seq.tolist() == load_cert(name)["gpu_seq"].tolist()
            assert audc(ranks, int(z["max_rank"]), n) == float(z["score"])
    finally:
        e.close()


def test_precomputed_first_layer_tables(monkeypatch):
    """Unit cost: the first-layer tables of every dmax precomputed at load (md_h0_kernel)
    give the same rollouts and Q as rebuilding them in phase A (MD_H0G=0), also after the
    weights are replaced on a loaded context."""
    w_a = engine.load_weights(engine.DEFAULT_UNIT)
    w_b = engine.load_weights(engine.DEFAULT_UNIT_REAL)
    z = load_golden("gmm1000_s2")
    g = (int(z["n_nodes"]), z["edges0"], z["edges1"])
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("MD_H0G", mode)
        e = _lib.Engine(w_b)
        try:
            e.load_graphs([g])
            e.set_weights(w_a)
            e.reset()
            q, _, _, _ = e.predict()
            out[mode] = (q.copy(), [(s.tolist(), r.tolist()) for s, r in e.rollout()])
            e.set_weights(w_b)
            e.reset()
            out[mode] += ([(s.tolist(), r.tolist()) for s, r in e.rollout()],)
        finally:
            e.close()
    assert np.array_equal(out["1"][0], out["0"][0])
    assert out["1"][1] == out["0"][1] and out["1"][2] == out["0"][2]


def test_native_tie_selection_matches_callback():
    """Ties resolved on the library's host thread with numpy's argsort routine give the same
    rollouts as the Python selection callback (np.argsort(-q)[:step]), single and batched."""
    z = load_golden("gmm1000_s0")
    g = (int(z["n_nodes"]), z["edges0"], z["edges1"])
    graphs = [g] + [(int(load_golden(nm)["n_nodes"]), load_golden(nm)["edges0"], load_golden(nm)["edges1"])
                    for nm in ("gmm200_s7", "er100")]
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
    try:
        for batch in ([g], graphs * 6):
            e.load_graphs(batch)
            e.reset()
            native = [(s.tolist(), r.tolist()) for s, r in e.rollout()]
            e.selector = lambda q, n_out: np.argsort(-q)[:n_out]  # forces the callback path
            e.reset()
            cb = [(s.tolist(), r.tolist()) for s, r in e.rollout()]
            e.selector = _lib._argsort_select
            assert native == cb
    finally:
        e.close()


def test_k2_endgame_in_one_handshake_matches_per_step(monkeypatch):
    """Unit-cost rollouts that reach a K2 end-game (every live node in a pair joined in both
    layers) let the host pick all remaining removals in one hand-shake; the rollouts equal the
    per-step protocol's (MD_VARIANT bit 2048), single graphs and a queue-mode batch."""
    names = ["gmm1000_s0", "gmm1000_s1", "gmm1000_s2", "er1000", "gmm200_s7", "er100"]
    graphs = [(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in map(load_golden, names)]

    def run(variant):
        monkeypatch.setenv("MD_VARIANT", str(variant))
        e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
        try:
            out = []
            for g in graphs:
                e.load_graphs([g])
                e.reset()
                out.append([(s.tolist(), r.tolist()) for s, r in e.rollout()])
                out.append([len(e.trace(0)["n_live"])])
            e.load_graphs(graphs * 3)
            e.reset()
            out.append([(s.tolist(), r.tolist()) for s, r in e.rollout()])
            return out
        finally:
            e.close()

    fast, slow = run(0), run(2048)
    for i in range(len(graphs)):
        assert fast[2 * i] == slow[2 * i], names[i]
        assert fast[2 * i + 1][0] <= slow[2 * i + 1][0]  # fewer forward passes recorded
    assert fast[-1] == slow[-1]
    # the GMM rollouts do end in K2 end-games: the shortcut skipped forward passes
    assert fast[1][0] < slow[1][0]


def test_k2_endgame_one_pass_apply_same_state(monkeypatch):
    """The K2 end-game answer applied in one pass (md_env.h env_endgame_apply) against action by
    action (MD_EG_APPLY=0): identical sequences, LMCC traces and final states (covered set,
    removed edges per layer, counters), single graphs (the synchronous hand-shake) and a batch
    (the asynchronous one); the LMCC trace also against the oracle environment stepped along
    the sequence (U/mvc_env.py:74-87, U/Mcc.py:30-38)."""
    from oracle import refenv
    from edge_graphs import cases
    names = ["gmm1000_s0", "gmm1000_s1", "gmm1000_s2", "er1000", "gmm200_s7", "er100"]
    graphs = [(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in map(load_golden, names)]
    graphs += [(n, e0, e1) for _, n, e0, e1 in cases()]

    def run(apply):
        monkeypatch.setenv("MD_EG_APPLY", str(apply))
        e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
        try:
            out = []
            for g in graphs:
                e.load_graphs([g])
                e.reset()
                (s, r), = e.rollout()
                cov, r0, r1, cnt = e.get_state(0)
                out.append((s.tolist(), r.tolist(), cov.tobytes(), r0.tobytes(), r1.tobytes(), cnt.tolist()))
            e.load_graphs(graphs * 2)
            e.reset()
            out.append([(s.tolist(), r.tolist()) for s, r in e.rollout()])
            return out
        finally:
            e.close()

    one, each = run(1), run(0)
    assert one == each
    for (n, e0, e1), got in zip(graphs, one):
        env = refenv.RefEnv(refenv.RefGraph(n, e0, e1), "unit")
        assert [env.step(int(a)) for a in got[0]] == got[1]
        assert env.terminal()


@pytest.mark.parametrize("name", ["gmm1000_s0", "gmm1000_s2", "er1000", "er300_dense"])
def test_speculative_steps_match_plain(monkeypatch, name):
    """Speculative environment workgroups (MD_SPEC, single-graph rollouts) change nothing:
    the same removal sequence and LMCC trace as without them, with most removals served by a
    speculative result, for the per-step protocol and the K2 end-game alike; 16 and 32 of
    them, with early requests (the next state built from the result phase A takes) and
    without (MD_EARLY=0: restaged from HBM after phase A's write-back), and with the fixed
    points of unusable results stopped early or run to the end (MD_SPEC_ABORT=0)."""
    z = load_golden(name)
    n = int(z["n_nodes"])
    w = engine.load_weights(engine.DEFAULT_UNIT)
    out = {}
    for spec, early, abort in (("0", "1", "1"), ("16", "1", "1"), ("32", "1", "1"), ("32", "0", "1"), ("32", "1", "0")):
        for variant in ("0", "2048"):
            monkeypatch.setenv("MD_SPEC", spec)
            monkeypatch.setenv("MD_EARLY", early)
            monkeypatch.setenv("MD_SPEC_ABORT", abort)
            monkeypatch.setenv("MD_VARIANT", variant)
            e = _lib.Engine(w)
            e.load_graphs([(n, z["edges0"], z["edges1"])])
            for rep in range(2):
                e.reset()
                seq, ranks = e.rollout()[0]
                out.setdefault((spec, early, abort, variant), []).append((seq.tolist(), ranks.tolist(), e.spec_stats(0)))
            e.close()
    base = out[("0", "1", "1", "0")][0]
    for key, runs in out.items():
        for seq, ranks, (hits, rem) in runs:
            assert seq == base[0] and ranks == base[1], key
            assert rem == len(seq)
            if key[0] == "0":
                assert hits == 0
            else:
                # how many removals a speculative workgroup serves depends on timing (whether it
                # started before phase A read the tags): only that the path ran is asserted
                assert hits > 0, (key, hits, len(seq))


def test_grid_wide_environment_step(monkeypatch):
    """One global-mode graph per launch runs its environment step on every workgroup
    (team_env_step: grid-strided union-find in HBM, grid barriers between the passes).
    MD_ENV_MODE=0 + MD_VARIANT=64 force it on small graphs; MD_VARIANT bit 2 restores the
    one-workgroup step.  Both give the certified sequences and AUDC, the same Q at s0, the same
    single-action steps (md_step) and the same multi-action rollouts (step > 1, host picks)."""
    monkeypatch.setenv("MD_ENV_MODE", "0")
    out = {}
    for variant in ("64", "66"):
        monkeypatch.setenv("MD_VARIANT", variant)
        e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
        try:
            for name in ("er100", "gmm200_s7", "er300_dense", "gmm1000_s0"):
                z = load_golden(name)
                n = int(z["n_nodes"])
                e.load_graphs([(n, z["edges0"], z["edges1"])])
                assert int(e.reset()[0]) == int(z["max_rank"]), (variant, name)
                q, _, _, _ = e.predict()
                seq, ranks = e.rollout()[0]
                assert seq.tolist() == load_cert(name)["gpu_seq"].tolist(), (variant, name)
                assert audc(ranks, int(z["max_rank"]), n) == float(z["score"]), (variant, name)
                e.reset()
                steps = [int(e.step(np.array([a], np.int32))[0][0]) for a in seq[:5].tolist()]
                assert steps == ranks[:5].tolist(), (variant, name)
                e.reset()
                s3, r3 = e.rollout(step=3)[0]
                out[(variant, name)] = (q.tobytes(), s3.tolist(), r3.tolist())
        finally:
            e.close()
    for name in ("er100", "gmm200_s7", "er300_dense", "gmm1000_s0"):
        assert out[("64", name)] == out[("66", name)], name


@pytest.mark.timeout(300)
def test_grid_wide_incremental_steps_random(monkeypatch):
    """The grid-wide step keeps the previous fixed point's class labels and sizes between its own
    steps (lab_ok) and runs each new fixed point on the removed node's class only; every other
    state change must drop them.  Random md_step calls (one action each; multi-action steps are
    the step > 1 rollouts of test_grid_wide_environment_step) on gmm1000_s0 in the grid-wide
    mode, with md_get_state / md_set_state round trips and md_predict calls in between, against
    the oracle environment stepped along the same actions: the LMCC, the covered set, the
    covered-edge counters (edges killed by a cover, not by an earlier prune) and the pruned-edge
    counts after every call."""
    from oracle import refenv
    monkeypatch.setenv("MD_ENV_MODE", "0")
    monkeypatch.setenv("MD_VARIANT", "64")
    z = load_golden("gmm1000_s0")
    n = int(z["n_nodes"])
    g = refenv.RefGraph(n, z["edges0"], z["edges1"])
    env = refenv.RefEnv(g, "unit")
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
    try:
        e.load_graphs([(n, z["edges0"], z["edges1"])])
        assert int(e.reset()[0]) == g.max_rank
        rng = np.random.default_rng(11)
        for it in range(40):
            live = refenv.featurize(g, env.covered, env.removed)[0]
            if not live:
                break
            a = int(rng.choice(np.asarray(live, np.int64)))
            lm, term = e.step(np.array([a], np.int32))
            r = env.step(a)
            assert int(lm[0]) == r, (it, a)
            cov, r0, r1, cnt = e.get_state(0)
            assert set(np.flatnonzero(cov).tolist()) == env.covered, it
            assert [int(cnt[0]), int(cnt[1])] == env.num_covered, it
            assert [int(cnt[2]), int(cnt[3])] == [len(env.removed[0]) // 2, len(env.removed[1]) // 2], it
            if bool(term[0]) or env.terminal():
                assert bool(term[0]) == env.terminal()
                break
            if it % 7 == 3:  # a state change outside the grid-wide step: the labels must be dropped
                e.set_state(0, cov, r0, r1)
            if it % 5 == 2:
                e.predict()
    finally:
        e.close()


@pytest.mark.timeout(300)
def test_grid_wide_two_graphs_alternating(monkeypatch):
    """Two loaded graphs share the grid-wide step's scratch (gscr_team: class labels and sizes);
    a step of one graph must drop the labels the other's steps left there (team_owner / lab_ok,
    md_abi.cpp).  md_step alternates between gmm1000_s0 and gmm1000_s2 in the grid-wide mode
    (each launch runs one graph), against one oracle environment per graph: LMCC, covered set
    and edge counters after every call."""
    from oracle import refenv
    monkeypatch.setenv("MD_ENV_MODE", "0")
    monkeypatch.setenv("MD_VARIANT", "64")
    names = ("gmm1000_s0", "gmm1000_s2")
    zs = [load_golden(nm) for nm in names]
    gs = [refenv.RefGraph(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in zs]
    envs = [refenv.RefEnv(g, "unit") for g in gs]
    e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
    try:
        e.load_graphs([(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in zs])
        assert [int(x) for x in e.reset()] == [g.max_rank for g in gs]
        rng = np.random.default_rng(5)
        done = [False, False]
        for it in range(40):
            k = it % 2
            if done[k]:
                continue
            live = refenv.featurize(gs[k], envs[k].covered, envs[k].removed)[0]
            if not live:
                done[k] = True
                continue
            a = int(rng.choice(np.asarray(live, np.int64)))
            acts = np.full(2, -1, np.int32)
            acts[k] = a
            lm, term = e.step(acts)
            r = envs[k].step(a)
            assert int(lm[k]) == r, (it, k, a)
            cov, _, _, cnt = e.get_state(k)
            assert set(np.flatnonzero(cov).tolist()) == envs[k].covered, (it, k)
            assert [int(cnt[0]), int(cnt[1])] == envs[k].num_covered, (it, k)
            assert [int(cnt[2]), int(cnt[3])] == [len(envs[k].removed[0]) // 2, len(envs[k].removed[1]) // 2], (it, k)
            if bool(term[k]) or envs[k].terminal():
                assert bool(term[k]) == envs[k].terminal()
                done[k] = True
    finally:
        e.close()


def test_iteration1_prebuild_same_rollouts(monkeypatch):
    """Single-graph rollouts build iteration 1 (rows, alive-neighbour lists, and the whole
    first message-passing iteration) during phase A from the speculative result phase A
    announces, and keep it when phase A confirms it.  The rollouts equal the ones without it
    (MD_VARIANT bit 1) and with lists only (bit 128), and the certified sequences."""
    out = {}
    for variant in ("0", "1", "128"):
        monkeypatch.setenv("MD_VARIANT", variant)
        e = _lib.Engine(engine.load_weights(engine.DEFAULT_UNIT))
        try:
            for name in ("gmm1000_s0", "gmm1000_s1", "gmm1000_s2", "er1000"):
                z = load_golden(name)
                e.load_graphs([(int(z["n_nodes"]), z["edges0"], z["edges1"])])
                e.reset()
                seq, ranks = e.rollout()[0]
                out[(variant, name)] = (seq.tolist(), ranks.tolist())
                assert seq.tolist() == load_cert(name)["gpu_seq"].tolist(), (variant, name)
        finally:
            e.close()
    for name in ("gmm1000_s0", "gmm1000_s1", "gmm1000_s2", "er1000"):
        assert out[("0", name)] == out[("1", name)] == out[("128", name)], name


def _hub_layer(n, hub, hub_deg, rng):
    m = 2 * n
    u = rng.integers(0, n, size=3 * m)
    v = rng.integers(0, n, size=3 * m)
    e = sorted({(min(a, b), max(a, b)) for a, b in zip(u.tolist(), v.tolist()) if a != b})[:m]
    nb = rng.choice(np.setdiff1d(np.arange(n), [hub]), size=hub_deg, replace=False)
    return np.array(sorted(set(e) | {(min(hub, int(x)), max(hub, int(x))) for x in nb}), np.int32)


@pytest.mark.parametrize("cost", ["unit", "degree"])
def test_paired_tiles_match_single_tiles(monkeypatch, cost):
    """Queue mode runs the two tiles of a 2-tile work item jointly (queue_pair: 32 rows per
    piece); MD_PAIR=0 runs them one after the other (queue_tile).  Same rollouts, for unit and
    degree cost, on a batch with a hub graph whose tiles overflow the LDS neighbour lists
    (the per-row CSR gather) and with odd tile counts (a last single-tile item)."""
    rng = np.random.default_rng(5)
    hub = (3000, _hub_layer(3000, 3, 2400, rng), _hub_layer(3000, 3, 2400, rng))
    names = ["gmm200_s7", "er100", "er300_dense", "gmm1000_s1"]
    graphs = [(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in map(load_golden, names)]
    batch = [hub] + [graphs[i % len(graphs)] for i in range(19)]
    w, mode = ((engine.load_weights(engine.DEFAULT_UNIT), _lib.MD_COST_UNIT) if cost == "unit" else
               (engine.load_weights(engine.DEFAULT_DEGREE), _lib.MD_COST_DEGREE))
    node_w = None
    if cost == "degree":
        from mdcommunity_amd import graph as mgraph
        node_w = mgraph.node_weight_array([mgraph.Graph_test.from_edges(n, e0, e1) for n, e0, e1 in batch])
    out = {}
    for pair in ("0", "1"):
        monkeypatch.setenv("MD_PAIR", pair)
        e = _lib.Engine(w, cost_mode=mode)
        try:
            e.load_graphs(batch, node_w=node_w)
            e.reset()
            out[pair] = [(s.tolist(), r.tolist()) for s, r in e.rollout()]
        finally:
            e.close()
    assert len(out["1"]) == len(batch)
    for i, (a, b) in enumerate(zip(out["0"], out["1"])):
        assert a == b, i


@pytest.mark.parametrize("cost", ["unit", "degree"])
def test_wave_items_match_workgroup_items(monkeypatch, cost):
    """Batch rollouts with one work item per wave (md_wq_kernel, default: each wave runs a whole
    tile, both layers, or a virtual-node step; environment steps in a workgroup group section)
    give the removal sequences and LMCC traces of the per-workgroup queue kernel (MD_WQ=0,
    md_queue_kernel): unit and degree cost, a hub graph whose tiles overflow the neighbour lists
    (the per-row CSR gather), odd tile counts."""
    rng = np.random.default_rng(5)
    hub = (3000, _hub_layer(3000, 3, 2400, rng), _hub_layer(3000, 3, 2400, rng))
    names = ["gmm200_s7", "er100", "er300_dense", "gmm1000_s1"]
    graphs = [(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in map(load_golden, names)]
    batch = [hub] + [graphs[i % len(graphs)] for i in range(19)]
    w, mode = ((engine.load_weights(engine.DEFAULT_UNIT), _lib.MD_COST_UNIT) if cost == "unit" else
               (engine.load_weights(engine.DEFAULT_DEGREE), _lib.MD_COST_DEGREE))
    node_w = None
    if cost == "degree":
        from mdcommunity_amd import graph as mgraph
        node_w = mgraph.node_weight_array([mgraph.Graph_test.from_edges(n, e0, e1) for n, e0, e1 in batch])
    out = {}
    # (MD_WQPARK=0: the wave kernel runs this 20-graph batch to the end -- by default a launch of
    # at most MD_WQPARK graphs goes to md_queue_kernel)
    monkeypatch.setenv("MD_WQPARK", "0")
    for wq in ("0", "1"):
        monkeypatch.setenv("MD_WQ", wq)
        e = _lib.Engine(w, cost_mode=mode)
        try:
            e.load_graphs(batch, node_w=node_w)
            e.reset()
            out[wq] = [(s.tolist(), r.tolist()) for s, r in e.rollout()]
        finally:
            e.close()
    assert len(out["1"]) == len(batch)
    for i, (a, b) in enumerate(zip(out["0"], out["1"])):
        assert a == b, i


@pytest.mark.parametrize("wq", ["1", "0"])
def test_iteration3_order_and_staging_same_rollouts(monkeypatch, wq):
    """Queue launches (wave items and md_queue_kernel, no tail hand-off): the iteration-3 tiles
    queued beside virtual-node part 2 (default) or after it (MD_VARIANT bit 12), and the
    environment staged in one pass (default) or in the batched two-pass form (bit 8), give
    identical rollouts; and a single-graph rollout whose applied speculative results compact
    the alive list (bit 15) equals the default's."""
    rng = np.random.default_rng(11)
    hub = (3000, _hub_layer(3000, 3, 2400, rng), _hub_layer(3000, 3, 2400, rng))
    names = ["gmm200_s7", "er100", "er300_dense", "gmm1000_s1"]
    graphs = [(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in map(load_golden, names)]
    batch = [hub] + [graphs[i % len(graphs)] for i in range(19)]
    w = engine.load_weights(engine.DEFAULT_UNIT)
    monkeypatch.setenv("MD_WQPARK", "0")
    monkeypatch.setenv("MD_QPARK", "0")
    monkeypatch.setenv("MD_WQ", wq)
    out = {}
    for v in ("0", "4096", "256"):
        monkeypatch.setenv("MD_VARIANT", v)
        e = _lib.Engine(w)
        try:
            e.load_graphs(batch)
            e.reset()
            out[v] = [(s_.tolist(), r.tolist()) for s_, r in e.rollout()]
        finally:
            e.close()
    assert out["0"] == out["4096"] == out["256"]
    z = load_golden("gmm1000_s0")
    single = {}
    for v in ("0", "32768"):
        monkeypatch.setenv("MD_VARIANT", v)
        e = _lib.Engine(w)
        try:
            e.load_graphs([(int(z["n_nodes"]), z["edges0"], z["edges1"])])
            e.reset()
            single[v] = [(s_.tolist(), r.tolist()) for s_, r in e.rollout()]
        finally:
            e.close()
    assert single["0"] == single["32768"]


@pytest.mark.parametrize("cost", ["unit", "degree"])
@pytest.mark.parametrize("wq", ["1", "0"])
def test_batch_speculation_same_rollouts(monkeypatch, cost, wq):
    """Queue launches with speculative environment items (MD_BSPEC=1; off by default: the environment
    item of step t queues the fixed point of the likely next pick, the live node of largest Q(t-1);
    step t + 1 applies it when it picks that node) give the removal sequences and LMCC traces of
    queue launches without them (MD_BSPEC=0), in the wave-item kernel and md_queue_kernel, unit and
    degree cost, over two rollouts of the same load (slots reused across launches); the
    speculation takes part in a good share of the steps (md_spec_stats)."""
    rng = np.random.default_rng(7)
    hub = (3000, _hub_layer(3000, 3, 2400, rng), _hub_layer(3000, 3, 2400, rng))
    names = ["gmm200_s7", "er100", "er300_dense", "gmm1000_s1", "gmm1000_s0"]
    graphs = [(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in map(load_golden, names)]
    batch = [hub] + [graphs[i % len(graphs)] for i in range(23)]
    w, mode = ((engine.load_weights(engine.DEFAULT_UNIT), _lib.MD_COST_UNIT) if cost == "unit" else
               (engine.load_weights(engine.DEFAULT_DEGREE), _lib.MD_COST_DEGREE))
    node_w = None
    if cost == "degree":
        from mdcommunity_amd import graph as mgraph
        node_w = mgraph.node_weight_array([mgraph.Graph_test.from_edges(n, e0, e1) for n, e0, e1 in batch])
    monkeypatch.setenv("MD_WQPARK", "0")
    monkeypatch.setenv("MD_QPARK", "0")
    monkeypatch.setenv("MD_WQ", wq)
    out, hits, rem = {}, 0, 0
    for bs in ("0", "1"):
        monkeypatch.setenv("MD_BSPEC", bs)
        e = _lib.Engine(w, cost_mode=mode)
        try:
            e.load_graphs(batch, node_w=node_w)
            runs = []
            for _ in range(2):
                e.reset()
                runs.append([(s.tolist(), r.tolist()) for s, r in e.rollout()])
            assert runs[0] == runs[1]
            out[bs] = runs[0]
            if bs == "1":
                for g in range(len(batch)):
                    h, r = e.spec_stats(g)
                    hits += h
                    rem += r
        finally:
            e.close()
    for i, (a, b) in enumerate(zip(out["0"], out["1"])):
        assert a == b, i
    assert hits > 0.2 * rem, (hits, rem)


@pytest.mark.parametrize("cost", ["unit", "degree"])
def test_dataflow_mode_same_rollouts(monkeypatch, cost):
    """The barrier-free dataflow mode of single-graph rollouts (MD_DF=1, default: tagged granules
    for the step record, rows and partials; the tiles derive phase A's pick from the arg-max
    partials and prebuild iteration 1 from it before phase A's slot check) gives the removal
    sequences and LMCC traces of the grid-barrier protocol (MD_DF=0, which also keeps the
    barrier-mode prebuild from phase A's early word), over repeated rollouts (timing-dependent
    paths), for graphs of 100 to 1000 nodes, with and without the K2 end-game shortcut."""
    if cost == "unit":
        names, w = ["gmm200_s7", "er100", "gmm1000_s0", "er300_dense", "gmm1000_s1"], engine.load_weights(engine.DEFAULT_UNIT)
    else:
        names, w = ["deg_gmm200_s7", "deg_er100"], engine.load_weights(engine.DEFAULT_DEGREE)
    for name in names:
        z = load_golden(name)
        n = int(z["n_nodes"])
        out = {}
        for df in ("0", "1"):
            for variant in (("0", "2048") if cost == "unit" else ("0",)):
                monkeypatch.setenv("MD_DF", df)
                monkeypatch.setenv("MD_VARIANT", variant)
                if cost == "unit":
                    e = _lib.Engine(w)
                    e.load_graphs([(n, z["edges0"], z["edges1"])])
                else:
                    from mdcommunity_amd import graph as mgraph
                    g = mgraph.Graph_test.from_edges(n, z["edges0"], z["edges1"])
                    mgraph.ensure_degree_weights(g)
                    e = _lib.Engine(w, cost_mode=_lib.MD_COST_DEGREE)
                    e.load_graphs([(n, z["edges0"], z["edges1"])], node_w=mgraph.node_weight_array([g]))
                for rep in range(3):
                    e.reset()
                    seq, ranks = e.rollout()[0]
                    out.setdefault(variant, []).append((df, seq.tolist(), ranks.tolist()))
                e.close()
        for variant, runs in out.items():
            for df, seq, ranks in runs:
                assert (seq, ranks) == (runs[0][1], runs[0][2]), (name, variant, df)


def test_fixed_point_shortcut_same_rollouts(monkeypatch):
    """MD_FP_SHORTCUT=0 (every mutual-LMCC fixed point runs its confirmation round) and
    MD_FP_SKIP=0 (every round re-unites both layers, also those the last prune left unchanged)
    give the removal sequences and LMCC traces of the defaults, alone and together
    (tests/test_fixed_point_shortcut.py checks the certificate itself on the CPU): single-graph
    launches (phase A, speculative workgroups, dataflow mode) and a 24-graph queue-mode launch
    (environment items)."""
    from mdcommunity_amd import gmm
    w = engine.load_weights(engine.DEFAULT_UNIT)
    singles = [load_golden(k) for k in ("gmm200_s7", "er100", "gmm1000_s0", "er300_dense")]
    batch = [(1000,) + gmm.gmm_pair(1000, seed=s) for s in range(24)]
    out = {}
    for fs in ("00", "01", "10", "11"):
        monkeypatch.setenv("MD_FP_SHORTCUT", fs[0])
        monkeypatch.setenv("MD_FP_SKIP", fs[1])
        e = _lib.Engine(w)
        res = []
        for z in singles:
            e.load_graphs([(int(z["n_nodes"]), z["edges0"], z["edges1"])])
            e.reset()
            seq, ranks = e.rollout()[0]
            res.append((seq.tolist(), ranks.tolist()))
        e.load_graphs(batch)
        e.reset()
        res += [(s.tolist(), r.tolist()) for s, r in e.rollout()]
        e.close()
        out[fs] = res
    assert out["00"] == out["11"] and out["01"] == out["11"] and out["10"] == out["11"]


def test_deferred_reset_same_rollouts():
    """md_reset_deferred (MvcEnv.s0's prune as the rollout launch's first environment step, the
    bench's path) gives the removal sequences, LMCC traces and max_rank of md_reset + md_rollout:
    single-graph launches (dataflow mode) and a 24-graph queue-mode launch, twice each (the
    deferred reset after a finished rollout)."""
    from mdcommunity_amd import gmm
    w = engine.load_weights(engine.DEFAULT_UNIT)
    singles = [load_golden(k) for k in ("gmm200_s7", "er100", "gmm1000_s0")]
    sets = [[(int(z["n_nodes"]), z["edges0"], z["edges1"])] for z in singles]
    sets.append([(1000,) + gmm.gmm_pair(1000, seed=s) for s in range(24)])
    e = _lib.Engine(w)
    try:
        for graphs in sets:
            e.load_graphs(graphs)
            mr = e.reset().copy()
            ref = [(s.tolist(), r.tolist()) for s, r in e.rollout()]
            for _ in range(2):
                e.reset_deferred()
                got = [(s.tolist(), r.tolist()) for s, r in e.rollout()]
                assert got == ref
                assert np.array_equal(e.max_rank(), mr)
    finally:
        e.close()


def test_deferred_reset_then_rollout_empty_layer_graph():
    """md_rollout after md_reset_deferred launches only graphs with edges in both
    layers; a graph with an empty layer (terminal from the start) must still get the s0 prune,
    so md_get_state and md_max_rank after the rollout equal md_reset's (U/mvc_env.py:52)."""
    w = engine.load_weights(engine.DEFAULT_UNIT)
    rng = np.random.default_rng(5)
    iu = np.array([(i, j) for i in range(20) for j in range(i + 1, 20)], np.int32)
    e0 = iu[rng.random(len(iu)) < 0.3]
    z = load_golden("er100")
    graphs = [(int(z["n_nodes"]), z["edges0"], z["edges1"]), (20, e0, np.zeros((0, 2), np.int32))]
    e = _lib.Engine(w)
    try:
        e.load_graphs(graphs)
        mr = e.reset().copy()
        st_ref = e.get_state(1)
        e.rollout()
        e.reset_deferred()
        e.rollout()
        for a, b in zip(e.get_state(1), st_ref):
            assert np.array_equal(a, b)
        assert np.array_equal(e.max_rank(), mr)
    finally:
        e.close()


def test_deferred_reset_then_step_predict_state():
    """After md_reset_deferred, md_step / md_predict / md_get_state / md_max_rank run the pending
    s0 prune first (U/mvc_env.py:52 before :74-87): the state, LMCC, max_rank and Q equal those
    after md_reset, on a single graph and on a 3-graph batch."""
    w = engine.load_weights(engine.DEFAULT_UNIT)
    singles = [load_golden(k) for k in ("gmm200_s7", "er100", "gmm1000_s0")]
    sets = [[(int(z["n_nodes"]), z["edges0"], z["edges1"])] for z in singles[:1]]
    sets.append([(int(z["n_nodes"]), z["edges0"], z["edges1"]) for z in singles])
    e = _lib.Engine(w)
    try:
        for graphs in sets:
            e.load_graphs(graphs)
            ng = len(graphs)
            mr = e.reset().copy()
            q_ref = e.predict()[0].copy()
            acts = np.array([int(np.argmax(q_ref[int(e.node_off[g]):int(e.node_off[g + 1])])) for g in range(ng)], np.int32)
            lm_ref, term_ref = e.step(acts)
            st_ref = [e.get_state(g) for g in range(ng)]
            # md_step straight after the deferred reset
            e.reset_deferred()
            lm, term = e.step(acts)
            assert np.array_equal(lm, lm_ref) and np.array_equal(term, term_ref)
            for g in range(ng):
                got = e.get_state(g)
                for a, b in zip(got, st_ref[g]):
                    assert np.array_equal(a, b)
            assert np.array_equal(e.max_rank(), mr)
            # md_predict / md_get_state / md_max_rank straight after the deferred reset
            e.reset_deferred()
            assert np.array_equal(e.predict()[0], q_ref)
            e.reset_deferred()
            s0_state = e.get_state(0)
            e.reset()
            for a, b in zip(s0_state, e.get_state(0)):
                assert np.array_equal(a, b)
            e.reset_deferred()
            assert np.array_equal(e.max_rank(), mr)
    finally:
        e.close()
