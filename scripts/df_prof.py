"""Per-step phase profile of a dataflow-mode single-graph rollout (md_profile stamps: phase A
of the environment workgroup, tile 0's layer-0 workgroup, the graph-head workgroup)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from mdcommunity_amd import _lib, engine
W = engine.load_weights(engine.DEFAULT_UNIT)
name = sys.argv[1] if len(sys.argv) > 1 else "gmm1000_s0"
z = np.load(os.path.join(ROOT, f"tests/golden/rollout_{name}.npz"))
e = _lib.Engine(W)
e.load_graphs([(int(z["n_nodes"]), z["edges0"], z["edges1"])])
e.reset(); e.rollout()
ks = []
for _ in range(10):
    e.reset(); e.rollout(); ks.append(e.last_timing()[0])
e.reset(); e.profile(512); e.rollout(); ms, _ = e.last_timing()
P = e.profile_read().astype(np.int64); e.profile(0)
TR = e.trace(0)
S = len(P)
full = P[(P[:, 10] > 0) & (P[:, 0] > 0)]
nxt = np.append(P[1:, 0], 0)[(P[:, 10] > 0) & (P[:, 0] > 0)]
ok = nxt > 0
d = lambda a, b: (full[:, b] - full[:, a]) / 100.0
segs = [("phaseA", 0, 3), ("rec->tile", 3, 4), ("it1", 4, 5), ("it2 gather", 5, 23), ("it2 rest", 23, 6),
        ("it3 gather", 6, 29), ("it3 upd+norm", 29, 30), ("L1 recv", 30, 8), ("attn+Q", 8, 9)]
print(f"{name}: unprofiled kernel ms median {np.median(ks):.3f}; profiled {ms:.3f} ms, {len(full)} steps", flush=True)
print("  median us: " + "  ".join(f"{s}={np.median(d(a, b)):.1f}" for s, a, b in segs) +
      f"  tile end->next phaseA={np.median((nxt[ok] - full[ok, 9]) / 100.0):.1f}  step={np.median((nxt[ok] - full[ok, 0]) / 100.0):.1f}", flush=True)
print("  mean us:   " + "  ".join(f"{s}={np.mean(d(a, b)):.1f}" for s, a, b in segs) +
      f"  tile end->next phaseA={np.mean((nxt[ok] - full[ok, 9]) / 100.0):.1f}  step={np.mean((nxt[ok] - full[ok, 0]) / 100.0):.1f}", flush=True)
h = lambda a, b: np.median((full[:, b] - full[:, a]) / 100.0)
# critical path from the step record (slot 3): the latest tile at each point, phase A's side
R = P[:-1]
nx3 = P[1:, 3]
m = (R[:, 3] > 0) & (R[:, 46] > 0) & (nx3 > 0) & (R[:, 11] > 0)
rel = lambda col: np.median((R[m, col] - R[m, 3]) / 100.0)
print("  from the record (latest tile): seen %.1f  it1 %.1f  it2 %.1f  L1 rows out %.1f  arg-max out %.1f | phase A: "
      "partials in %.1f  spec check %.1f-%.1f  next record %.1f us (%d steps)" % (
          rel(43), rel(44), rel(45), rel(47), rel(46), rel(11), rel(69) if np.all(R[m, 69] > 0) else float("nan"),
          rel(71) if np.all(R[m, 71] > 0) else float("nan"), np.median((nx3[m] - R[m, 3]) / 100.0), int(m.sum())), flush=True)
Rn = P[1:]
print("  phase A tail (from the spec check end): apply %.1f  features %.1f  write-back %.1f  request+h0 %.1f  record %.1f us" % (
    np.median((Rn[m, 2] - R[m, 71]) / 100.0), np.median((Rn[m, 34] - Rn[m, 2]) / 100.0), np.median((Rn[m, 14] - Rn[m, 34]) / 100.0),
    np.median((Rn[m, 15] - Rn[m, 14]) / 100.0), np.median((Rn[m, 3] - Rn[m, 15]) / 100.0)), flush=True)
mm = m & (Rn[:, 56] > 0)
print("  prebuild of step t+1 (latest tile, from the record of t): early word seen %.1f  lists %.1f  iteration 1 %.1f us" % (
    np.median((Rn[mm, 54] - R[mm, 3]) / 100.0) if mm.any() else float("nan"), np.median((Rn[mm, 55] - R[mm, 3]) / 100.0) if mm.any() else float("nan"),
    np.median((Rn[mm, 56] - R[mm, 3]) / 100.0) if mm.any() else float("nan")), flush=True)
print("  tiles seeing the record, latest (from the record): with prebuild %.1f  without %.1f us; tiles without the confirmed prebuild per step: median %.0f mean %.1f max %d" % (
    np.median((R[m & (R[:, 77] > 0), 77] - R[m & (R[:, 77] > 0), 3]) / 100.0) if (m & (R[:, 77] > 0)).any() else float("nan"),
    np.median((R[m & (R[:, 76] > 0), 76] - R[m & (R[:, 76] > 0), 3]) / 100.0) if (m & (R[:, 76] > 0)).any() else float("nan"),
    np.median(R[m, 79]), np.mean(R[m, 79]), int(R[m, 79].max())), flush=True)
print("  phase A check (from the record): start %.1f end %.1f; steps whose check polled a running slot: %d of %d, longest poll median %.1f us" % (
    np.median((R[m, 69] - R[m, 3]) / 100.0), np.median((R[m, 71] - R[m, 3]) / 100.0), int((R[m, 31] > 0).sum()), int(m.sum()),
    np.median(R[m & (R[:, 31] > 0), 32] / 100.0) if (m & (R[:, 31] > 0)).any() else 0.0), flush=True)
mp = (P[:, 28] > 0) & (P[:, 24] > 0) & (P[:, 25] > 0) & (P[:, 63] > 0) & (P[:, 26] > 0) & (P[:, 27] > 0) & (P[:, 35] > 0)
if mp.any():
    q = lambda a, b: np.median((P[mp, b] - P[mp, a]) / 100.0)
    print("  tile 0 / layer 0 prebuild pieces (us, %d steps): poll %.1f  rows+kills %.1f  lists: prefix %.1f scan %.1f write %.1f  gather %.1f  update+norm %.1f  store %.1f  | total %.1f" % (
        int(mp.sum()), q(28, 24), q(24, 25), q(25, 61), q(61, 62), q(62, 63), q(63, 26), q(26, 27), q(27, 35), q(28, 35)), flush=True)
print("  request -> next record: spec wg0 done %.1f features %.1f" % (
    np.median((R[m, 68] - R[m, 64]) / 100.0), np.median((R[m, 74] - R[m, 64]) / 100.0)), flush=True)
mq = m & (R[:, 65] > 0) & (R[:, 73] > 0) & (R[:, 66] > 0) & (R[:, 67] > 0) & (R[:, 68] > 0) & (R[:, 74] > 0)
if mq.any():
    dd = lambda a, b: np.median((R[mq, b] - R[mq, a]) / 100.0)
    print("  spec wg0 (from the request): seen %.1f  staged %.1f  ranked %.1f  taken %.1f  fixed point %.1f  features %.1f us; request at %.1f from the record" % (
        dd(64, 65), dd(64, 73), dd(64, 66), dd(64, 67), dd(64, 68), dd(64, 74), np.median((R[mq, 64] - R[mq, 3]) / 100.0)), flush=True)
me = (P[1:, 33] == 1) & (P[:-1, 71] > 0) & (P[1:, 65] > 0)
if me.any():
    print("  early requests (wg0): %d of %d; phase A's early word -> wg0 sees it %.1f  staged %.1f  fixed point done %.1f  features %.1f us" % (
        int(me.sum()), len(me), np.median((P[1:, 65][me] - P[:-1, 71][me]) / 100.0), np.median((P[1:, 73][me] - P[:-1, 71][me]) / 100.0),
        np.median((P[1:, 68][me] - P[:-1, 71][me]) / 100.0), np.median((P[1:, 74][me] - P[:-1, 71][me]) / 100.0)), flush=True)
print("  head it3 from record: start %.1f graph_sum(S2) done %.1f vrow %.1f head %.1f published %.1f us" % (
    h(3, 49), h(3, 50), h(3, 51), h(3, 52), h(3, 53)), flush=True)
e.close()
# per-step table (us from the record of step t): next record, latest tile seeing the next record,
# spec wg0 done / features (from the request), phase A's spec check end, prebuild stamps of t+1
print("  step: next_rec seen_next | req->done req->feat | check_end | pre: ew lists it1 | hit_slot | no-prebuild tiles", flush=True)
for t in range(min(len(P) - 2, 40)):
    a, b, c = P[t], P[t + 1], P[t + 2] if t + 2 < len(P) else P[t + 1]
    if a[3] == 0 or b[3] == 0:
        continue
    f = lambda x: "%.1f" % ((x - a[3]) / 100.0) if x > 0 else "-"
    print("  %3d: %s %s | %s %s | %s | %s %s %s | %d | %d" % (t, f(b[3]), "%.1f" % ((b[43] - b[3]) / 100.0) if b[43] > 0 else "-",
          "%.1f" % ((a[68] - a[64]) / 100.0) if a[68] > 0 else "-", "%.1f" % ((a[74] - a[64]) / 100.0) if a[74] > 0 else "-",
          f(a[71]), f(b[54]), f(b[55]), f(b[56]), int(a[70]), int(b[79])), flush=True)
# where the long steps come from: misses (no speculative result taken), cascade steps (the
# taken result's fixed point ran > 60 us), the rest
rows = []
for t in range(len(P) - 1):
    a, b = P[t], P[t + 1]
    if a[3] == 0 or b[3] == 0:
        continue
    rows.append(((b[3] - a[3]) / 100.0, int(a[70]), (a[68] - a[64]) / 100.0 if a[68] > 0 and a[64] > 0 else -1.0))
if rows:
    st = np.array([r[0] for r in rows]); hit = np.array([r[1] for r in rows]); fp = np.array([r[2] for r in rows])
    miss = hit == 0; casc = (~miss) & (fp > 60); rest = ~miss & ~casc
    print("  step classes: misses %d (%.0f us total, median %.1f), cascade %d (%.0f us, median %.1f), others %d (%.0f us, median %.1f); slot hits by rank: %s" % (
        miss.sum(), st[miss].sum(), np.median(st[miss]) if miss.any() else 0, casc.sum(), st[casc].sum(), np.median(st[casc]) if casc.any() else 0,
        rest.sum(), st[rest].sum(), np.median(st[rest]) if rest.any() else 0, np.bincount(hit).tolist()), flush=True)
    nt, gp = TR["n_tie"], TR["gap"]
    print("  misses (row: step us, ties / top-2 gap of predictions row-1..row+1): " + "; ".join(
        "%d: %.0f us, %s" % (t, st[t], [(int(nt[k]), float(gp[k])) for k in range(max(0, t - 1), min(len(nt), t + 2))])
        for t in np.nonzero(miss)[0]), flush=True)
# per-tile distribution (rows 128 + 4 t + k): iteration-2 start and prebuild end, from the record
# of step t (prebuild of step t+1 from the record of t)
os.environ["MD_PROF_ALL"] = "1"
e = _lib.Engine(W)
e.load_graphs([(int(z["n_nodes"]), z["edges0"], z["edges1"])])
e.reset(); e.rollout()
e.reset(); e.profile(512); e.rollout()
P2 = e.profile_read().astype(np.int64); e.profile(0)
del os.environ["MD_PROF_ALL"]
st_rel, pb_rel = [], []
for t in range(1, min(60, (len(P2) - 132) // 4)):
    rec = P2[t, 3]
    if rec == 0:
        continue
    s = np.concatenate([P2[128 + 4 * t, :64], P2[129 + 4 * t, :64]])
    b = np.concatenate([P2[130 + 4 * t, :64], P2[131 + 4 * t, :64]])
    s = s[s > 0]; b = b[b > 0]
    if len(s):
        st_rel.append(np.percentile((s - rec) / 100.0, [10, 50, 90, 100]))
    if len(b):
        pb_rel.append(np.percentile((b - rec) / 100.0, [10, 50, 90, 100]))
late = []
for t in range(1, min(60, (len(P2) - 132) // 4)):
    rec = P2[t, 3]
    if rec == 0:
        continue
    s = np.concatenate([P2[128 + 4 * t, :64], P2[129 + 4 * t, :64]]).astype(np.float64)
    s[s <= 0] = np.nan
    if np.isfinite(s).any():
        late.append(int(np.nanargmax(s)))
if late:
    lt = np.bincount(np.array(late), minlength=128)
    top = np.argsort(-lt)[:8]
    print("  latest tile workgroup to start iteration 2 (tile workgroup tb = 2 j + layer: steps): " +
          ", ".join("%d: %d" % (int(k), int(lt[k])) for k in top if lt[k] > 0), flush=True)
if st_rel:
    print("  per tile, iteration-2 start after the record (median over steps of the p10/p50/p90/max over tiles):",
          np.round(np.median(np.array(st_rel), axis=0), 1).tolist(), flush=True)
if pb_rel:
    print("  per tile, prebuild end after the record:", np.round(np.median(np.array(pb_rel), axis=0), 1).tolist(), flush=True)
e.close()
