// md_env.h — phase A of the rollout kernel: the MvcEnv step of one graph on one workgroup
// (cover the chosen node U/mvc_env.py:74-85, the mutual-LMCC fixed point U/Mcc.py:30-38, and
// the per-step graph features of U/PrepareBatchGraph.py:35-74).  Included by md_kernels.hip.
//
// Two storage modes share the code: LDS mode (the graph's edges, states, union-find and
// degree arrays staged in LDS; every graph of the reference's synthetic sizes) and global mode
// (arrays in HBM scratch, for graphs too large for one workgroup's LDS).  LDS-mode accesses go
// through address-space-3 pointers so they compile to ds_* instructions, and edge passes read
// eight edges per vector load.
#pragma once
#include <type_traits>

typedef __attribute__((address_space(3))) int lds_i32;
typedef __attribute__((address_space(3))) uint16_t lds_u16;
typedef __attribute__((address_space(3))) uint8_t lds_u8;
typedef __attribute__((address_space(3))) unsigned lds_u32;
typedef unsigned int v2u __attribute__((ext_vector_type(2)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v2u lds_u2;
typedef __attribute__((address_space(3))) v4u lds_u4;

// Phase-A sub-step timestamps of workgroup 0 (diagnostics; step index stashed in LDS misc[60]).
#define MD_PROF_A(slot)                                                                          \
  do {                                                                                           \
    if (p.prof != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {                              \
      const int ps_ = ((volatile int*)(lds_base + L_MISC))[60];                                  \
      if (ps_ < p.prof_cap) p.prof[(size_t)ps_ * PROF_SLOTS + (slot)] = wall_clock64();          \
    }                                                                                            \
  } while (0)

// Profile accumulators (slots 16.. of a profiled step; workgroup 0, thread 0 writes).
enum { PA_ROUNDS = 0, PA_UNITE = 1, PA_LABEL = 2, PA_PRUNE = 3, PA_COUNT = 4, PA_CALLS = 5, PA_COVER = 6,
       PA_INIT = 40, PA_FINDONLY = 41, PA_EDGES = 42, PA_UNIONS = 43 };  // 40+: slots 56.. of the step
#define PACC(acc, slot, t0)                                                          \
  do {                                                                               \
    if ((acc) != nullptr && threadIdx.x == 0) (acc)[slot] += wall_clock64() - (t0);  \
  } while (0)

// ------------------------------------------------------------------ union-find
// Parents always point to smaller ids, so the root of a tree is its minimum node id (the
// canonical label compared across layers).  Lock-free hooking of roots with compare-and-swap.
// Global-mode arrays are plain (flat) int pointers with agent-scope atomics; LDS-mode arrays
// are address-space-3 pointers (ds_* instructions, no aperture conversion, and no aliasing
// with the private stack, so view fields stay in registers).
// Queue-mode environment-item piece profile (builds with -DMD_QPROF, MD_VARIANT bit 8): device
// ticks per piece summed over items in md_profile slots 80.. (scripts/batch_prof.py)
#ifdef MD_QPROF
#define QENV_INIT() unsigned long long tqe_ = wall_clock64()
#define QENV(k)                                                                        \
  do {                                                                                 \
    if (p.prof != nullptr && p.qmode && (p.variant & 8) && threadIdx.x == 0) {         \
      const unsigned long long now_ = wall_clock64();                                  \
      atomicAdd(p.prof + 80 + (k), now_ - tqe_);                                       \
      tqe_ = now_;                                                                     \
    }                                                                                  \
  } while (0)
#else
#define QENV_INIT() do {} while (0)
#define QENV(k) do {} while (0)
#endif

__device__ __forceinline__ int uf_load(int* a, int i) {
  return __hip_atomic_load(a + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int uf_load(lds_i32* a, int i) {
  return __hip_atomic_load(a + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void uf_store(int* a, int i, int v) {
  __hip_atomic_store(a + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void uf_store(lds_i32* a, int i, int v) {
  __hip_atomic_store(a + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ int uf_cas(int* a, int i, int expect, int v) { return atomicCAS(a + i, expect, v); }
__device__ __forceinline__ int uf_cas(lds_i32* a, int i, int expect, int v) {
  __hip_atomic_compare_exchange_strong(a + i, &expect, v, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
  return expect;
}
__device__ __forceinline__ void uf_add(int* a, int i, int v) {
  __hip_atomic_fetch_add(a + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void uf_add(lds_i32* a, int i, int v) {
  __hip_atomic_fetch_add(a + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <class P>
__device__ __forceinline__ int uf_find(P par, int v) {
  int cur = uf_load(par, v);
  if (cur != v) {
    int prev = v, next;
    while (cur > (next = uf_load(par, cur))) {
      uf_store(par, prev, next);  // path halving; benign race (values only shrink)
      prev = cur;
      cur = next;
    }
  }
  return cur;
}
template <class P>
__device__ __forceinline__ void uf_unite(P par, int a, int b) {
  while (true) {
    a = uf_find(par, a);
    b = uf_find(par, b);
    if (a == b) return;
    if (a > b) { const int t = a; a = b; b = t; }
    if (uf_cas(par, b, b, a) == b) return;
  }
}

// uf_unite that reports whether it linked two trees (the edge is then a spanning-forest edge)
template <class P>
__device__ __forceinline__ bool uf_link(P par, int a, int b) {
  while (true) {
    a = uf_find(par, a);
    b = uf_find(par, b);
    if (a == b) return false;
    if (a > b) { const int t = a; a = b; b = t; }
    if (uf_cas(par, b, b, a) == b) return true;
  }
}

// Union of the trees holding a and b, climbing both paths in lockstep (two independent LDS
// loads per hop instead of two dependent find loops), path splitting on the way; stops when
// the paths meet or after hooking root hi -> lo (a failed compare-and-swap re-reads).
template <class P>
__device__ __forceinline__ void uf_unite2(P par, int a, int b) {
  int ap = -1, bp = -1;
  while (a != b) {
    const int na = uf_load(par, a), nb = uf_load(par, b);
    if (na == a && nb == b) {
      const int hi = a > b ? a : b, lo = a > b ? b : a;
      if (uf_cas(par, hi, hi, lo) == hi) return;
      continue;
    }
    if (na != a) {
      if (ap >= 0) uf_store(par, ap, na);
      ap = a;
      a = na;
    }
    if (nb != b) {
      if (bp >= 0) uf_store(par, bp, nb);
      bp = b;
      b = nb;
    }
  }
}

// Union-find for the grid-wide step: roots linked by a random priority (a bijective hash of the
// node id) instead of the id -- concurrent min-id linking of a large component builds deep
// chains (one edge's union took ~30 us over HBM at N = 18000); random linking keeps the trees
// shallow in expectation.  A component's root is its node of least priority: still one
// canonical label per node set, so the layers' partitions compare root for root.
__device__ __forceinline__ unsigned uf_pri(int x) { return (unsigned)x * 2654435761u; }
template <class P>
__device__ __forceinline__ int uf_find_h(P par, int v) {
  int cur = uf_load(par, v);
  if (cur != v) {
    int prev = v, next;
    while (cur != (next = uf_load(par, cur))) {
      uf_store(par, prev, next);  // path halving; any ancestor is a valid parent
      prev = cur;
      cur = next;
    }
  }
  return cur;
}
template <class P>
__device__ __forceinline__ void uf_unite_h(P par, int a, int b) {
  while (true) {
    a = uf_find_h(par, a);
    b = uf_find_h(par, b);
    if (a == b) return;
    if (uf_pri(a) > uf_pri(b)) { const int t = a; a = b; b = t; }
    if (uf_cas(par, b, b, a) == b) return;
  }
}
// Union by a static rank (rk, LDS): node x's position when the graph's nodes are ordered by
// descending static degree (both layers), ties by uf_pri.  A hub is the root of its tree from its
// first union on, so its neighbours hook under it with a compare-and-swap on their OWN parent
// word: with the hashed priority, a hub's root was in turn the larger-priority side of many
// concurrent unions, every one retrying its compare-and-swap on that one word (the union pass's
// stragglers at N = 18 000).  Roots are still one canonical node per node set (the least rank),
// the same in both layers.
// Both endpoints' paths are climbed in lockstep: one round trip per hop serves both
// climbs (two independent device-coherent loads in flight instead of two dependent find loops),
// path splitting on the way; two roots: the lower-ranked one is hooked under the other (a
// failed compare-and-swap re-reads); paths that meet stop.
// (CNT: diagnostics, the round trips in *ops -- a hop's two loads count once -- and the failed
// compare-and-swaps in *fails)
template <bool CNT = false, class P>
__device__ __forceinline__ void uf_unite_r2(P par, int a, int b, const lds_u16* rk, int* ops = nullptr,
                                            int* fails = nullptr) {
  int ap = -1, bp = -1;
  while (a != b) {
    const int na = uf_load(par, a), nb = uf_load(par, b);
    if (CNT) ++*ops;
    if (na == a && nb == b) {
      const bool sw = rk[a] > rk[b];
      const int hi = sw ? a : b, lo = sw ? b : a;  // hi: the root of lower rank (larger value)
      if (CNT) ++*ops;
      if (uf_cas(par, hi, hi, lo) == hi) return;
      if (CNT) ++*fails;
      continue;
    }
    if (na != a) {
      if (ap >= 0) uf_store(par, ap, na);
      ap = a;
      a = na;
    }
    if (nb != b) {
      if (bp >= 0) uf_store(par, bp, nb);
      bp = b;
      b = nb;
    }
  }
}
// the roots of x in both layers' parent arrays, the two climbs in lockstep (path halving)
template <class P>
__device__ __forceinline__ int2 uf_find2_h(P p0, P p1, int x) {
  int a = x, b = x, qa = -1, qb = -1;
  while (true) {
    const int na = uf_load(p0, a), nb = uf_load(p1, b);
    if (na == a && nb == b) return make_int2(a, b);
    if (na != a) {
      if (qa >= 0) uf_store(p0, qa, na);  // halving: qa's parent was a
      qa = a;
      a = na;
    }
    if (nb != b) {
      if (qb >= 0) uf_store(p1, qb, nb);
      qb = b;
      b = nb;
    }
  }
}
// ------------------------------------------------------------------ layout and view
// LDS layout of a graph's environment (words from the start of the phase-A area): the edge
// region first (u16 endpoints, state, state at the last write-back, covered flags) so a
// dedicated environment workgroup keeps it across steps, then union-find / degree arrays,
// the reduction temp and the first-layer-table scratch.
struct EnvLayout {
  int ew;                        // words of the edge region
  int cov;                       // byte offset of the covered flags
  int al0, al1, dl;              // byte offsets of the alive-edge lists (ping-pong) and the dead list
  int hdr;                       // word offset of {alive count, dead count, current list}
  int par0, par1, deg0, deg1, tmp, rp, total;
};
__host__ __device__ inline EnvLayout env_layout(int n, int et) {
  EnvLayout L;
  const int e8 = (et + 7) & ~7, e16 = (et + 15) & ~15;
  L.cov = 4 * e8 + e16;                       // u16 u, u16 v, u8 state
  L.al0 = L.cov + ((n + 15) & ~15);           // u16 edge ids
  L.al1 = L.al0 + 2 * e8;
  L.dl = L.al1 + 2 * e8;
  const int eb = L.dl + 2 * e8;
  L.ew = ((eb + 15) / 16) * 4;
  L.hdr = L.ew;
  L.par0 = L.hdr + 4;
  L.par1 = L.par0 + n;
  L.deg0 = L.par1 + n;
  L.deg1 = L.deg0 + n;
  L.tmp = ((L.deg1 + n + 3) / 4) * 4;
  L.rp = L.tmp + A_TMP_WORDS;                 // static CSR row pointers of both layers, n + 1 each
  L.total = L.rp + 2 * (n + 1);
  return L;
}
__host__ __device__ inline bool phase_a_fits_lds(int n, int et) {
  return env_layout(n, et).total <= A_WORDS && n <= 65535;
}

// Edge arrays of one graph: LDS-staged (u16 endpoints) or the global arrays themselves.
template <bool GL>
struct EnvView {
  typedef typename std::conditional<GL, int*, lds_i32*>::type IP;
  const GraphInfo* gi;
  int e0, et;                   // edges of layer 0, both layers
  int variant;
  lds_u16* u16;                 // LDS mode: endpoints [et]
  lds_u16* v16;
  lds_u8* st;                   // LDS mode: edge states [et]
  lds_u8* cov8;                 // LDS mode: covered flags [n]
  lds_u16* al;                  // LDS mode: alive edge ids (current list, al_n() entries)
  lds_u16* al_other;            //           the other half of the ping-pong pair
  lds_u16* dl;                  //           edges killed since the last write-back
  lds_i32* hdr;                 //           {alive count, dead count, current list 0/1}
  const int* gu[2];             // global mode
  const int* gv[2];
  uint8_t* gst[2];
  uint8_t* gcov;                // covered flags in HBM (both modes keep them current)
  IP par0, par1, deg0, deg1;    // union-find parents / labels, degrees
  int* tmp;                     // always LDS (generic pointer for the block helpers)
  uint8_t* calive[2];
  const int* epos[2];
  const int* grp[2];            // static CSR row pointers (global)
  lds_i32* rp[2];               // LDS mode: their staged copy

  __device__ __forceinline__ int layer_of(int e) const { return e < e0 ? 0 : 1; }
  __device__ __forceinline__ int local(int e) const { return e < e0 ? e : e - e0; }
  __device__ __forceinline__ int u(int e) const {
    if constexpr (GL) return gu[layer_of(e)][local(e)]; else return u16[e];
  }
  __device__ __forceinline__ int v(int e) const {
    if constexpr (GL) return gv[layer_of(e)][local(e)]; else return v16[e];
  }
  __device__ __forceinline__ int state(int e) const {
    if constexpr (GL) return ldc(gst[layer_of(e)] + local(e)); else return st[e];
  }
  __device__ __forceinline__ int covered(int x) const {
    if constexpr (GL) return ldc(gcov + x); else return cov8[x];
  }
  // alive -> dead transition (the LDS mode writes back at the end of phase A)
  __device__ __forceinline__ void kill(int e, uint8_t s) const {
    if constexpr (GL) {
      const int l = layer_of(e), k = local(e);
      stc(gst[l] + k, s);
      stc(calive[l] + epos[l][2 * k], (uint8_t)0);
      stc(calive[l] + epos[l][2 * k + 1], (uint8_t)0);
    } else {
      st[e] = s;
    }
  }
};

__device__ __forceinline__ unsigned sel4(const v4u& w, int i) {
  return i == 0 ? w.x : i == 1 ? w.y : i == 2 ? w.z : w.w;
}

// Visits this thread's edges: f(e, u, v, state).  LDS mode reads eight edges per vector load
// (edge groups g = tid, tid + NTHREADS, ...).
template <bool GL, class F>
__device__ __forceinline__ void for_each_edge(const EnvView<GL>& E, F&& f) {
  if constexpr (GL) {
    for (int e = threadIdx.x; e < E.et; e += NTHREADS) f(e, E.u(e), E.v(e), E.state(e));
  } else {
    const int ng = (E.et + 7) >> 3;
    for (int g = threadIdx.x; g < ng; g += NTHREADS) {
      const v4u U = ((const lds_u4*)E.u16)[g];
      const v4u V = ((const lds_u4*)E.v16)[g];
      const v2u S = ((const lds_u2*)E.st)[g];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int e = 8 * g + k;
        if (e >= E.et) break;
        const unsigned uw = sel4(U, k >> 1), vw = sel4(V, k >> 1), sw = k < 4 ? S.x : S.y;
        f(e, (int)((uw >> (16 * (k & 1))) & 0xffffu), (int)((vw >> (16 * (k & 1))) & 0xffffu),
          (int)((sw >> (8 * (k & 3))) & 0xffu));
      }
    }
  }
}

// ------------------------------------------------------------------ block reductions (fused)
// Sums of two ints over the block.  Leading barrier only: the caller must pass another
// __syncthreads before tmp is written again (every helper here starts with one).
__device__ __forceinline__ int2 block_sum2(int a, int b, int* tmp) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  __syncthreads();
  lds_i32* t = (lds_i32*)tmp;
  if (lane_id() == 0) {
    t[2 * wave_id()] = a;
    t[2 * wave_id() + 1] = b;
  }
  __syncthreads();
  int2 r = make_int2(0, 0);
#pragma unroll
  for (int w = 0; w < NTHREADS / 64; ++w) {
    r.x += t[2 * w];
    r.y += t[2 * w + 1];
  }
  return r;
}

// Sums of four ints over the block (leading barrier only, as block_sum2).
__device__ __forceinline__ int4 block_sum4(int a, int b, int c, int d, int* tmp) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
    c += __shfl_xor(c, o, 64);
    d += __shfl_xor(d, o, 64);
  }
  __syncthreads();
  lds_i32* t = (lds_i32*)tmp;
  if (lane_id() == 0) {
    t[4 * wave_id()] = a;
    t[4 * wave_id() + 1] = b;
    t[4 * wave_id() + 2] = c;
    t[4 * wave_id() + 3] = d;
  }
  __syncthreads();
  int4 r = make_int4(0, 0, 0, 0);
#pragma unroll
  for (int w = 0; w < NTHREADS / 64; ++w) {
    r.x += t[4 * w];
    r.y += t[4 * w + 1];
    r.z += t[4 * w + 2];
    r.w += t[4 * w + 3];
  }
  return r;
}

// ------------------------------------------------------------------ alive-edge list
// LDS mode keeps the ids of the alive edges in a compact list (edges only die during a
// rollout), so the per-step passes -- cover, unions, prune, degrees -- touch the alive edges
// only and every lane of a wave has work; the edges killed since the last write-back are kept
// in the dead list.  Global mode scans all edges.
template <bool GL, class F>
__device__ __forceinline__ void for_each_alive(const EnvView<GL>& E, F&& f) {
  if constexpr (GL) {
    for (int e = threadIdx.x; e < E.et; e += NTHREADS)
      if (E.state(e) == E_ALIVE) f(e, E.u(e), E.v(e));
  } else {
    const int na = E.hdr[0];
    const lds_u16* al = E.hdr[2] ? E.al_other : E.al;
    for (int i = threadIdx.x; i < na; i += NTHREADS) {
      const int e = al[i];
      if (E.st[e] == E_ALIVE) f(e, (int)E.u16[e], (int)E.v16[e]);
    }
  }
}

// Union-pass order: in LDS mode every thread takes a contiguous run of the alive list, so the
// edges in flight at one time are spread over the graph (few threads contend for the same
// roots) while each thread's consecutive edges share endpoints (short, compressed paths).
template <bool GL, class F>
__device__ __forceinline__ void for_each_alive_runs(const EnvView<GL>& E, F&& f) {
  if constexpr (GL) {
    for_each_alive<GL>(E, f);
  } else {
    const int na = E.hdr[0];
    const lds_u16* al = E.hdr[2] ? E.al_other : E.al;
    const int chunk = (na + NTHREADS - 1) / NTHREADS;
    const int i0 = min(na, (int)threadIdx.x * chunk), i1 = min(na, i0 + chunk);
    for (int i = i0; i < i1; ++i) {
      const int e = al[i];
      if (E.st[e] == E_ALIVE) f(e, (int)E.u16[e], (int)E.v16[e]);
    }
  }
}

// Builds the alive list from the staged edge states (ascending edge ids).
template <bool GL>
__device__ void build_alive(const EnvView<GL>& E) {
  if constexpr (!GL) {
    const int chunk = (E.et + NTHREADS - 1) / NTHREADS;
    const int e0 = min(E.et, (int)threadIdx.x * chunk), e1 = min(E.et, e0 + chunk);
    int keep = 0;
    for (int e = e0; e < e1; ++e) keep += E.st[e] == E_ALIVE;
    int tot = 0;
    int k = block_excl_scan(keep, E.tmp, &tot);
    for (int e = e0; e < e1; ++e)
      if (E.st[e] == E_ALIVE) E.al[k++] = (uint16_t)e;
    __syncthreads();
    if (threadIdx.x == 0) {
      E.hdr[0] = tot;
      E.hdr[1] = 0;
      E.hdr[2] = 0;
    }
    __syncthreads();
  }
}

// Drops the entries whose edge died from the alive list (kept entries stay in order) and
// appends them to the dead list.
template <bool GL>
__device__ void compact_alive(const EnvView<GL>& E) {
  if constexpr (!GL) {
    const int na = E.hdr[0], nd0 = E.hdr[1], cur = E.hdr[2];
    const lds_u16* src = cur ? E.al_other : E.al;
    lds_u16* dst = cur ? E.al : E.al_other;
    const int chunk = (na + NTHREADS - 1) / NTHREADS;
    const int i0 = min(na, (int)threadIdx.x * chunk), i1 = min(na, i0 + chunk);
    int keep = 0;
    for (int i = i0; i < i1; ++i) keep += E.st[src[i]] == E_ALIVE;
    int totk = 0, totd = 0;
    int k = block_excl_scan(keep, E.tmp, &totk);
    int d = nd0 + block_excl_scan(i1 - i0 - keep, E.tmp, &totd);
    for (int i = i0; i < i1; ++i) {
      const int e = src[i];
      if (E.st[e] == E_ALIVE) dst[k++] = (uint16_t)e;
      else E.dl[d++] = (uint16_t)e;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      E.hdr[0] = totk;
      E.hdr[1] = nd0 + totd;
      E.hdr[2] = 1 - cur;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ mutual LMCC
// Mutual-LMCC fixed point (U/Mcc.py:30-38) on the alive edges.  Both layers' components are
// found simultaneously; while the partitions differ, every alive edge of a layer that crosses
// the other layer's partition is pruned (both layers per round).  The fixed point (the
// coarsest partition connected in both layers) and the pruned-edge set equal the reference's
// alternating order.  Returns the LMCC size (over non-covered nodes); pruned counts in pr[2].
// Component labels (root ids) go to the degree arrays, free until after the fixed point: a
// path-halving find may rewrite a parent slot with a non-root ancestor after its owner stored
// the root, so the parent array itself is not a label map.
// `cover` >= 0: first cover that node (U/mvc_env.py:74-85) inside the first union pass -- its
// alive edges become covered instead of being united -- and return the covered edge counts
// per layer in cc[2].
// Confirmation shortcut (LDS mode; MD_FP_SHORTCUT=0: off): a round whose partitions differ is
// normally followed by one more union round, often only to confirm that the pruned partition
// P = C0 ^ C1 is connected in both layers.  The union pass records which alive edges linked two
// trees (a spanning forest F_l of each layer: |F_l| = n - #C_l); after the prune, F_l minus its
// t_l pruned edges is a forest whose n - |F_l| + t_l pieces each lie inside one class of P, so
// when #C_l + t_l == #P for both layers every class of P is connected in both layers by
// surviving edges: P is the fixed point and no edge crosses it unpruned -- the same result the
// next round would confirm.  #P counts the distinct (C0, C1) label pairs through an LDS hash
// table in the parent arrays (free between the label pass and the next round), whose slots
// then label P for the LMCC count.
// Speculative workgroups (spec_loop): the fixed point of a request's candidate stops after a
// round once the result cannot be used -- phase A's early word names another result of the same
// request, or a later request is out -- so a workgroup stuck in a long cascade is free for the
// next request sooner.  Returns -1 then (the LDS state is partial).
struct SpecAbort {
  const unsigned long long* ew;   // phase A's early word
  const unsigned long long* ew2;  // tile 0's derivation of it (nullptr: none)
  const unsigned long long* req;  // the request word
  unsigned tag;                   // this request's tag
  int slot;                       // this workgroup's result slot (parity included)
  int step;                       // this request's step
};
template <bool GL>
__device__ __forceinline__ int mcc_fixed_point(const EnvView<GL>& Ein, int* pr, unsigned long long* acc, int cover, int* cc,
                               const SpecAbort* ab = nullptr) {
  const EnvView<GL> E = Ein;  // fields in registers
  const int n = E.gi->n;
  int pruned0 = 0, pruned1 = 0;
  if (acc != nullptr && threadIdx.x == 0) acc[PA_CALLS] += 1;
  bool first = true, dirty = cover >= 0;  // dead entries in the alive list
  bool skipped = false;                   // ended by the confirmation shortcut (labels: table slots in deg1)
  const bool shortcut = !GL && kp().fp_short;
  // Unchanged layers (LDS mode; MD_FP_SKIP=0: off): a layer none of whose edges the last prune
  // removed has the same alive edges, hence the same components, labels and spanning forest as
  // in the last round -- its union and label work is skipped, and so is pruning the other
  // layer's edges by it (every edge crossing its partition went in that prune).  ch0 / ch1:
  // the layer's edge set changed since its last union pass (the shortcut's table overwrites
  // both parent arrays and layer 1's labels: a failed check marks layer 1 changed).  The
  // alive list is in ascending edge id, so a layer's entries are one range ([0, na0) layer 0).
  const bool lskip = !GL && kp().fp_skip;
  bool ch0 = true, ch1 = true;
  int na0 = -1;  // layer 0's alive-list entries (found at the first skip)
  unsigned long long ab_ew = 0ull, ab_ew2 = 0ull, ab_req = 0ull;  // thread 0: loaded during the previous round's prune
  while (true) {
    unsigned long long tp = wall_clock64();
    if (acc != nullptr && threadIdx.x == 0) acc[PA_ROUNDS] += 1;
    if constexpr (!GL) {
      if (ab != nullptr && !first && threadIdx.x == 0) {
        const bool taken_elsewhere = ((unsigned)(ab_ew >> 32) == ab->tag && (int)(ab_ew & 0xffffu) != ab->slot) ||
                                     ((unsigned)(ab_ew2 >> 32) == ab->tag && (int)(ab_ew2 & 0xffffu) != ab->slot);
        const bool newer = ab_req != 0ull && ab_req != SPEC_EXIT && (int)(unsigned)(ab_req >> 32) > ab->step;
        E.hdr[3] = (taken_elsewhere || newer) ? 1 : 0;
      }
    }
    for (int x = threadIdx.x; x < n; x += NTHREADS) {
      if (ch0) uf_store(E.par0, x, x);
      if (ch1) uf_store(E.par1, x, x);
    }
    __syncthreads();
    if constexpr (!GL) {
      if (ab != nullptr && !first && E.hdr[3] != 0) return -1;
      if (!(ch0 && ch1) && na0 < 0) {
        // (every thread the same bisection: the first entry of layer 1)
        const lds_u16* al = E.hdr[2] ? E.al_other : E.al;
        int lo = 0, hi = E.hdr[0];
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if ((int)al[mid] < E.e0) lo = mid + 1;
          else hi = mid;
        }
        na0 = lo;
      }
    }
    PACC(acc, PA_INIT, tp);
    int k0 = 0, k1 = 0;
    const bool cv = first && cover >= 0;
    if constexpr (!GL) {
      // the union pass over contiguous runs of the alive list (for_each_alive_runs), recording
      // per list position whether the edge linked two trees (the other alive-list buffer is free
      // until the final compaction)
      const int na = E.hdr[0];
      const lds_u16* al = E.hdr[2] ? E.al_other : E.al;
      lds_u8* tf = (lds_u8*)(E.hdr[2] ? E.al : E.al_other);
      // (the changed layers' range of the list; a skipped layer keeps its forest flags)
      const int ra = ch0 ? 0 : na0, rb = ch1 ? na : na0;
      const int chunk = (rb - ra + NTHREADS - 1) / NTHREADS;
      const int i0 = min(rb, ra + (int)threadIdx.x * chunk), i1 = min(rb, i0 + chunk);
#ifdef MD_UNION_PIPE
      // diagnostic variant (timing perturbation only): the next entry's id, state and endpoints
      // loaded one step ahead
      int e_n = i0 < i1 ? (int)al[i0] : 0;
      int s_n = i0 < i1 ? (int)E.st[e_n] : 0, u_n = i0 < i1 ? (int)E.u16[e_n] : 0, v_n = i0 < i1 ? (int)E.v16[e_n] : 0;
      for (int i = i0; i < i1; ++i) {
        const int e = e_n, s = s_n, u = u_n, v = v_n;
        if (i + 1 < i1) {
          e_n = al[i + 1];
          s_n = E.st[e_n];
          u_n = E.u16[e_n];
          v_n = E.v16[e_n];
        }
        if (s != E_ALIVE) continue;
#else
      for (int i = i0; i < i1; ++i) {
        const int e = al[i];
        if (E.st[e] != E_ALIVE) continue;
        const int u = (int)E.u16[e], v = (int)E.v16[e];
#endif
        if (cv && (u == cover || v == cover)) {
          E.kill(e, E_COVERED);
          if (e < E.e0) k0++; else k1++;
        } else {
          const bool lk = uf_link(e < E.e0 ? E.par0 : E.par1, u, v);
          if (shortcut) tf[i] = lk ? 1 : 0;
        }
      }
    } else if (cv) {
      for_each_alive_runs<GL>(E, [&](int e, int u, int v) {
        if (u == cover || v == cover) {
          E.kill(e, E_COVERED);
          if (e < E.e0) k0++; else k1++;
        } else {
          uf_unite(e < E.e0 ? E.par0 : E.par1, u, v);
        }
      });
    } else {
      for_each_alive_runs<GL>(E, [&](int e, int u, int v) { uf_unite(e < E.e0 ? E.par0 : E.par1, u, v); });
    }
    __syncthreads();
    PACC(acc, PA_UNITE, tp);
    if (acc != nullptr && (E.variant & 8)) {
      // diagnostics: alive edges per round
      int ne = 0;
      for_each_alive<GL>(E, [&](int, int, int) { ne++; });
      // depth of every node in the union-find forest after the union pass
      int dsum = 0;
      for (int x = threadIdx.x; x < n; x += NTHREADS) {
        for (int l = 0; l < 2; ++l) {
          auto par = l ? E.par1 : E.par0;
          int c = x, d = 0;
          while (uf_load(par, c) != c) { c = uf_load(par, c); ++d; }
          dsum += d;
        }
      }
      const int2 c = block_sum2(ne, dsum, E.tmp);
      if (threadIdx.x == 0) {
        acc[PA_EDGES] += c.x;
        acc[PA_FINDONLY] += c.y;
      }
    }
    tp = wall_clock64();
    int diff = 0, nr0 = 0, nr1 = 0;
    for (int x = threadIdx.x; x < n; x += NTHREADS) {
      const int r0 = ch0 ? uf_find(E.par0, x) : uf_load(E.deg0, x);
      const int r1 = ch1 ? uf_find(E.par1, x) : uf_load(E.deg1, x);
      if (ch0) uf_store(E.deg0, x, r0);
      if (ch1) uf_store(E.deg1, x, r1);
      diff |= (r0 != r1);
      nr0 += r0 == x;  // components per layer (their roots)
      nr1 += r1 == x;
    }
    int nc0 = 0, nc1 = 0;
    if (cv) {
      // covered-edge counts, the component counts and the partition test in one block exchange
      // (per layer at most n - 1 < 2^16 covered edges and n < 2^16 roots; at most 512 threads
      // with diff set)
      const int4 c = block_sum4(k0, k1, nr0, nr1 + (diff ? 1 << 16 : 0), E.tmp);
      cc[0] = c.x;
      cc[1] = c.y;
      nc0 = c.z;
      nc1 = c.w & 0xffff;
      diff = (c.w >> 16) != 0;
    } else if (shortcut) {
      const int2 c = block_sum2(nr0, nr1 + (diff ? 1 << 16 : 0), E.tmp);
      nc0 = c.x;
      nc1 = c.y & 0xffff;
      diff = (c.y >> 16) != 0;
    } else {
      diff = __syncthreads_or(diff);
    }
    first = false;
    PACC(acc, PA_LABEL, tp);
    tp = wall_clock64();
    if (!diff) {
      // the covered / pruned edges leave the alive list for the dead list once, at the end
      // (later rounds skip them by their state)
      if (dirty) compact_alive<GL>(E);
      break;
    }
    int c0 = 0, c1 = 0, t0 = 0, t1 = 0;
    if constexpr (!GL) {
      if (ab != nullptr && threadIdx.x == 0) {  // (used at the next round's start)
        ab_ew = __hip_atomic_load((const g_u64*)ab->ew, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ab_req = __hip_atomic_load((const g_u64*)ab->req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ab->ew2 != nullptr) ab_ew2 = __hip_atomic_load((const g_u64*)ab->ew2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      // the prune pass (for_each_alive's order), counting the pruned spanning-forest edges
      const int na = E.hdr[0];
      const lds_u16* al = E.hdr[2] ? E.al_other : E.al;
      const lds_u8* tf = (const lds_u8*)(E.hdr[2] ? E.al : E.al_other);
      // (layer-0 edges only when layer 1's labels were redone this round, and vice versa)
      const int ra = ch1 ? 0 : na0, rb = ch0 ? na : na0;
      for (int i = ra + (int)threadIdx.x; i < rb; i += NTHREADS) {
        const int e = al[i];
        if (E.st[e] != E_ALIVE) continue;
        const int u = (int)E.u16[e], v = (int)E.v16[e];
        auto other = e < E.e0 ? E.deg1 : E.deg0;  // layer-0 edges are pruned by layer-1 components
        if (uf_load(other, u) != uf_load(other, v)) {
          E.kill(e, E_PRUNED);
          const int f = shortcut ? (int)tf[i] : 0;
          if (e < E.e0) { c0++; t0 += f; } else { c1++; t1 += f; }
        }
      }
    } else {
      for_each_alive<GL>(E, [&](int e, int u, int v) {
        auto other = e < E.e0 ? E.deg1 : E.deg0;
        if (uf_load(other, u) != uf_load(other, v)) {
          E.kill(e, E_PRUNED);
          if (e < E.e0) c0++; else c1++;
        }
      });
    }
    const int4 c = block_sum4(c0, c1, t0, t1, E.tmp);
    pruned0 += c.x;
    pruned1 += c.y;
    dirty = true;
    if (lskip) {
      ch0 = c.x > 0;
      ch1 = c.y > 0;
    }
    PACC(acc, PA_PRUNE, tp);
    if constexpr (!GL) {
      // confirmation shortcut (see above): #C0 + t0 == #C1 + t1 is necessary; then count the
      // classes of P = C0 ^ C1 (distinct label pairs) in a hash table over both parent arrays
      if (shortcut && nc0 + c.z == nc1 + c.w) {
        auto ht = E.par0;  // par0, par1: 2n words, contiguous (env_layout)
        const unsigned hs = 2u * (unsigned)n;
        for (int x = threadIdx.x; x < 2 * n; x += NTHREADS) uf_store(ht, x, -1);
        __syncthreads();
        int np = 0;
        for (int x = threadIdx.x; x < n; x += NTHREADS) {
          const int key = (int)(((unsigned)uf_load(E.deg0, x) << 16) | (unsigned)uf_load(E.deg1, x));
          unsigned h = ((unsigned)key * 2654435761u) % hs;
          while (true) {
            const int old = uf_cas(ht, (int)h, -1, key);
            if (old == -1) { np++; break; }
            if (old == key) break;
            h = h + 1u == hs ? 0u : h + 1u;
          }
          uf_store(E.deg1, x, (int)h);  // x's class of P: its table slot (only this thread reads deg1[x] here)
        }
        const int2 q = block_sum2(np, 0, E.tmp);
        if (nc0 + c.z == q.x && nc1 + c.w == q.x) {
          skipped = true;
          compact_alive<GL>(E);
          break;
        }
        ch1 = true;  // (its labels hold table slots now; layer 0 keeps its labels in deg0)
        __syncthreads();  // (the next round's init overwrites the table)
      }
    }
  }
  const unsigned long long tc = wall_clock64();
  pr[0] = pruned0;
  pr[1] = pruned1;
  int best = 0;
  if (skipped) {
    // LMCC over the classes of P: sizes by table slot (deg1), in the table's words
    auto ht = E.par0;
    for (int x = threadIdx.x; x < 2 * n; x += NTHREADS) uf_store(ht, x, 0);
    __syncthreads();
    for (int x = threadIdx.x; x < n; x += NTHREADS)
      if (!E.covered(x)) uf_add(ht, uf_load(E.deg1, x), 1);
    __syncthreads();
    for (int x = threadIdx.x; x < 2 * n; x += NTHREADS) best = max(best, uf_load(ht, x));
  } else {
    for (int x = threadIdx.x; x < n; x += NTHREADS) uf_store(E.par1, x, 0);
    __syncthreads();
    for (int x = threadIdx.x; x < n; x += NTHREADS)
      if (!E.covered(x)) uf_add(E.par1, uf_load(E.deg0, x), 1);
    __syncthreads();
    for (int x = threadIdx.x; x < n; x += NTHREADS) best = max(best, uf_load(E.par1, x));
  }
  best = block_max_int(best, E.tmp);
  PACC(acc, PA_COUNT, tc);
  return best;
}

// Aggregates of one environment state (U/PrepareBatchGraph.py:35-74).
struct EnvAgg {
  int nlive, dm0, dm1, sd0, sd1, bad;
  long long th0, th1;
  int cand;  // (qs given) the live node of largest previous Q, least id first; -1 none
};

// Block arg-max of (v, i) pairs: the largest v, the least i among equal v; -1 when no thread
// has a finite v.  All threads get the result.
__device__ __forceinline__ int block_argmax_f(float v, int i, int* tmp) {
  const int lane = lane_id(), w = wave_id();
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float v2 = __shfl_xor(v, o, 64);
    const int i2 = __shfl_xor(i, o, 64);
    if (v2 > v || (v2 == v && i2 < i)) {
      v = v2;
      i = i2;
    }
  }
  __syncthreads();
  if (lane == 0) {
    tmp[2 * w] = __float_as_int(v);
    tmp[2 * w + 1] = i;
  }
  __syncthreads();
  float bv = NEG_INF;
  int bi = -1;
#pragma unroll
  for (int k = 0; k < NTHREADS / 64; ++k) {
    const float v2 = __int_as_float(tmp[2 * k]);
    const int i2 = tmp[2 * k + 1];
    if (v2 > bv || (v2 == bv && i2 < bi && i2 >= 0)) {
      bv = v2;
      bi = i2;
    }
  }
  __syncthreads();
  return bv > NEG_INF ? bi : -1;
}

// Residual degrees (edge-parallel atomics over the alive edges), then the ascending live list,
// the degrees and the per-layer aggregates of the current state, stored to (gdeg0, gdeg1, lv)
// -- the graph's HBM arrays (phase A) or a speculative result slot -- and q = -inf for every
// node when q is given.  One fused block exchange for the scan and all reductions.
template <bool GL>
__device__ __forceinline__ EnvAgg env_features(const EnvView<GL>& E, int n, int* gdeg0, int* gdeg1, float* lv, float* q,
                                               const float* qs = nullptr) {
  const int e0 = E.e0;
  // residual degrees by edge-parallel atomics
  for (int x = threadIdx.x; x < n; x += NTHREADS) {
    uf_store(E.deg0, x, 0);
    uf_store(E.deg1, x, 0);
  }
  __syncthreads();
  for_each_alive<GL>(E, [&](int e, int u, int v) {
    auto d = e < e0 ? E.deg0 : E.deg1;
    uf_add(d, u, 1);
    uf_add(d, v, 1);
  });
  __syncthreads();
  // live list (ascending ids), per-layer aggregates (U/PrepareBatchGraph.py:35-74): one
  // fused block exchange for the scan and all reductions
  const int chunk = (n + NTHREADS - 1) / NTHREADS;
  const int x0 = min(n, (int)threadIdx.x * chunk), x1 = min(n, x0 + chunk);
  int nlive = 0, dm0 = 0, dm1 = 0, sd0 = 0, sd1 = 0, bad = 0;
  long long th0 = 0, th1 = 0;
  float cq = NEG_INF;
  int ci = -1;
  for (int x = x0; x < x1; ++x) {
    const int d0 = uf_load(E.deg0, x), d1 = uf_load(E.deg1, x);
    stc(gdeg0 + x, d0);
    stc(gdeg1 + x, d1);
    if (q != nullptr) stc(q + x, NEG_INF);
    if (qs != nullptr && d0 > 0 && qs[x] > cq) {  // ascending x: the least id keeps a tie
      cq = qs[x];
      ci = x;
    }
    bad |= ((d0 > 0) != (d1 > 0));
    if (d0 > 0) {
      nlive++;
      dm0 = max(dm0, d0);
      dm1 = max(dm1, d1);
      th0 += (long long)d0 * (d0 - 1) / 2;
      th1 += (long long)d1 * (d1 - 1) / 2;
    }
    sd0 += d0;
    sd1 += d1;
  }
  int tot = 0, base = 0;
  {
    const int lane = lane_id(), w = wave_id();
    int incl = nlive;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    int r_nl = nlive, r_m0 = dm0, r_m1 = dm1, r_s0 = sd0, r_s1 = sd1, r_bad = bad;
    long long r_t0 = th0, r_t1 = th1;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      r_nl += __shfl_xor(r_nl, o, 64);
      r_m0 = max(r_m0, __shfl_xor(r_m0, o, 64));
      r_m1 = max(r_m1, __shfl_xor(r_m1, o, 64));
      r_s0 += __shfl_xor(r_s0, o, 64);
      r_s1 += __shfl_xor(r_s1, o, 64);
      r_bad |= __shfl_xor(r_bad, o, 64);
      r_t0 += __shfl_xor(r_t0, o, 64);
      r_t1 += __shfl_xor(r_t1, o, 64);
    }
    __syncthreads();
    lds_i32* t = (lds_i32*)E.tmp;  // 12 words per wave
    if (lane == 0) {
      t[12 * w + 0] = r_nl;
      t[12 * w + 1] = r_m0;
      t[12 * w + 2] = r_m1;
      t[12 * w + 3] = r_s0;
      t[12 * w + 4] = r_s1;
      t[12 * w + 5] = r_bad;
      t[12 * w + 6] = (int)(r_t0 & 0xffffffffll);
      t[12 * w + 7] = (int)(r_t0 >> 32);
      t[12 * w + 8] = (int)(r_t1 & 0xffffffffll);
      t[12 * w + 9] = (int)(r_t1 >> 32);
    }
    __syncthreads();
    dm0 = dm1 = sd0 = sd1 = bad = 0;
    th0 = th1 = 0;
    int before = 0;
#pragma unroll
    for (int i = 0; i < NTHREADS / 64; ++i) {
      const int nl_i = t[12 * i];
      if (i < w) before += nl_i;
      tot += nl_i;
      dm0 = max(dm0, (int)t[12 * i + 1]);
      dm1 = max(dm1, (int)t[12 * i + 2]);
      sd0 += t[12 * i + 3];
      sd1 += t[12 * i + 4];
      bad |= t[12 * i + 5];
      th0 += (long long)(((unsigned long long)(unsigned)t[12 * i + 7] << 32) | (unsigned)t[12 * i + 6]);
      th1 += (long long)(((unsigned long long)(unsigned)t[12 * i + 9] << 32) | (unsigned)t[12 * i + 8]);
    }
    base = before + incl - nlive;
  }
  {
    // live list entries {node, CSR begin layer 0, layer 1, CSR extents (u16 | u16 << 16)}: a tile
    // reads its rows and their neighbour ranges with one 16-byte load each
    int k = base;
    for (int x = x0; x < x1; ++x) {
      if (uf_load(E.deg0, x) > 0) {
        int b0, e0_, b1, e1_;
        if constexpr (GL) {
          b0 = E.grp[0][x]; e0_ = E.grp[0][x + 1]; b1 = E.grp[1][x]; e1_ = E.grp[1][x + 1];
        } else {
          b0 = E.rp[0][x]; e0_ = E.rp[0][x + 1]; b1 = E.rp[1][x]; e1_ = E.rp[1][x + 1];
        }
        if (MD_BOK(k < n, 9))
          stc4(lv, k * 16, make_float4(__int_as_float(x), __int_as_float(b0), __int_as_float(b1),
                                       __int_as_float((e0_ - b0) | ((e1_ - b1) << 16))));
        ++k;
      }
    }
  }

  EnvAgg ag;
  ag.nlive = tot;
  ag.dm0 = dm0;
  ag.dm1 = dm1;
  ag.sd0 = sd0;
  ag.sd1 = sd1;
  ag.bad = bad;
  ag.th0 = th0;
  ag.th1 = th1;
  ag.cand = qs != nullptr ? block_argmax_f(cq, ci, E.tmp) : -1;
  return ag;
}

// Phase A's copy of a speculative slot's degrees, live list and aggregates (env_features of
// the same state) to the graph's HBM arrays; q = -inf for every node.
// (ld0, ld1: the degrees also into the LDS degree arrays, for the neighbour-list builder)
__device__ __forceinline__ EnvAgg env_copy_features(const int* slot, int n, int et, int* gdeg0, int* gdeg1, float* lv,
                                                    float* q, const float* qs = nullptr, int* tmp = nullptr,
                                                    lds_i32* ld0 = nullptr, lds_i32* ld1 = nullptr) {
  const int* sd = slot + sres_deg(et);
  const float* sl = (const float*)(slot + sres_live(et, n));
  // every load in one round trip: the header words, the degrees and the live entries up to n
  // (the first n_live of them are used)
  int h[10];
#pragma unroll
  for (int i = 0; i < 10; ++i) h[i] = ldc(slot + 12 + i);
  constexpr int U = 4;
  int d0[U], d1[U];
  float4 le[U];
  float cq = NEG_INF;
  int ci = -1;
  for (int x0 = threadIdx.x; x0 < n; x0 += U * NTHREADS) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int x = x0 + u * NTHREADS;
      if (x < n) {
        d0[u] = ldc(sd + x);
        d1[u] = ldc(sd + n + x);
        le[u] = ldc4(sl, x * 16);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int x = x0 + u * NTHREADS;
      if (x < n) {
        stc(gdeg0 + x, d0[u]);
        stc(gdeg1 + x, d1[u]);
        if (ld0 != nullptr) {
          uf_store(ld0, x, d0[u]);
          uf_store(ld1, x, d1[u]);
        }
        stc(q + x, NEG_INF);
        if (x < h[0]) stc4(lv, x * 16, le[u]);
        if (qs != nullptr && d0[u] > 0 && (qs[x] > cq || (qs[x] == cq && x < ci))) {
          cq = qs[x];
          ci = x;
        }
      }
    }
  }
  EnvAgg ag;
  ag.cand = qs != nullptr ? block_argmax_f(cq, ci, tmp) : -1;
  ag.nlive = h[0];
  ag.dm0 = h[1];
  ag.dm1 = h[2];
  ag.sd0 = h[3];
  ag.sd1 = h[4];
  ag.bad = h[5];
  ag.th0 = (long long)(((unsigned long long)(unsigned)h[7] << 32) | (unsigned)h[6]);
  ag.th1 = (long long)(((unsigned long long)(unsigned)h[9] << 32) | (unsigned)h[8]);
  return ag;
}

// Queue launches: the speculative environment-step result slot of graph gi for the state after
// `steps` removals (two per graph, by removal-count parity; md_abi.cpp sizes them).  SRES layout
// plus word 24: the tag of the last speculative item that left the slot (the slot is free when
// it equals the STARTED word's tag).
__device__ __forceinline__ int* bspec_slot(KParams& p, const GraphInfo& gi, int steps) {
  return p.bspec + (size_t)(steps & 1) * (size_t)p.bspec_half +
         4 * ((size_t)9 * gi.gidx + (size_t)gi.eoff[0] + (size_t)gi.eoff[1] + 2 * (size_t)gi.node_off);
}
constexpr int BSPEC_EXITED = 24;

// ------------------------------------------------------------------ the environment step
// Everything phase A does for one graph once the actions to apply are known: cover each
// queued node and run the fixed point (s0 first if not done), then residual degrees, the
// ascending live-node list and the per-layer aggregates, the write-back of edge states and
// the unit-cost first-layer table.  Returns 0 or an ERR_* code.
// Not inlined: the environment step has its own register allocation (inlined, it raised the
// register pressure of the whole rollout loop -- spills in the tile phases).
// View of graph gi's environment arrays: LDS mode places them in the phase-A area `ia`
// (env_layout), global mode uses the HBM arrays (and gscr for the union-find / degrees).
template <bool GL>
__device__ __forceinline__ EnvView<GL> env_view(KParams& p, const GraphInfo& gi, int* ia) {
  const int n = gi.n, e0 = gi.e[0], e1 = gi.e[1], et = e0 + e1;
  EnvView<GL> E;
  E.gi = &gi;
  E.e0 = e0;
  E.et = et;
  E.variant = p.variant;
  for (int l = 0; l < 2; ++l) {
    E.gu[l] = p.eu[l] + gi.eoff[l];
    E.gv[l] = p.ev[l] + gi.eoff[l];
    E.gst[l] = p.estate[l] + gi.eoff[l];
    E.calive[l] = p.calive[l] + gi.coff[l];
    E.epos[l] = p.epos[l] + 2 * (size_t)gi.eoff[l];
    E.grp[l] = p.rowptr[l] + gi.roff[l];
  }
  E.gcov = p.covered + gi.node_off;
  if constexpr (GL) {
    // par0, par1, deg0, deg1 (env_layout's global-mode counterpart; GSCR_WORDS per node)
    int* gs = p.gscr + GSCR_WORDS * (size_t)gi.node_off;
    E.par0 = gs;
    E.par1 = gs + n;
    E.deg0 = gs + 2 * n;
    E.deg1 = gs + 3 * n;
    E.tmp = ia;
  } else {
    const EnvLayout L = env_layout(n, et);
    lds_i32* la = (lds_i32*)ia;
    E.par0 = la + L.par0;
    E.par1 = la + L.par1;
    E.deg0 = la + L.deg0;
    E.deg1 = la + L.deg1;
    E.tmp = ia + L.tmp;
    lds_u8* base8 = (lds_u8*)(uint8_t*)ia;
    E.u16 = (lds_u16*)base8;
    E.v16 = E.u16 + ((et + 7) & ~7);
    E.st = base8 + 4 * ((et + 7) & ~7);
    E.cov8 = base8 + L.cov;
    E.al = (lds_u16*)(base8 + L.al0);
    E.al_other = (lds_u16*)(base8 + L.al1);
    E.dl = (lds_u16*)(base8 + L.dl);
    E.hdr = la + L.hdr;
    E.rp[0] = la + L.rp;
    E.rp[1] = la + L.rp + n + 1;
  }
  return E;
}

// LDS mode: stage the graph's static arrays (edge endpoints, CSR row pointers) from HBM.
__device__ __forceinline__ void env_stage_static(const EnvView<false>& E, int n) {
  const int et = E.et, e0 = E.e0;
  for (int x = threadIdx.x; x <= n; x += NTHREADS) {
    E.rp[0][x] = E.grp[0][x];
    E.rp[1][x] = E.grp[1][x];
  }
  // batched so every thread keeps 8 independent global loads in flight
  for (int e0b = 0; e0b < et; e0b += 8 * NTHREADS) {
    int uu[8], vv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int e = e0b + k * NTHREADS + threadIdx.x;
      if (e < et) {
        const int l = e < e0 ? 0 : 1, kk = e < e0 ? e : e - e0;
        uu[k] = E.gu[l][kk];
        vv[k] = E.gv[l][kk];
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int e = e0b + k * NTHREADS + threadIdx.x;
      if (e < et) {
        E.u16[e] = (uint16_t)uu[k];
        E.v16[e] = (uint16_t)vv[k];
      }
    }
  }
}

// LDS mode: stage the dynamic state (edge states, covered flags: the last write-back) from HBM,
// sixteen independent loads per thread in flight.
__device__ __forceinline__ void env_stage_dynamic(const EnvView<false>& E, int n) {
  const int et = E.et, e0 = E.e0;
  for (int e0b = 0; e0b < et; e0b += 16 * NTHREADS) {
    int ss[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = e0b + k * NTHREADS + threadIdx.x;
      if (e < et) ss[k] = ldc(E.gst[e < e0 ? 0 : 1] + (e < e0 ? e : e - e0));
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int e = e0b + k * NTHREADS + threadIdx.x;
      if (e < et) E.st[e] = (uint8_t)ss[k];
    }
  }
  for (int x = threadIdx.x; x < n; x += NTHREADS) E.cov8[x] = ldc(E.gcov + x);
}

// LDS mode, one pass: every segment of the environment (endpoints and CSR row pointers of both
// layers, edge states, covered flags) read as 16-byte chunks from its 16-byte-aligned start
// (the bytes before and after a segment are other graphs' or allocation padding, discarded),
// all of a thread's chunks in flight before the first is written to LDS -- one or two round
// trips where env_stage_static + env_stage_dynamic take ~7 dependent batches on a C3 graph.
// The states and covered flags are written by other workgroups: agent-coherent buffer loads.
__device__ __forceinline__ v4u ld16_sc1(const void* base, int byte_off) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(base), 0, 0x7fffffff, 0x00020000);
  return __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16 /* sc1 */));
}
// bytes [16 c - lead, 16 c - lead + 16) of a byte segment of cnt bytes -> dst
__device__ __forceinline__ void stage_bytes(lds_u8* dst, const v4u& w, int c, int lead, int cnt) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int x = 16 * c + i - lead;
    if (x >= 0 && x < cnt) dst[x] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
  }
}
__device__ __forceinline__ void env_stage_wide(const EnvView<false>& E, int n, const float* gq = nullptr,
                                               lds_u8* qdst = nullptr) {
  const int tid = threadIdx.x, e0 = E.e0, e1 = E.et - E.e0;
  // dynamic segments (uniform bases): states of layer 0 / 1, covered flags, and (gq: batch
  // speculation) the graph's Q row as bytes; two chunks per thread in flight per segment (up to
  // 16 K edges per layer and 16 K nodes), the rest after
  const uint8_t* dp[4] = {E.gst[0], E.gst[1], E.gcov, qdst != nullptr ? (const uint8_t*)gq : E.gcov};
  const int dn[4] = {e0, e1, n, qdst != nullptr ? 4 * n : 0};
  constexpr int DQ = 2;
  v4u dv[4][DQ];
  int dlead[4], dch[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    dlead[s] = (int)((uintptr_t)dp[s] & 15);
    dch[s] = (dlead[s] + dn[s] + 15) >> 4;
    const uint8_t* a = dp[s] - dlead[s];
#pragma unroll
    for (int k = 0; k < DQ; ++k) {
      const int c = tid + k * NTHREADS;
      dv[s][k] = ld16_sc1(a, min(c, max(dch[s] - 1, 0)) * 16);  // clamped: branch-free loads
    }
  }
  // static segments by one chunk index: u0, u1, v0, v1 (e_l ints), rp0, rp1 (n + 1 ints)
  const int* sp[6] = {E.gu[0], E.gu[1], E.gv[0], E.gv[1], E.grp[0], E.grp[1]};
  const int sn[6] = {e0, e1, e0, e1, n + 1, n + 1};
  int slead[6], pre[7];
  pre[0] = 0;
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    slead[s] = (int)(((uintptr_t)sp[s] & 15) >> 2);  // ints before the segment in its first chunk
    pre[s + 1] = pre[s] + ((slead[s] + sn[s] + 3) >> 2);
  }
  constexpr int SQ = 10;
  lds_i32* const rp0 = E.rp[0];
  lds_i32* const rp1 = E.rp[1];
  for (int b = 0; b < pre[6]; b += SQ * NTHREADS) {
    v4u w[SQ];
#pragma unroll
    for (int k = 0; k < SQ; ++k) {
      const int q = min(b + k * NTHREADS + tid, pre[6] - 1);
      const int* a = sp[0] - slead[0];
      int c = q;
#pragma unroll
      for (int s = 1; s < 6; ++s)
        if (q >= pre[s]) {
          a = sp[s] - slead[s];
          c = q - pre[s];
        }
      w[k] = *(const v4u*)(a + 4 * c);
    }
#pragma unroll
    for (int k = 0; k < SQ; ++k) {
      const int q = b + k * NTHREADS + tid;
      if (q >= pre[6]) break;
      int s = 0;
#pragma unroll
      for (int t = 1; t < 6; ++t) s += q >= pre[t];
      int c = q, lead = slead[0], cnt = sn[0];
#pragma unroll
      for (int t = 1; t < 6; ++t)
        if (s == t) {
          c = q - pre[t];
          lead = slead[t];
          cnt = sn[t];
        }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int x = 4 * c + i - lead;
        if (x < 0 || x >= cnt) continue;
        const unsigned v = w[k][i];
        if (s < 2) E.u16[(s ? e0 : 0) + x] = (uint16_t)v;
        else if (s < 4) E.v16[(s == 3 ? e0 : 0) + x] = (uint16_t)v;
        else (s == 4 ? rp0 : rp1)[x] = (int)v;
      }
    }
  }
  lds_u8* const ddst[4] = {E.st, E.st + e0, E.cov8, qdst};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (s == 3 && qdst == nullptr) break;
#pragma unroll
    for (int k = 0; k < DQ; ++k) {
      const int c = tid + k * NTHREADS;
      if (c < dch[s]) stage_bytes(ddst[s], dv[s][k], c, dlead[s], dn[s]);
    }
    const uint8_t* a = dp[s] - dlead[s];
    for (int c = tid + DQ * NTHREADS; c < dch[s]; c += NTHREADS) stage_bytes(ddst[s], ld16_sc1(a, c * 16), c, dlead[s], dn[s]);
  }
}

// LDS mode: the whole environment of the last write-back, and its alive-edge list.
// (gq, qdst: also the graph's Q row into LDS, for the batch speculation's candidate)
__device__ __forceinline__ void env_stage_lds(const EnvView<false>& E, int n, const float* gq = nullptr,
                                              lds_u8* qdst = nullptr) {
  if ((E.variant & 0x100) && qdst == nullptr) {  // MD_VARIANT bit 8 (diagnostics): the batched two-pass staging
    env_stage_static(E, n);
    env_stage_dynamic(E, n);
  } else {
    env_stage_wide(E, n, gq, qdst);
  }
  __syncthreads();
  build_alive<false>(E);
}

// Applies a speculative workgroup's result (spec_loop, md_kernels.hip) in place of the
// fixed point: the killed edges get their new states and leave the alive list exactly as
// mcc_fixed_point's final compaction would move them, and their write-back to HBM (edge
// state, both CSR flags) is issued here.  The caller has covered the node.
__device__ __forceinline__ int env_apply_spec(const EnvView<false>& E, const int* slot, int nd, int* pr, int* cc) {
  // the header (and whether the features are published too) in the kill list's round trip
  int h[5] = {0, 0, 0, 0, 0}, fa[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long ft = 0ull, dt = 0ull;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < 5; ++i) h[i] = ldc(slot + 2 + i);
    // the result's aggregates (live count, dmax, degree sums, mismatch flag): the dataflow
    // mode's early step record
#pragma unroll
    for (int i = 0; i < 6; ++i) fa[i] = ldc(slot + 12 + i);
    ft = __hip_atomic_load((const g_u64*)(slot + SRES_FEAT), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    dt = __hip_atomic_load((const g_u64*)slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  int bad_slot = 0;
  for (int i0 = threadIdx.x; i0 < nd; i0 += 4 * NTHREADS) {
    int v[4], c0[4], c1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * NTHREADS;
      if (i < nd) {
        v[u] = ldc(slot + SRES_HDR + 3 * i);
        c0[u] = ldc(slot + SRES_HDR + 3 * i + 1);
        c1[u] = ldc(slot + SRES_HDR + 3 * i + 2);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (i0 + u * NTHREADS >= nd) continue;
      const int e = v[u] & 0xffff, l = e < E.e0 ? 0 : 1;
      const uint8_t s = (uint8_t)(v[u] >> 16);
      // indices from another workgroup's result: checked before any write (a result that is
      // not consistent raises ERR_SPEC_SLOT instead of writing out of range)
      const int csr = 2 * (l ? E.et - E.e0 : E.e0);
      if (!(e < E.et && c0[u] >= 0 && c0[u] < csr && c1[u] >= 0 && c1[u] < csr)) {
        bad_slot = 1;
        continue;
      }
      E.st[e] = s;
      stc(E.gst[l] + (e < E.e0 ? e : e - E.e0), s);
      stc(E.calive[l] + c0[u], (uint8_t)0);
      stc(E.calive[l] + c1[u], (uint8_t)0);
    }
  }
  if (__syncthreads_or(bad_slot) && threadIdx.x == 0) raise_err(kp(), ERR_SPEC_SLOT);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int i = 0; i < 5; ++i) E.tmp[A_TMP_WORDS - 8 + i] = h[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) E.tmp[A_TMP_WORDS - 16 + i] = fa[i];
    // features of the same result already published? (used after this point only)
    E.tmp[A_TMP_WORDS - 3] = (unsigned)ft == (unsigned)dt && (ft >> 32) == ((dt >> 32) & 0xffffu);
  }
  __syncthreads();
  const int lm = E.tmp[A_TMP_WORDS - 8];
  pr[0] = E.tmp[A_TMP_WORDS - 7];
  pr[1] = E.tmp[A_TMP_WORDS - 6];
  cc[0] = E.tmp[A_TMP_WORDS - 5];
  cc[1] = E.tmp[A_TMP_WORDS - 4];
  // the killed edges stay in the alive list (every pass skips them by their state; the next
  // fixed point's final compaction drops them): no compaction on the step's critical path
  // (MD_VARIANT bit 15: compact here)
  if (nd > 0 && (E.variant & 0x8000)) compact_alive<false>(E);
  if (threadIdx.x == 0) E.hdr[1] = 0;  // written back above
  __syncthreads();
  return lm;
}

// ------------------------------------------------------------------ the environment step
// Everything phase A does for one graph once the actions to apply are known: cover each
// queued node and run the fixed point (s0 first if not done), then residual degrees, the
// ascending live-node list and the per-layer aggregates, the write-back of edge states and
// the unit-cost first-layer table.  Returns 0 or an ERR_* code.
// Not inlined: the environment step has its own register allocation (inlined, it raised the
// register pressure of the whole rollout loop -- spills in the tile phases).
// First-layer embedding by degree (unit cost): X = [d/dmax, d/dmax] (net :252-261),
// normalize(relu(X . w_n2l)) with the 2-term FMA chain of MKL's sgemm; one thread per row
// d = 1..dmax (the row recomputed for the norm pass and the store pass; w_n2l arrives as
// scalar loads), the norm in torch's order (wave_norm64's).  The table depends on dmax
// only, so it is rebuilt only when dmax changed (hd0, hd1: the dmax of the current tables).
__device__ __forceinline__ void h0_update(KParams& p, const GraphInfo& gi, GraphVar& gv, int dm0, int dm1, int hd0, int hd1) {
  if (p.node_w == nullptr) {
    const float* wn = p.w + W_N2L;
    for (int l = 0; l < 2; ++l) {
      const int dm = l ? dm1 : dm0;
      if (dm == (l ? hd1 : hd0)) continue;
      float* tab = p.h0tab[l] + (size_t)gi.node_off * EMB;  // degrees <= n-1 fit the graph's rows
      if (dm <= p.h0g_dm && p.h0g != nullptr) continue;  // the tiles read the precomputed table
      if (dm <= p.h0g_dm) {
        // the table of this dmax is precomputed (md_h0_kernel at load): a 16-byte copy
        const float* src = p.h0g + h0g_row(dm, 1) * EMB;
        const int nq = 16 * dm;
        for (int i0 = threadIdx.x; i0 < nq; i0 += 4 * NTHREADS) {
          float4 x[4];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (i0 + k * NTHREADS < nq) x[k] = ldc4(src, (i0 + k * NTHREADS) * 16);
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (i0 + k * NTHREADS < nq) stc4(tab, EMB * 4 + (i0 + k * NTHREADS) * 16, x[k]);
        }
        continue;
      }
      for (int d = 1 + (int)threadIdx.x; d <= dm; d += NTHREADS) {
        const float f = (float)d / (float)dm;
        float acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
        for (int c = 0; c < 64; ++c) {
          const float x = fmaxf(fmaf(f, wn[64 + c], fmaf(f, wn[c], 0.f)), 0.f);
          acc[c & 7] = fmaf(x, x, acc[c & 7]);
        }
        const float den = fmaxf(sqrtf(sumsq8_finish(acc)), 1e-12f);
#pragma unroll
        for (int c4 = 0; c4 < 16; ++c4) {
          float o[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int c = 4 * c4 + k;
            o[k] = fmaxf(fmaf(f, wn[64 + c], fmaf(f, wn[c], 0.f)), 0.f) / den;
          }
          stc4(tab, d * 256 + c4 * 16, make_float4(o[0], o[1], o[2], o[3]));
        }
      }
    }
    if (threadIdx.x == 0) {
      gv.hdmax[0] = dm0;
      gv.hdmax[1] = dm1;
    }
  }
}

// Dataflow mode, early step record (thread 0): with the taken result's features published,
// the state after this step is known before phase A has applied it (live count, and whether it
// stays running: alive edges in both layers, no K2 end-game, no live-set mismatch -- the
// result's aggregates in E.tmp[A_TMP_WORDS - 16, -11)); tile workgroups whose iteration-1
// prebuild used this result start their step on it while this phase A finishes (the others,
// and the graph head, wait for the record's "full" granule; the tiles' Q stores come after the
// graph head, so after phase A's reset of Q).
template <bool GL>
__device__ __forceinline__ void df_early_record(KParams& p, const EnvView<GL>& E, int n) {
  const int nl = E.tmp[A_TMP_WORDS - 16], dm0 = E.tmp[A_TMP_WORDS - 15], dm1 = E.tmp[A_TMP_WORDS - 14];
  const int sd0 = E.tmp[A_TMP_WORDS - 13], sd1 = E.tmp[A_TMP_WORDS - 12], bad = E.tmp[A_TMP_WORDS - 11];
  const bool eg = p.endgame && p.node_w == nullptr && n < 32768 && nl > 0 && dm0 == 1 && dm1 == 1;
  volatile int* misc = (volatile int*)(md::lds_base() + L_MISC);
  if (!bad && sd0 > 0 && sd1 > 0 && !eg && misc[56] != 0) {
    const unsigned tag = (unsigned)(misc[60] + 1);
    const int v[6] = {ST_RUN, nl, misc[56], misc[57], misc[56], misc[57]};
#pragma unroll
    for (int i = 0; i < 6; ++i) df_st(p.df + DF_REC + i, __int_as_float(v[i]), tag);
    misc[48] = 1;
  }
}

// env_step's pend_first when the actions were applied already (env_endgame_apply): the step
// only recomputes the features
constexpr int PEND_APPLIED = -2;

// K2 end-game answer applied in one pass (LDS mode; p.endgame bit 2, MD_EG_APPLY=0: off).  The
// answer's state (endgame_state: residual degree <= 1 in both layers after a fixed point) is a
// set of pairs joined in both layers plus isolated nodes.  Covering a node of a pair kills its
// two edges and isolates its partner; nothing is pruned and the other pairs stay components of
// both layers, so after action j the LMCC (U/Mcc.py:30-38, over non-covered nodes) is 2 while
// pairs remain, else 1 while a non-covered node remains, else 0; the loop stops after the
// action that takes the last pair (env_step's terminal check).  Returns the actions applied,
// with the trace, covered flags, killed edges (dead list) and books as env_step's loop leaves
// them, or -1 when the state or the actions do not have that form (nothing changed: the
// caller's loop runs).  Scratch: the parent and degree arrays (free until the fixed point /
// the features pass).  Stages the state into LDS first unless `staged`.
__device__ __noinline__ int env_endgame_apply(KParams&, const GraphInfo gi, int pend_n, bool staged) {
  KParams& p = kp();
  GraphVar& gv = *(GraphVar*)(md::lds_base() + L_GV);
  const EnvView<false> E = env_view<false>(p, gi, (int*)(md::lds_base() + L_W));
  if (!staged) {
    env_stage_lds(E, gi.n);
    __syncthreads();
  }
  const int n = gi.n;
  lds_i32* mark = E.par0;  // node -> 1 + its action index (0: not picked)
  lds_i32* act = E.par1;   // action index -> node
  lds_i32* part = E.deg0;  // node -> layer-0 partner (-1: isolated)
  int* w = E.tmp + A_TMP_WORDS - 32;  // {bad, first action that takes the last pair}
  if (pend_n <= 0 || pend_n > n || gv.dmax[0] > 1 || gv.dmax[1] > 1 || gv.alive[0] != gv.alive[1] || gv.alive[0] <= 0 ||
      !gv.s0_done)
    return -1;
  for (int x = threadIdx.x; x < n; x += NTHREADS) {
    mark[x] = 0;
    part[x] = -1;
  }
  if (threadIdx.x == 0) {
    w[0] = 0;
    w[1] = pend_n;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < pend_n; i += NTHREADS) {
    const int a = __hip_atomic_load(p.pend + gi.node_off + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    act[i] = a;
    if (a < 0 || a >= n || E.covered(a)) w[0] = 1;
    else mark[a] = i + 1;
  }
  const int na = E.hdr[0];
  const lds_u16* al = E.hdr[2] ? E.al_other : E.al;
  for (int i = threadIdx.x; i < na; i += NTHREADS) {
    const int e = al[i];
    if (e < E.e0 && E.st[e] == E_ALIVE) {
      const int u = E.u16[e], v = E.v16[e];
      part[u] = v;
      part[v] = u;
    }
  }
  __syncthreads();
  // (duplicates: one index per node survives; layer 1 must join the same pairs)
  for (int i = threadIdx.x; i < pend_n; i += NTHREADS) {
    const int a = act[i];
    if (a >= 0 && a < n && mark[a] != i + 1) w[0] = 1;
  }
  for (int i = threadIdx.x; i < na; i += NTHREADS) {
    const int e = al[i];
    if (e >= E.e0 && E.st[e] == E_ALIVE) {
      const int u = E.u16[e], v = E.v16[e];
      if (part[u] != v || part[v] != u) w[0] = 1;
    }
  }
  __syncthreads();
  if (w[0]) return -1;
  // action i takes a pair when its partner is not picked before it; pairs left after it
  const int P = gv.alive[0];
  const int chunk = (pend_n + NTHREADS - 1) / NTHREADS;
  const int i0 = min(pend_n, (int)threadIdx.x * chunk), i1 = min(pend_n, i0 + chunk);
  int hits = 0;
  for (int i = i0; i < i1; ++i) {
    const int b = part[act[i]];
    hits += b >= 0 && (mark[b] == 0 || mark[b] > i + 1);
  }
  int tot = 0;
  int h = block_excl_scan(hits, E.tmp, &tot);
  const int ncov0 = gv.n_cov, steps0 = gv.steps;
  for (int i = i0; i < i1; ++i) {
    const int b = part[act[i]];
    h += b >= 0 && (mark[b] == 0 || mark[b] > i + 1);
    if (h == P) atomicMin(w + 1, i + 1);
    E.deg1[i] = P - h;  // pairs left after action i
  }
  __syncthreads();
  const int m = w[1];
  for (int i = threadIdx.x; i < m; i += NTHREADS) {
    const int a = act[i];
    stc(E.gcov + a, (uint8_t)1);
    E.cov8[a] = 1;
    const int lm = E.deg1[i] > 0 ? 2 : (n - ncov0 - (i + 1) > 0 ? 1 : 0);
    if (MD_BOK(steps0 + i < n, 8)) {
      stc(p.tr_action + gi.node_off + steps0 + i, a);
      stc(p.tr_rank + gi.node_off + steps0 + i, lm);
    }
  }
  int k0 = 0, k1 = 0;
  for (int i = threadIdx.x; i < na; i += NTHREADS) {
    const int e = al[i];
    if (E.st[e] != E_ALIVE) continue;
    const int mu = mark[E.u16[e]], mv = mark[E.v16[e]];
    if ((mu > 0 && mu <= m) || (mv > 0 && mv <= m)) {
      E.st[e] = E_COVERED;
      if (e < E.e0) k0++; else k1++;
    }
  }
  const int2 kk = block_sum2(k0, k1, E.tmp);
  __syncthreads();
  compact_alive(E);
  if (threadIdx.x == 0) {
    gv.counter[0] += kk.x;
    gv.counter[1] += kk.y;
    gv.alive[0] -= kk.x;
    gv.alive[1] -= kk.y;
    gv.n_cov += m;
    gv.lmcc = E.deg1[m - 1] > 0 ? 2 : (n - ncov0 - m > 0 ? 1 : 0);
    gv.steps += m;
  }
  __syncthreads();
  return m;
}

template <bool GL>
__device__ __noinline__ int env_step(KParams&, const GraphInfo gi, GraphVar&, float*, int pend_n,
                        int pend_first, const float*, bool staged) {
  KParams& p = kp();  // kernel arguments through the implicit-argument SGPRs (uniform)
  // LDS from the kernel's dynamic-LDS base (compile-time addresses, ds_* accesses)
  const float* const lds_base = md::lds_base();
  GraphVar& gv = *(GraphVar*)(md::lds_base() + L_GV);
  float* const area = md::lds_base() + L_W;
  const int n = gi.n, e0 = gi.e[0], et = e0 + gi.e[1];
  (void)et;  // bounds checks only
  int* ia = (int*)area;
  QENV_INIT();
  // (this step changes the state without the grid-wide step's class labels: they go stale)
  if (threadIdx.x == 0 && p.lab_ok != nullptr) stc(p.lab_ok + gi.gidx, 0);
  const EnvView<GL> E = env_view<GL>(p, gi, ia);
  // batch speculation (queue launches): the graph's previous Q row staged beside the state, for
  // the next step's candidate (after the environment arrays: free until the neighbour lists)
  const float* qs = nullptr;
  if constexpr (!GL) {
    const int qoff = env_layout(n, et).total;
    const bool bq = p.bspec != nullptr && !staged && qoff + n <= A_WORDS;
    if (bq) qs = (const float*)(ia + qoff);
    if (!staged) env_stage_lds(E, n, bq ? p.q + gi.node_off : nullptr, bq ? (lds_u8*)(uint8_t*)(ia + qoff) : nullptr);
    __syncthreads();
  }
  QENV(0);
  // a speculative workgroup may already have run this step's fixed point for the chosen node
  // (single-node steps picked by the device or the host; results are tagged with the launch,
  // the removals so far and the node)
  int spec_slot = -1, spec_nd = 0;
  if constexpr (!GL) {
    if (p.n_spec > 0 && pend_n == 1 && gv.s0_done && ((const volatile int*)(lds_base + L_MISC))[5]) {
      const int a = pend_first >= 0 ? pend_first : __hip_atomic_load(p.pend + gi.node_off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned want = spec_tag(p.launch_seq, gv.steps);
      const int ps = ((volatile int*)(lds_base + L_MISC))[60] - 1;  // the request's step
      unsigned long long* sts = p.prof != nullptr && ps >= 0 && ps < p.prof_cap ? p.prof + (size_t)ps * PROF_SLOTS : nullptr;
      if (sts != nullptr && threadIdx.x == 0) sts[69] = wall_clock64();
      if (threadIdx.x == 0) {
        E.tmp[A_TMP_WORDS - 1] = -1;
        E.tmp[A_TMP_WORDS - 10] = 0;  // the taken result's features were published at the pre-read
      }
      __syncthreads();
      if ((int)threadIdx.x < p.n_spec) {
        // done, or taken and still running: a taken fixed point started earlier than this one
        // could, so waiting for it is never slower than computing it here
        // tags as phase A read them beside the arg-max partials (L_PREF, free until the tile
        // prefix), polled again only while a taken result is still running
        const g_u64* tp = (const g_u64*)(p.sres + (size_t)spec_slot_index(threadIdx.x, ps) * p.sres_stride);
        const unsigned long long* pre = (const unsigned long long*)(lds_base + L_PREF) + 2 * threadIdx.x;
        unsigned long long v = pre[0];
        const unsigned long long st = pre[1];
        bool done = (unsigned)v == want && (int)((v >> 32) & 0xffffu) == a;
        if (!done && (unsigned)st == want && (int)(st >> 32) == a) {
          const unsigned long long t0 = wall_clock64();
          while (true) {
            v = __hip_atomic_load(tp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((unsigned)v == want && (int)((v >> 32) & 0xffffu) == a) { done = true; break; }
            if (wall_clock64() - t0 > BARRIER_TIMEOUT_TICKS ||
                (__hip_atomic_load((g_u32*)p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & BAR_ERR))
              break;
            __builtin_amdgcn_s_sleep(1);
          }
          if (sts != nullptr) {  // diagnostics: longest poll (slot 32), polling lanes (slot 31)
            atomicMax(sts + 32, wall_clock64() - t0);
            atomicAdd(sts + 31, 1ull);
          }
        }
        if (done) {
          E.tmp[A_TMP_WORDS - 1] = spec_slot_index(threadIdx.x, ps);  // the slot, parity included
          E.tmp[A_TMP_WORDS - 2] = (int)(v >> 48);  // killed edges
          if (sts != nullptr) sts[70] = threadIdx.x + 1;
          if (p.df != nullptr) {
            const int* pf = (const int*)(lds_base + L_PREF) + PREF_FEAT + 8 * threadIdx.x;
            if ((unsigned)pf[0] == want && pf[1] == a) {
#pragma unroll
              for (int i = 0; i < 6; ++i) E.tmp[A_TMP_WORDS - 16 + i] = pf[2 + i];
              E.tmp[A_TMP_WORDS - 10] = 1;
            }
          }
        }
      }
      __syncthreads();
      if (sts != nullptr && threadIdx.x == 0) sts[71] = wall_clock64();
      spec_slot = E.tmp[A_TMP_WORDS - 1];
      spec_nd = E.tmp[A_TMP_WORDS - 2];
      if (p.pre_ew != nullptr && threadIdx.x == 0) {
        // the tile workgroups may build their iteration-1 lists from this result meanwhile (and
        // the speculative workgroups the next state: spec_loop's early requests)
        const unsigned long long ew = spec_slot >= 0 ? ((unsigned long long)want << 32) | ((unsigned)a << 16) | (unsigned)spec_slot : 0ull;
        ((volatile unsigned*)(lds_base + L_MISC))[56] = (unsigned)ew;
        ((volatile unsigned*)(lds_base + L_MISC))[57] = (unsigned)(ew >> 32);
        if (ew != 0ull) __hip_atomic_store((g_u64*)p.pre_ew, ew, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // dataflow mode: with the taken result's features already published, the state after
        // this step is known now; the step record goes out before the result is applied (see
        // the early record below; the same conditions, from the pre-read aggregates)
        if (ew != 0ull && p.df != nullptr && pend_n == 1 && p.run_mode == RUN_ROLLOUT && E.tmp[A_TMP_WORDS - 10])
          df_early_record(p, E, n);
      }
      if (sts != nullptr && threadIdx.x == 0 && spec_slot >= 0)
        sts[72] = __hip_atomic_load((const g_u64*)(p.sres + (size_t)spec_slot * p.sres_stride) + 5, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
    }
  }
  // queue launches: a speculative environment item (bspec_spec_step) may have run this step for
  // the node now chosen, from exactly this state (tag: launch, removals so far, node)
  const int* spec_ptr = spec_slot >= 0 ? p.sres + (size_t)spec_slot * p.sres_stride : nullptr;
  if constexpr (!GL) {
    if (p.bspec != nullptr && p.n_spec == 0 && pend_n == 1 && gv.s0_done && !(p.variant & 0x2000)) {
      const int* sl = bspec_slot(p, gi, gv.steps);
      if (threadIdx.x == 0) {
        const int a = pend_first >= 0 ? pend_first
                                      : __hip_atomic_load(p.pend + gi.node_off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long v = __hip_atomic_load((const g_u64*)sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool hit = (unsigned)v == spec_tag(p.launch_seq, gv.steps) && (int)((v >> 32) & 0xffffu) == a;
        E.tmp[A_TMP_WORDS - 1] = hit ? 1 : 0;
        E.tmp[A_TMP_WORDS - 2] = (int)(v >> 48);
      }
      __syncthreads();
      if (E.tmp[A_TMP_WORDS - 1]) {
        spec_ptr = sl;
        spec_nd = E.tmp[A_TMP_WORDS - 2];
      }
      __syncthreads();
    }
  }
  bool spec_used = false;
  MD_PROF_A(1);
  unsigned long long* acc = nullptr;
  if (p.prof != nullptr && blockIdx.x == 0) {
    const int ps = ((volatile int*)(lds_base + L_MISC))[60];
    if (ps < p.prof_cap) acc = p.prof + (size_t)ps * PROF_SLOTS + 16;
  }
  int err = 0;
  for (int k = pend_first == PEND_APPLIED ? pend_n : 0; k < pend_n; ++k) {
    if (gv.alive[0] == 0 || gv.alive[1] == 0) break;  // terminal between queued actions
    const int a = k == 0 && pend_first >= 0
                      ? pend_first
                      : __hip_atomic_load(p.pend + gi.node_off + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a < 0 || a >= n) { err = ERR_BADNODE; break; }
    if (E.covered(a)) { err = ERR_COVERED; break; }
    // cover a in both layers (U/mvc_env.py:74-85) -- its alive edges become "covered", done
    // inside the first union pass of the fixed point -- then the mutual-LMCC fixed point
    const unsigned long long tcv = wall_clock64();
    __syncthreads();  // every thread has read covered(a) before it is set
    if (threadIdx.x == 0) {
      stc(E.gcov + a, (uint8_t)1);
      if constexpr (!GL) E.cov8[a] = 1;
    }
    __syncthreads();
    PACC(acc, PA_COVER, tcv);
    int pr[2], c[2];
    int lm;
    if constexpr (!GL) {
      if (k == 0 && spec_ptr != nullptr) {
        lm = env_apply_spec(E, spec_ptr, spec_nd, pr, c);
        spec_used = true;
        if (threadIdx.x == 0) gv.spec_hits += 1;
        if (p.df != nullptr && pend_n == 1 && p.run_mode == RUN_ROLLOUT && E.tmp[A_TMP_WORDS - 3] && threadIdx.x == 0 &&
            ((volatile int*)(lds_base + L_MISC))[48] == 0)
          df_early_record(p, E, n);
      } else {
        lm = mcc_fixed_point<GL>(E, pr, acc, a, c);
      }
    } else {
      lm = mcc_fixed_point<GL>(E, pr, acc, a, c);
    }
    if (threadIdx.x == 0) {
      gv.counter[0] += c[0];
      gv.counter[1] += c[1];
      gv.removed[0] += pr[0];
      gv.removed[1] += pr[1];
      gv.alive[0] -= c[0] + pr[0];
      gv.alive[1] -= c[1] + pr[1];
      gv.n_cov += 1;
      gv.lmcc = lm;
      if (MD_BOK(gv.steps < gi.n, 8)) {
        stc(p.tr_action + gi.node_off + gv.steps, a);
        stc(p.tr_rank + gi.node_off + gv.steps, lm);
      }
      gv.steps += 1;
    }
    __syncthreads();
  }
  if (!gv.s0_done && !err) {
    int pr[2];
    const int lm = mcc_fixed_point<GL>(E, pr, acc, -1, nullptr);
    if (threadIdx.x == 0) {
      gv.removed[0] += pr[0];
      gv.removed[1] += pr[1];
      gv.max_rank = lm;
      gv.lmcc = lm;
      gv.s0_done = 1;
    }
  }
  MD_PROF_A(2);
  QENV(1);
  float* q = p.q + gi.node_off;
  int* gdeg0 = p.deg[0] + gi.node_off;
  int* gdeg1 = p.deg[1] + gi.node_off;
  float* lv = (float*)(p.live + 4 * (size_t)gi.node_off);
  EnvAgg ag;
  if (spec_used && E.tmp[A_TMP_WORDS - 3]) {
    // the speculative workgroup also produced this step's degrees, live list and aggregates
    lds_i32* ld0 = nullptr;
    lds_i32* ld1 = nullptr;
    if constexpr (!GL) {
      ld0 = E.deg0;
      ld1 = E.deg1;
    }
    ag = env_copy_features(spec_ptr, n, et, gdeg0, gdeg1, lv, q, qs, E.tmp, ld0, ld1);
    if (acc != nullptr && threadIdx.x == 0) acc[59] = 1;  // diagnostics: slot 75, features copied
  } else {
    ag = env_features<GL>(E, n, gdeg0, gdeg1, lv, q, qs);
  }
  // the next step's candidate for the batch speculation (-1: none)
  if (threadIdx.x == 0) ((volatile int*)(lds_base + L_MISC))[20] = qs != nullptr ? ag.cand : -1;
  const int tot = ag.nlive, dm0 = ag.dm0, dm1 = ag.dm1, sd0 = ag.sd0, sd1 = ag.sd1, bad = ag.bad;
  const long long th0 = ag.th0, th1 = ag.th1;
  MD_PROF_A(34);
  QENV(2);
  if (bad && !err) err = ERR_LIVE_MISMATCH;
  const int hd0 = gv.hdmax[0], hd1 = gv.hdmax[1];
  __syncthreads();
  if (threadIdx.x == 0) {
    gv.n_live = tot;
    gv.dmax[0] = dm0;
    gv.dmax[1] = dm1;
    gv.alive[0] = sd0 / 2;
    gv.alive[1] = sd1 / 2;
    gv.twohop[0] = th0;
    gv.twohop[1] = th1;
  }
  if constexpr (!GL) {
    // write back the edges killed since the last write-back; dead edges drop out of the
    // gather's CSR view
    const int nd = E.hdr[1];
    for (int i = threadIdx.x; i < nd; i += NTHREADS) {
      const int e = E.dl[i];
      const int l = e < e0 ? 0 : 1, kk = e < e0 ? e : e - e0;
      if (!MD_BOK(e < et && i < et, 10)) continue;
      stc(E.gst[l] + kk, (uint8_t)E.st[e]);
      stc(E.calive[l] + E.epos[l][2 * kk], (uint8_t)0);
      stc(E.calive[l] + E.epos[l][2 * kk + 1], (uint8_t)0);
    }
    __syncthreads();
    if (threadIdx.x == 0) E.hdr[1] = 0;
  }
  MD_PROF_A(14);
  QENV(3);
  // a rollout's first environment step (no action, no prediction yet) asks too, with the
  // candidates ranked by residual degree (both layers) instead of the previous Q: the first
  // pick is a hub (rank 1-2 by degree on the GMM seeds), so step 1 needs no fixed point of its
  // own (MD_FIRST_REQ=0: off)
  const bool first_req = !GL && p.first_req && p.n_spec > 0 && p.run_mode == RUN_ROLLOUT && pend_n == 0 &&
                         p.qspec != nullptr && !((const volatile int*)(lds_base + L_MISC))[5];
  if (p.n_spec > 0 && !err && gv.alive[0] > 0 && gv.alive[1] > 0 &&
      (((const volatile int*)(lds_base + L_MISC))[5] || first_req)) {
    if constexpr (!GL) {
      if (first_req) {  // the ranking keys where the speculative workgroups read Q(t - 1)
        const int ps = ((const volatile int*)(lds_base + L_MISC))[60];
        float* qs = p.qspec + (size_t)((ps - 1) & 1) * p.qspec_n + gi.node_off;
        for (int x = threadIdx.x; x < n; x += NTHREADS) stc(qs + x, (float)(uf_load(E.deg0, x) + uf_load(E.deg1, x)));
      }
    }
    // the state after this step is in HBM once every store has drained: ask the speculative
    // workgroups for the next step's fixed point of the likely next removals (before the
    // first-layer table, which they do not read)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const int ps = ((const volatile int*)(lds_base + L_MISC))[60];
      __hip_atomic_store((g_u64*)p.spec_req, ((unsigned long long)(unsigned)ps << 32) | spec_tag(p.launch_seq, gv.steps),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (p.prof != nullptr && ps < p.prof_cap) p.prof[(size_t)ps * PROF_SLOTS + 64] = wall_clock64();
    }
  }
  h0_update(p, gi, gv, dm0, dm1, hd0, hd1);
  __syncthreads();
  MD_PROF_A(15);
  QENV(4);
  return err;
}

// ------------------------------------------------------------------ grid-wide environment step
// A graph too large for one workgroup's LDS (global mode: testReal sizes, N ~ 10^4 - 10^5)
// running alone in a launch: instead of one workgroup scanning every edge of the graph in HBM
// while the others wait at the barrier, every workgroup of the launch takes part -- edges and
// nodes grid-strided, the union-find forests in HBM with agent-scope atomics, a grid barrier
// between passes.  The passes are the one-workgroup code's (mcc_fixed_point, env_features):
// the same Jacobi rounds reach the same unique fixed point and pruned-edge set, the same LMCC
// count, degrees, ascending live list and aggregates.  Cross-workgroup sums go through
// per-workgroup partials (two alternating slots: a slot is rewritten two reductions later, after
// every workgroup has passed the barrier that follows its reads).
struct Team {
  int gt, gs;      // this thread's index in the grid, grid stride (threads)
  int use;         // reductions so far (partial slot = use & 1)
  unsigned* target;
  int* flag;
  int* tmp;        // LDS, >= 2 * (8 * 17 + 17) words (team_reduce's long longs)
  unsigned long long* acc;  // diagnostics (md_profile): per-step piece ticks of workgroup 0, else null
  unsigned long long t;
  unsigned long long* prof_any;  // diagnostics: the step's record (every workgroup), else null
  unsigned long long t0any;
};
// Team-step piece profile (md_profile, workgroup 0): slots 80.. of the step's record:
// 80 rounds, 81 union passes, 82 label passes + reduction, 83 prune passes + reduction,
// 84 LMCC count, 85 features, 86 fixed-point inits
#define TEAM_ACC(T, k)                                                    \
  do {                                                                    \
    if ((T).acc != nullptr && threadIdx.x == 0) {                         \
      const unsigned long long now_ = wall_clock64();                     \
      (T).acc[k] += now_ - (T).t;                                         \
      (T).t = now_;                                                       \
    }                                                                     \
  } while (0)

// arr[idx] += 1 for every lane with `on`; lanes of the wave that share an index are combined
// into one atomic -- a hub's edges and a giant component's nodes would otherwise serialise
// thousands of returning atomics on one word.  Every lane of the wave calls it (wave-uniform
// loops).
template <class P>
__device__ __forceinline__ void agg_add1(P arr, int idx, bool on) {
  unsigned long long m = __ballot(on);
  while (m != 0ull) {  // one atomic per distinct index of the wave
    const int leader = __ffsll((long long)m) - 1;
    const int key = __shfl(idx, leader, 64);
    const unsigned long long same = __ballot(on && idx == key);
    if (lane_id() == leader) uf_add(arr, key, (int)__popcll(same));
    if (idx == key) on = false;
    m &= ~same;
  }
}

// agg_add1 on an HBM array, returning the largest count any of this lane's adds produced (the
// lane that makes a word's last add sees the word's final count).
__device__ __forceinline__ int agg_add1_max(int* arr, int idx, bool on) {
  unsigned long long m = __ballot(on);
  int best = 0;
  while (m != 0ull) {  // one atomic per distinct index of the wave
    const int leader = __ffsll((long long)m) - 1;
    const int key = __shfl(idx, leader, 64);
    const unsigned long long same = __ballot(on && idx == key);
    if (lane_id() == leader) {
      const int k = (int)__popcll(same);
      best = max(best, __hip_atomic_fetch_add(arr + key, k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + k);
    }
    if (idx == key) on = false;
    m &= ~same;
  }
  return best;
}

// Reduces K 64-bit values over the grid (bit k of maxmask: max, else sum; every value >= 0 for
// a max) into tot[k]; `before`, when given, receives the sum of value 0 over the lower
// workgroups (the base of an ascending scan).  Returns true on a grid error.
template <int K>
__device__ bool team_reduce(KParams& p, Team& T, const long long (&v)[K], unsigned maxmask, long long (&tot)[K],
                            long long* before) {
  static_assert(K <= 16, "16 partials per workgroup");
  const int lane = lane_id(), w = wave_id();
  long long r[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    r[k] = v[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const long long y = __shfl_xor(r[k], o, 64);
      r[k] = (maxmask >> k & 1u) ? (r[k] > y ? r[k] : y) : r[k] + y;
    }
  }
  long long* lt = (long long*)T.tmp;  // [8 waves][K], then [K + 1] totals
  __syncthreads();
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) lt[w * K + k] = r[k];
  }
  __syncthreads();
  const int slot = T.use & 1;
  if (threadIdx.x < K) {
    const int k = threadIdx.x;
    long long a = 0;
    for (int i = 0; i < NTHREADS / 64; ++i) {
      const long long y = lt[i * K + k];
      a = (maxmask >> k & 1u) ? (a > y ? a : y) : a + y;
    }
    __hip_atomic_store((g_u64*)(p.tpart + ((size_t)slot * TEAM_MAX_WG + blockIdx.x) * 16 + k), (unsigned long long)a,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  T.use++;
  if (grid_sync(p, *T.target, T.flag)) return true;
  // every thread reads one workgroup's partials (its K loads in flight together): one round
  // trip for up to NTHREADS workgroups, where one wave looping over them took n_main / 64
  long long a[K];
  long long pre = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) a[k] = 0;
  for (int b = threadIdx.x; b < p.n_main; b += NTHREADS) {
    const g_u64* src = (const g_u64*)(p.tpart + ((size_t)slot * TEAM_MAX_WG + b) * 16);
    long long y[K];
#pragma unroll
    for (int k = 0; k < K; ++k) y[k] = (long long)__hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int k = 0; k < K; ++k) a[k] = (maxmask >> k & 1u) ? (a[k] > y[k] ? a[k] : y[k]) : a[k] + y[k];
    if (b < (int)blockIdx.x) pre += y[0];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const long long y = __shfl_xor(a[k], o, 64);
      a[k] = (maxmask >> k & 1u) ? (a[k] > y ? a[k] : y) : a[k] + y;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pre += __shfl_xor(pre, o, 64);
  if (lane == 0) {  // per wave (lt's first stage is dead: read before the barrier)
#pragma unroll
    for (int k = 0; k < K; ++k) lt[w * (K + 1) + k] = a[k];
    lt[w * (K + 1) + K] = pre;
  }
  __syncthreads();
  if (threadIdx.x <= K) {
    const int k = threadIdx.x;
    long long c = 0;
    for (int i = 0; i < NTHREADS / 64; ++i) {
      const long long y = lt[i * (K + 1) + k];
      c = (k < K && (maxmask >> k & 1u)) ? (c > y ? c : y) : c + y;
    }
    lt[8 * 17 + k] = c;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < K; ++k) tot[k] = lt[8 * 17 + k];
  if (before != nullptr) *before = lt[8 * 17 + K];
  __syncthreads();
  return false;
}

// Mutual-LMCC fixed point of mcc_fixed_point on the whole grid (cover >= 0: cover that node in
// the first union pass; its covered edge counts per layer in cc).  LMCC size in lm, pruned edge
// counts in pr.  Labels (component roots) end in E.deg0 / E.deg1 as there.
// Two grid barriers per round instead of three: the prune of round r (by round r's labels) and
// the union of round r + 1 are one edge pass -- each thread decides per alive edge whether the
// other layer's labels separate its endpoints (pruned) or it is united -- on parent arrays
// double-buffered by round (round r + 1's are reset during round r's label pass).  The edge set
// each union pass sees, and so every partition, label and pruned edge, is the three-pass loop's.
// deg_zero (the features' degree arrays, grid-wide scratch): zeroed in the init pass.
// Class restriction (cls != nullptr, cover >= 0): cls[x] is x's class (its root label) in the
// mutual partition the previous fixed point left, and cnt[r] the non-covered size of the class
// rooted at r.  Every alive edge lies inside one class there (crossing edges were pruned), so
// covering node a changes only a's class C_a: every other class stays connected in both layers
// with no edge leaving it, hence a class of the new fixed point as well.  The passes then run on
// C_a's nodes and edges alone (the others are skipped by their class), and the LMCC is the
// largest of the untouched classes' sizes and the recounted sizes inside C_a -- the same fixed
// point, pruned edges, labels and LMCC as the unrestricted loop (which runs when cls == nullptr
// and establishes cls and cnt).  cls is updated to the new labels in the count pass.
__device__ bool team_fixed_point(KParams& p, Team& T, const EnvView<true>& E, int* cnt, int cover, bool set_cover, int& lm,
                                 int* pr, int* cc, int* deg_zero = nullptr, int* cls = nullptr, bool restrict_cls = false,
                                 const lds_u16* rk = nullptr) {
  const int n = E.gi->n, et = E.et, e0 = E.e0;
  int* const pb[2][2] = {{E.par0, E.par1}, {p.gscr_team + n, p.gscr_team + 2 * n}};  // par0, par1 | par0', par1'
  const bool rs = restrict_cls && cls != nullptr && cover >= 0;
  const int La = rs ? uf_load(cls, cover) : -1;  // a's class
  if (T.acc != nullptr && threadIdx.x == 0) T.t = wall_clock64();
  for (int x = T.gt; x < n; x += T.gs) {
    if (!rs || uf_load(cls, x) == La) {
      uf_store(pb[0][0], x, x);
      uf_store(pb[0][1], x, x);
      uf_store(cnt, x, 0);  // (unrestricted: every class is recounted)
    }
    if (deg_zero != nullptr) {
      uf_store(deg_zero, x, 0);
      uf_store(deg_zero, n + x, 0);
    }
  }
  if (grid_sync(p, *T.target, T.flag)) return true;
  TEAM_ACC(T, 6);
  if (set_cover && cover >= 0 && threadIdx.x == 0) stc(E.gcov + cover, (uint8_t)1);  // read by the count pass
  pr[0] = pr[1] = 0;
  // The thread's first edge (e = T.gt: the grid has at least as many threads as most graphs have
  // edges) stays in registers for the whole fixed point -- alive flag, endpoints, class test --
  // instead of three dependent loads per round: only this thread changes its state here.
  const bool e1 = T.gt < et;
  bool a1 = false;
  int u1 = 0, v1 = 0;
  if (e1) {
    a1 = E.state(T.gt) == E_ALIVE;
    u1 = E.u(T.gt);
    v1 = E.v(T.gt);
    if (a1 && rs && uf_load(cls, u1) != La) a1 = false;  // an edge of another class (both ends in it)
  }
  // (node passes likewise: the thread's first node's class test)
  const bool x1in = T.gt < n && (!rs || uf_load(cls, T.gt) == La);
  // Unchanged layers (MD_FP_SKIP, as in mcc_fixed_point): a pass that pruned no edge of layer
  // 1 - l left layer 1 - l's partition as it was, so the next pass has no layer-l edge to prune
  // (the pass before pruned every one crossing it) and layer l's union would rebuild its last
  // labels: that pass skips layer l's edges and the label pass its finds.  (From the third
  // pass on: the first prunes nothing.)  cq0 / cq1: the last pass's pruned counts per layer.
  long long cq0 = -1, cq1 = -1;
  for (int round = 0;; ++round) {
    const bool first = round == 0;
    const bool sk0 = p.fp_skip && round >= 2 && cq1 == 0, sk1 = p.fp_skip && round >= 2 && cq0 == 0;
    int* const P0 = pb[round & 1][0];
    int* const P1 = pb[round & 1][1];
    long long k0 = 0, k1 = 0, c0 = 0, c1 = 0;
    int d_ops = 0, d_fails = 0, d_un = 0;  // diagnostics (prof_any)
    unsigned long long d_tmax = 0;
    if (T.prof_any != nullptr) T.t0any = wall_clock64();
    for (int e = T.gt; e < et; e += T.gs) {
      const bool own = e == T.gt;
      if (own ? !a1 : E.state(e) != E_ALIVE) continue;
      if (e < e0 ? sk0 : sk1) continue;  // (a skipped layer's edges stay alive and out of this pass)
      const int u = own ? u1 : E.u(e), v = own ? v1 : E.v(e);
      if (!own && rs && uf_load(cls, u) != La) continue;  // an edge of another class (both ends in it)
      if (own) a1 = false;  // (set again below when it stays alive)
      if (!first) {
        // the previous round's prune: layer-0 edges by the layer-1 components and vice versa
        auto other = e < e0 ? E.deg1 : E.deg0;
        if (uf_load(other, u) != uf_load(other, v)) {
          E.kill(e, E_PRUNED);
          if (e < e0) c0++; else c1++;
          continue;
        }
      }
      if (first && cover >= 0 && (u == cover || v == cover)) {
        E.kill(e, E_COVERED);
        if (e < e0) k0++; else k1++;
      } else {
        if (rk != nullptr && T.prof_any != nullptr) {
          const unsigned long long t0 = wall_clock64();
          uf_unite_r2<true>(e < e0 ? P0 : P1, u, v, rk, &d_ops, &d_fails);
          const unsigned long long dt = wall_clock64() - t0;
          d_tmax = dt > d_tmax ? dt : d_tmax;
          d_un++;
        } else if (rk != nullptr) {
          uf_unite_r2(e < e0 ? P0 : P1, u, v, rk);
        } else {
          uf_unite_h(e < e0 ? P0 : P1, u, v);
        }
        if (own) a1 = true;
      }
    }
    if (T.acc != nullptr) {  // diagnostics: workgroup 0's own union work (slot 88), before the barrier
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) T.acc[8] += wall_clock64() - T.t;
    }
    if (T.prof_any != nullptr) {  // slowest workgroup's union work (slot 89)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_fetch_max(T.prof_any + 9, wall_clock64() - T.t0any, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // per-thread union counts: 90 max parent loads + CASes of a thread, 91 their sum, 92 unions,
      // 93 the longest union (ticks), 94 failed CASes (summed over the step's rounds; maxima over
      // them); one set of atomics per workgroup
      unsigned long long mo = (unsigned long long)d_ops, so = mo, su = (unsigned long long)d_un,
                         sf = (unsigned long long)d_fails, mt = d_tmax;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const unsigned long long x = __shfl_xor(mo, o, 64), y = __shfl_xor(mt, o, 64);
        mo = x > mo ? x : mo;
        mt = y > mt ? y : mt;
        so += __shfl_xor(so, o, 64);
        su += __shfl_xor(su, o, 64);
        sf += __shfl_xor(sf, o, 64);
      }
      unsigned long long* lt = (unsigned long long*)T.tmp;  // [8 waves][5]
      if (lane_id() == 0) {
        lt[wave_id() * 5 + 0] = mo;
        lt[wave_id() * 5 + 1] = so;
        lt[wave_id() * 5 + 2] = su;
        lt[wave_id() * 5 + 3] = mt;
        lt[wave_id() * 5 + 4] = sf;
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        for (int w = 1; w < NTHREADS / 64; ++w) {
          mo = max(mo, lt[w * 5 + 0]);
          so += lt[w * 5 + 1];
          su += lt[w * 5 + 2];
          mt = max(mt, lt[w * 5 + 3]);
          sf += lt[w * 5 + 4];
        }
        __hip_atomic_fetch_max(T.prof_any + 10, mo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(T.prof_any + 11, so, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(T.prof_any + 12, su, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_max(T.prof_any + 13, mt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(T.prof_any + 14, sf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
    }
    if (grid_sync(p, *T.target, T.flag)) return true;
    TEAM_ACC(T, 1);
    if (T.acc != nullptr && threadIdx.x == 0) T.acc[0] += 1;
    // labels of this round; the next round's parents reset (nobody reads them in this round)
    int* const Q0 = pb[(round + 1) & 1][0];
    int* const Q1 = pb[(round + 1) & 1][1];
    long long diff = 0;
    const unsigned long long tl0 = T.prof_any != nullptr ? wall_clock64() : 0ull;
    for (int x = T.gt; x < n; x += T.gs) {
      if (x == T.gt ? !x1in : (rs && uf_load(cls, x) != La)) continue;  // labels of the untouched classes stay
      int r0, r1;
      if (sk0) {
        r0 = uf_load(E.deg0, x);
        r1 = uf_find_h(P1, x);
        uf_store(E.deg1, x, r1);
      } else if (sk1) {
        r0 = uf_find_h(P0, x);
        r1 = uf_load(E.deg1, x);
        uf_store(E.deg0, x, r0);
      } else {
        const int2 rr = uf_find2_h(P0, P1, x);
        r0 = rr.x;
        r1 = rr.y;
        uf_store(E.deg0, x, r0);
        uf_store(E.deg1, x, r1);
      }
      uf_store(Q0, x, x);
      uf_store(Q1, x, x);
      diff += r0 != r1;
    }
    if (T.prof_any != nullptr) {  // slowest workgroup's label work (slot 95: the largest of the step's rounds)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_fetch_max(T.prof_any + 15, wall_clock64() - tl0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const long long v5[5] = {diff, k0, k1, c0, c1};
    long long t5[5];
    if (team_reduce<5>(p, T, v5, 0u, t5, nullptr)) return true;
    TEAM_ACC(T, 2);
    if (first && cover >= 0) {
      cc[0] = (int)t5[1];
      cc[1] = (int)t5[2];
    }
    pr[0] += (int)t5[3];
    pr[1] += (int)t5[4];
    cq0 = t5[3];
    cq1 = t5[4];
    if (t5[0] == 0) break;
  }
  // the LMCC: non-covered nodes per component (layer-0 label = layer-1 label at the fixed point);
  // the largest count is the maximum over the adds' results (each word's last add sees its total)
  // (restricted: the untouched classes' sizes from cnt at their roots, C_a's recounted; cls takes
  // the new labels)
  long long best = 0;
  for (int xb = T.gt - lane_id(); xb < n; xb += T.gs) {
    const int x = xb + lane_id();
    const int cx = x < n && rs ? uf_load(cls, x) : La;
    const bool mine = x < n && cx == La;  // (unrestricted: every node)
    if (x < n && !mine && cx == x) best = max(best, (long long)uf_load(cnt, x));
    const int lab = mine ? uf_load(E.deg0, x) : 0;
    const bool on = mine && !E.covered(x);
    best = max(best, (long long)agg_add1_max(cnt, on ? lab : 0, on));
    if (mine && cls != nullptr) uf_store(cls, x, lab);
  }
  const long long vb[1] = {best};
  long long tb[1];
  if (team_reduce<1>(p, T, vb, 1u, tb, nullptr)) return true;
  TEAM_ACC(T, 4);
  lm = (int)tb[0];
  return false;
}

// env_features on the whole grid: residual degrees by edge-parallel atomics, then per workgroup a
// contiguous node range (workgroup order = ascending ids) for the live list, its base from the
// live counts of the lower workgroups.
// dg: the degree arrays (2n words of gscr); zeroed: already zeroed (by the fixed point's init pass).
__device__ bool team_features(KParams& p, Team& T, const EnvView<true>& E, int n, int* gdeg0, int* gdeg1, float* lv,
                              float* q, EnvAgg& ag, int* dg, bool zeroed) {
  const int e0 = E.e0;
  if (T.acc != nullptr && threadIdx.x == 0) T.t = wall_clock64();
  if (!zeroed) {
    for (int x = T.gt; x < n; x += T.gs) {
      uf_store(dg, x, 0);
      uf_store(dg, n + x, 0);
    }
    if (grid_sync(p, *T.target, T.flag)) return true;
  }
  // (layer 1's degrees follow layer 0's: one index space l * n + node for the combined atomics)
  for (int eb = T.gt - lane_id(); eb < E.et; eb += T.gs) {
    const int e = eb + lane_id();
    const bool on = e < E.et && E.state(e) == E_ALIVE;
    const int base = e < e0 ? 0 : n;
    agg_add1(dg, on ? base + E.u(e) : 0, on);
    agg_add1(dg, on ? base + E.v(e) : 0, on);
  }
  if (grid_sync(p, *T.target, T.flag)) return true;
  const int cw = (n + p.n_main - 1) / p.n_main;
  const int w0 = min(n, (int)blockIdx.x * cw), w1 = min(n, w0 + cw);
  const int ct = (w1 - w0 + NTHREADS - 1) / NTHREADS;
  const int x0 = min(w1, w0 + (int)threadIdx.x * ct), x1 = min(w1, x0 + ct);
  long long nlive = 0, dm0 = 0, dm1 = 0, sd0 = 0, sd1 = 0, bad = 0, th0 = 0, th1 = 0;
  for (int x = x0; x < x1; ++x) {
    const int d0 = uf_load(dg, x), d1 = uf_load(dg, n + x);
    stc(gdeg0 + x, d0);
    stc(gdeg1 + x, d1);
    stc(q + x, NEG_INF);
    bad |= ((d0 > 0) != (d1 > 0));
    if (d0 > 0) {
      nlive++;
      dm0 = max(dm0, (long long)d0);
      dm1 = max(dm1, (long long)d1);
      th0 += (long long)d0 * (d0 - 1) / 2;
      th1 += (long long)d1 * (d1 - 1) / 2;
    }
    sd0 += d0;
    sd1 += d1;
  }
  int wtot = 0;
  const int off = block_excl_scan((int)nlive, T.tmp, &wtot);
  const long long v8[8] = {nlive, sd0, sd1, bad, th0, th1, dm0, dm1};
  long long t8[8], before = 0;
  if (team_reduce<8>(p, T, v8, 0xc0u, t8, &before)) return true;
  int k = (int)before + off;
  for (int x = x0; x < x1; ++x) {
    if (uf_load(dg, x) > 0) {
      const int b0 = E.grp[0][x], b1 = E.grp[1][x];
      const int x0e = E.grp[0][x + 1], x1e = E.grp[1][x + 1];
      if (MD_BOK(k < n, 9))
        stc4(lv, k * 16, make_float4(__int_as_float(x), __int_as_float(b0), __int_as_float(b1),
                                     __int_as_float((x0e - b0) | ((x1e - b1) << 16))));
      ++k;
    }
  }
  TEAM_ACC(T, 5);
  ag.nlive = (int)t8[0];
  ag.sd0 = (int)t8[1];
  ag.sd1 = (int)t8[2];
  ag.bad = t8[3] != 0;
  ag.th0 = t8[4];
  ag.th1 = t8[5];
  ag.dm0 = (int)t8[6];
  ag.dm1 = (int)t8[7];
  return false;
}

// ------------------------------------------------------------------ batched prefixes (stepRatio)
// A prediction with stepRatio > 0 applies k picks a_1..a_k one by one, each followed by the
// mutual-LMCC cascade (U/MultiDismantler_torch.py:725-735, U/mvc_env.py:74-87, U/Mcc.py:30-38):
// k dependent grid-wide fixed points.  But the state after a_1..a_j has the same alive edges,
// partition and LMCC as ONE cascade of the prediction's start state with all of a_1..a_j covered
// (the fixed point is the coarsest partition whose classes are connected in both layers by
// edges inside them; the partitions only refine as nodes go, so an edge pruned earlier crosses
// every later partition: tests/test_prefix_states.py checks it on the oracle).  So the k
// prefixes are independent: workgroup j - 1 computes prefix j's fixed point in its own LDS, all
// at once, from the start state's alive edges (a compact list in HBM, read from L2 by every
// workgroup), and publishes its LMCC, alive counts and alive bitmap; then every alive edge's
// death step d(e) -- the first prefix without it (the bitmaps are nested) -- decides its fate:
// covered when it touches a_d(e) (numCoveredEdges, U/mvc_env.py:81-84), pruned otherwise
// (remove_edge).  The picks stop at the first terminal prefix (GetSolution's `continue`).
// pfx (HBM, md_abi.cpp): [0, et) compact start list u | v << 16, [et, 2 et) its edge ids,
// [2 et, + 4 TEAM_MAX_WG) per-prefix records {lmcc, alive 0, alive 1, -}, then per prefix the
// alive bitmap of the compact list (pfx_bw words).
__host__ __device__ inline int pfx_bw(int et) { return (et + 31) >> 5; }
constexpr int PFX_PROF_ROW = 2048;  // diagnostics: per-prefix rounds and ticks of the last batch (md_profile)
__host__ __device__ inline long long pfx_words(int et) { return 2LL * et + 4LL * TEAM_MAX_WG + (long long)TEAM_MAX_WG * pfx_bw(et); }
// LDS words of one prefix's fixed point: u16 parents of both layers, the prefix's cover bitmap,
// the alive bitmap of the compact list, reduction words
__host__ __device__ inline int pfx_lds_words(int n, int et) { return 2 * ((n + 1) >> 1) + ((n + 31) >> 5) + pfx_bw(et) + 64; }
__host__ __device__ inline bool pfx_fits(int n, int et) { return n <= 65535 && pfx_lds_words(n, et) <= A_WORDS; }

// u16 union-find in LDS (two parents per word; parents point to smaller ids, so a tree's root is
// its least node): 16-bit loads and path-halving stores, the hook a 32-bit compare-and-swap of
// the word holding the root (a change of the other half fails it, and it is retried on the new
// word: the root's own half decides)
__device__ __forceinline__ int p16_ld(lds_u16* P, int i) {
  return __hip_atomic_load(P + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void p16_st(lds_u16* P, int i, int v) {
  __hip_atomic_store(P + i, (uint16_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ bool p16_hook(lds_u16* P, int r, int to) {
  lds_u32* w = (lds_u32*)(P) + (r >> 1);
  const int sh = (r & 1) << 4;
  unsigned old = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (true) {
    if (((old >> sh) & 0xffffu) != (unsigned)r) return false;
    const unsigned nw = (old & ~(0xffffu << sh)) | ((unsigned)to << sh);
    unsigned ex = old;
    if (__hip_atomic_compare_exchange_strong(w, &ex, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
      return true;
    old = ex;
  }
}
__device__ __forceinline__ int p16_find(lds_u16* P, int v) {
  int cur = p16_ld(P, v);
  if (cur != v) {
    int prev = v, next;
    while (cur > (next = p16_ld(P, cur))) {
      p16_st(P, prev, next);  // path halving; benign race (values only shrink)
      prev = cur;
      cur = next;
    }
  }
  return cur;
}
// a root without path stores (the label pass: a halving store could replace a root another
// thread just stored as x's label with an older ancestor)
__device__ __forceinline__ int p16_root(lds_u16* P, int v) {
  int next;
  while ((next = p16_ld(P, v)) != v) v = next;
  return v;
}
// both layers' roots of x, the two read-only walks in lockstep
__device__ __forceinline__ int2 p16_root2(lds_u16* P0, lds_u16* P1, int x) {
  int a = x, b = x;
  while (true) {
    const int na = p16_ld(P0, a), nb = p16_ld(P1, b);
    if (na == a && nb == b) return make_int2(a, b);
    a = na;
    b = nb;
  }
}
__device__ __forceinline__ void p16_unite(lds_u16* P, int a, int b) {
  while (true) {
    a = p16_find(P, a);
    b = p16_find(P, b);
    if (a == b) return;
    if (a > b) { const int t = a; a = b; b = t; }
    if (p16_hook(P, b, a)) return;
  }
}

// The next kc actions (from index k0) of graph E.gi as batched prefixes.  Returns -1 on a grid
// error, 0 when the batch cannot take this path (an action out of range, covered or repeated: the
// sequential loop applies the actions before it and reports it, as the reference's assert would),
// else 1 with *J the actions applied (fewer than kc when a prefix is terminal), cnt the covered /
// pruned edges per layer {c0, c1, pr0, pr1}, and workgroup 0's books (covered flags, trace,
// GraphVar counters) updated.  Uses the LDS from L_W on (the caller reloads the weight image).
__device__ __forceinline__ int pfx_act(KParams& p, const GraphInfo& gi, int k, int pend_first) {
  return k == 0 && pend_first >= 0 ? pend_first : __hip_atomic_load(p.pend + gi.node_off + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __noinline__ int team_prefix_step(KParams& p, Team& T, const EnvView<true>& E, int k0, int kc, int pend_first, bool books,
                                int* Jout, int (&cnt)[4]) {
  const GraphInfo& gi = *E.gi;
  const int n = gi.n, et = E.et, e0 = E.e0;
  const int lane = lane_id(), wv = wave_id();
  int* const puv = p.pfx;
  int* const pe = p.pfx + et;
  int* const rec = p.pfx + 2 * et;
  int* const dbm = p.pfx + 2 * et + 4 * TEAM_MAX_WG;
  const int bw = pfx_bw(et);
  // diagnostics (md_profile, scripts/prefix_prof.py): slots 80.. of the step -- 80 most rounds of
  // any prefix, 81 list + validation (workgroup 0), 82 the slowest prefix's fixed point, 83 death
  // steps + reduction (workgroup 0), and the last prefix's pieces: 84 init + alive bits, 86 union,
  // 88 labels, 89 prune, 90 LMCC + stores, 91 its rounds; 92 prefixes, 93 applied
  unsigned long long* const pa = T.prof_any;
  unsigned long long tp0 = pa != nullptr ? wall_clock64() : 0ull, tp1 = tp0;
  // ---- the compact list of the start state's alive edges, in edge order (layer 0 first): each
  // workgroup a contiguous edge range, each thread a contiguous part of it
  const int cw = (et + p.n_main - 1) / p.n_main;
  const int w0 = min(et, (int)blockIdx.x * cw), w1 = min(et, w0 + cw);
  const int ct = (w1 - w0 + NTHREADS - 1) / NTHREADS;
  const int x0 = min(w1, w0 + (int)threadIdx.x * ct), x1 = min(w1, x0 + ct);
  long long na = 0, na0 = 0;
  for (int e = x0; e < x1; ++e) {
    const bool a = E.state(e) == E_ALIVE;
    na += a;
    na0 += a && e < e0;
  }
  int wtot = 0;
  const int off = block_excl_scan((int)na, T.tmp, &wtot);
  const long long v2[2] = {na, na0};
  long long t2[2], before = 0;
  if (team_reduce<2>(p, T, v2, 0u, t2, &before)) return -1;
  const int mc = (int)t2[0], mc0 = (int)t2[1];
  {
    int k = (int)before + off;
    for (int e = x0; e < x1; ++e) {
      if (E.state(e) != E_ALIVE) continue;
      stc(puv + k, E.u(e) | (E.v(e) << 16));
      stc(pe + k, e);
      ++k;
    }
  }
  // ---- LDS (from L_W): P0, P1 (u16), cover bitmap of the prefix, alive bitmap of the list
  const int h = (n + 1) >> 1, nb = (n + 31) >> 5, ab = (mc + 31) >> 5;
  lds_u32* const R = (lds_u32*)(unsigned*)(lds_base() + L_W);
  lds_u16* const P0 = (lds_u16*)(R);
  lds_u16* const P1 = (lds_u16*)(R + h);
  lds_u32* const cb = R + 2 * h;
  lds_u32* const abm = cb + nb;
  int* const tmp = (int*)(lds_base() + L_W) + 2 * h + nb + ab;
  // validation (every workgroup, same verdict): range, not covered, no repeats
  for (int i = threadIdx.x; i < nb; i += NTHREADS) cb[i] = 0u;
  __syncthreads();
  bool bad = false;
  for (int k = threadIdx.x; k < kc; k += NTHREADS) {
    const int a = pfx_act(p, gi, k0 + k, pend_first);
    if (a < 0 || a >= n || E.covered(a)) {
      bad = true;
    } else {
      const unsigned m = 1u << (a & 31);
      if (__hip_atomic_fetch_or(cb + (a >> 5), m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) & m) bad = true;
    }
  }
  bad = __syncthreads_or(bad);
  // (the list's stores must be visible before anyone reads it: every path below crosses a barrier)
  if (grid_sync(p, *T.target, T.flag)) return -1;
  if (bad) return 0;
  // The list is read-only from here to the next batch: one L1 invalidate (an agent-scope acquire)
  // and then plain loads, which the L1 serves (a thread's run of the union pass walks its lines
  // 16 bytes at a time) -- the agent-coherent loads elsewhere in this file always go to the L2.
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const unsigned* const puvc = (const unsigned*)puv;
  const uint4* const puv4 = (const uint4*)puv;  // (p.pfx is 256-byte aligned)
  const int j = (int)blockIdx.x + 1;  // this workgroup's prefix
  const bool plast = pa != nullptr && j == kc && threadIdx.x == 0;
  if (pa != nullptr && blockIdx.x == 0 && threadIdx.x == 0) pa[1] = wall_clock64() - tp0;
  if (pa != nullptr) tp0 = tp1 = wall_clock64();
  auto lap = [&](int k) {  // the last prefix's piece k (diagnostics)
    if (plast) {
      const unsigned long long t = wall_clock64();
      pa[k] += t - tp1;
      tp1 = t;
    }
  };
  if (j <= kc) {
    for (int i = threadIdx.x; i < nb; i += NTHREADS) cb[i] = 0u;
    for (int x = threadIdx.x; x < n; x += NTHREADS) {
      p16_st(P0, x, x);
      p16_st(P1, x, x);
    }
    __syncthreads();
    for (int k = threadIdx.x; k < j; k += NTHREADS) {
      const int a = pfx_act(p, gi, k0 + k, pend_first);
      __hip_atomic_fetch_or(cb + (a >> 5), 1u << (a & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    // alive bits: the start's alive edges without the prefix's covered nodes (a wave's 64 entries
    // per ballot)
    for (int ib = wv * 64; ib < mc; ib += NTHREADS) {
      const int i = ib + lane;
      bool al = false;
      if (i < mc) {
        const unsigned uv = puvc[i];
        const int u = (int)(uv & 0xffffu), v = (int)(uv >> 16);
        al = !((cb[u >> 5] >> (u & 31)) & 1u) && !((cb[v >> 5] >> (v & 31)) & 1u);
      }
      const unsigned long long m = __ballot(al);
      if (lane == 0) abm[ib >> 5] = (unsigned)m;
      if (lane == 1 && (ib >> 5) + 1 < ab) abm[(ib >> 5) + 1] = (unsigned)(m >> 32);
    }
    __syncthreads();
    lap(4);
    // Jacobi rounds (mcc_fixed_point's): union both layers, label, prune each layer's edges by
    // the other layer's labels; a layer that lost no edge keeps its labels (no reset, union or
    // relabel); no edge pruned = the partitions agree = the fixed point
    bool ch0 = true, ch1 = true;
    // the union pass's runs: whole 4-entry chunks per thread
    const int nq = (mc + 3) >> 2, cq = (nq + NTHREADS - 1) / NTHREADS;
    const int q0 = min(nq, (int)threadIdx.x * cq), q1 = min(nq, q0 + cq);
    int nrounds = 0;
    for (int round = 0;; ++round) {
      if (round > 0) {
        for (int x = threadIdx.x; x < n; x += NTHREADS) {
          if (ch0) p16_st(P0, x, x);
          if (ch1) p16_st(P1, x, x);
        }
        __syncthreads();
      }
      // union: a contiguous run of the list per thread (consecutive edges share endpoints)
      {
        const int ia = ch0 ? 0 : mc0, ib = ch1 ? mc : mc0;  // entries of the layers to unite
        const int qa = max(q0, ia >> 2), qb = min(q1, (ib + 3) >> 2);
        uint4 nxt = qa < qb ? puv4[qa] : make_uint4(0u, 0u, 0u, 0u);
        for (int q = qa; q < qb; ++q) {
          const uint4 w = nxt;
          if (q + 1 < qb) nxt = puv4[q + 1];  // one chunk ahead
          const unsigned bits = abm[q >> 3] >> ((q & 7) << 2);  // the chunk's 4 alive bits
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int i = 4 * q + k;
            if (i < ia || i >= ib || !((bits >> k) & 1u)) continue;
            const unsigned uv = k == 0 ? w.x : k == 1 ? w.y : k == 2 ? w.z : w.w;
            p16_unite(i < mc0 ? P0 : P1, (int)(uv & 0xffffu), (int)(uv >> 16));
          }
        }
      }
      __syncthreads();
      lap(6);
      // labels: every node's root, stored as its parent
      for (int x = threadIdx.x; x < n; x += NTHREADS) {
        if (ch0 && ch1) {
          const int2 r = p16_root2(P0, P1, x);
          p16_st(P0, x, r.x);
          p16_st(P1, x, r.y);
        } else {
          if (ch0) p16_st(P0, x, p16_root(P0, x));
          if (ch1) p16_st(P1, x, p16_root(P1, x));
        }
      }
      __syncthreads();
      lap(8);
      // prune (coalesced: entries strided over the block)
      int c0 = 0, c1 = 0;
      for (int i = threadIdx.x; i < mc; i += NTHREADS) {
        if (!((abm[i >> 5] >> (i & 31)) & 1u)) continue;
        const unsigned uv = puvc[i];
        const int u = (int)(uv & 0xffffu), v = (int)(uv >> 16);
        lds_u16* const other = i < mc0 ? P1 : P0;  // layer-0 edges by the layer-1 labels
        if (p16_ld(other, u) != p16_ld(other, v)) {
          __hip_atomic_fetch_and(abm + (i >> 5), ~(1u << (i & 31)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (i < mc0) c0++; else c1++;
        }
      }
      const int2 cs = block_sum2(c0, c1, tmp);
      __syncthreads();
      lap(9);
      ++nrounds;
      if (plast) pa[11] += 1;
      if (pa != nullptr && threadIdx.x == 0)
        __hip_atomic_fetch_max(pa, (unsigned long long)(round + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (cs.x == 0 && cs.y == 0) break;
      ch0 = cs.x > 0;
      ch1 = cs.y > 0;
    }
    // LMCC: non-covered nodes per layer-0 label, counted in P1's words (two u16 counts each)
    for (int i = threadIdx.x; i < h; i += NTHREADS) R[h + i] = 0u;
    __syncthreads();
    for (int x = threadIdx.x; x < n; x += NTHREADS) {
      if ((cb[x >> 5] >> (x & 31)) & 1u) continue;
      if (E.covered(x)) continue;
      const int r = p16_ld(P0, x);
      __hip_atomic_fetch_add(R + h + (r >> 1), 1u << ((r & 1) << 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    int best = 0, al0 = 0, al1 = 0;
    for (int i = threadIdx.x; i < h; i += NTHREADS) {
      const unsigned w = R[h + i];
      best = max(best, (int)max(w & 0xffffu, w >> 16));
    }
    for (int i = threadIdx.x; i < ab; i += NTHREADS) {
      const unsigned w = abm[i];
      stc(dbm + (size_t)(j - 1) * bw + i, (int)w);
      // bits of entries [32 i, 32 i + 32): layer 0 below mc0
      const int lo = 32 * i;
      const unsigned m0 = mc0 <= lo ? 0u : (mc0 >= lo + 32 ? ~0u : ((1u << (mc0 - lo)) - 1u));
      al0 += __popc(w & m0);
      al1 += __popc(w & ~m0);
    }
    best = block_max_int(best, tmp);
    const int2 al = block_sum2(al0, al1, tmp);
    __syncthreads();
    if (threadIdx.x == 0) {
      stc(rec + 4 * (j - 1), best);
      stc(rec + 4 * (j - 1) + 1, al.x);
      stc(rec + 4 * (j - 1) + 2, al.y);
    }
    lap(10);
    if (pa != nullptr && threadIdx.x == 0) {
      const unsigned long long dt = wall_clock64() - tp0;
      __hip_atomic_fetch_max(pa + 2, dt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // per prefix (rows PFX_PROF_ROW..; MD_PROF_ALL=1 reads them): rounds, device ticks
      if (p.prof_cap > PFX_PROF_ROW + 24 && j <= 1024) {
        p.prof[(size_t)PFX_PROF_ROW * PROF_SLOTS + (j - 1)] = (unsigned long long)nrounds;
        p.prof[(size_t)PFX_PROF_ROW * PROF_SLOTS + 1024 + (j - 1)] = dt;
      }
    }
  }
  if (grid_sync(p, *T.target, T.flag)) return -1;
  if (pa != nullptr) tp0 = wall_clock64();
  // ---- the applied prefix: the first terminal one, else kc (every workgroup, same answer)
  int jt = kc;
  for (int q = threadIdx.x; q < kc; q += NTHREADS) {
    if (ldc(rec + 4 * q + 1) == 0 || ldc(rec + 4 * q + 2) == 0) {
      jt = q + 1;
      break;
    }
  }
  for (int o = 32; o > 0; o >>= 1) jt = min(jt, __shfl_xor(jt, o, 64));
  int* const ltmp = T.tmp;
  if (lane == 0) ltmp[wv] = jt;
  __syncthreads();
  int J = ltmp[0];
#pragma unroll
  for (int q = 1; q < NTHREADS / 64; ++q) J = min(J, ltmp[q]);
  __syncthreads();
  // ---- each start edge's death step (the bitmaps are nested: binary search over 1..J)
  long long c0 = 0, c1 = 0, q0 = 0, q1 = 0;
  for (int i = T.gt; i < mc; i += T.gs) {
    const unsigned m = 1u << (i & 31);
    if ((unsigned)ldc(dbm + (size_t)(J - 1) * bw + (i >> 5)) & m) continue;  // alive after the batch
    int lo = 1, hi = J;  // first prefix without the edge
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if ((unsigned)ldc(dbm + (size_t)(mid - 1) * bw + (i >> 5)) & m) lo = mid + 1; else hi = mid;
    }
    const int a = pfx_act(p, gi, k0 + lo - 1, pend_first);
    const unsigned uv = (unsigned)ldc(puv + i);
    const bool cov = (int)(uv & 0xffffu) == a || (int)(uv >> 16) == a;
    E.kill(ldc(pe + i), cov ? E_COVERED : E_PRUNED);
    if (i < mc0) { if (cov) c0++; else q0++; } else { if (cov) c1++; else q1++; }
  }
  const long long v4[4] = {c0, c1, q0, q1};
  long long t4[4];
  if (team_reduce<4>(p, T, v4, 0u, t4, nullptr)) return -1;
  for (int k = 0; k < 4; ++k) cnt[k] = (int)t4[k];
  if (pa != nullptr && blockIdx.x == 0 && threadIdx.x == 0) {
    pa[3] = wall_clock64() - tp0;
    pa[12] = (unsigned long long)kc;
    pa[13] = (unsigned long long)J;
  }
  if (books) {
    GraphVar& gv = *(GraphVar*)(lds_base() + L_GV);
    const int st0 = gv.steps;
    for (int q = threadIdx.x; q < J; q += NTHREADS) {
      const int a = pfx_act(p, gi, k0 + q, pend_first);
      stc(E.gcov + a, (uint8_t)1);
      if (MD_BOK(st0 + q < gi.n, 8)) {
        stc(p.tr_action + gi.node_off + st0 + q, a);
        stc(p.tr_rank + gi.node_off + st0 + q, ldc(rec + 4 * q));
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      gv.counter[0] += cnt[0];
      gv.counter[1] += cnt[1];
      gv.removed[0] += cnt[2];
      gv.removed[1] += cnt[3];
      gv.alive[0] -= cnt[0] + cnt[2];
      gv.alive[1] -= cnt[1] + cnt[3];
      gv.n_cov += J;
      gv.lmcc = ldc(rec + 4 * (J - 1));
      gv.steps += J;
    }
    __syncthreads();
  }
  *Jout = J;
  return 1;
}

// The environment step of graph g on every workgroup of the launch (env_step's work once the
// actions are known): workgroup 0 holds the graph's GraphVar in LDS and keeps its books (the
// others read the counts they need from the partials); pend_n actions, the first pend_first
// (or p.pend[0] when < 0).  Returns an ERR_* code (0: ok) in *err; true on a grid error.
// (*err bit 30: the weight image's LDS was used -- the caller reloads it)
constexpr int TEAM_WDIRTY = 1 << 30;
__device__ bool team_env_step(KParams& p, Team& T, int g, int pend_n, int pend_first, int* err) {
  const GraphInfo gi = p.ginfo[g];
  const int n = gi.n;
  GraphVar& gv = *(GraphVar*)(lds_base() + L_GV);
  const bool books = blockIdx.x == 0;
  const EnvView<true> E = env_view<true>(p, gi, (int*)(lds_base() + L_SCR));
  // (gscr_team: graph-local, sized for the largest loaded graph; md_abi.cpp clears lab_ok of a
  // graph whenever another graph ran the grid-wide step since it last did)
  int* cnt = p.gscr_team;                // LMCC counts (n)
  int* dg = p.gscr_team + 3 * n;         // the features' degrees (2n)
  int* cls = p.gscr_team + 5 * n;        // class labels (team_fixed_point)
  bool zeroed = false;  // dg zeroed by a fixed point's init pass

  // every workgroup follows the same control flow: alive counts and s0 from the graph's
  // GraphVar as the last phase A stored it
  int alive0 = ldc(&p.gvar[g].alive[0]), alive1 = ldc(&p.gvar[g].alive[1]);
  const int s0_done = ldc(&p.gvar[g].s0_done);
  // the class labels and sizes are current when the last state change was this step's (every
  // workgroup reads the flag before workgroup 0 can set it: the first fixed point's barrier)
  bool labels = p.lab_ok != nullptr && ldc(p.lab_ok + g) != 0 && s0_done;
  // the static union ranks (md_abi.cpp, at load) in the tile scratch, free during the step (after
  // the team's own reduction words)
  const lds_u16* rk = nullptr;
  if (p.prank != nullptr && gi.rank_off >= 0 && n <= TEAM_RANK_MAX) {
    lds_u16* dst = (lds_u16*)(uint16_t*)(lds_base() + L_SCR + TEAM_RANK_OFF);
    const unsigned* src = (const unsigned*)(p.prank + gi.rank_off);  // (rank_off even)
    const int nw = (n + 1) >> 1;
    for (int i = threadIdx.x; i < nw; i += NTHREADS) ((lds_u32*)(unsigned*)dst)[i] = src[i];
    __syncthreads();
    rk = dst;
  }
  *err = 0;
  // batched prefixes (stepRatio): chunks of up to n_main actions at once while at least
  // pfx_min remain (team_prefix_step); an invalid action leaves them to the loop below
  int k0 = 0;
  bool wdirty = false;
  while (p.pfx != nullptr && p.pfx_min > 0 && s0_done && pend_n - k0 >= p.pfx_min && alive0 > 0 && alive1 > 0 &&
         pfx_fits(n, E.et)) {
    const int kc = min(pend_n - k0, p.n_main);
    int J = 0, cnt[4];
    wdirty = true;  // (the LDS from L_W on, even when the batch is refused)
    const int r = team_prefix_step(p, T, E, k0, kc, pend_first, books, &J, cnt);
    if (r < 0) return true;
    if (r == 0) break;
    labels = false;  // (the class labels are the last fixed point's of the sequential loop)
    alive0 -= cnt[0] + cnt[2];
    alive1 -= cnt[1] + cnt[3];
    k0 += J;
    if (J < kc) {  // terminal
      k0 = pend_n;
      break;
    }
  }
  if (wdirty && rk != nullptr) {  // the static ranks again (their LDS was the prefixes')
    lds_u16* dst = (lds_u16*)(uint16_t*)(lds_base() + L_SCR + TEAM_RANK_OFF);
    const unsigned* src = (const unsigned*)(p.prank + gi.rank_off);
    for (int i = threadIdx.x; i < ((n + 1) >> 1); i += NTHREADS) ((lds_u32*)(unsigned*)dst)[i] = src[i];
    __syncthreads();
  }
  for (int k = k0; k < pend_n; ++k) {
    if (alive0 == 0 || alive1 == 0) break;  // terminal between queued actions
    const int a = k == 0 && pend_first >= 0 ? pend_first
                                            : __hip_atomic_load(p.pend + gi.node_off + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a < 0 || a >= n) { *err = ERR_BADNODE; break; }
    if (E.covered(a)) { *err = ERR_COVERED; break; }
    int pr[2], c[2], lm = 0;
    // (workgroup 0 sets covered(a) after the fixed point's first barrier: every workgroup has
    // read it by then)
    if (team_fixed_point(p, T, E, cnt, a, books, lm, pr, c, zeroed ? nullptr : dg, cls, labels, rk)) return true;
    zeroed = true;
    labels = true;
    alive0 -= c[0] + pr[0];
    alive1 -= c[1] + pr[1];
    if (books && threadIdx.x == 0) {
      gv.counter[0] += c[0];
      gv.counter[1] += c[1];
      gv.removed[0] += pr[0];
      gv.removed[1] += pr[1];
      gv.alive[0] -= c[0] + pr[0];
      gv.alive[1] -= c[1] + pr[1];
      gv.n_cov += 1;
      gv.lmcc = lm;
      if (MD_BOK(gv.steps < gi.n, 8)) {
        stc(p.tr_action + gi.node_off + gv.steps, a);
        stc(p.tr_rank + gi.node_off + gv.steps, lm);
      }
      gv.steps += 1;
    }
  }
  if (!s0_done && *err == 0) {
    int pr[2], lm = 0;
    if (team_fixed_point(p, T, E, cnt, -1, false, lm, pr, nullptr, zeroed ? nullptr : dg, cls, false, rk)) return true;
    zeroed = true;
    labels = true;
    if (books && threadIdx.x == 0) {
      gv.removed[0] += pr[0];
      gv.removed[1] += pr[1];
      gv.max_rank = lm;
      gv.lmcc = lm;
      gv.s0_done = 1;
    }
  }
  // the labels stay current for the next step only when every fixed point ran here (a step with
  // no fixed point, e.g. a terminal graph's queued action, changes nothing)
  if (books && threadIdx.x == 0 && p.lab_ok != nullptr) stc(p.lab_ok + g, (labels && *err == 0) ? 1 : 0);
  EnvAgg ag;
  if (team_features(p, T, E, n, p.deg[0] + gi.node_off, p.deg[1] + gi.node_off, (float*)(p.live + 4 * (size_t)gi.node_off),
                    p.q + gi.node_off, ag, dg, zeroed))
    return true;
  if (books) {
    if (ag.bad && *err == 0) *err = ERR_LIVE_MISMATCH;
    const int hd0 = gv.hdmax[0], hd1 = gv.hdmax[1];
    __syncthreads();
    if (threadIdx.x == 0) {
      gv.n_live = ag.nlive;
      gv.dmax[0] = ag.dm0;
      gv.dmax[1] = ag.dm1;
      gv.alive[0] = ag.sd0 / 2;
      gv.alive[1] = ag.sd1 / 2;
      gv.twohop[0] = ag.th0;
      gv.twohop[1] = ag.th1;
    }
    h0_update(p, gi, gv, ag.dm0, ag.dm1, hd0, hd1);
    __syncthreads();
  }
  if (wdirty) *err |= TEAM_WDIRTY;
  return false;
}
