// md_abi.cpp — C ABI of libmdroll.so (declared in include/mdroll.h).
//
// Owns all device memory of a context, builds the CSR adjacency in the reference's
// neighbour order, drives the persistent rollout kernel and resolves exact Q ties on the
// host through the caller's callback (the reference's np.argsort order).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <string>
#include <unordered_set>
#include <thread>
#include <chrono>
#include <vector>

#include "../../include/mdroll.h"
#include "md_common.h"

namespace md {
int lds_bytes();
int weight_image_floats();
bool phase_a_fits_lds_host(int n, int edges);
bool spec_fits_lds_host(int n, int edges);
bool pfx_fits_host(int n, int edges);
long long pfx_words_host(int edges);
void build_weight_image(const float* w, float* img);
hipError_t launch_rollout(const Params& p, const float* wimg, int grid, hipStream_t s);
hipError_t launch_h0(const float* w, float* tab, int dm_lo, int dm_hi, hipStream_t s);
hipError_t launch_reset(const Params& p, hipStream_t s);
hipError_t launch_clear(void* const* ptr, const size_t* bytes, int n, hipStream_t s);
hipError_t set_kernel_attrs();
}  // namespace md

using namespace md;

namespace {

constexpr double QMASK = -(2147483647.0 / 2.0);  // U/MultiDismantler_torch.py:60

// MD_TRACE=1 (diagnostics): every device allocation and every kernel launch to stderr, flushed,
// so a GPU memory-fault report (its faulting address) can be mapped to a buffer and a launch.
bool trace_on() {
  static const bool on = std::getenv("MD_TRACE") != nullptr && std::atoi(std::getenv("MD_TRACE")) != 0;
  return on;
}

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  hipError_t alloc(size_t count) {
    release();
    n = count;
    if (count == 0) return hipSuccess;
    const hipError_t e = hipMalloc((void**)&p, count * sizeof(T));
    if (trace_on())
      std::fprintf(stderr, "md trace: alloc %p .. %p (%zu B)\n", (void*)p, (void*)((char*)p + count * sizeof(T)),
                   count * sizeof(T));
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

// Mapped, coherent pinned host memory (the in-kernel host selection hand-shake).
template <class T>
struct HostBuf {
  T* h = nullptr;  // host pointer
  T* d = nullptr;  // device pointer
  hipError_t alloc(size_t count) {
    release();
    if (count == 0) return hipSuccess;
    hipError_t e = hipHostMalloc((void**)&h, count * sizeof(T), hipHostMallocMapped | hipHostMallocCoherent);
    if (e != hipSuccess) return e;
    std::memset(h, 0, count * sizeof(T));
    e = hipHostGetDevicePointer((void**)&d, h, 0);
    if (trace_on())
      std::fprintf(stderr, "md trace: host alloc %p .. %p (%zu B)\n", (void*)d, (void*)((char*)d + count * sizeof(T)),
                   count * sizeof(T));
    return e;
  }
  void release() {
    if (h) (void)hipHostFree(h);
    h = d = nullptr;
  }
};

}  // namespace

struct md_ctx {
  int device = 0;
  int cost_mode = MD_COST_UNIT;
  int cus = 256;
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::string err;
  int team_size_req = 0;
  int env_mode = 1;  // 1: dedicated environment workgroups for small batches
  int variant = 0;   // diagnostics knob (MD_VARIANT)
  int pair_on = 1;   // queue mode: paired tiles (MD_PAIR=0: one tile at a time)
  int bspec_on = 0;  // queue launches: speculative environment steps of the likely next pick (MD_BSPEC=1: on)
  DevBuf<int> bspec;
  long long bspec_half = 0;
  int wq_on = 1;     // queue mode: one work item per wave (md_wq_kernel; MD_WQ=0: per workgroup, md_queue_kernel)
  int wqpark = 128;  // wave-item launches of more than this many graphs; at most this many still running ->
                     // they continue in md_queue_kernel (whose per-step latency is lower; MD_WQPARK)
  int qpark = 4;     // queue mode: at most this many graphs left -> the lock-step kernel (MD_QPARK, 0 = off)
  double last_ms = 0.0;
  int last_launches = 0;

  DevBuf<float> w, wimg;
  DevBuf<float> h0g;  // unit cost: precomputed first-layer tables, dmax 1..h0g_dm
  int h0g_dm = 0;
  bool h0g_on = true;  // MD_H0G=0: rebuild the tables in phase A instead (tests)
  // graphs
  int ng = 0;
  std::vector<GraphInfo> hinfo;
  std::vector<GraphVar> hvar;
  size_t tot_n = 0, tot_e[2] = {0, 0}, tot_c[2] = {0, 0}, tot_r[2] = {0, 0};
  DevBuf<GraphInfo> ginfo;
  DevBuf<GraphVar> gvar;
  size_t tot_tiles = 0;
  DevBuf<int> rowptr[2], adj[2], adjx[2], epos[2], eu[2], ev[2];
  DevBuf<uint8_t> estate[2], calive[2], covered;
  DevBuf<int> deg[2], live, gscr, pend, tr_action, tr_rank, tr_stat, glist, ctl;
  DevBuf<long long> tpart;  // grid-wide environment step: per-workgroup partials [2][TEAM_MAX_WG][16]
  DevBuf<int> lab_ok;       // per graph: the grid-wide step's class labels are current
  DevBuf<int> gscr_team;    // the grid-wide step's graph-local scratch (GSCR_TEAM_WORDS x the largest n)
  int team_owner = -1;      // the graph whose class labels gscr_team holds
  DevBuf<uint16_t> prank;   // static union ranks (team_env_step), graphs of <= 65535 nodes
  DevBuf<float> H[2][2], h0tab[2], q, spart, apart, ybuf, hbuf, tr_q, node_w;
  DevBuf<unsigned long long> xbuf;
  DevBuf<int> nbc;  // neighbour-list cache slots (tiles of the largest launch)
  int nbc_slots = 0;
  DevBuf<int> gtoff;  // per launch graph slot: first tile within the launch (queue-mode cache slots)
  int max_tiles = 0;  // tiles of the largest loaded graph
  DevBuf<unsigned long long> qslot;  // queue-mode work items
  DevBuf<int> qg;                    // queue-mode per-graph stage counters
  DevBuf<unsigned> bars;  // grid-barrier counter shards
  // speculative environment steps (single-graph rollouts): result slots, Q of the last two
  // predictions; spec_n workgroups per launch when the CUs are free (MD_SPEC, 0 = off).
  // Default 32 (= SPEC_MAX): on gmm1000_s0 the pick is the previous prediction's rank 16-31 in
  // 2 of 65 steps (a miss costs ~45 us): 16 -> 32 gave 4.19 -> 4.11 ms, er1000 8.10 -> 7.73 ms
  DevBuf<int> sres;
  DevBuf<float> qspec;
  int sres_stride = 0;
  int spec_n = 32;
  unsigned launch_seq = 0;
  // host selection hand-shake
  int host_mode = 1;  // 1: ties / multi-node steps are answered inside the launch (MD_HOST_HANDSHAKE)
  md_argsort_f64 tie_argsort = nullptr;  // numpy's float64 argsort (md_set_tie_argsort), else the callback
  int poll_us = 0;    // host poll interval while serving (MD_POLL_US)
  HostBuf<unsigned> h_req, h_ans;
  HostBuf<int> h_nact, h_act;
  HostBuf<float> h_q;
  HostBuf<float> h_chk;
  HostBuf<unsigned> h_done;  // launch completion record {tag, error word} (kernel_exit)
  HostBuf<int> h_gvar;       // GraphVars of the last launch, copied by kernel_exit
  bool vars_stale = false;   // a launch ended without its completion record
  // md_reset_deferred left MvcEnv.s0's prune to the next md_rollout's first environment step;
  // any other call that reads or changes the state runs that prune first (finish_deferred_s0)
  bool s0_pending = false;
  bool need_gscr = false;
  DevBuf<unsigned long long> prof;
  int prof_cap = 0;
  // dataflow mode (single-graph rollouts without grid barriers, md_kernels.hip df_*): tagged
  // granule buffer sized for the largest graph that qualifies (df_graph); MD_DF=0 turns it off
  bool df_on = true;
  // speculative workgroups build the next step's state from the result phase A takes, before
  // its write-back (spec_loop early requests); MD_EARLY=0 turns it off
  bool early_on = true;
  // a speculative fixed point stops once phase A has taken another result of its request or a
  // later request is out (MD_SPEC_ABORT=0: always runs to the end)
  bool abort_on = true;
  bool fp_short = true;  // MD_FP_SHORTCUT=0: every fixed point runs its confirmation round
  bool fp_skip = true;   // MD_FP_SKIP=0: every LDS fixed-point round re-unites both layers
  int last_served = 0;   // host selection requests served by the last API call's launches
  int pfx_min = 8;       // MD_PREFIX: grid-wide steps take >= this many actions as batched prefixes (0: off)
  bool dev_topk = true;  // MD_DEVTOPK=0: every stepRatio prediction goes to the host's numpy routine
  bool eg_apply = true;  // MD_EG_APPLY=0: a K2 end-game answer is applied action by action
  DevBuf<int> pfx;       // their scratch (md_env.h pfx_words)
  HostBuf<int> h_tr;         // mapped host mirrors of tr_action [tot_n] and tr_rank [tot_n] (trace_publish)
  bool first_req = true;  // MD_FIRST_REQ=0: no speculative request at a rollout's first step
  DevBuf<unsigned long long> dfbuf;
  int df_mt = 0, df_n = 0;
  std::vector<char> df_graph;
  std::vector<unsigned long long> prof_host;

  ~md_ctx() {
    if (stream) {
      (void)hipStreamSynchronize(stream);
      (void)hipStreamDestroy(stream);
    }
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    w.release();
    wimg.release();
    prof.release();
    free_graphs();
  }
  void free_graphs() {
    ginfo.release();
    gvar.release();
    for (int l = 0; l < 2; ++l) {
      rowptr[l].release(); adj[l].release(); adjx[l].release(); epos[l].release(); eu[l].release(); ev[l].release();
      estate[l].release(); calive[l].release(); deg[l].release(); h0tab[l].release();
      H[l][0].release(); H[l][1].release();
    }
    covered.release(); live.release(); gscr.release(); pend.release(); tr_action.release(); tr_rank.release();
    tr_stat.release(); glist.release(); gtoff.release(); ctl.release(); tpart.release(); lab_ok.release(); gscr_team.release(); pfx.release(); bspec.release(); prank.release(); q.release(); spart.release();
    apart.release(); ybuf.release(); hbuf.release(); xbuf.release(); nbc.release(); qslot.release(); qg.release(); tr_q.release(); node_w.release();
    sres.release(); qspec.release(); bars.release(); dfbuf.release();
    df_graph.clear();
    h_req.release(); h_ans.release(); h_nact.release(); h_act.release(); h_q.release(); h_chk.release();
    h_done.release(); h_gvar.release(); h_tr.release();
    ng = 0;
    hinfo.clear();
    hvar.clear();
  }
};

namespace {

md_status fail(md_ctx* c, md_status s, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) c->err = buf;
  return s;
}

#define HIPCHK(ctx, call)                                                                          \
  do {                                                                                             \
    hipError_t e_ = (call);                                                                        \
    if (e_ != hipSuccess) return fail(ctx, e_ == hipErrorOutOfMemory ? MD_EOOM : MD_EHIP, "%s: %s", \
                                      #call, hipGetErrorString(e_));                               \
  } while (0)

// Control block layout (ints): [0] barrier counter, [1] error word (zeroed before each launch).
constexpr int CTL_BAR = 0, CTL_ERR = 1, CTL_Q = 2, CTL_SPEC = 8, CTL_TEAM = 12, CTL_EXIT = 14, CTL_SELF = 32, CTL_PRE = 64,
              CTL_RING = 96, CTL_WORDS = 96 + 32 * 8;  // CTL_PRE and each ring's tickets on lines of their own
constexpr int SPEC_MAX = 32;  // speculative workgroups per launch at most (CTL_SPEC: the u64 request word)

Params make_params(md_ctx* c) {
  Params p{};
  p.fp_short = c->fp_short ? 1 : 0;
  p.fp_skip = c->fp_skip ? 1 : 0;
  p.pfx = c->pfx_min > 0 ? c->pfx.p : nullptr;
  p.pfx_min = c->pfx_min;
  p.first_req = c->first_req ? 1 : 0;
  p.w = c->w.p;
  p.ginfo = c->ginfo.p;
  p.gvar = c->gvar.p;
  for (int l = 0; l < 2; ++l) {
    p.rowptr[l] = c->rowptr[l].p;
    p.adj[l] = c->adj[l].p;
    p.adjx[l] = c->adjx[l].p;
    p.calive[l] = c->calive[l].p;
    p.epos[l] = c->epos[l].p;
    p.eu[l] = c->eu[l].p;
    p.ev[l] = c->ev[l].p;
    p.estate[l] = c->estate[l].p;
    p.deg[l] = c->deg[l].p;
    p.h0tab[l] = c->h0tab[l].p;
    p.H[l][0] = c->H[l][0].p;
    p.H[l][1] = c->H[l][1].p;
  }
  p.covered = c->covered.p;
  p.live = c->live.p;
  p.q = c->q.p;
  p.gscr = c->gscr.p;
  p.tpart = c->tpart.p;
  p.tctl = c->ctl.p + CTL_TEAM;
  p.lab_ok = c->lab_ok.p;
  p.gscr_team = c->gscr_team.p;
  p.bspec = c->bspec.p;
  p.bspec_half = c->bspec_half;
  p.prank = c->prank.p;
  p.spart = c->spart.p;
  p.apart = c->apart.p;
  p.ybuf = c->ybuf.p;
  p.hbuf = c->hbuf.p;
  p.xbuf = c->xbuf.p;
  p.nbc = c->nbc.p;
  p.nbc_slots = c->nbc_slots;
  p.pend = c->pend.p;
  p.tr_action = c->tr_action.p;
  p.tr_rank = c->tr_rank.p;
  p.h_tra = c->h_tr.d;
  p.h_trr = c->h_tr.d != nullptr ? c->h_tr.d + c->tot_n : nullptr;
  p.tr_stat = c->tr_stat.p;
  p.tr_q = c->tr_q.p;
  p.node_w = c->cost_mode == MD_COST_DEGREE ? c->node_w.p : nullptr;
  p.h0g = c->h0g.p;
  p.h0g_dm = c->h0g.p ? c->h0g_dm : 0;
  p.bar = (unsigned*)(c->ctl.p + CTL_BAR);
  p.bars = c->bars.p;
  p.err = c->ctl.p + CTL_ERR;
  p.qctl = (unsigned*)(c->ctl.p + CTL_Q);
  p.qslot = c->qslot.p;
  p.qring = (unsigned*)(c->ctl.p + CTL_RING);
  p.qg = c->qg.p;
  p.gtoff = c->gtoff.p;
  p.glist = c->glist.p;
  p.prof = c->prof_cap > 0 ? c->prof.p : nullptr;
  p.prof_cap = c->prof_cap;
  return p;
}

const char* err_name(int e) {
  switch (e) {
    case 1: return "team barrier timeout";
    case 2: return "action on an already covered node";
    case 3: return "live node sets differ between layers (U/PrepareBatchGraph.py:73)";
    case 4: return "action out of range";
    case 5: return "host selection failed";
    case 6: return "kernel argument layout differs from the compiled assumption";
    case 7: return "dataflow mode: a tile's alive-neighbour list exceeded NB_CAP";
    case 8: return "dataflow mode: phase A's state differs from its early step record";
    case 9: return "a speculative result's kill list is out of range";
    default: return e >= 1000 ? "bounds check failed (debug build; site = code - 1000)" : "unknown device error";
  }
}

md_status pull_vars(md_ctx* c) {
  HIPCHK(c, hipMemcpyAsync(c->hvar.data(), c->gvar.p, sizeof(GraphVar) * c->ng, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return MD_OK;
}
md_status push_vars(md_ctx* c) {
  HIPCHK(c, hipMemcpyAsync(c->gvar.p, c->hvar.data(), sizeof(GraphVar) * c->ng, hipMemcpyHostToDevice, c->stream));
  return MD_OK;
}

// Small batches whose environments fit LDS get dedicated environment workgroups.
constexpr int DEDICATED_MAX_GRAPHS = 16;

int env_workgroups(md_ctx* c, const std::vector<int>& gl) {
  if (c->env_mode == 0 || (int)gl.size() > DEDICATED_MAX_GRAPHS || (int)gl.size() * 4 > c->cus) return 0;
  for (int g : gl)
    if (!phase_a_fits_lds_host(c->hinfo[g].n, c->hinfo[g].e[0] + c->hinfo[g].e[1])) return 0;
  return (int)gl.size();
}

// Workgroups of one launch: enough for every graph's phase A and every 16-row tile, at most
// one per CU (the kernel is persistent and relies on co-residency for its grid barrier).
int grid_size(md_ctx* c, const std::vector<int>& gl, int n_env) {
  long tiles = 0;
  for (int g : gl) tiles += (c->hinfo[g].n + TILE - 1) / TILE;
  if (c->team_size_req > 0) tiles = c->team_size_req;
  // dedicated mode: two tile workgroups per tile when they fit (the kernel's layer split)
  const long want = n_env > 0 ? 2 * n_env + 2 * std::max<long>(1, tiles) : std::max<long>((long)gl.size(), tiles);
  return (int)std::max<long>(2 * n_env + 1, std::min<long>(want, c->cus));
}

// One launch of the persistent kernel over the graphs in gl (<= G_CAP of them).
// Host side of the in-kernel selection hand-shake: the callback and what it needs.
struct Selector {
  md_select_cb cb = nullptr;
  void* user = nullptr;
  int step = 1;
  std::string err;  // first failure, reported after the launch drained
};

// The reference's pick np.argsort(-q)[:n_out] on the masked float64 row: numpy's own float64
// argsort routine when the caller registered it (no Python on the hand-shake path), else the
// selection callback.  Returns 0 on success.
int select_actions(md_ctx* c, md_select_cb cb, void* user, int g, const std::vector<double>& qd, int n, int nout,
                   int32_t* acts) {
  if (c->tie_argsort) {
    thread_local std::vector<double> neg;
    thread_local std::vector<int64_t> idx;
    neg.resize(n);
    idx.resize(n);
    for (int i = 0; i < n; ++i) {
      neg[i] = -qd[i];
      idx[i] = i;
    }
    if (c->tie_argsort(neg.data(), idx.data(), n, nullptr) < 0) return 1;
    for (int i = 0; i < nout; ++i) acts[i] = (int32_t)idx[i];
    return 0;
  }
  if (!cb) return 1;
  return cb(user, g, qd.data(), n, nout, acts);
}

// K2 end-game request of graph g (md_kernels.hip, endgame_request): the row holds each live
// node's partner (int bits), -inf elsewhere.  Runs every remaining step's pick as the per-step
// protocol would: the masked double row with one common value at the live nodes,
// np.argsort(-q)[0] by numpy's own routine, then the pick and its partner leave the live set.
// Writes the picks to h_act and returns their count (-1 on a malformed request).
int serve_endgame(md_ctx* c, Selector* sel, int g, int nlive, std::vector<double>& qd) {
  const GraphInfo& gi = c->hinfo[g];
  const volatile float* hq = c->h_q.h + gi.node_off;
  thread_local std::vector<int> part;
  part.assign(gi.n, -1);
  qd.assign(gi.n, QMASK);
  int live = 0;
  for (int i = 0; i < gi.n; ++i) {
    const float x = hq[i];
    if (std::isinf(x)) continue;
    int pt;
    std::memcpy(&pt, &x, sizeof pt);
    part[i] = pt;
    qd[i] = -0.5;  // any common value above the mask: the picks depend only on the live set
    ++live;
  }
  bool ok = live == nlive && live % 2 == 0;
  for (int i = 0; ok && i < gi.n; ++i)
    if (part[i] >= 0) ok = part[i] < gi.n && part[i] != i && part[part[i]] == i;
  if (!ok) {
    if (sel->err.empty()) sel->err = "graph " + std::to_string(g) + ": malformed end-game request";
    return -1;
  }
  int k = 0;
  int32_t a = -1;
  while (live > 0) {
    if (select_actions(c, sel->cb, sel->user, g, qd, gi.n, 1, &a) != 0 || a < 0 || a >= gi.n || part[a] < 0) {
      if (sel->err.empty()) sel->err = "graph " + std::to_string(g) + ": end-game selection failed";
      return -1;
    }
    c->h_act.h[gi.node_off + k++] = a;
    qd[a] = QMASK;
    qd[part[a]] = QMASK;
    part[part[a]] = -1;
    part[a] = -1;
    live -= 2;
  }
  return k;
}

// Answers graph g's request `tag`: Q row (float, -inf = masked) -> the reference's masked
// double row, the callback's actions into mapped memory, then the answer tag.
void serve_request(md_ctx* c, Selector* sel, int g, unsigned tag, std::vector<double>& qd, std::vector<int32_t>& acts) {
  const GraphInfo& gi = c->hinfo[g];
  int k = -1;
  if (!sel->cb && !c->tie_argsort) {
    if (sel->err.empty()) {
      char b[160];
      snprintf(b, sizeof b, "graph %d: nodes tie at the max Q and no selection callback was given", g);
      sel->err = b;
    }
  } else {
    qd.resize(gi.n);
    const volatile float* hq = c->h_q.h + gi.node_off;
    // the row must carry the device's own max and tie count (a stale or torn row would
    // silently change the selection)
    float mx = -INFINITY;
    int nt = 0;
    for (int i = 0; i < gi.n; ++i) {
      const float x = hq[i];
      qd[i] = std::isinf(x) ? QMASK : (double)x;
      if (x > mx) {
        mx = x;
        nt = 1;
      } else if (x == mx) {
        ++nt;
      }
    }
    const float cmax = c->h_chk.h[2 * g];
    int cnt;
    std::memcpy(&cnt, c->h_chk.h + 2 * g + 1, sizeof cnt);
    if (cnt < 0) {
      k = serve_endgame(c, sel, g, -cnt, qd);
      c->h_nact.h[g] = k;
      __atomic_store_n(c->h_ans.h + g, tag, __ATOMIC_RELEASE);
      return;
    }
    if (mx != cmax || nt != cnt) {
      if (sel->err.empty()) {
        char b[200];
        snprintf(b, sizeof b, "graph %d: host Q row (max %.9g, %d at max) disagrees with the device (%.9g, %d)", g,
                 (double)mx, nt, (double)cmax, cnt);
        sel->err = b;
      }
      c->h_nact.h[g] = -1;
      __atomic_store_n(c->h_ans.h + g, tag, __ATOMIC_RELEASE);
      return;
    }
    const int nout = std::min(sel->step, gi.n);
    acts.assign(nout, -1);
    if (select_actions(c, sel->cb, sel->user, g, qd, gi.n, nout, acts.data()) != 0) {
      if (sel->err.empty()) sel->err = "selection callback failed (graph " + std::to_string(g) + ")";
    } else {
      k = 0;
      for (int i = 0; i < nout; ++i) {
        if (acts[i] < 0 || acts[i] >= gi.n) {
          if (sel->err.empty()) sel->err = "callback returned node " + std::to_string(acts[i]) + " out of range";
          k = -1;
          break;
        }
        c->h_act.h[gi.node_off + k++] = acts[i];
      }
    }
  }
  c->h_nact.h[g] = k;
  __atomic_store_n(c->h_ans.h + g, tag, __ATOMIC_RELEASE);
}

// Whole-batch rollouts run through the device work queue (MD_VARIANT bit 32: the lock-step
// shared mode instead) when every loaded graph fits the work items' tile field.
bool queue_mode_ok(const md_ctx* c, int run_mode) {
  return run_mode == RUN_ROLLOUT && !(c->variant & 32) && c->max_tiles < Q_MAX_TILES;
}

md_status launch_chunk(md_ctx* c, const int* gl_in, int ngl, int run_mode, int host_select, Selector* sel) {
  const auto t_fn = std::chrono::steady_clock::now();
  std::vector<int> v(gl_in, gl_in + ngl);
  // graphs with more edges first: the queue's first round-robin positions go to the longest
  // rollouts (the rollout length grows with the edge count), so the launch does not end on a
  // few long graphs running alone; the graph-slot order has no other meaning
  std::stable_sort(v.begin(), v.end(), [&](int a, int b) {
    return (long)c->hinfo[a].e[0] + c->hinfo[a].e[1] > (long)c->hinfo[b].e[0] + c->hinfo[b].e[1];
  });
  const int* gl = v.data();
  const int n_env = env_workgroups(c, v);
  // batches of whole rollouts run through the device work queue (MD_VARIANT bit 32: the
  // lock-step shared mode instead), one workgroup per CU
  // (one graph too large for LDS: the lock-step kernel, whose environment step runs on every
  // workgroup of the launch -- team_env_step -- unless MD_VARIANT bit 2 turns that off)
  const bool team_env = ngl == 1 && !(c->variant & 2) &&
                        (!phase_a_fits_lds_host(c->hinfo[gl[0]].n, c->hinfo[gl[0]].e[0] + c->hinfo[gl[0]].e[1]) ||
                         (c->variant & 64));
  const bool qmode = queue_mode_ok(c, run_mode) && n_env == 0 && !team_env;
  if (team_env && c->team_owner != gl[0]) {
    // gscr_team is shared by the loaded graphs: class labels another graph's grid-wide step
    // left there are not this graph's
    HIPCHK(c, hipMemsetAsync(c->lab_ok.p + gl[0], 0, sizeof(int), c->stream));
    c->team_owner = gl[0];
  }
  const int grid = qmode ? c->cus : grid_size(c, v, n_env);
  // speculative environment workgroups on the CUs a single-graph rollout leaves free
  // (single-node steps only: step > 1 takes several removals per prediction)
  const int n_spec = run_mode == RUN_ROLLOUT && n_env == 1 && ngl == 1 && !host_select && c->sres.p != nullptr &&
                             spec_fits_lds_host(c->hinfo[gl[0]].n, c->hinfo[gl[0]].e[0] + c->hinfo[gl[0]].e[1]) &&
                             // word-aligned state arrays (the speculative staging reads 4 states per load)
                             c->hinfo[gl[0]].eoff[0] % 4 == 0 && c->hinfo[gl[0]].eoff[1] % 4 == 0 &&
                             c->hinfo[gl[0]].node_off % 4 == 0
                         ? std::max(0, std::min(c->spec_n, c->cus - grid))
                         : 0;
  // dataflow mode: a single-graph rollout in dedicated mode with the layer split, no grid
  // barrier (md_kernels.hip df_*; the graph qualified at load, MD_DF=0 keeps the barriers)
  const bool df = run_mode == RUN_ROLLOUT && n_env == 1 && ngl == 1 && !team_env && c->dfbuf.p != nullptr &&
                  c->df_graph[gl[0]] && 2 * ((c->hinfo[gl[0]].n + TILE - 1) / TILE) <= grid - 2;
  HIPCHK(c, hipMemcpyAsync(c->glist.p, gl, sizeof(int) * ngl, hipMemcpyHostToDevice, c->stream));
  // (the host side of an async upload must outlive the copy: `to`, like `v`, lives until the
  // launch below has been waited for)
  std::vector<int> to;
  if (qmode) {
    // queue-mode neighbour-list cache slots: each graph slot's tiles from its launch prefix
    to.assign(ngl + 1, 0);
    for (int i = 0; i < ngl; ++i) to[i + 1] = to[i] + (c->hinfo[gl[i]].n + TILE - 1) / TILE;
    HIPCHK(c, hipMemcpyAsync(c->gtoff.p, to.data(), sizeof(int) * (ngl + 1), hipMemcpyHostToDevice, c->stream));
  }
  {
    // per-launch clears in one dispatch: control words, barrier shards; graph-head hand-off
    // granules carry the step as their tag (stale tags from earlier launches must not match);
    // the split hand-off slots a launch of this grid can use (split tiles <= tile workgroups / 2);
    // the work queue
    void* ptr[6] = {c->ctl.p, c->bars.p, nullptr, nullptr, nullptr, nullptr};
    size_t bytes[6] = {sizeof(int) * CTL_WORDS, sizeof(unsigned) * c->bars.n, 0, 0, 0, 0};
    if (n_env > 0) {
      ptr[2] = c->hbuf.p;
      bytes[2] = sizeof(float) * c->hbuf.n;
      ptr[3] = c->xbuf.p;
      bytes[3] = sizeof(unsigned long long) * 2048 * std::min(XB_SLOTS, grid / 2 + 1);
    }
    if (qmode) {
      // (wave items: the head granules carry the forward pass's prediction count as their tag)
      ptr[2] = c->hbuf.p;
      bytes[2] = sizeof(float) * c->hbuf.n;
      ptr[4] = c->qslot.p;
      bytes[4] = sizeof(unsigned long long) * c->qslot.n;
      ptr[5] = c->qg.p;
      bytes[5] = sizeof(int) * c->qg.n;
    }
    if (df) {  // the tagged granules (no tag of an earlier launch may match)
      ptr[4] = c->dfbuf.p;
      bytes[4] = sizeof(unsigned long long) * c->dfbuf.n;
    }
    HIPCHK(c, launch_clear(ptr, bytes, 6, c->stream));
  }
  Params p = make_params(c);
  p.n_main = grid;
  p.n_spec = n_spec;
  if (n_spec > 0) {
    p.spec_req = (unsigned long long*)(c->ctl.p + CTL_SPEC);
    p.sres = c->sres.p;
    p.sres_stride = c->sres_stride;
    p.qspec = c->qspec.p;
    p.qspec_n = (int)c->tot_n;
    if (!(c->variant & 1)) {  // MD_VARIANT bit 1: no iteration-1 prebuild
      p.pre_ew = (unsigned long long*)(c->ctl.p + CTL_PRE);
      p.pre_cw = (unsigned long long*)(c->ctl.p + CTL_PRE + 2);
      p.spec_early = c->early_on ? 1 : 0;
      p.spec_abort = c->abort_on ? 1 : 0;
    }
  }
  if (df) {
    p.df = c->dfbuf.p;
    p.df_mt = c->df_mt;
    p.df_n = c->df_n;
    // tile 0 hands its derivation of phase A's early word to the speculative workgroups
    if (p.pre_ew != nullptr) p.self_ew = (unsigned long long*)(c->ctl.p + CTL_SELF);
  }
  // wave items for launches with enough graphs to fill the chip's waves; the last wqpark running
  // graphs of such a launch leave it (parked) and continue in the per-workgroup queue kernel, which
  // in turn hands its last qpark to the lock-step kernel
  const bool wq = qmode && c->wq_on && ngl > c->wqpark;
  p.qmode = qmode ? (wq ? 2 : 1) : 0;
  p.qpair = c->pair_on ? 1 : 0;
  p.qpark = p.qmode == 2 ? c->wqpark : c->qpark;
  if (!qmode) p.bspec = nullptr;  // (speculative environment items run in the queue kernels only)
  p.nglist = ngl;
  p.n_env = n_env;
  p.variant = c->variant;
  p.launch_seq = ++c->launch_seq;
  if ((c->launch_seq & 0xffffu) == 0) {
    // speculative-result tags carry the low 16 bits of launch_seq (spec_tag): every 65536
    // launches the slots are wiped and the all-zero tag value is skipped, so no slot can hold
    // a tag of an earlier launch that matches this one's
    p.launch_seq = ++c->launch_seq;
    if (c->sres.p) HIPCHK(c, hipMemsetAsync(c->sres.p, 0, sizeof(int) * c->sres.n, c->stream));
    // the batch-speculation slots carry the same 16-bit launch tag
    if (c->bspec.p) HIPCHK(c, hipMemsetAsync(c->bspec.p, 0, sizeof(int) * (size_t)(2 * c->bspec_half), c->stream));
  }
  p.run_mode = run_mode;
  p.host_select = host_select;
  // the k largest Q of a grid-wide step's prediction on the device when tie-free (numpy's own
  // routine is the selection rule: a Python selector keeps every request; MD_DEVTOPK=0: off)
  p.sel_step = sel != nullptr ? sel->step : 1;
  p.dev_topk = host_select && sel != nullptr && c->tie_argsort != nullptr && c->dev_topk ? 1 : 0;
  const bool hs = sel != nullptr && c->host_mode != 0 && c->h_req.d != nullptr;
  if (hs) {
    for (int g : v) {
      __atomic_store_n(c->h_req.h + g, 0u, __ATOMIC_RELAXED);
      __atomic_store_n(c->h_ans.h + g, 0u, __ATOMIC_RELAXED);
    }
    p.h_req = c->h_req.d;
    p.h_ans = c->h_ans.d;
    p.h_nact = c->h_nact.d;
    p.h_act = c->h_act.d;
    p.h_q = c->h_q.d;
    p.h_chk = c->h_chk.d;
    // K2 end-games in one hand-shake: single-node steps picked by numpy's own argsort routine
    // (the callback path keeps one request per step); MD_VARIANT bit 2048 turns it off
    // (bit 2: the answer applied in one pass, env_endgame_apply; MD_EG_APPLY=0: action by action)
    p.endgame = run_mode == RUN_ROLLOUT && c->tie_argsort != nullptr && sel->step == 1 &&
                c->cost_mode == MD_COST_UNIT && !(c->variant & 2048)
                    ? 1 | (c->eg_apply ? 2 : 0)
                    : 0;
  }
  // completion record: the last workgroup copies the GraphVars and the error word to mapped
  // host memory and then writes the launch tag (kernel_exit)
  const bool rec = c->h_done.h != nullptr && c->h_gvar.h != nullptr;
  if (rec) {
    __atomic_store_n(c->h_done.h, 0u, __ATOMIC_RELAXED);
    p.exit_ctr = (unsigned*)(c->ctl.p + CTL_EXIT);
    p.h_done = c->h_done.d;
    p.h_gvar = c->h_gvar.d;
  }
  if (trace_on())
    std::fprintf(stderr, "md trace: ctx %p launch %u run %d grid %d spec %d env %d df %d qmode %d graphs %d\n", (void*)c,
                 p.launch_seq, run_mode, grid, n_spec, n_env, df ? 1 : 0, qmode ? 1 : 0, ngl);
  HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  HIPCHK(c, launch_rollout(p, c->wimg.p, grid + n_spec, c->stream));
  HIPCHK(c, hipEventRecord(c->ev1, c->stream));
  // Wait for the launch while serving selection requests (hs): the completion tag is read on
  // every pass (host memory, no runtime call); the launch's completion event only every 20 us
  // (a launch that ended without its record: a fault, or an early exit) and, once the tag is
  // there, until the kernel has retired.
  bool tagged = false;
  {
    std::vector<double> qd;
    std::vector<int32_t> acts;
    auto last = std::chrono::steady_clock::now();
    const auto t_launch = last;
    auto t_tag = last;
    static const bool host_stats = std::getenv("MD_HOST_STATS") != nullptr;  // diagnostics
    double serve_s = 0.0;
    int n_served = 0;
    bool done = false;
    while (true) {
      bool served = false;
      if (hs) {
        for (int g : v) {
          const unsigned r = __atomic_load_n(c->h_req.h + g, __ATOMIC_ACQUIRE);
          if (r != 0 && r != __atomic_load_n(c->h_ans.h + g, __ATOMIC_RELAXED)) {
            const auto ts = std::chrono::steady_clock::now();
            serve_request(c, sel, g, r, qd, acts);
            c->last_served += 1;
            if (host_stats) {
              serve_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - ts).count();
              ++n_served;
            }
            served = true;
          }
        }
      }
      if (done) break;
      if (rec && !tagged && __atomic_load_n(c->h_done.h, __ATOMIC_ACQUIRE) == p.launch_seq) {
        tagged = true;
        if (host_stats) t_tag = std::chrono::steady_clock::now();
      }
      const auto now = std::chrono::steady_clock::now();
      if (tagged || (!served && now - last >= std::chrono::microseconds(20))) {
        last = now;
        const hipError_t q = hipEventQuery(c->ev1);
        if (q != hipSuccess && q != hipErrorNotReady) HIPCHK(c, q);
        done = q == hipSuccess;
      }
      if (!hs && !done && !tagged) {
        if (!rec) {
          HIPCHK(c, hipEventSynchronize(c->ev1));
          done = true;
        }
      } else if (c->poll_us > 0 && !tagged) {
        std::this_thread::sleep_for(std::chrono::microseconds(c->poll_us));
      }
    }
    if (hs && host_stats)
      std::fprintf(stderr, "md host: prelude %.3f ms; %d requests served in %.3f ms of a %.3f ms launch wait (tag seen at %.3f ms)\n",
                   1e3 * std::chrono::duration<double>(t_launch - t_fn).count(), n_served, 1e3 * serve_s,
                   1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t_launch).count(),
                   1e3 * std::chrono::duration<double>(t_tag - t_launch).count());
  }
  if (trace_on()) std::fprintf(stderr, "md trace: ctx %p launch %u done\n", (void*)c, p.launch_seq);
  int dev_err = 0;
  if (rec && __atomic_load_n(c->h_done.h, __ATOMIC_ACQUIRE) == p.launch_seq) {
    dev_err = (int)__atomic_load_n(c->h_done.h + 1, __ATOMIC_RELAXED);
    constexpr int GVW = (int)(sizeof(GraphVar) / sizeof(int));
    for (int g : v) std::memcpy(&c->hvar[g], c->h_gvar.h + (size_t)g * GVW, sizeof(GraphVar));
  } else {
    c->vars_stale = true;  // launch() pulls every GraphVar
    HIPCHK(c, hipMemcpyAsync(&dev_err, c->ctl.p + CTL_ERR, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  float ms = 0.f;
  HIPCHK(c, hipEventElapsedTime(&ms, c->ev0, c->ev1));
  c->last_ms += ms;
  c->last_launches += 1;
  if (dev_err == 5 && sel != nullptr && !sel->err.empty()) return fail(c, MD_ECALLBACK, "%s", sel->err.c_str());
  if (dev_err) return fail(c, dev_err == 1 ? MD_ETIMEOUT : MD_EINVAL, "device: %s (code %d)", err_name(dev_err), dev_err);
  if (c->prof_cap > 0) {
    std::vector<unsigned long long> tmp((size_t)c->prof_cap * PROF_SLOTS);
    HIPCHK(c, hipMemcpy(tmp.data(), c->prof.p, sizeof(unsigned long long) * tmp.size(), hipMemcpyDeviceToHost));
    // the step records up to the first empty one (MD_PROF_ALL=1: every row up to the last
    // non-empty one -- the dataflow mode's per-tile rows 128.. follow the step records)
    const bool all = std::getenv("MD_PROF_ALL") != nullptr && std::atoi(std::getenv("MD_PROF_ALL")) != 0;
    int rows = 0;
    for (int s = 0; s < c->prof_cap; ++s) {
      bool any = tmp[(size_t)s * PROF_SLOTS] != 0;
      for (int k = 1; all && !any && k < PROF_SLOTS; ++k) any = tmp[(size_t)s * PROF_SLOTS + k] != 0;
      if (any) rows = s + 1;
      else if (!all) break;
    }
    c->prof_host.insert(c->prof_host.end(), tmp.begin(), tmp.begin() + (size_t)rows * PROF_SLOTS);
    HIPCHK(c, hipMemset(c->prof.p, 0, sizeof(unsigned long long) * tmp.size()));
  }
  return MD_OK;
}

md_status launch(md_ctx* c, const std::vector<int>& gl, int run_mode, int host_select, Selector* sel = nullptr) {
  c->vars_stale = false;
  // a queue-mode batch runs in one launch of up to QG_CAP graphs (one launch tail instead of
  // one per G_CAP chunk); lock-step launches take G_CAP
  const size_t cap = queue_mode_ok(c, run_mode) && gl.size() > (size_t)DEDICATED_MAX_GRAPHS ? QG_CAP : G_CAP;
  for (size_t i = 0; i < gl.size(); i += cap) {
    const int k = (int)std::min<size_t>(cap, gl.size() - i);
    md_status st = launch_chunk(c, gl.data() + i, k, run_mode, host_select, sel);
    if (st != MD_OK) {
      (void)pull_vars(c);
      return st;
    }
  }
  // the launches' completion records carried their GraphVars; otherwise copy them all back
  return c->vars_stale ? pull_vars(c) : MD_OK;
}

void host_first_layer(const float* w, const float* nw, float* out) {
  // degree cost: X = [w_l(i), 1.0] (D/PrepareBatchGraph.py:133-136); normalize(relu(X . w_n2l))
  float x[64];
  for (int c = 0; c < 64; ++c) {
    float a = std::fma(nw[0], w[W_N2L + c], 0.f);
    a = std::fma(1.0f, w[W_N2L + 64 + c], a);
    x[c] = a > 0.f ? a : 0.f;
  }
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int c = 0; c < 64; ++c) acc[c & 7] = std::fma(x[c], x[c], acc[c & 7]);
  float s = acc[0];
  for (int j = 1; j < 8; ++j) s = s + acc[j];
  const float den = std::max(std::sqrt(s), 1e-12f);
  for (int c = 0; c < 64; ++c) out[c] = x[c] / den;
}

}  // namespace

extern "C" {

const char* md_version(void) { return "libmdroll 0.1 (gfx950, HIP " HIP_VERSION_BUILD_NAME ")"; }

int md_device_count(void) {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

const char* md_last_error(const md_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

md_status md_create(int device, const float* weights, size_t n_floats, int cost_mode, md_ctx** out) {
  if (!out || !weights) return MD_EINVAL;
  *out = nullptr;
  if (n_floats != MD_WEIGHT_FLOATS) return MD_EINVAL;
  if (cost_mode != MD_COST_UNIT && cost_mode != MD_COST_DEGREE) return MD_EINVAL;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MD_EHIP;
  if (device < 0 || device >= ndev) return MD_EINVAL;
  md_ctx* c = new md_ctx();
  c->device = device;
  c->cost_mode = cost_mode;
  if (const char* v = std::getenv("MD_VARIANT")) c->variant = std::atoi(v);
  if (const char* v = std::getenv("MD_ENV_MODE")) c->env_mode = std::atoi(v);
  if (const char* v = std::getenv("MD_PAIR")) c->pair_on = std::atoi(v) != 0;
  if (const char* v = std::getenv("MD_WQ")) c->wq_on = std::atoi(v) != 0;
  if (const char* v = std::getenv("MD_BSPEC")) c->bspec_on = std::atoi(v) != 0;
  if (const char* v = std::getenv("MD_WQPARK")) c->wqpark = std::max(0, std::min(4096, std::atoi(v)));
  if (const char* v = std::getenv("MD_QPARK")) c->qpark = std::max(0, std::min(16, std::atoi(v)));
  if (const char* v = std::getenv("MD_HOST_HANDSHAKE")) c->host_mode = std::atoi(v);
  if (const char* v = std::getenv("MD_POLL_US")) c->poll_us = std::atoi(v);
  if (const char* v = std::getenv("MD_H0G")) c->h0g_on = std::atoi(v) != 0;
  if (const char* v = std::getenv("MD_EARLY")) c->early_on = std::atoi(v) != 0;
  if (const char* v = std::getenv("MD_SPEC_ABORT")) c->abort_on = std::atoi(v) != 0;
  if (const char* v = std::getenv("MD_FP_SHORTCUT")) c->fp_short = std::atoi(v) != 0;
  if (const char* v = std::getenv("MD_FP_SKIP")) c->fp_skip = std::atoi(v) != 0;
  if (const char* v = std::getenv("MD_PREFIX")) c->pfx_min = std::max(0, std::atoi(v));
  if (const char* v = std::getenv("MD_DEVTOPK")) c->dev_topk = std::atoi(v) != 0;
  if (const char* v = std::getenv("MD_EG_APPLY")) c->eg_apply = std::atoi(v) != 0;
  if (const char* v = std::getenv("MD_FIRST_REQ")) c->first_req = std::atoi(v) != 0;
  if (const char* v = std::getenv("MD_DF")) c->df_on = std::atoi(v) != 0;
  if (const char* v = std::getenv("MD_SPEC")) c->spec_n = std::max(0, std::min(SPEC_MAX, std::atoi(v)));
  md_status st = MD_OK;
  do {
    if (hipSetDevice(device) != hipSuccess) { st = MD_EHIP; break; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) { st = MD_EHIP; break; }
    c->cus = prop.multiProcessorCount;
    // MD_MAX_CUS: use at most this many CUs (one workgroup per CU), e.g. several ranks sharing
    // one GPU, whose persistent grids must all be resident at once
    if (const char* v = std::getenv("MD_MAX_CUS")) c->cus = std::max(8, std::min(c->cus, std::atoi(v)));
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) { st = MD_EHIP; break; }
    if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) { st = MD_EHIP; break; }
    if (set_kernel_attrs() != hipSuccess) { st = MD_EHIP; break; }
    st = md_set_weights(c, weights, n_floats);
  } while (0);
  if (st != MD_OK) {
    delete c;
    return st;
  }
  *out = c;
  if (trace_on())
    std::fprintf(stderr, "md trace: create ctx %p df %d variant %d spec %d\n", (void*)c, c->df_on ? 1 : 0, c->variant,
                 c->spec_n);
  return MD_OK;
}

void md_destroy(md_ctx* ctx) {
  if (trace_on()) std::fprintf(stderr, "md trace: destroy ctx %p\n", (void*)ctx);
  delete ctx;
}

// Unit cost: the first-layer tables of every dmax up to the largest loaded graph's n - 1
// (tables of dmax <= H0G_MAX_DM only: 2048 dmax values are 537 MB; larger dmax values are
// rebuilt in phase A).  Recomputed from scratch when the weights change.
constexpr int H0G_MAX_DM = 2048;
md_status ensure_h0g(md_ctx* c, int need, bool weights_changed) {
  if (c->cost_mode != MD_COST_UNIT || !c->h0g_on) return MD_OK;
  need = std::min(need, H0G_MAX_DM);
  if (weights_changed && c->h0g.p) c->h0g_dm = 0;
  if (need <= c->h0g_dm) return MD_OK;
  const size_t rows = (size_t)h0g_row(need + 1, 1);
  if (!c->h0g.p || c->h0g.n < rows * EMB) {
    c->h0g.release();
    HIPCHK(c, c->h0g.alloc(rows * EMB));
    c->h0g_dm = 0;
  }
  HIPCHK(c, launch_h0(c->w.p, c->h0g.p, c->h0g_dm + 1, need, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->h0g_dm = need;
  return MD_OK;
}

md_status md_set_weights(md_ctx* c, const float* weights, size_t n_floats) {
  if (!c || !weights || n_floats != MD_WEIGHT_FLOATS) return fail(c, MD_EINVAL, "weights: expected %d floats", MD_WEIGHT_FLOATS);
  HIPCHK(c, hipSetDevice(c->device));
  if (!c->w.p) HIPCHK(c, c->w.alloc(W_TOTAL + 3));
  const int ni = weight_image_floats();
  if (!c->wimg.p) HIPCHK(c, c->wimg.alloc(ni));
  std::vector<float> img(ni);
  build_weight_image(weights, img.data());
  HIPCHK(c, hipMemcpyAsync(c->w.p, weights, sizeof(float) * W_TOTAL, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->wimg.p, img.data(), sizeof(float) * ni, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // degree cost: the static first-layer input depends on the weights
  if (c->ng > 0 && c->cost_mode == MD_COST_DEGREE) {
    std::vector<float> nw(2 * c->tot_n);
    HIPCHK(c, hipMemcpy(nw.data(), c->node_w.p, sizeof(float) * nw.size(), hipMemcpyDeviceToHost));
    for (int l = 0; l < 2; ++l) {
      std::vector<float> tab(c->tot_n * EMB);
      for (size_t v = 0; v < c->tot_n; ++v) host_first_layer(weights, &nw[l * c->tot_n + v], &tab[v * EMB]);
      HIPCHK(c, hipMemcpy(c->h0tab[l].p, tab.data(), sizeof(float) * tab.size(), hipMemcpyHostToDevice));
    }
  } else if (c->ng > 0) {
    // unit cost: the per-graph degree tables were built from the old weights
    int maxn = 0;
    for (const auto& gi : c->hinfo) maxn = std::max(maxn, gi.n);
    md_status st = ensure_h0g(c, maxn - 1, true);
    if (st != MD_OK) return st;
    for (auto& v : c->hvar) v.hdmax[0] = v.hdmax[1] = 0;
    return push_vars(c);
  } else if (c->h0g.p) {
    c->h0g_dm = 0;
  }
  return MD_OK;
}

md_status md_set_tie_argsort(md_ctx* c, md_argsort_f64 fn) {
  if (!c) return MD_EINVAL;
  c->tie_argsort = fn;
  return MD_OK;
}

md_status md_set_team_size(md_ctx* c, int team_size) {
  if (!c || team_size < 0) return MD_EINVAL;
  c->team_size_req = team_size;
  return MD_OK;
}

md_status md_load_graphs(md_ctx* c, int n_graphs, const int32_t* n_nodes, const int64_t* edge_off0,
                         const int32_t* edges0, const int64_t* edge_off1, const int32_t* edges1,
                         const float* node_w) {
  if (!c) return MD_EINVAL;
  if (n_graphs <= 0 || !n_nodes || !edge_off0 || !edge_off1) return fail(c, MD_EINVAL, "bad graph batch");
  if (c->cost_mode == MD_COST_DEGREE && !node_w) return fail(c, MD_EINVAL, "degree cost needs node_w");
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->free_graphs();
  const int64_t* eo[2] = {edge_off0, edge_off1};
  const int32_t* ed[2] = {edges0, edges1};
  std::vector<GraphInfo> info(n_graphs);
  size_t tn = 0, te[2] = {0, 0}, tt = 0;
  bool big = false;
  for (int g = 0; g < n_graphs; ++g) {
    const int n = n_nodes[g];
    if (n <= 0) return fail(c, MD_EINVAL, "graph %d: n_nodes must be > 0", g);
    GraphInfo& gi = info[g];
    gi.n = n;
    gi.node_off = (int)tn;
    gi.tile_off = (int)tt;
    gi.gidx = g;
    for (int l = 0; l < 2; ++l) {
      const int64_t ne = eo[l][g + 1] - eo[l][g];
      if (ne < 0) return fail(c, MD_EINVAL, "graph %d layer %d: negative edge count", g, l);
      gi.e[l] = (int)ne;
      gi.eoff[l] = (int)te[l];
      gi.roff[l] = (int)(tn + g);
      gi.coff[l] = (int)(2 * te[l]);
      te[l] += ne;
    }
    tn += n;
    tt += (n + TILE - 1) / TILE;
    if (!phase_a_fits_lds_host(n, gi.e[0] + gi.e[1])) big = true;
  }
  if (tn > (size_t)INT32_MAX / EMB || te[0] > (size_t)INT32_MAX / 4 || te[1] > (size_t)INT32_MAX / 4)
    return fail(c, MD_EINVAL, "batch too large");
  // static CSR in reference order: row i lists i's neighbours in the order the edges appear
  // in G.edges() (the in_edges order of U/PrepareBatchGraph.py:151-160, U/graph_struct.py:63)
  std::vector<int> rowptr[2], adj[2], adjx[2], epos[2], eu[2], ev[2];
  for (int l = 0; l < 2; ++l) {
    rowptr[l].assign(tn + n_graphs, 0);
    adj[l].resize(2 * te[l]);
    adjx[l].resize(2 * te[l]);
    epos[l].resize(2 * te[l]);
    eu[l].resize(te[l]);
    ev[l].resize(te[l]);
    for (int g = 0; g < n_graphs; ++g) {
      const GraphInfo& gi = info[g];
      const int n = gi.n;
      int* rp = rowptr[l].data() + gi.roff[l];
      std::unordered_set<uint64_t> seen;
      seen.reserve(gi.e[l] * 2 + 1);
      for (int k = 0; k < gi.e[l]; ++k) {
        const int u = ed[l][2 * (eo[l][g] + k)], v = ed[l][2 * (eo[l][g] + k) + 1];
        if (u < 0 || v < 0 || u >= n || v >= n) return fail(c, MD_EINVAL, "graph %d layer %d edge %d: node out of range", g, l, k);
        if (u == v) return fail(c, MD_EINVAL, "graph %d layer %d edge %d: self-loop", g, l, k);
        const uint64_t key = ((uint64_t)std::min(u, v) << 32) | (uint32_t)std::max(u, v);
        if (!seen.insert(key).second) return fail(c, MD_EINVAL, "graph %d layer %d: duplicate edge %d-%d", g, l, u, v);
        eu[l][gi.eoff[l] + k] = u;
        ev[l][gi.eoff[l] + k] = v;
        rp[u + 1]++;
        rp[v + 1]++;
      }
      for (int i = 0; i < n; ++i) rp[i + 1] += rp[i];
      std::vector<int> fill(rp, rp + n);
      int* a = adj[l].data() + gi.coff[l];
      int* ax = adjx[l].data() + gi.coff[l];
      int* ep = epos[l].data() + 2 * (size_t)gi.eoff[l];
      // packed words are read only for layer-local edge ids < 2^15 (env_build_lists tests x >= 0
      // for liveness, and k = 65535, u = 65535 would pack to the -1 'not packed' marker)
      const bool packs = gi.e[l] < ADJX_EDGE_LIMIT && n <= 65536;
      for (int k = 0; k < gi.e[l]; ++k) {
        const int u = eu[l][gi.eoff[l] + k], v = ev[l][gi.eoff[l] + k];
        ep[2 * k] = fill[v];
        ax[fill[v]] = packs ? (k << 16) | u : -1;
        a[fill[v]++] = u;  // in_edges[v] gets u (U/PrepareBatchGraph.py:157)
        ep[2 * k + 1] = fill[u];
        ax[fill[u]] = packs ? (k << 16) | v : -1;
        a[fill[u]++] = v;  // in_edges[u] gets v (:159)
      }
    }
  }
  // static union ranks of the grid-wide environment step (md_env.h uf_unite_r2): per graph the
  // nodes ordered by descending static degree (both layers), ties by the hashed priority
  // (uf_pri), rank = position; every graph's block starts at an even index
  std::vector<uint16_t> ranks;
  {
    // (only graphs the grid-wide step can run: too large for LDS, or any graph of a small batch,
    // where MD_VARIANT=64 forces that step; rank_off = -1 otherwise)
    size_t off = 0;
    for (int g = 0; g < n_graphs; ++g) {
      const bool want = info[g].n <= 65535 &&
                        (n_graphs <= DEDICATED_MAX_GRAPHS || !phase_a_fits_lds_host(info[g].n, info[g].e[0] + info[g].e[1]));
      info[g].rank_off = want ? (int)off : -1;
      if (want) off += (size_t)((info[g].n + 1) & ~1);
    }
    ranks.assign(std::max<size_t>(2, off), 0);
    std::vector<int> ord;
    for (int g = 0; g < n_graphs; ++g) {
      const GraphInfo& gi = info[g];
      if (gi.rank_off < 0) continue;
      const int* r0 = rowptr[0].data() + gi.roff[0];
      const int* r1 = rowptr[1].data() + gi.roff[1];
      ord.resize(gi.n);
      for (int x = 0; x < gi.n; ++x) ord[x] = x;
      auto deg = [&](int x) { return (r0[x + 1] - r0[x]) + (r1[x + 1] - r1[x]); };
      std::sort(ord.begin(), ord.end(), [&](int a, int b) {
        const int da = deg(a), db = deg(b);
        if (da != db) return da > db;
        return (unsigned)a * 2654435761u < (unsigned)b * 2654435761u;
      });
      for (int k = 0; k < gi.n; ++k) ranks[gi.rank_off + ord[k]] = (uint16_t)k;
    }
  }
  c->ng = n_graphs;
  c->hinfo = info;
  c->hvar.assign(n_graphs, GraphVar{});
  c->s0_pending = false;  // a deferred prune belonged to the graphs this load replaces
  c->tot_n = tn;
  c->tot_tiles = tt;
  c->need_gscr = big;
  HIPCHK(c, c->ginfo.alloc(n_graphs));
  HIPCHK(c, c->gvar.alloc(n_graphs));
  for (int l = 0; l < 2; ++l) {
    c->tot_e[l] = te[l];
    HIPCHK(c, c->rowptr[l].alloc(rowptr[l].size() + 4));  // + 4: env_stage_wide's 16-byte chunks
    HIPCHK(c, c->adj[l].alloc(std::max<size_t>(1, adj[l].size())));
    HIPCHK(c, c->adjx[l].alloc(std::max<size_t>(1, adjx[l].size())));
    HIPCHK(c, c->epos[l].alloc(std::max<size_t>(1, epos[l].size())));
    HIPCHK(c, c->calive[l].alloc(std::max<size_t>(1, 2 * te[l])));
    HIPCHK(c, c->eu[l].alloc(eu[l].size() + 4));
    HIPCHK(c, c->ev[l].alloc(ev[l].size() + 4));
    HIPCHK(c, c->estate[l].alloc(te[l] + 16));  // + 16: whole-chunk reads of the last states
    HIPCHK(c, c->deg[l].alloc(tn));
    HIPCHK(c, c->h0tab[l].alloc(tn * EMB));
    HIPCHK(c, c->H[l][0].alloc(tn * EMB));
    HIPCHK(c, c->H[l][1].alloc(tn * EMB));
    HIPCHK(c, hipMemcpyAsync(c->rowptr[l].p, rowptr[l].data(), sizeof(int) * rowptr[l].size(), hipMemcpyHostToDevice, c->stream));
    if (te[l]) {
      HIPCHK(c, hipMemcpyAsync(c->adj[l].p, adj[l].data(), sizeof(int) * adj[l].size(), hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipMemcpyAsync(c->adjx[l].p, adjx[l].data(), sizeof(int) * adjx[l].size(), hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipMemcpyAsync(c->epos[l].p, epos[l].data(), sizeof(int) * epos[l].size(), hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipMemcpyAsync(c->eu[l].p, eu[l].data(), sizeof(int) * eu[l].size(), hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipMemcpyAsync(c->ev[l].p, ev[l].data(), sizeof(int) * ev[l].size(), hipMemcpyHostToDevice, c->stream));
    }
  }
  HIPCHK(c, c->covered.alloc(tn + 16));
  HIPCHK(c, c->live.alloc(4 * tn));  // {node, CSR begin l0, l1, extents} per live position
  HIPCHK(c, c->gscr.alloc(GSCR_WORDS * tn));  // global-mode environment scratch (always, so MD_VARIANT=64 can force that mode)
  HIPCHK(c, c->pend.alloc(tn));
  HIPCHK(c, c->tr_action.alloc(tn));
  HIPCHK(c, c->tr_rank.alloc(tn));
  HIPCHK(c, c->h_tr.alloc(2 * tn));
  HIPCHK(c, c->tr_stat.alloc(4 * tn));
  HIPCHK(c, c->tr_q.alloc(2 * tn));
  // (+4: env_stage_wide stages the last graph's Q row as 16-byte unclipped buffer loads)
  HIPCHK(c, c->q.alloc(tn + 4));
  HIPCHK(c, c->glist.alloc(n_graphs));
  HIPCHK(c, c->ctl.alloc(CTL_WORDS));
  if (c->tpart.p == nullptr) HIPCHK(c, c->tpart.alloc(2 * (size_t)TEAM_MAX_WG * 16));
  HIPCHK(c, c->lab_ok.alloc(n_graphs));
  {
    int max_n = 1;
    for (int g = 0; g < n_graphs; ++g) max_n = std::max(max_n, (int)n_nodes[g]);
    HIPCHK(c, c->gscr_team.alloc((size_t)GSCR_TEAM_WORDS * max_n));
    // batched-prefix scratch, sized by the largest graph that can take the prefix path
    int max_et = 0;
    for (int g = 0; g < n_graphs; ++g) {
      const int et = (int)(c->hinfo[g].e[0] + c->hinfo[g].e[1]);
      if (pfx_fits_host(c->hinfo[g].n, et)) max_et = std::max(max_et, et);
    }
    c->pfx.release();
    if (c->pfx_min > 0 && max_et > 0) HIPCHK(c, c->pfx.alloc((size_t)pfx_words_host(max_et)));
    c->team_owner = -1;
  }
  // speculative environment-step slots of queue launches (bspec_slot): per graph and removal-count
  // parity 4 (9 + e + 2 n) ints >= the SRES layout's 35 + 3 e + 6 n; zeroed (every slot free)
  c->bspec_half = 0;
  c->bspec.release();
  if (c->bspec_on && n_graphs > DEDICATED_MAX_GRAPHS) {
    c->bspec_half = 4 * (9 * (long long)n_graphs + (long long)te[0] + (long long)te[1] + 2 * (long long)tn);
    HIPCHK(c, c->bspec.alloc((size_t)(2 * c->bspec_half)));
    HIPCHK(c, hipMemsetAsync(c->bspec.p, 0, sizeof(int) * (size_t)(2 * c->bspec_half), c->stream));
  }
  HIPCHK(c, c->prank.alloc(ranks.size()));
  HIPCHK(c, hipMemcpyAsync(c->prank.p, ranks.data(), sizeof(uint16_t) * ranks.size(), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemsetAsync(c->lab_ok.p, 0, sizeof(int) * n_graphs, c->stream));
  HIPCHK(c, c->bars.alloc(8 * 64));
  HIPCHK(c, c->spart.alloc(tt * 384));
  HIPCHK(c, c->apart.alloc(tt * 4));
  HIPCHK(c, c->ybuf.alloc((size_t)n_graphs * 128));
  HIPCHK(c, c->hbuf.alloc((size_t)n_graphs * 144 * 2));
  HIPCHK(c, c->xbuf.alloc((size_t)XB_SLOTS * 2048));
  {
    // cache slots: every launch addresses its own tile prefix (the lock-step modes: the launch's
    // tile index; queue mode: gtoff[graph slot] + tile), so the tiles of the QG_CAP largest
    // graphs bound every launch -- not the whole loaded set
    std::vector<long> nt(n_graphs);
    for (int g = 0; g < n_graphs; ++g) nt[g] = (n_nodes[g] + TILE - 1) / TILE;
    std::sort(nt.begin(), nt.end(), std::greater<long>());
    long slots = 0;
    for (int g = 0; g < std::min(n_graphs, QG_CAP); ++g) slots += nt[g];
    c->nbc_slots = (int)std::min<long>(slots, INT32_MAX / NBC_INTS);
    c->max_tiles = (int)std::max<long>(1, nt[0]);
    HIPCHK(c, c->nbc.alloc((size_t)std::max(1, c->nbc_slots) * NBC_INTS));
    HIPCHK(c, c->gtoff.alloc(QG_CAP + 1));
  }  // split tiles of a launch <= CUs / 2 <= XB_SLOTS
  HIPCHK(c, c->h_req.alloc((size_t)n_graphs));
  HIPCHK(c, c->h_ans.alloc((size_t)n_graphs));
  HIPCHK(c, c->h_nact.alloc((size_t)n_graphs));
  HIPCHK(c, c->h_act.alloc(c->tot_n));
  HIPCHK(c, c->h_q.alloc(c->tot_n));
  HIPCHK(c, c->h_chk.alloc(2 * (size_t)n_graphs));
  if (c->h_done.h == nullptr) HIPCHK(c, c->h_done.alloc(2));
  HIPCHK(c, c->h_gvar.alloc((size_t)n_graphs * (sizeof(GraphVar) / sizeof(int))));
  HIPCHK(c, hipMemcpyAsync(c->ginfo.p, info.data(), sizeof(GraphInfo) * n_graphs, hipMemcpyHostToDevice, c->stream));
  if (c->cost_mode == MD_COST_DEGREE) {
    HIPCHK(c, c->node_w.alloc(2 * tn));
    HIPCHK(c, hipMemcpyAsync(c->node_w.p, node_w, sizeof(float) * 2 * tn, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    std::vector<float> wv(W_TOTAL);
    HIPCHK(c, hipMemcpy(wv.data(), c->w.p, sizeof(float) * W_TOTAL, hipMemcpyDeviceToHost));
    for (int l = 0; l < 2; ++l) {
      std::vector<float> tab(tn * EMB);
      for (size_t v = 0; v < tn; ++v) host_first_layer(wv.data(), &node_w[l * tn + v], &tab[v * EMB]);
      HIPCHK(c, hipMemcpy(c->h0tab[l].p, tab.data(), sizeof(float) * tab.size(), hipMemcpyHostToDevice));
    }
  }
  HIPCHK(c, hipStreamSynchronize(c->stream));
  // queue-mode buffers last (allocation order moves the other buffers' addresses)
  HIPCHK(c, c->qslot.alloc(Q_CAP));
  HIPCHK(c, c->qg.alloc(3 * QG_CAP));  // stage counter, stage size per graph slot; lists-built flag
  {
    // speculative-step slots: killed-edge lists of one graph, sized by the graphs a single-graph
    // rollout can run with speculative workgroups (launch_chunk's conditions: the state fits
    // LDS, word-aligned offsets); none at all when MD_SPEC=0 or no graph qualifies
    int maxw = 0;
    if (c->spec_n > 0)
      for (int g = 0; g < n_graphs; ++g) {
        const int et = info[g].e[0] + info[g].e[1];
        if (spec_fits_lds_host(info[g].n, et) && info[g].eoff[0] % 4 == 0 && info[g].eoff[1] % 4 == 0 &&
            info[g].node_off % 4 == 0)
          maxw = std::max(maxw, sres_words(et, info[g].n));
      }
    c->sres_stride = ((maxw + 63) / 64) * 64;
    if (maxw > 0) {
      // two slots per speculative workgroup: requests alternate between them (spec_slot_index)
      HIPCHK(c, c->sres.alloc((size_t)2 * SPEC_SLOTS * c->sres_stride));
      HIPCHK(c, hipMemset(c->sres.p, 0, sizeof(int) * (size_t)2 * SPEC_SLOTS * c->sres_stride));
      HIPCHK(c, c->qspec.alloc(2 * tn));
    } else {
      c->sres.release();
      c->qspec.release();
    }
  }
  {
    int maxn = 0;
    for (int g = 0; g < n_graphs; ++g) maxn = std::max(maxn, (int)n_nodes[g]);
    md_status st = ensure_h0g(c, maxn - 1, false);
    if (st != MD_OK) return st;
  }
  {
    // dataflow mode: a graph qualifies when its single-graph rollout runs with the layer split
    // (environment in LDS, two tile workgroups per tile) and no tile's alive-neighbour list can
    // exceed NB_CAP in either layer (the 16 largest degrees sum to at most NB_CAP: a tile's
    // list holds the alive entries of 16 live rows)
    c->df_graph.assign(n_graphs, 0);
    int dn = 0, dmt = 0;
    if (c->df_on)
      for (int g = 0; g < n_graphs; ++g) {
        const GraphInfo& gi = info[g];
        const int tiles = (gi.n + TILE - 1) / TILE;
        if (!phase_a_fits_lds_host(gi.n, gi.e[0] + gi.e[1]) || 2 + 2 * tiles > c->cus || tiles > XB_SLOTS) continue;
        bool ok = true;
        for (int l = 0; l < 2 && ok; ++l) {
          const int* rp = rowptr[l].data() + gi.roff[l];
          std::vector<int> d(gi.n);
          for (int i = 0; i < gi.n; ++i) d[i] = rp[i + 1] - rp[i];
          const int k = std::min(gi.n, TILE);
          std::partial_sort(d.begin(), d.begin() + k, d.end(), std::greater<int>());
          long s = 0;
          for (int i = 0; i < k; ++i) s += d[i];
          ok = s <= NB_CAP_ENTRIES;
        }
        if (!ok) continue;
        c->df_graph[g] = 1;
        dn = std::max(dn, gi.n);
        dmt = std::max(dmt, tiles);
      }
    if (dn > 0) {
      HIPCHK(c, c->dfbuf.alloc((size_t)df_granules(dn, dmt)));
      c->df_n = dn;
      c->df_mt = dmt;
    }
  }
  return md_reset(c, nullptr);
}

md_status md_reset(md_ctx* c, int32_t* max_rank_out) {
  if (!c) return MD_EINVAL;
  if (c->ng == 0) return fail(c, MD_ESTATE, "no graphs loaded");
  HIPCHK(c, hipSetDevice(c->device));
  c->s0_pending = false;
  std::vector<int> gl(c->ng);
  for (int g = 0; g < c->ng; ++g) gl[g] = g;
  HIPCHK(c, hipMemcpyAsync(c->glist.p, gl.data(), sizeof(int) * gl.size(), hipMemcpyHostToDevice, c->stream));
  Params p = make_params(c);
  p.nglist = c->ng;
  HIPCHK(c, launch_reset(p, c->stream));
  c->last_ms = 0.0;
  c->last_served = 0;
  c->last_launches = 0;
  md_status st = launch(c, gl, RUN_STEP, 0);  // s0: initial prune (U/mvc_env.py:52)
  if (st != MD_OK) return st;
  if (max_rank_out)
    for (int g = 0; g < c->ng; ++g) max_rank_out[g] = c->hvar[g].max_rank;
  return MD_OK;
}

md_status md_reset_deferred(md_ctx* c) {
  if (!c) return MD_EINVAL;
  if (c->ng == 0) return fail(c, MD_ESTATE, "no graphs loaded");
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<int> gl(c->ng);
  for (int g = 0; g < c->ng; ++g) gl[g] = g;
  HIPCHK(c, hipMemcpyAsync(c->glist.p, gl.data(), sizeof(int) * gl.size(), hipMemcpyHostToDevice, c->stream));
  Params p = make_params(c);
  p.nglist = c->ng;
  HIPCHK(c, launch_reset(p, c->stream));
  c->last_ms = 0.0;
  c->last_served = 0;
  c->last_launches = 0;
  // the host view md_rollout starts from (it pushes it to the device): as md_reset_kernel left
  // the GraphVar, with the edge counts as alive counts (a graph with edges in both layers runs;
  // its first environment step, s0 not done, prunes and recomputes them)
  for (int g = 0; g < c->ng; ++g) {
    GraphVar v = {};
    v.status = ST_RUN;
    v.argmax = -1;
    v.alive[0] = c->hinfo[g].e[0];
    v.alive[1] = c->hinfo[g].e[1];
    c->hvar[g] = v;
  }
  c->s0_pending = true;
  return MD_OK;
}

namespace {
// The s0 prune md_reset_deferred left pending, as md_reset runs it (one RUN_STEP launch over
// every graph from the state md_reset_kernel left on the device): called by every entry point
// except md_rollout (whose first environment step runs it) before it reads or changes the
// state, so an action is never applied before the initial prune (U/mvc_env.py:52 then :74-87).
md_status finish_deferred_s0(md_ctx* c) {
  if (!c->s0_pending) return MD_OK;
  c->s0_pending = false;
  std::vector<int> gl(c->ng);
  for (int g = 0; g < c->ng; ++g) gl[g] = g;
  return launch(c, gl, RUN_STEP, 0);
}
}  // namespace

md_status md_max_rank(md_ctx* c, int32_t* max_rank_out) {
  if (!c || !max_rank_out) return MD_EINVAL;
  if (c->ng > 0) {
    HIPCHK(c, hipSetDevice(c->device));
    md_status st = finish_deferred_s0(c);
    if (st != MD_OK) return st;
  }
  for (int g = 0; g < c->ng; ++g) max_rank_out[g] = c->hvar[g].max_rank;
  return MD_OK;
}

md_status md_predict(md_ctx* c, float* q_out, int32_t* argmax, int32_t* n_tie, float* top_gap) {
  if (!c) return MD_EINVAL;
  if (c->ng == 0) return fail(c, MD_ESTATE, "no graphs loaded");
  HIPCHK(c, hipSetDevice(c->device));
  {
    md_status st0 = finish_deferred_s0(c);
    if (st0 != MD_OK) return st0;
  }
  std::vector<int> gl;
  for (int g = 0; g < c->ng; ++g) {
    GraphVar& v = c->hvar[g];
    if (v.alive[0] > 0 && v.alive[1] > 0 && v.n_live > 0) {
      v.status = ST_RUN;
      v.npend = 0;
      gl.push_back(g);
    }
  }
  md_status st = push_vars(c);
  if (st != MD_OK) return st;
  c->last_ms = 0.0;
  c->last_served = 0;
  c->last_launches = 0;
  if (!gl.empty()) {
    // graphs with no live node keep their (all masked) q
    st = launch(c, gl, RUN_PREDICT, 0);
    if (st != MD_OK) return st;
  }
  if (q_out) HIPCHK(c, hipMemcpy(q_out, c->q.p, sizeof(float) * c->tot_n, hipMemcpyDeviceToHost));
  for (int g = 0; g < c->ng; ++g) {
    const bool ran = std::find(gl.begin(), gl.end(), g) != gl.end();
    if (argmax) argmax[g] = ran ? c->hvar[g].argmax : -1;
    if (n_tie) n_tie[g] = ran ? c->hvar[g].ntie : 0;
    if (top_gap) top_gap[g] = ran ? c->hvar[g].gap : 0.f;
  }
  return MD_OK;
}

md_status md_step(md_ctx* c, const int32_t* actions, int32_t* lmcc_out, uint8_t* terminal_out) {
  if (!c || !actions) return MD_EINVAL;
  if (c->ng == 0) return fail(c, MD_ESTATE, "no graphs loaded");
  HIPCHK(c, hipSetDevice(c->device));
  {
    md_status st0 = finish_deferred_s0(c);
    if (st0 != MD_OK) return st0;
  }
  std::vector<int> gl;
  for (int g = 0; g < c->ng; ++g) {
    const int a = actions[g];
    if (a < 0) continue;
    const GraphInfo& gi = c->hinfo[g];
    if (a >= gi.n) return fail(c, MD_EINVAL, "graph %d: action %d out of range", g, a);
    GraphVar& v = c->hvar[g];
    if (v.alive[0] == 0 || v.alive[1] == 0) continue;  // terminal: stepping is a no-op
    v.status = ST_RUN;
    v.npend = 1;
    HIPCHK(c, hipMemcpyAsync(c->pend.p + gi.node_off, &actions[g], sizeof(int), hipMemcpyHostToDevice, c->stream));
    gl.push_back(g);
  }
  md_status st = push_vars(c);
  if (st != MD_OK) return st;
  c->last_ms = 0.0;
  c->last_served = 0;
  c->last_launches = 0;
  st = launch(c, gl, RUN_STEP, 0);
  if (st != MD_OK) return st;
  for (int g = 0; g < c->ng; ++g) {
    const GraphVar& v = c->hvar[g];
    if (lmcc_out) lmcc_out[g] = v.lmcc;
    if (terminal_out) terminal_out[g] = (v.alive[0] == 0 || v.alive[1] == 0) ? 1 : 0;
  }
  return MD_OK;
}

// The device rollout loop of md_rollout / md_rollout_packed (launches until every graph stops).
md_status rollout_run(md_ctx* c, int step, md_select_cb cb, void* user) {
  if (c->ng == 0) return fail(c, MD_ESTATE, "no graphs loaded");
  HIPCHK(c, hipSetDevice(c->device));
  const int host_select = step > 1 ? 1 : 0;
  c->last_ms = 0.0;
  c->last_served = 0;
  c->last_launches = 0;
  std::vector<int> gl, idle;
  for (int g = 0; g < c->ng; ++g) {
    GraphVar& v = c->hvar[g];
    if (v.alive[0] > 0 && v.alive[1] > 0) {
      v.status = ST_RUN;
      v.npend = 0;
      gl.push_back(g);
    } else {
      idle.push_back(g);
    }
  }
  if (c->s0_pending) {
    // the first environment step of this rollout runs the deferred s0 prune for every graph it
    // launches; a graph it leaves out (a layer without edges: terminal from the start) gets the
    // prune here, exactly md_reset's launch, so its state and max_rank equal md_reset's
    c->s0_pending = false;
    if (!idle.empty()) {
      md_status st = launch(c, idle, RUN_STEP, 0);
      if (st != MD_OK) return st;
    }
  }
  std::vector<float> qrow;
  std::vector<double> qd;
  std::vector<int32_t> acts;
  std::vector<std::pair<int, int>> before;
  std::vector<int> stalled(c->ng, 0);
  while (!gl.empty()) {
    md_status st = push_vars(c);
    if (st != MD_OK) return st;
    Selector sel;
    sel.cb = cb;
    sel.user = user;
    sel.step = step;
    before.resize(c->ng);
    for (int g : gl) before[g] = {c->hvar[g].steps, c->hvar[g].npred};
    st = launch(c, gl, RUN_ROLLOUT, host_select, &sel);
    if (st != MD_OK) return st;
    std::vector<int> next;
    for (int g : gl) {
      GraphVar& v = c->hvar[g];
      if (v.status == ST_RUN) {
        // left by a queue-mode launch at its tail: the next launch continues it.  A graph
        // admitted late may be parked right after its first environment step, which removes
        // nothing and predicts nothing, but the launch after a park (at most MD_QPARK graphs:
        // the lock-step kernel, which never parks) always advances it -- a second launch in a
        // row without progress would mean a graph relaunched forever
        if (before[g] == std::make_pair(v.steps, v.npred)) {
          if (++stalled[g] >= 2)
            return fail(c, MD_ESTATE, "graph %d: two rollout launches in a row left it running without progress", g);
        } else {
          stalled[g] = 0;
        }
        v.npend = 0;
        next.push_back(g);
        continue;
      }
      if (v.status != ST_NEED_HOST) continue;
      const GraphInfo& gi = c->hinfo[g];
      if (!cb && !c->tie_argsort)
        return fail(c, MD_ECALLBACK, "graph %d: %d nodes tie at the max Q and no selection callback was given", g, v.ntie);
      qrow.resize(gi.n);
      qd.resize(gi.n);
      HIPCHK(c, hipMemcpy(qrow.data(), c->q.p + gi.node_off, sizeof(float) * gi.n, hipMemcpyDeviceToHost));
      for (int i = 0; i < gi.n; ++i) qd[i] = std::isinf(qrow[i]) ? QMASK : (double)qrow[i];
      const int nout = std::min(step, gi.n);
      acts.assign(nout, -1);
      if (select_actions(c, cb, user, g, qd, gi.n, nout, acts.data()) != 0)
        return fail(c, MD_ECALLBACK, "selection callback failed (graph %d)", g);
      int k = 0;
      for (int i = 0; i < nout; ++i) {
        if (acts[i] < 0 || acts[i] >= gi.n) return fail(c, MD_ECALLBACK, "callback returned node %d out of range", acts[i]);
        acts[k++] = acts[i];
      }
      HIPCHK(c, hipMemcpy(c->pend.p + gi.node_off, acts.data(), sizeof(int) * k, hipMemcpyHostToDevice));
      v.npend = k;
      v.status = ST_RUN;
      next.push_back(g);
    }
    gl.swap(next);
  }
  return MD_OK;
}

md_status md_rollout(md_ctx* c, int step, int32_t* seq_out, int32_t* lmcc_out, int32_t* seq_len, md_select_cb cb,
                     void* user) {
  if (!c || step < 1) return MD_EINVAL;
  const md_status st = rollout_run(c, step, cb, user);
  if (st != MD_OK) return st;
  // (every graph is terminal: its trace went to the host mirrors as it ended, trace_publish)
  if (seq_out) std::memcpy(seq_out, c->h_tr.h, sizeof(int) * c->tot_n);
  if (lmcc_out) std::memcpy(lmcc_out, c->h_tr.h + c->tot_n, sizeof(int) * c->tot_n);
  if (seq_len)
    for (int g = 0; g < c->ng; ++g) seq_len[g] = c->hvar[g].steps;
  return MD_OK;
}

md_status md_rollout_packed(md_ctx* c, int step, int32_t* seq_packed, int32_t* lmcc_packed, int32_t* seq_len,
                            md_select_cb cb, void* user) {
  if (!c || step < 1 || !seq_packed || !lmcc_packed || !seq_len) return MD_EINVAL;
  static const bool host_stats = std::getenv("MD_HOST_STATS") != nullptr;  // diagnostics
  const auto t0 = std::chrono::steady_clock::now();
  const md_status st = rollout_run(c, step, cb, user);
  if (st != MD_OK) return st;
  struct PackStats {
    std::chrono::steady_clock::time_point t0, t1;
    bool on;
    ~PackStats() {
      if (on)
        std::fprintf(stderr, "md host: rollout %.3f ms, outputs %.3f ms\n",
                     1e3 * std::chrono::duration<double>(t1 - t0).count(),
                     1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count());
    }
  } ps{t0, std::chrono::steady_clock::now(), host_stats};
  // (every graph is terminal: its trace went to the host mirrors as it ended, trace_publish;
  // only the removals are read, from host memory)
  int tot = 0;
  for (int g = 0; g < c->ng; ++g) {
    const int len = c->hvar[g].steps, off = (int)c->hinfo[g].node_off;
    std::memcpy(seq_packed + tot, c->h_tr.h + off, sizeof(int) * len);
    std::memcpy(lmcc_packed + tot, c->h_tr.h + c->tot_n + off, sizeof(int) * len);
    seq_len[g] = len;
    tot += len;
  }
  return MD_OK;
}

md_status md_spec_stats(md_ctx* c, int graph, int32_t* hits, int32_t* removals) {
  if (!c || graph < 0 || graph >= c->ng) return MD_EINVAL;
  if (hits) *hits = c->hvar[graph].spec_hits;
  if (removals) *removals = c->hvar[graph].steps;
  return MD_OK;
}

md_status md_rollout_trace(md_ctx* c, int graph, int32_t* n_live, int32_t* m0, int32_t* m1, int32_t* n_tie,
                           float* qmax, float* gap, int32_t* n_pred) {
  if (!c || graph < 0 || graph >= c->ng) return MD_EINVAL;
  const GraphInfo& gi = c->hinfo[graph];
  const int np = std::min(c->hvar[graph].npred, gi.n);
  std::vector<int> st(4 * (size_t)np);
  std::vector<float> tq(2 * (size_t)np);
  if (np > 0) {
    HIPCHK(c, hipMemcpy(st.data(), c->tr_stat.p + 4 * (size_t)gi.node_off, sizeof(int) * st.size(), hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemcpy(tq.data(), c->tr_q.p + 2 * (size_t)gi.node_off, sizeof(float) * tq.size(), hipMemcpyDeviceToHost));
  }
  for (int t = 0; t < np; ++t) {
    if (n_live) n_live[t] = st[4 * t + 0];
    if (m0) m0[t] = st[4 * t + 1];
    if (m1) m1[t] = st[4 * t + 2];
    if (n_tie) n_tie[t] = st[4 * t + 3];
    if (qmax) qmax[t] = tq[2 * t + 0];
    if (gap) gap[t] = tq[2 * t + 1];
  }
  if (n_pred) *n_pred = np;
  return MD_OK;
}

md_status md_get_state(md_ctx* c, int graph, uint8_t* covered, uint8_t* removed0, uint8_t* removed1, int32_t* counters) {
  if (!c || graph < 0 || graph >= c->ng) return MD_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  {
    md_status st0 = finish_deferred_s0(c);
    if (st0 != MD_OK) return st0;
  }
  const GraphInfo& gi = c->hinfo[graph];
  if (covered) HIPCHK(c, hipMemcpy(covered, c->covered.p + gi.node_off, gi.n, hipMemcpyDeviceToHost));
  uint8_t* outs[2] = {removed0, removed1};
  for (int l = 0; l < 2; ++l) {
    if (!outs[l] || gi.e[l] == 0) continue;
    HIPCHK(c, hipMemcpy(outs[l], c->estate[l].p + gi.eoff[l], gi.e[l], hipMemcpyDeviceToHost));
    for (int e = 0; e < gi.e[l]; ++e) outs[l][e] = outs[l][e] == E_PRUNED ? 1 : 0;
  }
  if (counters) {
    const GraphVar& v = c->hvar[graph];
    counters[0] = v.counter[0];
    counters[1] = v.counter[1];
    counters[2] = v.removed[0];
    counters[3] = v.removed[1];
    counters[4] = v.lmcc;
    counters[5] = (v.alive[0] == 0 || v.alive[1] == 0) ? 1 : 0;
  }
  return MD_OK;
}

md_status md_set_state(md_ctx* c, int graph, const uint8_t* covered, const uint8_t* removed0, const uint8_t* removed1) {
  if (!c || graph < 0 || graph >= c->ng || !covered) return MD_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  {
    md_status st0 = finish_deferred_s0(c);
    if (st0 != MD_OK) return st0;
  }
  const GraphInfo& gi = c->hinfo[graph];
  GraphVar& v = c->hvar[graph];
  std::vector<int> eu, ev;
  int ncov = 0;
  for (int i = 0; i < gi.n; ++i) ncov += covered[i] ? 1 : 0;
  const uint8_t* rem[2] = {removed0, removed1};
  for (int l = 0; l < 2; ++l) {
    std::vector<uint8_t> st(std::max(1, gi.e[l]));
    eu.resize(gi.e[l]);
    ev.resize(gi.e[l]);
    if (gi.e[l]) {
      HIPCHK(c, hipMemcpy(eu.data(), c->eu[l].p + gi.eoff[l], sizeof(int) * gi.e[l], hipMemcpyDeviceToHost));
      HIPCHK(c, hipMemcpy(ev.data(), c->ev[l].p + gi.eoff[l], sizeof(int) * gi.e[l], hipMemcpyDeviceToHost));
    }
    int ccov = 0, cpr = 0, calive = 0;
    std::vector<int> ep(2 * (size_t)std::max(1, gi.e[l]));
    std::vector<uint8_t> ca(2 * (size_t)std::max(1, gi.e[l]), 1);
    if (gi.e[l]) HIPCHK(c, hipMemcpy(ep.data(), c->epos[l].p + 2 * (size_t)gi.eoff[l], sizeof(int) * 2 * gi.e[l], hipMemcpyDeviceToHost));
    for (int e = 0; e < gi.e[l]; ++e) {
      if (rem[l] && rem[l][e]) { st[e] = E_PRUNED; cpr++; }
      else if (covered[eu[e]] || covered[ev[e]]) { st[e] = E_COVERED; ccov++; }
      else { st[e] = E_ALIVE; calive++; }
      if (st[e] != E_ALIVE) ca[ep[2 * e]] = ca[ep[2 * e + 1]] = 0;
    }
    if (gi.e[l]) {
      HIPCHK(c, hipMemcpy(c->estate[l].p + gi.eoff[l], st.data(), gi.e[l], hipMemcpyHostToDevice));
      HIPCHK(c, hipMemcpy(c->calive[l].p + gi.coff[l], ca.data(), 2 * (size_t)gi.e[l], hipMemcpyHostToDevice));
    }
    v.counter[l] = ccov;
    v.removed[l] = cpr;
    v.alive[l] = calive;
  }
  HIPCHK(c, hipMemcpy(c->covered.p + gi.node_off, covered, gi.n, hipMemcpyHostToDevice));
  HIPCHK(c, hipMemset(c->lab_ok.p + graph, 0, sizeof(int)));  // the grid-wide step's class labels are stale
  v.n_cov = ncov;
  v.s0_done = 1;
  v.npend = 0;
  v.status = ST_RUN;
  v.n_live = 1;  // recomputed by the next prediction's phase A
  v.hdmax[0] = v.hdmax[1] = 0;
  return push_vars(c);
}

md_status md_profile(md_ctx* c, int steps) {
  if (!c || steps < 0) return MD_EINVAL;
  HIPCHK(c, hipSetDevice(c->device));
  c->prof.release();
  c->prof_cap = 0;
  c->prof_host.clear();
  if (steps > 0) {
    HIPCHK(c, c->prof.alloc((size_t)steps * PROF_SLOTS));
    HIPCHK(c, hipMemset(c->prof.p, 0, sizeof(unsigned long long) * (size_t)steps * PROF_SLOTS));
    c->prof_cap = steps;
  }
  return MD_OK;
}

md_status md_profile_read(md_ctx* c, uint64_t* out, int capacity_steps, int32_t* n_steps) {
  if (!c || capacity_steps < 0) return MD_EINVAL;
  const int have = (int)(c->prof_host.size() / PROF_SLOTS);
  const int k = std::min(have, capacity_steps);
  if (out) std::memcpy(out, c->prof_host.data(), sizeof(uint64_t) * PROF_SLOTS * (size_t)k);
  if (n_steps) *n_steps = k;
  return MD_OK;
}

md_status md_host_requests(md_ctx* c, int32_t* n_requests) {
  if (!c || !n_requests) return MD_EINVAL;
  *n_requests = c->last_served;
  return MD_OK;
}

md_status md_last_timing(md_ctx* c, double* kernel_ms, int32_t* launches) {
  if (!c) return MD_EINVAL;
  if (kernel_ms) *kernel_ms = c->last_ms;
  if (launches) *launches = c->last_launches;
  return MD_OK;
}

}  // extern "C"
