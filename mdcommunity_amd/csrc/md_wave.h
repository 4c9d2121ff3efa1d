// md_wave.h — batch rollouts with one work item per WAVE (md_wq_kernel), included by
// md_kernels.hip inside namespace md.
//
// The queue kernel (md_queue_kernel, queue_loop) runs every work item on a whole 512-thread
// workgroup: the item's eight waves move through its pieces together (neighbour-list header,
// gather batches, MFMA update, normalisation, stores), separated by workgroup barriers, so the
// two waves a SIMD holds are always in the same piece and wait for memory together (MFMA busy
// 15 %, waves waiting 55 %: VERDICT r04 item 1).  Here each of the eight waves of a workgroup
// is an independent worker: it pops its own items from the same device queue and runs a whole
// 16-row tile (both layers) or a virtual-node step by itself, with no workgroup barrier -- the
// two waves of a SIMD belong to different items, so one's gather round trips overlap the
// other's MFMA chains.  Every output is computed by the same operations in the same order as the
// workgroup pieces (MFMA k-chains per 16x16 accumulator, CSR-order neighbour sums, torch-order
// row norms, ascending-row column sums, the attention / Q-head chains), so rollouts are
// identical (GPU tests: MD_WQ=0 against the default).
//
// The environment step (phase A: U/mvc_env.py:74-87, U/Mcc.py:30-38, U/PrepareBatchGraph.py:35-74)
// keeps its 512-thread LDS-resident code: a wave that pops an ENV item queues it in the
// workgroup's group words and every wave joins a group section at its next item boundary (or
// while it waits for an item), where the workgroup runs the queued environment steps together
// and reloads the weight image they overwrote.
//
// Per-wave LDS (WQ_AREA floats in the tile scratch): WA, a 16-row block transposed (wq_o) or
// gather staging rows; WL, the alive-neighbour lists of both layers (u16).  The weight image is
// shared.

constexpr int WQ_AREA = 2048;                  // floats of LDS per wave
constexpr int WQ_WA = 0, WQ_WL = 64 * LDT;     // WA [64][17] floats, WL [2][WQ_LIST_MAX] u16
constexpr int WQ_LIST_MAX = 960;               // alive entries per layer the list area holds
constexpr int WQ_SPEC_WORDS = 256;             // list words per layer loaded with the header
static_assert(WQ_WL + WQ_LIST_MAX <= WQ_AREA, "list area");
// A 16-row block in WA is transposed with a 17-float pitch (wq_o(k, row)): every access pattern
// below is one lane base plus immediate offsets (the rotated paired-tile layout needs a lane
// offset per k-step, which the compiler hoists out of the item loop as hundreds of live
// registers), and the MFMA A-operand reads conflict in one lane pair per 32-lane half only.
__device__ __forceinline__ int wq_o(int k, int row) { return k * LDT + row; }
constexpr int WQ_WAVES = NTHREADS / 64;
static_assert(WQ_WAVES * WQ_AREA <= S_END, "per-wave areas inside the tile scratch");
// group words (ints at L_PREF; phase A uses L_PREF only with speculative workgroups or the
// dataflow buffer, neither of which a queue launch has): queued ENV items, the items, waves done
constexpr int WQC_REQ = 0, WQC_ITEMS = 1, WQC_DONE = 1 + WQ_WAVES;
static_assert(WQC_DONE + 1 <= G_CAP + 4, "group words fit L_PREF");
constexpr unsigned WQ_GROUP = 0xfffffff8u;     // wq_wait: go to the group section (ticket kept)

__device__ __forceinline__ int wq_wave() { return __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6); }
__device__ __forceinline__ float* wq_area() { return lds_base() + L_SCR + wq_wave() * WQ_AREA; }
__device__ __forceinline__ volatile int* wq_ctl() { return (volatile int*)(lds_base() + L_PREF); }
// LDS hand-off between lanes of one wave (a wave's LDS operations complete in order; the fences
// keep the compiler from moving them across)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ int wq_uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
// The lane index, opaque to the optimiser: every lane-dependent address of an item derives from
// it, so none is hoisted out of the item loop (hoisted, the offsets of all the items' pieces stay
// live across the loop and spill, and each scratch reload -- a vector-memory load -- makes the
// wave wait for every load in flight before it)
__device__ __forceinline__ int wq_lane() {
  int l = (int)threadIdx.x & 63;
  asm volatile("" : "+v"(l));
  return l;
}
__device__ __forceinline__ unsigned long long wq_uni64(unsigned long long x) {
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)x), hi = __builtin_amdgcn_readfirstlane((unsigned)(x >> 32));
  return ((unsigned long long)hi << 32) | lo;
}

// Piece profile of the wave items (builds with -DMD_QPROF, md_profile with MD_VARIANT bit 8):
// device ticks per piece summed over items in prof[20 + 8 (it - 1) + piece] (scripts/batch_prof.py)
#ifdef MD_QPROF
#define WQTS_INIT(it_)                                                                                \
  unsigned long long* wqd_ = (kp().prof != nullptr && (kp().variant & 8)) ? kp().prof + 20 + 8 * ((it_) - 1) : nullptr; \
  unsigned long long wqt_ = wall_clock64()
#define WQTS(k)                                                        \
  do {                                                                 \
    if (wqd_ != nullptr && lane_id() == 0) {                           \
      const unsigned long long now_ = wall_clock64();                  \
      atomicAdd(wqd_ + (k), now_ - wqt_);                              \
      wqt_ = now_;                                                     \
    }                                                                  \
  } while (0)
#define WQTS_RESET() wqt_ = wall_clock64()
#define WQTA_INIT()                                                                                      \
  unsigned long long* wqd_ = (kp().prof != nullptr && (kp().variant & 8)) ? kp().prof + 88 : nullptr; \
  unsigned long long wqt_ = wall_clock64()
// the ENV item's pieces in prof[44 + piece] (thread 0 of the group section)
#define WQTE_INIT()                                                                                      \
  unsigned long long* wqe_ = (kp().prof != nullptr && (kp().variant & 8)) ? kp().prof + 44 : nullptr; \
  unsigned long long wqte_ = wall_clock64()
#define WQTE(k)                                                        \
  do {                                                                 \
    if (wqe_ != nullptr && threadIdx.x == 0) {                         \
      const unsigned long long now_ = wall_clock64();                  \
      atomicAdd(wqe_ + (k), now_ - wqte_);                             \
      wqte_ = now_;                                                    \
    }                                                                  \
  } while (0)
#else
#define WQTE_INIT() do {} while (0)
#define WQTE(k) do {} while (0)
#define WQTA_INIT() do {} while (0)
#define WQTS_INIT(it_) do {} while (0)
#define WQTS(k) do {} while (0)
#define WQTS_RESET() do {} while (0)
#endif

// Event log of graph slot 0 (diagnostics, md_profile with MD_VARIANT bit 4): {event, wall clock}
// pairs after the first 8 profile records -- 6 ENV item taken, 0 environment step starts (group
// section), 5 its tiles pushed, 1..3 tile stage 1..3 complete, 4 virtual-node part 2 done
// (scripts/wq_timeline.py)
__device__ __forceinline__ void wq_event(KParams& p, int gl, int ev) {
  if (p.prof == nullptr || !(p.variant & 4) || gl != 0 || p.prof_cap < 16) return;
  const unsigned long long k = atomicAdd(p.prof + 8 * PROF_SLOTS - 1, 1ull);
  if (8 * PROF_SLOTS + 2 * k + 1 < (unsigned long long)p.prof_cap * PROF_SLOTS) {
    p.prof[8 * PROF_SLOTS + 2 * k] = (unsigned long long)ev;
    p.prof[8 * PROF_SLOTS + 2 * k + 1] = wall_clock64();
  }
}

// ------------------------------------------------------------------ per-wave queue operations
__device__ __forceinline__ unsigned wq_take(KParams& p) {
  unsigned t = 0u;
  if (lane_id() == 0) t = __hip_atomic_fetch_add(q_ctl(p) + QC_HEAD, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (unsigned)wq_uni((int)t);
}
__device__ __forceinline__ unsigned long long wq_peek(KParams& p, unsigned tk) {
  unsigned long long v = 0ull;
  if (lane_id() == 0) v = __hip_atomic_load((const g_u64*)q_slot(p, tk), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return wq_uni64(v);
}
__device__ __forceinline__ bool wq_error(KParams& p) {
  unsigned e = 0u;
  if (lane_id() == 0) e = __hip_atomic_load((g_u32*)p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & BAR_ERR;
  return wq_uni((int)e) != 0;
}
// The item of ticket tk (pre: its slot as read earlier), QK_EXIT on an error anywhere, or
// WQ_GROUP when a group section is requested while the slot is still empty (the ticket stays
// held: the caller comes back for it).
__device__ __noinline__ unsigned wq_wait(KParams&, unsigned tk, unsigned long long pre) {
  KParams& p = kp();
  unsigned long long v = pre;
  if ((v >> 32) == (unsigned long long)(tk + 1u)) return (unsigned)v;
  const unsigned long long t0 = wall_clock64();
  while (true) {
    if (wq_ctl()[WQC_REQ] != 0) return WQ_GROUP;
    if (wq_error(p)) return QK_EXIT;
    v = wq_peek(p, tk);
    if ((v >> 32) == (unsigned long long)(tk + 1u)) return (unsigned)v;
    __builtin_amdgcn_s_sleep(2);
    if (wall_clock64() - t0 > (p.h_req != nullptr ? HOST_TIMEOUT_TICKS : BARRIER_TIMEOUT_TICKS)) {
      if (lane_id() == 0) raise_err(p, ERR_TIMEOUT);
      return QK_EXIT;
    }
  }
}
// n items f(0..n-1) pushed by one wave, after its own data stores have drained (they are all
// the data the items read that this wave produced; the other producers drained theirs before
// their stage-counter adds, which the caller's add came after).
template <class F>
__device__ __forceinline__ void wq_push(KParams& p, int n, F&& f) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned base = 0u;
  if (lane_id() == 0) base = __hip_atomic_fetch_add(q_ctl(p) + QC_TAIL, (unsigned)n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  base = (unsigned)wq_uni((int)base);
  for (int i = lane_id(); i < n; i += 64) {
    const unsigned tk = base + (unsigned)i;
    __hip_atomic_store((g_u64*)q_slot(p, tk), ((unsigned long long)(tk + 1u) << 32) | f(i), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ------------------------------------------------------------------ one wave's tile pieces
// Row norms of a 16 x 64 block given in MFMA accumulator layout (lane (ak, ar) holds rows
// 4 ak + r, columns 16 cb + ar in x[cb][r]): written to WA, per-row torch-order sums of
// squares (accumulator j = columns j, 8 + j, ... as an FMA chain, then acc0 + ... + acc7), and
// x divided by max(sqrt(sum), 1e-12) in place.  WA is free afterwards (written again by the
// caller before reads).
__device__ __forceinline__ void wq_norm_rows(float* wa, f4 (&x)[4]) {
  const int lane = wq_lane(), ar = lane & 15, ak = lane >> 4;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) wa[wq_o(16 * cb + ar, 4 * ak + r)] = x[cb][r];
  wave_lds_sync();
  const int row = lane >> 2, jp = lane & 3;
  float pa = 0.f, pb = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float va = wa[wq_o(8 * i + 2 * jp, row)], vb = wa[wq_o(8 * i + 2 * jp + 1, row)];
    pa = fmaf(va, va, pa);
    pb = fmaf(vb, vb, pb);
  }
  const int b0 = lane & ~3;
  float acc8[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    acc8[2 * k] = __shfl(pa, b0 + k, 64);
    acc8[2 * k + 1] = __shfl(pb, b0 + k, 64);
  }
  const float den = fmaxf(sqrtf(sumsq8_finish(acc8)), 1e-12f);
  wave_lds_sync();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float d = __shfl(den, 4 * (4 * ak + r), 64);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) x[cb][r] = x[cb][r] / d;
  }
}

// x (accumulator layout) into WA as the transposed rotated block: WA[wq_o(col, row)]
__device__ __forceinline__ void wq_put_acc(float* wa, const f4 (&x)[4]) {
  const int lane = wq_lane(), ar = lane & 15, ak = lane >> 4;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) wa[wq_o(16 * cb + ar, 4 * ak + r)] = x[cb][r];
}

// Neighbour sums of the 16 rows from the alive-neighbour list in WL (CSR order per row, rows'
// entries contiguous; off/cnt per row from the cached header): batches of 16 list entries, each
// lane loading one 16-byte quarter-row of four entries, a window of WQ_WIN batches in flight;
// each batch is staged in WA and every lane adds, for each of its four rows, that row's entries
// of the batch in list order (sequential float adds from 0, gather_pair's order).  Result:
// WA[wq_o(k, r)] = P[r][k].
#ifndef MD_WQ_WIN
#define MD_WQ_WIN 4
#endif
constexpr int WQ_WIN = MD_WQ_WIN;
__device__ __forceinline__ void wq_gather_list(KParams& p, const float* hp, int tot, int hdw, int l, float* wa,
                                               const lds_u16* wl) {
  const int lane = wq_lane(), q = lane & 15, rs = lane >> 4;
  int offm[4], endm[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    offm[m] = __shfl(hdw, l * 16 + rs + 4 * m, 64);
    endm[m] = offm[m] + __shfl(hdw, 32 + l * 16 + rs + 4 * m, 64);
  }
  float4 acc[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) acc[m] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int nb = (tot + 15) >> 4;
  // loads without branches (entries past the list's end re-read its last row, unused): an
  // exec-masked load makes the compiler's wait counting give up (vmcnt(0) at the join)
  const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(hp), 0, 0x7fffffff, 0x00020000);
  v4f xw[WQ_WIN][4];
  auto issue = [&](int b, v4f (&x)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = min(16 * b + rs + 4 * i, tot - 1);
      x[i] = __builtin_amdgcn_raw_buffer_load_b128(rsc, (int)wl[e] * 256 + q * 16, 0, 16 /* sc1 */);
    }
  };
  float4* stg = (float4*)wa;
  auto consume = [&](int b, const v4f (&x)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (16 * b + rs + 4 * i < tot) stg[(rs + 4 * i) * 16 + q] = make_float4(x[i].x, x[i].y, x[i].z, x[i].w);
    wave_lds_sync();
    // a row's entries of the batch in order, eight staged loads in flight before their adds
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int lo = max(offm[m], 16 * b), hi = min(endm[m], 16 * b + 16);
      for (int k = lo; k < hi; k += 8) {
        float4 y[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
          if (k + jj < hi) y[jj] = stg[(k + jj - 16 * b) * 16 + q];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
          if (k + jj < hi) {
            acc[m].x = acc[m].x + y[jj].x;
            acc[m].y = acc[m].y + y[jj].y;
            acc[m].z = acc[m].z + y[jj].z;
            acc[m].w = acc[m].w + y[jj].w;
          }
      }
    }
    wave_lds_sync();
  };
  if (nb > 0) {
#pragma unroll
    for (int u = 0; u < WQ_WIN; ++u) issue(u, xw[u]);
  }
  for (int b = 0; b < nb; b += WQ_WIN) {
#pragma unroll
    for (int u = 0; u < WQ_WIN; ++u) {
      if (b + u < nb) {
        consume(b + u, xw[u]);
        issue(b + u + WQ_WIN, xw[u]);
      }
    }
  }
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int r = rs + 4 * m;
    wa[wq_o(4 * q + 0, r)] = acc[m].x;
    wa[wq_o(4 * q + 1, r)] = acc[m].y;
    wa[wq_o(4 * q + 2, r)] = acc[m].z;
    wa[wq_o(4 * q + 3, r)] = acc[m].w;
  }
  wave_lds_sync();
}

// Neighbour sums straight from the CSR (no usable cached list: not built, over WQ_LIST_MAX or
// NB_CAP entries): rows one after the other, the row's CSR entries 64 at a time (alive flag,
// neighbour), its alive ones in CSR order four per load (a 16-lane group each), added in order
// by the group-0 lanes.  Same result layout.
__device__ __forceinline__ void wq_gather_csr(KParams& p, const GraphInfo& gi, const float* hp, bool table, int l,
                                              int vrow, float* wa) {
  const int lane = wq_lane(), q = lane & 15, grp = lane >> 4;
  const int* rp = p.rowptr[l] + gi.roff[l];
  const int* adj = p.adj[l] + gi.coff[l];
  const uint8_t* ca = p.calive[l] + gi.coff[l];
  const int* deg = p.deg[l] + gi.node_off;
  for (int r = 0; r < TILE; ++r) {
    const int v = __shfl(vrow, r, 64);
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    if (v >= 0) {
      const int rb = rp[v], re = rp[v + 1];
      for (int c0 = rb; c0 < re; c0 += 64) {
        const int e = c0 + lane;
        int nb = -1;
        if (e < re && ldc(ca + e)) nb = adj[e];
        if (table && nb >= 0) nb = ldc(deg + nb);
        unsigned long long m = __ballot(nb >= 0);
        while (m != 0ull) {
          int src[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int b = m != 0ull ? __builtin_ctzll(m) : -1;
            if (m != 0ull) m &= m - 1ull;
            src[k] = b < 0 ? -1 : __shfl(nb, b, 64);
          }
          const int mine = src[grp];
          float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
          if (mine >= 0) x = ldc4(hp, mine * 256 + q * 16);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float4 y = make_float4(__shfl(x.x, 16 * k + q, 64), __shfl(x.y, 16 * k + q, 64),
                                         __shfl(x.z, 16 * k + q, 64), __shfl(x.w, 16 * k + q, 64));
            if (src[k] >= 0) {
              acc.x = acc.x + y.x;
              acc.y = acc.y + y.y;
              acc.z = acc.z + y.z;
              acc.w = acc.w + y.w;
            }
          }
        }
      }
    }
    if (grp == 0) {
      wa[wq_o(4 * q + 0, r)] = acc.x;
      wa[wq_o(4 * q + 1, r)] = acc.y;
      wa[wq_o(4 * q + 2, r)] = acc.z;
      wa[wq_o(4 * q + 3, r)] = acc.w;
    }
  }
  wave_lds_sync();
}

// Layer l's source rows of iteration it: the previous iteration's H, or (it == 1) the first-layer
// rows, by residual degree (unit cost: the precomputed table of the step's dmax, `table`) or by
// node (degree cost).
__device__ __forceinline__ const float* wq_src(KParams& p, const GraphInfo& gi, int it, int l, bool& table) {
  table = false;
  if (it == 1) {
    table = p.node_w == nullptr;
    return table ? first_layer_rows(p, gi, l) : p.h0tab[l] + (size_t)gi.node_off * EMB;
  }
  return p.H[l][(it - 2) & 1] + (size_t)gi.node_off * EMB;
}
// The 16 own rows as MFMA A operands: lane (ak, ar) holds X[ar][4 s + ak] (vx: row ar's source
// row in lane ar's group, -1 for an empty row).
__device__ __forceinline__ void wq_xload(const float* hp, int vx, float (&xa)[16]) {
  const int ak = wq_lane() >> 4;
  const __amdgpu_buffer_rsrc_t rsc = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(hp), 0, 0x7fffffff, 0x00020000);
  const int base = max(vx, 0) * 256 + 4 * ak;  // (an empty row reads row 0, then zeroes it: no branch)
#pragma unroll
  for (int s = 0; s < 16; ++s)
    xa[s] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsc, base + 16 * s, 0, 16 /* sc1 */));
#pragma unroll
  for (int s = 0; s < 16; ++s) xa[s] = vx >= 0 ? xa[s] : 0.f;
}

// One layer of one tile on one wave (iteration it), in two parts so the caller can issue the next
// layer's loads between them.  Front: S0 (it == 1: column sums of the first-layer input rows) and
// the gather; back: node update relu([P.P1 | X.P2] . P3) on the MFMA chains of update_pair, row
// normalisation, the H rows and (it < 3) the virtual-node partial sums S1 / S2.  `en` returns
// the normalised rows in accumulator layout (the attention's input at it == 3).
__device__ __forceinline__ void wq_layer_front(KParams& p, const GraphInfo& gi, int it, int j, int l, int vrow, int nv,
                                               int hdw, int tot, bool listed, float* wa, const lds_u16* wl,
                                               const float (&xa)[16]) {
  const int lane = wq_lane(), ar = lane & 15, ak = lane >> 4;
  WQTS_INIT(it);
  bool table;
  const float* hp = wq_src(p, gi, it, l, table);
  if (it == 1) {
    // S0: column sums of the first-layer input rows (col_sum16's order)
#pragma unroll
    for (int s = 0; s < 16; ++s) wa[wq_o(4 * s + ak, ar)] = xa[s];
    wave_lds_sync();
    float v[TILE];
#pragma unroll
    for (int r = 0; r < TILE; ++r) v[r] = wa[wq_o(lane, r)];
    float s0 = 0.f;
#pragma unroll
    for (int r = 0; r < TILE; ++r)
      if (r < nv) s0 = s0 + v[r];
    stc(p.spart + (size_t)(gi.tile_off + j) * 384 + l * 64 + lane, s0);
    wave_lds_sync();
  }
  WQTS(1);  // own rows' wait, S0
  if (listed) wq_gather_list(p, hp, tot, hdw, l, wa, wl);
  else wq_gather_csr(p, gi, hp, table, l, vrow, wa);
  WQTS(2);  // gather
}

__device__ __forceinline__ void wq_layer_back(KParams& p, const GraphInfo& gi, int it, int j, int l, int vrow, int nv,
                                              float* wa, const float (&xa)[16], f4 (&en)[4]) {
  const int lane = wq_lane(), ar = lane & 15, ak = lane >> 4;
  WQTS_INIT(it);
  const float* wi = lds_base() + L_W;
  // update, part 1: P.P1 and X.P2 (update_pair's chains for each column block)
  f4 a1[4], a2[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    a1[cb] = f4{0.f, 0.f, 0.f, 0.f};
    a2[cb] = f4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const float ap = wa[wq_o(4 * s + ak, ar)];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      a1[cb] = mfma16(ap, wi[W_IP1 + (cb * 16 + s) * 64 + lane], a1[cb]);
      a2[cb] = mfma16(xa[s], wi[W_IP2 + (cb * 16 + s) * 64 + lane], a2[cb]);
    }
  }
  wave_lds_sync();
  // part 2: M = [P.P1 | X.P2] through WA in two halves, relu(M.P3) (k-steps 0..31 in order)
  f4 a3[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) a3[cb] = f4{0.f, 0.f, 0.f, 0.f};
  wq_put_acc(wa, a1);
  wave_lds_sync();
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const float am = wa[wq_o(4 * s + ak, ar)];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) a3[cb] = mfma16(am, wi[W_IP3 + (cb * 32 + s) * 64 + lane], a3[cb]);
  }
  wave_lds_sync();
  wq_put_acc(wa, a2);
  wave_lds_sync();
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const float am = wa[wq_o(4 * s + ak, ar)];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) a3[cb] = mfma16(am, wi[W_IP3 + (cb * 32 + 16 + s) * 64 + lane], a3[cb]);
  }
  wave_lds_sync();
#pragma unroll
  for (int cb = 0; cb < 4; ++cb)
#pragma unroll
    for (int r = 0; r < 4; ++r) en[cb][r] = fmaxf(a3[cb][r], 0.f);
  WQTS(3);  // update
  wq_norm_rows(wa, en);
  if (it < 3) {
    wq_put_acc(wa, en);
    wave_lds_sync();
    // S1 / S2 (col_sum16 of the normalised rows)
    float v[TILE];
#pragma unroll
    for (int r = 0; r < TILE; ++r) v[r] = wa[wq_o(lane, r)];
    float sn = 0.f;
#pragma unroll
    for (int r = 0; r < TILE; ++r)
      if (r < nv) sn = sn + v[r];
    stc(p.spart + (size_t)(gi.tile_off + j) * 384 + (it == 1 ? 128 : 256) + l * 64 + lane, sn);
    // the rows, a 16-byte quarter per lane and row
    float* hb = p.H[l][(it - 1) & 1] + (size_t)gi.node_off * EMB;
    const int q = lane & 15, rs = lane >> 4;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int r = rs + 4 * m;
      const int v = __shfl(vrow, r, 64);
      if (v >= 0)
        stc4(hb, v * 256 + q * 16,
             make_float4(wa[wq_o(4 * q, r)], wa[wq_o(4 * q + 1, r)], wa[wq_o(4 * q + 2, r)], wa[wq_o(4 * q + 3, r)]));
    }
    wave_lds_sync();
  }
  WQTS(4);  // normalisation, sums and stores
}

// Iteration 3 of one tile on one wave after both layers: attention_q_tile's pieces --
// F_l = tanh(E_l.T + b), the gate dot products, E'_l = F_l + g_l F_other normalised, the
// outer-product chain e = sum_b (h y_b) cp_b, relu(e.H1), the Q head, q = w0 Q0 + w1 Q1 and the
// tile's arg-max partial.  y and the graph scalars come from the head granules of this forward
// pass (tag htag = the graph's predictions so far + 1; the granules are cleared per launch): the
// iteration-3 tiles are queued beside virtual-node part 2 and wait here for its hand-off.
__device__ __forceinline__ void wq_attention(KParams& p, const GraphInfo& gi, int g, int j, int vrow,
                                             f4 (&e0)[4], f4 (&e1)[4], float* wa, unsigned htag) {
  const int lane = wq_lane(), ar = lane & 15, ak = lane >> 4;
  const float* wi = lds_base() + L_W;
  WQTA_INIT();
  // head granules: y of both layers (lanes), the graph scalars (lanes 0..15)
  float yv[2], gsv = 0.f;
  {
    const g_u64* hb = (const g_u64*)(p.hbuf + 2 * ((size_t)g * HB_FLOATS));
    unsigned long long gr[3];
    const unsigned long long t0 = wall_clock64();
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int idx = lane + 64 * k;
      gr[k] = (unsigned long long)htag << 32;
      if (idx < HB_FLOATS) {
        while (((gr[k] = __hip_atomic_load(hb + idx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) != htag) {
          __builtin_amdgcn_s_sleep(1);
          if (wall_clock64() - t0 > BARRIER_TIMEOUT_TICKS ||
              (__hip_atomic_load((g_u32*)p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & BAR_ERR)) {
            raise_err(p, ERR_TIMEOUT);
            gr[k] = 0ull;
            break;
          }
        }
      }
    }
    yv[0] = __uint_as_float((unsigned)gr[0]);
    yv[1] = __uint_as_float((unsigned)gr[1]);
    gsv = __uint_as_float((unsigned)gr[2]);
  }
  WQTS(3);  // head granules
  // F_l = tanh(E_l . T + b)
  f4 f[2][4];
#pragma unroll
  for (int l = 0; l < 2; ++l) {
    wq_put_acc(wa, l == 0 ? e0 : e1);
    wave_lds_sync();
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) f[l][cb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const float ax = wa[wq_o(4 * s + ak, ar)];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) f[l][cb] = mfma16(ax, wi[W_IT + (cb * 16 + s) * 64 + lane], f[l][cb]);
    }
    wave_lds_sync();
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const float b = wi[W_ITB + 16 * cb + ar];
#pragma unroll
      for (int r = 0; r < 4; ++r) f[l][cb][r] = tanhf(f[l][cb][r] + b);
    }
  }
  WQTS(0);  // tanh GEMM
  // gate dot products per row: kind 0 F0F0, 1 F1F1, 2 F0F1 (the product rounded, then the
  // lw-weighted FMA chain over the columns in order)
  float dk[3];
#pragma unroll
  for (int kind = 0; kind < 3; ++kind) {
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        wa[wq_o(16 * cb + ar, 4 * ak + r)] = f[kind == 1 ? 1 : 0][cb][r] * f[kind == 0 ? 0 : 1][cb][r];
    wave_lds_sync();
    float a = 0.f;
    if (lane < TILE) {
#pragma unroll
      for (int h = 0; h < 64; h += 32) {
        float xv[32], wv[32];
#pragma unroll
        for (int c = 0; c < 32; ++c) {
          xv[c] = wa[wq_o(h + c, lane)];
          wv[c] = wi[W_ILW + h + c];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < 32; ++c) a = fmaf(xv[c], wv[c], a);
      }
    }
    dk[kind] = a;
    wave_lds_sync();
  }
  const float lb = wi[W_ILB];
  const float g0 = other_gate(0, dk[0], dk[1], dk[2], lb), g1 = other_gate(1, dk[0], dk[1], dk[2], lb);
  WQTS(1);  // dots + gates
  // E'_l = F_l + g_l F_other (mul then add), normalised
  f4 m[2][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const float ga = __shfl(g0, 4 * ak + r, 64), gb = __shfl(g1, 4 * ak + r, 64);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      m[0][cb][r] = f[0][cb][r] + ga * f[1][cb][r];
      m[1][cb][r] = f[1][cb][r] + gb * f[0][cb][r];
    }
  }
  wq_norm_rows(wa, m[0]);
  wq_norm_rows(wa, m[1]);
  WQTS(2);  // mix + norm
  const float cpl = wi[W_ICP + lane];
  // per layer: e = sum_b (h y_b) cp_b as the hidden layer's A operands, then relu(e . H1)
  f4 hid[2][2];
#pragma unroll
  for (int l = 0; l < 2; ++l) {
    wq_put_acc(wa, m[l]);
    wave_lds_sync();
    typedef float f2v __attribute__((ext_vector_type(2)));
    f2v h[8], acc[8];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      h[s >> 1][s & 1] = wa[wq_o(4 * s + ak, ar)];
      acc[s >> 1][s & 1] = 0.f;
    }
    wave_lds_sync();
    // {y_b, cp_b} pairs in WA, read by every lane at one address (an LDS broadcast), four b per
    // 2 x 16-byte read issued one block ahead; per b the eight products first (independent),
    // then the eight FMAs
    wa[2 * lane] = yv[l];
    wa[2 * lane + 1] = cpl;
    wave_lds_sync();
    const float4* yc = (const float4*)wa;
    auto term = [&](float y, float c) {
      const f2v yy = {y, y}, cc = {c, c};
      f2v t[8];
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) t[k2] = h[k2] * yy;
#pragma unroll
      for (int k2 = 0; k2 < 8; ++k2) acc[k2] = __builtin_elementwise_fma(t[k2], cc, acc[k2]);
    };
    float4 n0 = yc[0], n1 = yc[1];
#pragma unroll 2
    for (int bb = 0; bb < 64; bb += 4) {
      const float4 c0 = n0, c1 = n1;
      if (bb + 4 < 64) {
        n0 = yc[(bb + 4) / 2];
        n1 = yc[(bb + 4) / 2 + 1];
      }
      term(c0.x, c0.y);
      term(c0.z, c0.w);
      term(c1.x, c1.y);
      term(c1.z, c1.w);
    }
    wave_lds_sync();
#pragma unroll
    for (int cb = 0; cb < 2; ++cb) {
      hid[l][cb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 16; ++s) hid[l][cb] = mfma16(acc[s >> 1][s & 1], wi[W_IH1 + (cb * 16 + s) * 64 + lane], hid[l][cb]);
    }
  }
  WQTS(4);  // e-chain + hidden GEMM
  // Q head per (layer, row): relu(hidden) . w2[0..31] then the aux terms, as one FMA chain
  float* hq = wa;  // [2][16][33] (WA and WL: the lists are dead here)
#pragma unroll
  for (int l = 0; l < 2; ++l)
#pragma unroll
    for (int cb = 0; cb < 2; ++cb)
#pragma unroll
      for (int r = 0; r < 4; ++r) hq[(l * 16 + 4 * ak + r) * 33 + 16 * cb + ar] = fmaxf(hid[l][cb][r], 0.f);
  wave_lds_sync();
  float ql = 0.f;
  {
    const int ll = (lane >> 4) & 1, row = lane & 15;
    float a = fma_chain<32>(0.f, 0, [&](int k) { return hq[(ll * 16 + row) * 33 + k]; },
                            [&](int k) { return wi[W_IW2 + k]; });
#pragma unroll
    for (int k = 0; k < 4; ++k) a = fmaf(__shfl(gsv, 4 + ll * 4 + k, 64), wi[W_IW2 + 32 + k], a);
    ql = a;
  }
  wave_lds_sync();
  WQTS(5);  // Q head
  const float q1 = __shfl(ql, 16 + (lane & 15), 64);
  const float w0 = __shfl(gsv, 0, 64), w1 = __shfl(gsv, 1, 64);
  float bm = NEG_INF, bs = NEG_INF;
  int bi = 0x7fffffff, bc = 0;
  if (lane < TILE && vrow >= 0) {
    const float qq = w0 * ql + w1 * q1;
    stc(p.q + gi.node_off + vrow, qq);
    bm = qq;
    bi = vrow;
    bc = 1;
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(bm, o, 64), s2 = __shfl_xor(bs, o, 64);
    const int i2 = __shfl_xor(bi, o, 64), c2 = __shfl_xor(bc, o, 64);
    if (c2 != 0) argmax_combine(bm, bs, bi, bc, m2, s2, i2, c2);
  }
  if (lane == 0) stc4(p.apart + (size_t)(gi.tile_off + j) * 4, 0, make_float4(bm, bs, __int_as_float(bi), __int_as_float(bc)));
  WQTS(6);  // q, arg-max partial, stores
}

// Work item TILE(it, j) of graph g (slot gl) on one wave: both layers, then (it == 3) the
// attention and Q head.
__device__ __forceinline__ void wq_tile(KParams&, int g, int gl, int it, int j) {
  KParams& p = kp();
  const int lane = wq_lane();
  WQTS_INIT(it);
  float* const wa = wq_area() + WQ_WA;
  lds_u16* const wl = (lds_u16*)(uint16_t*)(wq_area() + WQ_WL);
  const GraphInfo gi = p.ginfo[g];
  // rows (live list), the cached alive-neighbour lists' header and flag, one round trip
  const int nl = wq_uni(ldc(&p.gvar[g].n_live));
  const int npred = it == 3 ? wq_uni(ldc(&p.gvar[g].npred)) : 0;  // the head granules' tag - 1
  int vrow = -1;
  if (lane < TILE) {
    const int r = j * TILE + lane;
    const float4 e = ldc4((const float*)(p.live + 4 * (size_t)gi.node_off), min(r, gi.n - 1) * 16);
    const int v = __float_as_int(e.x);
    if (r < nl && MD_BOK(v >= 0 && v < gi.n && nl <= gi.n, 6)) vrow = v;
  }
  const int slot = p.gtoff[gl] + j;
  const bool cacheable = slot < p.nbc_slots;
  int hdw = 0, hdx = 0, built = 0;
  const int* hd = p.nbc + (size_t)slot * NBC_INTS;
  // the first WQ_SPEC_WORDS list words of each layer go out with the header (the lists' lengths
  // are not known yet; longer lists load the rest after it)
  constexpr int NS = WQ_SPEC_WORDS / 64;
  int w0[NS], w1[NS];
  if (cacheable) {
    hdw = ldc(hd + lane);
    if (lane < 3) hdx = ldc(hd + 64 + lane);
    built = ldc(p.qg + 2 * QG_CAP + gl);
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      w0[u] = ldc(hd + NBC_HDR + lane + 64 * u);
      w1[u] = ldc(hd + NBC_HDR + NBC_LWORDS + lane + 64 * u);
    }
  }
  const int nv = __popcll(__ballot(lane < TILE && vrow >= 0));
  built = wq_uni(built);
  const int tot0 = __shfl(hdx, 0, 64), tot1 = __shfl(hdx, 1, 64), okf = __shfl(hdx, 2, 64);
  const bool ok = cacheable && built != 0 && okf != 0;
  const bool listed0 = ok && tot0 <= WQ_LIST_MAX, listed1 = ok && tot1 <= WQ_LIST_MAX;
  // both layers' list entries (packed two per int) into WL
  {
    const int nw0 = listed0 ? (tot0 + 1) >> 1 : 0, nw1 = listed1 ? (tot1 + 1) >> 1 : 0;
    lds_i32* ww = (lds_i32*)(int*)(wq_area() + WQ_WL);
#pragma unroll
    for (int u = 0; u < NS; ++u) {
      const int i = lane + 64 * u;
      if (i < nw0) ww[i] = w0[u];
      if (i < nw1) ww[WQ_LIST_MAX / 2 + i] = w1[u];
    }
    if (nw0 > WQ_SPEC_WORDS || nw1 > WQ_SPEC_WORDS) {
      for (int i = WQ_SPEC_WORDS + lane; i < max(nw0, nw1); i += 64) {
        if (i < nw0) ww[i] = ldc(hd + NBC_HDR + i);
        if (i < nw1) ww[WQ_LIST_MAX / 2 + i] = ldc(hd + NBC_HDR + NBC_LWORDS + i);
      }
    }
    wave_lds_sync();
  }
  // own-row sources of both layers; unit cost, iteration 1: rows and list entries by residual
  // degree (the entries of both lists resolved in one round trip)
  bool table;
  const float* hp0 = wq_src(p, gi, it, 0, table);
  const float* hp1 = wq_src(p, gi, it, 1, table);
  int vs0 = vrow, vs1 = vrow;
  if (table && lane < TILE && vrow >= 0) {
    vs0 = ldc(p.deg[0] + gi.node_off + vrow);
    vs1 = ldc(p.deg[1] + gi.node_off + vrow);
  }
  float xa0[16], xa1[16];
  wq_xload(hp0, __shfl(vs0, lane & 15, 64), xa0);
  if (table && (listed0 || listed1)) {
    const int* dg0 = p.deg[0] + gi.node_off;
    const int* dg1 = p.deg[1] + gi.node_off;
    lds_u16* w1 = wl + WQ_LIST_MAX;
    const int t0 = listed0 ? tot0 : 0, t1 = listed1 ? tot1 : 0;
    for (int i0 = 0; i0 < max(t0, t1); i0 += 128) {
      int d0[2], d1[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = i0 + lane + 64 * u;
        d0[u] = i < t0 ? ldc(dg0 + (int)wl[i]) : 0;
        d1[u] = i < t1 ? ldc(dg1 + (int)w1[i]) : 0;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = i0 + lane + 64 * u;
        if (i < t0) wl[i] = (uint16_t)d0[u];
        if (i < t1) w1[i] = (uint16_t)d1[u];
      }
    }
    wave_lds_sync();
  }
  f4 e0[4], e1[4];
  WQTS(0);  // header, rows, lists (and their first-layer rows)
  wq_layer_front(p, gi, it, j, 0, vrow, nv, hdw, tot0, listed0, wa, wl, xa0);
  wq_xload(hp1, __shfl(vs1, lane & 15, 64), xa1);  // (arrives under layer 0's update)
  wq_layer_back(p, gi, it, j, 0, vrow, nv, wa, xa0, e0);
  wq_layer_front(p, gi, it, j, 1, vrow, nv, hdw, tot1, listed1, wa, wl + WQ_LIST_MAX, xa1);
  wq_layer_back(p, gi, it, j, 1, vrow, nv, wa, xa1, e1);
  if (it == 3) {
    WQTS_RESET();
    wq_attention(p, gi, g, j, vrow, e0, e1, wa, (unsigned)npred + 1u);
    WQTS(6);  // attention + Q head
  }
}

// ------------------------------------------------------------------ one wave's virtual node
// graph_sum of slot k on one wave: lane c adds both layers' column c (outputs c, 64 + c), four
// quarters of the tiles each in order, then the quarters in order.
__device__ __forceinline__ void wq_graph_sum(KParams& p, const GraphInfo& gi, int nt, int k, float& s0, float& s1) {
  const int lane = wq_lane();
  const float* sp = p.spart + (size_t)gi.tile_off * 384 + k * 128 + lane;
  const int per = (nt + 3) >> 2;
  float part[2][4];
#pragma unroll
  for (int qt = 0; qt < 4; ++qt) {
    part[0][qt] = 0.f;
    part[1][qt] = 0.f;
  }
  for (int jb = 0; jb < per; jb += 8) {
    float x[4][2][8];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      const int j0 = min(nt, qt * per), j1 = min(nt, j0 + per);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int jj = j0 + jb + u;
        x[qt][0][u] = jj < j1 ? ldc(sp + (size_t)jj * 384) : 0.f;
        x[qt][1][u] = jj < j1 ? ldc(sp + (size_t)jj * 384 + 64) : 0.f;
      }
    }
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      const int j0 = min(nt, qt * per), j1 = min(nt, j0 + per);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (j0 + jb + u < j1) {
          part[0][qt] = part[0][qt] + x[qt][0][u];
          part[1][qt] = part[1][qt] + x[qt][1][u];
        }
    }
  }
  s0 = ((part[0][0] + part[0][1]) + part[0][2]) + part[0][3];
  s1 = ((part[1][0] + part[1][1]) + part[1][2]) + part[1][3];
}

// vrow_update on one wave: y' = normalize(relu([s.P1 | y.P2] . P3)) for both layers, each
// output column's chains split in vrow_update's four partial chains, summed in order.
__device__ __forceinline__ void wq_vrow(float s0, float s1, float& y0, float& y1, float* wa) {
  const int c = wq_lane();
  const float* wi = lds_base() + L_W;
  wa[c] = s0;
  wa[64 + c] = s1;
  wa[128 + c] = y0;
  wa[192 + c] = y1;
  wave_lds_sync();
#pragma unroll
  for (int l = 0; l < 2; ++l) {
    float p1[4], p2[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      p1[q] = fma_chain<16>(0.f, 16 * q, [&](int k) { return wa[l * 64 + k]; }, [&](int k) { return wget(wi + W_IP1, 16, k, c); });
      p2[q] = fma_chain<16>(0.f, 16 * q, [&](int k) { return wa[128 + l * 64 + k]; },
                            [&](int k) { return wget(wi + W_IP2, 16, k, c); });
    }
    wa[256 + l * 128 + c] = ((p1[0] + p1[1]) + p1[2]) + p1[3];
    wa[256 + l * 128 + 64 + c] = ((p2[0] + p2[1]) + p2[2]) + p2[3];
  }
  wave_lds_sync();
#pragma unroll
  for (int l = 0; l < 2; ++l) {
    float p3[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      p3[q] = fma_chain<32>(0.f, 32 * q, [&](int k) { return wa[256 + l * 128 + k]; },
                            [&](int k) { return wget(wi + W_IP3, 32, k, c); });
    float o = ((p3[0] + p3[1]) + p3[2]) + p3[3];
    o = fmaxf(o, 0.f);
    const float nr = wave_norm64(o);
    (l == 0 ? y0 : y1) = o / fmaxf(nr, 1e-12f);
  }
  wave_lds_sync();
}

// Virtual-node item of graph g on one wave: part 1 Y1, Y2 from S0, S1 (stored to ybuf); part 2
// Y3 from S2, then graph_head (y, layer-mix weights, aux features) published as the head
// granules (tag: the graph's predictions so far + 1) for the iteration-3 tiles.
__device__ __forceinline__ void wq_vn(KParams&, int g, int part) {
  KParams& p = kp();
  const int lane = wq_lane();
  float* const wa = wq_area() + WQ_WA;
  const float* wi = lds_base() + L_W;
  const GraphInfo gi = p.ginfo[g];
  const int nl = wq_uni(ldc(&p.gvar[g].n_live));
  const int npred = part == 2 ? wq_uni(ldc(&p.gvar[g].npred)) : 0;
  const int nt = (nl + TILE - 1) / TILE;
  float y0, y1;
  if (part == 1) {
    y0 = y1 = lds_base()[L_Y0 + lane];
  } else {
    y0 = ldc(p.ybuf + (size_t)g * 128 + lane);
    y1 = ldc(p.ybuf + (size_t)g * 128 + 64 + lane);
  }
  for (int k = part == 1 ? 0 : 2; k < (part == 1 ? 2 : 3); ++k) {
    float s0, s1;
    wq_graph_sum(p, gi, nt, k, s0, s1);
    wq_vrow(s0, s1, y0, y1, wa);
  }
  if (part == 1) {
    stc(p.ybuf + (size_t)g * 128 + lane, y0);
    stc(p.ybuf + (size_t)g * 128 + 64 + lane, y1);
    return;
  }
  // graph head (graph_head's chains)
  wa[lane] = y0;
  wa[64 + lane] = y1;
  wave_lds_sync();
  float fl[2];
#pragma unroll
  for (int l = 0; l < 2; ++l) {
    const float a = fma_chain<64>(0.f, 0, [&](int k) { return wa[l * 64 + k]; }, [&](int k) { return wget(wi + W_IT, 16, k, lane); });
    fl[l] = tanhf(a + wi[W_ITB + lane]);
  }
  wa[128 + lane] = fl[0];
  wa[192 + lane] = fl[1];
  wave_lds_sync();
  float dt = 0.f;
  if (lane < 3) {
    const float* fa = wa + 128 + (lane == 1 ? 64 : 0);
    const float* fb = wa + 128 + (lane == 0 ? 0 : 64);
    dt = fma_chain<64>(0.f, 0, [&](int c) { return fa[c] * fb[c]; }, [&](int c) { return wi[W_ILW + c]; });
  }
  const float d00 = __shfl(dt, 0, 64), d11 = __shfl(dt, 1, 64), d01 = __shfl(dt, 2, 64);
  float ys[2];
#pragma unroll
  for (int l = 0; l < 2; ++l) {
    const float gg = other_gate(l, d00, d11, d01, wi[W_ILB]);
    const float m = fl[l] + gg * fl[1 - l];
    const float nr = wave_norm64(m);
    ys[l] = m / fmaxf(nr, 1e-12f);
  }
  wave_lds_sync();
  wa[256 + lane] = ys[0];
  wa[320 + lane] = ys[1];
  wave_lds_sync();
  // zh[ll][j] = relu(ys_ll . WL1[:, j]), j = lane, 64 + lane (w_layer1 read from the weights)
  float zh[2][2];
  {
    const float* wl1 = p.w + W_WL1;
    float wv[2][64];
#pragma unroll
    for (int k = 0; k < 64; ++k) {
      wv[0][k] = wl1[k * 128 + lane];
      wv[1][k] = wl1[k * 128 + 64 + lane];
    }
#pragma unroll
    for (int ll = 0; ll < 2; ++ll)
#pragma unroll
      for (int jh = 0; jh < 2; ++jh) {
        float a = 0.f;
#pragma unroll
        for (int k = 0; k < 64; ++k) a = fmaf(wa[256 + ll * 64 + k], wv[jh][k], a);
        zh[ll][jh] = fmaxf(a, 0.f);
      }
  }
#pragma unroll
  for (int ll = 0; ll < 2; ++ll) {
    wa[384 + ll * 128 + lane] = zh[ll][0];
    wa[384 + ll * 128 + 64 + lane] = zh[ll][1];
  }
  wave_lds_sync();
  float z = 0.f;
  if (lane < 2)
    z = fma_chain<128>(0.f, 0, [&](int jj) { return wa[384 + lane * 128 + jj]; }, [&](int jj) { return wi[W_IWL2 + jj]; });
  const float z0 = __shfl(z, 0, 64), z1 = __shfl(z, 1, 64);
  const float mz = fmaxf(z0, z1);
  const float ex0 = expf(z0 - mz), ex1 = expf(z1 - mz);
  const float inv = 1.f / (ex0 + ex1);
  // graph scalars: mix weights, aux features (graph_aux), published with y
  float gsv = 0.f;
  if (lane == 0) gsv = ex0 * inv;
  if (lane == 1) gsv = ex1 * inv;
  if (lane >= 4 && lane < 12) {
    const int ll = (lane - 4) >> 2, k = (lane - 4) & 3;
    const double N = (double)gi.n;
    const GraphVar* gvp = p.gvar + g;
    if (k == 0) gsv = (float)((double)ldc(&gvp->n_cov) / N);
    else if (k == 1) gsv = (float)((double)ldc(&gvp->counter[ll]) / (double)(ll == 0 ? gi.e[0] : gi.e[1]));
    else if (k == 2) {
      const long long th = __hip_atomic_load((const __attribute__((address_space(1))) long long*)&gvp->twohop[ll],
                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      gsv = (float)((double)th / (N * N));
    } else gsv = 1.0f;
  }
  wave_lds_sync();
  g_u64* hb = (g_u64*)(p.hbuf + 2 * ((size_t)g * HB_FLOATS));
  const unsigned long long tag = (unsigned long long)((unsigned)npred + 1u) << 32;
  __hip_atomic_store(hb + lane, tag | (unsigned)__float_as_uint(ys[0]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(hb + 64 + lane, tag | (unsigned)__float_as_uint(ys[1]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (lane < 16)
    __hip_atomic_store(hb + 128 + lane, tag | (unsigned)__float_as_uint(gsv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ------------------------------------------------------------------ group section (ENV items)
// The environment step of queued item `item` on the whole workgroup: queue_loop's ENV branch
// (phase A, tail park, this step's neighbour lists, the iteration-1 tiles pushed one per item).
__device__ void wq_env(KParams& p, float* lds, unsigned item) {
  int* misc = (int*)(lds + L_MISC);
  int* bc = misc + 48;
  const int ng = p.nglist;
  const int it = (int)((item >> 3) & 3u), gl = q_item_gl(item);
  const int g = p.glist[gl];
  if (it == 2) {  // batch speculation: the next step's fixed point for the candidate
    bspec_step(p, gl, q_item_j(item));
    return;
  }
  if (threadIdx.x == 0) {
    wq_event(p, gl, 0);
    misc[20] = -1;  // (env_step sets the candidate)
  }
  WQTE_INIT();
  // the tail-park test's words, read before phase A instead of after it (both only move toward
  // parking -- QC_REM down, QC_ADMIT up -- so an early read parks no graph too soon)
  int padm = 0, prem = 0x7fffffff;
  const bool ptest = p.qpark > 0 && ng > p.qpark;
  if (ptest && threadIdx.x == 0) {
    padm = ldc((const int*)(p.qctl + QC_ADMIT));
    prem = ldc((const int*)(p.qctl + QC_REM));
  }
  const bool lds_env = phase_a(p, g, it != 0, lds, false);
  WQTE(0);  // phase A
  const GraphVar& gv = *(const GraphVar*)(lds + L_GV);
  const int st = gv.status, nl = gv.n_live;
  __syncthreads();
  if (st == ST_RUN && nl <= 0) {
    if (threadIdx.x == 0) raise_err(p, ERR_LIVE_MISMATCH);
    return;
  }
  bool park = false;
  if (st == ST_RUN && ptest) {
    if (threadIdx.x == 0) bc[6] = padm >= ng && prem <= p.qpark;
    __syncthreads();
    park = bc[6] != 0;
  }
  WQTE(1);  // park check
  if (st == ST_RUN && !park) {
    const int nt = (nl + TILE - 1) / TILE;
    // batch speculation: the slot words of the new state's parity (the loads' round trip
    // overlaps the neighbour lists), then the claim
    const bool bsp = p.bspec != nullptr && lds_env;
    unsigned long long bst = 0ull;
    unsigned bex = 1u;
    if (bsp && threadIdx.x == 0) {
      const int* sl = bspec_slot(p, p.ginfo[g], gv.steps);
      bst = __hip_atomic_load((const g_u64*)(sl + SRES_STARTED), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      bex = (unsigned)ldc(sl + BSPEC_EXITED);
    }
    const bool built = lds_env && env_build_lists(p, p.ginfo[g], gl);
    WQTE(2);  // neighbour lists
    if (threadIdx.x == 0) {
      stc(p.qg + 2 * gl + 1, nt | (nt << 16) | (1 << 28));
      stc(p.qg + 2 * QG_CAP + gl, built ? 1 : 0);
      misc[21] = bsp && !(p.variant & 0x4000) && bspec_claim(p, p.ginfo[g], gv.steps, misc[20], bst, bex) ? 1 : 0;
    }
    __syncthreads();
    const int ns = misc[21], steps = gv.steps;
    q_push(p, nt + ns, [&](int i) { return i < nt ? q_item(QK_TILE, 1, gl, i) : bspec_item(gl, steps); }, bc);
    if (threadIdx.x == 0) wq_event(p, gl, 5);
    WQTE(3);  // stage word, push
  } else if (st == ST_WAIT_HOST) {
    q_push(p, 1, [&](int) { return q_item(QK_ENV, 1, gl, 0); }, bc);  // poll again later
  } else {
    if (threadIdx.x == 0) {
      bc[2] = (int)__hip_atomic_fetch_add((g_u32*)(p.qctl + QC_REM), 0xffffffffu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int a;
      while ((a = (int)__hip_atomic_fetch_add((g_u32*)(p.qctl + QC_ADMIT), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) <
                 ng &&
             ldc(&p.gvar[p.glist[a]].status) != ST_RUN) {
      }
      bc[4] = a < ng ? a : -1;
    }
    __syncthreads();
    if (bc[4] >= 0) q_push(p, 1, [&](int) { return q_item(QK_ENV, 0, bc[4], 0); }, bc);
    // two EXIT items per wave of the launch (a wave may hold one ticket it never uses)
    if (bc[2] == 1) q_push(p, 2 * WQ_WAVES * gridDim.x, [&](int) { return (unsigned)QK_EXIT; }, bc);
  }
}

// Every wave of the workgroup: run the queued ENV items together, reload the weight image.
__device__ __noinline__ void wq_group(KParams&, const float* __restrict__ wimg) {
  KParams& p = kp();
  float* const lds = lds_base();
  __syncthreads();
  volatile int* ctl = wq_ctl();
  const int n = ctl[WQC_REQ];
  unsigned items[WQ_WAVES];
#pragma unroll
  for (int i = 0; i < WQ_WAVES; ++i) items[i] = (unsigned)ctl[WQC_ITEMS + i];
  unsigned long long* qp = p.prof;
  const unsigned long long t0 = wall_clock64();
  __syncthreads();
  const bool err = (__hip_atomic_load((g_u32*)p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & BAR_ERR) != 0;
  __syncthreads();
  if (!err) {
    for (int i = 0; i < n && i < WQ_WAVES; ++i) wq_env(p, lds, items[i]);
    WQTE_INIT();
    load_weights(lds + L_W, wimg);
    __syncthreads();
    WQTE(4);  // weight reload
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    ctl[WQC_REQ] = 0;
    if (qp != nullptr) {
      atomicAdd(qp + QK_ENV, wall_clock64() - t0);
      atomicAdd(qp + 8 + QK_ENV, (unsigned long long)n);
    }
  }
  __syncthreads();
}

// ------------------------------------------------------------------ the loop
__device__ __forceinline__ void wq_loop(KParams&, const float* __restrict__ wimg) {
  KParams& p = kp();
  float* const lds = lds_base();
  int* misc = (int*)(lds + L_MISC);
  int* bc = misc + 48;
  volatile int* ctl = wq_ctl();
  const int ng = p.nglist;
  if (threadIdx.x == 0) {
    ctl[WQC_REQ] = 0;
    ctl[WQC_DONE] = 0;
    misc[60] = 1 << 30;  // no per-step phase stamps in queue mode
  }
  if (blockIdx.x == 0) {
    // queue_loop's start: the running graphs in slot order, the first q_admit of them
    int* run = (int*)(lds + L_SCR + S_M);
    int tot = 0;
    for (int base = 0; base < ng; base += NTHREADS) {
      const int s = base + (int)threadIdx.x;
      const int mine = s < ng && ldc(&p.gvar[p.glist[s]].status) == ST_RUN;
      int cnt = 0;
      const int at = block_excl_scan(mine, (int*)(lds + L_SCR + S_RED), &cnt);
      if (mine) run[tot + at] = s;
      tot += cnt;
      __syncthreads();
    }
    // admission: every wave of the chip runs its own items, so more graphs run at once than in
    // md_queue_kernel: up to two per workgroup (sweep over 4096 graphs: 160 / 512 / 1024 / all ->
    // 366 / 265 / 271 / 281 ms), one per workgroup when no more than two per workgroup wait
    // (512 graphs, the C5 shard at world 8: 256 / 384 / 512 admitted -> 37.2 / 37.8 / 38.0 ms;
    // 256 graphs: 128 / 192 / 256 -> 26.4 / 25.0 / 24.8 ms); MD_VARIANT bits 16+ override
    const int vadm = (int)((unsigned)p.variant >> 16);
    const int grid = (int)gridDim.x;
    const int first = min(tot, vadm > 0 ? vadm : (tot > 2 * grid ? 2 * grid : grid));
    if (threadIdx.x == 0) {
      __hip_atomic_store((g_u32*)(p.qctl + QC_REM), (unsigned)tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((g_u32*)(p.qctl + QC_ADMIT), (unsigned)(first < tot ? run[first] : ng), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (tot > 0) q_push(p, first, [&](int i) { return q_item(QK_ENV, 0, run[i], 0); }, bc);
    else q_push(p, 2 * WQ_WAVES * gridDim.x, [&](int) { return (unsigned)QK_EXIT; }, bc);
  }
  __syncthreads();
  // diagnostics (md_profile): per item kind device ticks and counts summed over waves in
  // prof[kind] / prof[8 + kind] (ENV: group sections), waiting ticks in prof[16]
  unsigned long long* qp = p.prof;
  if (qp != nullptr && blockIdx.x == 0 && threadIdx.x == 0) qp[0] = 1;
  const int lane = lane_id();
  unsigned tk = wq_take(p);
  unsigned long long pre = 0ull;
  unsigned cont = 0u;
  bool done = false;
  unsigned long long tq = wall_clock64();
  const unsigned long long tq0 = tq;
  while (true) {
    // (a held continuation runs first: the iteration-3 tiles of its graph, maybe a wave of this
    // workgroup among them, wait for part 2's head granules and would never reach the group's
    // barrier)
    if (ctl[WQC_REQ] != 0 && cont == 0u) {
      wq_group(p, wimg);
      continue;
    }
    if (done) {
      if (ctl[WQC_DONE] == WQ_WAVES) break;
      __builtin_amdgcn_s_sleep(4);
      continue;
    }
    unsigned item;
    if (cont != 0u) {
      item = cont;
      cont = 0u;
    } else {
      item = wq_wait(p, tk, pre);
      if (item == WQ_GROUP) continue;
      pre = 0ull;
      tk = wq_take(p);
    }
    const unsigned kind = item & 7u;
    unsigned long long ti = 0;
    if (qp != nullptr && lane == 0) {
      ti = wall_clock64();
      atomicAdd(qp + 16, ti - tq);
      // waiting ticks over the launch in 1.31 ms buckets (slots 20..63; with MD_VARIANT bit 8
      // those slots hold the item pieces instead)
      if (!(p.variant & 8)) atomicAdd(qp + 20 + min(43, (int)((ti - tq0) >> 17)), ti - tq);
    }
    if (kind == QK_EXIT || kind == 0u) {
      done = true;
      if (lane == 0) __hip_atomic_fetch_add((int*)(ctl + WQC_DONE), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      continue;
    }
    if (kind == QK_ENV) {
      if (lane == 0) wq_event(p, q_item_gl(item), 6);
      if (lane == 0) {
        const int s = __hip_atomic_fetch_add((int*)(ctl + WQC_REQ), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        ctl[WQC_ITEMS + s] = (int)item;
      }
      wave_lds_sync();
      tq = wall_clock64();
      continue;
    }
    const int it = (int)((item >> 3) & 3u), gl = q_item_gl(item), j = q_item_j(item);
    const int g = p.glist[gl];
    int next = 0;
    if (kind == QK_TILE || it == 1) {
      if (kind == QK_TILE) wq_tile(p, g, gl, it, j);
      else wq_vn(p, g, 1);
      const int stage = kind == QK_TILE ? it : 2;
      pre = wq_peek(p, tk);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's outputs are stored
      int nx = 0;
      if (lane == 0) {
        const int tasks = (ldc(p.qg + 2 * gl + 1) & 0xffff) + (stage == 2 ? 1 : 0);
        const int old = __hip_atomic_fetch_add(p.qg + 2 * gl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == tasks - 1) {
          stc(p.qg + 2 * gl, 0);
          nx = stage;
        }
      }
      next = wq_uni(nx);
    } else {  // QK_VN part 2
      wq_vn(p, g, 2);
      pre = wq_peek(p, tk);
      // (the iteration-3 tiles went out with this item; MD_VARIANT bit 12: after it)
      next = (p.variant & 4096) ? 4 : 0;
      if (!(p.variant & 4096) && lane == 0) wq_event(p, gl, 4);
    }
    if (next != 0) {
      if (lane == 0) wq_event(p, gl, next);
      const int nt = (wq_uni(ldc(p.qg + 2 * gl + 1)) >> 16) & 0xfff;
      if (next == 1) {
        wq_push(p, nt + 1, [&](int i) { return i < nt ? q_item(QK_TILE, 2, gl, i) : q_item(QK_VN, 1, gl, 0); });
      } else if (next == 2) {
        // the iteration-3 tiles now: their layer pieces need only the iteration-2 rows, and
        // their attention waits for this step's head granules, which part 2 publishes
        if (!(p.variant & 4096)) wq_push(p, nt, [&](int i) { return q_item(QK_TILE, 3, gl, i); });
        cont = q_item(QK_VN, 2, gl, 0);
      } else if (next == 3) {
        cont = q_item(QK_ENV, 1, gl, 0);
      } else {
        wq_push(p, nt, [&](int i) { return q_item(QK_TILE, 3, gl, i); });
      }
    }
    if (qp != nullptr && lane == 0) {
      tq = wall_clock64();
      const int slotk = kind == QK_TILE ? 4 + it : kind == QK_VN ? 2 + it : (int)kind;
      atomicAdd(qp + slotk, tq - ti);
      atomicAdd(qp + 8 + (int)kind, 1ull);
    } else {
      tq = wall_clock64();
    }
  }
}

__global__ void __launch_bounds__(NTHREADS, 1) md_wq_kernel(Params p, const float* __restrict__ wimg) {
  if (!kargs_layout_ok()) {
    if (threadIdx.x == 0) __hip_atomic_store(p.err, ERR_ABI, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  extern __shared__ __attribute__((aligned(16))) float lds[];
  KParams& kpp = kp();
  load_weights(lds + L_W, wimg);
  __syncthreads();
  if (wave_id() == 0) {
    // constant virtual-node input: normalize(relu([1,1] . w_n2l))  (net :247,272-283)
    const int lane = lane_id();
    const float x = fmaxf(fmaf(1.f, lds[L_W + W_IWN + 64 + lane], fmaf(1.f, lds[L_W + W_IWN + lane], 0.f)), 0.f);
    const float nr = wave_norm64(x);
    lds[L_Y0 + lane] = x / fmaxf(nr, 1e-12f);
  }
  __syncthreads();
  wq_loop(kpp, wimg);
  kernel_exit(kpp);
}
