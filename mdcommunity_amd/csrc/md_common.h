// md_common.h — structures shared by the host ABI (md_abi.cpp) and the gfx950 kernels
// (md_kernels.hip) of libmdroll.so.  Everything lives in device memory, laid out as flat
// arrays over all loaded graphs (graph g's nodes at [node_off, node_off+n), its layer-l
// undirected edges at [eoff[l], eoff[l]+e[l]), its CSR entries at [coff[l], coff[l]+2e[l]),
// its 16-row tiles at [tile_off, tile_off + ceil(n/16))).
#pragma once
#include <stdint.h>

namespace md {

constexpr int EMB = 64;          // EMBEDDING_SIZE, U/MultiDismantler_torch.py:36
constexpr int REG_HIDDEN = 32;   // REG_HIDDEN, :57
constexpr int AUX_DIM = 4;       // aux_dim, :64
constexpr int BP_ITERS = 3;      // max_bp_iter, :62
constexpr int NTHREADS = 512;    // 8 waves: waves 0-3 work on layer 0, waves 4-7 on layer 1
constexpr int TILE = 16;         // node rows per MFMA tile (v_mfma_f32_16x16x4_f32)
constexpr int G_CAP = 512;       // graphs per kernel launch (the host chunks larger batches)
// queue-mode launches (whole-batch rollouts) take up to QG_CAP graphs: a work item holds a
// 12-bit graph slot and a 13-bit first tile (graphs of < Q_MAX_TILES tiles; a batch with a
// larger graph runs in the lock-step kernel)
constexpr int QG_CAP = 4096;
constexpr int Q_MAX_TILES = 8192;
constexpr int PROF_SLOTS = 96;
constexpr int NB_CAP_ENTRIES = 2052;   // alive neighbour entries per layer kept for a tile (NB_CAP)
// neighbour-list cache slot: header (off[2][16], cnt[2][16], tot[2], ok) then per layer the u16
// entries packed two per int
constexpr int NBC_HDR = 80, NBC_LWORDS = NB_CAP_ENTRIES / 2, NBC_INTS = 2176;
static_assert(NBC_HDR + 2 * NBC_LWORDS <= NBC_INTS, "cache slot");
constexpr int XB_SLOTS = 256;
constexpr int TEAM_MAX_WG = 1024;  // workgroups of a launch the grid-wide environment step supports
constexpr int Q_CAP = 1 << 18;   // queue-mode ring slots (items in flight << Q_CAP)

// Offsets (floats) of each tensor in the packed weight blob (see include/mdroll.h).
enum WOff : int {
  W_N2L = 0, W_P1 = 128, W_P2 = 4224, W_P3 = 8320, W_H1 = 16512, W_W2 = 18560, W_CP = 18596,
  W_WL1 = 18660, W_WL2 = 26852, W_T = 26980, W_TB = 31076, W_LW = 31140, W_LB = 31204,
  W_TOTAL = 31205
};

// Edge state (per undirected edge and layer).
enum : uint8_t { E_ALIVE = 0, E_COVERED = 1, E_PRUNED = 2 };

// Per-graph run status.
enum : int { ST_RUN = 0, ST_TERMINAL = 1, ST_NEED_HOST = 2, ST_PAUSED = 3, ST_WAIT_HOST = 4 };

// What a launch does with each graph.
enum : int { RUN_ROLLOUT = 0, RUN_PREDICT = 1, RUN_STEP = 2 };

// Row of degree d (1 <= d <= dm) in the precomputed first-layer tables: dmax dm's rows are
// contiguous, tables in ascending dmax.
__host__ __device__ inline long long h0g_row(int dm, int d) { return (long long)dm * (dm - 1) / 2 + (d - 1); }

struct GraphInfo {           // immutable after md_load_graphs
  int n;                     // nodes
  int node_off;              // into per-node arrays
  int e[2];                  // undirected edges per layer
  int eoff[2];               // into per-edge arrays
  int roff[2];               // into row-pointer arrays (n + 1 entries per graph)
  int coff[2];               // into CSR entry arrays (2 e entries per graph)
  int tile_off;              // into per-tile arrays (ceil(n / 16) tiles per graph)
  int gidx;                  // the graph's index (its GraphVar)
  int rank_off;              // into the static union ranks (even: read as u32 pairs)
};

struct GraphVar {            // mutable per-graph state
  int status;                // ST_*
  int s0_done;               // initial MCC prune done (MvcEnv.s0)
  int npend;                 // actions queued by the host (pend[node_off ..])
  int max_rank;              // LMCC after s0 (Graph_test.max_rank)
  int lmcc;                  // LMCC after the last step
  int n_cov;                 // covered nodes
  int n_live;                // nodes with an alive edge (compact list length)
  int steps;                 // removals applied since reset
  int npred;                 // predictions made since reset
  int dmax[2];               // max residual degree over live nodes
  int counter[2];            // numCoveredEdges (U/mvc_env.py:81-84)
  int removed[2];            // |remove_edge[l]| / 2
  int alive[2];              // alive edges
  long long twohop[2];       // sum over live nodes of C(deg, 2) (U/PrepareBatchGraph.py:62-72)
  int argmax;                // last prediction: best node (-1 when tied / none)
  int ntie;                  // last prediction: nodes tied at the max
  float qmax, gap;           // last prediction: best Q and top-2 gap
  int hdmax[2];              // dmax the unit-cost first-layer table was built for (0 = none)
  unsigned long long t_req;  // ST_WAIT_HOST: device wall clock of the pending host request
  int spec_hits;             // removals whose fixed point came from a speculative workgroup
};

// adjx packs a layer's CSR entries only below this many edges (positive words, never -1)
constexpr int ADJX_EDGE_LIMIT = 32768;

struct Params {
  const float* w;                  // packed weights (reference layout)
  const GraphInfo* ginfo;
  GraphVar* gvar;
  const int* rowptr[2];            // static CSR (neighbour order = reference in_edges order)
  const int* adj[2];
  const int* adjx[2];              // per CSR entry: (layer-local edge id << 16) | neighbour, packed only
                                   //   when e_l < ADJX_EDGE_LIMIT and n <= 2^16 (else -1): the word stays
                                   //   >= 0, the reader's liveness test (env_build_lists)
  uint8_t* calive[2];              // per CSR entry: 1 while its edge is alive
  const int* epos[2];              // per undirected edge: its two CSR entry positions
  const int* eu[2];                // undirected endpoints (graph-local ids)
  const int* ev[2];
  uint8_t* estate[2];
  uint8_t* covered;
  int* deg[2];                     // residual degree per node
  int* live;                       // compact ascending live-node list per graph: int4 {node,
                                   //   CSR begin layer 0, layer 1, extents l0 | l1 << 16}
  float* H[2][2];                  // [layer][buffer] node embeddings, node-major x 64
  float* h0tab[2];                 // [layer] first-layer embedding: by degree (unit) / by node (degree cost)
  float* q;                        // per node (-inf = masked)
  int* gscr;                       // phase-A scratch in global memory for graphs too big for LDS: GSCR_WORDS per node
  int* bspec;                      // queue launches: speculative environment-step results, two per graph
                                   // (removal-count parity), SRES layout (md_kernels.hip bspec_slot); nullptr = off
  long long bspec_half;            // ints per parity half
  int* gscr_team;                  // the grid-wide step's graph-local scratch (GSCR_TEAM_WORDS x the largest n):
                                   //   LMCC counts, second parent buffers, feature degrees, class labels
  long long* tpart;                // grid-wide environment step: per-workgroup partials [2][TEAM_MAX_WG][16]
  int* tctl;                       // grid-wide environment step: {actions (-1: none), first action}
  const uint16_t* prank;           // per node: static union rank (descending degree; team_env_step), or null
  int* lab_ok;                     // per graph: 1 while gscr's class labels and class sizes describe the
                                   //   current state (team_env_step keeps them; every other state change clears)
  float* spart;                    // per tile: [3 sums][2 layers][64] virtual-node partial sums
  float* apart;                    // per tile: arg-max partial {max, second, idx, count}
  float* ybuf;                     // per graph: [2][64] virtual-node embedding after iteration 2
  float* hbuf;                     // per graph: [144][2] graph-head hand-off granules {value, step tag}
  int* nbc;                        // per launch tile slot: its alive neighbour lists (NBC_INTS ints), built at
                                   //   iteration 1, reloaded by iterations 2-3 of multi-tile workgroups
  int nbc_slots;
  const int* gtoff;                // per launch graph slot: its first tile in the launch (prefix of the
                                   //   slots' tile counts; queue-mode cache slot = gtoff[slot] + tile)
  unsigned long long* xbuf;        // layer split: per launch tile slot [2 layers][1024] E-row granules {tag, value}
  int* pend;                       // per node slot: host-queued actions
  int* tr_action;                  // per node slot: removal order
  int* tr_rank;                    // per node slot: LMCC after each removal
  int* tr_stat;                    // per node slot x 4: n_live, m0, m1, ntie per prediction
  float* tr_q;                     // per node slot x 2: qmax, gap per prediction
  const float* node_w;             // degree cost: [2][total nodes] static features, else null
  unsigned* bar;                   // error word of the grid barrier (bit 31; zeroed per launch)
  unsigned* bars;                  // grid barrier arrival counters: 8 shards x 64 words (zeroed per launch)
  // host selection hand-shake (mapped pinned host memory; null: end the launch instead)
  // launch completion record in mapped host memory (null: the host reads the device words):
  // the last workgroup to exit copies the launch's GraphVars and the error word there, then
  // writes the launch tag, so the host needs no runtime call to learn that a launch is done
  unsigned* exit_ctr;              // device: workgroups that finished this launch (cleared per launch)
  unsigned* h_done;                // mapped host: {launch tag, error word}
  int* h_gvar;                     // mapped host: GraphVar copies [n_graphs]
  int* h_tra;                      // mapped host: mirrors of tr_action / tr_rank, a graph's range
  int* h_trr;                      //   written once it is final (trace_publish)
  unsigned* h_req;                 // per graph: request tag (device writes)
  unsigned* h_ans;                 // per graph: answer tag (host writes)
  int* h_nact;                     // per graph: actions answered (-1: abort)
  int* h_act;                      // per node slot: answered actions
  float* h_q;                      // per node slot: Q of the request (-inf = masked)
  float* h_chk;                    // per graph: {max Q, tie count (int bits)} of the request
  const float* h0g;                // unit cost: first-layer rows of every dmax <= h0g_dm (h0g_row)
  int h0g_dm;
  const int* glist;                // graphs processed by this launch (<= G_CAP)
  int nglist;
  int n_env;                       // dedicated environment workgroups (0 = shared mode)
  unsigned launch_seq;             // launches of this context so far (tags hand-offs)
  int variant;                     // diagnostics: algorithm variant (MD_VARIANT env, 0 = default)
  int run_mode;                    // RUN_*
  int host_select;                 // 1: every prediction goes to the host (step > 1)
  int sel_step;                    // step > 1: picks per prediction; dev_topk: the grid-wide step's
  int dev_topk;                    //   prediction picks its k largest Q on the device when they are
                                   //   distinct and above the rest (md_kernels.hip device_topk)
  int* err;                        // device error word (nonzero = failure code)
  unsigned long long* prof;        // optional phase timestamps of workgroup 0 (wall clock)
  int prof_cap;                    // steps of 16 timestamp slots available in prof
  int qmode;                       // 1: batch rollout through the device work queue (queue_loop)
  int qpair;                       // queue mode: a 2-tile item's tiles run jointly (queue_pair; MD_PAIR)
  int qpark;                       // queue mode: graphs left to the lock-step kernel at the tail (MD_QPARK)
  unsigned* qring;                 // queue mode: the ring's {head, tail} tickets (a line of their own)
  unsigned* qctl;                  // queue mode: {head ticket, tail ticket, running graphs}
  unsigned long long* qslot;       // queue mode: Q_CAP item slots {ticket + 1, item}
  int* qg;                         // queue mode: per graph slot {tiles done in the stage, tiles}
  int endgame;                     // bit 1: the host runs K2 end-games in one hand-shake (see md_kernels.hip);
                                   // bit 2: the device applies the answer in one pass (env_endgame_apply)
  // speculative environment steps (single-graph rollouts, md_kernels.hip spec_loop): workgroups
  // [n_main, n_main + n_spec) precompute the next step's mutual-LMCC cascade for the likely
  // next removals while the tiles compute Q; the grid barrier counts the n_main others only
  int n_main;                      // workgroups taking part in the grid barrier
  int n_spec;                      // speculative workgroups after them (0: off)
  unsigned long long* spec_req;    // request {previous-Q buffer << 32 | request tag}; SPEC_EXIT ends the loop
  int* sres;                       // per speculative workgroup: result slot of sres_stride ints
  int sres_stride;
  float* qspec;                    // [2][qspec_n]: Q of the last two predictions (never masked)
  // iteration-1 prebuild (single-graph rollouts with speculative steps): phase A publishes the
  // speculative result it takes as soon as it knows it (pre_ew: {request tag << 32 | node << 16 |
  // slot}) and, at its end, the same word again when the step's final state is exactly that
  // result (pre_cw, else 0); the tile workgroups build their rows and alive-neighbour lists from
  // the result while phase A runs and keep them when the confirmation matches
  unsigned long long* pre_ew;
  unsigned long long* pre_cw;
  // dataflow mode with the self-pick: tile 0's derivation of phase A's early word, published when
  // the result it names is finished (speculative workgroups start the next state from it)
  unsigned long long* self_ew;
  int spec_early;                  // 1: speculative workgroups serve the next request from pre_ew (spec_loop)
  int spec_abort;                  // 1: a speculative fixed point stops once its result cannot be used
  int qspec_n;                     // total nodes of the loaded batch
  // dataflow mode (single-graph rollouts in dedicated mode with the layer split, md_kernels.hip
  // df_*): no grid barrier; the step record, the H rows, the virtual-node and arg-max partials
  // move as data-tagged granules {value, tag} in this buffer (graph-local node / tile indices,
  // zeroed per launch; layout df_ap / df_sp / df_hb, rows and sums by step parity).  null: the
  // barrier protocol.
  unsigned long long* df;
  int df_mt;                       // tiles of the largest graph the buffer is sized for
  int df_n;                        // nodes of that graph
  int fp_short;                    // 1: mutual-LMCC fixed points end by the confirmation shortcut (mcc_fixed_point)
  int fp_skip;                     // 1: LDS fixed-point rounds skip the layers the last prune left unchanged
  int first_req;                   // 1: a rollout's first step requests degree-ranked speculative results (env_step)
  // batched prefixes (md_env.h team_prefix_step): the grid-wide step applies a prediction's
  // actions as independent prefix fixed points, one per workgroup, when at least pfx_min remain
  int* pfx;                        // scratch, pfx_words(largest et) ints; null: off
  int pfx_min;                     // MD_PREFIX (0: off)
};
// global-mode environment scratch words per node (md_env.h env_view: parents, degrees) and the
// grid-wide step's own words per node of the graph it runs (team_env_step, one graph per launch)
constexpr int GSCR_WORDS = 4, GSCR_TEAM_WORDS = 6;
// dataflow buffer size (granules) for graphs of at most n nodes / mt tiles
inline long long df_granules(int n, int mt) { return 64 + 772LL * mt + 8LL * 64 * n; }

// Speculative-step result slot (ints):
//   [0..1] u64 done tag {nd << 48 | candidate << 32 | request tag}, written last
//   [2] LMCC  [3..4] pruned edges per layer  [5..6] covered edges per layer  [7] killed edges nd
//   [8..9] u64 started tag {candidate << 32 | request tag}, written when the candidate is taken
//   [10..11] u64 device time of the result (diagnostics)
//   [12] live nodes  [13..14] dmax per layer  [15..16] degree sums  [17] live-set mismatch
//   [18..21] two-hop sums (2 x i64)  [22..23] u64 features tag {candidate << 32 | request tag},
//   written after the degrees, live list and aggregates (later than the done tag)
//   [SRES_HDR, +3 nd) killed edges {edge (LDS id) | new state << 16, CSR slot, CSR slot}
//   [sres_deg, +2 n) residual degrees per layer; [sres_live, +4 n) live-list entries
constexpr int SRES_HDR = 32, SRES_STARTED = 8, SRES_FEAT = 22;
// Result slots are double-buffered by the parity of the request's step: slot k of request step
// ps is k + SPEC_SLOTS * (ps & 1), so the next request never rewrites a slot that the tile
// workgroups may still be reading for their iteration-1 prebuild.
constexpr int SPEC_SLOTS = 32;
__host__ __device__ inline int spec_slot_index(int k, int ps) { return k + SPEC_SLOTS * (ps & 1); }
__host__ __device__ inline int sres_deg(int et) { return SRES_HDR + 3 * et; }
__host__ __device__ inline int sres_live(int et, int n) { return (sres_deg(et) + 2 * n + 3) & ~3; }
__host__ __device__ inline int sres_words(int et, int n) { return sres_live(et, n) + 4 * n; }
constexpr unsigned long long SPEC_EXIT = ~0ull;
__host__ __device__ inline unsigned spec_tag(unsigned launch_seq, int steps) {
  return ((launch_seq & 0xffffu) << 16) | ((unsigned)steps & 0xffffu);
}

}  // namespace md
