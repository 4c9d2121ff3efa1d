/*
 * mdroll.h — C ABI of libmdroll.so, the MI355X (gfx950) MultiDismantler inference-rollout engine.
 *
 * The reference (KelvinRyman/MDCommunity, Python) runs the rollout as
 *   GetSol / GetSolution          U/MultiDismantler_torch.py:759-784 / :711-736
 *     -> PredictWithCurrentQNet   :304-306 -> Predict :263-302 -> test_forward
 *                                 (U/MultiDismantler_net_graphsage.py:243-394)
 *     -> np.argsort(-q)[:step]    :769 / :725
 *     -> MvcEnv.stepWithoutReward U/mvc_env.py:74-87 -> getReward -> Mcc.MCC (U/Mcc.py:30-38)
 * Each entry point below replaces one of those interfaces; the Python package
 * `mdcommunity_amd` binds them with ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions: plain pointers and explicit sizes only; the caller owns every host buffer,
 * the library owns every device allocation of a context; weights and graphs are copied in.
 * Every function returns an md_status and never aborts across the ABI; md_last_error()
 * gives the detail string of the last failure on that context.
 * Threading: one context per (process, device); calls on one context must be serialised
 * by the caller (the reference is single-threaded Python).  Contexts on different devices
 * may be used concurrently (one process per GPU for the sharded configuration).
 */
#ifndef MDROLL_H
#define MDROLL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  MD_OK = 0,
  MD_EINVAL = 1,   /* bad argument (shape, id range, self-loop, ...)             */
  MD_EHIP = 2,     /* HIP runtime error (launch, copy, device fault)              */
  MD_EOOM = 3,     /* device allocation failed                                    */
  MD_ESTATE = 4,   /* call not valid in the current state (e.g. no graphs loaded) */
  MD_ETIMEOUT = 5, /* a device-side team barrier timed out (kernel drained)       */
  MD_ECALLBACK = 6 /* the host tie-selection callback reported an error           */
} md_status;

/* Cost model: unit cost (U/) or degree cost (D/, D/mvc_env.py:127-134). */
enum { MD_COST_UNIT = 0, MD_COST_DEGREE = 1 };

/* Number of fp32 values in a packed weight blob (A.3 of SURVEY.md; state_dict of
 * U/MultiDismantler_net_graphsage.py:42-89 + U/MRGNN/mutil_layer_weight.py:252-262),
 * packed in this order, each row-major as in the state_dict:
 *   w_n2l[2][64], p_node_conv[64][64], p_node_conv2[64][64], p_node_conv3[128][64],
 *   h1_weight[64][32], h2_weight(=last_w)[36], cross_product[64], w_layer1[64][128],
 *   w_layer2[128], trans[64][64], bias[64], logis.weight[64], logis.bias[1]          */
#define MD_WEIGHT_FLOATS 31205

typedef struct md_ctx md_ctx;

/* Host tie-resolution callback.  The device picks the arg-max itself whenever the
 * maximum Q is unique.  When k > 1 live nodes tie exactly at the maximum, the reference's
 * choice is `np.argsort(-q)[:step]` (U/MultiDismantler_torch.py:769), i.e. numpy's
 * unstable sort order, so the library hands the masked Q row (float64, masked entries =
 * -1073741823.5 as U/MultiDismantler_torch.py:60,291-299) to the host, which writes
 * `n_out` node ids, best first, into `actions`.  Return 0 on success.
 * The callback runs on the calling thread while the rollout kernel waits for its answer
 * (the Q row and the answer travel through mapped pinned memory; no relaunch), so it must
 * return within 60 s (else MD_ETIMEOUT); MD_HOST_HANDSHAKE=0 in the environment falls back
 * to ending the launch and relaunching after the callback. */
typedef int (*md_select_cb)(void* user, int graph, const double* q, int n_nodes, int n_out,
                            int32_t* actions);

/* numpy's own float64 argsort routine (its ArrFuncs argsort[NPY_QUICKSORT] entry, the code
 * np.argsort(x) runs for a contiguous float64 array; the package's _npsel helper module hands
 * its address over).  Registered with md_set_tie_argsort, the tie hand-shake computes
 * np.argsort(-q)[:step] (U/MultiDismantler_torch.py:725,769) on the host thread itself
 * instead of calling the selection callback; NULL restores the callback. */
typedef int (*md_argsort_f64)(void* data, int64_t* idx, int64_t n, void* unused);

/* Create a context on HIP device `device`.  `weights` holds MD_WEIGHT_FLOATS floats
 * (replaces MultiDismantler.LoadModel, U/MultiDismantler_torch.py:791-797). */
md_status md_create(int device, const float* weights, size_t n_floats, int cost_mode, md_ctx** out);
void md_destroy(md_ctx* ctx);
const char* md_last_error(const md_ctx* ctx);

/* Replace the weights of an existing context (LoadModel on a live agent). */
md_status md_set_weights(md_ctx* ctx, const float* weights, size_t n_floats);

/* Load a batch of two-layer graphs (replaces graph.Graph_test, U/graph.py:69-84, and
 * MultiDismantler.InsertGraph :171-178).  Graph g has n_nodes[g] nodes (ids 0..n-1).
 * Layer l's undirected edges of graph g are the pairs
 *   edges_l[2*k], edges_l[2*k+1]   for k in [edge_off_l[g], edge_off_l[g+1])
 * given in the reference's edge order (networkx G.edges(), U/graph.py:76): it fixes the
 * neighbour-aggregation order (U/PrepareBatchGraph.py:151-160).  Self-loops and duplicate
 * edges are rejected (MD_EINVAL).  `node_w` (degree cost only, else NULL) holds
 * 2*sum(n_nodes) per-node weights: layer 0 of all graphs, then layer 1 (D/graph.py:91-115).
 * Loading replaces any previously loaded batch and resets every graph (md_reset). */
md_status md_load_graphs(md_ctx* ctx, int n_graphs, const int32_t* n_nodes,
                         const int64_t* edge_off0, const int32_t* edges0,
                         const int64_t* edge_off1, const int32_t* edges1,
                         const float* node_w);

/* MvcEnv.s0 for every loaded graph (U/mvc_env.py:31-52): clear covered/removed state and
 * run the initial mutual-LMCC prune.  max_rank_out[g] (may be NULL) receives the initial
 * LMCC size = Graph_test.max_rank (U/graph.py:80-84). */
md_status md_reset(md_ctx* ctx, int32_t* max_rank_out);

/* md_reset with MvcEnv.s0's prune deferred: the state is cleared now, and the initial
 * mutual-LMCC prune runs as the first environment step of the next md_rollout, inside the same
 * launch (every rollout kernel starts with an environment step; no separate s0 launch and host
 * round trip).  Any other call that reads or changes the state (md_predict, md_step,
 * md_get_state, md_set_state, md_max_rank) first runs that prune exactly as md_reset does, so an
 * action is never applied before it; md_max_rank after the md_rollout reads max_rank. */
md_status md_reset_deferred(md_ctx* ctx);

/* Graph_test.max_rank of every loaded graph as of the last launch (after md_reset, or after the
 * md_rollout that followed md_reset_deferred): max_rank_out[g]. */
md_status md_max_rank(md_ctx* ctx, int32_t* max_rank_out);

/* One Q evaluation of the current state of every graph (Predict, U/MultiDismantler_torch.py:263-302).
 * q_out (may be NULL): sum(n_nodes) floats, graph-major; non-live nodes get -1073741823.5.
 * argmax/n_tie/top_gap (may be NULL): per graph, arg-max node (-1 if terminal), number of
 * nodes tied at the max, and the gap between the best and second-best live Q. */
md_status md_predict(md_ctx* ctx, float* q_out, int32_t* argmax, int32_t* n_tie, float* top_gap);

/* MvcEnv.stepWithoutReward for every graph with actions[g] >= 0 (U/mvc_env.py:74-87):
 * cover the node, cascade the mutual-LMCC prune.  lmcc_out[g] (may be NULL) = LMCC size
 * after the step (the `rank` of getReward :133-137); terminal_out[g] = isTerminal (:128-131). */
md_status md_step(md_ctx* ctx, const int32_t* actions, int32_t* lmcc_out, uint8_t* terminal_out);

/* The whole rollout of every graph from its current state to terminal, on the device
 * (GetSol / GetSolution loop).  `step` = nodes removed per prediction (stepRatio, :676-679);
 * with step > 1 every prediction goes through `cb`.  Outputs, per graph g with capacity
 * n_nodes[g] entries at node_off(g) = sum_{h<g} n_nodes[h]:
 *   seq_out   removal order;  lmcc_out  LMCC size after each removal;  seq_len[g] count.
 * cb may be NULL only if no tie occurs (else MD_ECALLBACK). */
md_status md_rollout(md_ctx* ctx, int step, int32_t* seq_out, int32_t* lmcc_out, int32_t* seq_len,
                     md_select_cb cb, void* user);

/* md_rollout with the outputs packed: graph g's removal order and LMCC trace at offsets
 * sum_{h<g} seq_len[h] of seq_packed / lmcc_packed (capacity sum(n_nodes) each; only the
 * removals are read: each graph's trace reaches mapped host memory as the graph ends, so no
 * copy follows the launch).  seq_len is required. */
md_status md_rollout_packed(md_ctx* ctx, int step, int32_t* seq_packed, int32_t* lmcc_packed, int32_t* seq_len,
                            md_select_cb cb, void* user);

/* Per-step diagnostics of the last md_rollout for graph g (capacity n_nodes[g] rows):
 * live nodes, alive edges in layer 0 and 1, number of nodes tied at the max, per prediction,
 * and (float) the best Q and top-2 gap.  Returns the number of predictions made. */
md_status md_rollout_trace(md_ctx* ctx, int graph, int32_t* n_live, int32_t* m0, int32_t* m1,
                           int32_t* n_tie, float* qmax, float* gap, int32_t* n_pred);

/* Speculative environment steps of the last md_rollout for graph g: removals whose mutual-LMCC
 * fixed point was taken from a speculative workgroup (hits) out of all removals.  A
 * single-graph rollout runs up to MD_SPEC (default 32) extra workgroups on CUs it leaves
 * free; each runs the next step's fixed point for one likely next removal while the tiles
 * compute Q.  Results never depend on it (diagnostics). */
md_status md_spec_stats(md_ctx* ctx, int graph, int32_t* hits, int32_t* removals);

/* Read back the environment state of graph g (MvcEnv attributes, U/mvc_env.py:8-29):
 * covered[n] (0/1), removed_l[e_l] (1 = pruned by MCC, i.e. in remove_edge[l]),
 * counters[6] = {numCoveredEdges[0], numCoveredEdges[1], |removed0|, |removed1|, lmcc, terminal}. */
md_status md_get_state(md_ctx* ctx, int graph, uint8_t* covered, uint8_t* removed0, uint8_t* removed1,
                       int32_t* counters);

/* Overwrite the state of graph g (PredictWithCurrentQNet on an arbitrary state): covered
 * nodes and pruned edges; no MCC is run (the reference's Predict runs none). */
md_status md_set_state(md_ctx* ctx, int graph, const uint8_t* covered, const uint8_t* removed0,
                       const uint8_t* removed1);

/* Host tie selection through numpy's argsort routine (see md_argsort_f64), NULL = callback. */
md_status md_set_tie_argsort(md_ctx* ctx, md_argsort_f64 fn);

/* Execution geometry override: number of tile workgroups of a launch, 0 = automatic
 * (one per 16-node tile, at most one workgroup per CU).  Results do not depend on it. */
md_status md_set_team_size(md_ctx* ctx, int team_size);

/* Device time (ms) of the kernel launches of the last md_reset / md_predict / md_step /
 * md_rollout call, measured with HIP events on the context's stream, and their count. */
md_status md_last_timing(md_ctx* ctx, double* kernel_ms, int32_t* launches);

/* Host selection requests (ties, stepRatio predictions the device did not pick itself) served
 * during the last md_reset / md_predict / md_step / md_rollout call. */
md_status md_host_requests(md_ctx* ctx, int32_t* n_requests);

/* Diagnostics: record device wall-clock (100 MHz) phase timestamps of workgroup 0,
 * MD_PROF_SLOTS slots per removal step (0-15 timestamps, 16-31 accumulated sub-phase
 * durations and counters of the environment step, 64-72 speculative-step timeline), for up to `steps` steps per launch of the
 * following calls (0 disables).
 * md_profile_read copies the timestamps accumulated since md_profile was called and returns
 * the number of steps recorded in *n_steps. */
#define MD_PROF_SLOTS 96
md_status md_profile(md_ctx* ctx, int steps);
md_status md_profile_read(md_ctx* ctx, uint64_t* out, int capacity_steps, int32_t* n_steps);

/* Library build string (arch, version). */
const char* md_version(void);

/* Number of visible GPUs (0 when there is none or the runtime fails): the agent's
 * "CUDA: <bool>" line (U/MultiDismantler_torch.py:107, torch.cuda.is_available()). */
int md_device_count(void);

/* ---------------------------------------------------------------- synthetic graph generator
 * Geometric Multiplex Model (U/GMM.py:6-68 with U/Hyperbolic.py:18-117, g = 0.5, nu = 0.2,
 * gamma = 2.5, T = 0.4, kbar ~ U(2, 10)) on the device, SURVEY.md §8(f3).  Context-free (own
 * device allocations; errors in md_gmm_last_error()).  mdcommunity_amd.gmm_gpu drives them. */
const char* md_gmm_last_error(void);

/* Per-node values of n_graphs graphs of n nodes: kbar_out [G][2], kappa_out / theta_out
 * [G][2][n] (layer 0 then the conditioned layer 1: GMM.py:10-25).  Randomness: Philox4x32-10
 * streams keyed by seeds[G] (not the reference's numpy stream), or -- for checks against the
 * reference's own functions -- the caller's uniforms [4][G][n] (kappa1, kappa2, theta1, theta2)
 * and kbar_in [G][2]. */
md_status md_gmm_nodes(int device, int n_graphs, int n, const uint64_t* seeds, const double* uniforms,
                       const double* kbar_in, double* kbar_out, double* kappa_out, double* theta_out);

/* Links of n_layers layers of n nodes (CreateNetworks, U/Hyperbolic.py:101-117): pairs (i < j)
 * in row-major order, kept when u < 1 / (1 + r^(1/T)); kappa / theta [L][n], mu [L].  Edges
 * (u < v, lexicographic: the reference's networkx order) to edges_out [L][edge_cap][2], counts
 * to edge_count [L].  uniforms [L][n(n-1)/2]: the reference's pair stream (exact mode; pairs
 * within a relative 1e-9 of the threshold go to amb_out [L][amb_cap] / amb_count [L] for the
 * caller to re-decide with the reference's own expression); else Philox pair streams keyed by
 * seeds [L/2] (layers 2g, 2g + 1 of graph g). */
md_status md_gmm_links(int device, int n_layers, int n, const double* kappa, const double* theta, const double* mu,
                       const double* uniforms, const uint64_t* seeds, int32_t* edges_out, int64_t* edge_count,
                       int64_t edge_cap, int64_t* amb_out, int64_t* amb_count, int64_t amb_cap);

/*
 * Environment switches, read once by md_create.  None changes any result: each selects between
 * equivalent execution strategies (for A/B measurement and for exercising fallbacks), and each
 * has a GPU identity test that checks identical rollouts (named after the switch):
 *   MD_VARIANT        bit mask, default 0:
 *                       1     single-graph rollouts: no iteration-1 prebuild during phase A
 *                             (test_iteration1_prebuild_same_rollouts)
 *                       2     one graph too large for LDS: its environment step on one workgroup
 *                             instead of on every workgroup (team_env_step); with 64 and
 *                             MD_ENV_MODE=0 that step also runs for graphs that fit
 *                             (test_grid_wide_environment_step)
 *                       32    lock-step shared mode instead of the device work queue (> 16
 *                             graphs; the path batches with graphs of >= 8192 tiles take)
 *                             (test_shared_mode_batch_matches_dedicated)
 *                       64    environment state in HBM even when it fits in LDS
 *                             (test_global_memory_environment_mode, test_grid_wide_environment_step)
 *                       128   iteration-1 prebuild limited to the rows and neighbour lists
 *                             (test_iteration1_prebuild_same_rollouts)
 *                       512..1536 (bits 9-10 = 1..3)  tiles per queue work item (default 2)
 *                             (test_queue_admission_limit_matches_single)
 *                       256   environment staged in batched passes instead of one pass of
 *                             16-byte chunks (test_iteration3_order_and_staging_same_rollouts)
 *                       2048  K2 end-game shortcut off: one forward pass per removal step (the
 *                             bench's per_step_protocol_value;
 *                             test_k2_endgame_in_one_handshake_matches_per_step)
 *                       4096  queue launches: iteration-3 tiles queued after virtual-node part 2
 *                             instead of beside it (test_iteration3_order_and_staging_same_rollouts)
 *                       8192, 16384  with MD_BSPEC=1: speculative results not used / not queued
 *                             by wave items (test_batch_speculation_same_rollouts's diagnostics)
 *                       32768 an applied speculative result compacts the alive list at once
 *                             (test_iteration3_order_and_staging_same_rollouts)
 *                       bits 16+  queue-mode admission limit (graphs running at once)
 *                             (test_queue_admission_limit_matches_single)
 *   MD_ENV_MODE       0: no dedicated environment workgroups for small batches (shared
 *                     mode); default 1 (test_grid_wide_environment_step)
 *   MD_PAIR           0: queue-mode work items run their two tiles one after the other
 *                     instead of jointly (default 1; test_paired_tiles_match_single_tiles)
 *   MD_QPARK          queue mode: once every graph is admitted and at most this many still
 *                     run, they continue in one lock-step launch (default 4, 0 = off, <= 16;
 *                     tests/test_gpu_batch.py test_tail_handoff_off_same_rollouts)
 *   MD_WQ             0: queue launches run one work item per workgroup (md_queue_kernel) from
 *                     the start instead of one per wave (md_wq_kernel, default 1;
 *                     test_wave_items_match_workgroup_items)
 *   MD_WQPARK         wave-item launches of more than this many graphs park the graphs still
 *                     running once at most this many are left; md_queue_kernel continues them
 *                     (default 128, 0 = never; test_wave_items_match_workgroup_items runs 0)
 *   MD_BSPEC          1: queue launches run speculative environment items for the likely next
 *                     pick (default 0; test_batch_speculation_same_rollouts)
 *   MD_HOST_HANDSHAKE 0: end the launch on a tie and relaunch after the host selection
 *                     (default 1: in-kernel hand-shake through mapped host memory;
 *                     test_host_handshake_modes_same_rollouts)
 *   MD_H0G            0: rebuild the unit-cost first-layer tables per step instead of the
 *                     precomputed per-dmax tables (test_precomputed_first_layer_tables)
 *   MD_SPEC           speculative environment workgroups of a single-graph rollout (0..32,
 *                     default 32, 0 = off; md_spec_stats; test_speculative_steps_match_plain)
 *   MD_EARLY          0: speculative workgroups wait for phase A's write-back and restage the
 *                     state instead of building the next state from the result phase A takes
 *                     (test_speculative_steps_match_plain)
 *   MD_SPEC_ABORT     0: a speculative fixed point runs to the end even when phase A has taken
 *                     another result of its request (default 1: it stops after the round;
 *                     test_speculative_steps_match_plain)
 *   MD_DF             single-graph rollouts in dedicated mode with the layer split: 1 (default)
 *                     dataflow mode (no grid barrier, tagged hand-offs) whose tiles derive
 *                     phase A's pick from the arg-max partials and prebuild from it; 0 grid
 *                     barriers (the tiles prebuild from phase A's early word)
 *                     (test_dataflow_mode_same_rollouts)
 *   MD_FP_SHORTCUT    0: every mutual-LMCC fixed point runs its confirmation round (default 1:
 *                     a pruned partition certified by its spanning forests ends the fixed point;
 *                     test_fixed_point_shortcut_same_rollouts)
 *   MD_FP_SKIP        0: every round of a mutual-LMCC fixed point re-unites both layers
 *                     (default 1: a layer the last prune left unchanged keeps its components
 *                     and labels -- the LDS-resident and the grid-wide fixed point;
 *                     test_fixed_point_shortcut_same_rollouts, and the grid-wide step's
 *                     certified N = 18 000 sequences)
 *   MD_PREFIX         k: the grid-wide environment step applies a prediction's picks
 *                     (stepRatio > 0) as independent prefix fixed points, one per workgroup,
 *                     while at least k remain (default 8; 0: one cascade after another;
 *                     test_gpu_prefix.py, and the certified N = 18 000 stepRatio sequence)
 *   MD_DEVTOPK        0: every stepRatio prediction of the grid-wide step goes to the host's
 *                     numpy routine (default 1: the device takes the k largest Q when they are
 *                     tie-free; test_device_topk_same_rollouts)
 *   MD_EG_APPLY       0: a K2 end-game answer is applied action by action (default 1: in one
 *                     pass, env_endgame_apply; test_k2_endgame_one_pass_apply_same_state)
 *   MD_FIRST_REQ      0: no speculative request at a rollout's first environment step (default
 *                     1: candidates ranked by residual degree, as no prediction exists yet;
 *                     test_first_request_same_rollouts)
 * Diagnostics and resources (no effect on any computation):
 *   MD_VARIANT 4      event log of graph slot 0 in wave-item launches (md_profile;
 *                     scripts/wq_timeline.py)
 *   MD_VARIANT bit 8  per-piece queue-mode profile stamps (md_profile; qprof build)
 *   MD_POLL_US        host-thread polling interval of the hand-shake (µs)
 *   MD_HOST_STATS     set: print hand-shake and host-side timing (launch prelude, wait,
 *                     outputs) to stderr
 *   MD_PROF_ALL       md_profile_read returns every non-empty record row (the dataflow mode's
 *                     per-tile rows after the step records), not only the step records
 *   MD_TRACE          1: every device allocation and kernel launch to stderr (maps a GPU
 *                     memory-fault address to a buffer and a launch)
 *   MD_MAX_CUS        use at most this many CUs (>= 8; default: all), e.g. for several ranks
 *                     sharing one GPU, whose persistent grids must be co-resident
 */

#ifdef __cplusplus
}
#endif
#endif /* MDROLL_H */
