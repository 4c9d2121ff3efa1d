// md_kernels.hip — gfx950 (MI355X, CDNA4) kernels of the MultiDismantler inference rollout.
//
// One persistent kernel runs whole rollouts of a batch of graphs (1 ... G_CAP per launch).
// All workgroups of the grid cooperate; per removal step they run four phases separated by
// grid barriers (placement-independent agent-scope release/acquire):
//   A  environment, one workgroup per graph: apply the chosen node (U/mvc_env.py:74-87),
//      mutual-LMCC cascade by union-find over the graph's edges staged in LDS
//      (U/Mcc.py:30-38), residual degrees, ascending live-node list and aux features
//      (U/PrepareBatchGraph.py:35-101), first-layer embedding table.
//   1,2 message passing (U/MultiDismantler_net_graphsage.py:288-321) over 16-row tiles of all
//      graphs, spread over the grid in contiguous tile ranges: CSR neighbour gather-sum in the
//      reference's in_edges order, the node-update MLP on v_mfma_f32_16x16x4_f32 (a k-ordered
//      fp32 FMA chain == MKL's sgemm order), ReLU, row L2 norm in torch's reduction order,
//      per-tile virtual-node partial sums.
//   3  last iteration + inter-layer attention (U/MRGNN/mutil_layer_weight.py:266-313) + Q head
//      (net :343-394) on the same rows, per-tile arg-max partials.
// Phase A of the next step reduces a graph's arg-max partials in tile order (deterministic,
// independent of the grid size).  Exact ties go back to the host: the reference breaks them
// with numpy's unstable argsort (U/MultiDismantler_torch.py:769).
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "md_common.h"

namespace md {

typedef float f4 __attribute__((ext_vector_type(4)));

// The dynamic LDS of every kernel here, as a compile-time base: device functions derive their
// LDS pointers from it instead of from pointer arguments, so their LDS addresses stay
// constants whichever kernel (and however many call levels) they are reached from.
__device__ __forceinline__ float* lds_base() {
  extern __shared__ __attribute__((aligned(16))) float lds_dyn[];
  return lds_dyn;
}

// ------------------------------------------------------------------ weight image (floats)
// Weights in MFMA B-fragment order: frag[cb][s][lane] = W[4s + (lane>>4)][16cb + (lane&15)].
constexpr int W_IP1 = 0;                // 4 x 16 x 64
constexpr int W_IP2 = W_IP1 + 4096;
constexpr int W_IP3 = W_IP2 + 4096;     // 4 x 32 x 64
constexpr int W_IT = W_IP3 + 8192;      // 4 x 16 x 64
constexpr int W_IH1 = W_IT + 4096;      // 2 x 16 x 64
constexpr int W_ITB = W_IH1 + 2048;     // 64
constexpr int W_ILW = W_ITB + 64;       // 64
constexpr int W_ICP = W_ILW + 64;       // 64
constexpr int W_IW2 = W_ICP + 64;       // 36 (+4)
constexpr int W_ILB = W_IW2 + 40;       // 1 (+3)
constexpr int W_IWN = W_ILB + 4;        // 128 (w_n2l row-major)
constexpr int W_IWL2 = W_IWN + 128;     // 128
constexpr int W_IEND = W_IWL2 + 128;

// ------------------------------------------------------------------ LDS layout (floats)
constexpr int L_PREF = 0;                        // int [G_CAP + 4] tile prefix of this step
constexpr int L_MISC = L_PREF + G_CAP + 4;       // 64 words of broadcast scalars
// dataflow mode, phase A: per speculative slot {features tag (2 words), aggregates (6)} read
// beside the slot tags (L_PREF words [0, 4 SPEC_MAX) hold the tags)
constexpr int PREF_FEAT = 4 * 32;
static_assert(PREF_FEAT + 8 * 32 <= G_CAP + 4, "speculative slot words must fit L_PREF");
constexpr int L_GV = L_MISC + 64;                // 32 words: phase-A copy of a GraphVar
constexpr int L_Y0 = L_GV + 32;                  // [64] virtual-node input embedding (constant)
constexpr int L_YW = L_Y0 + 64;                  // [2][64] virtual-node embedding being iterated
constexpr int L_YS = L_YW + 128;                 // [2][64] final graph vector y per layer
constexpr int L_GS = L_YS + 128;                 // graph scalars: mix w0,w1; aux per layer
constexpr int L_W = L_GS + 16;                   // weight image
constexpr int L_SCR = L_W + W_IEND;              // tile scratch
// tile scratch (offsets from L_SCR)
constexpr int LDT = 17;                 // transposed tile: At[k][row], 16 rows + 1 pad
constexpr int S_P = 0;                  // [2][64][17] gathered neighbour sums
constexpr int S_X = S_P + 2 * 64 * LDT; // [2][64][17] own embedding
constexpr int S_M = S_X + 2 * 64 * LDT; // [2][128][17] [P.P1 | X.P2]
constexpr int S_E = S_M + 2 * 128 * LDT;// [2][64][17] new embedding / attention output
constexpr int S_F = S_E + 2 * 64 * LDT; // [2][64][17] tanh features / Q-head input
constexpr int S_HID = S_F + 2 * 64 * LDT;   // [2][16][33]
constexpr int S_RED = S_HID + 2 * 16 * 33;  // [2][16][8] sum-of-squares partials
constexpr int S_DOT = S_RED + 256;          // [16][3] attention gate dot products, [2][16] gates
constexpr int S_Q = S_DOT + 96;             // [2][16]
constexpr int S_ROW = S_Q + 32;             // [16] node id per tile row (int)
constexpr int S_YP = S_ROW + 16;            // [2][4][128] virtual-node GEMV partials
constexpr int S_YM = S_YP + 1024;           // [2][128]
// The neighbour lists alias the virtual-node scratch S_YP/S_YM: the graph-head workgroup
// never gathers, and shared-mode tile workgroups rebuild the lists after each chain.
constexpr int S_NBH = S_YP;                 // neighbour-list header (ints, see build_nb_lists)
constexpr int S_NBL = S_NBH + 172;          // [2][NB_CAP] u16 alive neighbour ids, CSR order
constexpr int NB_CAP = NB_CAP_ENTRIES;      // alive neighbour entries per layer kept for a tile
constexpr int S_END = S_NBL + NB_CAP;
constexpr int STG_ROWS = 68;                // neighbour rows per layer staged per batch ([S_M, S_HID))
constexpr int L_TOTAL = L_SCR + S_END;      // floats of dynamic LDS per workgroup
// grid-wide environment step (md_env.h team_env_step) in the tile scratch: env_view's block-scan
// temp at 0, the team reductions' words at TEAM_TMP_OFF, the static union ranks (u16) after them
constexpr int TEAM_TMP_OFF = 1024, TEAM_RANK_OFF = 2048;
constexpr int TEAM_RANK_MAX = 2 * (S_END - TEAM_RANK_OFF);  // nodes whose ranks fit
// Paired tiles (queue mode, md_kernels.hip queue_pair): the two tiles of a 2-tile work item run
// every piece once for their 32 rows.  Transposed blocks [layer][row block][K][LDT] (a row
// block = one tile's 16 rows, the single-tile layout twice); M aliases P and X once their
// reads are done, E aliases M, the attention features F the dead X, the hidden layer the
// dead E, and the gather stages its neighbour rows in P and X before it writes them.  The
// first tile keeps its lists at S_NBH, the second at P2_NB1.
constexpr int P2_LD = 16;                      // P / X / M blocks: K-rows of 16 rows, rotated (p2o)
constexpr int P2_P = 0;                         // [2][2][64][16] gathered neighbour sums
constexpr int P2_X = 2 * 2 * 64 * LDT;          // [2][2][64][16] own embedding (F's offset)
constexpr int P2_M = 0;                         // [2][2][128][16] [P.P1 | X.P2]
constexpr int P2_E = 0;                         // [2][2][64][17] new embedding / attention output
constexpr int P2_F = P2_X;                      // [2][2][64][17] tanh features / Q-head input
constexpr int P2_HID = 0;                       // [2][32][33]
constexpr int P2_NB1 = S_NBH - (S_END - S_NBH); // second tile's list region (header + lists)
constexpr int P2_ROW = P2_NB1 - 784;            // [32] node id per row (int)
constexpr int P2_RED = P2_ROW + 32;             // [2][32][8] sum-of-squares partials
constexpr int P2_DOT = P2_RED + 512;            // [32][3] gate dot products, [2][32] gates at +96
constexpr int P2_Q = P2_DOT + 160;              // [2][32]
constexpr int P2_FLAG = P2_Q + 64;              // ints: [0] lists cached, [1..2] lists ok, [8..15] wave totals
constexpr int P2_STG = 0;                       // gather staging, [2][STG2_ROWS][16] float4 (P, X and beyond)
constexpr int STG2_ROWS = 88, STG2_LD = (STG2_ROWS * 16 + 255) / 256;  // rows per layer, loads per thread
static_assert(P2_FLAG + 16 == P2_NB1 && 2 * P2_X <= P2_ROW, "paired-tile scratch below the second list region");
static_assert(2 * STG2_ROWS * 64 <= P2_ROW, "paired gather staging below the row ids");
static_assert(2 * 32 * 33 <= P2_X, "paired hidden layer inside the E region");
__device__ __forceinline__ int p2b(int l, int rb, int K) { return (l * 2 + rb) * K * LDT; }
// The update's operand blocks P, X and M are [K][16] with K-row k holding its 16 rows rotated
// by 5 * (k >> 1) (p2m block bases, p2o elements): the MFMA A-operand reads (a wave half reads
// K-rows k, k + 1 for k even, rows 0..15) then cover all 32 banks of ds_read_b32, where [k][17]
// put row 15 of k + 1 on row 0's bank (2-way on every A read); the gather and MFMA D writes
// conflict no more than with [k][17].  E and F keep [k][17] (their row-wise and column-wise
// accesses would pay a rotated offset per element).
__device__ __forceinline__ int p2m(int l, int rb, int K) { return (l * 2 + rb) * K * P2_LD; }
__device__ __forceinline__ int p2o(int k, int row) { return k * P2_LD + ((row + 5 * (k >> 1)) & 15); }
// A-operand offsets of a lane (ak = lane >> 4, ar = lane & 15): p2o(4 * s + ak, ar) is
// 64 * s + ro[s & 7] (the rotation 5 * (2 * s + (ak >> 1)) repeats every 8 k-steps), so the
// reads of every k-step take an immediate offset from one of 8 lane registers.
struct P2Rot {
  int ro[8];
  __device__ __forceinline__ P2Rot(int ak, int ar) {
#pragma unroll
    for (int q = 0; q < 8; ++q) ro[q] = ak * P2_LD + ((ar + 10 * q + 5 * (ak >> 1)) & 15);
  }
  __device__ __forceinline__ int operator()(int s) const { return 64 * s + ro[s & 7]; }
};
// phase A uses [L_W, L_TOTAL) (weights are reloaded afterwards)
constexpr int A_WORDS = L_TOTAL - L_W;
constexpr int A_TMP_WORDS = 1024;

static_assert(L_W % 4 == 0 && L_SCR % 4 == 0, "16-byte aligned regions");
static_assert(sizeof(GraphVar) <= 32 * 4, "GraphVar must fit its LDS slot");
static_assert(L_TOTAL * 4 + 1024 <= 163840, "LDS budget");
static_assert(S_END >= 64 * 128 + 128 + 4 + 256, "scratch must hold w_layer1 for the graph head");
static_assert(2 * STG_ROWS * 64 <= S_HID - S_M, "neighbour staging fits [S_M, S_HID)");

constexpr float NEG_INF = -__builtin_huge_valf();
constexpr unsigned long long BARRIER_TIMEOUT_TICKS = 400000000ull;  // 4 s at 100 MHz
enum : int { ERR_TIMEOUT = 1, ERR_COVERED = 2, ERR_LIVE_MISMATCH = 3, ERR_BADNODE = 4, ERR_HOST = 5, ERR_ABI = 6,
             ERR_DF_LISTS = 7, ERR_DF_EARLY = 8, ERR_SPEC_SLOT = 9 };

// Kernel arguments of md_rollout_kernel / md_env_kernel, (Params, const float*), read in every
// device function through the implicit-argument pointer (SGPRs s[8:9] in callees) at a fixed
// offset below it: s_load of uniform fields straight from the kernarg segment.  A Params
// reference passed to a non-inlined function would travel as a per-lane (VGPR) pointer to a
// private copy: flat loads from scratch and waterfall loops around every buffer resource.
typedef const __attribute__((address_space(4))) Params KParams;
constexpr int KARG_BYTES = (int)((sizeof(Params) + 7) & ~(size_t)7) + 8;  // Params, wimg
__device__ __forceinline__ KParams& kp() {
  return *(KParams*)((const __attribute__((address_space(4))) char*)__builtin_amdgcn_implicitarg_ptr() - KARG_BYTES);
}
__device__ __forceinline__ bool kargs_layout_ok() {
  return (const __attribute__((address_space(4))) char*)__builtin_amdgcn_implicitarg_ptr() -
             (const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr() == KARG_BYTES;
}
constexpr unsigned long long HOST_TIMEOUT_TICKS = 6000000000ull;  // 60 s at 100 MHz

// ------------------------------------------------------------------ small helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

__device__ __forceinline__ f4 mfma16(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Sequential chain acc = fmaf(a(k), b(k), acc), k = k0 .. k0 + K - 1 in order (the reference's
// MKL k-ascending chain), the operands of each block of B terms loaded together ahead of its
// arithmetic: LDS latency is paid once per block, not once per term.  Small register
// footprint on purpose: a callee's VGPR count is what its callers must keep clear.
template <int K, int B = 16, class FA, class FB>
__device__ __forceinline__ float fma_chain(float acc, int k0, FA&& fa, FB&& fb) {
  static_assert(K % B == 0, "block size");
#pragma unroll
  for (int blk = 0; blk < K / B; ++blk) {
    float x[B], y[B];
#pragma unroll
    for (int i = 0; i < B; ++i) {
      x[i] = fa(k0 + blk * B + i);
      y[i] = fb(k0 + blk * B + i);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < B; ++i) acc = fmaf(x[i], y[i], acc);
    __builtin_amdgcn_sched_barrier(0);
  }
  return acc;
}

// Weight element W[k][c] of a [K][64] matrix stored in B-fragment order at `base`.
__device__ __forceinline__ float wget(const float* base, int ksteps, int k, int c) {
  return base[((c >> 4) * ksteps + (k >> 2)) * 64 + ((k & 3) << 4) + (c & 15)];
}

// torch's CPU L2 norm reduction order for a 64-wide row (checked against
// torch.linalg.vector_norm on the build host): element c -> accumulator c % 8 as an FMA
// chain in ascending c, then acc0 + acc1 + ... + acc7, then sqrt.
__device__ __forceinline__ float sumsq8_finish(const float* acc8) {
  float s = acc8[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) s = s + acc8[j];
  return s;
}

// Wave-level: every lane holds x[c] (c = lane); returns sqrt(sum of squares) in torch order.
__device__ __forceinline__ float wave_norm64(float x) {
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = __shfl(x, 8 * i + j, 64);
      acc[j] = fmaf(v, v, acc[j]);
    }
  }
  return sqrtf(sumsq8_finish(acc));
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

// ------------------------------------------------------------------ inter-workgroup data
// Every array one workgroup writes and another reads inside a launch moves with agent-scope
// (sc1) global stores and loads: the hand-off protocol of MI355X_MICROARCH.md
// (inter-workgroup visibility, first table row: every storing wave drains vmcnt before the
// barrier arrival, one lane signals with an agent-scope atomic, the consumer polls with an
// sc1 load and reads after a workgroup barrier), so the grid barrier needs neither an L2
// write-back nor an L1 invalidate.  Static data (CSR, weights, graph info) use plain loads.
typedef __attribute__((address_space(1))) int g_i32;
typedef __attribute__((address_space(1))) unsigned g_u32;
typedef __attribute__((address_space(1))) float g_f32;
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(1))) unsigned long long g_u64;
typedef float v4f __attribute__((ext_vector_type(4)));
__device__ __forceinline__ int ldc(const int* a) {
  return __hip_atomic_load((g_i32*)a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ldc(const float* a) {
  return __hip_atomic_load((g_f32*)a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint8_t ldc(const uint8_t* a) {
  return __hip_atomic_load((g_u8*)a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stc(int* a, int v) {
  __hip_atomic_store((g_i32*)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stc(float* a, float v) {
  __hip_atomic_store((g_f32*)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void stc(uint8_t* a, uint8_t v) {
  __hip_atomic_store((g_u8*)a, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-byte sc1 accesses through a buffer resource on a wave-uniform base.
// The base must be wave-uniform (every caller passes an array base): it is moved to SGPRs so
// the buffer resource is scalar (no waterfall loop when the base arrived in VGPRs).
__device__ __forceinline__ void* uniform_ptr(const void* q) {
  const unsigned long long a = (unsigned long long)q;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return (void*)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ float4 ldc4(const float* base, int byte_off) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(base), 0, 0x7fffffff, 0x00020000);
  const v4f v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16 /* sc1 */);
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ float2 ldc2(const float* base, int byte_off) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(base), 0, 0x7fffffff, 0x00020000);
  typedef float v2f __attribute__((ext_vector_type(2)));
  const v2f v = __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, 16 /* sc1 */);
  return make_float2(v.x, v.y);
}
__device__ __forceinline__ void stc4(float* base, int byte_off, float4 x) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(base), 0, 0x7fffffff, 0x00020000);
  const v4f v = {x.x, x.y, x.z, x.w};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, byte_off, 0, 16 /* sc1 */);
}
constexpr int GV_WORDS = (int)(sizeof(GraphVar) / 4);
// GraphVar of graph g into `dst` (LDS), GV_WORDS threads in parallel; the caller syncs.
__device__ __forceinline__ void gv_load(KParams& p, int g, GraphVar* dst) {
  if (threadIdx.x < GV_WORDS) ((int*)dst)[threadIdx.x] = ldc((const int*)(p.gvar + g) + threadIdx.x);
}
__device__ __forceinline__ void gv_store(KParams& p, int g, const GraphVar* src) {
  if (threadIdx.x < GV_WORDS) stc((int*)(p.gvar + g) + threadIdx.x, ((const int*)src)[threadIdx.x]);
}


// ------------------------------------------------------------------ grid barrier
// Monotonic counter: every wave drains its stores (vmcnt), the workgroup syncs, one lane adds
// to the counter (agent-scope atomic) and polls it with sc1 loads; all data crossing the
// barrier is sc1 on both sides.  An error sets bit 31 of the counter (BAR_ERR) besides the
// error word: every barrier then falls through and reports it, so no workgroup needs a
// separate load of the error word on the critical path.  Bounded spin: a timeout raises
// ERR_TIMEOUT the same way, so the grid drains.
constexpr unsigned BAR_ERR = 0x80000000u;
constexpr int BAR_SHARDS = 8, BAR_STRIDE = 64;  // grid-barrier counter shards, one 256-byte line each
__device__ __forceinline__ void raise_err(KParams& p, int code) {
  // the first error wins (later ones are usually its consequences: a workgroup that gave up
  // waiting on data the failed one never produced)
  int zero = 0;
  __hip_atomic_compare_exchange_strong(p.err, &zero, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_fetch_or((g_u32*)p.bar, BAR_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Debug builds (-DMD_DEBUG_BOUNDS): index checks that raise error 1000 + site instead of
// letting a bad index reach memory.
#ifdef MD_DEBUG_BOUNDS
__device__ __forceinline__ bool md_bok(bool ok, int site) {
  if (!ok) raise_err(kp(), 1000 + site);
  return ok;
}
#define MD_BOK(cond, site) md_bok((cond), (site))
#else
#define MD_BOK(cond, site) true
#endif
// Torn-slot diagnostic build (-DMD_TORN_SLOT, make torn-slot; with MD_DEBUG_BOUNDS): the first-
// layer row reads of a speculated iteration 1 are checked against [1, dmax] instead of clamped
// to it; a blocked read is counted (md_profile buffer, step row 0, slot 70 + site: 92 own rows,
// 93 neighbour rows) and skipped.
#ifdef MD_TORN_SLOT
__device__ __forceinline__ bool md_brec(bool ok, int site) {
  KParams& p = kp();
  if (!ok && p.prof != nullptr && p.prof_cap > 0) atomicAdd(p.prof + 70 + site, 1ull);
  return ok;
}
#endif

// ------------------------------------------------------------------ dataflow mode: granules
// Single-graph rollouts in dedicated mode with the layer split run without any grid barrier
// when p.df is set (md_abi.cpp decides; MD_DF=0 keeps the barriers).  Everything one workgroup
// hands to another inside a step moves as data-tagged 8-byte granules {value bits (low word),
// tag (high word)}, each written by ONE sc1 store and polled by the consumer until its tag
// matches (MI355X_MICROARCH.md price list, handoff-1to1: one round trip, no flag, no drain):
//   step record  environment workgroup -> all: {status, n_live, confirmation, early word} of
//                step pstep, tag pstep + 1, after phase A's stores drained (replaces barrier A
//                and the tiles' read of the GraphVar)
//   H rows       tiles -> tiles: the iteration-1 / -2 embeddings, 64 granules per node row
//                (replaces barriers 1 and 2: an iteration waits for exactly its neighbours)
//   spart        tiles -> graph-head workgroup: virtual-node partial sums S0..S2
//   apart        tiles -> phase A: the arg-max partial {max, second, index, count}, written
//                after the tile's q stores drained (replaces barrier 3)
// Data of step pstep carry tag (pstep + 1) << 1; iteration-1 data that an iteration-1 prebuild
// wrote from the speculative result (before phase A confirmed it) carry that | 1, and are
// accepted only when the step record confirms that result (the step's one early word).  The
// buffer is zeroed before each launch.  Write-after-read safety without barriers: a step's
// rows and sums are read within the step, and the next step's writers start after the next
// step record, which phase A publishes only after every active tile's arg-max partial (each
// written after that tile's last read, and after the layer-1 hand-off and the graph head it
// waited for) has arrived.
constexpr int DF_REC = 0;  // record granules: status, n_live, confirmation lo / hi, early word lo / hi
__device__ __forceinline__ unsigned df_tag(int pstep) { return (unsigned)(pstep + 1) << 1; }
__device__ __forceinline__ unsigned long long* df_ap(KParams& p) { return p.df + 64; }
// Rows and virtual-node partial sums are double-buffered by step parity (the parity of a step's
// data comes from its tag): the iteration-1 prebuild of step t + 1 may start while tiles still
// read step t's rows.
__device__ __forceinline__ int df_par(unsigned tag) { return (int)(((tag & 0xffffffu) >> 1) - 1u) & 1; }
__device__ __forceinline__ unsigned long long* df_sp(KParams& p, int par) {
  return p.df + 64 + 4 * (size_t)p.df_mt + (size_t)par * 384 * p.df_mt;
}
__device__ __forceinline__ unsigned long long* df_hb(KParams& p, int l, int b, int par) {
  return p.df + 64 + 772 * (size_t)p.df_mt + (size_t)(4 * l + 2 * par + b) * 64 * p.df_n;
}
// tag of iteration-1 data a prebuild wrote from the speculative result ew (its slot in bits 24-29)
__device__ __forceinline__ unsigned df_ptag(unsigned tn, unsigned long long ew) {
  return tn | 1u | ((unsigned)(ew & 63u) << 24);
}
__device__ __forceinline__ void df_st(unsigned long long* a, float v, unsigned tag) {
  __hip_atomic_store((g_u64*)a, ((unsigned long long)tag << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool df_ok(unsigned t, unsigned ta, unsigned tb) { return t == ta || t == tb; }
// granule pair {v0, tag, v1, tag} as loaded by one 16-byte sc1 load
__device__ __forceinline__ bool df_ok4(const float4& x, unsigned ta, unsigned tb) {
  return df_ok(__float_as_uint(x.y), ta, tb) && df_ok(__float_as_uint(x.w), ta, tb);
}
// the slow path of a granule poll: true when the caller should stop (an error anywhere, or the
// time-out, which raises one); t0 = the poll's start
__device__ __forceinline__ bool df_give_up(KParams& p, unsigned long long t0, unsigned long long limit) {
  if (__hip_atomic_load((g_u32*)p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & BAR_ERR) return true;
  if (wall_clock64() - t0 > limit) {
    raise_err(p, ERR_TIMEOUT);
    return true;
  }
  return false;
}
// 16-byte granule pair at byte offset off of the (wave-uniform) base, polled until both tags
// are ta or tb (zeros when the grid gave up)
__device__ __forceinline__ float4 df_ld4(KParams& p, const float* base, int off, unsigned ta, unsigned tb) {
  float4 x = ldc4(base, off);
  if (!df_ok4(x, ta, tb)) {
    const unsigned long long t0 = wall_clock64();
    do {
      __builtin_amdgcn_s_sleep(1);
      if (df_give_up(p, t0, 400000000ull)) return make_float4(0.f, 0.f, 0.f, 0.f);
      x = ldc4(base, off);
    } while (!df_ok4(x, ta, tb));
  }
  return x;
}
// one granule, polled until its tag is ta or tb; returns its value (0 when the grid gave up)
__device__ __forceinline__ float df_ld(KParams& p, const unsigned long long* a, unsigned ta, unsigned tb) {
  unsigned long long g = __hip_atomic_load((const g_u64*)a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!df_ok((unsigned)(g >> 32), ta, tb)) {
    const unsigned long long t0 = wall_clock64();
    do {
      __builtin_amdgcn_s_sleep(1);
      if (df_give_up(p, t0, 400000000ull)) return 0.f;
      g = __hip_atomic_load((const g_u64*)a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } while (!df_ok((unsigned)(g >> 32), ta, tb));
  }
  return __uint_as_float((unsigned)g);
}
// arg-max partial of tile j written in the step whose tag is tag: {max, second, index, count}
__device__ __forceinline__ float4 df_apart(KParams& p, int j, unsigned tag) {
  const float* b = (const float*)df_ap(p);
  const float4 a = df_ld4(p, b, j * 32, tag, tag), c = df_ld4(p, b, j * 32 + 16, tag, tag);
  return make_float4(a.x, a.z, c.x, c.z);
}
// returns true (uniformly) when an error was raised anywhere in the grid.
// The arrival counter is sharded over BAR_SHARDS words on lines of their own (workgroup b adds
// to shard b % BAR_SHARDS): one-word fan-in serialises every arrival at the memory side
// (~12 ns each, MI355X_MICROARCH.md fanin row), the shards take 1/8 of them each.  Wave 0
// polls every shard and the error word in one instruction; `target` counts this workgroup's
// barriers.  Speculative workgroups (blockIdx >= n_main) take no part.
__device__ __forceinline__ void grid_arrive(KParams& p, unsigned& target) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  target += 1;
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add((g_u32*)(p.bars + BAR_STRIDE * (blockIdx.x % BAR_SHARDS)), 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
// Waits for the barrier `target` (after grid_arrive); *flag = 1 (uniform) when an error was
// raised anywhere, as grid_sync.  With `watch` set it also returns early when the 8-byte word
// *watch differs from `seen` (the new value in *seen_out, LDS): the return value is then 2, else
// 1 (released or error).  One workgroup barrier either way.
__device__ __forceinline__ int grid_wait(KParams& p, unsigned target, int* flag, const unsigned long long* watch = nullptr,
                                         unsigned long long seen = 0ull, unsigned long long* seen_out = nullptr) {
  int* code = flag + 2;  // the word after the caller's flag pair (misc[63] for bflag = misc + 61)
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned want = lane < BAR_SHARDS ? target * (unsigned)((p.n_main - lane + BAR_SHARDS - 1) / BAR_SHARDS) : 0u;
    const g_u32* w = (const g_u32*)(lane < BAR_SHARDS ? p.bars + BAR_STRIDE * lane : p.bar);
    const unsigned long long t0 = wall_clock64();
    int err = 0, res = 1;
    while (true) {
      const unsigned v = lane <= BAR_SHARDS ? __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
      const bool lag = lane < BAR_SHARDS && v < want;
      if (__ballot(lane == BAR_SHARDS && (v & BAR_ERR))) { err = 1; break; }
      if (!__ballot(lag)) break;
      if (watch != nullptr) {
        const unsigned long long x = __hip_atomic_load((const g_u64*)watch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (x != seen) {
          if (lane == 0) *seen_out = x;
          res = 2;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > (p.h_req != nullptr ? HOST_TIMEOUT_TICKS : BARRIER_TIMEOUT_TICKS)) {
        if (lane == 0) raise_err(p, ERR_TIMEOUT);
        err = 1;
        break;
      }
    }
    if (lane == 0) {
      *flag = err;
      *code = res;
    }
  }
  __syncthreads();
  return *code;
}
__device__ __forceinline__ bool grid_sync(KParams& p, unsigned& target, int* flag) {
  grid_arrive(p, target);
  grid_wait(p, target, flag);
  return *flag != 0;
}

// ------------------------------------------------------------------ block reductions
__device__ __forceinline__ int block_sum_int(int v, int* tmp) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane_id() == 0) tmp[wave_id()] = v;
  __syncthreads();
  int s = 0;
#pragma unroll
  for (int w = 0; w < NTHREADS / 64; ++w) s += tmp[w];
  __syncthreads();
  return s;
}

__device__ __forceinline__ int block_max_int(int v, int* tmp) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  __syncthreads();
  if (lane_id() == 0) tmp[wave_id()] = v;
  __syncthreads();
  int s = tmp[0];
#pragma unroll
  for (int w = 1; w < NTHREADS / 64; ++w) s = max(s, tmp[w]);
  __syncthreads();
  return s;
}

__device__ __forceinline__ long long block_sum_ll(long long v, long long* tmp) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane_id() == 0) tmp[wave_id()] = v;
  __syncthreads();
  long long s = 0;
#pragma unroll
  for (int w = 0; w < NTHREADS / 64; ++w) s += tmp[w];
  __syncthreads();
  return s;
}

// Exclusive scan over the block (thread order); returns this thread's offset, total in *tot.
__device__ __forceinline__ int block_excl_scan(int v, int* tmp, int* tot) {
  const int lane = lane_id(), w = wave_id();
  int x = v;
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  __syncthreads();
  if (lane == 63) tmp[w] = x;
  __syncthreads();
  int base = 0, all = 0;
  for (int i = 0; i < NTHREADS / 64; ++i) {
    if (i < w) base += tmp[i];
    all += tmp[i];
  }
  __syncthreads();
  *tot = all;
  return base + x - v;
}

#include "md_env.h"

// Sum of one column of a transposed tile (a[row], rows 0..15) over its first nv rows (the valid
// rows are a prefix), added in row order; every LDS read is issued before the first add (a
// break-at-the-first-invalid-row loop is a chain of dependent LDS round trips).
__device__ __forceinline__ float col_sum16(const float* a, int nv) {
  float v[TILE];
#pragma unroll
  for (int r = 0; r < TILE; ++r) v[r] = a[r];
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < TILE; ++r)
    if (r < nv) s = s + v[r];
  return s;
}
// col_sum16 of K-row k of a rotated block (rows read at their rotated positions, summed in
// row order).
__device__ __forceinline__ float col_sum16_p2(const float* blk, int k, int nv) {
  float v[TILE];
#pragma unroll
  for (int r = 0; r < TILE; ++r) v[r] = blk[p2o(k, r)];
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < TILE; ++r)
    if (r < nv) s = s + v[r];
  return s;
}
__device__ __forceinline__ int tile_rows_valid(const int* rows) {
  int nv = 0;
#pragma unroll
  for (int r = 0; r < TILE; ++r) nv += rows[r] >= 0;
  return nv;
}

// Merge arg-max partial (m2, s2, i2, c2) into (bm, bs, bi, bc); c = 0 marks an empty partial.
__device__ __forceinline__ void argmax_combine(float& bm, float& bs, int& bi, int& bc, float m2, float s2,
                                               int i2, int c2) {
  if (bc == 0) {
    bm = m2; bs = s2; bi = i2; bc = c2;
  } else if (m2 > bm) {
    bs = fmaxf(bm, s2);
    bm = m2; bi = i2; bc = c2;
  } else if (m2 == bm) {
    bc += c2;
    bi = min(bi, i2);
    bs = fmaxf(bs, s2);
  } else {
    bs = fmaxf(bs, m2);
  }
}

// Host selection hand-shake for graph g (ties at the max Q, or a multi-node step): publish
// the graph's Q row, its max and tie count to mapped host memory and raise the request tag;
// the host answers with its selection callback (the reference's np.argsort pick).  All host
// memory traffic is system-scope (uncached) and in program order over the link, so no cache
// write-back / invalidate is needed (those would flush the whole L2 under the running grid).
__device__ __forceinline__ unsigned host_tag(KParams& p, int npred) {
  return (p.launch_seq << 16) ^ (unsigned)(npred + 1);
}
__device__ __noinline__ void host_request(KParams&, const GraphInfo gi, int g, int npred, float qmax, int ntie) {
  KParams& p = kp();  // kernel arguments through the implicit-argument SGPRs (uniform)
  for (int x = threadIdx.x; x < gi.n; x += NTHREADS)
    __hip_atomic_store(p.h_q + gi.node_off + x, ldc(p.q + gi.node_off + x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (threadIdx.x == 0) {
    __hip_atomic_store(p.h_chk + 2 * g, qmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(p.h_chk + 2 * g + 1, __int_as_float(ntie), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(p.h_req + g, host_tag(p, npred), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// End-game requests carry bit 15 (n < 32768, so npred + 1 never sets it).
__device__ __forceinline__ unsigned host_tag_eg(KParams& p, int npred, bool endgame) {
  return host_tag(p, npred) ^ (endgame ? 0x8000u : 0u);
}
// Thread 0 only: whether the host answered request `npred` of graph g.  Returns the number of
// actions, 0 when not answered yet, -1 on a bad answer; host_copy_actions then moves them.
__device__ __forceinline__ int host_answer(KParams& p, const GraphInfo& gi, int g, int npred, bool endgame = false) {
  if (__hip_atomic_load(p.h_ans + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != host_tag_eg(p, npred, endgame))
    return 0;
  const int k = __hip_atomic_load(p.h_nact + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return k <= 0 || k > gi.n ? -1 : k;
}
// Whole workgroup, after the answer's count was seen: the k actions from mapped host memory to
// p.pend, one load per thread (each is a bus round trip: a stepRatio or end-game answer no longer
// waits k of them back to back).  Ends with the workgroup's stores drained.
__device__ __forceinline__ void host_copy_actions(KParams& p, const GraphInfo& gi, int k) {
  for (int i = threadIdx.x; i < k; i += NTHREADS)
    __hip_atomic_store(p.pend + gi.node_off + i,
                       __hip_atomic_load(p.h_act + gi.node_off + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}
// K2 end-game (unit cost): when every live node has residual degree 1 in both layers, the
// graph is a set of disjoint pairs joined in both layers, every live node's Q is the same
// number (same inputs, same arithmetic: checked on 676 such states of 40 GMM rollouts,
// scripts/k2_check.py), and the reference's pick np.argsort(-q)[0] depends only on which
// nodes are live.  Removing a node isolates its partner and leaves the other pairs as they
// were, so the host can run every remaining step's pick in one hand-shake (the same numpy
// routine on the same masked rows, live nodes at one value) instead of one forward pass and
// one hand-shake per step.  The request row carries each live node's partner (int bits)
// and -inf elsewhere; the tie-count word carries -n_live.
__device__ __noinline__ void endgame_request(KParams&, const GraphInfo gi, int g, int npred, int nlive) {
  KParams& p = kp();
  const int* rp = p.rowptr[0] + gi.roff[0];
  const int* adj = p.adj[0] + gi.coff[0];
  const uint8_t* ca = p.calive[0] + gi.coff[0];
  const int* deg = p.deg[0] + gi.node_off;
  for (int x = threadIdx.x; x < gi.n; x += NTHREADS) {
    float v = NEG_INF;
    if (ldc(deg + x) > 0) {
      int part = -1;
      for (int i = rp[x]; i < rp[x + 1]; ++i)
        if (ldc(ca + i)) {
          part = adj[i];
          break;
        }
      v = __int_as_float(part);
    }
    __hip_atomic_store(p.h_q + gi.node_off + x, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x == 0) {
    __hip_atomic_store(p.h_chk + 2 * g, 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(p.h_chk + 2 * g + 1, __int_as_float(-nlive), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(p.h_req + g, host_tag_eg(p, npred, true), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool endgame_state(KParams& p, const GraphInfo& gi, const GraphVar& gv) {
  return p.endgame && p.node_w == nullptr && gi.n < 32768 && gv.status == ST_RUN && gv.n_live > 0 &&
         gv.dmax[0] == 1 && gv.dmax[1] == 1;
}

// stepRatio picks on the device: np.argsort(-q)[:k] (U/MultiDismantler_torch.py:725) is the
// unique descending order of the k largest Q when those are distinct and the k-th is above the
// (k+1)-th -- then no tie order of numpy's sort can matter.  Radix select of the k-th largest
// key (four 8-bit digit passes over the graph's Q row), a count of the keys equal to it, the k
// candidates collected and bitonic-sorted in LDS, a check for equal neighbours.  Returns k with
// the picks in p.pend, or 0 (a tie at or above the k-th value, or k > TOPK_MAX): the host's
// numpy routine then decides, as for every tie.  k <= the live nodes (the finite Q), so the
// k-th largest is above the masked -inf rows.  Grid-wide step only: the tile scratch of
// workgroup 0 is free at phase A there.
constexpr int TOPK_MAX = 1024;
__device__ __forceinline__ unsigned topk_key(float f) {
  const unsigned u = __float_as_uint(f == 0.f ? 0.f : f);  // (-0 == +0 for numpy's compare)
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);       // unsigned order = float order
}
__device__ __noinline__ int device_topk(KParams&, const GraphInfo gi, int k) {
  KParams& p = kp();
  const float* q = p.q + gi.node_off;
  const int n = gi.n;
  int* const hist = (int*)(lds_base() + L_SCR);  // [256]
  int* const ctl = hist + 256;                    // [8]: prefix, need, equal count, collected
  unsigned* const ck = (unsigned*)(ctl + 8);      // [TOPK_MAX] keys
  int* const ci = (int*)(ck + TOPK_MAX);          // [TOPK_MAX] node ids
  if (k < 1 || k > TOPK_MAX || k > n) return 0;
  const int lane = lane_id();
  unsigned prefix = 0u, pmask = 0u;
  int need = k, eq = 0;
  for (int shift = 24; shift >= 0; shift -= 8) {
    if (threadIdx.x < 256) hist[threadIdx.x] = 0;
    __syncthreads();
    for (int x = threadIdx.x; x < n; x += NTHREADS) {
      const unsigned key = topk_key(ldc(q + x));
      if ((key & pmask) == prefix) atomicAdd(hist + ((key >> shift) & 255u), 1);
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      // the digit holding the need-th largest key: lane l sums digits 255 - 4l .. 252 - 4l,
      // an inclusive scan over the lanes from the top digit down
      const int b0 = 255 - 4 * lane;
      const int h0 = hist[b0], h1 = hist[b0 - 1], h2 = hist[b0 - 2], h3 = hist[b0 - 3];
      const int s = h0 + h1 + h2 + h3;
      int incl = s;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
      }
      const int before = incl - s;
      const unsigned long long m = __ballot(incl >= need);
      const int hit = __ffsll((long long)m) - 1;  // first lane whose range reaches rank `need`
      if (lane == hit) {
        int c = before, d = b0, hd = h0;
        const int hs[4] = {h0, h1, h2, h3};
        for (int t = 0; t < 4; ++t) {
          d = b0 - t;
          hd = hs[t];
          if (c + hd >= need) break;
          c += hd;
        }
        ctl[0] = d;
        ctl[1] = need - c;  // rank inside the digit's group
        ctl[2] = hd;
      }
    }
    __syncthreads();
    prefix |= (unsigned)ctl[0] << shift;
    pmask |= 255u << shift;
    need = ctl[1];
    eq = ctl[2];
    __syncthreads();
  }
  // prefix is the k-th largest key; eq keys equal it, k - need of them are larger
  if (eq != 1) return 0;  // a tie at the k-th value (need == 1 then: k - 1 keys above it)
  if (threadIdx.x == 0) ctl[3] = 0;
  for (int i = threadIdx.x; i < TOPK_MAX; i += NTHREADS) ck[i] = 0u;  // (pads sort last)
  __syncthreads();
  for (int x = threadIdx.x; x < n; x += NTHREADS) {
    const unsigned key = topk_key(ldc(q + x));
    if (key >= prefix) {
      const int at = atomicAdd(ctl + 3, 1);
      if (at < TOPK_MAX) {
        ck[at] = key;
        ci[at] = x;
      }
    }
  }
  __syncthreads();
  if (ctl[3] != k) return 0;  // (cannot happen: k - 1 above, one equal)
  // bitonic sort, descending by key, over the next power of two >= k
  int m2 = 1;
  while (m2 < k) m2 <<= 1;
  for (int size = 2; size <= m2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < m2; i += NTHREADS) {
        const int jx = i ^ stride;
        if (jx > i) {
          const bool desc = (i & size) == 0;
          const unsigned a = ck[i], b = ck[jx];
          if (desc ? a < b : a > b) {
            ck[i] = b;
            ck[jx] = a;
            const int t = ci[i];
            ci[i] = ci[jx];
            ci[jx] = t;
          }
        }
      }
      __syncthreads();
    }
  }
  bool dup = false;
  for (int i = threadIdx.x; i + 1 < k; i += NTHREADS) dup |= ck[i] == ck[i + 1];
  if (__syncthreads_or(dup)) return 0;
  for (int i = threadIdx.x; i < k; i += NTHREADS)
    __hip_atomic_store(p.pend + gi.node_off + i, ci[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return k;
}

// Synchronous form (one graph per launch: nothing else could run meanwhile): request, then
// wait for the answer.  Returns the number of actions (0 on error; the error word is set).
__device__ __noinline__ int host_handshake(KParams&, const GraphInfo gi, int g, int npred, float qmax, int ntie, int* misc,
                                           bool endgame = false) {
  KParams& p = kp();
  if (endgame) endgame_request(p, gi, g, npred, ntie);
  else host_request(p, gi, g, npred, qmax, ntie);
  if (threadIdx.x == 0) {
    const unsigned long long t0 = wall_clock64();
    int k;
    while ((k = host_answer(p, gi, g, npred, endgame)) == 0) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > HOST_TIMEOUT_TICKS) {
        k = -1;
        break;
      }
    }
    if (k < 0) raise_err(p, ERR_HOST);
    misc[3] = k;
  }
  __syncthreads();
  const int k = misc[3];
  if (k > 0) host_copy_actions(p, gi, k);
  return max(k, 0);
}

// K2 end-game answer of k actions (LDS mode): applied in one pass when the state has the
// end-game form (env_endgame_apply; env_step then gets PEND_APPLIED and only recomputes the
// features).  Stages the state first when it is not (staged: in LDS afterwards either way).
__device__ __forceinline__ bool eg_apply(KParams& p, const GraphInfo& gi, int k, bool& staged) {
  if (!(p.endgame & 2) || k < 2) return false;
  const bool ok = env_endgame_apply(p, gi, k, staged) >= 0;
  staged = true;
  return ok;
}

// A graph's final removal trace [0, steps) to the mapped host mirrors (p.h_tra / p.h_trr), so
// md_rollout reads it without a copy after the launch.  Launches of at most PUB_EXIT_MAX graphs
// publish in kernel_exit, once every workgroup is done (a system-scope store during the
// single-graph rollout showed as ~0.25 MB of extra WRITE_SIZE each, no time); queue launches
// publish each graph as it becomes terminal (the workgroup that ended it).  Whole workgroup;
// the trace slots may have been written by other threads or workgroups (agent-coherent
// stores).
constexpr int PUB_EXIT_MAX = 16;
__device__ __forceinline__ void trace_publish(KParams& p, const GraphInfo& gi, int steps) {
  if (p.h_tra == nullptr) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < min(steps, gi.n); i += NTHREADS) {
    __hip_atomic_store(p.h_tra + gi.node_off + i, ldc(p.tr_action + gi.node_off + i), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(p.h_trr + gi.node_off + i, ldc(p.tr_rank + gi.node_off + i), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Phase A of one graph: reduce the previous prediction, then apply / MCC / features.
// team_out (grid-wide environment step): when the step would run in global mode, phase A stops
// once the actions are known: {pend_n, pend_first, 1} in team_out, the GraphVar left in LDS for
// the caller to finish (team_env_step); team_out[2] = 0 otherwise.
__device__ __forceinline__ bool phase_a(KParams&, int g, bool have_q, float* lds, bool staged, int* team_out = nullptr) {
  KParams& p = kp();  // kernel arguments through the implicit-argument SGPRs (uniform)
  GraphVar& gv = *(GraphVar*)(lds + L_GV);
  int* misc = (int*)(lds + L_MISC);
  const GraphInfo gi = p.ginfo[g];
  // a dedicated environment workgroup that already stepped this graph in this launch holds
  // its current GraphVar in LDS (nobody else writes it during a launch)
  if (!(staged && p.n_env > 0)) gv_load(p, g, &gv);
  if (threadIdx.x == 0) {
    misc[5] = 0;
    misc[56] = misc[57] = 0;  // the speculative result this phase A takes (iteration-1 prebuild)
    if (team_out != nullptr) team_out[2] = 0;
  }
  __syncthreads();
  int pend_n = 0, pend_first = -1;
  bool eg_ans = false;  // the actions answer an end-game request
  bool stop = false;
  if (gv.status == ST_WAIT_HOST) {
    // asynchronous hand-shake (several graphs per launch): the graph sat out the steps since
    // its request while the others went on; poll the host's answer once per step
    if (threadIdx.x == 0) {
      int k = host_answer(p, gi, g, gv.npred, gv.ntie < 0);  // ntie < 0: an end-game request
      if (k == 0 && wall_clock64() - gv.t_req > HOST_TIMEOUT_TICKS) k = -1;
      if (k < 0) raise_err(p, ERR_HOST);
      misc[3] = k;
    }
    __syncthreads();
    if (misc[3] <= 0) return staged;
    pend_n = misc[3];
    eg_ans = gv.ntie < 0;
    host_copy_actions(p, gi, pend_n);
  } else if (gv.status != ST_RUN) {
    return staged;
  } else if (have_q) {
    float bm = NEG_INF, bs = NEG_INF;
    int bi = 0x7fffffff, bc = 0;
    if (threadIdx.x < 64) {
      // arg-max over the graph's tile partials {max, second, min index at max, count at max}:
      // lanes combine strided tiles, then a butterfly; every combine step is max / min / sum,
      // so the result does not depend on the order.
      const int lane = threadIdx.x;
      const int nt = (gv.n_live + TILE - 1) / TILE;
      for (int j = lane; j < nt; j += 64) {
        // (dataflow mode: the partials of the previous step, polled as tagged granules)
        const float4 ap = p.df != nullptr ? df_apart(p, j, (unsigned)misc[60] << 1) : ldc4(p.apart, (gi.tile_off + j) * 16);
        const int c = __float_as_int(ap.w);
        if (c == 0) continue;
        argmax_combine(bm, bs, bi, bc, ap.x, ap.y, __float_as_int(ap.z), c);
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float m2 = __shfl_xor(bm, o, 64), s2 = __shfl_xor(bs, o, 64);
        const int i2 = __shfl_xor(bi, o, 64), c2 = __shfl_xor(bc, o, 64);
        if (c2 != 0) argmax_combine(bm, bs, bi, bc, m2, s2, i2, c2);
      }
    } else if ((int)threadIdx.x < 64 + p.n_spec && p.df == nullptr) {
      // speculative results' tags, read beside the partials (env_step matches them against
      // the chosen node without a round trip of its own); the previous step's request's slots
      const g_u64* tp = (const g_u64*)(p.sres + (size_t)spec_slot_index(threadIdx.x - 64, misc[60] - 1) * p.sres_stride);
      unsigned long long* pre = (unsigned long long*)(lds + L_PREF) + 2 * (threadIdx.x - 64);
      pre[0] = __hip_atomic_load(tp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      pre[1] = __hip_atomic_load(tp + SRES_STARTED / 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (p.df != nullptr) {
      // dataflow mode: phase A starts polling the partials as the step's tiles start, so the
      // tags are read once every partial has arrived (as fresh as beside barrier mode's partials)
      if (p.prof != nullptr && threadIdx.x == 0 && misc[60] - 1 < p.prof_cap)  // diagnostics: slot 11 of the step
        p.prof[(size_t)(misc[60] - 1) * PROF_SLOTS + 11] = wall_clock64();
      __syncthreads();
      if (threadIdx.x >= 64 && (int)threadIdx.x < 64 + p.n_spec) {
        const g_u64* tp = (const g_u64*)(p.sres + (size_t)spec_slot_index(threadIdx.x - 64, misc[60] - 1) * p.sres_stride);
        unsigned long long* pre = (unsigned long long*)(lds + L_PREF) + 2 * (threadIdx.x - 64);
        // (and the features tag and aggregates: a result taken with its features published
        // lets env_step publish the step record at its slot check)
        int* pf = (int*)(lds + L_PREF) + PREF_FEAT + 8 * (threadIdx.x - 64);
        const unsigned long long ft = __hip_atomic_load(tp + SRES_FEAT / 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int fa[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) fa[i] = ldc((const int*)tp + 12 + i);
        pre[0] = __hip_atomic_load(tp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pre[1] = __hip_atomic_load(tp + SRES_STARTED / 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pf[0] = (int)(unsigned)ft;
        pf[1] = (int)(unsigned)(ft >> 32);
#pragma unroll
        for (int i = 0; i < 6; ++i) pf[2 + i] = fa[i];
      }
    }
    if (threadIdx.x == 0) {
      const int t = gv.npred;
      if (t < gi.n) {
        int* ts = p.tr_stat + (size_t)(gi.node_off + t) * 4;
        ts[0] = gv.n_live;
        ts[1] = gv.alive[0];
        ts[2] = gv.alive[1];
        ts[3] = bc;
        p.tr_q[(size_t)(gi.node_off + t) * 2 + 0] = bm;
        p.tr_q[(size_t)(gi.node_off + t) * 2 + 1] = bm - bs;
      }
      gv.npred = t + 1;
      gv.ntie = bc;
      gv.qmax = bm;
      gv.gap = bm - bs;
      gv.argmax = bc == 1 ? bi : -1;
      misc[1] = bi;
      misc[2] = bc;
      misc[5] = 1;  // speculative tags pre-read in L_PREF
    }
    __syncthreads();
    if (p.run_mode == RUN_PREDICT) {
      if (threadIdx.x == 0) gv.status = ST_PAUSED;
      stop = true;
    } else if (p.host_select && p.dev_topk && team_out != nullptr && p.nglist == 1 &&
               (pend_n = device_topk(p, gi, min(p.sel_step, gv.n_live))) > 0) {
      // (stepRatio picks of the grid-wide step taken on the device: see device_topk; with
      // fewer live nodes than picks only the live ones -- the graph is terminal once they are
      // gone, so the masked picks after them are never applied)
    } else if (p.host_select || misc[2] != 1) {
#ifndef MD_NO_HS
      if (p.h_req != nullptr) {
#else
      if (false) {
#endif
        // ask the host without ending the launch; the actions land in p.pend
        if (p.nglist > 1) {
          // several graphs: the others keep stepping while the host answers
          host_request(p, gi, g, gv.npred, gv.qmax, gv.ntie);
          if (threadIdx.x == 0) {
            gv.status = ST_WAIT_HOST;
            gv.t_req = wall_clock64();
          }
          stop = true;
        } else {
          pend_n = host_handshake(p, gi, g, gv.npred, gv.qmax, gv.ntie, misc);
          stop = pend_n <= 0;
        }
      } else {
        if (threadIdx.x == 0) gv.status = ST_NEED_HOST;
        stop = true;
      }
    } else {
      pend_n = 1;
      pend_first = misc[1];
    }
  } else {
    pend_n = gv.npend;
  }
  __syncthreads();
  unsigned long long cw = 0ull;  // the prebuild confirmation (see below)
  if (!stop) {
    const int et = gi.e[0] + gi.e[1];
    const bool fits = phase_a_fits_lds(gi.n, et) && !(p.variant & 64);  // 64: force global mode (tests)
    if (team_out != nullptr && !fits) {
      if (threadIdx.x == 0) {
        team_out[0] = pend_n;
        team_out[1] = pend_first;
        team_out[2] = 1;
      }
      __syncthreads();
      return staged;
    }
    float* area = lds + L_W;
    bool was_staged = staged && fits;
    staged = fits;
    if (eg_ans && fits && eg_apply(p, gi, pend_n, was_staged)) pend_first = PEND_APPLIED;
    int err = fits ? env_step<false>(p, gi, gv, area, pend_n, pend_first, lds, was_staged)
                   : env_step<true>(p, gi, gv, area, pend_n, pend_first, lds, false);
    // the prebuild confirmation: the state after this phase A is exactly the speculative
    // result published early (one action, taken from it; an end-game below withdraws it)
    cw = ((unsigned long long)(unsigned)misc[57] << 32) | (unsigned)misc[56];
    if (err || pend_n != 1) cw = 0ull;
    if (threadIdx.x == 0) {
      gv.npend = 0;
      if (err) raise_err(p, err);
      const bool term = gv.alive[0] == 0 || gv.alive[1] == 0;
      if (term) gv.status = ST_TERMINAL;
      else if (p.run_mode == RUN_STEP) gv.status = ST_PAUSED;
      else gv.status = ST_RUN;
    }
    __syncthreads();
    if (!err && p.run_mode == RUN_ROLLOUT && p.h_req != nullptr && endgame_state(p, gi, gv)) {
      // K2 end-game: the host picks every remaining removal in one hand-shake (no forward
      // pass for these steps, no prediction recorded)
      if (p.nglist > 1) {
        endgame_request(p, gi, g, gv.npred, gv.n_live);
        if (threadIdx.x == 0) {
          gv.status = ST_WAIT_HOST;
          gv.ntie = -1;
          gv.t_req = wall_clock64();
        }
      } else {
        const int k = host_handshake(p, gi, g, gv.npred, 0.f, gv.n_live, misc, true);
        cw = 0ull;
        if (k > 0) {
          err = fits ? env_step<false>(p, gi, gv, area, k, eg_apply(p, gi, k, staged) ? PEND_APPLIED : -1, lds, true)
                     : env_step<true>(p, gi, gv, area, k, -1, lds, false);
          if (threadIdx.x == 0) {
            if (err) raise_err(p, err);
            gv.status = gv.alive[0] == 0 || gv.alive[1] == 0 ? ST_TERMINAL : ST_RUN;
          }
        }
      }
    }
  }
  __syncthreads();
  // (phase A never starts on a terminal graph)
  if (gv.status == ST_TERMINAL && p.nglist > PUB_EXIT_MAX) trace_publish(p, gi, gv.steps);
  gv_store(p, g, &gv);
  if (p.pre_cw != nullptr && threadIdx.x == 0)  // every phase A: a stale confirmation must not match
    __hip_atomic_store((g_u64*)p.pre_cw, cw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (p.df != nullptr && threadIdx.x == 0) {  // dataflow mode: the confirmation goes into the step record
    misc[54] = (int)(unsigned)cw;
    misc[55] = (int)(unsigned)(cw >> 32);
  }
  __syncthreads();
  return staged;
}

// Diagnostic timestamp into a profiled step's slots (ts == nullptr: off).
#define TSTAMP(k)                                                  \
  do {                                                             \
    if (ts != nullptr && threadIdx.x == 0) ts[k] = wall_clock64(); \
  } while (0)

// ------------------------------------------------------------------ tile pieces
// Gather for one tile: waves 0-3 layer 0, 4-7 layer 1; each wave handles rows 4*(w&3)..+3
// concurrently, one 16-lane group per row, every lane owning 4 features (float4 loads).
// it == 1: previous embedding = first-layer table (by degree, unit cost) or static input.
// Iteration 1, unit cost: first-layer rows by residual degree d (row d of the returned base).
// The precomputed table of the step's dmax (md_h0_kernel, at load) when it exists -- phase A
// then copies nothing -- else the graph's own table, rebuilt by phase A.  The dmax load goes
// out beside the degree loads it is needed with.
__device__ __forceinline__ const float* first_layer_rows(KParams& p, const GraphInfo& gi, int l) {
  if (p.h0g != nullptr) {
    const int dm = ldc(&p.gvar[gi.gidx].dmax[l]);
    if (dm >= 1 && dm <= p.h0g_dm) return p.h0g + (h0g_row(dm, 1) - 1) * EMB;  // row d at base + d rows
  }
  return p.h0tab[l] + (size_t)gi.node_off * EMB;
}

__device__ __noinline__ void gather_tile(KParams&, const GraphInfo gi, int it, const int*, float*) {
  const int* const rows = (const int*)(lds_base() + L_SCR + S_ROW);
  float* const scr = lds_base() + L_SCR;

  KParams& p = kp();  // kernel arguments through the implicit-argument SGPRs (uniform)
  const int w = wave_id(), l = w >> 2, lane = lane_id();
  const int grp = lane >> 4, qd = lane & 15;
  const int* rp = p.rowptr[l] + gi.roff[l];
  const int* adj = p.adj[l] + gi.coff[l];
  const uint8_t* ca = p.calive[l] + gi.coff[l];
  const int* deg = p.deg[l] + gi.node_off;
  const float* hp;
  bool table = false;
  if (it == 1) {
    table = p.node_w == nullptr;
    hp = table ? first_layer_rows(p, gi, l) : p.h0tab[l] + (size_t)gi.node_off * EMB;
  } else {
    hp = p.H[l][(it - 2) & 1] + (size_t)gi.node_off * EMB;
  }
  const int r = 4 * (w & 3) + grp;
  const int v = rows[r];
  int rb = 0, re = 0;
  float4 own = {0.f, 0.f, 0.f, 0.f}, acc = {0.f, 0.f, 0.f, 0.f};
  if (v >= 0) {
    rb = rp[v];
    re = rp[v + 1];
    const int ov = table ? ldc(deg + v) : v;
    if (MD_BOK(v < gi.n && ov >= 0 && ov < gi.n, 1)) own = ldc4(hp, ov * 256 + qd * 16);
  }
  int nch = (re - rb + 15) >> 4;
  nch = max(nch, __shfl_xor(nch, 16, 64));
  nch = max(nch, __shfl_xor(nch, 32, 64));
  for (int ch = 0; ch < nch; ++ch) {
    const int e = rb + 16 * ch + qd;
    int nb = -1;
    if (e < re && ldc(ca + e)) nb = adj[e];
    if (table && nb >= 0) nb = ldc(deg + nb);
    const unsigned long long m = __ballot(nb >= 0);
    unsigned gm = (unsigned)(m >> (16 * grp)) & 0xFFFFu;
    // the alive neighbours in CSR order (== reference in_edges order), 4 rows x 4 loads in flight
    while (__any(gm != 0)) {
      int j[4] = {-1, -1, -1, -1};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (gm) {
          const int b = __builtin_ctz(gm);
          gm &= gm - 1;
          j[k] = b;
        }
      }
      int src[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) src[k] = __shfl(nb, 16 * grp + (j[k] < 0 ? 0 : j[k]), 64);
      float4 x[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) x[k] = j[k] >= 0 ? ldc4(hp, src[k] * 256 + qd * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (j[k] >= 0) {
          acc.x = acc.x + x[k].x;
          acc.y = acc.y + x[k].y;
          acc.z = acc.z + x[k].z;
          acc.w = acc.w + x[k].w;
        }
      }
    }
  }
  float* atp = scr + S_P + l * 64 * LDT;
  float* atx = scr + S_X + l * 64 * LDT;
  const int c = 4 * qd;
  atp[(c + 0) * LDT + r] = acc.x;
  atp[(c + 1) * LDT + r] = acc.y;
  atp[(c + 2) * LDT + r] = acc.z;
  atp[(c + 3) * LDT + r] = acc.w;
  atx[(c + 0) * LDT + r] = own.x;
  atx[(c + 1) * LDT + r] = own.y;
  atx[(c + 2) * LDT + r] = own.z;
  atx[(c + 3) * LDT + r] = own.w;
}

// Alive neighbour lists of the tile's rows for both layers (waves 0-3: layer 0, 4-7: layer
// 1), in CSR order (= reference in_edges order), kept in LDS for the three iterations of a
// step.  Header (ints at S_NBH): off[2][16], cnt[2][16] (alive, per row), rawb[2][16],
// rawc[2][16] (CSR extent), tot[2].  Returns false when a layer has more than NB_CAP alive
// entries (the tile then uses gather_tile).
// Killed-edge set of an iteration-1 prebuild (CSR positions of one layer, open addressing in LDS).
constexpr int KH_SIZE = 1024;
__device__ __forceinline__ unsigned kh_slot(int key) { return ((unsigned)key * 2654435761u) >> 22; }
__device__ __forceinline__ void kh_insert(lds_i32* h, int key) {
  unsigned i = kh_slot(key);
  while (true) {
    const int prev = uf_cas(h, (int)i, -1, key);
    if (prev == -1 || prev == key) return;
    i = (i + 1) & (KH_SIZE - 1);
  }
}
__device__ __forceinline__ bool kh_has(const lds_i32* h, int key) {
  unsigned i = kh_slot(key);
  while (true) {
    const int v = h[i];
    if (v == key) return true;
    if (v == -1) return false;
    i = (i + 1) & (KH_SIZE - 1);
  }
}

// nbo: the header and lists at S_NBH + nbo / S_NBL + nbo (a paired tile's second list region),
// tmpo: 8 words of wave totals at that scratch offset.
__device__ __noinline__ bool build_nb_lists(KParams&, const GraphInfo gi, const int*, float*,
                                            unsigned long long* ts, int L, bool killed_set = false,
                                            int nbo = 0, int tmpo = S_RED) {
  float* const scr = lds_base() + L_SCR;

  KParams& p = kp();  // kernel arguments through the implicit-argument SGPRs (uniform)
  // L < 0: both layers (waves 0-3 layer 0, 4-7 layer 1); L = 0 / 1: that layer, all waves
  const int NT = L < 0 ? 256 : NTHREADS;
  const int w = wave_id(), l = L < 0 ? w >> 2 : L, lane = lane_id(), t = L < 0 ? threadIdx.x & 255 : threadIdx.x;
  lds_i32* hdr = (lds_i32*)(int*)(scr + S_NBH + nbo);
  lds_i32* tmp = (lds_i32*)(int*)(scr + tmpo);  // [2][4] wave totals
  lds_u16* nbl = (lds_u16*)(uint16_t*)(scr + S_NBL + nbo) + l * NB_CAP;
  const int* adj = p.adj[l] + gi.coff[l];
  const uint8_t* ca = p.calive[l] + gi.coff[l];
  // killed_set: CSR positions killed by the step in flight (an iteration-1 prebuild during phase
  // A: its write-back may or may not have reached these flags yet) count as dead
  const lds_i32* kh = killed_set ? (const lds_i32*)(int*)(scr + S_M) : nullptr;
  // rows' CSR begin / extent are in hdr[64 + 16 l + r] / hdr[96 + 16 l + r] (from the live list)
  TSTAMP(60);
  // CSR-extent prefix per row in LDS (a per-thread array indexed at run time would live in
  // scratch memory)
  lds_i32* pre = hdr + 136 + l * 17;
  if (t < 16) {
    // 16-lane inclusive scan of the extents
    int a = hdr[96 + l * 16 + t];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const int y = __shfl_up(a, o, 64);
      if (t >= o) a += y;
    }
    pre[t + 1] = a;
    if (t == 0) pre[0] = 0;
  }
  __syncthreads();
  TSTAMP(61);
  const int T = pre[16];
  const int chunk = (T + NT - 1) / NT;
  const int i0 = min(T, t * chunk), i1 = min(T, i0 + chunk);
  // my entries: alive flags and neighbour ids, the first four of them with all their loads in
  // flight together and kept in registers for the second pass
  int keep = 0;
  int r = 0;
  while (r < 15 && pre[r + 1] <= i0) ++r;
  const int r0 = r;
  int posv[4], nbv[4], fl[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = i0 + k;
    posv[k] = -1;
    if (i < i1) {
      while (pre[r + 1] <= i) ++r;
      posv[k] = hdr[64 + l * 16 + r] + (i - pre[r]);
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    fl[k] = 0;
    nbv[k] = 0;
    if (posv[k] >= 0) {
      if (MD_BOK(posv[k] < 2 * gi.e[l], 2)) {
        fl[k] = ldc(ca + posv[k]);
        nbv[k] = adj[posv[k]];
      }
      if (kh != nullptr && fl[k] && kh_has(kh, posv[k])) fl[k] = 0;
      if (!MD_BOK(nbv[k] >= 0 && nbv[k] < gi.n, 3)) nbv[k] = 0;
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) keep += fl[k] != 0;
  const int rt = r;
  for (int i = i0 + 4; i < i1; ++i) {
    while (pre[r + 1] <= i) ++r;
    const int pos = hdr[64 + l * 16 + r] + (i - pre[r]);
    keep += ldc(ca + pos) != 0 && !(kh != nullptr && kh_has(kh, pos));
  }
  // exclusive scan of keep over the layer's 256 threads
  int incl = keep;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) tmp[w] = incl;
  __syncthreads();
  TSTAMP(62);
  int base = 0, tot = 0;
  if (L < 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int x = tmp[l * 4 + k];
      if (k < (w & 3)) base += x;
      tot += x;
    }
  } else {
#pragma unroll
    for (int k = 0; k < NTHREADS / 64; ++k) {
      const int x = tmp[k];
      if (k < w) base += x;
      tot += x;
    }
  }
  int o = base + incl - keep;
  // row offsets without atomics: the owner of a row's first CSR position writes the row's
  // offset (= alive entries before it); rows starting at T get the total
  int rs = r0;
  while (rs > 0 && pre[rs - 1] == i0) --rs;
  if (rs < 16 && pre[rs] < i0) ++rs;
  r = r0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int i = i0 + k;
    if (i < i1) {
      while (rs < 16 && pre[rs] == i) hdr[l * 16 + rs++] = o;
      if (fl[k]) {
        if (o < NB_CAP) nbl[o] = (uint16_t)nbv[k];
        ++o;
      }
    }
  }
  r = rt;
  for (int i = i0 + 4; i < i1; ++i) {
    while (rs < 16 && pre[rs] == i) hdr[l * 16 + rs++] = o;
    while (pre[r + 1] <= i) ++r;
    const int pos = hdr[64 + l * 16 + r] + (i - pre[r]);
    if (ldc(ca + pos) && !(kh != nullptr && kh_has(kh, pos))) {
      if (o < NB_CAP) nbl[o] = (uint16_t)adj[pos];
      ++o;
    }
  }
  if (t < 16 && pre[t] == T) hdr[l * 16 + t] = tot;
  if (t == 0) hdr[128 + l] = tot;
  __syncthreads();
  TSTAMP(63);
  if (t < 16) hdr[32 + l * 16 + t] = (t < 15 ? hdr[l * 16 + t + 1] : tot) - hdr[l * 16 + t];
  const int over = __syncthreads_or(tot > NB_CAP);
  return !over;
}

// Iteration-1 prebuild of tile j, layer L (single-graph rollouts with speculative steps): while
// phase A applies the speculative result `ew` names (published as soon as phase A knows it takes
// it), the tile workgroup builds its rows and alive-neighbour lists from that result -- its live
// list for the rows, the CSR flags with the result's killed edges removed (phase A's write-back
// of them may be in flight) -- so iteration 1 starts at the gather when phase A confirms the
// result (pre_cw).  Returns 1 (rows and lists ready), 2 (rows ready, lists over NB_CAP: the
// per-row gather), 0 (not built: the result's features not published in time, or too many
// killed edges for the LDS set).
__device__ __noinline__ int prebuild_lists(KParams&, const GraphInfo gi, int j, int L, unsigned long long ew,
                                           unsigned long long* ts = nullptr, unsigned long long sv = 0ull) {
  KParams& p = kp();
  float* const lds = lds_base();
  float* const scr = lds + L_SCR;
  int* rows = (int*)(scr + S_ROW);
  lds_i32* hdr = (lds_i32*)(int*)(scr + S_NBH);
  int* misc = (int*)(lds + L_MISC);
  const int slot = (int)(ew & 0xffffu), a = (int)((ew >> 16) & 0xffffu);
  const unsigned want = (unsigned)(ew >> 32);
  const int* sl = p.sres + (size_t)slot * p.sres_stride;
  const int n = gi.n, et = gi.e[0] + gi.e[1];
  lds_i32* kh = (lds_i32*)(int*)(scr + S_M);
  TSTAMP(28);  // diagnostics: prebuild start
  for (int i = threadIdx.x; i < KH_SIZE; i += NTHREADS) kh[i] = -1;
  if (threadIdx.x == 0) {
    // the features tag, the done tag and the live count polled together (one round trip when
    // the result is complete, as it usually is once phase A took it)
    const unsigned long long ft_want = ((unsigned long long)(unsigned)a << 32) | want;
    const unsigned long long t0 = wall_clock64();
    int ok = 0;
    unsigned long long dt;
    int nl;
    while (true) {
      const unsigned long long ft = __hip_atomic_load((const g_u64*)(sl + SRES_FEAT), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      dt = __hip_atomic_load((const g_u64*)sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      nl = ldc(sl + 12);
      // sv != 0 (a prebuild ahead of phase A's pick): stop once phase A's early word (same
      // round trip) names another result
      const unsigned long long now = sv != 0ull && p.pre_ew != nullptr
                                         ? __hip_atomic_load((const g_u64*)p.pre_ew, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                         : 0ull;
      if (now != 0ull && now != sv && now != ew) break;
      if (ft == ft_want) {
        ok = 1;
        break;
      }
      if (wall_clock64() - t0 > 3000 ||  // 30 us: phase A will not wait for it either
          (__hip_atomic_load((g_u32*)p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & BAR_ERR))
        break;
      __builtin_amdgcn_s_sleep(1);
    }
    // (the features tag is written after the done tag and the live count, but loads of one
    // round trip are not ordered: the data round trip below reads both again to confirm)
    const int nd = (int)(dt >> 48);
    // (at most KH_SIZE / 2 CSR slots in the killed-edge set: the probes always find a free entry)
    if (ok && ((unsigned)dt != want || (int)((dt >> 32) & 0xffffu) != a || nd > KH_SIZE / 4)) ok = 0;
    misc[44] = ok;
    misc[45] = nd;
    misc[46] = nl;
  }
  __syncthreads();
  TSTAMP(24);  // diagnostics (one tile's prebuild): slot polled
  if (!misc[44]) return 0;
  const int nd = misc[45], nl = misc[46];
#ifdef MD_TORN_SLOT
  const int ndk = misc[25] ? 0 : nd;  // (torn step: the kill list read stale, after the tag checks)
#else
  const int ndk = nd;
#endif
  // the tile's rows from the result's live list (entries as in phase A's list) and every killed
  // edge's three words, all in one round trip
  float4 e = make_float4(0.f, 0.f, 0.f, 0.f);
  if (threadIdx.x < TILE) e = ldc4((const float*)(sl + sres_live(et, n)), min(j * TILE + (int)threadIdx.x, n - 1) * 16);
  constexpr int KPT = (KH_SIZE / 4 + NTHREADS - 1) / NTHREADS;
  int kv[KPT], k1[KPT], k2[KPT];
#pragma unroll
  for (int u = 0; u < KPT; ++u) {
    const int i = threadIdx.x + u * NTHREADS;
    if (i < nd) {
      kv[u] = ldc(sl + SRES_HDR + 3 * i);
      k1[u] = ldc(sl + SRES_HDR + 3 * i + 1);
      k2[u] = ldc(sl + SRES_HDR + 3 * i + 2);
    }
  }
  if (threadIdx.x == 0) {
    const unsigned long long dt2 = __hip_atomic_load((const g_u64*)sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    misc[47] = ((int)(dt2 >> 48) == nd && (unsigned)dt2 == want && ldc(sl + 12) == nl && nl <= n);
    // in the same round trip: layer L's dmax of the result (spec_iteration1's first-layer
    // table) and the early word as it stands now (a prebuild phase A has already overtaken
    // stops after its lists)
    misc[40] = ldc(sl + 13 + L);
    const unsigned long long now = p.pre_ew != nullptr ? __hip_atomic_load((const g_u64*)p.pre_ew, __ATOMIC_RELAXED,
                                                                            __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    misc[36] = (int)(unsigned)now;
    misc[37] = (int)(unsigned)(now >> 32);
  }
  __syncthreads();
  TSTAMP(25);  // rows and kill list in
  if (!misc[47]) return 0;  // (else not built: the tile builds after the record)
  if (threadIdx.x < TILE) {
    // entries validated whatever the slot holds: a workgroup that lags may read a slot being
    // rewritten (its prebuild is then never used, but every address it forms stays in bounds)
    const int r = j * TILE + threadIdx.x;
    const unsigned c = (unsigned)__float_as_int(e.w);
    const bool ok = r < nl && __float_as_int(e.x) >= 0 && __float_as_int(e.x) < n && __float_as_int(e.y) >= 0 &&
                    __float_as_int(e.y) + (int)(c & 0xffffu) <= 2 * gi.e[0] && __float_as_int(e.z) >= 0 &&
                    __float_as_int(e.z) + (int)(c >> 16) <= 2 * gi.e[1];
    rows[threadIdx.x] = ok ? __float_as_int(e.x) : -1;
    hdr[64 + threadIdx.x] = ok ? __float_as_int(e.y) : 0;
    hdr[96 + threadIdx.x] = ok ? (int)(c & 0xffffu) : 0;
    hdr[64 + 16 + threadIdx.x] = ok ? __float_as_int(e.z) : 0;
    hdr[96 + 16 + threadIdx.x] = ok ? (int)(c >> 16) : 0;
  }
  // the killed edges of layer L: both CSR positions into the set
#pragma unroll
  for (int u = 0; u < KPT; ++u) {
    const int i = threadIdx.x + u * NTHREADS;
    if (i < ndk && ((kv[u] & 0xffff) < gi.e[0] ? 0 : 1) == L) {
      kh_insert(kh, k1[u]);
      kh_insert(kh, k2[u]);
    }
  }
  __syncthreads();
  return build_nb_lists(p, gi, rows, scr, ts, L, true) ? 1 : 2;
}

// Gather for one tile from the alive neighbour lists: per batch the layer's 256 threads stage
// up to STG_ROWS neighbour rows (five 16-byte loads in flight per thread) into [S_M, S_HID),
// then each 16-lane group adds its row's neighbours in CSR order (the reference's sequential
// scatter-add order).  Same results as gather_tile; high-degree rows no longer serialise
// their loads.
__device__ __noinline__ void gather_tile2(KParams&, const GraphInfo gi, int it, const int*, float*) {
  const int* const rows = (const int*)(lds_base() + L_SCR + S_ROW);
  float* const scr = lds_base() + L_SCR;

  KParams& p = kp();  // kernel arguments through the implicit-argument SGPRs (uniform)
  const int w = wave_id(), l = w >> 2, lane = lane_id(), t = threadIdx.x & 255;
  const int grp = lane >> 4, qd = lane & 15;
  const int* deg = p.deg[l] + gi.node_off;
  const float* hp;
  bool table = false;
  if (it == 1) {
    table = p.node_w == nullptr;
    hp = table ? first_layer_rows(p, gi, l) : p.h0tab[l] + (size_t)gi.node_off * EMB;
  } else {
    hp = p.H[l][(it - 2) & 1] + (size_t)gi.node_off * EMB;
  }
  const lds_i32* hdr = (const lds_i32*)(const int*)(scr + S_NBH);
  const lds_u16* nbl = (const lds_u16*)(const uint16_t*)(scr + S_NBL) + l * NB_CAP;
  const int r = 4 * (w & 3) + grp;
  const int v = rows[r];
  float4 own = {0.f, 0.f, 0.f, 0.f}, acc = {0.f, 0.f, 0.f, 0.f};
  if (v >= 0) {
    const int ov = table ? ldc(deg + v) : v;
    if (MD_BOK(v < gi.n && ov >= 0 && ov < gi.n, 1)) own = ldc4(hp, ov * 256 + qd * 16);
  }
  const int myoff = hdr[l * 16 + r], mycnt = hdr[32 + l * 16 + r];
  const int totl = hdr[128 + l];
  const int nbat = (max(hdr[128], hdr[129]) + STG_ROWS - 1) / STG_ROWS;
  float4* stg = (float4*)(scr + S_M) + l * STG_ROWS * 16;
  // Batch b's five 16-byte loads per thread go out while batch b - 1 is summed (register
  // double buffer: the global latency of a batch overlaps the previous batch's adds); the
  // per-row adds read eight staged rows ahead of their (in-order) accumulation.
  auto issue = [&](int b, float4 (&x)[5], bool (&ok)[5]) {
    const int base = b * STG_ROWS;
    int src[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int k = t + 256 * i, row = base + (k >> 4);
      src[i] = -1;
      if (b < nbat && k < STG_ROWS * 16 && row < totl) {
        const int id = nbl[row];
        src[i] = MD_BOK(id < gi.n, 4) ? (table ? ldc(deg + id) : id) : -1;
        if (!MD_BOK(src[i] < gi.n, 5)) src[i] = -1;
      }
    }
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      ok[i] = src[i] >= 0;
      if (ok[i]) x[i] = ldc4(hp, src[i] * 256 + ((t + 256 * i) & 15) * 16);
    }
  };
  auto consume = [&](int b, const float4 (&x)[5], const bool (&ok)[5]) {
    const int base = b * STG_ROWS;
#pragma unroll
    for (int i = 0; i < 5; ++i)
      if (ok[i]) stg[t + 256 * i] = x[i];
    __syncthreads();
    const int lo = max(myoff, base), hi = min(myoff + mycnt, base + STG_ROWS);
    int k = lo;
    for (; k + 8 <= hi; k += 8) {
      float4 y[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = stg[(k + j - base) * 16 + qd];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc.x = acc.x + y[j].x;
        acc.y = acc.y + y[j].y;
        acc.z = acc.z + y[j].z;
        acc.w = acc.w + y[j].w;
      }
    }
    for (; k < hi; ++k) {
      const float4 y = stg[(k - base) * 16 + qd];
      acc.x = acc.x + y.x;
      acc.y = acc.y + y.y;
      acc.z = acc.z + y.z;
      acc.w = acc.w + y.w;
    }
    __syncthreads();
  };
  float4 xa[5], xb[5];
  bool oka[5], okb[5];
  if (nbat > 0) issue(0, xa, oka);
  for (int b = 0; b < nbat; b += 2) {
    issue(b + 1, xb, okb);
    consume(b, xa, oka);
    if (b + 1 >= nbat) break;
    issue(b + 2, xa, oka);
    consume(b + 1, xb, okb);
  }
  float* atp = scr + S_P + l * 64 * LDT;
  float* atx = scr + S_X + l * 64 * LDT;
  const int c = 4 * qd;
  atp[(c + 0) * LDT + r] = acc.x;
  atp[(c + 1) * LDT + r] = acc.y;
  atp[(c + 2) * LDT + r] = acc.z;
  atp[(c + 3) * LDT + r] = acc.w;
  atx[(c + 0) * LDT + r] = own.x;
  atx[(c + 1) * LDT + r] = own.y;
  atx[(c + 2) * LDT + r] = own.z;
  atx[(c + 3) * LDT + r] = own.w;
}

// Iteration 1 of a workgroup with several tiles: its tiles' alive neighbour lists and
// headers go to the tile's cache slot (agent-scope stores), so iterations 2 and 3 reload them
// in one round trip instead of rebuilding them from the CSR flags.
__device__ __noinline__ void nbc_store(KParams&, int slot, const float*, bool ok, int nbo = 0) {
  float* const scr = lds_base() + L_SCR;

  KParams& p = kp();
  int* dst = p.nbc + (size_t)slot * NBC_INTS;
  const lds_i32* hdr = (const lds_i32*)(const int*)(scr + S_NBH + nbo);
  const lds_i32* words = (const lds_i32*)(const int*)(scr + S_NBL + nbo);
  const int t = threadIdx.x;
  if (t < 64) stc(dst + t, hdr[t]);
  else if (t < 66) stc(dst + t, hdr[128 + t - 64]);
  else if (t == 66) stc(dst + t, ok ? 1 : 0);
  if (!ok) return;
#pragma unroll
  for (int l = 0; l < 2; ++l) {
    const int nw = (hdr[128 + l] + 1) >> 1;
    for (int i = t; i < nw; i += NTHREADS) stc(dst + NBC_HDR + l * NBC_LWORDS + i, words[l * NBC_LWORDS + i]);
  }
}

// ------------------------------------------------------------------ layer-split tile pieces
// Dedicated mode with at least two tile workgroups per tile: workgroup (tile, L) runs layer L
// of iterations 1 and 2 with all eight waves (the two layers only meet in the attention of
// iteration 3, which the L = 0 workgroup runs for both).  Same arithmetic, same order.

// Gather of layer L from its alive neighbour list: the 512 threads stage up to 2 * STG_ROWS
// neighbour rows per batch (register double buffer as in gather_tile2), 32 lanes per row add
// two features each in CSR order.
// deg_ovr / hp_ovr (iteration 1 speculated during phase A): the residual degrees and the
// first-layer rows of the speculative result instead of the graph's arrays.
// dcap: first-layer rows by degree are clamped to [1, dcap] (the prebuild's table of the result's
// dmax, whose row d sits at hp + d rows: a prebuild from a slot being rewritten must not address
// outside it -- row 0 of the dmax-1 table would lie 256 B before the h0g allocation; every node on
// a tile's rows or lists has degree >= 1, so consistent data are unaffected).
__device__ __noinline__ void gather_tile2s(KParams&, const GraphInfo gi, int it, const int*, float*, int L,
                                           const int* deg_ovr = nullptr, const float* hp_ovr = nullptr,
                                           int dcap = 0x7fffffff) {
  const int* const rows = (const int*)(lds_base() + L_SCR + S_ROW);
  float* const scr = lds_base() + L_SCR;

  KParams& p = kp();  // kernel arguments through the implicit-argument SGPRs (uniform)
  constexpr int SROWS = 2 * STG_ROWS, NLD = (SROWS * 16 + NTHREADS - 1) / NTHREADS;
  const int w = wave_id(), lane = lane_id(), t = threadIdx.x, l = L;
  const int q = lane & 31;
  const int r = 2 * w + (lane >> 5);
  const int* deg = deg_ovr != nullptr ? deg_ovr : p.deg[l] + gi.node_off;
  const float* hp;
  bool table = false;
  if (it == 1) {
    table = p.node_w == nullptr;
    hp = table ? (hp_ovr != nullptr ? hp_ovr : first_layer_rows(p, gi, l)) : p.h0tab[l] + (size_t)gi.node_off * EMB;
  } else {
    hp = p.H[l][(it - 2) & 1] + (size_t)gi.node_off * EMB;
  }
  const lds_i32* hdr = (const lds_i32*)(const int*)(scr + S_NBH);
  const lds_u16* nbl = (const lds_u16*)(const uint16_t*)(scr + S_NBL) + l * NB_CAP;
  const int v = rows[r];
  float2 own = {0.f, 0.f}, acc = {0.f, 0.f};
#ifdef MD_TORN_SLOT
  // (a torn speculative slot, this step: the degree words of odd nodes read as 0)
  const bool torn = deg_ovr != nullptr && ((const int*)(lds_base() + L_MISC))[25] != 0;
  auto rdeg = [&](int x) { return torn && (x & 1) ? 0 : ldc(deg + x); };
  auto row_of = [&](int d, int site) { return md_brec(d >= 1 && d <= dcap, site) ? d : -1; };
#else
  auto rdeg = [&](int x) { return ldc(deg + x); };
  auto row_of = [&](int d, int) { return min(max(d, 1), dcap); };
#endif
  if (v >= 0) {
    const int ov = table ? row_of(rdeg(v), 22) : v;
    if (ov >= 0 && MD_BOK(v < gi.n && ov < gi.n, 1)) own = ldc2(hp, ov * 256 + q * 8);
  }
  const int myoff = hdr[l * 16 + r], mycnt = hdr[32 + l * 16 + r];
  const int totl = hdr[128 + l];
  const int nbat = (totl + SROWS - 1) / SROWS;
  float4* stg = (float4*)(scr + S_M);
  const float2* stg2 = (const float2*)(scr + S_M);
  auto issue = [&](int b, float4 (&x)[NLD], bool (&ok)[NLD]) {
    const int base = b * SROWS;
    int src[NLD];
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int k = t + NTHREADS * i, row = base + (k >> 4);
      src[i] = -1;
      if (b < nbat && k < SROWS * 16 && row < totl) {
        const int id = nbl[row];
        src[i] = MD_BOK(id < gi.n, 4) ? (table ? row_of(rdeg(id), 23) : id) : -1;
        if (!MD_BOK(src[i] < gi.n, 5)) src[i] = -1;
      }
    }
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      ok[i] = src[i] >= 0;
      if (ok[i]) x[i] = ldc4(hp, src[i] * 256 + ((t + NTHREADS * i) & 15) * 16);
    }
  };
  auto consume = [&](int b, const float4 (&x)[NLD], const bool (&ok)[NLD]) {
    const int base = b * SROWS;
#pragma unroll
    for (int i = 0; i < NLD; ++i)
      if (ok[i]) stg[t + NTHREADS * i] = x[i];
    __syncthreads();
    const int lo = max(myoff, base), hi = min(myoff + mycnt, base + SROWS);
    int k = lo;
    for (; k + 8 <= hi; k += 8) {
      float2 y[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) y[j] = stg2[(k + j - base) * 32 + q];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc.x = acc.x + y[j].x;
        acc.y = acc.y + y[j].y;
      }
    }
    for (; k < hi; ++k) {
      const float2 y = stg2[(k - base) * 32 + q];
      acc.x = acc.x + y.x;
      acc.y = acc.y + y.y;
    }
    __syncthreads();
  };
  float4 xa[NLD], xb[NLD];
  bool oka[NLD], okb[NLD];
  if (nbat > 0) issue(0, xa, oka);
  for (int b = 0; b < nbat; b += 2) {
    issue(b + 1, xb, okb);
    consume(b, xa, oka);
    if (b + 1 >= nbat) break;
    issue(b + 2, xa, oka);
    consume(b + 1, xb, okb);
  }
  float* atp = scr + S_P + l * 64 * LDT;
  float* atx = scr + S_X + l * 64 * LDT;
  const int c = 2 * q;
  atp[(c + 0) * LDT + r] = acc.x;
  atp[(c + 1) * LDT + r] = acc.y;
  atx[(c + 0) * LDT + r] = own.x;
  atx[(c + 1) * LDT + r] = own.y;
}

// Dataflow mode, iterations 2-3 of layer L: gather_tile2s with the previous iteration's rows
// read as tagged granules (df_hb) -- 32 lanes per row, each loading its two features and their
// tags in one 16-byte load -- polled until every tag is ta or tb, so the gather itself waits for
// exactly the rows it needs instead of a grid barrier.  Same staging, same adds in CSR order.
__device__ __forceinline__ void gather_df(KParams&, const GraphInfo gi, int it, int L, unsigned ta, unsigned tb) {
  const int* const rows = (const int*)(lds_base() + L_SCR + S_ROW);
  float* const scr = lds_base() + L_SCR;

  KParams& p = kp();
  // 80 rows per batch: five 16-byte loads per thread and buffer (two buffers in flight) keep the
  // function clear of the callee-saved registers (no spill at its entry and exit)
  constexpr int SROWS = 80, NLD = SROWS * 32 / NTHREADS;
  static_assert(SROWS * 64 <= S_HID - S_M && SROWS * 32 % NTHREADS == 0, "dataflow staging fits [S_M, S_HID)");
  const int w = wave_id(), lane = lane_id(), t = threadIdx.x;
  const int q = lane & 31;
  const int r = 2 * w + (lane >> 5);
  const float* hb = (const float*)df_hb(p, L, it - 2, df_par(ta));
  const lds_i32* hdr = (const lds_i32*)(const int*)(scr + S_NBH);
  const lds_u16* nbl = (const lds_u16*)(const uint16_t*)(scr + S_NBL) + L * NB_CAP;
  const int v = rows[r];
  float4 ox = make_float4(0.f, 0.f, 0.f, 0.f);
  if (v >= 0 && MD_BOK(v < gi.n && v < p.df_n, 1)) ox = ldc4(hb, v * 512 + q * 16);
  float2 acc = {0.f, 0.f};
  const int myoff = hdr[L * 16 + r], mycnt = hdr[32 + L * 16 + r];
  const int totl = hdr[128 + L];
  const int nbat = (totl + SROWS - 1) / SROWS;
  float2* stg = (float2*)(scr + S_M);
  const float2* stg2 = (const float2*)(scr + S_M);
  auto src_of = [&](int base, int i) {
    const int k = t + NTHREADS * i, row = base + (k >> 5);
    const int id = nbl[row];
    return MD_BOK(id < gi.n && id < p.df_n, 23) ? id * 512 + (k & 31) * 16 : 0;
  };
  auto issue = [&](int b, float4 (&x)[NLD], bool (&ok)[NLD]) {
    const int base = b * SROWS;
#pragma unroll
    for (int i = 0; i < NLD; ++i) {
      const int k = t + NTHREADS * i, row = base + (k >> 5);
      ok[i] = b < nbat && row < totl;
      if (ok[i]) x[i] = ldc4(hb, src_of(base, i));
    }
  };
  auto consume = [&](int b, float4 (&x)[NLD], const bool (&ok)[NLD]) {
    const int base = b * SROWS;
    // rows whose producer has not stored them yet: poll those (rare once a tile's neighbours
    // are ahead of it)
    unsigned bad = 0;
#pragma unroll
    for (int i = 0; i < NLD; ++i)
      if (ok[i] && !df_ok4(x[i], ta, tb)) bad |= 1u << i;
    if (__any(bad != 0)) {
      const unsigned long long t0 = wall_clock64();
      while (__any(bad != 0)) {
        __builtin_amdgcn_s_sleep(1);
        if (df_give_up(p, t0, BARRIER_TIMEOUT_TICKS)) break;
#pragma unroll
        for (int i = 0; i < NLD; ++i)
          if (bad & (1u << i)) x[i] = ldc4(hb, src_of(base, i));
#pragma unroll
        for (int i = 0; i < NLD; ++i)
          if ((bad & (1u << i)) && df_ok4(x[i], ta, tb)) bad &= ~(1u << i);
      }
    }
#pragma unroll
    for (int i = 0; i < NLD; ++i)
      if (ok[i]) stg[t + NTHREADS * i] = make_float2(x[i].x, x[i].z);
    __syncthreads();
    const int lo = max(myoff, base), hi = min(myoff + mycnt, base + SROWS);
    int k = lo;
    for (; k + 8 <= hi; k += 8) {
      float2 y[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) y[jj] = stg2[(k + jj - base) * 32 + q];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        acc.x = acc.x + y[jj].x;
        acc.y = acc.y + y[jj].y;
      }
    }
    for (; k < hi; ++k) {
      const float2 y = stg2[(k - base) * 32 + q];
      acc.x = acc.x + y.x;
      acc.y = acc.y + y.y;
    }
    __syncthreads();
  };
  float4 xa[NLD], xb[NLD];
  bool oka[NLD], okb[NLD];
  if (nbat > 0) issue(0, xa, oka);
  for (int b = 0; b < nbat; b += 2) {
    issue(b + 1, xb, okb);
    consume(b, xa, oka);
    if (b + 1 >= nbat) break;
    issue(b + 2, xa, oka);
    consume(b + 1, xb, okb);
  }
  if (v >= 0 && !df_ok4(ox, ta, tb)) ox = df_ld4(p, hb, v * 512 + q * 16, ta, tb);
  float* atp = scr + S_P + L * 64 * LDT;
  float* atx = scr + S_X + L * 64 * LDT;
  const int c = 2 * q;
  atp[(c + 0) * LDT + r] = acc.x;
  atp[(c + 1) * LDT + r] = acc.y;
  atx[(c + 0) * LDT + r] = ox.x;
  atx[(c + 1) * LDT + r] = ox.z;
}

// Node update of layer L: waves 0-3 P.P1 (column block w), waves 4-7 X.P2, then waves 0-3
// relu(M.P3).  Each output's k-chain is update_tile's.
__device__ __noinline__ void update_tile_split(const float*, float*, int L) {
  const float* const wi = lds_base() + L_W;
  float* const scr = lds_base() + L_SCR;

  const int w = wave_id(), cb = w & 3, lane = lane_id();
  const int ar = lane & 15, ak = lane >> 4;
  const bool second = w >= 4;
  const float* at_in = scr + (second ? S_X : S_P) + L * 64 * LDT;
  float* atm = scr + S_M + L * 128 * LDT;
  const float* wsrc = wi + (second ? W_IP2 : W_IP1) + cb * 16 * 64;
  const float* p3 = wi + W_IP3 + cb * 32 * 64;
  float xa[16], wa[16], wc[32];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    xa[s] = at_in[(4 * s + ak) * LDT + ar];
    wa[s] = wsrc[s * 64 + lane];
  }
  if (!second) {
#pragma unroll
    for (int s = 0; s < 32; ++s) wc[s] = p3[s * 64 + lane];
  }
  __builtin_amdgcn_sched_barrier(0);
  f4 a1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 16; ++s) a1 = mfma16(xa[s], wa[s], a1);
  const int col = 16 * cb + ar;
#pragma unroll
  for (int r = 0; r < 4; ++r) atm[((second ? 64 : 0) + col) * LDT + 4 * ak + r] = a1[r];
  __syncthreads();
  if (!second) {
    float xm[32];
#pragma unroll
    for (int s = 0; s < 32; ++s) xm[s] = atm[(4 * s + ak) * LDT + ar];
    __builtin_amdgcn_sched_barrier(0);
    f4 a3 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 32; ++s) a3 = mfma16(xm[s], wc[s], a3);
    float* ate = scr + S_E + L * 64 * LDT;
#pragma unroll
    for (int r = 0; r < 4; ++r) ate[col * LDT + 4 * ak + r] = fmaxf(a3[r], 0.f);
  }
}

// Row-normalise layer L of the transposed tile at `at` in place (normalize_tile's order).
__device__ __noinline__ void normalize_tile_split(float*, float*, int L) {
  float* const scr = lds_base() + L_SCR;
  float* const at = scr + S_E;

  float* red = scr + S_RED;
  const int t = threadIdx.x;
  float* a = at + L * 64 * LDT;
  if (t < 128) {
    const int row = t >> 3, j = t & 7;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float v = a[(8 * i + j) * LDT + row];
      acc = fmaf(v, v, acc);
    }
    red[(L * 16 + row) * 8 + j] = acc;
  }
  __syncthreads();
  const int w = wave_id(), lane = lane_id();
  if (w < 4) {
    const int col = 16 * w + (lane & 15), rq = lane >> 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * rq + r;
      const float den = fmaxf(sqrtf(sumsq8_finish(red + (L * 16 + row) * 8)), 1e-12f);
      a[col * LDT + row] = a[col * LDT + row] / den;
    }
  }
}

// Node update for one tile: H' = relu([P.P1 | X.P2] . P3) into S_E (normalised separately).
// Iteration 1 of tile j, layer L speculated during phase A (after prebuild_lists): the gather
// with the speculative result's degrees and first-layer rows, the update, the normalisation,
// the partial sums S0 / S1 and the H1 stores -- the layer-split iteration-1 work exactly.  Its
// stores land where iteration 1's do and nobody reads them before barrier 1; without phase A's
// confirmation the tile runs iteration 1 again and overwrites them.  Returns false when the
// first-layer rows of the result's dmax are not precomputed (nothing done).
// Dataflow mode: the outputs of iteration it (1 or 2) of tile j, layer L (graph-local) as tagged
// granules -- the virtual-node partial sums (S0 and S1 at iteration 1, S2 at 2, the barrier
// path's values) and the new embedding rows, thread t storing row t / 32's features 2 (t % 32)
// and 2 (t % 32) + 1 as one 16-byte pair of granules.  Reads E / X in LDS: the caller syncs
// before overwriting them.
__device__ __forceinline__ void df_store_tile(KParams&, int j, int L, int it, unsigned tag) {
  KParams& p = kp();
  float* const scr = lds_base() + L_SCR;
  const int* rows = (const int*)(scr + S_ROW);
  if (threadIdx.x < 64) {
    const int c = threadIdx.x;
    const float* ate = scr + S_E + L * 64 * LDT + c * LDT;
    const float* atx = scr + S_X + L * 64 * LDT + c * LDT;
    const int nv = tile_rows_valid(rows);
    unsigned long long* sp = df_sp(p, df_par(tag)) + (size_t)j * 384;
    const float s_new = col_sum16(ate, nv);
    if (it == 1) {
      df_st(sp + L * 64 + c, col_sum16(atx, nv), tag);  // S0 (first-layer input)
      df_st(sp + 128 + L * 64 + c, s_new, tag);         // S1
    } else {
      df_st(sp + 256 + L * 64 + c, s_new, tag);         // S2
    }
  }
  const int rr = threadIdx.x >> 5, c2 = threadIdx.x & 31;
  const int v = rows[rr];
  const float* e = scr + S_E + L * 64 * LDT;
  const float tf = __uint_as_float(tag);
  if (v >= 0 && MD_BOK(v < p.df_n && j < p.df_mt, 21))
    stc4((float*)df_hb(p, L, it - 1, df_par(tag)), v * 512 + c2 * 16,
         make_float4(e[(2 * c2) * LDT + rr], tf, e[(2 * c2 + 1) * LDT + rr], tf));
}

// dft != 0 (dataflow mode): the outputs go out as granules tagged dft (df_store_tile).
__device__ __forceinline__ bool spec_iteration1(KParams&, const GraphInfo gi, int j, int L, unsigned long long ew,
                                             unsigned dft = 0, unsigned long long* ts = nullptr) {
  KParams& p = kp();
  float* const lds = lds_base();
  float* const scr = lds + L_SCR;
  const int* rows = (const int*)(scr + S_ROW);
  const int* sl = p.sres + (size_t)(ew & 0xffffu) * p.sres_stride;
  const int n = gi.n, et = gi.e[0] + gi.e[1];
  const float* hp = nullptr;
  int dm = 0x7fffffff;
  if (p.node_w == nullptr) {  // unit cost: rows by degree, from the precomputed table of the result's dmax
    dm = ((const int*)(lds + L_MISC))[40];  // (read by prebuild_lists, which runs just before)
    if (p.h0g == nullptr || dm < 1 || dm > p.h0g_dm) return false;
    hp = p.h0g + (h0g_row(dm, 1) - 1) * EMB;
  }
  gather_tile2s(p, gi, 1, rows, scr, L, sl + sres_deg(et) + L * n, hp, dm);
  __syncthreads();
  TSTAMP(26);  // diagnostics: gathered
  update_tile_split(lds + L_W, scr, L);
  __syncthreads();
  normalize_tile_split(scr + S_E, scr, L);
  __syncthreads();
  TSTAMP(27);  // updated, normalised
  if (dft != 0) {
    df_store_tile(p, j, L, 1, dft);
    __syncthreads();
    TSTAMP(35);  // stored
    return true;
  }
  if (threadIdx.x < 64) {
    const int c = threadIdx.x;
    const float* ate = scr + S_E + L * 64 * LDT + c * LDT;
    const float* atx = scr + S_X + L * 64 * LDT + c * LDT;
    const int nv = tile_rows_valid(rows);
    const float s_new = col_sum16(ate, nv), s_old = col_sum16(atx, nv);
    float* sp = p.spart + (size_t)(gi.tile_off + j) * 384;
    stc(sp + L * 64 + c, s_old);        // S0 (first-layer input)
    stc(sp + 128 + L * 64 + c, s_new);  // S1
  }
  {
    const int w = wave_id(), lane = lane_id();
    float* hb = p.H[L][0] + (size_t)gi.node_off * EMB;
    const int r = 4 * (w & 3) + (lane >> 4), q4 = lane & 15;
    const int v = rows[r];
    const float* e = scr + S_E + L * 64 * LDT + 4 * q4 * LDT + r;
    if (v >= 0 && w < 4) stc4(hb, v * 256 + q4 * 16, make_float4(e[0], e[LDT], e[2 * LDT], e[3 * LDT]));
  }
  __syncthreads();
  return true;
}

__device__ __noinline__ void update_tile(const float*, float*) {
  const float* const wi = lds_base() + L_W;
  float* const scr = lds_base() + L_SCR;

  const int w = wave_id(), l = w >> 2, cb = w & 3, lane = lane_id();
  const int ar = lane & 15, ak = lane >> 4;
  const float* atp = scr + S_P + l * 64 * LDT;
  const float* atx = scr + S_X + l * 64 * LDT;
  float* atm = scr + S_M + l * 128 * LDT;
  const float* p1 = wi + W_IP1 + cb * 16 * 64;
  const float* p2 = wi + W_IP2 + cb * 16 * 64;
  const float* p3 = wi + W_IP3 + cb * 32 * 64;
  // operands of both chains loaded up front (every LDS read in flight before the first
  // MFMA), the P3 fragments before the workgroup barrier
  float xa[16], xb[16], wa[16], wb[16], wc[32];
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    xa[s] = atp[(4 * s + ak) * LDT + ar];
    wa[s] = p1[s * 64 + lane];
    xb[s] = atx[(4 * s + ak) * LDT + ar];
    wb[s] = p2[s * 64 + lane];
  }
#pragma unroll
  for (int s = 0; s < 32; ++s) wc[s] = p3[s * 64 + lane];
  __builtin_amdgcn_sched_barrier(0);  // keep every read ahead of the MFMA chains
  f4 a1 = {0.f, 0.f, 0.f, 0.f}, a2 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    a1 = mfma16(xa[s], wa[s], a1);
    a2 = mfma16(xb[s], wb[s], a2);
  }
  const int col = 16 * cb + ar;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    atm[col * LDT + 4 * ak + r] = a1[r];
    atm[(64 + col) * LDT + 4 * ak + r] = a2[r];
  }
  __syncthreads();
  float xm[32];
#pragma unroll
  for (int s = 0; s < 32; ++s) xm[s] = atm[(4 * s + ak) * LDT + ar];
  __builtin_amdgcn_sched_barrier(0);
  f4 a3 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 32; ++s) a3 = mfma16(xm[s], wc[s], a3);
  float* ate = scr + S_E + l * 64 * LDT;
#pragma unroll
  for (int r = 0; r < 4; ++r) ate[col * LDT + 4 * ak + r] = fmaxf(a3[r], 0.f);
}

// Row-normalise the [2][64][16] transposed tile at `at` in place (torch reduction order).
__device__ __noinline__ void normalize_tile(float*, float*) {
  float* const scr = lds_base() + L_SCR;
  float* const at = scr + S_E;

  float* red = scr + S_RED;
  const int t = threadIdx.x;
  if (t < 256) {
    const int l = t >> 7, row = (t >> 3) & 15, j = t & 7;
    const float* a = at + l * 64 * LDT;
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float v = a[(8 * i + j) * LDT + row];
      acc = fmaf(v, v, acc);
    }
    red[(l * 16 + row) * 8 + j] = acc;
  }
  __syncthreads();
  const int w = wave_id(), l = w >> 2, cb = w & 3, lane = lane_id();
  const int col = 16 * cb + (lane & 15), rq = lane >> 4;
  float* a = at + l * 64 * LDT;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 4 * rq + r;
    const float den = fmaxf(sqrtf(sumsq8_finish(red + (l * 16 + row) * 8)), 1e-12f);
    a[col * LDT + row] = a[col * LDT + row] / den;
  }
}

// ------------------------------------------------------------------ virtual node (1 row)
// Sum of one graph's per-tile partial sums (slot) -> out[2][64]: four threads per output each
// add a contiguous quarter of the tiles in order, then the quarters are added in order
// (a fixed order, identical in every workgroup).
// ta != 0 (dataflow mode): the partials are tagged granules (df_sp, graph-local tiles) polled
// until their tag is ta or tb.
__device__ void graph_sum(KParams& p, const GraphInfo& gi, int nt, int slot, float*, float*, unsigned ta = 0,
                          unsigned tb = 0) {
  float* const out = lds_base() + L_SCR + S_HID;
  float* const tmp4 = lds_base() + L_SCR + S_YP;

  const int o = threadIdx.x & 127, qt = threadIdx.x >> 7;
  const int per = (nt + 3) >> 2;
  const int j0 = min(nt, qt * per), j1 = min(nt, j0 + per);
  const float* sp = p.spart + (size_t)gi.tile_off * 384 + slot * 128 + o;
  float a = 0.f;
  if (ta != 0) {
    const unsigned long long* sg = df_sp(p, df_par(ta)) + slot * 128 + o;
    for (int jb = j0; jb < j1; jb += 16) {
      unsigned long long gx[16];
#pragma unroll
      for (int k = 0; k < 16; ++k)
        gx[k] = jb + k < j1 ? __hip_atomic_load((const g_u64*)(sg + (size_t)(jb + k) * 384), __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT)
                            : 0ull;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (jb + k < j1) {
          const float x = df_ok((unsigned)(gx[k] >> 32), ta, tb) ? __uint_as_float((unsigned)gx[k])
                                                                 : df_ld(p, sg + (size_t)(jb + k) * 384, ta, tb);
          a = a + x;
        }
      }
    }
  } else {
    for (int jb = j0; jb < j1; jb += 16) {
      float x[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) x[k] = jb + k < j1 ? ldc(sp + (size_t)(jb + k) * 384) : 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (jb + k < j1) a = a + x[k];
    }
  }
  tmp4[qt * 128 + o] = a;
  __syncthreads();
  if (threadIdx.x < 128) out[o] = ((tmp4[o] + tmp4[128 + o]) + tmp4[256 + o]) + tmp4[384 + o];
  __syncthreads();
}

// One virtual-node iteration for both layers: y' = normalize(relu([s.P1 | y.P2] . P3)),
// computed by the 4 waves of each layer group as 4 partial chains summed in order.
__device__ __noinline__ void vrow_update(const float*, float*, const float* /*[2][64]*/, float* /*[2][64]*/) {
  const float* const wi = lds_base() + L_W;
  float* const scr = lds_base() + L_SCR;
  const float* const s = scr + S_HID;
  float* const y = lds_base() + L_YW;

  const int w = wave_id(), l = w >> 2, q = w & 3, lane = lane_id();
  float* yp = scr + S_YP + l * 512;
  float* ym = scr + S_YM + l * 128;
  {
    const int k0 = q * 16;
    const float a1 = fma_chain<16>(0.f, k0, [&](int k) { return s[l * 64 + k]; },
                                   [&](int k) { return wget(wi + W_IP1, 16, k, lane); });
    const float a2 = fma_chain<16>(0.f, k0, [&](int k) { return y[l * 64 + k]; },
                                   [&](int k) { return wget(wi + W_IP2, 16, k, lane); });
    yp[q * 128 + lane] = a1;
    yp[q * 128 + 64 + lane] = a2;
  }
  __syncthreads();
  if (q == 0) {
    ym[lane] = ((yp[lane] + yp[128 + lane]) + yp[256 + lane]) + yp[384 + lane];
    ym[64 + lane] = ((yp[64 + lane] + yp[192 + lane]) + yp[320 + lane]) + yp[448 + lane];
  }
  __syncthreads();
  {
    const int k0 = q * 32;
    const float a = fma_chain<32>(0.f, k0, [&](int k) { return ym[k]; },
                                  [&](int k) { return wget(wi + W_IP3, 32, k, lane); });
    yp[q * 128 + lane] = a;
  }
  __syncthreads();
  if (q == 0) {
    float o = ((yp[lane] + yp[128 + lane]) + yp[256 + lane]) + yp[384 + lane];
    o = fmaxf(o, 0.f);
    const float nr = wave_norm64(o);
    y[l * 64 + lane] = o / fmaxf(nr, 1e-12f);
  }
  __syncthreads();
}

// Attention gate of one row (U/MRGNN/mutil_layer_weight.py:266-285, LogisticVector :304-313):
// weight of the OTHER layer for target layer l, from dots d00 = F0F0.lw, d11, d01.
__device__ __forceinline__ float other_gate(int l, float d00, float d11, float d01, float lb) {
  float a0, a1;
  if (l == 0) {
    a0 = sigmoidf_(d00 + lb);  // k = 0: self
    a1 = sigmoidf_(d01 + lb);  // k = 1: other (F1*F0)
  } else {
    a0 = sigmoidf_(d01 + lb);  // k = 0: other (F0*F1)
    a1 = sigmoidf_(d11 + lb);  // k = 1: self
  }
  const float m = fmaxf(a0, a1);
  const float e0 = expf(a0 - m), e1 = expf(a1 - m);
  const float inv = 1.f / (e0 + e1);  // torch CPU softmax: x * (1 / sum)
  return l == 0 ? e1 * inv : e0 * inv;
}

// w_layer1 [64][128] into LDS (the graph-head workgroup keeps it for the whole launch).
__device__ __forceinline__ void stage_wl1(KParams& p, float* wl1) {
  constexpr int N4 = 64 * 128 / 4, K = N4 / NTHREADS;
  const float4* src = (const float4*)(p.w + W_WL1);
  float4 t[K];
#pragma unroll
  for (int k = 0; k < K; ++k) t[k] = src[k * NTHREADS + threadIdx.x];
#pragma unroll
  for (int k = 0; k < K; ++k) ((float4*)wl1)[k * NTHREADS + threadIdx.x] = t[k];
}

// Aux features of layer ll (U/PrepareBatchGraph.py:92-101): fp64 division, then fp32 as
// torch.tensor(...).type(FloatTensor).  They depend on the environment state only.
__device__ __forceinline__ void graph_aux(float* gs, const GraphInfo& gi, const GraphVar& gv, int ll) {
  const double N = (double)gi.n;
  gs[4 + ll * 4 + 0] = (float)((double)gv.n_cov / N);
  gs[4 + ll * 4 + 1] = (float)((double)gv.counter[ll] / (double)gi.e[ll]);
  gs[4 + ll * 4 + 2] = (float)((double)gv.twohop[ll] / (N * N));
  gs[4 + ll * 4 + 3] = 1.0f;
}

// Graph rows: y_l from the final virtual-node embeddings E_l = Y3_l (in L_YW), the layer-mix
// weights softmax(relu(y_l.WL1).WL2) and the aux features (U/PrepareBatchGraph.py:92-101).
__device__ __forceinline__ void head_publish_part(KParams& p, const float* lds, int g, unsigned long long htag, bool mix);
__device__ __noinline__ void graph_head(KParams&, float*, float*, const GraphInfo gi,
                                        const GraphVar&, bool wl1_resident, bool aux_ready,
                                        unsigned long long pub_tag = 0ull, int pub_g = -1) {
  float* const lds = lds_base();
  float* const scr = lds + L_SCR;
  const GraphVar& gv = *(const GraphVar*)(lds + L_GV);

  KParams& p = kp();  // kernel arguments through the implicit-argument SGPRs (uniform)
  const int w = wave_id(), l = w >> 2, q = w & 3, lane = lane_id();
  const float* wi = lds + L_W;
  float* gs = lds + L_GS;
  float* ys = lds + L_YS;
  const float* y = lds + L_YW;
  float* wl1 = scr;                 // [64][128] staged w_layer1
  float* f = scr + 64 * 128;        // [2][64] tanh features
  float* dots = f + 128;            // [4]
  float* zh = dots + 4;             // [2][128] hidden, then the 2 layer logits
  if (!wl1_resident) stage_wl1(p, wl1);
  if (q == 0) {
    // F = tanh(E.T + b): the graph row is part of the reference's [n+1, 64] sgemm -> FMA chain
    const float a = fma_chain<64>(0.f, 0, [&](int k) { return y[l * 64 + k]; },
                                  [&](int k) { return wget(wi + W_IT, 16, k, lane); });
    f[l * 64 + lane] = tanhf(a + wi[W_ITB + lane]);
  }
  __syncthreads();
  if (w == 0 && lane < 3) {
    const float* fa = f + (lane == 1 ? 64 : 0);
    const float* fb = f + (lane == 0 ? 0 : 64);
    dots[lane] = fma_chain<64>(0.f, 0, [&](int c) { return fa[c] * fb[c]; },
                               [&](int c) { return wi[W_ILW + c]; });  // 0: F0F0, 1: F1F1, 2: F0F1
  }
  __syncthreads();
  if (q == 0) {
    const float g = other_gate(l, dots[0], dots[1], dots[2], wi[W_ILB]);
    const float m = f[l * 64 + lane] + g * f[(1 - l) * 64 + lane];
    const float nr = wave_norm64(m);
    ys[l * 64 + lane] = m / fmaxf(nr, 1e-12f);
  }
  __syncthreads();
  // (dedicated mode: y and the aux features go to the tiles now, the layer-mix weights below
  // when they are done -- the tiles' attention needs them only for the final combine)
  if (pub_tag != 0ull) head_publish_part(p, lds, pub_g, pub_tag, false);
  if (threadIdx.x < 256) {
    const int ll = threadIdx.x >> 7, j = threadIdx.x & 127;
    const float a = fma_chain<64>(0.f, 0, [&](int k) { return ys[ll * 64 + k]; },
                                  [&](int k) { return wl1[k * 128 + j]; });
    zh[ll * 128 + j] = fmaxf(a, 0.f);
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    // the two layer logits, one lane each
    const int ll = threadIdx.x;
    zh[256 + ll] = fma_chain<128>(0.f, 0, [&](int j) { return zh[ll * 128 + j]; },
                                  [&](int j) { return wi[W_IWL2 + j]; });
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float z[2] = {zh[256], zh[257]};
    const float m = fmaxf(z[0], z[1]);
    const float e0 = expf(z[0] - m), e1 = expf(z[1] - m);
    const float inv = 1.f / (e0 + e1);
    gs[0] = e0 * inv;
    gs[1] = e1 * inv;
  }
  if (!aux_ready && threadIdx.x < 2) graph_aux(gs, gi, gv, threadIdx.x);
  __syncthreads();
}

// ------------------------------------------------------------------ graph-head hand-off
// Dedicated mode: the graph-head workgroup publishes y (L_YS, 128 floats) and the graph
// scalars (L_GS, 16) of graph g as 144 data-tagged 8-byte granules {value, tag} (one agent-
// scope `sc1` store each, tag = step + 1; the host zeroes the buffer before each launch), and
// each of 144 tile threads polls its own granule until the tag matches: one memory round trip
// for the hand-off, no separate flag (MI355X_MICROARCH.md, handoff-1to1 row: 8-byte granules).
constexpr int HB_FLOATS = 144;
constexpr int HB_MIX = 128;  // granules 128, 129: the layer-mix weights (L_GS[0..1])
__device__ __forceinline__ void head_publish(KParams& p, const float* lds, int g, unsigned long long htag) {
  if (threadIdx.x < HB_FLOATS) {
    const unsigned long long gr = (htag << 32) | (unsigned)__float_as_uint(lds[L_YS + threadIdx.x]);
    __hip_atomic_store((g_u64*)(p.hbuf + 2 * ((size_t)g * HB_FLOATS + threadIdx.x)), gr, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}
// the granules of head_publish without the layer-mix weights (mix = false), or those two alone
__device__ __forceinline__ void head_publish_part(KParams& p, const float* lds, int g, unsigned long long htag, bool mix) {
  const int t = threadIdx.x;
  if (t < HB_FLOATS && ((t == HB_MIX || t == HB_MIX + 1) == mix)) {
    const unsigned long long gr = (htag << 32) | (unsigned)__float_as_uint(lds[L_YS + t]);
    __hip_atomic_store((g_u64*)(p.hbuf + 2 * ((size_t)g * HB_FLOATS + t)), gr, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}
// skip_mix: every granule but the layer-mix weights (head_mix_weights polls those)
__device__ __forceinline__ void head_receive(KParams& p, float* lds, int g, unsigned long long htag, bool skip_mix = false) {
  if (threadIdx.x < HB_FLOATS && !(skip_mix && (threadIdx.x == HB_MIX || threadIdx.x == HB_MIX + 1))) {
    const g_u64* src = (const g_u64*)(p.hbuf + 2 * ((size_t)g * HB_FLOATS + threadIdx.x));
    const unsigned long long t0 = wall_clock64();
    unsigned long long gr;
    while (((gr = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) != htag) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > BARRIER_TIMEOUT_TICKS ||
          (__hip_atomic_load((g_u32*)p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & BAR_ERR)) {
        raise_err(p, ERR_TIMEOUT);
        gr = 0;
        break;
      }
    }
    lds[L_YS + threadIdx.x] = __uint_as_float((unsigned)gr);
  }
  __syncthreads();
}
// The layer-mix weights (w0, w1) of the head hand-off, polled by lanes 0 and 1 of the calling
// wave and broadcast to it.
__device__ __forceinline__ float2 head_mix_weights(KParams& p, int g, unsigned long long htag) {
  const int lane = lane_id();
  unsigned long long gr = 0ull;
  if (lane < 2) {
    const g_u64* src = (const g_u64*)(p.hbuf + 2 * ((size_t)g * HB_FLOATS + HB_MIX + lane));
    const unsigned long long t0 = wall_clock64();
    while (((gr = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) != htag) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > BARRIER_TIMEOUT_TICKS ||
          (__hip_atomic_load((g_u32*)p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & BAR_ERR)) {
        raise_err(p, ERR_TIMEOUT);
        gr = 0;
        break;
      }
    }
  }
  return make_float2(__uint_as_float((unsigned)__shfl((int)(unsigned)gr, 0, 64)),
                     __uint_as_float((unsigned)__shfl((int)(unsigned)gr, 1, 64)));
}

// Layer split, iteration 3: workgroup (tile, 1) hands its normalised layer-1 rows (S_E layer 1,
// 64 x 16) to workgroup (tile, 0) as 1024 data-tagged 8-byte granules in tile slot `slot`
// (tag = step + 1; the host zeroes the slots before each launch); the receiver polls each
// granule until its tag matches (one round trip, no flag), as the graph-head hand-off.
__device__ __forceinline__ void split_publish(KParams& p, const float* scr, int slot, unsigned long long tag) {
  g_u64* dst = (g_u64*)(p.xbuf + (size_t)slot * 2048 + 1024);
  const float* e = scr + S_E + 64 * LDT;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = threadIdx.x + NTHREADS * h, c = k >> 4, r = k & 15;
    __hip_atomic_store(dst + k, (tag << 32) | (unsigned)__float_as_uint(e[c * LDT + r]), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ void split_receive(KParams& p, float* scr, int slot, unsigned long long tag) {
  const g_u64* src = (const g_u64*)(p.xbuf + (size_t)slot * 2048 + 1024);
  float* e = scr + S_E + 64 * LDT;
  const unsigned long long t0 = wall_clock64();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = threadIdx.x + NTHREADS * h, c = k >> 4, r = k & 15;
    unsigned long long gr;
    while (((gr = __hip_atomic_load(src + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) != tag) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > BARRIER_TIMEOUT_TICKS ||
          (__hip_atomic_load((g_u32*)p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & BAR_ERR)) {
        raise_err(p, ERR_TIMEOUT);
        gr = 0;
        break;
      }
    }
    e[c * LDT + r] = __uint_as_float((unsigned)gr);
  }
  __syncthreads();
}

// One iteration of the graph-head workgroup (dedicated mode) for graph g: it == 2 builds
// Y1, Y2 from the S0 / S1 tile partials of iteration 1; it == 3 builds Y3 from S2, runs the
// graph head and publishes it.  Same arithmetic as the shared-mode path in the tile loop.
// ta / tb (dataflow mode): the tags the tiles' partial sums of this step carry (0: barrier mode).
__device__ __noinline__ void head_iteration(KParams&, float*, float*, int g, int it,
                                            unsigned long long htag, unsigned ta = 0, unsigned tb = 0) {
  float* const lds = lds_base();
  float* const scr = lds + L_SCR;

  KParams& p = kp();  // kernel arguments through the implicit-argument SGPRs (uniform)
  // diagnostics: iteration-3 timestamps of the first graph's head workgroup (slots 48-53)
  unsigned long long* hts = nullptr;
  if (p.prof != nullptr && it == 3 && (int)blockIdx.x == p.n_env && threadIdx.x == 0) {
    const int ps = ((volatile int*)(lds + L_MISC))[60];
    if (ps < p.prof_cap) hts = p.prof + (size_t)ps * PROF_SLOTS;
  }
#define HSTAMP(k)                              \
  do {                                         \
    if (hts != nullptr) hts[k] = wall_clock64(); \
  } while (0)
  HSTAMP(48);
  // graph info and state (fixed until the next phase A) are read at iteration 2 and kept in
  // LDS for iteration 3, whose head work is on the critical path
  GraphInfo* gic = (GraphInfo*)((int*)(lds + L_MISC) + 16);
  if (it == 2) {
    if (threadIdx.x < (int)(sizeof(GraphInfo) / 4)) ((int*)gic)[threadIdx.x] = ((const int*)(p.ginfo + g))[threadIdx.x];
    gv_load(p, g, (GraphVar*)(lds + L_GV));
  }
  __syncthreads();
  // references into LDS (a private copy would go through scratch memory)
  const GraphInfo& gi = *gic;
  const GraphVar& gv = *(const GraphVar*)(lds + L_GV);
  if (gv.status != ST_RUN) return;
  if (it == 2 && threadIdx.x < 2) graph_aux(lds + L_GS, gi, gv, threadIdx.x);
  const int nt = (gv.n_live + TILE - 1) / TILE;
  float* sbuf = scr + S_HID;  // [2][64]
  float* yw = lds + L_YW;
  if (it == 2) {
    if (threadIdx.x < 128) yw[threadIdx.x] = lds[L_Y0 + (threadIdx.x & 63)];
    graph_sum(p, gi, nt, 0, sbuf, scr + S_YP, ta, tb);
    vrow_update(lds + L_W, scr, sbuf, yw);  // Y1 from S0
    graph_sum(p, gi, nt, 1, sbuf, scr + S_YP, ta, tb);
    vrow_update(lds + L_W, scr, sbuf, yw);  // Y2 from S1
  } else {
    HSTAMP(49);
    graph_sum(p, gi, nt, 2, sbuf, scr + S_YP, ta, tb);
    HSTAMP(50);
    vrow_update(lds + L_W, scr, sbuf, yw);  // Y3 from S2
    HSTAMP(51);
    graph_head(p, lds, scr, gi, gv, true, true, htag, g);  // (y and the aux features published inside)
    HSTAMP(52);
    head_publish_part(p, lds, g, htag, true);
    HSTAMP(53);
  }
}

// Attention + Q head for one tile whose final embeddings are in S_E (both layers).
// Writes q for valid rows and this tile's arg-max partial.
__device__ __noinline__ void attention_q_tile(KParams&, float*, float*, const GraphInfo gi, int g,
                                              const int*, float* apart_out, unsigned long long htag,
                                              unsigned long long* ts) {
  float* const lds = lds_base();
  float* const scr = lds + L_SCR;
  const int* const rows = (const int*)(scr + S_ROW);

  KParams& p = kp();  // kernel arguments through the implicit-argument SGPRs (uniform)
  const float* wi = lds + L_W;
#ifdef MD_QPROF
  // queue-mode piece profile (qprof build, MD_VARIANT bit 8): slots 88.. of the launch record
  unsigned long long* qa = p.prof != nullptr && p.qmode && (p.variant & 8) ? p.prof + 88 : nullptr;
  unsigned long long tqa = qa != nullptr ? wall_clock64() : 0ull;
#define QATS(k)                                                   \
  do {                                                            \
    if (qa != nullptr && threadIdx.x == 0) {                      \
      const unsigned long long now_ = wall_clock64();             \
      atomicAdd(qa + (k), now_ - tqa);                            \
      tqa = now_;                                                 \
    }                                                             \
  } while (0)
#else
#define QATS(k) do {} while (0)
#endif
  const int w = wave_id(), l = w >> 2, cb = w & 3, lane = lane_id();
  const int ar = lane & 15, ak = lane >> 4;
  const int col = 16 * cb + ar;
  float* ate = scr + S_E + l * 64 * LDT;
  float* atf = scr + S_F + l * 64 * LDT;
  {
    // F_l = tanh(E_l . T + b)
    const float* tf = wi + W_IT + cb * 16 * 64;
    float xa[16], wa[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      xa[s] = ate[(4 * s + ak) * LDT + ar];
      wa[s] = tf[s * 64 + lane];
    }
    __builtin_amdgcn_sched_barrier(0);
    f4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 16; ++s) a = mfma16(xa[s], wa[s], a);
    const float b = wi[W_ITB + col];
#pragma unroll
    for (int r = 0; r < 4; ++r) atf[col * LDT + 4 * ak + r] = tanhf(a[r] + b);
  }
  __syncthreads();
  TSTAMP(38);
  QATS(0);
  float* dot = scr + S_DOT;
  float* gate = dot + 48;  // [2][16] weight of the other layer per (layer, row)
  if (w == 0) {
    if (lane < 48) {
      const int row = lane & 15, kind = lane >> 4;  // 0: F0F0, 1: F1F1, 2: F0F1
      const float* fa = scr + S_F + (kind == 1 ? 64 * LDT : 0);
      const float* fb = scr + S_F + (kind == 0 ? 0 : 64 * LDT);
      float a = 0.f;
#pragma unroll
      for (int h = 0; h < 64; h += 32) {
        float xa[32], xb[32], ww[32];
#pragma unroll
        for (int c = 0; c < 32; ++c) {
          xa[c] = fa[(h + c) * LDT + row];
          xb[c] = fb[(h + c) * LDT + row];
          ww[c] = wi[W_ILW + h + c];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < 32; ++c) a = fmaf(xa[c] * xb[c], ww[c], a);
      }
      dot[row * 3 + kind] = a;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes are done
    __builtin_amdgcn_wave_barrier();
    if (lane < 32) {
      const int ll = lane >> 4, row = lane & 15;
      gate[ll * 16 + row] = other_gate(ll, dot[row * 3 + 0], dot[row * 3 + 1], dot[row * 3 + 2], wi[W_ILB]);
    }
  }
  __syncthreads();
  TSTAMP(33);
  QATS(1);
  TSTAMP(35);
  // mix E_l = F_l + gate * F_other (mul then add, as the reference) fused into the first pass
  // of the row normalisation (each element is read there by exactly one thread)
  {
    float* red = scr + S_RED;
    const int t = threadIdx.x;
    if (t < 256) {
      const int ll = t >> 7, row = (t >> 3) & 15, j = t & 7;
      const float* f = scr + S_F + ll * 64 * LDT;
      const float* o = scr + S_F + (1 - ll) * 64 * LDT;
      float* e = scr + S_E + ll * 64 * LDT;
      const float gt = gate[ll * 16 + row];
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = 8 * i + j;
        const float v = f[c * LDT + row] + gt * o[c * LDT + row];
        e[c * LDT + row] = v;
        acc = fmaf(v, v, acc);
      }
      red[(ll * 16 + row) * 8 + j] = acc;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * ak + r;
      const float den = fmaxf(sqrtf(sumsq8_finish(red + (l * 16 + row) * 8)), 1e-12f);
      ate[col * LDT + row] = ate[col * LDT + row] / den;
    }
  }
  __syncthreads();
  TSTAMP(39);
  QATS(2);
  if (htag != 0ull) head_receive(p, lds, g, htag, true);  // (the layer-mix weights at the combine below)
  TSTAMP(40);
  QATS(3);
  {
    // e[a] = sum_b (h[a] * y[b]) * cp[b]: the reference's outer product then x cross_product
    // (net :356-363), a batched [64,64]x[64,1] matmul = an FMA chain over b.  Each thread
    // runs four independent chains of one layer (256 threads per layer).
    const int ll = threadIdx.x >> 8, t = threadIdx.x & 255;
    const float* at = scr + S_E + ll * 64 * LDT;
    typedef float f2v __attribute__((ext_vector_type(2)));
    f2v h[2], acc[2];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = t + 256 * k, row = idx >> 6, a = idx & 63;
      h[k >> 1][k & 1] = at[a * LDT + row];
      acc[k >> 1][k & 1] = 0.f;
    }
    const float4* y4 = (const float4*)(lds + L_YS + ll * 64);
    const float4* c4 = (const float4*)(wi + W_ICP);
    // chains k = 0..3 in pairs: packed multiply then packed FMA per b (each component rounds
    // exactly as h * y then fmaf(., cp, acc))
#pragma unroll 4
    for (int b4 = 0; b4 < 16; ++b4) {
      const float4 yv = y4[b4], cv = c4[b4];
      const float ys[4] = {yv.x, yv.y, yv.z, yv.w}, cs[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f2v yy = {ys[q], ys[q]}, cc = {cs[q], cs[q]};
#pragma unroll
        for (int k2 = 0; k2 < 2; ++k2) acc[k2] = __builtin_elementwise_fma(h[k2] * yy, cc, acc[k2]);
      }
    }
    float* af = scr + S_F + ll * 64 * LDT;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int idx = t + 256 * k, row = idx >> 6, a = idx & 63;
      af[a * LDT + row] = acc[k >> 1][k & 1];
    }
  }
  __syncthreads();
  TSTAMP(41);
  QATS(4);
  float* hid = scr + S_HID;
  if (cb < 2) {
    const float* hf = wi + W_IH1 + cb * 16 * 64;
    float xa[16], wa[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      xa[s] = atf[(4 * s + ak) * LDT + ar];
      wa[s] = hf[s * 64 + lane];
    }
    __builtin_amdgcn_sched_barrier(0);
    f4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 16; ++s) a = mfma16(xa[s], wa[s], a);
#pragma unroll
    for (int r = 0; r < 4; ++r) hid[(l * 16 + 4 * ak + r) * 33 + col] = fmaxf(a[r], 0.f);
  }
  __syncthreads();
  float* ql = scr + S_Q;
  if (threadIdx.x < 32) {
    const int ll = threadIdx.x >> 4, row = threadIdx.x & 15;
    const float* gs = lds + L_GS;
    float a = fma_chain<32>(0.f, 0, [&](int k) { return hid[(ll * 16 + row) * 33 + k]; },
                            [&](int k) { return wi[W_IW2 + k]; });
    for (int k = 0; k < 4; ++k) a = fmaf(gs[4 + ll * 4 + k], wi[W_IW2 + 32 + k], a);
    ql[ll * 16 + row] = a;
  }
  // the arg-max partial below runs on the same wave: its LDS writes are visible to itself
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  TSTAMP(42);
  QATS(5);
  if (threadIdx.x < 64) {
    // q = w0 * Q0 + w1 * Q1 per row, and the tile's arg-max partial by a 16-lane butterfly
    // (max / min index / count / second: order-free, as the sequential scan)
    const float* gs = lds + L_GS;
    const int lane = threadIdx.x;
    float bm = NEG_INF, bs = NEG_INF;
    int bi = 0x7fffffff, bc = 0;
    const float2 mw = htag != 0ull ? head_mix_weights(p, g, htag) : make_float2(gs[0], gs[1]);
    if (lane < 16) {
      const int v = rows[lane];
      if (v >= 0) {
        const float qq = mw.x * ql[lane] + mw.y * ql[16 + lane];
        stc(p.q + gi.node_off + v, qq);
        if (p.qspec != nullptr)  // this step's Q for the speculative workgroups (buffer = step & 1)
          stc(p.qspec + (size_t)(((const int*)(lds + L_MISC))[60] & 1) * p.qspec_n + gi.node_off + v, qq);
        bm = qq;
        bi = v;
        bc = 1;
      }
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      const float m2 = __shfl_xor(bm, o, 64), s2 = __shfl_xor(bs, o, 64);
      const int i2 = __shfl_xor(bi, o, 64), c2 = __shfl_xor(bc, o, 64);
      if (c2 != 0) argmax_combine(bm, bs, bi, bc, m2, s2, i2, c2);
    }
    if (p.df != nullptr) {
      // dataflow mode: four tagged granules, once this wave's q / qspec stores are done (phase A
      // and the speculative workgroups read q after seeing the partial)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane < 4)
        df_st((unsigned long long*)apart_out + lane, lane == 0 ? bm : lane == 1 ? bs : __int_as_float(lane == 2 ? bi : bc),
              (unsigned)htag << 1);
    } else if (lane == 0) {
      stc4(apart_out, 0, make_float4(bm, bs, __int_as_float(bi), __int_as_float(bc)));
    }
  }
  __syncthreads();
  QATS(6);
#undef QATS
}


// Phase timestamps of workgroup 0 (diagnostics only; p.prof == nullptr in normal runs).
#define MD_PROF(slot)                                                                            \
  do {                                                                                           \
    if (p.prof != nullptr && blockIdx.x == 0 && threadIdx.x == 0 && pstep < p.prof_cap)          \
      p.prof[(size_t)pstep * PROF_SLOTS + (slot)] = wall_clock64();                                      \
  } while (0)

// Tile-side timestamps of the first tile workgroup (slots 23-31: per iteration after the
// gather, after update / normalize / stores, at the tile's end).
#ifdef MD_NO_PROFT
#define MD_PROF_T(slot) do {} while (0)
#else
#define MD_PROF_T(slot)                                                                          \
  do {                                                                                           \
    if (p.prof != nullptr && (int)blockIdx.x == twg0 && t == t0 && threadIdx.x == 0 &&            \
        pstep < p.prof_cap)                                                                      \
      p.prof[(size_t)pstep * PROF_SLOTS + (slot)] = wall_clock64();                              \
  } while (0)
#endif

__device__ __forceinline__ void load_weights(float* dst, const float* src) {
  constexpr int N4 = W_IEND / 4, K = (N4 + NTHREADS - 1) / NTHREADS;
  const float4* s4 = (const float4*)src;
  float4* d4 = (float4*)dst;
  float4 t[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = k * NTHREADS + threadIdx.x;
    if (i < N4) t[k] = s4[i];
  }
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = k * NTHREADS + threadIdx.x;
    if (i < N4) d4[i] = t[k];
  }
}
static_assert(W_IEND % 4 == 0, "weight image is copied as float4");

// Graph-list index of global tile t (prefix in LDS, ng + 1 entries).
__device__ __forceinline__ int tile_graph(const int* pref, int ng, int t) {
  int lo = 0, hi = ng - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (pref[mid] <= t) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// ------------------------------------------------------------------ queue mode (batches)
// Rollouts of many graphs without lock-step grid barriers: every workgroup pops work items
// from one device queue and pushes the items they enable, so one graph's environment step,
// another's virtual node and the tiles of a third run at the same time, and a graph that
// waits for a host answer or finished early holds nobody up.  Per graph and removal step:
//   ENV  phase A (arg-max of the last Q, action, mutual-LMCC fixed point, features)
//   -> TILE(1, j) for its tiles -> TILE(2, j) -> VN (virtual node Y1..Y3 + graph head,
//   published as tagged granules) -> TILE(3, j) (attention, Q, arg-max partials) -> ENV.
// The last tile of a stage (per-graph counter) pushes the next stage.  Items are 32-bit
// {kind, iteration, graph slot, tile} in a ring of 8-byte slots tagged with their ticket + 1:
// a consumer takes a ticket (atomic add) and polls its slot; a producer reserves tickets and
// writes the slots after draining its data stores (the fence-free sc1 protocol of the grid
// barrier).  Every item runs to completion without waiting on another item, so the queue
// cannot deadlock; when the last graph stops, one EXIT item per workgroup is pushed.
enum : unsigned { QK_ENV = 1, QK_TILE = 2, QK_VN = 3, QK_EXIT = 4 };
enum : int { QC_HEAD = 0, QC_TAIL = 1, QC_REM = 2, QC_ADMIT = 3 };
// Graphs running at once in queue mode: the larger of 3/8 of the workgroups and 5/16 of the
// launch's graphs, the latter at most Q_ADMIT_MAX (sweeps of 64..192 and all: 96 best for 256
// GMM N=1000 graphs on 256 CUs, 160 for 512; for 4096-graph launches see DESIGN.md).
// MD_VARIANT bits 16+ override.
constexpr int Q_ADMIT_MAX = 160;
__device__ __forceinline__ int q_admit(KParams& p) {
  const int v = (int)((unsigned)p.variant >> 16);
  return v > 0 ? v : max(1, max((int)(3 * gridDim.x) / 8, min(Q_ADMIT_MAX, (5 * p.nglist) / 16)));
}
__device__ __forceinline__ unsigned q_item(unsigned kind, int it, int gl, int j) {
  return kind | ((unsigned)it << 3) | ((unsigned)gl << 5) | ((unsigned)j << 17);
}
__device__ __forceinline__ int q_item_gl(unsigned item) { return (int)((item >> 5) & (QG_CAP - 1)); }
// Tile item i of a stage with nt tiles and tpi tiles per item: first tile j = i * tpi (bits
// 17-29, < Q_MAX_TILES), the number of further tiles in bits 30-31 (they run back to back on one workgroup:
// one stage signal and one pop for all of them).
__device__ __forceinline__ unsigned q_item_tile(int it, int gl, int i, int nt, int tpi) {
  const int j = i * tpi, extra = min(tpi, nt - j) - 1;
  return q_item(QK_TILE, it, gl, j) | ((unsigned)extra << 30);
}
__device__ __forceinline__ int q_item_j(unsigned item) { return (int)((item >> 17) & (Q_MAX_TILES - 1)); }
__device__ __forceinline__ int q_item_extra(unsigned item) { return (int)(item >> 30); }
// Tiles per item: 2 (MD_VARIANT bits 9-10 = 1..3 override; sweep of 1..4 tiles x admission
// 96..160 on 256 / 512 graphs: 2 best, -3 % / -5 % against 1).  Per-graph stage size word in
// qg[2 gl + 1]: items of a tile stage | tiles << 16.
__device__ __forceinline__ int q_tiles_per_item(KParams& p) {
  const int f = (p.variant >> 9) & 3;
  return f == 0 ? 2 : f;
}
// In the launch's tail (every graph admitted and at most 1/8 of the workgroups' count still
// running) a step's tiles go one per item: fewer graphs share the chip, so each stage's items
// are spread over more workgroups (per graph and step the tiles per item are fixed: qg word
// bits 28-29).
__device__ __forceinline__ int q_tail(KParams&) { return (int)gridDim.x / 8; }
// Pushes n items f(0..n-1); every thread of the workgroup calls it.  The ring's head / tail
// tickets sit on a line of their own (p.qring); Q_CAP slots.
__device__ __forceinline__ g_u32* q_ctl(KParams& p) { return (g_u32*)p.qring; }
__device__ __forceinline__ unsigned long long* q_slot(KParams& p, unsigned tk) {
  return p.qslot + (tk & (unsigned)(Q_CAP - 1));
}
template <class F>
__device__ __forceinline__ void q_push(KParams& p, int n, F&& f, int* bc) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's data stores are done
  __syncthreads();
  if (threadIdx.x == 0)
    bc[0] = (int)__hip_atomic_fetch_add(q_ctl(p) + QC_TAIL, (unsigned)n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const unsigned base = (unsigned)bc[0];
  for (int i = threadIdx.x; i < n; i += NTHREADS) {
    const unsigned tk = base + (unsigned)i;
    const unsigned long long v = ((unsigned long long)(tk + 1u) << 32) | f(i);
    __hip_atomic_store((g_u64*)q_slot(p, tk), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
}
// EXIT items, two per workgroup of the launch (a workgroup may hold one ticket it never uses)
__device__ __forceinline__ void q_push_exit(KParams& p, int* bc) {
  q_push(p, 2 * gridDim.x, [&](int) { return (unsigned)QK_EXIT; }, bc);
}
// Thread 0 takes the next ticket; it is taken one item ahead (the atomic's latency overlaps
// the current item), so a workgroup may hold one ticket it never uses when it exits: EXIT
// items are pushed twice per workgroup.
__device__ __forceinline__ unsigned q_take(KParams& p) {
  return threadIdx.x == 0
             ? __hip_atomic_fetch_add(q_ctl(p) + QC_HEAD, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
             : 0u;
}
// Thread 0 reads ticket tk's slot without waiting for it (issued beside an item's last memory
// round trip, so a slot that is already filled costs no round trip of its own in q_wait).
__device__ __forceinline__ unsigned long long q_peek(KParams& p, unsigned tk) {
  return threadIdx.x == 0
             ? __hip_atomic_load((const g_u64*)q_slot(p, tk), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
             : 0ull;
}
__device__ __forceinline__ unsigned q_wait(KParams& p, unsigned tk, int* bc, unsigned long long pre) {
  if (threadIdx.x == 0) {
    unsigned long long v = pre;
    // an error anywhere: stop taking work (the grid drains).  Checked only when the item is not
    // there yet: a workgroup that keeps finding work sees the error once the queue runs dry.
    const bool ready = (v >> 32) == (unsigned long long)(tk + 1u);
    if (!ready) v = QK_EXIT;
    if (!ready && !(__hip_atomic_load((g_u32*)p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & BAR_ERR)) {
      const g_u64* slot = (const g_u64*)q_slot(p, tk);
      const unsigned long long t0 = wall_clock64();
      while (((v = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) != (unsigned long long)(tk + 1u)) {
        __builtin_amdgcn_s_sleep(2);
        if (__hip_atomic_load((g_u32*)p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & BAR_ERR) {
          v = QK_EXIT;
          break;
        }
        if (wall_clock64() - t0 > (p.h_req != nullptr ? HOST_TIMEOUT_TICKS : BARRIER_TIMEOUT_TICKS)) {
          raise_err(p, ERR_TIMEOUT);
          v = QK_EXIT;
          break;
        }
      }
    }
    bc[1] = (int)(unsigned)v;
  }
  __syncthreads();
  const unsigned item = (unsigned)bc[1];
  __syncthreads();
  return item;
}

// Queue mode, after phase A of graph slot gl in LDS mode: the alive neighbour lists of every
// tile of the step, both layers, written to the tiles' neighbour-list cache slots in
// nbc_store's format, so the iteration-1 tiles reload them like iterations 2-3 instead of each
// building its own.  The same lists: live rows in ascending id order, 16 per tile, each row's
// alive CSR entries in CSR order (the reference's in_edges order); a tile whose layer has more
// than NB_CAP entries gets ok = 0 (the per-row gather).  Each CSR entry comes from the static
// packed adjacency (adjx: layer-local edge id and neighbour in one word) and is alive when its
// edge's state in LDS is, so both layers' entries are one round of independent loads (no
// alive-flag reads: the flags in HBM are the same states' write-back).  Returns false (the tiles
// build their lists) when the scratch does not fit.
__device__ __forceinline__ bool env_build_lists(KParams&, const GraphInfo gi, int gl) {
  KParams& p = kp();
  float* const lds = lds_base();
  int* ia = (int*)(lds + L_W);
  const int n = gi.n, e0 = gi.e[0], et = gi.e[0] + gi.e[1];
  const EnvLayout Lo = env_layout(n, et);
  const EnvView<false> E = env_view<false>(p, gi, ia);
  const int nl = ((const GraphVar*)(lds + L_GV))->n_live, nt = (nl + TILE - 1) / TILE;
  // (the per-thread packed counts below need fewer than 2^16 CSR entries per layer)
  if (Lo.total + 5 * nl + 2 * nt + 8 > A_WORDS || p.gtoff[gl] + nt > p.nbc_slots || nl <= 0 || gi.e[0] >= ADJX_EDGE_LIMIT ||
      gi.e[1] >= ADJX_EDGE_LIMIT || n > 65536)
    return false;
  // scratch after the environment: node of each live position, per layer the per-position
  // prefixes of the CSR extent and of the alive count (nl + 1 each), per-tile alive totals
  int* pn = ia + Lo.total;
  int* px[2] = {pn + nl, pn + 2 * nl + 1};
  int* pd[2] = {pn + 3 * nl + 2, pn + 4 * nl + 3};
  int* tt = pn + 5 * nl + 4;
  int* tmp = E.tmp;
  int* base_slot = p.nbc + (size_t)p.gtoff[gl] * NBC_INTS;
#ifdef MD_QPROF
  // diagnostics (qprof build, MD_VARIANT bit 8): the builder's pieces in prof[50 + k]
  unsigned long long* lqd = p.prof != nullptr && (p.variant & 8) ? p.prof + 50 : nullptr;
  unsigned long long lqt = wall_clock64();
#define LQTS(k)                                                                        \
  do {                                                                                 \
    if (lqd != nullptr && threadIdx.x == 0) {                                          \
      const unsigned long long now_ = wall_clock64();                                  \
      atomicAdd(lqd + (k), now_ - lqt);                                                \
      lqt = now_;                                                                      \
    }                                                                                  \
  } while (0)
#else
#define LQTS(k) do {} while (0)
#endif
  {
    // live positions (ascending ids, as the live list)
    const int chunk = (n + NTHREADS - 1) / NTHREADS;
    const int x0 = min(n, (int)threadIdx.x * chunk), x1 = min(n, x0 + chunk);
    int c = 0;
    for (int x = x0; x < x1; ++x) c += uf_load(E.deg0, x) > 0;
    int tot = 0;
    int k = block_excl_scan(c, tmp, &tot);
    for (int x = x0; x < x1; ++x)
      if (uf_load(E.deg0, x) > 0) pn[k++] = x;
  }
  __syncthreads();
  LQTS(0);
  // prefixes over live positions of both layers' CSR extents and alive counts (residual degrees)
  {
    const int chunk = (nl + NTHREADS - 1) / NTHREADS;
    const int i0 = min(nl, (int)threadIdx.x * chunk), i1 = min(nl, i0 + chunk);
    int sx[2] = {0, 0}, sd[2] = {0, 0};
    for (int i = i0; i < i1; ++i) {
      const int x = pn[i];
      sx[0] += E.rp[0][x + 1] - E.rp[0][x];
      sx[1] += E.rp[1][x + 1] - E.rp[1][x];
      sd[0] += uf_load(E.deg0, x);
      sd[1] += uf_load(E.deg1, x);
    }
    int tx = 0, td = 0;
    const int ox = block_excl_scan(sx[0] | (sx[1] << 16), tmp, &tx);
    const int od = block_excl_scan(sd[0] | (sd[1] << 16), tmp, &td);
    int ax[2] = {ox & 0xffff, ox >> 16}, ad[2] = {od & 0xffff, od >> 16};
    for (int i = i0; i < i1; ++i) {
      const int x = pn[i];
#pragma unroll
      for (int l = 0; l < 2; ++l) {
        px[l][i] = ax[l];
        pd[l][i] = ad[l];
        ax[l] += E.rp[l][x + 1] - E.rp[l][x];
        ad[l] += uf_load(l ? E.deg1 : E.deg0, x);
      }
    }
    if (threadIdx.x == 0) {
      px[0][nl] = tx & 0xffff;
      px[1][nl] = tx >> 16;
      pd[0][nl] = td & 0xffff;
      pd[1][nl] = td >> 16;
    }
  }
  __syncthreads();
  LQTS(1);
  // each thread: a contiguous run of the live rows' CSR entries per layer; the first R of both
  // layers loaded in one round (kept for the write pass), longer runs in further rounds.  A run
  // is walked row by row with the row's boundary and CSR base in registers (LDS reads only where
  // the run crosses into the next live row).
  constexpr int R = 20;
  struct Walk {
    int i, nxt, base;  // live position, its CSR-extent end, CSR position - extent index
  };
  int eb[2], ee[2];
  Walk w0[2];
  int xs[2][R];
  const int* adjx[2] = {p.adjx[0] + gi.coff[0], p.adjx[1] + gi.coff[1]};
#pragma unroll
  for (int l = 0; l < 2; ++l) {
    const int te = px[l][nl], ce = (te + NTHREADS - 1) / NTHREADS;
    eb[l] = min(te, (int)threadIdx.x * ce);
    ee[l] = min(te, eb[l] + ce);
    int lo = 0, hi = nl - 1;  // last position with px[i] <= eb
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (px[l][mid] <= eb[l]) lo = mid; else hi = mid - 1;
    }
    w0[l].i = lo;
    w0[l].nxt = px[l][lo + 1];
    w0[l].base = E.rp[l][pn[lo]] - px[l][lo];
  }
  auto advance = [&](int l, Walk& w, int e) {
    while (e >= w.nxt) {
      ++w.i;
      w.nxt = px[l][w.i + 1];
      w.base = E.rp[l][pn[w.i]] - px[l][w.i];
    }
  };
  {
    int cp[2][R];
#pragma unroll
    for (int l = 0; l < 2; ++l) {
      Walk w = w0[l];
#pragma unroll
      for (int u = 0; u < R; ++u) {
        const int e = eb[l] + u;
        cp[l][u] = -1;
        if (e < ee[l]) {
          advance(l, w, e);
          cp[l][u] = w.base + e;
        }
      }
    }
#pragma unroll
    for (int l = 0; l < 2; ++l)
#pragma unroll
      for (int u = 0; u < R; ++u) xs[l][u] = cp[l][u] >= 0 ? adjx[l][cp[l][u]] : -1;
  }
  auto alive = [&](int l, int x) { return x >= 0 && E.st[(x >> 16) + (l ? e0 : 0)] == E_ALIVE; };
  int keep[2] = {0, 0};
#pragma unroll
  for (int l = 0; l < 2; ++l) {
#pragma unroll
    for (int u = 0; u < R; ++u) keep[l] += alive(l, xs[l][u]);
    if (eb[l] + R < ee[l]) {
      Walk w = w0[l];
      advance(l, w, eb[l] + R);
      for (int b = eb[l] + R; b < ee[l]; b += R) {
        int xr[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
          xr[u] = -1;
          if (b + u < ee[l]) {
            advance(l, w, b + u);
            xr[u] = adjx[l][w.base + b + u];
          }
        }
#pragma unroll
        for (int u = 0; u < R; ++u) keep[l] += alive(l, xr[u]);
      }
    }
  }
  LQTS(2);
  int tk = 0;
  const int o01 = block_excl_scan(keep[0] | (keep[1] << 16), tmp, &tk);
#pragma unroll
  for (int l = 0; l < 2; ++l) {
    int o = l ? o01 >> 16 : o01 & 0xffff;
    Walk w = w0[l];
    // an alive entry's place in its tile's list: its index among the layer's alive entries,
    // minus that of the tile's first row
    auto put = [&](int x, int e) {
      advance(l, w, e);
      if (!alive(l, x)) return;
      const int j = w.i >> 4, wo = o - pd[l][j << 4];
      if (wo < NB_CAP) {
        uint16_t* ent = (uint16_t*)(base_slot + (size_t)j * NBC_INTS + NBC_HDR + l * NBC_LWORDS);
        __hip_atomic_store((__attribute__((address_space(1))) uint16_t*)(ent + wo), (uint16_t)(x & 0xffff),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      ++o;
    };
#pragma unroll
    for (int u = 0; u < R; ++u)
      if (eb[l] + u < ee[l]) put(xs[l][u], eb[l] + u);
    for (int b = eb[l] + R; b < ee[l]; b += R) {
      int xr[R];
      Walk w2 = w;
#pragma unroll
      for (int u = 0; u < R; ++u) {
        xr[u] = -1;
        if (b + u < ee[l]) {
          advance(l, w2, b + u);
          xr[u] = adjx[l][w2.base + b + u];
        }
      }
#pragma unroll
      for (int u = 0; u < R; ++u)
        if (b + u < ee[l]) put(xr[u], b + u);
    }
  }
  LQTS(3);
  // headers: per row its offset and count in the tile's list, per tile the total
  for (int q = threadIdx.x; q < 2 * nt * TILE; q += NTHREADS) {
    const int l = q >= nt * TILE, qq = q - l * nt * TILE;
    const int j = qq >> 4, r = qq & 15, at = (j << 4) + r, end = min(nl, (j + 1) << 4);
    const int* d = pd[l];
    int* hd = base_slot + (size_t)j * NBC_INTS;
    const int tot = d[end] - d[j << 4];
    stc(hd + l * 16 + r, at < nl ? d[at] - d[j << 4] : tot);
    stc(hd + 32 + l * 16 + r, at < nl ? d[at + 1] - d[at] : 0);
    if (r == 0) {
      stc(hd + 64 + l, tot);
      tt[l * nt + j] = tot;
    }
  }
  __syncthreads();
  for (int j = threadIdx.x; j < nt; j += NTHREADS)
    stc(base_slot + (size_t)j * NBC_INTS + 66, (tt[j] <= NB_CAP && tt[nt + j] <= NB_CAP) ? 1 : 0);
  __syncthreads();
  LQTS(4);
#undef LQTS
  return true;
}

// ------------------------------------------------------------------ batch speculation
// Queue launches (wave items, md_queue_kernel): the environment item of step t queues, beside
// its iteration-1 tiles, a speculative item for the graph's likely next pick -- the live node of
// largest Q(t - 1) after step t (env_features' candidate) -- that stages the state after step t,
// covers that node, runs the same mutual-LMCC fixed point and publishes the result in the
// graph's slot of this removal-count parity (spec_loop's SRES layout and tags) while the forward
// pass of step t runs.  The environment item of step t + 1 takes it when it picks that node
// (env_step: apply the kill list, copy the features) and runs the fixed point itself otherwise.
// Slot ownership: the environment item claims a slot (STARTED = {node, tag}) only when the last
// item on it has left (EXITED = that item's tag, written after all its stores drained), so no
// two items ever write one slot; step t + 1 reads a result only through its done and features
// tags, each written after the data it covers drained, and naming its own launch, removal count
// and node.  A state staged while step t + 1 already rewrites it can only give a result tagged
// for removal count t, which no later step asks for.
__device__ __forceinline__ unsigned bspec_item(int gl, int steps) { return q_item(QK_ENV, 2, gl, steps & 1); }

// The speculative item of graph slot gl (the whole workgroup; phase A's LDS area, so the caller
// reloads the weights afterwards).
__device__ __noinline__ void bspec_step(KParams&, int gl, int par) {
  KParams& p = kp();
  float* const lds = lds_base();
  int* misc = (int*)(lds + L_MISC);
  const int g = p.glist[gl];
  const GraphInfo gi = p.ginfo[g];
  const int n = gi.n, et = gi.e[0] + gi.e[1];
  int* slot = bspec_slot(p, gi, par);
  if (threadIdx.x == 0) {
    const unsigned long long stw = __hip_atomic_load((const g_u64*)(slot + SRES_STARTED), __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
    const int s_now = ldc(&p.gvar[g].steps), st = ldc(&p.gvar[g].status);
    const unsigned tag = (unsigned)stw;
    const int c = (int)(stw >> 32);
    // still the state this item was queued for (a later environment step already took its place
    // otherwise), and a state the LDS environment holds
    const bool ok = tag == spec_tag(p.launch_seq, s_now) && st == ST_RUN && c >= 0 && c < n &&
                    phase_a_fits_lds(n, et) && (s_now & 1) == par;
    misc[22] = ok ? 1 : 0;
    misc[23] = c;
    misc[24] = (int)tag;
  }
  __syncthreads();
  const unsigned tag = (unsigned)misc[24];
  if (misc[22]) {
    const int c = misc[23];
    int* ia = (int*)(lds + L_W);
    const EnvView<false> E = env_view<false>(p, gi, ia);
    env_stage_lds(E, n);
    __syncthreads();
    if (threadIdx.x == 0) E.cov8[c] = 1;  // c is live, hence not covered
    __syncthreads();
    int pr[2], cc[2];
    const int lm = mcc_fixed_point<false>(E, pr, nullptr, c, cc);
    const int nd = E.hdr[1];
    for (int i = threadIdx.x; i < nd; i += NTHREADS) {
      const int e = E.dl[i];
      if (!MD_BOK(e < et, 24)) continue;
      const int l = e < E.e0 ? 0 : 1, kk = e < E.e0 ? e : e - E.e0;
      stc(slot + SRES_HDR + 3 * i, e | ((int)E.st[e] << 16));
      stc(slot + SRES_HDR + 3 * i + 1, E.epos[l][2 * kk]);
      stc(slot + SRES_HDR + 3 * i + 2, E.epos[l][2 * kk + 1]);
    }
    if (threadIdx.x == 0) {
      stc(slot + 2, lm);
      stc(slot + 3, pr[0]);
      stc(slot + 4, pr[1]);
      stc(slot + 5, cc[0]);
      stc(slot + 6, cc[1]);
      stc(slot + 7, nd);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)  // {killed edges << 48 | node << 32 | tag}
      __hip_atomic_store((g_u64*)slot, ((unsigned long long)(unsigned)(c | (nd << 16)) << 32) | tag, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    const EnvAgg ag = env_features<false>(E, n, slot + sres_deg(et), slot + sres_deg(et) + n,
                                          (float*)(slot + sres_live(et, n)), nullptr);
    if (threadIdx.x == 0) {
      stc(slot + 12, ag.nlive);
      stc(slot + 13, ag.dm0);
      stc(slot + 14, ag.dm1);
      stc(slot + 15, ag.sd0);
      stc(slot + 16, ag.sd1);
      stc(slot + 17, ag.bad);
      stc(slot + 18, (int)(ag.th0 & 0xffffffffll));
      stc(slot + 19, (int)(ag.th0 >> 32));
      stc(slot + 20, (int)(ag.th1 & 0xffffffffll));
      stc(slot + 21, (int)(ag.th1 >> 32));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_store((g_u64*)(slot + SRES_FEAT), ((unsigned long long)(unsigned)c << 32) | tag, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  // leave the slot (after every store of this item drained)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) stc(slot + BSPEC_EXITED, (int)tag);
}

// The environment item's side (thread 0, after phase A; the candidate in misc[20]): the slot of
// the new state's parity, free (EXITED == STARTED) -> claimed for the candidate.  Returns
// whether to queue the speculative item (bspec_item) with the tiles.  stw / exw: the slot's
// words, loaded earlier (their round trip overlaps the neighbour lists).
__device__ __forceinline__ bool bspec_claim(KParams& p, const GraphInfo& gi, int steps, int cand, unsigned long long stw,
                                            unsigned exw) {
  if (cand < 0 || (unsigned)stw != exw) return false;
  __hip_atomic_store((g_u64*)(bspec_slot(p, gi, steps) + SRES_STARTED),
                     ((unsigned long long)(unsigned)cand << 32) | spec_tag(p.launch_seq, steps), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  return true;
}

// One tile of one graph for iteration `it` (queue mode; the same pieces and order as the
// lock-step tile loop).  Neighbour lists: built and cached at iteration 1, reloaded at 2-3.
__device__ __noinline__ void queue_tile(KParams&, float* lds, int g, int gl, int it, int j) {
  KParams& p = kp();
  float* scr = lds + L_SCR;
  int* rows = (int*)(scr + S_ROW);
  const GraphInfo gi = p.ginfo[g];
  // iteration 3: the head granules' tag (predictions so far + 1), read now, used at the attention
  const int npv = it == 3 ? ldc(&p.gvar[g].npred) : 0;
  lds_i32* hdr = (lds_i32*)(int*)(scr + S_NBH);
  // diagnostics (builds with -DMD_QPROF, md_profile with MD_VARIANT bit 8): per-piece device
  // ticks of the tile items, summed over items in slots 20.. (8 per iteration)
#ifdef MD_QPROF
  unsigned long long* qd = p.prof != nullptr && (p.variant & 8) ? p.prof + 20 + 8 * (it - 1) : nullptr;
  unsigned long long tqd = qd != nullptr ? wall_clock64() : 0ull;
#else
  constexpr unsigned long long* qd = nullptr;
  unsigned long long tqd = 0ull;
#endif
#define QTS(k)                                                    \
  do {                                                            \
    if (qd != nullptr && threadIdx.x == 0) {                      \
      const unsigned long long now_ = wall_clock64();             \
      atomicAdd(qd + (k), now_ - tqd);                            \
      tqd = now_;                                                 \
    }                                                             \
  } while (0)
  const int slot = p.gtoff[gl] + j;  // neighbour-list cache slot: the graph's tile within the launch
  const bool cacheable = slot < p.nbc_slots;
  // iteration 1: the environment item built this step's lists when its flag says so (read in
  // the same round trip as the speculative reload)
  const bool want = cacheable;
  int cw = 0, ch = 0, built = 0;
  if (want) {
    const int* src = p.nbc + (size_t)slot * NBC_INTS;
    cw = ldc(src + NBC_HDR + (threadIdx.x >> 8) * NBC_LWORDS + (threadIdx.x & 255));
    if (threadIdx.x < 67) ch = ldc(src + threadIdx.x);
    if (it == 1 && threadIdx.x == 67) built = ldc(p.qg + 2 * QG_CAP + gl);
  }
  if (threadIdx.x < TILE) {
    const int r = j * TILE + threadIdx.x;
    const int nl = ldc(&p.gvar[g].n_live);
    const float4 e = ldc4((const float*)(p.live + 4 * (size_t)gi.node_off), min(r, gi.n - 1) * 16);
    const bool ok = r < nl && MD_BOK(__float_as_int(e.x) >= 0 && __float_as_int(e.x) < gi.n && nl <= gi.n, 6);
    const unsigned c = (unsigned)__float_as_int(e.w);
    rows[threadIdx.x] = ok ? __float_as_int(e.x) : -1;
    hdr[64 + threadIdx.x] = ok ? __float_as_int(e.y) : 0;
    hdr[96 + threadIdx.x] = ok ? (int)(c & 0xffffu) : 0;
    hdr[64 + 16 + threadIdx.x] = ok ? __float_as_int(e.z) : 0;
    hdr[96 + 16 + threadIdx.x] = ok ? (int)(c >> 16) : 0;
  }
  int* misc = (int*)(lds + L_MISC);
  if (threadIdx.x == 67) misc[58] = it > 1 || built;
  __syncthreads();
  const bool cached = want && misc[58] != 0;
  if (cached) {
    ((lds_i32*)(int*)(scr + S_NBL))[(threadIdx.x >> 8) * NBC_LWORDS + (threadIdx.x & 255)] = cw;
    if (threadIdx.x < 64) hdr[threadIdx.x] = ch;
    else if (threadIdx.x < 66) hdr[128 + threadIdx.x - 64] = ch;
    else if (threadIdx.x == 66) misc[59] = ch;
  }
  __syncthreads();
  QTS(0);
  bool nb_ok;
  if (cached) {
    nb_ok = misc[59] != 0;
    const int nw0 = (hdr[128] + 1) >> 1, nw1 = (hdr[129] + 1) >> 1;
    if (nb_ok && (nw0 > 256 || nw1 > 256)) {
      const int* src = p.nbc + (size_t)slot * NBC_INTS + NBC_HDR;
      lds_i32* words = (lds_i32*)(int*)(scr + S_NBL);
      for (int i = 256 + (int)threadIdx.x; i < nw0; i += NTHREADS) words[i] = ldc(src + i);
      for (int i = 256 + (int)threadIdx.x; i < nw1; i += NTHREADS) words[NBC_LWORDS + i] = ldc(src + NBC_LWORDS + i);
      __syncthreads();
    }
  } else {
    nb_ok = build_nb_lists(p, gi, rows, scr, nullptr, -1);
    if (cacheable) nbc_store(p, slot, scr, nb_ok);
  }
  QTS(1);
  if (nb_ok) gather_tile2(p, gi, it, rows, scr);
  else gather_tile(p, gi, it, rows, scr);
  __syncthreads();
  QTS(2);
  update_tile(lds + L_W, scr);
  __syncthreads();
  QTS(3);
  normalize_tile(scr + S_E, scr);
  __syncthreads();
  QTS(4);
  if (threadIdx.x < 128 && it < 3) {
    // tile partial sums of the virtual node (rows in ascending compact order from 0)
    const int l = threadIdx.x >> 6, c = threadIdx.x & 63;
    const float* ate = scr + S_E + l * 64 * LDT + c * LDT;
    const float* atx = scr + S_X + l * 64 * LDT + c * LDT;
    const int nv = tile_rows_valid(rows);
    const float s_new = col_sum16(ate, nv), s_old = it == 1 ? col_sum16(atx, nv) : 0.f;
    float* sp = p.spart + (size_t)(gi.tile_off + j) * 384;
    if (it == 1) {
      stc(sp + l * 64 + c, s_old);        // S0 (first-layer input)
      stc(sp + 128 + l * 64 + c, s_new);  // S1
    } else {
      stc(sp + 256 + l * 64 + c, s_new);  // S2
    }
  }
  if (it < 3) {
    const int w = wave_id(), l = w >> 2, lane = lane_id();
    float* hb = p.H[l][(it - 1) & 1] + (size_t)gi.node_off * EMB;
    const int r = 4 * (w & 3) + (lane >> 4), q4 = lane & 15;
    const int v = rows[r];
    const float* e = scr + S_E + l * 64 * LDT + 4 * q4 * LDT + r;
    if (v >= 0) stc4(hb, v * 256 + q4 * 16, make_float4(e[0], e[LDT], e[2 * LDT], e[3 * LDT]));
  }
  __syncthreads();
  QTS(5);
  // iteration 3: the graph head was published (tag 1) before this item was pushed
  if (it == 3)
    attention_q_tile(p, lds, scr, gi, g, rows, p.apart + (size_t)(gi.tile_off + j) * 4,
                     (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane(npv) + 1ull, nullptr);
  QTS(6);
#undef QTS
}

// ------------------------------------------------------------------ paired tiles (queue mode)
// A 2-tile work item (tiles j, j + 1 of one graph) runs header, gather, update, normalisation,
// sums / stores and the attention + Q head once for its 32 rows instead of twice for 16: one
// chain of memory and LDS round trips and workgroup barriers per item instead of two, each
// MFMA weight fragment read from LDS serves both row blocks, and the waves run two
// independent MFMA chains.  Every element is computed by the same operations in the same
// order as the single-tile pieces (the MFMA chains per 16-row block, the CSR-order neighbour
// sums, the torch-order norms, per-tile partial sums and arg-max partials), so results are
// identical (GPU test: MD_PAIR=0 against the default).

// Gather of both tiles from their alive-neighbour lists: the layer's two lists staged as one
// concatenated list (batches of STG_ROWS rows per layer, register double buffer as
// gather_tile2); thread (row r, quad) adds rows r and 16 + r in list (CSR) order.
__device__ __noinline__ void gather_pair(KParams&, const GraphInfo gi, int it) {
  float* const scr = lds_base() + L_SCR;
  const int* const rows = (const int*)(scr + P2_ROW);

  KParams& p = kp();
  const int w = wave_id(), l = w >> 2, lane = lane_id(), t = threadIdx.x & 255;
  const int grp = lane >> 4, qd = lane & 15;
  const int* deg = p.deg[l] + gi.node_off;
  const float* hp;
  bool table = false;
  if (it == 1) {
    table = p.node_w == nullptr;
    hp = table ? first_layer_rows(p, gi, l) : p.h0tab[l] + (size_t)gi.node_off * EMB;
  } else {
    hp = p.H[l][(it - 2) & 1] + (size_t)gi.node_off * EMB;
  }
  const lds_i32* h0 = (const lds_i32*)(const int*)(scr + S_NBH);
  const lds_i32* h1 = (const lds_i32*)(const int*)(scr + P2_NB1);
  const lds_u16* nb0 = (const lds_u16*)(const uint16_t*)(scr + S_NBL) + l * NB_CAP;
  const lds_u16* nb1 = (const lds_u16*)(const uint16_t*)(scr + P2_NB1 + (S_NBL - S_NBH)) + l * NB_CAP;
  const int r = 4 * (w & 3) + grp;
  float4 own[2], acc[2];
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    own[rb] = make_float4(0.f, 0.f, 0.f, 0.f);
    acc[rb] = make_float4(0.f, 0.f, 0.f, 0.f);
    const int v = rows[16 * rb + r];
    if (v >= 0) {
      const int ov = table ? ldc(deg + v) : v;
      if (MD_BOK(v < gi.n && ov >= 0 && ov < gi.n, 1)) own[rb] = ldc4(hp, ov * 256 + qd * 16);
    }
  }
  const int t0 = h0[128 + l], totl = t0 + h1[128 + l];
  const int nbat = (max(h0[128] + h1[128], h0[129] + h1[129]) + STG2_ROWS - 1) / STG2_ROWS;
  const int off0 = h0[l * 16 + r], cnt0 = h0[32 + l * 16 + r];
  const int off1 = t0 + h1[l * 16 + r], cnt1 = h1[32 + l * 16 + r];
  float4* stg = (float4*)(scr + P2_STG) + l * STG2_ROWS * 16;
  auto issue = [&](int b, float4 (&x)[STG2_LD], bool (&ok)[STG2_LD]) {
    const int base = b * STG2_ROWS;
    int src[STG2_LD];
#pragma unroll
    for (int i = 0; i < STG2_LD; ++i) {
      const int k = t + 256 * i, row = base + (k >> 4);
      src[i] = -1;
      if (b < nbat && k < STG2_ROWS * 16 && row < totl) {
        const int id = row < t0 ? nb0[row] : nb1[row - t0];
        src[i] = MD_BOK(id < gi.n, 4) ? (table ? ldc(deg + id) : id) : -1;
        if (!MD_BOK(src[i] < gi.n, 5)) src[i] = -1;
      }
    }
#pragma unroll
    for (int i = 0; i < STG2_LD; ++i) {
      ok[i] = src[i] >= 0;
      if (ok[i]) x[i] = ldc4(hp, src[i] * 256 + ((t + 256 * i) & 15) * 16);
    }
  };
  auto add_range = [&](float4& a, int lo, int hi, int base) {
    int k = lo;
    for (; k + 8 <= hi; k += 8) {
      float4 y[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) y[jj] = stg[(k + jj - base) * 16 + qd];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        a.x = a.x + y[jj].x;
        a.y = a.y + y[jj].y;
        a.z = a.z + y[jj].z;
        a.w = a.w + y[jj].w;
      }
    }
    for (; k < hi; ++k) {
      const float4 y = stg[(k - base) * 16 + qd];
      a.x = a.x + y.x;
      a.y = a.y + y.y;
      a.z = a.z + y.z;
      a.w = a.w + y.w;
    }
  };
#ifdef MD_QPROF
  // (qprof build, iterations 2-3: slot 64 = waiting for a batch's loads, slot 65 = staging
  // stores + adds + barriers; the next batch's six loads stay in flight)
  unsigned long long* gw = p.prof != nullptr && (p.variant & 8) && it > 1 ? p.prof + 64 : nullptr;
#endif
  auto consume = [&](int b, const float4 (&x)[STG2_LD], const bool (&ok)[STG2_LD]) {
    const int base = b * STG2_ROWS;
#ifdef MD_QPROF
    unsigned long long tw0 = 0, tw1 = 0;
    if (gw != nullptr) {
      tw0 = wall_clock64();
      if (b + 1 < nbat) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // every thread's loads of this batch are in
      tw1 = wall_clock64();
    }
#endif
#pragma unroll
    for (int i = 0; i < STG2_LD; ++i)
      if (ok[i]) stg[t + 256 * i] = x[i];
    __syncthreads();
    add_range(acc[0], max(off0, base), min(off0 + cnt0, base + STG2_ROWS), base);
    add_range(acc[1], max(off1, base), min(off1 + cnt1, base + STG2_ROWS), base);
    __syncthreads();
#ifdef MD_QPROF
    if (gw != nullptr && threadIdx.x == 0) {
      atomicAdd(gw + 0, tw1 - tw0);
      atomicAdd(gw + 1, wall_clock64() - tw1);
    }
#endif
  };
  float4 xa[STG2_LD], xb[STG2_LD];
  bool oka[STG2_LD], okb[STG2_LD];
#ifdef MD_QPROF
  // gather sub-pieces (qprof build, MD_VARIANT bit 8): slots 60 (own loads and first issue
  // complete), 61 (batch loop), 62 (batches), 63 (list entries)
  unsigned long long* gq = p.prof != nullptr && (p.variant & 8) ? p.prof + 60 : nullptr;
  unsigned long long tg0 = gq != nullptr ? wall_clock64() : 0ull;
#endif
  if (nbat > 0) issue(0, xa, oka);
#ifdef MD_QPROF
  if (gq != nullptr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned long long t1 = wall_clock64();
      atomicAdd(gq + 0, t1 - tg0);
      atomicAdd(gq + 2, (unsigned long long)nbat);
      atomicAdd(gq + 3, (unsigned long long)(h0[128] + h1[128] + h0[129] + h1[129]));
      tg0 = t1;
    }
  }
#endif
  for (int b = 0; b < nbat; b += 2) {
    issue(b + 1, xb, okb);
    consume(b, xa, oka);
    if (b + 1 >= nbat) break;
    issue(b + 2, xa, oka);
    consume(b + 1, xb, okb);
  }
#ifdef MD_QPROF
  if (gq != nullptr && threadIdx.x == 0) atomicAdd(gq + 1, wall_clock64() - tg0);
#endif
  const int c = 4 * qd;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    float* atp = scr + P2_P + p2m(l, rb, 64);
    float* atx = scr + P2_X + p2m(l, rb, 64);
    atp[p2o(c + 0, r)] = acc[rb].x;
    atp[p2o(c + 1, r)] = acc[rb].y;
    atp[p2o(c + 2, r)] = acc[rb].z;
    atp[p2o(c + 3, r)] = acc[rb].w;
    atx[p2o(c + 0, r)] = own[rb].x;
    atx[p2o(c + 1, r)] = own[rb].y;
    atx[p2o(c + 2, r)] = own[rb].z;
    atx[p2o(c + 3, r)] = own[rb].w;
  }
}

// Gather of both tiles straight from the CSR (a list over NB_CAP entries): gather_tile per row
// block.
__device__ __noinline__ void gather_pair_csr(KParams&, const GraphInfo gi, int it) {
  float* const scr = lds_base() + L_SCR;
  const int* const rows = (const int*)(scr + P2_ROW);

  KParams& p = kp();
  const int w = wave_id(), l = w >> 2, lane = lane_id();
  const int grp = lane >> 4, qd = lane & 15;
  const int* rp = p.rowptr[l] + gi.roff[l];
  const int* adj = p.adj[l] + gi.coff[l];
  const uint8_t* ca = p.calive[l] + gi.coff[l];
  const int* deg = p.deg[l] + gi.node_off;
  const float* hp;
  bool table = false;
  if (it == 1) {
    table = p.node_w == nullptr;
    hp = table ? first_layer_rows(p, gi, l) : p.h0tab[l] + (size_t)gi.node_off * EMB;
  } else {
    hp = p.H[l][(it - 2) & 1] + (size_t)gi.node_off * EMB;
  }
  const int r = 4 * (w & 3) + grp;
  for (int rb = 0; rb < 2; ++rb) {
    const int v = rows[16 * rb + r];
    int rbeg = 0, rend = 0;
    float4 own = {0.f, 0.f, 0.f, 0.f}, acc = {0.f, 0.f, 0.f, 0.f};
    if (v >= 0) {
      rbeg = rp[v];
      rend = rp[v + 1];
      const int ov = table ? ldc(deg + v) : v;
      if (MD_BOK(v < gi.n && ov >= 0 && ov < gi.n, 1)) own = ldc4(hp, ov * 256 + qd * 16);
    }
    int nch = (rend - rbeg + 15) >> 4;
    nch = max(nch, __shfl_xor(nch, 16, 64));
    nch = max(nch, __shfl_xor(nch, 32, 64));
    for (int ch = 0; ch < nch; ++ch) {
      const int e = rbeg + 16 * ch + qd;
      int nb = -1;
      if (e < rend && ldc(ca + e)) nb = adj[e];
      if (table && nb >= 0) nb = ldc(deg + nb);
      const unsigned long long m = __ballot(nb >= 0);
      unsigned gm = (unsigned)(m >> (16 * grp)) & 0xFFFFu;
      while (__any(gm != 0)) {
        int jx[4] = {-1, -1, -1, -1};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (gm) {
            const int b = __builtin_ctz(gm);
            gm &= gm - 1;
            jx[k] = b;
          }
        }
        int src[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) src[k] = __shfl(nb, 16 * grp + (jx[k] < 0 ? 0 : jx[k]), 64);
        float4 x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = jx[k] >= 0 ? ldc4(hp, src[k] * 256 + qd * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (jx[k] >= 0) {
            acc.x = acc.x + x[k].x;
            acc.y = acc.y + x[k].y;
            acc.z = acc.z + x[k].z;
            acc.w = acc.w + x[k].w;
          }
        }
      }
    }
    float* atp = scr + P2_P + p2m(l, rb, 64);
    float* atx = scr + P2_X + p2m(l, rb, 64);
    const int c = 4 * qd;
    atp[p2o(c + 0, r)] = acc.x;
    atp[p2o(c + 1, r)] = acc.y;
    atp[p2o(c + 2, r)] = acc.z;
    atp[p2o(c + 3, r)] = acc.w;
    atx[p2o(c + 0, r)] = own.x;
    atx[p2o(c + 1, r)] = own.y;
    atx[p2o(c + 2, r)] = own.z;
    atx[p2o(c + 3, r)] = own.w;
  }
}

// Node update of both row blocks: wave (layer, column block) runs the chains of update_tile for
// each block on one set of weight fragments (four independent chains, then two).
__device__ __noinline__ void update_pair() {
  const float* const wi = lds_base() + L_W;
  float* const scr = lds_base() + L_SCR;

  const int w = wave_id(), l = w >> 2, cb = w & 3, lane = lane_id();
  const int ar = lane & 15, ak = lane >> 4;
  const P2Rot rot(ak, ar);
  const float* p1 = wi + W_IP1 + cb * 16 * 64;
  const float* p2 = wi + W_IP2 + cb * 16 * 64;
  const float* p3 = wi + W_IP3 + cb * 32 * 64;
  const int col = 16 * cb + ar;
  f4 a1[2], a2[2];
  {
    float xa[2][16], xb[2][16], wa[16], wb[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        xa[rb][s] = scr[P2_P + p2m(l, rb, 64) + rot(s)];
        xb[rb][s] = scr[P2_X + p2m(l, rb, 64) + rot(s)];
      }
      wa[s] = p1[s * 64 + lane];
      wb[s] = p2[s * 64 + lane];
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      a1[rb] = f4{0.f, 0.f, 0.f, 0.f};
      a2[rb] = f4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) {
        a1[rb] = mfma16(xa[rb][s], wa[s], a1[rb]);
        a2[rb] = mfma16(xb[rb][s], wb[s], a2[rb]);
      }
    }
    // the LDS reads of k-steps s + 4.. issue under the MFMAs of step s (-0.9 ms per 256-graph
    // launch against all reads first)
    __builtin_amdgcn_sched_group_barrier(0x100, 24, 0);
#pragma unroll
    for (int s = 0; s < 12; ++s) {
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 16, 0);
  }
  __syncthreads();  // every P / X read done: M overwrites them
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    float* atm = scr + P2_M + p2m(l, rb, 128);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      atm[p2o(col, 4 * ak + r)] = a1[rb][r];
      atm[p2o(64 + col, 4 * ak + r)] = a2[rb][r];
    }
  }
  __syncthreads();
  f4 a3[2];
  {
    float xm[2][32], wc[32];
#pragma unroll
    for (int s = 0; s < 32; ++s) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) xm[rb][s] = scr[P2_M + p2m(l, rb, 128) + rot(s)];
      wc[s] = p3[s * 64 + lane];
    }
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) a3[rb] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 32; ++s) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) a3[rb] = mfma16(xm[rb][s], wc[s], a3[rb]);
    }
    __builtin_amdgcn_sched_group_barrier(0x100, 12, 0);
#pragma unroll
    for (int s = 0; s < 28; ++s) {
      __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
  }
  __syncthreads();  // every M read done: E overwrites it
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    float* ate = scr + P2_E + p2b(l, rb, 64);
#pragma unroll
    for (int r = 0; r < 4; ++r) ate[col * LDT + 4 * ak + r] = fmaxf(a3[rb][r], 0.f);
  }
}

// Row normalisation of both blocks of E in place (normalize_tile's order).
__device__ __noinline__ void normalize_pair() {
  float* const scr = lds_base() + L_SCR;
  float* red = scr + P2_RED;
  {
    const int t = threadIdx.x, l = t >> 8, row = (t >> 3) & 31, jj = t & 7;
    const float* a = scr + P2_E + p2b(l, row >> 4, 64);
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float v = a[(8 * i + jj) * LDT + (row & 15)];
      acc = fmaf(v, v, acc);
    }
    red[(l * 32 + row) * 8 + jj] = acc;
  }
  __syncthreads();
  const int w = wave_id(), l = w >> 2, cb = w & 3, lane = lane_id();
  const int col = 16 * cb + (lane & 15), rq = lane >> 4;
#pragma unroll
  for (int rb = 0; rb < 2; ++rb) {
    float* a = scr + P2_E + p2b(l, rb, 64);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * rq + r;
      const float den = fmaxf(sqrtf(sumsq8_finish(red + (l * 32 + 16 * rb + row) * 8)), 1e-12f);
      a[col * LDT + row] = a[col * LDT + row] / den;
    }
  }
}

// Iteration 3 of both tiles: attention_q_tile's pieces for 32 rows; the arg-max partials stay
// per tile (tiles j, j + 1).
__device__ __noinline__ void attention_q_pair(KParams&, const GraphInfo gi, int g, int j, unsigned long long htag) {
  float* const lds = lds_base();
  float* const scr = lds + L_SCR;
  const int* const rows = (const int*)(scr + P2_ROW);

  KParams& p = kp();
  const float* wi = lds + L_W;
#ifdef MD_QPROF
  unsigned long long* qa = p.prof != nullptr && (p.variant & 8) ? p.prof + 88 : nullptr;
  unsigned long long tqa = qa != nullptr ? wall_clock64() : 0ull;
#define QATS(k)                                                   \
  do {                                                            \
    if (qa != nullptr && threadIdx.x == 0) {                      \
      const unsigned long long now_ = wall_clock64();             \
      atomicAdd(qa + (k), now_ - tqa);                            \
      tqa = now_;                                                 \
    }                                                             \
  } while (0)
#else
#define QATS(k) do {} while (0)
#endif
  const int w = wave_id(), l = w >> 2, cb = w & 3, lane = lane_id();
  const int ar = lane & 15, ak = lane >> 4;
  const int col = 16 * cb + ar;
  {
    // F_l = tanh(E_l . T + b)
    const float* tf = wi + W_IT + cb * 16 * 64;
    float xa[2][16], wa[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) xa[rb][s] = scr[P2_E + p2b(l, rb, 64) + (4 * s + ak) * LDT + ar];
      wa[s] = tf[s * 64 + lane];
    }
    f4 a[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < 16; ++s) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) a[rb] = mfma16(xa[rb][s], wa[s], a[rb]);
    }
    __builtin_amdgcn_sched_barrier(0);
    const float b = wi[W_ITB + col];
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      float* atf = scr + P2_F + p2b(l, rb, 64);
#pragma unroll
      for (int r = 0; r < 4; ++r) atf[col * LDT + 4 * ak + r] = tanhf(a[rb][r] + b);
    }
  }
  __syncthreads();
  QATS(0);
  float* dot = scr + P2_DOT;
  float* gate = dot + 96;  // [2][32] weight of the other layer per (layer, row)
  if (w < 2) {
    // wave rb: the gate dot products and gates of row block rb
    const int rb = w;
    if (lane < 48) {
      const int row = lane & 15, kind = lane >> 4;  // 0: F0F0, 1: F1F1, 2: F0F1
      const float* fa = scr + P2_F + p2b(kind == 1 ? 1 : 0, rb, 64);
      const float* fb = scr + P2_F + p2b(kind == 0 ? 0 : 1, rb, 64);
      float a = 0.f;
#pragma unroll
      for (int h = 0; h < 64; h += 32) {
        float xa[32], xb[32], ww[32];
#pragma unroll
        for (int c = 0; c < 32; ++c) {
          xa[c] = fa[(h + c) * LDT + row];
          xb[c] = fb[(h + c) * LDT + row];
          ww[c] = wi[W_ILW + h + c];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int c = 0; c < 32; ++c) a = fmaf(xa[c] * xb[c], ww[c], a);
      }
      dot[(16 * rb + row) * 3 + kind] = a;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes are done
    __builtin_amdgcn_wave_barrier();
    if (lane < 32) {
      const int ll = lane >> 4, row = 16 * rb + (lane & 15);
      gate[ll * 32 + row] = other_gate(ll, dot[row * 3 + 0], dot[row * 3 + 1], dot[row * 3 + 2], wi[W_ILB]);
    }
  }
  __syncthreads();
  QATS(1);
  {
    // mix E_l = F_l + gate * F_other fused into the first pass of the row normalisation
    float* red = scr + P2_RED;
    const int t = threadIdx.x;
    const int ll = t >> 8, row = (t >> 3) & 31, jj = t & 7, rb = row >> 4, rr = row & 15;
    const float* f = scr + P2_F + p2b(ll, rb, 64);
    const float* o = scr + P2_F + p2b(1 - ll, rb, 64);
    float* e = scr + P2_E + p2b(ll, rb, 64);
    const float gt = gate[ll * 32 + row];
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = 8 * i + jj;
      const float v = f[c * LDT + rr] + gt * o[c * LDT + rr];
      e[c * LDT + rr] = v;
      acc = fmaf(v, v, acc);
    }
    red[(ll * 32 + row) * 8 + jj] = acc;
    __syncthreads();
#pragma unroll
    for (int b2 = 0; b2 < 2; ++b2) {
      float* at = scr + P2_E + p2b(l, b2, 64);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rw = 4 * ak + r;
        const float den = fmaxf(sqrtf(sumsq8_finish(red + (l * 32 + 16 * b2 + rw) * 8)), 1e-12f);
        at[col * LDT + rw] = at[col * LDT + rw] / den;
      }
    }
  }
  __syncthreads();
  QATS(2);
  head_receive(p, lds, g, htag);
  QATS(3);
  {
    // e[a] = sum_b (h[a] * y[b]) * cp[b] (attention_q_tile's chains, eight per thread)
    const int ll = threadIdx.x >> 8, t = threadIdx.x & 255;
    typedef float f2v __attribute__((ext_vector_type(2)));
    f2v h[4], acc[4];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int idx = t + 256 * k, row = idx >> 6, a = idx & 63;
      h[k >> 1][k & 1] = scr[P2_E + p2b(ll, row >> 4, 64) + a * LDT + (row & 15)];
      acc[k >> 1][k & 1] = 0.f;
    }
    const float4* y4 = (const float4*)(lds + L_YS + ll * 64);
    const float4* c4 = (const float4*)(wi + W_ICP);
#pragma unroll 4
    for (int b4 = 0; b4 < 16; ++b4) {
      const float4 yv = y4[b4], cv = c4[b4];
      const float ys[4] = {yv.x, yv.y, yv.z, yv.w}, cs[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f2v yy = {ys[q], ys[q]}, cc = {cs[q], cs[q]};
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) acc[k2] = __builtin_elementwise_fma(h[k2] * yy, cc, acc[k2]);
      }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int idx = t + 256 * k, row = idx >> 6, a = idx & 63;
      scr[P2_F + p2b(ll, row >> 4, 64) + a * LDT + (row & 15)] = acc[k >> 1][k & 1];
    }
  }
  __syncthreads();
  QATS(4);
  float* hid = scr + P2_HID;
  if (cb < 2) {
    const float* hf = wi + W_IH1 + cb * 16 * 64;
    float xa[2][16], wa[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) xa[rb][s] = scr[P2_F + p2b(l, rb, 64) + (4 * s + ak) * LDT + ar];
      wa[s] = hf[s * 64 + lane];
    }
    f4 a[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int s = 0; s < 16; ++s) {
#pragma unroll
      for (int rb = 0; rb < 2; ++rb) a[rb] = mfma16(xa[rb][s], wa[s], a[rb]);
    }
    __builtin_amdgcn_sched_barrier(0);
    // hid overwrites the (dead) E region only, not the F being read
#pragma unroll
    for (int rb = 0; rb < 2; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) hid[(l * 32 + 16 * rb + 4 * ak + r) * 33 + col] = fmaxf(a[rb][r], 0.f);
  }
  __syncthreads();
  float* ql = scr + P2_Q;
  if (threadIdx.x < 64) {
    const int ll = threadIdx.x >> 5, row = threadIdx.x & 31;
    const float* gs = lds + L_GS;
    float a = fma_chain<32>(0.f, 0, [&](int k) { return hid[(ll * 32 + row) * 33 + k]; },
                            [&](int k) { return wi[W_IW2 + k]; });
    for (int k = 0; k < 4; ++k) a = fmaf(gs[4 + ll * 4 + k], wi[W_IW2 + 32 + k], a);
    ql[ll * 32 + row] = a;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  QATS(5);
  if (threadIdx.x < 64) {
    // q = w0 * Q0 + w1 * Q1 per row, and each tile's arg-max partial by a 16-lane butterfly
    const float* gs = lds + L_GS;
    const int ln = threadIdx.x;
    float bm = NEG_INF, bs = NEG_INF;
    int bi = 0x7fffffff, bc = 0;
    if (ln < 32) {
      const int v = rows[ln];
      if (v >= 0) {
        const float qq = gs[0] * ql[ln] + gs[1] * ql[32 + ln];
        stc(p.q + gi.node_off + v, qq);
        if (p.qspec != nullptr)
          stc(p.qspec + (size_t)(((const int*)(lds + L_MISC))[60] & 1) * p.qspec_n + gi.node_off + v, qq);
        bm = qq;
        bi = v;
        bc = 1;
      }
    }
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      const float m2 = __shfl_xor(bm, o, 64), s2 = __shfl_xor(bs, o, 64);
      const int i2 = __shfl_xor(bi, o, 64), c2 = __shfl_xor(bc, o, 64);
      if (c2 != 0) argmax_combine(bm, bs, bi, bc, m2, s2, i2, c2);
    }
    // (stc4 takes a wave-uniform base: the tile goes in the byte offset)
    if (ln == 0 || ln == 16)
      stc4(p.apart + (size_t)(gi.tile_off + j) * 4, (ln >> 4) * 16, make_float4(bm, bs, __int_as_float(bi), __int_as_float(bc)));
  }
  __syncthreads();
  QATS(6);
#undef QATS
}

// Queue work item of tiles j and j + 1 of graph g (slot gl), iteration it: queue_tile for both
// at once.
__device__ __noinline__ void queue_pair(KParams&, float* lds, int g, int gl, int it, int j) {
  KParams& p = kp();
  float* scr = lds + L_SCR;
  int* rows = (int*)(scr + P2_ROW);
  const GraphInfo gi = p.ginfo[g];
  const int npv = it == 3 ? ldc(&p.gvar[g].npred) : 0;  // (the head granules' tag - 1, iteration 3)
  lds_i32* flag = (lds_i32*)(int*)(scr + P2_FLAG);
#ifdef MD_QPROF
  unsigned long long* qd = p.prof != nullptr && (p.variant & 8) ? p.prof + 20 + 8 * (it - 1) : nullptr;
  unsigned long long tqd = qd != nullptr ? wall_clock64() : 0ull;
#else
  constexpr unsigned long long* qd = nullptr;
  unsigned long long tqd = 0ull;
#endif
#define QTS(k)                                                    \
  do {                                                            \
    if (qd != nullptr && threadIdx.x == 0) {                      \
      const unsigned long long now_ = wall_clock64();             \
      atomicAdd(qd + (k), now_ - tqd);                            \
      tqd = now_;                                                 \
    }                                                             \
  } while (0)
  const int t = threadIdx.x;
  const int slot0 = p.gtoff[gl] + j;  // neighbour-list cache slots: the graph's tiles within the launch
  const int nbo[2] = {0, P2_NB1 - S_NBH};
  bool cacheable[2], want[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    cacheable[b] = slot0 + b < p.nbc_slots;
    want[b] = cacheable[b];
  }
  // both tiles' cached lists (first 256 words per layer), headers and the "built" flag in one
  // round trip, with the rows from the live list
  int cw[2] = {0, 0}, ch = 0, built = 0;
#pragma unroll
  for (int b = 0; b < 2; ++b)
    if (want[b]) cw[b] = ldc(p.nbc + (size_t)(slot0 + b) * NBC_INTS + NBC_HDR + (t >> 8) * NBC_LWORDS + (t & 255));
  const int hb = t >> 7, hi = t & 127;
  if (hb < 2 && hi < 67 && want[hb]) ch = ldc(p.nbc + (size_t)(slot0 + hb) * NBC_INTS + hi);
  if (it == 1 && t == 67 && (want[0] || want[1])) built = ldc(p.qg + 2 * QG_CAP + gl);
  if (t < 2 * TILE) {
    const int r = j * TILE + t;
    lds_i32* hdr = (lds_i32*)(int*)(scr + S_NBH + nbo[t >> 4]);
    const int rr = t & 15;
    const int nl = ldc(&p.gvar[g].n_live);
    const float4 e = ldc4((const float*)(p.live + 4 * (size_t)gi.node_off), min(r, gi.n - 1) * 16);
    const bool ok = r < nl && MD_BOK(__float_as_int(e.x) >= 0 && __float_as_int(e.x) < gi.n && nl <= gi.n, 6);
    const unsigned c = (unsigned)__float_as_int(e.w);
    rows[t] = ok ? __float_as_int(e.x) : -1;
    hdr[64 + rr] = ok ? __float_as_int(e.y) : 0;
    hdr[96 + rr] = ok ? (int)(c & 0xffffu) : 0;
    hdr[64 + 16 + rr] = ok ? __float_as_int(e.z) : 0;
    hdr[96 + 16 + rr] = ok ? (int)(c >> 16) : 0;
  }
  if (t == 67) flag[0] = it > 1 || built;
  __syncthreads();
  bool cached[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) cached[b] = want[b] && flag[0] != 0;
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    if (cached[b]) {
      lds_i32* hdr = (lds_i32*)(int*)(scr + S_NBH + nbo[b]);
      ((lds_i32*)(int*)(scr + S_NBL + nbo[b]))[(t >> 8) * NBC_LWORDS + (t & 255)] = cw[b];
      if (hb == b) {
        if (hi < 64) hdr[hi] = ch;
        else if (hi < 66) hdr[128 + hi - 64] = ch;
        else if (hi == 66) flag[1 + b] = ch;
      }
    }
  }
  __syncthreads();
  QTS(0);
  bool nb_ok[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    if (cached[b]) {
      nb_ok[b] = flag[1 + b] != 0;
      const lds_i32* hdr = (const lds_i32*)(const int*)(scr + S_NBH + nbo[b]);
      const int nw0 = (hdr[128] + 1) >> 1, nw1 = (hdr[129] + 1) >> 1;
      if (nb_ok[b] && (nw0 > 256 || nw1 > 256)) {
        const int* src = p.nbc + (size_t)(slot0 + b) * NBC_INTS + NBC_HDR;
        lds_i32* words = (lds_i32*)(int*)(scr + S_NBL + nbo[b]);
        for (int i = 256 + t; i < nw0; i += NTHREADS) words[i] = ldc(src + i);
        for (int i = 256 + t; i < nw1; i += NTHREADS) words[NBC_LWORDS + i] = ldc(src + NBC_LWORDS + i);
        __syncthreads();
      }
    } else {
      nb_ok[b] = build_nb_lists(p, gi, nullptr, nullptr, nullptr, -1, false, nbo[b], P2_FLAG + 8);
      if (cacheable[b]) nbc_store(p, slot0 + b, scr, nb_ok[b], nbo[b]);
    }
  }
  QTS(1);
  if (nb_ok[0] && nb_ok[1]) gather_pair(p, gi, it);
  else gather_pair_csr(p, gi, it);
  __syncthreads();
  if (it == 1 && t < 256) {
    // S0 (first-layer input) partial sums before the update overwrites X
    const int b = t >> 7, l = (t >> 6) & 1, c = t & 63;
    const float s_old = col_sum16_p2(scr + P2_X + p2m(l, b, 64), c, tile_rows_valid(rows + 16 * b));
    stc(p.spart + (size_t)(gi.tile_off + j + b) * 384 + l * 64 + c, s_old);
  }
  QTS(2);
  update_pair();
  __syncthreads();
  QTS(3);
  normalize_pair();
  __syncthreads();
  QTS(4);
  if (it < 3) {
    if (t < 256) {
      const int b = t >> 7, l = (t >> 6) & 1, c = t & 63;
      const float s_new = col_sum16(scr + P2_E + p2b(l, b, 64) + c * LDT, tile_rows_valid(rows + 16 * b));
      stc(p.spart + (size_t)(gi.tile_off + j + b) * 384 + (it == 1 ? 128 : 256) + l * 64 + c, s_new);  // S1 / S2
    }
    const int w = wave_id(), l = w >> 2, lane = lane_id();
    float* hbuf = p.H[l][(it - 1) & 1] + (size_t)gi.node_off * EMB;
    const int r = 4 * (w & 3) + (lane >> 4), q4 = lane & 15;
#pragma unroll
    for (int rb = 0; rb < 2; ++rb) {
      const int v = rows[16 * rb + r];
      const float* e = scr + P2_E + p2b(l, rb, 64) + 4 * q4 * LDT + r;
      if (v >= 0) stc4(hbuf, v * 256 + q4 * 16, make_float4(e[0], e[LDT], e[2 * LDT], e[3 * LDT]));
    }
    __syncthreads();
  }
  QTS(5);
  if (it == 3) attention_q_pair(p, gi, g, j, (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane(npv) + 1ull);
  QTS(6);
#undef QTS
}

// Virtual-node chain Y1..Y3 from the tile partial sums S0..S2 and the graph head of graph g,
// published as tagged granules (tag 1) for its iteration-3 tiles.
// Virtual-node chain of graph g in two items: part 1 (Y1, Y2 from the iteration-1 partial sums
// S0, S1; runs beside the iteration-2 tiles, stored to ybuf) and part 2 (Y3 from S2 and the
// graph head, published as tagged granules (tag 1) for the iteration-3 tiles).
__device__ __noinline__ void queue_vn(KParams&, float* lds, int g, int part) {
  KParams& p = kp();
  float* scr = lds + L_SCR;
  const GraphInfo gi = p.ginfo[g];
  gv_load(p, g, (GraphVar*)(lds + L_GV));
  float* yw = lds + L_YW;
  if (threadIdx.x < 128) yw[threadIdx.x] = part == 1 ? lds[L_Y0 + (threadIdx.x & 63)] : ldc(p.ybuf + (size_t)g * 128 + threadIdx.x);
  __syncthreads();
  const GraphVar& gv = *(const GraphVar*)(lds + L_GV);
  const int nt = (gv.n_live + TILE - 1) / TILE;
  float* sbuf = scr + S_HID;  // [2][64]
  for (int k = part == 1 ? 0 : 2; k < (part == 1 ? 2 : 3); ++k) {
    graph_sum(p, gi, nt, k, sbuf, scr + S_YP);
    vrow_update(lds + L_W, scr, sbuf, yw);  // Y(k+1) from S(k)
  }
  if (part == 1) {
    if (threadIdx.x < 128) stc(p.ybuf + (size_t)g * 128 + threadIdx.x, yw[threadIdx.x]);
    return;
  }
  graph_head(p, lds, scr, gi, gv, false, false);
  head_publish(p, lds, g, (unsigned long long)(unsigned)gv.npred + 1ull);  // (this forward pass's tag)
}

__device__ __noinline__ void queue_loop(KParams&, float* lds, const float* __restrict__ wimg) {
  KParams& p = kp();
  int* misc = (int*)(lds + L_MISC);
  int* bc = misc + 48;
  const int ng = p.nglist;
  if (blockIdx.x == 0) {
    // the running graphs start with an environment step (no prediction yet); their slots in
    // order (up to QG_CAP) in the scratch's S_M region, unused before the first item
    int* run = (int*)(lds + L_SCR + S_M);
    static_assert(2 * 128 * LDT >= QG_CAP, "running-slot list must fit S_M");
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
    // admission: the first q_admit(p) running graphs (graph slots are ordered longest rollout
    // first) start now; every graph that stops admits the next one, so the long rollouts do
    // not wait behind the whole batch's backlog at every stage
    const int first = min(tot, q_admit(p));
    if (threadIdx.x == 0) {
      __hip_atomic_store((g_u32*)(p.qctl + QC_REM), (unsigned)tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store((g_u32*)(p.qctl + QC_ADMIT), (unsigned)(first < tot ? run[first] : ng), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (tot > 0) {
      q_push(p, first, [&](int i) { return q_item(QK_ENV, 0, run[i], 0); }, bc);
    } else {
      q_push_exit(p, bc);
    }
  }
  bool wdirty = false;
  // diagnostics (md_profile): per item kind, total device ticks and count in prof[kind] /
  // prof[8 + kind]; ticks waiting for items in prof[16]; weight reloads in prof[17]
  unsigned long long* qp = p.prof;
  unsigned long long tq = wall_clock64();
  const unsigned long long tq0 = tq;
  if (threadIdx.x == 0) misc[60] = 1 << 30;  // no per-step phase stamps (MD_PROF_A) in queue mode
  __syncthreads();
  if (qp != nullptr && blockIdx.x == 0 && threadIdx.x == 0) qp[0] = 1;  // the record is present
  unsigned tk = q_take(p);
  unsigned long long pre = 0ull;  // thread 0: early read of the next ticket's slot
  // A single-item stage that a workgroup enables (virtual-node part 2 after the last
  // iteration-2 task, the environment step after the last iteration-3 tile) runs on that
  // workgroup right away instead of queueing behind the backlog: one queue wait less on the
  // graph's critical path per stage.
  unsigned cont = 0u;
  while (true) {
    unsigned item;
    if (cont != 0u) {
      item = cont;
      cont = 0u;
    } else {
      if (qp != nullptr && (p.variant & 8) && threadIdx.x == 0) {
        // diagnostics (MD_VARIANT bit 8): pops whose slot was already filled at the early read
        // (slot 18), and the queue's backlog beyond the held ticket summed over pops (slot 19)
        if ((pre >> 32) == (unsigned long long)(tk + 1u)) atomicAdd(qp + 18, 1ull);
        const unsigned tl = __hip_atomic_load(q_ctl(p) + QC_TAIL, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        atomicAdd(qp + 19, (unsigned long long)max(0, (int)(tl - tk)));
      }
      item = q_wait(p, tk, bc, pre);
      pre = 0ull;
      tk = q_take(p);
    }
    const unsigned kind = item & 7u;
    unsigned long long ti = 0;
    if (qp != nullptr && threadIdx.x == 0) {
      ti = wall_clock64();
      atomicAdd(qp + 16, ti - tq);
      // waiting time over the launch in 1.31 ms buckets (slots 20..63; with MD_VARIANT bit 8
      // those slots hold the tile-item pieces instead)
      if (!(p.variant & 8)) atomicAdd(qp + 20 + min(43, (int)((ti - tq0) >> 17)), ti - tq);
      atomicAdd(qp + 8 + (kind & 7u), 1ull);
    }
    if (kind == QK_EXIT || kind == 0u) break;
    const int it = (int)((item >> 3) & 3u), gl = q_item_gl(item), j = q_item_j(item);
    const int g = p.glist[gl];
    if (kind == QK_ENV && it == 2) {  // batch speculation: the next step's fixed point for the candidate
      bspec_step(p, gl, j);
      pre = q_peek(p, tk);
      wdirty = true;
      if (qp != nullptr && threadIdx.x == 0) atomicAdd(qp + kind, (tq = wall_clock64()) - ti);
      continue;
    }
    if (kind == QK_ENV) {
#ifdef MD_QPROF
      const unsigned long long tqa = wall_clock64();
#endif
      if (threadIdx.x == 0) misc[20] = -1;  // (env_step sets the candidate)
      const bool lds_env = phase_a(p, g, it != 0, lds, false);
#ifdef MD_QPROF
      if (qp != nullptr && (p.variant & 8) && threadIdx.x == 0) atomicAdd(qp + 85, wall_clock64() - tqa);
#endif
      pre = q_peek(p, tk);
      wdirty = true;
      const GraphVar& gv = *(const GraphVar*)(lds + L_GV);
      const int st = gv.status, nl = gv.n_live;
      __syncthreads();
      if (st == ST_RUN && nl <= 0) {
        // cannot happen (alive edges in both layers imply live nodes); never strand the queue
        if (threadIdx.x == 0) raise_err(p, ERR_LIVE_MISMATCH);
        break;
      }
      // The launch's tail (every graph admitted, at most p.qpark still running): the graph
      // leaves the queue after this environment step and the host continues it in the
      // lock-step kernel (dedicated environment workgroups, speculative steps for a single
      // graph), whose per-step latency with few graphs is 1.5-2.5x lower; a launch begins
      // with phase A without an action, so the rollout continues exactly from this state.
      bool park = false;
      // (a launch of at most p.qpark graphs never parks: each launch makes progress)
      if (st == ST_RUN && p.qpark > 0 && ng > p.qpark) {
        if (threadIdx.x == 0)
          bc[6] = ldc((const int*)(p.qctl + QC_ADMIT)) >= ng && ldc((const int*)(p.qctl + QC_REM)) <= p.qpark;
        __syncthreads();
        park = bc[6] != 0;
      }
      if (st == ST_RUN && !park) {
        if (threadIdx.x == 0) {  // one decision for the workgroup
          int t = q_tiles_per_item(p);
          if (t > 1 && ldc((const int*)(p.qctl + QC_ADMIT)) >= ng && ldc((const int*)(p.qctl + QC_REM)) <= q_tail(p)) t = 1;
          bc[5] = t;
        }
        __syncthreads();
        const int tpi = bc[5];
        const int nt = (nl + TILE - 1) / TILE, ni = (nt + tpi - 1) / tpi;
        // this step's neighbour lists for the iteration-1 tiles
#ifdef MD_QPROF
        const unsigned long long tqb = wall_clock64();
#endif
        // batch speculation: the slot words of the new state's parity (loaded before the lists)
        const GraphVar& gvv = *(const GraphVar*)(lds + L_GV);
        const bool bsp = p.bspec != nullptr && lds_env;
        unsigned long long bst = 0ull;
        unsigned bex = 1u;
        if (bsp && threadIdx.x == 0) {
          const int* sl = bspec_slot(p, p.ginfo[g], gvv.steps);
          bst = __hip_atomic_load((const g_u64*)(sl + SRES_STARTED), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          bex = (unsigned)ldc(sl + BSPEC_EXITED);
        }
        // (in the tail -- one tile per item -- the iteration-1 tiles build their own lists: the
        // environment item is on the graph's critical path and most workgroups are idle)
        const bool built = lds_env && tpi > 1 && env_build_lists(p, p.ginfo[g], gl);
#ifdef MD_QPROF
        if (qp != nullptr && (p.variant & 8) && threadIdx.x == 0) atomicAdd(qp + 86, wall_clock64() - tqb);
#endif
        if (threadIdx.x == 0) {
          stc(p.qg + 2 * gl + 1, ni | (nt << 16) | (tpi << 28));
          stc(p.qg + 2 * QG_CAP + gl, built ? 1 : 0);
          misc[21] = bsp && bspec_claim(p, p.ginfo[g], gvv.steps, misc[20], bst, bex) ? 1 : 0;
        }
        __syncthreads();
        const int ns = misc[21], steps = gvv.steps;
        q_push(p, ni + ns, [&](int i) { return i < ni ? q_item_tile(1, gl, i, nt, tpi) : bspec_item(gl, steps); }, bc);
      } else if (st == ST_WAIT_HOST) {
        q_push(p, 1, [&](int) { return q_item(QK_ENV, 1, gl, 0); }, bc);  // poll again later
      } else {
        if (threadIdx.x == 0) {
          bc[2] = (int)__hip_atomic_fetch_add((g_u32*)(p.qctl + QC_REM), 0xffffffffu, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
          // admit the next graph that has not started (slots in order, skipping stopped ones)
          int a;
          while ((a = (int)__hip_atomic_fetch_add((g_u32*)(p.qctl + QC_ADMIT), 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT)) < ng &&
                 ldc(&p.gvar[p.glist[a]].status) != ST_RUN) {
          }
          bc[4] = a < ng ? a : -1;
        }
        __syncthreads();
        if (bc[4] >= 0) q_push(p, 1, [&](int) { return q_item(QK_ENV, 0, bc[4], 0); }, bc);
        if (bc[2] == 1) q_push_exit(p, bc);
      }
      if (qp != nullptr && threadIdx.x == 0) atomicAdd(qp + kind, (tq = wall_clock64()) - ti);
      continue;
    }
    if (wdirty) {
      load_weights(lds + L_W, wimg);
      __syncthreads();
      wdirty = false;
      if (qp != nullptr && threadIdx.x == 0) atomicAdd(qp + 17, wall_clock64() - ti);
    }
    int next = 0;
    if (kind == QK_TILE || (kind == QK_VN && it == 1)) {
      // a task of a stage: iteration-1/2/3 tiles; stage 2 also counts virtual-node part 1
      if (kind == QK_TILE) {
        const int ex = q_item_extra(item);
        if (ex == 1 && p.qpair) queue_pair(p, lds, g, gl, it, j);
        else
          for (int k = 0; k <= ex; ++k) queue_tile(p, lds, g, gl, it, j + k);
      } else {
        queue_vn(p, lds, g, 1);
      }
      const int stage = kind == QK_TILE ? it : 2;
      pre = q_peek(p, tk);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        const int tasks = (ldc(p.qg + 2 * gl + 1) & 0xffff) + (stage == 2 ? 1 : 0);
        const int old = __hip_atomic_fetch_add(p.qg + 2 * gl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == tasks - 1) {
          stc(p.qg + 2 * gl, 0);
          bc[3] = stage;
        } else {
          bc[3] = 0;
        }
      }
      __syncthreads();
      next = bc[3];
    } else {  // QK_VN part 2 (the iteration-3 tiles went out with it; MD_VARIANT bit 12: after it)
      queue_vn(p, lds, g, 2);
      pre = q_peek(p, tk);
      next = (p.variant & 4096) ? 4 : 0;
    }
    if (next != 0) {
      const int sz = ldc(p.qg + 2 * gl + 1), ni = sz & 0xffff, nt = (sz >> 16) & 0xfff, tpi = (sz >> 28) & 3;
      if (next == 1) {
        q_push(p, ni + 1, [&](int i) { return i < ni ? q_item_tile(2, gl, i, nt, tpi) : q_item(QK_VN, 1, gl, 0); }, bc);
      } else if (next == 2) {
        // the iteration-3 tiles now: their layer pieces need the iteration-2 rows only, their
        // attention waits for this forward pass's head granules (part 2, run here next)
        if (!(p.variant & 4096)) q_push(p, ni, [&](int i) { return q_item_tile(3, gl, i, nt, tpi); }, bc);
        cont = q_item(QK_VN, 2, gl, 0);
      } else if (next == 3) {
        cont = q_item(QK_ENV, 1, gl, 0);
      } else q_push(p, ni, [&](int i) { return q_item_tile(3, gl, i, nt, tpi); }, bc);
    }
    if (qp != nullptr && threadIdx.x == 0) atomicAdd(qp + (kind == QK_TILE ? 4 + it : kind == QK_VN ? 2 + it : kind), (tq = wall_clock64()) - ti);
  }
}

// ------------------------------------------------------------------ speculative steps
// Single-graph rollouts leave most CUs idle.  Workgroups [n_main, n_main + n_spec) of such a
// launch run the NEXT step's environment for likely next removals while the tiles compute Q:
// after phase A of step t publishes its state (spec_req), speculative workgroup k takes the
// live node of rank k in the previous prediction Q(t-1) (the next pick is among the top 8 in
// ~90 % of GMM steps), stages the state of step t from HBM into its own LDS, covers that
// node and runs the same mutual-LMCC fixed point (mcc_fixed_point, bit-identical: the result
// is unique and the code is the same), and publishes the killed edges, pruned / covered
// counts and LMCC, tagged {node, launch, removals so far}.  Phase A of step t + 1 uses a result
// only when its tag equals {the chosen node, this launch, the current removal count}: read
// before that phase A writes anything back, such a result was computed from step t's state.
// The workgroups take no part in the grid barrier and never write graph state; they stop at
// SPEC_EXIT (end of the launch), on an error anywhere, or after the host time-out.
// LDS words the candidate ranking needs beyond the environment: Q of the live nodes, group
// maxima, the candidate list.
constexpr int SPEC_CL = 256;
__host__ __device__ inline int spec_rank_words(int n) { return ((n + 15) & ~15) + ((n + 15) >> 4) + SPEC_CL + 16; }

__device__ __noinline__ void spec_loop(KParams&) {
  KParams& p = kp();
  float* const lds = lds_base();
  int* misc = (int*)(lds + L_MISC);
  const int k = (int)blockIdx.x - p.n_main;
  const GraphInfo gi = p.ginfo[p.glist[0]];
  const int n = gi.n, et = gi.e[0] + gi.e[1];
  int* ia = (int*)(lds + L_W);
  const EnvView<false> E = env_view<false>(p, gi, ia);
  // ranking scratch after the environment: qv[n] (Q of live nodes, -inf otherwise), gmx[G]
  // (maxima of 16-node groups), cl[SPEC_CL] (candidate list)
  float* qv = (float*)(ia + env_layout(n, et).total);
  const int G = (n + 15) >> 4;
  float* gmx = qv + ((n + 15) & ~15);
  int* cl = (int*)(gmx + G);
  env_stage_static(E, n);  // endpoints and row pointers: once per launch
  unsigned long long last = 0ull, last_ew = 0ull;
  // Early requests: phase A publishes the result it takes (pre_ew: {request tag << 32 | node <<
  // 16 | slot}) right after its slot check, about 12 us before its write-back and its request.
  // A workgroup whose LDS still holds the state of that request (own candidate's kills undoable:
  // `mine` >= -1) builds the next state itself -- undo its own kills, apply the taken result's
  // kill list -- and serves the next request (same step and tag as phase A's, which it then
  // ignores) without waiting for the write-back or restaging.  The state is the same bytes
  // phase A reaches: its step applies exactly that result's kill list (env_apply_spec).
  int mine = -2;  // -2: no state to build on; -1: state of request `last`, unmodified; else own candidate
  while (true) {
    if (threadIdx.x < 64) {
      // one round trip per poll: lane 0 the request word, lane 1 the early word, lane 2 the
      // error word
      const int lane = threadIdx.x;
      const bool we = p.pre_ew != nullptr && mine >= -1 && p.spec_early;
      const bool ws = we && p.self_ew != nullptr;
      const unsigned long long t0 = wall_clock64();
      unsigned long long v, ew = 0ull;
      int stop = 0, early = 0;
      while (true) {
        unsigned long long g = 0ull;
        if (lane == 0) g = __hip_atomic_load((const g_u64*)p.spec_req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (lane == 1 && we) g = __hip_atomic_load((const g_u64*)p.pre_ew, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (lane == 2) g = __hip_atomic_load((g_u32*)p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else if (lane == 3 && ws) g = __hip_atomic_load((const g_u64*)p.self_ew, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned lo = (unsigned)g, hi = (unsigned)(g >> 32);
        v = ((unsigned long long)(unsigned)__shfl((int)hi, 0, 64) << 32) | (unsigned)__shfl((int)lo, 0, 64);
        ew = ((unsigned long long)(unsigned)__shfl((int)hi, 1, 64) << 32) | (unsigned)__shfl((int)lo, 1, 64);
        const unsigned bw = (unsigned)__shfl((int)lo, 2, 64);
        if (ws && !(ew != last_ew && (unsigned)(ew >> 32) == (unsigned)last)) {
          // tile 0's self-pick: the word phase A's early word will be (its result finished)
          ew = ((unsigned long long)(unsigned)__shfl((int)hi, 3, 64) << 32) | (unsigned)__shfl((int)lo, 3, 64);
        }
        if (v == SPEC_EXIT) { stop = 1; break; }
        if (we && ew != last_ew && (unsigned)(ew >> 32) == (unsigned)last) {
          v = ((unsigned long long)((unsigned)(last >> 32) + 1u) << 32) |
              spec_tag(p.launch_seq, (int)((unsigned)last & 0xffffu) + 1);
          early = 1;
          break;
        }
        if (v != 0ull && v != last && ((unsigned)v >> 16) == (p.launch_seq & 0xffffu)) break;
        if (bw & BAR_ERR) { stop = 1; break; }
        if (wall_clock64() - t0 > HOST_TIMEOUT_TICKS) { stop = 1; break; }
        __builtin_amdgcn_s_sleep(2);
      }
      if (lane == 0) {
      misc[0] = stop;
      misc[1] = (int)(unsigned)v;
      misc[2] = (int)(unsigned)(v >> 32);
      misc[3] = -1;
      misc[4] = __float_as_int(NEG_INF);
      misc[5] = 0;
      misc[6] = early;
      misc[7] = (int)(ew & 0xffffu);          // the taken result's slot (parity included)
      misc[8] = (int)((ew >> 16) & 0xffffu);  // and node
      misc[9] = (int)(unsigned)ew;
      misc[10] = (int)(unsigned)(ew >> 32);
      }
    }
    __syncthreads();
    if (misc[0]) return;
    const unsigned tag = (unsigned)misc[1];
    const int qb = (misc[2] - 1) & 1;  // buffer of the previous prediction
    int* const slot = p.sres + (size_t)spec_slot_index(k, misc[2]) * p.sres_stride;  // this request's parity
    last = ((unsigned long long)(unsigned)misc[2] << 32) | tag;
    const bool early = misc[6] != 0;
    if (early) last_ew = ((unsigned long long)(unsigned)misc[10] << 32) | (unsigned)misc[9];
    // diagnostics (md_profile): workgroup 0's timeline in the request step's slots 65-68
    unsigned long long* ts = p.prof != nullptr && k == 0 && misc[2] < p.prof_cap ? p.prof + (size_t)misc[2] * PROF_SLOTS : nullptr;
    TSTAMP(65);
    if (ts != nullptr && threadIdx.x == 0) ts[33] = early ? 1 : 0;  // diagnostics: early request
    if (early) {
      // the next state from this LDS state: undo the own candidate's kills (its fixed point
      // killed only alive edges, listed in the dead list), apply the taken result's kill list
      const int a = misc[8];
      const int* const ts_ = p.sres + (size_t)misc[7] * p.sres_stride;
      // one round trip for Q(t-1) (first 4 x 512 nodes), the kill count and the first 512
      // kill entries (read before the count is known: entries past it are ignored)
      constexpr int QU = 4;
      float qq[QU];
#pragma unroll
      for (int u = 0; u < QU; ++u) {
        const int i = u * NTHREADS + threadIdx.x;
        if (i < n) qq[u] = ldc(p.qspec + (size_t)qb * p.qspec_n + gi.node_off + i);
      }
      if (mine != a) {
        const int nd_s = ldc(ts_ + 7);
        const int w0 = (int)threadIdx.x < et ? ldc(ts_ + SRES_HDR + 3 * threadIdx.x) : 0;
        if (mine >= 0) {
          const int nd = E.hdr[1];
          for (int i = threadIdx.x; i < nd; i += NTHREADS) E.st[E.dl[i]] = E_ALIVE;
          if (threadIdx.x == 0) E.cov8[mine] = 0;
          __syncthreads();
        }
        for (int i = threadIdx.x; i < nd_s; i += NTHREADS) {
          const int w = i < NTHREADS ? w0 : ldc(ts_ + SRES_HDR + 3 * i);
          const int e = w & 0xffff;
          if (MD_BOK(e < et, 11)) E.st[e] = (uint8_t)(w >> 16);
        }
        if (threadIdx.x == 0) E.cov8[a] = 1;
      }
      __syncthreads();
      build_alive<false>(E);
      // live nodes (residual layer-0 degree > 0, as phase A's degrees say) and Q(t-1)
      for (int x = threadIdx.x; x < n; x += NTHREADS) uf_store(E.deg0, x, 0);
      __syncthreads();
      for_each_alive<false>(E, [&](int e, int u, int v) {
        if (e < E.e0) {
          uf_store(E.deg0, u, 1);
          uf_store(E.deg0, v, 1);
        }
      });
      __syncthreads();
#pragma unroll
      for (int u = 0; u < QU; ++u) {
        const int i = u * NTHREADS + threadIdx.x;
        if (i < n) qv[i] = uf_load(E.deg0, i) > 0 ? qq[u] : NEG_INF;
      }
      for (int i = QU * NTHREADS + threadIdx.x; i < n; i += NTHREADS)
        qv[i] = uf_load(E.deg0, i) > 0 ? ldc(p.qspec + (size_t)qb * p.qspec_n + gi.node_off + i) : NEG_INF;
    } else {
    // step t's state and the previous prediction Q(t-1), loads batched; nodes live now were
    // live then, so their entries are that prediction's
    {
      // edge states and covered flags as whole words (4 per load; the single graph's arrays
      // start word-aligned and have 4 bytes of slack at the end)
      const int e0 = E.e0, e1 = et - e0, w0 = (e0 + 3) >> 2, w1 = (e1 + 3) >> 2, wn = (n + 3) >> 2;
      const int span = max(max(w0 + w1, wn), n);
      for (int b = 0; b < span; b += 4 * NTHREADS) {
        unsigned sw[4], cw[4];
        int dd[4];
        float qq[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = b + u * NTHREADS + threadIdx.x;
          if (i < w0 + w1) sw[u] = ldc((const int*)(i < w0 ? E.gst[0] + 4 * i : E.gst[1] + 4 * (i - w0)));
          if (i < wn) cw[u] = ldc((const int*)(E.gcov + 4 * i));
          if (i < n) {
            dd[u] = ldc(p.deg[0] + gi.node_off + i);
            qq[u] = ldc(p.qspec + (size_t)qb * p.qspec_n + gi.node_off + i);
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = b + u * NTHREADS + threadIdx.x;
          if (i < w0 + w1) {
            const int base = i < w0 ? 4 * i : e0 + 4 * (i - w0), lim = i < w0 ? e0 : et;
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (base + k < lim) E.st[base + k] = (uint8_t)(sw[u] >> (8 * k));
          }
          if (i < wn) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
              if (4 * i + k < n) E.cov8[4 * i + k] = (uint8_t)(cw[u] >> (8 * k));
          }
          if (i < n) qv[i] = dd[u] > 0 ? qq[u] : NEG_INF;
        }
      }
    }
    __syncthreads();
    build_alive<false>(E);
    }
    mine = -1;
    __syncthreads();
    TSTAMP(73);
    // candidate: the live node of rank k (descending Q, ties by ascending id).  Rank 0 (the
    // workgroup whose result phase A takes most often) is the arg-max, one block reduction;
    // ranks >= 1: the top n_spec all have Q >= T, the n_spec-th largest maximum of the 16-node
    // groups (those maxima are n_spec nodes at >= T), so only the nodes at >= T are ranked.
    if (k == 0) {
      float bv = NEG_INF;
      int bx = 0x7fffffff;
      for (int x = threadIdx.x; x < n; x += NTHREADS) {
        const float v = qv[x];
        if (v > bv) {  // ascending x per thread: the first maximum is the smallest id
          bv = v;
          bx = x;
        }
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        const float v2 = __shfl_xor(bv, o, 64);
        const int x2 = __shfl_xor(bx, o, 64);
        if (v2 > bv || (v2 == bv && x2 < bx)) {
          bv = v2;
          bx = x2;
        }
      }
      float* wv = gmx;  // the group maxima are not needed for rank 0
      int* wx = (int*)(gmx + NTHREADS / 64);
      if (lane_id() == 0) {
        wv[wave_id()] = bv;
        wx[wave_id()] = bx;
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        float v = wv[0];
        int x = wx[0];
        for (int i = 1; i < NTHREADS / 64; ++i)
          if (wv[i] > v || (wv[i] == v && wx[i] < x)) {
            v = wv[i];
            x = wx[i];
          }
        misc[3] = v != NEG_INF ? x : -1;
      }
      __syncthreads();
    } else {
    for (int r0 = 0; r0 < n; r0 += NTHREADS) {
      const int x = r0 + (int)threadIdx.x;
      float v = x < n ? qv[x] : NEG_INF;
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 16));
      if ((threadIdx.x & 15) == 0 && x < n) gmx[x >> 4] = v;
    }
    __syncthreads();
    const int K = p.n_spec;
    for (int gq = threadIdx.x; gq < G; gq += NTHREADS) {
      const float v = gmx[gq];
      int r = 0;
      for (int h = 0; h < G; ++h) {
        const float w = gmx[h];
        r += (w > v) || (w == v && h < gq);
      }
      if (r == K - 1) misc[4] = __float_as_int(v);
    }
    __syncthreads();
    const float T = __int_as_float(misc[4]);
    for (int x = threadIdx.x; x < n; x += NTHREADS) {
      const float v = qv[x];
      if (v != NEG_INF && v >= T) {
        const int at = atomicAdd(&misc[5], 1);
        if (at < SPEC_CL) cl[at] = x;
      }
    }
    __syncthreads();
    const int m = misc[5];
    if (m <= SPEC_CL && (int)threadIdx.x < m) {
      const int x = cl[threadIdx.x];
      const float v = qv[x];
      int r = 0;
      for (int i = 0; i < m; ++i) {
        const int y = cl[i];
        const float w = qv[y];
        r += (w > v) || (w == v && y < x);
      }
      if (r == k) misc[3] = x;
    }
    __syncthreads();
    }
    const int c = misc[3];
    __syncthreads();
    if (c < 0) continue;
    mine = c;
    TSTAMP(66);
    // taken: phase A of the next step waits for this result instead of recomputing it
    if (threadIdx.x == 0) {
      __hip_atomic_store((g_u64*)(slot + SRES_STARTED), ((unsigned long long)(unsigned)c << 32) | tag,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      E.cov8[c] = 1;  // c is live, hence not covered
    }
    __syncthreads();
    TSTAMP(67);
    int pr[2], cc[2];
    SpecAbort ab;
    ab.ew = p.pre_ew;
    ab.ew2 = p.self_ew;
    ab.req = p.spec_req;
    ab.tag = tag;
    ab.slot = spec_slot_index(k, misc[2]);
    ab.step = misc[2];
    const int lm = mcc_fixed_point<false>(E, pr, nullptr, c, cc, p.pre_ew != nullptr && p.spec_abort ? &ab : nullptr);
    if (lm < 0) {  // the result can no longer be used: the LDS state is partial, restage next
      mine = -2;
      if (ts != nullptr && threadIdx.x == 0) ts[36] = 1;  // diagnostics: aborted
      continue;
    }
    const int nd = E.hdr[1];
    for (int i = threadIdx.x; i < nd; i += NTHREADS) {
      const int e = E.dl[i];
      if (!(e < et)) continue;  // (cannot happen: dead-list entries are edge ids)
      const int l = e < E.e0 ? 0 : 1, kk = e < E.e0 ? e : e - E.e0;
      stc(slot + SRES_HDR + 3 * i, e | ((int)E.st[e] << 16));
      stc(slot + SRES_HDR + 3 * i + 1, E.epos[l][2 * kk]);
      stc(slot + SRES_HDR + 3 * i + 2, E.epos[l][2 * kk + 1]);
    }
    if (threadIdx.x == 0) {
      stc(slot + 2, lm);
      stc(slot + 3, pr[0]);
      stc(slot + 4, pr[1]);
      stc(slot + 5, cc[0]);
      stc(slot + 6, cc[1]);
      stc(slot + 7, nd);
      const unsigned long long tdone = wall_clock64();
      __hip_atomic_store((g_u64*)(slot + 10), tdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (ts != nullptr) ts[68] = tdone;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)  // {killed edges << 48 | node << 32 | request tag}, one 8-byte granule
      __hip_atomic_store((g_u64*)slot, ((unsigned long long)(unsigned)(c | (nd << 16)) << 32) | tag,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // then the features of the state after c (degrees, live list, aggregates), tagged apart:
    // phase A takes them when they are there, computes them itself otherwise
    const EnvAgg ag = env_features<false>(E, n, slot + sres_deg(et), slot + sres_deg(et) + n,
                                          (float*)(slot + sres_live(et, n)), nullptr);
    if (threadIdx.x == 0) {
      stc(slot + 12, ag.nlive);
      stc(slot + 13, ag.dm0);
      stc(slot + 14, ag.dm1);
      stc(slot + 15, ag.sd0);
      stc(slot + 16, ag.sd1);
      stc(slot + 17, ag.bad);
      stc(slot + 18, (int)(ag.th0 & 0xffffffffll));
      stc(slot + 19, (int)(ag.th0 >> 32));
      stc(slot + 20, (int)(ag.th1 & 0xffffffffll));
      stc(slot + 21, (int)(ag.th1 >> 32));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_store((g_u64*)(slot + SRES_FEAT), ((unsigned long long)(unsigned)c << 32) | tag, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    TSTAMP(74);
  }
}

// ------------------------------------------------------------------ the kernel
// One body, two entry points so profiles separate the work: md_rollout_kernel runs whole
// rollouts (RUN_ROLLOUT); md_env_kernel runs single environment steps and predictions
// (RUN_STEP: MvcEnv.s0 / queued actions, RUN_PREDICT).
// ------------------------------------------------------------------ dataflow mode: the loops
// (see "dataflow mode: granules" above).  Per step the environment workgroup runs phase A and
// publishes the step record; the graph-head workgroup and the tile workgroups wait for it (the
// tiles building the iteration-1 prebuild from phase A's early word meanwhile), then run the
// step with every hand-off polled as tagged granules.

// Waits for the step record tagged `tag`: 1 when it is there (its six words in misc[50..55];
// with `full`, also its "full" granule: phase A has finished, not just published the record
// early), 2 when `watch` is set and the early word changed first (new value in the LDS word at
// L_MISC + 42), 0 on an error anywhere.  Uniform.
// Self-pick (nt_self = the previous step's tile count, <= 64): the wave also polls the
// previous step's arg-max partials (phase A's inputs) and, once all are in, combines them exactly
// as phase A does; a unique maximum whose node is the candidate of a started or finished result
// of request req_step gives the early word phase A will publish, returned as 4 (L_MISC + 38) --
// the prebuild then starts before phase A's slot check, and stores at once: phase A takes the
// same node, so the same state and tile assignment, whether it then takes this result (the same
// early word, absorbed here without a return) or computes the state itself (a result that
// started after its slot pre-read: the confirmation does not match and the tile rebuilds the
// same rows untagged).  misc[30] = 1 once this step's self-pick is decided (or phase A's early
// word came first).
__device__ __forceinline__ int df_wait_rec(KParams&, unsigned tag, bool watch, bool full = false, int req_step = -1,
                                        int nt_self = 0) {
  KParams& p = kp();
  int* const misc = (int*)(lds_base() + L_MISC);
  unsigned long long* const seen = (unsigned long long*)(lds_base() + L_MISC + 42);
  unsigned long long* const tried0 = (unsigned long long*)(lds_base() + L_MISC + 38);
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const bool w = watch && p.pre_ew != nullptr;
    const bool wr = w && req_step >= 0 && p.sres != nullptr && p.spec_req != nullptr;
    bool ws = wr && nt_self > 0 && nt_self <= 64 && !p.host_select && misc[30] == 0;
    const unsigned ptag = (unsigned)(req_step + 1) << 1;  // the partials of step req_step (df_tag)
    const float* const apb = (const float*)df_ap(p);
    unsigned long long sv = *seen;
    const unsigned long long s0 = *tried0;
    const unsigned long long t0 = wall_clock64();
    int res = 0;
    while (true) {
      // lanes 0-6: the record's granules (6: "full"), lane 8: the error word, lane 7: the early word
      unsigned long long g = 0ull;
      if (lane < 7) g = __hip_atomic_load((const g_u64*)(p.df + DF_REC + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else if (lane == 8) g = __hip_atomic_load((g_u32*)p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else if (lane == 7 && w) g = __hip_atomic_load((const g_u64*)p.pre_ew, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else if (lane == 9 && ws) g = __hip_atomic_load((const g_u64*)p.spec_req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      float4 pa = make_float4(0.f, 0.f, 0.f, 0.f), pc = pa;
      if (ws && lane < nt_self) {
        pa = ldc4(apb, lane * 32);
        pc = ldc4(apb, lane * 32 + 16);
      }
      if (__ballot(lane == 8 && (g & BAR_ERR))) break;
      // a new early word first (phase A publishes it with, or just before, an early record: the
      // prebuild from it is the tile's fastest start)
      if (w) {
        const unsigned lo = __shfl((unsigned)g, 7, 64), hi = __shfl((unsigned)(g >> 32), 7, 64);
        const unsigned long long ew = ((unsigned long long)hi << 32) | lo;
        if (ew != sv) {
          if (lane == 0) {
            *seen = ew;
            misc[30] = 1;
          }
          sv = ew;
          // (phase A's early word equal to this step's self-pick: that prebuild is the one)
          if (!(ew == s0 && (unsigned)(ew >> 32) != 0u)) {
            res = 2;
            break;
          }
        }
      }
      if (!__ballot((lane < 6 || (lane == 6 && full)) && (unsigned)(g >> 32) != tag)) {
        if (lane < 6) misc[50 + lane] = (int)(unsigned)g;
        res = 1;
        break;
      }
      if (ws && !__ballot(lane < nt_self && !(df_ok4(pa, ptag, ptag) && df_ok4(pc, ptag, ptag)))) {
        // every partial of the step is in: phase A's combine (max / min / sum steps, so the
        // result does not depend on the order)
        float bm = NEG_INF, bs = NEG_INF;
        int bi = 0x7fffffff, bc = 0;
        const int c = lane < nt_self ? __float_as_int(pc.z) : 0;
        if (c != 0) argmax_combine(bm, bs, bi, bc, pa.x, pa.z, __float_as_int(pc.x), c);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
          const float m2 = __shfl_xor(bm, o, 64), s2 = __shfl_xor(bs, o, 64);
          const int i2 = __shfl_xor(bi, o, 64), c2 = __shfl_xor(bc, o, 64);
          if (c2 != 0) argmax_combine(bm, bs, bi, bc, m2, s2, i2, c2);
        }
        const unsigned rlo = __shfl((unsigned)g, 9, 64), rhi = __shfl((unsigned)(g >> 32), 9, 64);
        ws = false;
        if (lane == 0) misc[30] = 1;
        if (bc == 1 && (int)rhi == req_step && rlo != 0u) {
          // the result of the request whose candidate is the pick (started or finished): the
          // one phase A's slot check takes
          unsigned long long sd = 0ull, ss = 0ull;
          if (lane < p.n_spec) {
            const g_u64* tp = (const g_u64*)(p.sres + (size_t)spec_slot_index(lane, req_step) * p.sres_stride);
            sd = __hip_atomic_load(tp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            ss = __hip_atomic_load(tp + SRES_STARTED / 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          const bool fin = lane < p.n_spec && (unsigned)sd == rlo && (int)((sd >> 32) & 0xffffu) == bi;
          const bool hit = fin || (lane < p.n_spec && (unsigned)ss == rlo && (int)(ss >> 32) == bi);
          const unsigned long long m = __ballot(hit);
          if (m != 0ull) {
            const int k = __builtin_ctzll(m);
            const unsigned long long e0 = ((unsigned long long)rlo << 32) | ((unsigned long long)(unsigned)bi << 16) |
                                          (unsigned)spec_slot_index(k, req_step);
            // tile 0 (layer 0) hands a finished result's word to the speculative workgroups
            if (p.self_ew != nullptr && (int)blockIdx.x == 2 * p.n_env && lane == k && fin)
              __hip_atomic_store((g_u64*)p.self_ew, e0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (e0 != s0) {
              if (lane == 0) *tried0 = e0;
              res = 4;
              break;
            }
          }
        }
      }
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > (p.h_req != nullptr ? HOST_TIMEOUT_TICKS : BARRIER_TIMEOUT_TICKS)) {
        if (lane == 0) raise_err(p, ERR_TIMEOUT);
        break;
      }
    }
    if (lane == 0) misc[49] = res;
  }
  __syncthreads();
  const int r = misc[49];
  __syncthreads();
  return r;
}

// Environment workgroup: phase A, then the step record {status, n_live, confirmation, early
// word} once phase A's stores are done.
__device__ __noinline__ void df_env(KParams&) {
  KParams& p = kp();
  float* const lds = lds_base();
  int* const misc = (int*)(lds + L_MISC);
  const int g = p.glist[0];
  bool have_q = false, staged = false;
  unsigned long long last_ew = 0ull;  // the early word as the tiles see it after this phase A
  for (int pstep = 0;; ++pstep) {
    MD_PROF(0);
    if (threadIdx.x == 0) {
      misc[60] = pstep;
      misc[48] = 0;  // set by env_step when it published the step record early
    }
    __syncthreads();
    staged = phase_a(p, g, have_q, lds, staged);
    MD_PROF(3);
    const GraphVar& gv = *(const GraphVar*)(lds + L_GV);
    if (p.pre_ew != nullptr) {
      const unsigned long long ew = ((unsigned long long)(unsigned)misc[57] << 32) | (unsigned)misc[56];
      if (ew != 0ull) last_ew = ew;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every store of phase A is done
    __syncthreads();
    const int st = gv.status;
    const bool early = misc[48] != 0;
    if (early && threadIdx.x == 0 && (st != ST_RUN || (unsigned)misc[54] != (unsigned)last_ew))
      raise_err(p, ERR_DF_EARLY);  // (cannot happen: the early record promised this state)
    if (threadIdx.x < 7 && (threadIdx.x == 6 || !early)) {
      const int k = threadIdx.x;
      const int v = k == 0 ? st : k == 1 ? gv.n_live : k < 4 ? misc[52 + k] : k == 4 ? (int)(unsigned)last_ew : k == 5 ? (int)(unsigned)(last_ew >> 32) : 1;
      df_st(p.df + DF_REC + k, __int_as_float(v), (unsigned)(pstep + 1));
    }
    // the record lands before any later early word (a tile that sees the next step's early word
    // sees this record)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) misc[49] = (__hip_atomic_load((g_u32*)p.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & BAR_ERR) != 0;
    __syncthreads();
    const bool stop = st != ST_RUN || misc[49] != 0;
    __syncthreads();
    if (stop) break;
    have_q = true;
  }
  if (p.n_spec > 0 && threadIdx.x == 0)
    __hip_atomic_store((g_u64*)p.spec_req, SPEC_EXIT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Graph-head workgroup: the virtual-node chain and the graph head of each step from the tiles'
// tagged partial sums (S0 / S1 may come from a confirmed prebuild).
__device__ __noinline__ void df_head(KParams&) {
  KParams& p = kp();
  float* const lds = lds_base();
  float* const scr = lds + L_SCR;
  int* const misc = (int*)(lds + L_MISC);
  const int g = p.glist[0];
  for (int pstep = 0;; ++pstep) {
    if (threadIdx.x == 0) misc[60] = pstep;
    __syncthreads();
    if (df_wait_rec(p, (unsigned)(pstep + 1), false, true) != 1 || misc[50] != ST_RUN) break;
    const unsigned long long cw = ((unsigned long long)(unsigned)misc[53] << 32) | (unsigned)misc[52];
    const unsigned tn = df_tag(pstep), tp = cw != 0ull ? df_ptag(tn, cw) : tn;
    head_iteration(p, lds, scr, g, 2, (unsigned long long)(pstep + 1), tn, tp);
    head_iteration(p, lds, scr, g, 3, (unsigned long long)(pstep + 1), tn, tn);
  }
}

// Diagnostics (md_profile): stamps of tile 0's layer-0 workgroup in the step's slots: 4 record
// seen, 5 iteration 1 done, 23 / 6 iteration-2 gather / all done, 29 / 30 iteration-3 gather /
// update done, 8 layer-1 rows received, 9 = 10 attention and arg-max partial done.
#define DF_STAMP(slot)                                                                              \
  do {                                                                                              \
    if (p.prof != nullptr && tb == 0 && threadIdx.x == 0 && pstep < p.prof_cap)                     \
      p.prof[(size_t)pstep * PROF_SLOTS + (slot)] = wall_clock64();                                 \
  } while (0)
// ... and the latest over every active tile workgroup: 43 record seen, 44 iteration 1 done, 45
// iteration 2 done, 46 arg-max partial (layer 0) / layer-1 rows (layer 1) out
// ... and per tile workgroup (rows 128 + 4 pstep + k of the profile, slot tb % 64, k = tb / 64
// for the iteration-2 start, 2 + tb / 64 for the end of the prebuild)
#define DF_STAMP_TILE(k)                                                                            \
  do {                                                                                              \
    if (p.prof != nullptr && threadIdx.x == 0 && 128 + 4 * pstep + 4 < p.prof_cap)                  \
      p.prof[(size_t)(128 + 4 * pstep + (k) + (tb >> 6)) * PROF_SLOTS + (tb & 63)] = wall_clock64();  \
  } while (0)
#define DF_STAMP_MAX(slot)                                                                          \
  do {                                                                                              \
    if (p.prof != nullptr && threadIdx.x == 0 && pstep < p.prof_cap)                                \
      atomicMax(p.prof + (size_t)pstep * PROF_SLOTS + (slot), wall_clock64());                      \
  } while (0)
// Tile workgroup (tile j, layer L) of the layer split.
__device__ __noinline__ void df_tiles(KParams&) {
  KParams& p = kp();
  float* const lds = lds_base();
  float* const scr = lds + L_SCR;
  int* const misc = (int*)(lds + L_MISC);
  int* const rows = (int*)(scr + S_ROW);
  const int g = p.glist[0];
  const GraphInfo gi = p.ginfo[g];
  const int tb = (int)blockIdx.x - 2 * p.n_env, j = tb >> 1, L = tb & 1;
  unsigned long long* const seen = (unsigned long long*)(lds + L_MISC + 42);
  unsigned long long* const tried0 = (unsigned long long*)(lds + L_MISC + 38);
  if (threadIdx.x == 0) *seen = *tried0 = 0ull;
  int nl_prev = 0;  // live nodes of the previous step (its tile count: the self-pick's partials)
  for (int pstep = 0;; ++pstep) {
    if (threadIdx.x == 0) {
      misc[60] = pstep;
      misc[30] = 0;  // this step's self-pick not decided yet (df_wait_rec)
#ifdef MD_TORN_SLOT
      misc[25] = pstep % 3 == 1;  // every third step: the prebuild reads a torn slot
#endif
    }
    __syncthreads();
    // the step record; meanwhile the iteration-1 prebuild, first from the self-pick (the result
    // phase A will take, derived from the previous step's arg-max partials before phase A's slot
    // check), then, if phase A's early word names another result, from that one (rows and sums
    // are tagged with the result's slot; both store at once: phase A takes the same node, hence
    // the same state and tile assignment)
    int pre_state = 0, r;
    unsigned long long pre_used = 0ull;
#ifdef MD_TORN_SLOT
    unsigned long long torn_tried = 0ull;  // (a torn step's prebuild runs once per early word)
#endif
    while ((r = df_wait_rec(p, (unsigned)(pstep + 1), true, false, pstep - 1,
                            pstep >= 1 ? (nl_prev + TILE - 1) / TILE : 0)) >= 2) {
      const unsigned long long ew = r == 2 ? *seen : *tried0;  // (4: the self-pick)
#ifdef MD_TORN_SLOT
      if (misc[25] && ew == torn_tried) continue;
      torn_tried = ew;
#endif
      if (ew != 0ull && ew != pre_used) {
        DF_STAMP_MAX(54);
        pre_used = 0ull;
        // diagnostics: tile 0's layer-0 workgroup stamps the pieces of its prebuild
        unsigned long long* const pts = p.prof != nullptr && tb == 0 && pstep < p.prof_cap ? p.prof + (size_t)pstep * PROF_SLOTS : nullptr;
        pre_state = prebuild_lists(p, gi, j, L, ew, pts, r >= 3 ? *seen : 0ull);
        DF_STAMP_MAX(55);
        if (pre_state) pre_used = ew;
#ifdef MD_TORN_SLOT
        // a torn slot belongs to a result phase A does not take: the prebuild's early word (and
        // so its rows' tag) names the other slot of the pair
        const unsigned long long ewt = misc[25] ? ew ^ 1ull : ew;
        if (pre_state) pre_used = ewt;
#else
        const unsigned long long ewt = ew;
#endif
        // a self-pick prebuild that phase A's early word has already overtaken (it names another
        // result) stops after its lists
        const unsigned long long now = ((unsigned long long)(unsigned)misc[37] << 32) | (unsigned)misc[36];
        if (r >= 3 && pre_state == 1 && now != 0ull && now != *seen && now != ew) {
          pre_state = 0;
          pre_used = 0ull;
        }
        // the whole of iteration 1 too (MD_VARIANT bit 128: lists only)
        if (pre_state == 1 && !(p.variant & 128) && spec_iteration1(p, gi, j, L, ew, df_ptag(df_tag(pstep), ewt), pts))
          pre_state = 3;
        DF_STAMP_MAX(56);
        DF_STAMP_TILE(2);
      }
    }
    if (r != 1 || misc[50] != ST_RUN) break;
    DF_STAMP(4);
    const int nl = misc[51];
    nl_prev = nl;
    const unsigned long long cw = ((unsigned long long)(unsigned)misc[53] << 32) | (unsigned)misc[52];
    __syncthreads();
    // the next step's wait starts from this step's early word: a change is the next phase A's
    if (threadIdx.x == 0) *seen = ((unsigned long long)(unsigned)misc[55] << 32) | (unsigned)misc[54];
    if (j >= (nl + TILE - 1) / TILE) continue;
    const int pre_ok = pre_state != 0 && cw == pre_used ? pre_state : 0;
    if (p.prof != nullptr && threadIdx.x == 0 && pstep < p.prof_cap) {  // diagnostics
      unsigned long long* const ps = p.prof + (size_t)pstep * PROF_SLOTS;
      atomicMax(ps + (pre_ok == 3 ? 77 : 76), wall_clock64());  // latest record seen, with / without prebuild
      if (pre_ok != 3) atomicAdd(ps + 79, 1ull);                 // tiles without the confirmed prebuild
    }
    // a tile without the confirmed prebuild reads phase A's outputs: the whole of phase A first
    if (pre_ok != 3 && df_wait_rec(p, (unsigned)(pstep + 1), false, true) != 1) break;
    DF_STAMP_MAX(43);
    const unsigned tn = df_tag(pstep), tp = cw != 0ull ? df_ptag(tn, cw) : tn;
    bool nb_ok = true;
    // iteration 1 (skipped when the confirmed prebuild ran it)
    if (pre_ok != 3) {
      if (pre_ok == 0) {
        if (threadIdx.x < TILE) {
          const int rr = j * TILE + threadIdx.x;
          const float4 e = ldc4((const float*)(p.live + 4 * (size_t)gi.node_off), min(rr, gi.n - 1) * 16);
          const bool ok = rr < nl && MD_BOK(__float_as_int(e.x) >= 0 && __float_as_int(e.x) < gi.n && nl <= gi.n, 6);
          const unsigned c = (unsigned)__float_as_int(e.w);
          lds_i32* hdr = (lds_i32*)(int*)(scr + S_NBH);
          rows[threadIdx.x] = ok ? __float_as_int(e.x) : -1;
          hdr[64 + threadIdx.x] = ok ? __float_as_int(e.y) : 0;       // layer 0: CSR begin
          hdr[96 + threadIdx.x] = ok ? (int)(c & 0xffffu) : 0;        //          CSR extent
          hdr[64 + 16 + threadIdx.x] = ok ? __float_as_int(e.z) : 0;  // layer 1
          hdr[96 + 16 + threadIdx.x] = ok ? (int)(c >> 16) : 0;
        }
        __syncthreads();
        nb_ok = build_nb_lists(p, gi, rows, scr, nullptr, L);
      } else {
        nb_ok = pre_ok == 1;
      }
      // (the host enables this mode only when no tile's lists can exceed NB_CAP)
      if (!nb_ok) {
        if (threadIdx.x == 0) raise_err(p, ERR_DF_LISTS);
        break;
      }
      gather_tile2s(p, gi, 1, rows, scr, L);
      __syncthreads();
      update_tile_split(lds + L_W, scr, L);
      __syncthreads();
      normalize_tile_split(scr + S_E, scr, L);
      __syncthreads();
      df_store_tile(p, j, L, 1, tn);
      __syncthreads();
    }
    DF_STAMP(5);
    DF_STAMP_MAX(44);
    DF_STAMP_TILE(0);
    // iteration 2: the neighbours' iteration-1 rows (a confirmed prebuild's are valid too)
    gather_df(p, gi, 2, L, tn, tp);
    __syncthreads();
    DF_STAMP(23);
    update_tile_split(lds + L_W, scr, L);
    __syncthreads();
    normalize_tile_split(scr + S_E, scr, L);
    __syncthreads();
    df_store_tile(p, j, L, 2, tn);
    __syncthreads();
    DF_STAMP(6);
    DF_STAMP_MAX(45);
    // iteration 3, then the layer-1 rows to the layer-0 workgroup, which runs the attention and
    // the Q head and publishes the arg-max partial
    gather_df(p, gi, 3, L, tn, tn);
    __syncthreads();
    DF_STAMP(29);
    update_tile_split(lds + L_W, scr, L);
    __syncthreads();
    normalize_tile_split(scr + S_E, scr, L);
    __syncthreads();
    DF_STAMP(30);
    if (L == 1) {
      split_publish(p, scr, j, (unsigned long long)(pstep + 1));
      DF_STAMP_MAX(47);
    } else {
      split_receive(p, scr, j, (unsigned long long)(pstep + 1));
      DF_STAMP(8);
      attention_q_tile(p, lds, scr, gi, g, rows, (float*)(df_ap(p) + 4 * (size_t)j), (unsigned long long)(pstep + 1),
                       nullptr);
      DF_STAMP(9);
      DF_STAMP(10);
      DF_STAMP_MAX(46);
    }
  }
}
#undef DF_STAMP
#undef DF_STAMP_MAX
#undef DF_STAMP_TILE

__device__ __forceinline__ void engine_body(KParams& p, const float* __restrict__ wimg) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* scr = lds + L_SCR;
  int* pref = (int*)(lds + L_PREF);
  int* rows = (int*)(scr + S_ROW);

  // Dedicated mode (p.n_env > 0): workgroup b < n_env owns graph glist[b] and keeps its
  // environment in LDS across steps; workgroup n_env + b runs graph glist[b]'s virtual-node
  // chain and graph head while the tiles are computed and hands y / mix / aux to them; the
  // remaining workgroups own the weight image and do tiles.
  // Shared mode: every workgroup runs phase A for graphs b, b + grid, ... and then tiles
  // (the tile workgroups compute the virtual-node chain of the graphs they touch).
  if ((int)blockIdx.x >= p.n_main) {
    spec_loop(p);
    return;
  }
  const bool ded = p.n_env > 0;
  // grid-wide environment step: one graph too large for LDS (global mode) in shared mode
  // (MD_VARIANT bit 2: off, the one-workgroup step)
  const bool team = !ded && p.nglist == 1 && p.tctl != nullptr && !(p.variant & 2) && p.n_main <= TEAM_MAX_WG &&
                    (!phase_a_fits_lds(p.ginfo[p.glist[0]].n, p.ginfo[p.glist[0]].e[0] + p.ginfo[p.glist[0]].e[1]) ||
                     (p.variant & 64));
  const bool is_env = ded && (int)blockIdx.x < p.n_env;
  const bool is_head = ded && !is_env && (int)blockIdx.x < 2 * p.n_env;
  const int twg0 = ded ? 2 * p.n_env : 0;
  const int ntw = p.n_main - twg0;
  if (!is_env) {
    load_weights(lds + L_W, wimg);
    if (is_head) stage_wl1(p, scr);  // graph_head's w_layer1, resident for the launch
    __syncthreads();
    if (wave_id() == 0) {
      // constant virtual-node input: normalize(relu([1,1] . w_n2l))  (net :247,272-283)
      const int lane = lane_id();
      const float x = fmaxf(fmaf(1.f, lds[L_W + W_IWN + 64 + lane], fmaf(1.f, lds[L_W + W_IWN + lane], 0.f)), 0.f);
      const float nr = wave_norm64(x);
      lds[L_Y0 + lane] = x / fmaxf(nr, 1e-12f);
    }
    __syncthreads();
  }
  if (p.df != nullptr) {  // dataflow mode (single graph, layer split): no grid barrier
    if (is_env) df_env(p);
    else if (is_head) df_head(p);
    else df_tiles(p);
    return;
  }

  unsigned target = 0;
  int* bflag = (int*)(lds + L_MISC) + 61;  // barrier error broadcast
  const int my_gl = (int)threadIdx.x < p.nglist ? p.glist[threadIdx.x] : 0;  // nglist <= G_CAP = NTHREADS
  const GraphInfo spec_gi = p.ginfo[p.glist[0]];
  int pstep = 0;
  bool have_q = false, staged = false;
  const int ng = p.nglist;
  // iteration-1 prebuild (single graph, layer split, speculative steps on): this workgroup's tile
  // and layer, the last early word seen and the one its current prebuild used
  const bool pre_tile = ded && ng == 1 && p.pre_ew != nullptr && !is_env && !is_head &&
                        2 * ((spec_gi.n + TILE - 1) / TILE) <= p.n_main - 2 * p.n_env;
  const int pre_j = ((int)blockIdx.x - 2 * p.n_env) >> 1, pre_L = ((int)blockIdx.x - 2 * p.n_env) & 1;
  unsigned long long pre_seen = 0ull, pre_used = 0ull;
  while (true) {
    // ---------------- phase A
    MD_PROF(0);
    if (threadIdx.x == 0) ((int*)(lds + L_MISC))[60] = pstep;
    __syncthreads();
    bool wdirty = false;  // the weight image's LDS was used (reloaded below, one call site)
    if (ded) {
      if (is_env) staged = phase_a(p, p.glist[blockIdx.x], have_q, lds, staged);
    } else if (team) {
      // one global-mode graph: workgroup 0 decides the actions, then every workgroup runs the
      // environment step (team_env_step) and workgroup 0 finishes phase A
      int* tq = (int*)(lds + L_MISC) + 40;
      if (blockIdx.x == 0) {
        phase_a(p, p.glist[0], have_q, lds, false, tq);
        if (threadIdx.x == 0) {
          stc(p.tctl, tq[2] ? tq[0] : -1);
          stc(p.tctl + 1, tq[1]);
        }
      }
      if (grid_sync(p, target, bflag)) break;
      if (threadIdx.x == 0) {
        tq[0] = ldc(p.tctl);
        tq[1] = ldc(p.tctl + 1);
      }
      __syncthreads();
      const int pn = tq[0], pf = tq[1];
      __syncthreads();
      if (pn >= 0) {
        Team T;
        T.gt = (int)blockIdx.x * NTHREADS + (int)threadIdx.x;
        T.gs = p.n_main * NTHREADS;
        T.use = 0;
        T.target = &target;
        T.flag = bflag;
        T.tmp = (int*)(scr + TEAM_TMP_OFF);
        T.acc = nullptr;
        T.t = 0;
        T.prof_any = p.prof != nullptr && pstep < p.prof_cap ? p.prof + (size_t)pstep * PROF_SLOTS + 80 : nullptr;
        T.t0any = 0;
        if (p.prof != nullptr && blockIdx.x == 0 && pstep < p.prof_cap) {
          T.acc = p.prof + (size_t)pstep * PROF_SLOTS + 80;
          if (threadIdx.x == 0) p.prof[(size_t)pstep * PROF_SLOTS + 87] = wall_clock64();
        }
        int terr = 0;
        if (team_env_step(p, T, p.glist[0], pn, pf, &terr)) break;
        wdirty = (terr & TEAM_WDIRTY) != 0;
        terr &= ~TEAM_WDIRTY;
        if (T.acc != nullptr && threadIdx.x == 0) T.acc[7] = wall_clock64() - T.acc[7];  // slot 87: step total
        if (blockIdx.x == 0) {
          GraphVar& gv = *(GraphVar*)(lds + L_GV);
          if (threadIdx.x == 0) {
            gv.npend = 0;
            if (terr) raise_err(p, terr);
            if (gv.alive[0] == 0 || gv.alive[1] == 0) gv.status = ST_TERMINAL;
            else if (p.run_mode == RUN_STEP) gv.status = ST_PAUSED;
            else gv.status = ST_RUN;
          }
          __syncthreads();
          gv_store(p, p.glist[0], &gv);
          __syncthreads();
        }
      }
    } else {
      for (int gi = blockIdx.x; gi < ng; gi += p.n_main) {
        phase_a(p, p.glist[gi], have_q, lds, false);
        wdirty = true;
      }
    }
    if (wdirty) load_weights(lds + L_W, wimg);
    MD_PROF(3);
    // iteration-1 prebuild (p.pre_ew): a single graph's tile workgroups wait at barrier A for
    // the release or for phase A's early word, and build their iteration-1 rows and lists from
    // the speculative result it names meanwhile
    int pre_state = 0;
    bool errA;
    if (pre_tile) {
      grid_arrive(p, target);
      unsigned long long* seen_out = (unsigned long long*)(lds + L_MISC + 42);
      while (grid_wait(p, target, bflag, p.pre_ew, pre_seen, seen_out) == 2) {
        pre_seen = *seen_out;
        if (pre_state == 0 && pre_seen != 0ull) {
          pre_state = prebuild_lists(p, spec_gi, pre_j, pre_L, pre_seen);
          if (pre_state) pre_used = pre_seen;
          // the whole of iteration 1 too (MD_VARIANT bit 128: lists only)
          if (pre_state == 1 && !(p.variant & 128) && spec_iteration1(p, spec_gi, pre_j, pre_L, pre_seen)) pre_state = 3;
        }
      }
      errA = *bflag != 0;
    } else {
      errA = grid_sync(p, target, bflag);
    }
    MD_PROF(4);
    if (errA) break;
    // ---------------- tile prefix over the launch's graphs
    // (one graph, dedicated mode: the rows of tile blockIdx - twg0 are loaded speculatively in
    // the same round trip; they are this workgroup's tile whenever there are enough workgroups)
    const bool spec = ded && ng == 1 && !is_env && !is_head && threadIdx.x < TILE;
    float4 spec_e = make_float4(0.f, 0.f, 0.f, 0.f);
    // layer split (below) is certain for one graph whose every tile fits two workgroups
    const bool spec_split = 2 * ((spec_gi.n + TILE - 1) / TILE) <= ntw;
    const int spec_tile = spec_split ? ((int)blockIdx.x - twg0) >> 1 : (int)blockIdx.x - twg0;
    if (spec) {
      const int r = spec_tile * TILE + threadIdx.x;
      spec_e = ldc4((const float*)(p.live + 4 * (size_t)spec_gi.node_off), min(r, spec_gi.n - 1) * 16);
    }
    // phase A's confirmation of the speculative result a prebuild used (same round trip)
    if (pre_state != 0 && threadIdx.x == 64) {
      const unsigned long long cw = __hip_atomic_load((const g_u64*)p.pre_cw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ((int*)(lds + L_MISC))[47] = cw == pre_used ? pre_state : 0;
    }
    bool waiting = false;
    if (threadIdx.x < ng) {
      const GraphVar* gv = p.gvar + my_gl;
      const int st = ldc(&gv->status), nl = ldc(&gv->n_live);
      pref[threadIdx.x + 1] = st == ST_RUN ? (nl + TILE - 1) / TILE : 0;
      waiting = st == ST_WAIT_HOST;
      if (threadIdx.x == 0) ((int*)(lds + L_MISC))[62] = nl;  // n_live of the first graph
    }
    waiting = __syncthreads_or(waiting);
    if (threadIdx.x == 0) {
      pref[0] = 0;
      for (int i = 0; i < ng; ++i) pref[i + 1] += pref[i];
    }
    __syncthreads();
    const int ttot = pref[ng];
    const int pre_ok = pre_state != 0 ? ((int*)(lds + L_MISC))[47] : 0;  // 1 / 2: use the prebuilt rows (and lists)
    if (p.prof != nullptr && pre_tile && (int)blockIdx.x == twg0 && threadIdx.x == 0 && pstep < p.prof_cap)
      p.prof[(size_t)pstep * PROF_SLOTS + 78] = 1 + 10 * pre_state + pre_ok;  // diagnostics: prebuild state
    if (ttot == 0) {
      if (!waiting) break;
      // only graphs waiting for a host answer: one more barrier (nobody writes a GraphVar
      // before every workgroup has read the prefix), then phase A polls again
      if (grid_sync(p, target, bflag)) break;
      pstep++;
      continue;
    }
    const int per = (ttot + ntw - 1) / ntw;
    const int tb = (int)blockIdx.x - twg0;
    const bool tiles = !is_env && !is_head;
    // Layer split (dedicated mode, two tile workgroups per tile): workgroup (tile, L) runs layer
    // L of iterations 1 and 2; iteration 3 (attention mixes the layers) runs on L = 0 alone.
    const bool split = ded && 2 * ttot <= ntw && ttot <= XB_SLOTS;
    const int L = split ? (tb & 1) : 0;
    int t0, t1;
    if (split) {
      t0 = tiles ? min(ttot, tb >> 1) : 0;
      t1 = tiles ? min(ttot, t0 + 1) : 0;
    } else {
      t0 = tiles ? min(ttot, tb * per) : 0;
      t1 = tiles ? min(ttot, t0 + per) : 0;
    }
    bool nb_ok = false, failed = false;
    // hand-off tag of this step's graph head (unique per launch and step)
    const unsigned long long htag = ded ? (unsigned long long)(pstep + 1) : 0ull;

    for (int it = 1; it <= BP_ITERS; ++it) {
      MD_PROF(10 + it);
      if (is_head && it >= 2) head_iteration(p, lds, scr, p.glist[blockIdx.x - p.n_env], it, htag);
      int cur = ded ? 0x7fffffff : -1;  // graph-list index whose virtual node / graph head is loaded
      const bool sit = split;  // this iteration runs one layer per workgroup
      for (int t = t0; t < t1; ++t) {
        // iteration 1 done during phase A from the confirmed speculative result
        if (it == 1 && pre_ok == 3 && split && t == pre_j && L == pre_L) {
          nb_ok = true;  // its lists (in LDS) serve iterations 2 and 3
          continue;
        }
        const int gl = tile_graph(pref, ng, t);
        const int g = p.glist[gl];
        const GraphInfo gi = p.ginfo[g];
        const int j = t - pref[gl];  // tile within the graph
        if (it >= 2 && gl != cur && cur != 0x7fffffff) {
          // virtual-node chain of this graph (identical in every workgroup that needs it)
          gv_load(p, g, (GraphVar*)(lds + L_GV));
          __syncthreads();
          const GraphVar& gv = *(const GraphVar*)(lds + L_GV);
          const int nt = (gv.n_live + TILE - 1) / TILE;
          float* sbuf = scr + S_HID;  // [2][64]
          float* yw = lds + L_YW;
          if (it == 2) {
            if (threadIdx.x < 128) yw[threadIdx.x] = lds[L_Y0 + (threadIdx.x & 63)];
            graph_sum(p, gi, nt, 0, sbuf, scr + S_YP);
            vrow_update(lds + L_W, scr, sbuf, yw);  // Y1 from S0
            graph_sum(p, gi, nt, 1, sbuf, scr + S_YP);
            vrow_update(lds + L_W, scr, sbuf, yw);  // Y2 from S1
            if (threadIdx.x < 128) stc(p.ybuf + (size_t)g * 128 + threadIdx.x, yw[threadIdx.x]);
          } else {
            if (threadIdx.x < 128) yw[threadIdx.x] = ldc(p.ybuf + (size_t)g * 128 + threadIdx.x);
            graph_sum(p, gi, nt, 2, sbuf, scr + S_YP);
            vrow_update(lds + L_W, scr, sbuf, yw);  // Y3 from S2
            graph_head(p, lds, scr, gi, gv, false, false);
          }
          cur = gl;
        }
        // rows of the tile and their CSR ranges (unchanged during a step: a single-tile
        // workgroup of dedicated mode keeps them; in shared mode the virtual-node chain reuses
        // that LDS); one 16-byte live-list entry per row
        // several tiles per workgroup: iteration 1 caches the tile's neighbour lists in HBM
        // (slot t), iterations 2-3 reload them with the rows (first 256 words per layer
        // speculatively, the rest only when a layer has more than 512 entries)
        const bool multi = (t1 - t0 > 1 || !ded) && t < p.nbc_slots;
        const bool cached = multi && it > 1;
        int cw = 0, ch = 0;
        if (cached) {
          const int* src = p.nbc + (size_t)t * NBC_INTS;
          cw = ldc(src + NBC_HDR + (threadIdx.x >> 8) * NBC_LWORDS + (threadIdx.x & 255));
          if (threadIdx.x < 67) ch = ldc(src + threadIdx.x);
        }
        const bool prebuilt = it == 1 && (pre_ok == 1 || pre_ok == 2) && split && t == pre_j && L == pre_L;
        if ((it == 1 || t1 - t0 > 1 || !ded) && !prebuilt) {
          if (threadIdx.x < TILE) {
            const int r = j * TILE + threadIdx.x;
            int nl;
            float4 e;
            if (spec && it == 1 && t == spec_tile) {
              nl = ((const int*)(lds + L_MISC))[62];
              e = spec_e;
            } else {
              nl = ldc(&p.gvar[g].n_live);
              e = ldc4((const float*)(p.live + 4 * (size_t)gi.node_off), min(r, gi.n - 1) * 16);
            }
            const bool ok = r < nl && MD_BOK(__float_as_int(e.x) >= 0 && __float_as_int(e.x) < gi.n && nl <= gi.n, 6);
            const unsigned c = (unsigned)__float_as_int(e.w);
            lds_i32* hdr = (lds_i32*)(int*)(scr + S_NBH);
            rows[threadIdx.x] = ok ? __float_as_int(e.x) : -1;
            hdr[64 + threadIdx.x] = ok ? __float_as_int(e.y) : 0;       // layer 0: CSR begin
            hdr[96 + threadIdx.x] = ok ? (int)(c & 0xffffu) : 0;        //          CSR extent
            hdr[64 + 16 + threadIdx.x] = ok ? __float_as_int(e.z) : 0;  // layer 1
            hdr[96 + 16 + threadIdx.x] = ok ? (int)(c >> 16) : 0;
          }
        }
        if (cached) {
          lds_i32* hdr = (lds_i32*)(int*)(scr + S_NBH);
          ((lds_i32*)(int*)(scr + S_NBL))[(threadIdx.x >> 8) * NBC_LWORDS + (threadIdx.x & 255)] = cw;
          if (threadIdx.x < 64) hdr[threadIdx.x] = ch;
          else if (threadIdx.x < 66) hdr[128 + threadIdx.x - 64] = ch;
          else if (threadIdx.x == 66) ((int*)(lds + L_MISC))[59] = ch;
        }
        __syncthreads();
        // alive neighbour lists: built at iteration 1, kept for 2 and 3 when this workgroup
        // has a single tile (its LDS copy is intact)
        unsigned long long tg0 = 0;
        if (p.prof != nullptr && it == 2 && threadIdx.x == 0 && pstep < p.prof_cap) {
          tg0 = wall_clock64();
          atomicMax(p.prof + (size_t)pstep * PROF_SLOTS + 47, tg0);  // latest tile start (it 2)
        }
        {
          unsigned long long* ts = nullptr;
          if (p.prof != nullptr && it == 1 && (int)blockIdx.x == twg0 && t == t0 && pstep < p.prof_cap)
            ts = p.prof + (size_t)pstep * PROF_SLOTS;
          TSTAMP(54);
          if (cached) {
            nb_ok = ((const int*)(lds + L_MISC))[59] != 0;
            const lds_i32* hdr = (const lds_i32*)(const int*)(scr + S_NBH);
            const int nw0 = (hdr[128] + 1) >> 1, nw1 = (hdr[129] + 1) >> 1;
            if (nb_ok && (nw0 > 256 || nw1 > 256)) {
              const int* src = p.nbc + (size_t)t * NBC_INTS + NBC_HDR;
              lds_i32* words = (lds_i32*)(int*)(scr + S_NBL);
              for (int i = 256 + (int)threadIdx.x; i < nw0; i += NTHREADS) words[i] = ldc(src + i);
              for (int i = 256 + (int)threadIdx.x; i < nw1; i += NTHREADS) words[NBC_LWORDS + i] = ldc(src + NBC_LWORDS + i);
              __syncthreads();
            }
          } else if (prebuilt) {
            nb_ok = pre_ok == 1;  // (2: lists over NB_CAP, the per-row gather)
          } else if (it == 1 || t1 - t0 > 1 || !ded) {
            nb_ok = build_nb_lists(p, gi, rows, scr, ts, sit ? L : -1);
            if (multi) nbc_store(p, t, scr, nb_ok);
          }
          TSTAMP(55);
        }
        if (nb_ok) {
          if (sit) gather_tile2s(p, gi, it, rows, scr, L);
          else gather_tile2(p, gi, it, rows, scr);
        } else {
          gather_tile(p, gi, it, rows, scr);
        }
        __syncthreads();
        if (tg0 != 0) atomicMax(p.prof + (size_t)pstep * PROF_SLOTS + 46, wall_clock64() - tg0);  // longest gather (it 2)
        MD_PROF_T(23 + 3 * (it - 1));
        if (sit) update_tile_split(lds + L_W, scr, L);
        else update_tile(lds + L_W, scr);
        __syncthreads();
        if (it == 1) MD_PROF_T(36);
        if (sit) normalize_tile_split(scr + S_E, scr, L);
        else normalize_tile(scr + S_E, scr);
        __syncthreads();
        if (it == 1) MD_PROF_T(37);
        if (threadIdx.x < (sit ? 64 : 128)) {
          // tile partial sums of the virtual node (rows in ascending compact order from 0)
          const int l = sit ? L : (int)threadIdx.x >> 6, c = threadIdx.x & 63;
          const float* ate = scr + S_E + l * 64 * LDT + c * LDT;
          const float* atx = scr + S_X + l * 64 * LDT + c * LDT;
          const int nv = tile_rows_valid(rows);
          const float s_new = col_sum16(ate, nv), s_old = it == 1 ? col_sum16(atx, nv) : 0.f;
          float* sp = p.spart + (size_t)(gi.tile_off + j) * 384;
          if (it == 1) {
            stc(sp + l * 64 + c, s_old);        // S0 (first-layer input)
            stc(sp + 128 + l * 64 + c, s_new);  // S1
          } else if (it == 2) {
            stc(sp + 256 + l * 64 + c, s_new);  // S2
          }
        }
        if (it < 3) {
          // new embeddings to HBM as 16-byte sc1 stores: 16 lanes per row, 4 rows per wave
          const int w = wave_id(), l = sit ? L : w >> 2, lane = lane_id();
          float* hb = p.H[l][(it - 1) & 1] + (size_t)gi.node_off * EMB;
          const int r = 4 * (w & 3) + (lane >> 4), q4 = lane & 15;
          const int v = rows[r];
          const float* e = scr + S_E + l * 64 * LDT + 4 * q4 * LDT + r;
          if (v >= 0 && !(sit && w >= 4)) stc4(hb, v * 256 + q4 * 16, make_float4(e[0], e[LDT], e[2 * LDT], e[3 * LDT]));
        }
        __syncthreads();
        MD_PROF_T(24 + 3 * (it - 1));
        if (it == 3 && sit) {
          // the layer-1 rows go to the layer-0 workgroup, which runs the attention and Q head
          if (L == 1) {
            split_publish(p, scr, t, htag);
            continue;
          }
          split_receive(p, scr, t, htag);
        }
        if (it == 3) {
          unsigned long long* ts = nullptr;
          if (p.prof != nullptr && (int)blockIdx.x == twg0 && t == t0 && pstep < p.prof_cap)
            ts = p.prof + (size_t)pstep * PROF_SLOTS;
          attention_q_tile(p, lds, scr, gi, g, rows, p.apart + (size_t)(gi.tile_off + j) * 4, htag, ts);
        }
        MD_PROF_T(25 + 3 * (it - 1));
        if (p.prof != nullptr && threadIdx.x == 0 && pstep < p.prof_cap)
          atomicMax(p.prof + (size_t)pstep * PROF_SLOTS + 42 + it, wall_clock64());  // slowest tile's end
      }
      MD_PROF(3 + 2 * it);
      failed = grid_sync(p, target, bflag);
      MD_PROF(4 + 2 * it);
      if (failed) break;
    }
    if (failed) break;
    have_q = true;
    pstep++;
  }
  if (p.n_spec > 0 && blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store((g_u64*)p.spec_req, SPEC_EXIT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Completion record (p.h_done): every workgroup drains its stores and counts itself out; the
// last one copies the launch's GraphVars and the error word to mapped host memory with
// system-scope stores, drains them, then writes the launch tag.  The host polls the tag
// instead of querying the runtime, and reads the GraphVars without a copy.
__device__ __noinline__ void kernel_exit(KParams&) {
  KParams& p = kp();
  if (p.h_done == nullptr) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  __shared__ int last;
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add((g_u32*)p.exit_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  for (int i = threadIdx.x; i < p.nglist * GV_WORDS; i += NTHREADS) {
    const int g = p.glist[i / GV_WORDS], k = i % GV_WORDS;
    __hip_atomic_store(p.h_gvar + (size_t)g * GV_WORDS + k, ldc((const int*)(p.gvar + g) + k), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (p.nglist <= PUB_EXIT_MAX) {
    // the terminal graphs' traces (trace_publish: small launches publish here)
    for (int i = 0; i < p.nglist; ++i) {
      const int g = p.glist[i];
      const GraphVar* v = p.gvar + g;
      if (ldc(&v->status) == ST_TERMINAL) trace_publish(p, p.ginfo[g], ldc(&v->steps));
    }
  }
  if (threadIdx.x == 0)
    __hip_atomic_store(p.h_done + 1, (unsigned)__hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(p.h_done, p.launch_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(NTHREADS, 1) md_rollout_kernel(Params p, const float* __restrict__ wimg) {
  if (!kargs_layout_ok()) {
    if (threadIdx.x == 0) __hip_atomic_store(p.err, ERR_ABI, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  engine_body(kp(), wimg);
  kernel_exit(kp());
}

// Batched rollouts through the device work queue (queue_loop); its own entry point so the
// lock-step body's register allocation is not shaped by the queue code.
__global__ void __launch_bounds__(NTHREADS, 1) md_queue_kernel(Params p, const float* __restrict__ wimg) {
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
  queue_loop(kpp, lds, wimg);
  kernel_exit(kpp);
}

#include "md_wave.h"

__global__ void __launch_bounds__(NTHREADS, 1) md_env_kernel(Params p, const float* __restrict__ wimg) {
  if (!kargs_layout_ok()) {
    if (threadIdx.x == 0) __hip_atomic_store(p.err, ERR_ABI, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  engine_body(kp(), wimg);
  kernel_exit(kp());
}

// Clears up to six device ranges (bytes, multiples of 4) in one launch: the per-launch control
// words, barrier shards and hand-off tags that would otherwise take one memset dispatch each.
struct ClearList {
  void* ptr[6];
  unsigned long long bytes[6];
  int n;
};
__global__ void __launch_bounds__(256) md_clear_kernel(ClearList cl) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
  for (int k = 0; k < cl.n; ++k) {
    unsigned* w = (unsigned*)cl.ptr[k];
    const size_t nw = cl.bytes[k] / 4;
    for (size_t i = t; i < nw; i += stride) w[i] = 0u;
  }
}

// Reset every graph in glist to the initial (pre-s0) state.
// Unit-cost first-layer tables of every dmax 1..dm_max (the per-step rebuild of phase A
// becomes a copy): block dm, thread per row d, the same expressions as env_step's rebuild.
__global__ void __launch_bounds__(256) md_h0_kernel(const float* __restrict__ w, float* tab, int dm_lo, int dm_hi) {
  const int dm = dm_lo + (int)blockIdx.x;
  if (dm > dm_hi) return;
  const float* wn = w + W_N2L;
  for (int d = 1 + (int)threadIdx.x; d <= dm; d += blockDim.x) {
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
    float* row = tab + h0g_row(dm, d) * EMB;
#pragma unroll
    for (int c = 0; c < 64; ++c) row[c] = fmaxf(fmaf(f, wn[64 + c], fmaf(f, wn[c], 0.f)), 0.f) / den;
  }
}

__global__ void md_reset_kernel(Params p) {
  const int gidx = blockIdx.x;
  if (gidx >= p.nglist) return;
  const int g = p.glist[gidx];
  const GraphInfo gi = p.ginfo[g];
  for (int v = threadIdx.x; v < gi.n; v += blockDim.x) {
    p.covered[gi.node_off + v] = 0;
    p.q[gi.node_off + v] = NEG_INF;
  }
  for (int l = 0; l < 2; ++l) {
    for (int e = threadIdx.x; e < gi.e[l]; e += blockDim.x) p.estate[l][gi.eoff[l] + e] = E_ALIVE;
    for (int e = threadIdx.x; e < 2 * gi.e[l]; e += blockDim.x) p.calive[l][gi.coff[l] + e] = 1;
  }
  if (threadIdx.x == 0) {
    GraphVar v = {};
    v.status = ST_RUN;
    v.argmax = -1;
    p.gvar[g] = v;
    p.lab_ok[g] = 0;
  }
}

}  // namespace md

// ------------------------------------------------------------------ launch wrappers (C++)
namespace md {
int lds_bytes() { return L_TOTAL * 4; }
int weight_image_floats() { return W_IEND; }
bool phase_a_fits_lds_host(int n, int et) { return phase_a_fits_lds(n, et); }
bool pfx_fits_host(int n, int et) { return pfx_fits(n, et); }
long long pfx_words_host(int et) { return pfx_words(et); }
// speculative workgroups: the environment plus the candidate ranking keys in LDS
bool spec_fits_lds_host(int n, int et) {
  return phase_a_fits_lds(n, et) && env_layout(n, et).total + spec_rank_words(n) <= A_WORDS;
}

// Host-side permutation of the reference-layout weight blob into the LDS image.
void build_weight_image(const float* w, float* img) {
  auto frag = [&](int dst, int src, int K) {
    for (int cb = 0; cb < 4; ++cb)
      for (int s = 0; s < K / 4; ++s)
        for (int lane = 0; lane < 64; ++lane) {
          const int k = 4 * s + (lane >> 4), c = 16 * cb + (lane & 15);
          img[dst + (cb * (K / 4) + s) * 64 + lane] = w[src + k * 64 + c];
        }
  };
  for (int i = 0; i < W_IEND; ++i) img[i] = 0.f;
  frag(W_IP1, W_P1, 64);
  frag(W_IP2, W_P2, 64);
  frag(W_IP3, W_P3, 128);
  frag(W_IT, W_T, 64);
  for (int cb = 0; cb < 2; ++cb)
    for (int s = 0; s < 16; ++s)
      for (int lane = 0; lane < 64; ++lane) {
        const int k = 4 * s + (lane >> 4), c = 16 * cb + (lane & 15);
        img[W_IH1 + (cb * 16 + s) * 64 + lane] = w[W_H1 + k * 32 + c];
      }
  for (int i = 0; i < 64; ++i) {
    img[W_ITB + i] = w[W_TB + i];
    img[W_ILW + i] = w[W_LW + i];
    img[W_ICP + i] = w[W_CP + i];
  }
  for (int i = 0; i < 36; ++i) img[W_IW2 + i] = w[W_W2 + i];
  img[W_ILB] = w[W_LB];
  for (int i = 0; i < 128; ++i) {
    img[W_IWN + i] = w[W_N2L + i];
    img[W_IWL2 + i] = w[W_WL2 + i];
  }
}

hipError_t launch_rollout(const Params& p, const float* wimg, int grid, hipStream_t s) {
  if (p.qmode == 2)
    hipLaunchKernelGGL(md_wq_kernel, dim3(grid), dim3(NTHREADS), lds_bytes(), s, p, wimg);
  else if (p.qmode)
    hipLaunchKernelGGL(md_queue_kernel, dim3(grid), dim3(NTHREADS), lds_bytes(), s, p, wimg);
  else if (p.run_mode == RUN_ROLLOUT)
    hipLaunchKernelGGL(md_rollout_kernel, dim3(grid), dim3(NTHREADS), lds_bytes(), s, p, wimg);
  else
    hipLaunchKernelGGL(md_env_kernel, dim3(grid), dim3(NTHREADS), lds_bytes(), s, p, wimg);
  return hipGetLastError();
}

hipError_t launch_h0(const float* w, float* tab, int dm_lo, int dm_hi, hipStream_t s) {
  if (dm_hi < dm_lo) return hipSuccess;
  hipLaunchKernelGGL(md_h0_kernel, dim3(dm_hi - dm_lo + 1), dim3(256), 0, s, w, tab, dm_lo, dm_hi);
  return hipGetLastError();
}

hipError_t launch_clear(void* const* ptr, const size_t* bytes, int n, hipStream_t s) {
  ClearList cl;
  size_t tot = 0;
  cl.n = 0;
  for (int k = 0; k < n && cl.n < 6; ++k) {
    if (ptr[k] == nullptr || bytes[k] == 0) continue;
    cl.ptr[cl.n] = ptr[k];
    cl.bytes[cl.n] = bytes[k];
    tot += bytes[k];
    cl.n++;
  }
  if (cl.n == 0) return hipSuccess;
  const int blocks = (int)std::min<size_t>(1024, (tot / 4 + 255) / 256);
  hipLaunchKernelGGL(md_clear_kernel, dim3(std::max(1, blocks)), dim3(256), 0, s, cl);
  return hipGetLastError();
}

hipError_t launch_reset(const Params& p, hipStream_t s) {
  hipLaunchKernelGGL(md_reset_kernel, dim3(p.nglist), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t set_kernel_attrs() {
  hipError_t e = hipFuncSetAttribute((const void*)md_rollout_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     lds_bytes());
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)md_queue_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes());
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)md_wq_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes());
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)md_env_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes());
}
}  // namespace md
