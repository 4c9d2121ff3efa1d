// md_gmm.hip — Geometric Multiplex Model generator on the device.
//
// The reference draws its synthetic two-layer test graphs with U/GMM.py:6-68 (the hyperbolic
// helpers of U/Hyperbolic.py:18-117): per node a hidden degree kappa and an angle theta per
// layer (layer 2 conditioned on layer 1), then one uniform per node pair (i < j, row-major) per
// layer, and the pair is linked when u < 1 / (1 + r^(1/T)) with
// r = (n / 2pi) |pi - |pi - |theta_i - theta_j||| / (mu kappa_i kappa_j).  That pair loop is
// O(N^2) Python in the reference (~4 s per N = 1000 graph); here it is one workgroup per layer
// streaming the pairs row by row, with an ordered compaction so the edges come out in the
// reference's lexicographic (networkx G.edges()) order.
//
// Two sources of randomness:
//  * exact: the caller passes the per-node values and the pair uniforms of the reference's own
//    numpy stream (mdcommunity_amd.gmm_gpu draws them exactly as U/GMM.py does); the device
//    only evaluates the link test.  Pairs whose uniform lies within a relative 1e-9 of the
//    threshold are reported back as ambiguous (pow/division order of the host's numpy could
//    differ in the last bit), and the host re-decides them with the reference's expression,
//    so the edge lists equal U/GMM.py's bit for bit.
//  * device: counter-based Philox4x32-10 streams keyed by the seed (kbar, the four per-node
//    uniform vectors and the pair uniforms), the per-node values computed on the device
//    (Lambert W by Halley iteration, erfinv) -- the same model, not the numpy stream.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "../../include/mdroll.h"

namespace mdg {

constexpr int NT = 512;
constexpr double GAMMA = 2.5, NU = 0.2, GCORR = 0.5, TEMP = 0.4;
constexpr double PI = 3.14159265358979323846;

// ------------------------------------------------------------------ Philox4x32-10
struct u4 {
  unsigned x, y, z, w;
};
__device__ __forceinline__ u4 philox(u4 c, unsigned k0, unsigned k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c.x;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c.z;
    const unsigned h0 = (unsigned)(p0 >> 32), l0 = (unsigned)p0, h1 = (unsigned)(p1 >> 32), l1 = (unsigned)p1;
    c = {h1 ^ c.y ^ k0, l1, h0 ^ c.w ^ k1, l0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
// Uniform double in [0, 1) with 53 random bits (numpy's random_sample construction) from
// stream `s` at index i of the key.
__device__ __forceinline__ double uni(unsigned long long key, unsigned s, unsigned long long i) {
  const u4 r = philox({(unsigned)i, (unsigned)(i >> 32), s, 0x6d647267u}, (unsigned)key, (unsigned)(key >> 32));
  return ((double)(r.x >> 5) * 67108864.0 + (double)(r.y >> 6)) / 9007199254740992.0;
}
enum : unsigned { S_KBAR = 1, S_KAPPA1 = 2, S_KAPPA2 = 3, S_THETA1 = 4, S_THETA2 = 5, S_PAIR0 = 6, S_PAIR1 = 7 };

// ------------------------------------------------------------------ per-node values (device mode)
// Lambert W, principal branch, x > 0 (scipy.special.lambertw's real value there): Halley steps.
__device__ double lambert_w0(double x) {
  double w = x < 2.0 ? log1p(x) : log(x) - log(log(x));
  for (int it = 0; it < 12; ++it) {
    const double ew = exp(w), f = w * ew - x;
    const double d = ew * (w + 1.0) - (w + 2.0) * f / (2.0 * w + 2.0);
    const double nw = w - f / d;
    if (fabs(nw - w) <= 1e-15 * fabs(nw)) return nw;
    w = nw;
  }
  return w;
}
__device__ __forceinline__ double kmin_of(double kbar) { return kbar * (GAMMA - 2.0) / (GAMMA - 1.0); }
// U/Hyperbolic.py conditional kappa of layer 2 given layer 1 (gmm._conditional_kappa)
__device__ double cond_kappa(double kappa1, double u, double kmin1, double kmin2) {
  const double g1 = GAMMA, g2 = GAMMA, nu = NU;
  const double phi = -log(1.0 - pow(kmin1 / kappa1, g1 - 1.0));
  double z = 1.0 / kmin1 * pow(phi, nu / (nu - 1.0)) * pow(kappa1, -g1);
  z = z * (kmin1 * pow(kappa1, g1) - pow(kmin1, g1) * kappa1);
  double zr = z * u;
  zr = (nu / (1.0 - nu)) * lambert_w0(pow(zr, (nu - 1.0) / nu) / (nu / (1.0 - nu)));
  zr = pow(zr, 1.0 / (1.0 - nu)) - pow(phi, 1.0 / (1.0 - nu));
  zr = exp(-pow(fmax(zr, 0.0), 1.0 - nu));
  return kmin2 * pow(1.0 - zr, 1.0 / (1.0 - g2));
}
// gmm._conditional_theta
__device__ double cond_theta(double theta1, double u, int n) {
  const double two_pi = 2.0 * PI;
  double sigma0 = n / (4.0 * PI);
  if (sigma0 > 100.0) sigma0 = 100.0;
  const double sigma = sigma0 * (1.0 / GCORR - 1.0);
  const double ell = sqrt(2.0) * sigma * erfinv((-1.0 + 2.0 * u) * erf(n / (2.0 * sqrt(2.0) * sigma)));
  double t = fmod(theta1 + two_pi * ell / n, two_pi);
  if (t < 0.0) t += two_pi;
  return t;
}

// One workgroup per graph: kbar (2), kappa and theta of both layers.  `uin` (optional, tests):
// [4][G][n] uniforms (kappa1, kappa2, theta1, theta2) and kbar [G][2] instead of Philox.
__global__ void __launch_bounds__(NT) gmm_nodes_kernel(int n, const unsigned long long* keys, const double* uin,
                                                       const double* kbar_in, int G, double* kbar, double* kappa,
                                                       double* theta) {
  const int g = blockIdx.x;
  const unsigned long long key = keys != nullptr ? keys[g] : 0ull;
  double kb[2];
  for (int l = 0; l < 2; ++l)
    kb[l] = kbar_in != nullptr ? kbar_in[2 * g + l] : 2.0 + 8.0 * uni(key, S_KBAR, (unsigned long long)l);
  if (threadIdx.x == 0) {
    kbar[2 * g] = kb[0];
    kbar[2 * g + 1] = kb[1];
  }
  const double kmin1 = kmin_of(kb[0]), kmin2 = kmin_of(kb[1]);
  const size_t base = (size_t)g * n;
  for (int i = threadIdx.x; i < n; i += NT) {
    const double uk1 = uin ? uin[0 * (size_t)G * n + base + i] : uni(key, S_KAPPA1, i);
    const double uk2 = uin ? uin[1 * (size_t)G * n + base + i] : uni(key, S_KAPPA2, i);
    const double ut1 = uin ? uin[2 * (size_t)G * n + base + i] : uni(key, S_THETA1, i);
    const double ut2 = uin ? uin[3 * (size_t)G * n + base + i] : uni(key, S_THETA2, i);
    const double k1 = kmin1 * pow(1.0 - uk1, 1.0 / (1.0 - GAMMA));
    const double t1 = 2.0 * PI * ut1;
    kappa[2 * base + i] = k1;
    kappa[2 * base + n + i] = cond_kappa(k1, uk2, kmin1, kmin2);
    theta[2 * base + i] = t1;
    theta[2 * base + n + i] = cond_theta(t1, ut2, n);
  }
}

// ------------------------------------------------------------------ links
// One workgroup per layer: rows i = 0..n-2, the row's pairs (i, j > i) in chunks of NT lanes;
// kept pairs are compacted in order (wave ballots, then the waves' counts through LDS), so the
// layer's edges come out sorted (u, v) with u < v.  Exact mode reads the pair uniforms (row-major
// pair index, the reference's stream order); device mode draws them from Philox.
__global__ void __launch_bounds__(NT) gmm_links_kernel(int n, const double* kappa, const double* theta, const double* mu,
                                                       const double* uniforms, const unsigned long long* keys,
                                                       int* edges, long long* ecount, long long ecap, long long* amb,
                                                       long long* acount, long long acap) {
  __shared__ int wcnt[NT / 64], wamb[NT / 64];
  const int L = blockIdx.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double* ka = kappa + (size_t)L * n;
  const double* th = theta + (size_t)L * n;
  const double m = mu[L];
  const long long npairs = (long long)n * (n - 1) / 2;
  const double* un = uniforms != nullptr ? uniforms + (size_t)L * npairs : nullptr;
  const unsigned long long key = keys != nullptr ? keys[L >> 1] : 0ull;
  const unsigned stream = (L & 1) ? S_PAIR1 : S_PAIR0;
  int* out = edges + 2 * (size_t)L * ecap;
  long long* am = amb + (size_t)L * acap;
  const double two_pi = 2.0 * PI, inv_t = 1.0 / TEMP;
  long long cnt = 0, acnt = 0;
  for (int i = 0; i + 1 < n; ++i) {
    const long long row = (long long)i * n - (long long)i * (i + 1) / 2 - (i + 1);  // pair index of (i, j) = row + j
    const double ki = ka[i], ti = th[i];
    for (int j0 = i + 1; j0 < n; j0 += NT) {
      const int j = j0 + (int)threadIdx.x;
      bool keep = false, ambig = false;
      if (j < n) {
        const long long pidx = row + j;
        const double u = un != nullptr ? un[pidx] : uni(key, stream, (unsigned long long)pidx);
        // the reference's expression, operation for operation (no contraction)
        const double dth = n / two_pi * fabs(PI - fabs(PI - fabs(ti - th[j])));
        const double r = dth / (m * ki * ka[j]);
        const double thr = 1.0 / (1.0 + pow(r, inv_t));
        keep = u < thr;
        ambig = un != nullptr && fabs(u - thr) <= 1e-9 * thr;
      }
      const unsigned long long bk = __ballot(keep), ba = __ballot(ambig);
      const unsigned long long below = (1ull << lane) - 1ull;
      if (lane == 0) {
        wcnt[w] = (int)__popcll(bk);
        wamb[w] = (int)__popcll(ba);
      }
      __syncthreads();
      long long pre = cnt, apre = acnt;
      int tot = 0, atot = 0;
      for (int k = 0; k < NT / 64; ++k) {
        if (k < w) {
          pre += wcnt[k];
          apre += wamb[k];
        }
        tot += wcnt[k];
        atot += wamb[k];
      }
      if (keep) {
        const long long at = pre + __popcll(bk & below);
        if (at < ecap) {
          out[2 * at] = i;
          out[2 * at + 1] = j;
        }
      }
      if (ambig) {
        const long long at = apre + __popcll(ba & below);
        if (at < acap) am[at] = row + j;
      }
      cnt += tot;
      acnt += atot;
      __syncthreads();
    }
  }
  if (threadIdx.x == 0) {
    ecount[L] = cnt;
    acount[L] = acnt;
  }
}

thread_local char g_err[256] = "";

md_status fail(const char* what, hipError_t e) {
  snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
  return MD_EHIP;
}

template <class T>
struct Dev {
  T* p = nullptr;
  hipError_t alloc(size_t n) { return hipMalloc((void**)&p, (n ? n : 1) * sizeof(T)); }
  ~Dev() {
    if (p) (void)hipFree(p);
  }
};

#define GCHK(what, x)                  \
  do {                                 \
    const hipError_t e_ = (x);         \
    if (e_ != hipSuccess) return fail(what, e_); \
  } while (0)

}  // namespace mdg

extern "C" {

const char* md_gmm_last_error(void) { return mdg::g_err; }

md_status md_gmm_nodes(int device, int n_graphs, int n, const uint64_t* seeds, const double* uniforms,
                       const double* kbar_in, double* kbar_out, double* kappa_out, double* theta_out) {
  using namespace mdg;
  if (n_graphs <= 0 || n < 2 || (seeds == nullptr && uniforms == nullptr) || !kbar_out || !kappa_out || !theta_out) {
    snprintf(g_err, sizeof(g_err), "md_gmm_nodes: bad arguments");
    return MD_EINVAL;
  }
  GCHK("hipSetDevice", hipSetDevice(device));
  const size_t gn = (size_t)n_graphs * n;
  Dev<unsigned long long> dk;
  Dev<double> du, dkb, dkbo, dka, dth;
  if (seeds) {
    GCHK("alloc", dk.alloc(n_graphs));
    GCHK("copy", hipMemcpy(dk.p, seeds, sizeof(uint64_t) * n_graphs, hipMemcpyHostToDevice));
  }
  if (uniforms) {
    GCHK("alloc", du.alloc(4 * gn));
    GCHK("copy", hipMemcpy(du.p, uniforms, sizeof(double) * 4 * gn, hipMemcpyHostToDevice));
  }
  if (kbar_in) {
    GCHK("alloc", dkb.alloc(2 * (size_t)n_graphs));
    GCHK("copy", hipMemcpy(dkb.p, kbar_in, sizeof(double) * 2 * n_graphs, hipMemcpyHostToDevice));
  }
  GCHK("alloc", dkbo.alloc(2 * (size_t)n_graphs));
  GCHK("alloc", dka.alloc(2 * gn));
  GCHK("alloc", dth.alloc(2 * gn));
  hipLaunchKernelGGL(gmm_nodes_kernel, dim3(n_graphs), dim3(NT), 0, 0, n, dk.p, du.p, dkb.p, n_graphs, dkbo.p, dka.p, dth.p);
  GCHK("gmm_nodes_kernel", hipGetLastError());
  GCHK("copy", hipMemcpy(kbar_out, dkbo.p, sizeof(double) * 2 * n_graphs, hipMemcpyDeviceToHost));
  GCHK("copy", hipMemcpy(kappa_out, dka.p, sizeof(double) * 2 * gn, hipMemcpyDeviceToHost));
  GCHK("copy", hipMemcpy(theta_out, dth.p, sizeof(double) * 2 * gn, hipMemcpyDeviceToHost));
  return MD_OK;
}

md_status md_gmm_links(int device, int n_layers, int n, const double* kappa, const double* theta, const double* mu,
                       const double* uniforms, const uint64_t* seeds, int32_t* edges_out, int64_t* edge_count,
                       int64_t edge_cap, int64_t* amb_out, int64_t* amb_count, int64_t amb_cap) {
  using namespace mdg;
  if (n_layers <= 0 || n < 2 || !kappa || !theta || !mu || (uniforms == nullptr && seeds == nullptr) || !edges_out ||
      !edge_count || edge_cap <= 0 || (uniforms != nullptr && (!amb_out || !amb_count || amb_cap <= 0)) ||
      (uniforms == nullptr && (n_layers & 1))) {
    snprintf(g_err, sizeof(g_err), "md_gmm_links: bad arguments");
    return MD_EINVAL;
  }
  GCHK("hipSetDevice", hipSetDevice(device));
  const size_t ln = (size_t)n_layers * n;
  const size_t npairs = (size_t)n * (n - 1) / 2;
  Dev<double> dka, dth, dmu, dun;
  Dev<unsigned long long> dk;
  Dev<int> de;
  Dev<long long> dec, dam, dac;
  GCHK("alloc", dka.alloc(ln));
  GCHK("alloc", dth.alloc(ln));
  GCHK("alloc", dmu.alloc(n_layers));
  GCHK("copy", hipMemcpy(dka.p, kappa, sizeof(double) * ln, hipMemcpyHostToDevice));
  GCHK("copy", hipMemcpy(dth.p, theta, sizeof(double) * ln, hipMemcpyHostToDevice));
  GCHK("copy", hipMemcpy(dmu.p, mu, sizeof(double) * n_layers, hipMemcpyHostToDevice));
  if (uniforms) {
    GCHK("alloc", dun.alloc(npairs * n_layers));
    GCHK("copy", hipMemcpy(dun.p, uniforms, sizeof(double) * npairs * n_layers, hipMemcpyHostToDevice));
  } else {
    GCHK("alloc", dk.alloc(n_layers / 2));
    GCHK("copy", hipMemcpy(dk.p, seeds, sizeof(uint64_t) * (n_layers / 2), hipMemcpyHostToDevice));
  }
  const long long acap = uniforms ? amb_cap : 1;
  GCHK("alloc", de.alloc(2 * (size_t)edge_cap * n_layers));
  GCHK("alloc", dec.alloc(n_layers));
  GCHK("alloc", dam.alloc((size_t)acap * n_layers));
  GCHK("alloc", dac.alloc(n_layers));
  hipLaunchKernelGGL(gmm_links_kernel, dim3(n_layers), dim3(NT), 0, 0, n, dka.p, dth.p, dmu.p, dun.p, dk.p, de.p, dec.p,
                     (long long)edge_cap, dam.p, dac.p, acap);
  GCHK("gmm_links_kernel", hipGetLastError());
  GCHK("copy", hipMemcpy(edge_count, dec.p, sizeof(int64_t) * n_layers, hipMemcpyDeviceToHost));
  for (int l = 0; l < n_layers; ++l) {
    if (edge_count[l] > edge_cap) {
      snprintf(g_err, sizeof(g_err), "md_gmm_links: layer %d has %lld edges, capacity %lld", l, (long long)edge_count[l],
               (long long)edge_cap);
      return MD_EINVAL;
    }
  }
  GCHK("copy", hipMemcpy(edges_out, de.p, sizeof(int32_t) * 2 * (size_t)edge_cap * n_layers, hipMemcpyDeviceToHost));
  if (uniforms) {
    GCHK("copy", hipMemcpy(amb_count, dac.p, sizeof(int64_t) * n_layers, hipMemcpyDeviceToHost));
    for (int l = 0; l < n_layers; ++l) {
      if (amb_count[l] > amb_cap) {
        snprintf(g_err, sizeof(g_err), "md_gmm_links: layer %d has %lld ambiguous pairs, capacity %lld", l,
                 (long long)amb_count[l], (long long)amb_cap);
        return MD_EINVAL;
      }
    }
    GCHK("copy", hipMemcpy(amb_out, dam.p, sizeof(int64_t) * (size_t)amb_cap * n_layers, hipMemcpyDeviceToHost));
  } else if (amb_count) {
    for (int l = 0; l < n_layers; ++l) amb_count[l] = 0;
  }
  return MD_OK;
}

}  // extern "C"
