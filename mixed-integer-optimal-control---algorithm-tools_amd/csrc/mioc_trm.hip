// mioc_trm.hip -- the trust-region quantities around the DP, on gfx950: pred, TV_p and the step decision.
//
// Reference:
//   multi-trust.jl:117-121  int_val = Δt · Σ_{j=1..n} ∇f[:,j]'(u_old[:,j] − u[:,j])   (j in order, then ×Δt)
//   multi-trust.jl:123,126  TV_new = TV_p(u, p);  pred = int_val + β·(TV_old − TV_new)
//   multi-trust.jl:127-158  ared = J_old − J_new + β·(TV_old − TV_new);
//                           pred ≤ 0 → stop;  ared < σ·pred → halve Δ;  else accept
//   HelpFunctions.jl:251-268 TV_p(u, p) = Σ_{i=2..n} ‖u_i − u_{i−1}‖_p  (i in order; p = Inf: the max norm)
//
// One workgroup per subproblem.  The per-step terms of a chunk of steps depend only on their own step, so all
// four waves compute them into LDS; then one lane per quantity folds the chunk in the reference's sequential
// order (waves 0, 1, 2 fold int_val, TV(u_old), TV(u) concurrently).  Every sum therefore rounds exactly as the
// reference's loop does.  Terms:
//   TV, p = 1      Σ_m |d_m|                exact (integral controls)
//   TV, p = Inf    max_m |d_m|              exact
//   TV, int p ≥ 2  w[Σ_m |d_m|^p]           the host-supplied table of Julia's Float64(S)^(1/p) (MIOC_P_INTLUT)
//   TV, table      w[rank(u_{i-1})·L + rank(u_i)]   (MIOC_P_TABLE; both controls must be on the level grid)
//   int_val        ((0 + g_1 v_1) + g_2 v_2) + ...,  v = u_old − u (exact): the reference's BLAS ddot tail loop;
//                  MIOC_OPT_PRED_FMA = 1 accumulates with fma instead (an FMA-contracted BLAS build).
// The file is built with -ffp-contract=off, like the DP kernels.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mioc_internal.h"

namespace mioc {

namespace {

constexpr int kTrmThreads = 256;
constexpr int kTrmChunk = 2048;   // steps per LDS chunk: 3 x 16 KB of terms

__device__ __forceinline__ double trm_val(const TrmDev &T, int k, int j, int m, bool is_u) {
  if (!is_u) return T.uold[((size_t)k * T.nt + j) * T.M + m];
  if (T.u) return T.u[((size_t)k * T.nt + j) * T.M + m];
  return T.nuval[(size_t)T.ranks[(size_t)k * T.nt + j] * T.M + m];
}

// iterator rank of a control on the level grid, -1 when it is not an admissible tuple (k_uold_rank's lookup)
__device__ __forceinline__ int trm_rank(const TrmDev &T, const double *v) {
  if (!T.g2r) return -1;
  int g = 0, stride = 1;
  for (int m = 0; m < T.M; ++m) {
    const int q0 = T.voff[m], q1 = T.voff[m + 1];
    int q = q0;
    while (q < q1 && (double)T.vals[q] != v[m]) ++q;
    if (q == q1) return -1;
    g += (q - q0) * stride;
    stride *= q1 - q0;
  }
  return T.g2r[g];
}

// ‖b − a‖_p as TV_p's summand (HelpFunctions.jl:259-263); err bit 1: key / rank outside the weight table
__device__ double tv_term(const TrmDev &T, const double *a, const double *b, int ra, int rb, int *err) {
  if (T.p_kind == MIOC_P_TABLE) {
    if (ra < 0 || rb < 0) {
      *err |= 1;
      return 0.0;
    }
    return T.tvw[(size_t)ra * T.L + rb];
  }
  if (T.p_kind == MIOC_P_INF) {
    double mx = 0.0;
    for (int m = 0; m < T.M; ++m) mx = fmax(mx, fabs(b[m] - a[m]));
    return mx;
  }
  if (T.p_kind == MIOC_P_ONE) {
    double s = 0.0;
    for (int m = 0; m < T.M; ++m) s = s + fabs(b[m] - a[m]);
    return s;
  }
  long long key = 0;
  for (int m = 0; m < T.M; ++m) {
    const double d = fabs(b[m] - a[m]);
    if (!(d < 1048576.0)) {
      *err |= 1;
      return 0.0;
    }
    long long t = 1;
    for (int q = 0; q < T.p_int; ++q) t *= (long long)d;
    key += t;
  }
  if (key >= T.tvw_len) {
    *err |= 1;
    return 0.0;
  }
  return T.tvw[key];
}

__device__ __forceinline__ double fold(const double *x, int n, double acc) {
  int j = 0;
  for (; j + 8 <= n; j += 8) {
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = x[j + q];
#pragma unroll
    for (int q = 0; q < 8; ++q) acc = acc + v[q];
  }
  for (; j < n; ++j) acc = acc + x[j];
  return acc;
}

__global__ __launch_bounds__(kTrmThreads) void k_trm_pred(TrmDev T) {
  __shared__ double s_int[kTrmChunk], s_told[kTrmChunk], s_tnew[kTrmChunk];
  __shared__ int s_err;
  const int k = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const bool want_int = T.mode & 1, want_told = T.mode & 2, want_tnew = T.mode & 4;
  if (tid == 0) s_err = 0;
  int err = 0;
  double acc = 0.0;  // lane 0 of wave 0 / 1 / 2: int_val / TV(u_old) / TV(u)
  for (int s0 = 0; s0 < T.nt; s0 += kTrmChunk) {
    const int cnt = min(kTrmChunk, T.nt - s0);
    for (int jj = tid; jj < cnt; jj += kTrmThreads) {
      const int j = s0 + jj;
      double uo[kMaxM], uu[kMaxM], po[kMaxM], pu[kMaxM];
      for (int m = 0; m < T.M; ++m) {  // u_old is read only when a quantity needs it (mioc_tv_device has none)
        uo[m] = (want_int || want_told) ? trm_val(T, k, j, m, false) : 0.0;
        uu[m] = (want_int || want_tnew) ? trm_val(T, k, j, m, true) : 0.0;
      }
      if (want_int) {
        const double *g = T.df + ((size_t)k * T.nt + j) * T.M;
        double d = 0.0;
        for (int m = 0; m < T.M; ++m) d = T.fma ? fma(g[m], uo[m] - uu[m], d) : d + g[m] * (uo[m] - uu[m]);
        s_int[jj] = d;
      }
      if (want_told) {
        double t = 0.0;
        if (j > 0) {
          for (int m = 0; m < T.M; ++m) po[m] = trm_val(T, k, j - 1, m, false);
          const bool tab = T.p_kind == MIOC_P_TABLE;
          t = tv_term(T, po, uo, tab ? trm_rank(T, po) : 0, tab ? trm_rank(T, uo) : 0, &err);
        }
        s_told[jj] = t;
      }
      if (want_tnew) {
        double t = 0.0;
        if (j > 0) {
          for (int m = 0; m < T.M; ++m) pu[m] = trm_val(T, k, j - 1, m, true);
          int ra = 0, rb = 0;
          if (T.p_kind == MIOC_P_TABLE) {
            ra = T.u ? trm_rank(T, pu) : T.ranks[(size_t)k * T.nt + j - 1];
            rb = T.u ? trm_rank(T, uu) : T.ranks[(size_t)k * T.nt + j];
          }
          t = tv_term(T, pu, uu, ra, rb, &err);
        }
        s_tnew[jj] = t;
      }
    }
    __syncthreads();
    if (lane == 0) {
      if (wave == 0 && want_int) acc = fold(s_int, cnt, acc);
      if (wave == 1 && want_told) acc = fold(s_told, cnt, acc);
      if (wave == 2 && want_tnew) acc = fold(s_tnew, cnt, acc);
    }
    __syncthreads();
  }
  if (err) atomicOr(&s_err, err);
  // hand the three sums to wave 0 through LDS (the chunk arrays are free now)
  if (lane == 0 && wave < 3) s_int[wave] = acc;
  __syncthreads();
  if (tid == 0) {
    const double iv = s_int[0] * T.dt, to = s_int[1], tn = s_int[2];
    if (T.out_int) T.out_int[k] = iv;
    if (T.out_told) T.out_told[k] = to;
    if (T.out_tnew) T.out_tnew[k] = tn;
    if (T.out_pred) T.out_pred[k] = iv + T.beta * (to - tn);
    if (s_err) atomicOr(T.err, s_err);
  }
}

// multi-trust.jl:126-158 per subproblem: ared and the step decision (0 accept, 1 halve Δ, 2 stop)
__global__ void k_trm_decide(int K, const double *J_old, const double *J_new, const double *tv_old,
                             const double *tv_new, const double *pred, double beta, double sigma, double *ared,
                             int32_t *decision) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const double a = (J_old[k] - J_new[k]) + beta * (tv_old[k] - tv_new[k]);
  const double p = pred[k];
  if (ared) ared[k] = a;
  decision[k] = (p <= 0.0) ? 2 : (a < sigma * p) ? 1 : 0;
}

}  // namespace

hipError_t launch_trm_pred(hipStream_t s, const TrmDev &T) {
  hipLaunchKernelGGL(k_trm_pred, dim3(T.K), dim3(kTrmThreads), 0, s, T);
  return hipGetLastError();
}

hipError_t launch_trm_decide(hipStream_t s, int K, const double *J_old, const double *J_new, const double *tv_old,
                             const double *tv_new, const double *pred, double beta, double sigma, double *ared,
                             int32_t *decision) {
  hipLaunchKernelGGL(k_trm_decide, dim3((K + 255) / 256), dim3(256), 0, s, K, J_old, J_new, tv_old, tv_new, pred,
                     beta, sigma, ared, decision);
  return hipGetLastError();
}

}  // namespace mioc
