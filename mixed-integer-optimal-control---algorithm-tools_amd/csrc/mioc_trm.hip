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

#include <algorithm>

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
  if (gate_closed(T.gate)) return;
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

// ---- device-resident TRM control (multi-trust.jl:92-163) for K restarts ------------------------------------
// State block (TrmState, laid out by trm_state_layout): the gate word (any restart inside its inner loop: the
// gated kernels of an inner iteration return at once while it is 0), the any-active word (any restart not
// stopped), the copy word (any trial to copy), then per restart Δᵏ, TV_old, k, flags, outer iterations.
constexpr int TRM_INNER = 1, TRM_HALVED = 2, TRM_STOP = 4, TRM_COPY_U = 8, TRM_COPY_UOLD = 16;

struct TrmState {
  int32_t *gate, *any_active, *any_copy;
  double *Dk, *tv_old;
  int32_t *k, *flags, *iters;
};
__host__ __device__ inline TrmState trm_state_layout(void *base, int K) {
  TrmState S;
  char *b = static_cast<char *>(base);
  S.gate = reinterpret_cast<int32_t *>(b);
  S.any_active = S.gate + 1;
  S.any_copy = S.gate + 2;
  S.Dk = reinterpret_cast<double *>(b + 16);
  S.tv_old = S.Dk + K;
  S.k = reinterpret_cast<int32_t *>(S.tv_old + K);
  S.flags = S.k + K;
  S.iters = S.flags + K;
  return S;
}

// block-wide OR of one flag per thread into *out (one workgroup)
__device__ __forceinline__ void trm_block_or(int v, int32_t *out) {
  __shared__ int s_or;
  if (threadIdx.x == 0) s_or = 0;
  __syncthreads();
  if (__ballot(v) && (threadIdx.x & 63) == 0) atomicOr(&s_or, 1);
  __syncthreads();
  if (threadIdx.x == 0) *out = s_or;
}

// start of an outer iteration, multi-trust.jl:99-107: TV_old = TV_p(u), Δᵏ = Δ⁰, k = 1, every restart that has not
// stopped enters its inner loop with the full budget B; the gate opens if any did
__global__ __launch_bounds__(1024) void k_trm_outer_begin(int K, TrmState S, const double *tv_u, double D0, int B,
                                                          int32_t *budgets) {
  int any = 0;
  for (int r = threadIdx.x; r < K; r += blockDim.x) {
    const int f = S.flags[r];
    const bool active = !(f & TRM_STOP);
    S.tv_old[r] = tv_u[r];
    S.Dk[r] = D0;
    S.k[r] = 1;
    S.flags[r] = active ? TRM_INNER : f & TRM_STOP;
    S.iters[r] += active ? 1 : 0;
    budgets[r] = B;
    any |= active ? 1 : 0;
  }
  trm_block_or(any, S.gate);
  if (threadIdx.x == 0) {
    *S.any_active = *S.gate;
    *S.any_copy = 0;
  }
}

// end of an inner iteration, multi-trust.jl:117-158 for every restart still inside its inner loop: pred with the
// outer iteration's TV_old, ared and the decision (the reference's expressions, as k_trm_decide), obj.x = the
// trial (copied by k_trm_copy), accept (u_old = trial, J_old = J = J_new, TV_old = TV_new), halve Δᵏ, or stop
// (J = J_old); k += 1; the next budget floor(Δᵏ/Δt) after a halving; the gate stays open while any restart is
// inside its inner loop (k <= kmax, no accept, no stop)
__global__ __launch_bounds__(1024) void k_trm_inner_end(int K, TrmState S, double beta, double sigma, int kmax,
                                                        double tau, int B, const double *int_val, const double *tv_new,
                                                        const double *J_new, double *J_old, double *J, double *tv_u,
                                                        int32_t *budgets, int32_t *decision) {
  int any_inner = 0, any_act = 0, any_cp = 0;
  for (int r = threadIdx.x; r < K; r += blockDim.x) {
    int f = S.flags[r] & ~(TRM_COPY_U | TRM_COPY_UOLD);
    if (f & TRM_INNER) {
      const double tvo = S.tv_old[r], tvn = tv_new[r];
      const double pred = int_val[r] + beta * (tvo - tvn);                 // multi-trust.jl:126
      const double ared = (J_old[r] - J_new[r]) + beta * (tvo - tvn);      // :128
      const int d = (pred <= 0.0) ? 2 : (ared < sigma * pred) ? 1 : 0;     // :130, :140
      if (decision) decision[r] = d;
      f |= TRM_COPY_U;                                                     // obj.x = the trial, accepted or not
      tv_u[r] = tvn;
      if (d == 2) {                                                        // stop, J = J_old, :130-138
        J[r] = J_old[r];
        f |= TRM_STOP;
        f &= ~TRM_INNER;
      } else if (d == 0) {                                                 // accept, :148-154
        f |= TRM_COPY_UOLD;
        J_old[r] = J_new[r];
        J[r] = J_new[r];
        S.tv_old[r] = tvn;
        f &= ~TRM_INNER;
      } else {                                                             // halve Δᵏ, :140-146
        S.Dk[r] = S.Dk[r] / 2;
        f |= TRM_HALVED;
      }
      const int k = S.k[r] + 1;
      S.k[r] = k;
      if (k > kmax) f &= ~TRM_INNER;
      budgets[r] = (f & TRM_HALVED) ? (int)floor(S.Dk[r] / tau) : B;      // B_new = floor(Δᵏ/Δt), :109
      any_cp = 1;
    } else if (decision) {
      decision[r] = -1;
    }
    S.flags[r] = f;
    any_inner |= (f & TRM_INNER) ? 1 : 0;
    any_act |= (f & TRM_STOP) ? 0 : 1;
  }
  trm_block_or(any_cp, S.any_copy);
  trm_block_or(any_act, S.any_active);
  trm_block_or(any_inner, S.gate);
}

// the trial into u (every restart of the inner iteration) and into u_old (accepted ones); grid (chunks, K)
__global__ __launch_bounds__(256) void k_trm_copy(TrmState S, size_t n, const double *trial, double *u, double *u_old) {
  if (*S.any_copy == 0) return;
  const int r = blockIdx.y;
  const int f = S.flags[r];
  if (!(f & (TRM_COPY_U | TRM_COPY_UOLD))) return;
  const size_t base = (size_t)r * n;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (size_t)gridDim.x * blockDim.x) {
    const double v = trial[base + e];
    if (f & TRM_COPY_U) u[base + e] = v;
    if (f & TRM_COPY_UOLD) u_old[base + e] = v;
  }
}

}  // namespace

size_t trm_state_bytes(int K) { return 16 + (size_t)K * (2 * sizeof(double) + 3 * sizeof(int32_t)); }

hipError_t launch_trm_outer_begin(hipStream_t s, int K, void *state, const double *tv_u, double D0, int B,
                                  int32_t *budgets) {
  hipLaunchKernelGGL(k_trm_outer_begin, dim3(1), dim3(1024), 0, s, K, trm_state_layout(state, K), tv_u, D0, B,
                     budgets);
  return hipGetLastError();
}

hipError_t launch_trm_inner_end(hipStream_t s, int K, void *state, double beta, double sigma, int kmax, double tau,
                                int B, const double *int_val, const double *tv_new, const double *J_new,
                                double *J_old, double *J, double *tv_u, int32_t *budgets, int32_t *decision,
                                size_t n, const double *trial, double *u, double *u_old) {
  const TrmState S = trm_state_layout(state, K);
  hipLaunchKernelGGL(k_trm_inner_end, dim3(1), dim3(1024), 0, s, K, S, beta, sigma, kmax, tau, B, int_val, tv_new,
                     J_new, J_old, J, tv_u, budgets, decision);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const unsigned chunks = (unsigned)std::min<size_t>((n + 255) / 256, 64);
  hipLaunchKernelGGL(k_trm_copy, dim3(chunks, (unsigned)K), dim3(256), 0, s, S, n, trial, u, u_old);
  return hipGetLastError();
}

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
