// mioc_pinf.hip -- exact p = Inf collapse of bellman_TRM! / eval_u_TRM! for gfx950.
//
// With p = Inf the reference's switching weight is (sum_m |d_m|^Inf)^(1/Inf) = x^0.0 = 1.0 for every
// pair (l, j) (HelpFunctions.jl:63-67), so K(l, j) = fl(T1(l) + β) =: K_l does not depend on j and
//     Φ_i[c, l] = min_j fl(K_l + Φ_{i+1}[c - b̃_l, j]) = fl(K_l + R_{i+1}[c - b̃_l]),
//     R_i[c]    = min_l Φ_i[c, l]    = min_b fl(Kmin_i[b] + R_{i+1}[c - b])
// because fl(x + y) is monotone non-decreasing in each argument.  Kmin_i[b] is the minimum of K_l
// over the levels of budget class b = b̃(l, i).  The whole front is therefore a function of the
// (B+1)-vector R_{i+1} and per-class minima: the DP is O(nt * (L*M + (B+1)*BW)) and never
// materialises Φ or U.  The backtrack re-derives U_i[c, l] (the FIRST rank j with
// fl(K_l + Φ_{i+1}[c', j]) == Φ_i[c, l]) from the class tables; a class where a second distinct K
// could round to the same value is resolved by an exact scan of the row (counted in nfallback).
//
// Tables per subproblem k:  kmin/k2/kfirst [nt][BW]  (terminal row i = nt-1 holds T1 minima, no β)
//                           R              [nt][RP]
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "mioc_internal.h"

namespace mioc {

__device__ __forceinline__ double p_t1(const double *nuv, const double *dfi, int M, double dt) {
  double t = 0.0;
  for (int m = 0; m < M; ++m) t = t + (dt * dfi[m]) * nuv[m];
  return t;
}
__device__ __forceinline__ int p_bt(const double *nuv, const double *uoi, int M) {
  int b = 0;
  for (int m = 0; m < M; ++m) b += (int)fabs(nuv[m] - uoi[m]);
  return b;
}
// order-preserving key for finite doubles (inputs are validated finite)
__device__ __forceinline__ uint64_t okey(double v) {
  uint64_t u = (uint64_t)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double from_okey(uint64_t k) {
  if (k == ~0ull) return INFINITY;
  uint64_t u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __longlong_as_double((long long)u);
}
__device__ __forceinline__ uint64_t jl_key2(double v) {
  if (v != v) return 0ull;
  return okey(v);
}

// ---------------------------------------------------------------------------------------------
// per-step class tables, one workgroup per (step i, subproblem k); fully parallel over steps
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pinf_prep(ProblemDev P, LevelsDev Lv, PinfDev D) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int BW = D.BW;
  uint64_t *skmin = reinterpret_cast<uint64_t *>(smem);
  uint64_t *sk2 = skmin + BW;
  int32_t *sfirst = reinterpret_cast<int32_t *>(sk2 + BW);
  const int i = blockIdx.x, k = blockIdx.y, M = P.M;
  for (int b = threadIdx.x; b < BW; b += blockDim.x) {
    skmin[b] = ~0ull;
    sk2[b] = ~0ull;
    sfirst[b] = INT_MAX;
  }
  const double *dfi = P.df + ((size_t)k * P.nt + i) * M;
  const double *uoi = P.uold + ((size_t)k * P.nt + i) * M;
  const bool term = (i == P.nt - 1);
  __syncthreads();
  for (int r = threadIdx.x; r < Lv.L; r += blockDim.x) {
    const double *nuv = Lv.nuval + (size_t)r * M;
    const int b = p_bt(nuv, uoi, M);
    if (b >= BW) continue;
    const double t1 = p_t1(nuv, dfi, M, P.dt);
    const double v = term ? t1 : t1 + Lv.beta;  // fl(T1 + β·1.0)
    atomicMin(reinterpret_cast<unsigned long long *>(&skmin[b]), (unsigned long long)okey(v));
  }
  __syncthreads();
  for (int r = threadIdx.x; r < Lv.L; r += blockDim.x) {
    const double *nuv = Lv.nuval + (size_t)r * M;
    const int b = p_bt(nuv, uoi, M);
    if (b >= BW) continue;
    const double t1 = p_t1(nuv, dfi, M, P.dt);
    const double v = term ? t1 : t1 + Lv.beta;
    const uint64_t key = okey(v);
    if (key == skmin[b])
      atomicMin(&sfirst[b], r);
    else
      atomicMin(reinterpret_cast<unsigned long long *>(&sk2[b]), (unsigned long long)key);
  }
  __syncthreads();
  const size_t row = ((size_t)k * P.nt + i) * BW;
  for (int b = threadIdx.x; b < BW; b += blockDim.x) {
    D.kmin[row + b] = from_okey(skmin[b]);
    D.k2[row + b] = from_okey(sk2[b]);
    D.kfirst[row + b] = sfirst[b] == INT_MAX ? -1 : sfirst[b];
  }
}

hipError_t launch_pinf_prep(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PinfDev &D) {
  dim3 grid(P.nt, P.K);
  size_t lds = (size_t)D.BW * 20 + 16;
  hipLaunchKernelGGL(k_pinf_prep, grid, dim3(256), lds, s, P, Lv, D);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// sequential recursion over steps, one workgroup per subproblem; R_{i+1} and the class row live in
// LDS (double-buffered), R_i is streamed to HBM for the backtrack.
// ---------------------------------------------------------------------------------------------
constexpr int PR_MAXPF = 4;  // prefetch registers per thread: BW <= 4 * blockDim

__global__ __launch_bounds__(1024) void k_pinf_recur(ProblemDev P, PinfDev D) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int RP = P.RP, BW = D.BW, B = P.B, nt = P.nt, k = blockIdx.x;
  double *Ra = sm, *Rb = sm + RP, *Ka = Rb + RP, *Kb = Ka + BW;
  const double *kmin = D.kmin + (size_t)k * nt * BW;
  double *R = D.R + (size_t)k * nt * RP;
  for (int c = threadIdx.x; c < RP; c += blockDim.x) {
    const double v = (c < BW) ? kmin[(size_t)(nt - 1) * BW + c] : INFINITY;
    Ra[c] = v;
    Rb[c] = INFINITY;
    R[(size_t)(nt - 1) * RP + c] = v;
  }
  if (nt >= 2)
    for (int b = threadIdx.x; b < BW; b += blockDim.x) Ka[b] = kmin[(size_t)(nt - 2) * BW + b];
  __syncthreads();
  double *Rp = Ra, *Rn = Rb, *Kc = Ka, *Kn = Kb;
  for (int i = nt - 2; i >= 0; --i) {
    double pf[PR_MAXPF];
    if (i >= 1) {
#pragma unroll
      for (int q = 0; q < PR_MAXPF; ++q) {
        const int b = threadIdx.x + q * blockDim.x;
        pf[q] = (b < BW) ? kmin[(size_t)(i - 1) * BW + b] : INFINITY;
      }
    }
    for (int c = threadIdx.x; c <= B; c += blockDim.x) {
      double m = INFINITY;
      const int bl = c < BW - 1 ? c : BW - 1;
      for (int b = 0; b <= bl; ++b) m = fmin(m, Kc[b] + Rp[c - b]);
      Rn[c] = m;
      R[(size_t)i * RP + c] = m;
    }
    if (i >= 1) {
#pragma unroll
      for (int q = 0; q < PR_MAXPF; ++q) {
        const int b = threadIdx.x + q * blockDim.x;
        if (b < BW) Kn[b] = pf[q];
      }
    }
    __syncthreads();
    double *t = Rp;
    Rp = Rn;
    Rn = t;
    t = Kc;
    Kc = Kn;
    Kn = t;
  }
}

hipError_t launch_pinf_recur(hipStream_t s, const ProblemDev &P, const PinfDev &D) {
  int threads = ((P.B + 1 + 63) / 64) * 64;
  if (threads > 1024) threads = 1024;
  if (D.BW > PR_MAXPF * threads) return hipErrorInvalidValue;
  size_t lds = (size_t)(2 * P.RP + 2 * D.BW) * sizeof(double);
  hipLaunchKernelGGL(k_pinf_recur, dim3(P.K), dim3(threads), lds, s, P, D);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// backtrack start: argmin over (c <= B', l) of Φ_0[c, l] (HelpFunctions.jl:106) by exact scan
// ---------------------------------------------------------------------------------------------
struct PKey {
  uint64_t v, pos;
  double val;
  int32_t r, c;
};
__device__ __forceinline__ bool pkey_less(const PKey &a, const PKey &b) {
  return a.v < b.v || (a.v == b.v && a.pos < b.pos);
}

__global__ __launch_bounds__(1024) void k_pinf_start(ProblemDev P, LevelsDev Lv, PinfDev D, int Bu, Start *start) {
  extern __shared__ __attribute__((aligned(16))) double sR1[];
  __shared__ PKey red[16];
  const int k = blockIdx.x, M = P.M, nt = P.nt;
  const double *R1 = D.R + ((size_t)k * nt + 1) * P.RP;
  if (nt >= 2)
    for (int c = threadIdx.x; c <= Bu; c += blockDim.x) sR1[c] = R1[c];
  __syncthreads();
  const double *df0 = P.df + (size_t)k * nt * M;
  const double *uo0 = P.uold + (size_t)k * nt * M;
  PKey best;
  best.v = ~0ull;
  best.pos = ~0ull;
  best.val = INFINITY;
  best.r = -1;
  best.c = 0;
  for (int r = threadIdx.x; r < Lv.L; r += blockDim.x) {
    const double *nuv = Lv.nuval + (size_t)r * M;
    const int b = p_bt(nuv, uo0, M);
    if (b > Bu) continue;
    const double t1 = p_t1(nuv, df0, M, P.dt);
    const uint64_t g = (uint64_t)(uint32_t)Lv.gidx[r] << 32;
    if (nt == 1) {
      PKey a{jl_key2(t1), g | (uint32_t)b, t1, r, b};
      if (pkey_less(a, best)) best = a;
      continue;
    }
    const double K = t1 + Lv.beta;
    // first minimum over c for this l (strict), then compare (value, grid index, c)
    double bv = INFINITY;
    uint64_t bkey = ~0ull;
    int bc = -1;
    for (int c = b; c <= Bu; ++c) {
      const double v = K + sR1[c - b];
      const uint64_t kv = jl_key2(v);
      if (kv < bkey) {
        bkey = kv;
        bv = v;
        bc = c;
      }
    }
    if (bc >= 0) {
      PKey a{bkey, g | (uint32_t)bc, bv, r, bc};
      if (pkey_less(a, best)) best = a;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    PKey o;
    o.v = __shfl_xor(best.v, off);
    o.pos = __shfl_xor(best.pos, off);
    o.val = __shfl_xor(best.val, off);
    o.r = __shfl_xor(best.r, off);
    o.c = __shfl_xor(best.c, off);
    if (pkey_less(o, best)) best = o;
  }
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = best;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int q = 1; q < (int)(blockDim.x >> 6); ++q)
      if (pkey_less(red[q], best)) best = red[q];
    Start st;
    st.phi = best.val;
    st.c = best.c;
    st.r = best.r;
    st.status = (best.r >= 0 && best.val < INFINITY) ? MIOC_OK : MIOC_EINFEASIBLE;
    st.pad = 0;
    start[k] = st;
  }
}

hipError_t launch_pinf_start(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PinfDev &D, int Bu,
                             Start *start) {
  size_t lds = (size_t)(Bu + 1) * sizeof(double);
  hipLaunchKernelGGL(k_pinf_start, dim3(P.K), dim3(1024), lds, s, P, Lv, D, Bu, start);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// forward walk, one wave per subproblem.  State at step i: (c, l, K_l(i), b̃_l(i), Φ_i[c, l]).
// Lane b examines budget class b of step j = i+1: all levels of the class with K == Kmin give
// Φ_{i+1}[c', ·] = V_b = fl(Kmin + R_{i+2}[c' - b]), the first of them is kfirst; a level with a
// larger K gives at least fl(K2 + R_{i+2}[c' - b]).  If that second value could still satisfy
// fl(K_l + ·) == Φ_i[c, l], the step is resolved by an exact scan over all levels instead.
// R rows i+2.. are prefetched into an LDS ring (state-independent), so a step costs LDS reads,
// a few f64 ops and one wave reduction.
// ---------------------------------------------------------------------------------------------
constexpr int PW_RING = 8;
constexpr int PW_MAXRPL = 16;  // RP / 64 <= 16  (B < 1024)

__global__ __launch_bounds__(64) void k_pinf_walk(ProblemDev P, LevelsDev Lv, PinfDev D, const Start *start,
                                                  int32_t *ranks, int32_t *nfallback) {
  extern __shared__ __attribute__((aligned(16))) double ring[];
  const int k = blockIdx.x, lane = threadIdx.x, M = P.M, nt = P.nt, RP = P.RP, BW = D.BW;
  const Start st = start[k];
  if (st.status != MIOC_OK) return;
  int32_t *rk = ranks + (size_t)k * nt;
  if (lane == 0) rk[0] = st.r;
  if (nt == 1) return;
  const double *R = D.R + (size_t)k * nt * RP;
  const double *dfk = P.df + (size_t)k * nt * M;
  const double *uok = P.uold + (size_t)k * nt * M;
  const double beta = Lv.beta;
  const int rpl = RP / 64;  // R doubles per lane per row

  for (int q = 0; q < PW_RING; ++q) {
    const int row = 2 + q;
    if (row < nt)
      for (int c = lane; c < RP; c += 64) ring[(row % PW_RING) * RP + c] = R[(size_t)row * RP + c];
  }
  // state
  int r = st.r, c = st.c;
  double target = st.phi;
  double Kr, lvK;
  int br;
  {
    const double *nuv = Lv.nuval + (size_t)r * M;
    Kr = p_t1(nuv, dfk, M, P.dt) + beta;
    br = p_bt(nuv, uok, M);
  }
  (void)lvK;
  // class row prefetch (lane b; BW <= 64)
  const bool have_b = lane < BW;
  size_t crow = ((size_t)k * nt + 1) * BW + lane;
  double nkm = have_b ? D.kmin[crow] : INFINITY;
  double nk2 = have_b ? D.k2[crow] : INFINITY;
  int nkf = have_b ? D.kfirst[crow] : -1;
  __syncthreads();

  int fallbacks = 0;
  for (int i = 0; i + 1 < nt; ++i) {
    const int j = i + 1;
    const bool term = (j == nt - 1);
    // issue the ring refill for row i+2+RING (lands in the slot row i+2 occupies now)
    const int frow = i + 2 + PW_RING;
    double pf[PW_MAXRPL];
    if (frow < nt) {
#pragma unroll
      for (int q = 0; q < PW_MAXRPL; ++q)
        if (q < rpl) pf[q] = R[(size_t)frow * RP + lane + 64 * q];
    }
    const double km = nkm, k2 = nk2;
    const int kf = nkf;
    if (j + 1 < nt && have_b) {  // prefetch class row j+1
      crow += BW;
      nkm = D.kmin[crow];
      nk2 = D.k2[crow];
      nkf = D.kfirst[crow];
    }
    const int cp = c - br;
    int win = INT_MAX;
    double winV = INFINITY, winK = INFINITY;
    int winb = -1;
    bool amb = false;
    if (have_b && km < INFINITY) {
      const int b = lane;
      double x = INFINITY;
      if (term)
        x = (b == cp) ? 0.0 : INFINITY;
      else if (cp >= b)
        x = ring[((j + 1) % PW_RING) * RP + cp - b];
      if (x < INFINITY) {
        const double V = term ? km : km + x;
        if (Kr + V == target) {
          if (k2 < INFINITY) {
            const double V2 = term ? k2 : k2 + x;
            if (Kr + V2 == target) amb = true;
          }
          win = kf;
          winV = V;
          winK = km;
          winb = b;
        }
      }
    }
    // wave argmin over the first rank
    int wmin = win;
    for (int off = 32; off > 0; off >>= 1) wmin = min(wmin, __shfl_xor(wmin, off));
    const bool any_amb = __any(amb);
    if (!any_amb) {
      const unsigned long long bal = __ballot(win == wmin && wmin != INT_MAX);
      const int src = bal ? (__ffsll((long long)bal) - 1) : 0;
      winV = __shfl(winV, src);
      winK = __shfl(winK, src);
      winb = __shfl(winb, src);
      win = wmin;
    } else {
      // exact scan of row c' of Φ_{j}: first rank s with fl(K_l + Φ_j[c', s]) == Φ_i[c, l]
      ++fallbacks;
      const double *dfj = dfk + (size_t)j * M;
      const double *uoj = uok + (size_t)j * M;
      int sbest = INT_MAX;
      double sV = INFINITY, sK = INFINITY;
      int sb = -1;
      for (int s = lane; s < Lv.L; s += 64) {
        const double *nuv = Lv.nuval + (size_t)s * M;
        const int bs = p_bt(nuv, uoj, M);
        const double t1 = p_t1(nuv, dfj, M, P.dt);
        double val = INFINITY, Ks = t1;
        if (term) {
          if (bs == cp) val = t1;
        } else {
          Ks = t1 + beta;
          if (cp >= bs && bs < BW) val = Ks + ring[((j + 1) % PW_RING) * RP + cp - bs];
        }
        if (val < INFINITY && Kr + val == target && s < sbest) {
          sbest = s;
          sV = val;
          sK = Ks;
          sb = bs;
        }
      }
      int m2 = sbest;
      for (int off = 32; off > 0; off >>= 1) m2 = min(m2, __shfl_xor(m2, off));
      const unsigned long long bal = __ballot(sbest == m2 && m2 != INT_MAX);
      const int src = bal ? (__ffsll((long long)bal) - 1) : 0;
      win = m2;
      winV = __shfl(sV, src);
      winK = __shfl(sK, src);
      winb = __shfl(sb, src);
    }
    if (win == INT_MAX) {  // cannot happen for a consistent DP; mark and stop
      if (lane == 0) atomicAdd(nfallback + 1, 1);
      break;
    }
    if (lane == 0) rk[j] = win;
    r = win;
    c = cp;
    target = winV;
    Kr = winK;
    br = winb;
    // complete the ring refill
    if (frow < nt) {
#pragma unroll
      for (int q = 0; q < PW_MAXRPL; ++q)
        if (q < rpl) ring[(frow % PW_RING) * RP + lane + 64 * q] = pf[q];
    }
    __syncthreads();
  }
  (void)r;
  if (lane == 0 && fallbacks) atomicAdd(nfallback, fallbacks);
}

hipError_t launch_pinf_walk(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PinfDev &D,
                            const Start *start, int32_t *ranks, int32_t *nfallback) {
  if (D.BW > 64 || P.RP / 64 > PW_MAXRPL) return hipErrorInvalidValue;
  size_t lds = (size_t)PW_RING * P.RP * sizeof(double);
  hipLaunchKernelGGL(k_pinf_walk, dim3(P.K), dim3(64), lds, s, P, Lv, D, start, ranks, nfallback);
  return hipGetLastError();
}

}  // namespace mioc
