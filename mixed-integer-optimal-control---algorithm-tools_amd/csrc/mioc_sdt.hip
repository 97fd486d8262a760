// mioc_sdt.hip -- bellman_TRM! for p = 1 on 8^M product grids (gfx950): separable L1 distance transform
// with a certified argmin.
//
// For p = 1 the switching weight is the L1 distance d(l, j) = Σ_m |ν_lm - ν_jm| (HelpFunctions.jl:63-67).
// One source budget row c' of step i+1 holds Ψ_j = Φ_{i+1}[j, c'], and each target l of step i reads
// exactly that row (HelpFunctions.jl:69-77 with b = c'):
//     out(l) = min_j R(l, j),        R(l, j) = fl(fl(T1_l + fl(β·d(l,j))) + Ψ_j),
// U(l) = the first (lowest-rank) j attaining it (the reference's strict `>`, :73).
//
// In real arithmetic min_j (Ψ_j + β·d(l,j)) is an L1 distance transform, separable over the grid
// dimensions: M one-dimensional passes, each a forward and a backward sweep along the 8 levels of one
// dimension.  The transform runs in exact fixed-point arithmetic inside one binade of doubles:
//   - each finite Ψ_j becomes V_j = base + (Ψ_j - Ψmin)/β, truncated to the grid g = 2^13 ulp(base), with
//     the source rank j in the 12 low mantissa bits (the payload) and bit 12 as the "near tie" flag;
//   - a unit step costs exactly 1.0 (a multiple of g), so every sum is exact and keeps its payload, and
//     v_min_f64 carries the winner's rank through every pass for free;
//   - every merge of two disjoint candidate sets whose values differ by <= tol sets the flag.
// Invariant: an unflagged result's rank j* beats every other source by more than tol in the exact
// fixed-point values.  tol covers twice the stamping error (< g) plus twice the reference's own rounding
// error (<= 4u·|T1 + β·d + Ψ|), so then R(l, j) > R(l, j*) for all j != j*: j* is the reference's unique
// argmin and out(l) = R(l, j*), computed with the reference's expression.  Flagged targets (near ties),
// rows with very few targets and rows whose scale does not fit the binade are resolved by an exact scan
// of the reference loop.  Results are bit-identical to the reference in every case.
//
// Layout: the staging layout of the pyramid (mioc_pyramid.hip): S_i[c'][pos_i(l)] = Φ_i[l, c' + b̃_l(i)]
// (+Inf where c' + b̃_l > B) in the sphere order of u_old(i), UU_i[c'][l] = U_i[l, c' + b̃_l(i)] (uint16
// rank, natural order).  One workgroup of L/8 threads per source row; every pass gives each thread one
// line of 8 values.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mioc_internal.h"

namespace mioc {

constexpr int SD_RB = 12;                // payload rank bits (L <= 4096)
constexpr int SD_FLAG = 1 << SD_RB;      // near-tie flag (payload bit 12)
constexpr int SD_PAY = 2 * SD_FLAG - 1;  // payload mask: 13 low mantissa bits
constexpr int SD_COOP = 8;               // listed targets up to this many: whole-workgroup scans, else one wave each
constexpr int SD_FEW = 4;                // rows with at most this many targets go straight to the exact scan

// v_min_f64 without llvm.minnum's canonicalising v_max_f64 x,x on every operand (inputs are finite or +Inf)
__device__ __forceinline__ double sd_min(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// merge two disjoint candidate sets (their minima a, b): the smaller keeps its payload; a near tie sets
// the flag.  |a - b| is exact (one binade), +Inf - +Inf is NaN and never flags.
__device__ __forceinline__ double sd_merge(double a, double b, double tol) {
  const double m = sd_min(a, b);
  const bool close = fabs(a - b) <= tol;
  return __hiloint2double(__double2hiint(m), __double2loint(m) | (close ? SD_FLAG : 0));
}

// LDS position of rank r (3 bits per dimension): XOR swizzle so that each 32-lane half of a pass reads
// 32 distinct 8-byte bank slots in every pass: slot = (x0 ^ x1) + 8·((x1 ^ x2) & 3)
__device__ __forceinline__ int sd_swz(int r) { return r ^ ((r >> 3) & 7) ^ (((r >> 6) & 3) << 3); }

// rank of element x of line q in the pass over dimension m (q enumerates the other coordinates, lowest
// dimension fastest)
__device__ __forceinline__ int sd_rank(int q, int m, int x) {
  const int lo = q & ((1 << (3 * m)) - 1);
  return lo | (x << (3 * m)) | ((q >> (3 * m)) << (3 * (m + 1)));
}

// Exact scan of the listed targets: the reference loop (HelpFunctions.jl:60-77) for one cell each.
// COOP: the whole workgroup scans one target at a time (thread t: sources t + T·s, ascending), then a
// (value, rank) minimum, ties to the lower rank.  Otherwise one wave per target (lane: sources
// lane + 64·t).  Writes U (finite minimum) and the value (+Inf if none) into outnat.
template <int M, bool COOP>
__device__ __forceinline__ void sd_scan(const uint16_t *list, int nl, const double *psi, const double *a,
                                        const int *base, double beta, uint16_t *UU, double *outnat, double *redv,
                                        int *redj) {
  constexpr int L = 1 << (3 * M), T = L / 8, NW = T / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  auto target = [&](int r, int *xl) {
    double t1 = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      xl[m] = (r >> (3 * m)) & 7;
      t1 = t1 + a[m] * (double)(base[m] + xl[m]);  // ((0 + (Δt·df_1)·ν_1) + ...), HelpFunctions.jl:52-57
    }
    return t1;
  };
  auto wave_min = [&](double &bv, int &bj) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double ov = __shfl_xor(bv, off);
      const int oj = __shfl_xor(bj, off);
      if (oj >= 0 && (bj < 0 || ov < bv || (ov == bv && oj < bj))) {
        bv = ov;
        bj = oj;
      }
    }
  };
  if constexpr (COOP) {
    for (int e = 0; e < nl; ++e) {
      const int r = list[e];
      int xl[M];
      const double t1 = target(r, xl);
      unsigned dpre = 0;
#pragma unroll
      for (int m = 0; m < M - 1; ++m) dpre = __sad((tid >> (3 * m)) & 7, xl[m], dpre);
      double bv = INFINITY;
      int bj = -1;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int j = tid + T * s;
        const double val = (t1 + beta * (double)__sad(s, xl[M - 1], dpre)) + psi[j];
        if (val < bv) {
          bv = val;
          bj = j;
        }
      }
      wave_min(bv, bj);
      if (lane == 0) {
        redv[e * NW + w] = bv;
        redj[e * NW + w] = bj;
      }
    }
    __syncthreads();
    if (tid < nl) {
      double bv = INFINITY;
      int bj = -1;
      for (int q = 0; q < NW; ++q) {
        const double ov = redv[tid * NW + q];
        const int oj = redj[tid * NW + q];
        if (oj >= 0 && (bj < 0 || ov < bv || (ov == bv && oj < bj))) {
          bv = ov;
          bj = oj;
        }
      }
      const int r = list[tid];
      if (bj >= 0) UU[r] = (uint16_t)bj;
      outnat[r] = bj >= 0 ? bv : INFINITY;
    }
  } else {
    for (int e = w; e < nl; e += NW) {
      const int r = list[e];
      int xl[M];
      const double t1 = target(r, xl);
      double bv = INFINITY;
      int bj = -1;
      for (int t = 0; t < L / 64; ++t) {
        const int j = lane + 64 * t;
        unsigned d = 0;
#pragma unroll
        for (int m = 0; m < M; ++m) d = __sad((j >> (3 * m)) & 7, xl[m], d);
        const double val = (t1 + beta * (double)d) + psi[j];
        if (val < bv) {
          bv = val;
          bj = j;
        }
      }
      wave_min(bv, bj);
      if (lane == 0) {
        if (bj >= 0) UU[r] = (uint16_t)bj;
        outnat[r] = bj >= 0 ? bv : INFINITY;
      }
    }
  }
}

template <int M>
__global__ __launch_bounds__(1 << (3 * M - 3)) void k_sdt_step(ProblemDev P, LevelsDev Lv, PyrGeom G, int i,
                                                           const uint32_t *__restrict__ perm_all,
                                                           const double *__restrict__ Sin_all,
                                                           double *__restrict__ Sout_all,
                                                           uint16_t *__restrict__ UU_all, size_t s_stride,
                                                           size_t uu_stride_k, int32_t *__restrict__ counters) {
  constexpr int L = 1 << (3 * M), T = L / 8, NW = T / 64, Smax = 7 * M;
  extern __shared__ __attribute__((aligned(16))) unsigned char sds[];
  double *psi = reinterpret_cast<double *>(sds);      // [L] Ψ_j by rank
  double *dtv = psi + L;                              // [L] transform values (swizzled), then outputs (natural)
  uint16_t *list = reinterpret_cast<uint16_t *>(dtv + L);  // [L] targets for the exact scan
  __shared__ double redv[SD_COOP * NW];
  __shared__ int redj[SD_COOP * NW];
  __shared__ double rmn[NW], rmx[NW];
  __shared__ int rnv[NW];
  __shared__ int nlist;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int k = blockIdx.y, cp = (int)blockIdx.x, B = P.B;
  const double beta = Lv.beta;
  const double *Sin = Sin_all + (size_t)k * s_stride;
  double *Sout = Sout_all + (size_t)k * s_stride + (size_t)cp * L;
  uint16_t *UU = UU_all + (size_t)k * uu_stride_k + (size_t)i * ((size_t)(B + 1) * L) + (size_t)cp * L;
  const double *dfi = P.df + ((size_t)k * P.nt + i) * M;
  const double *uoi = P.uold + ((size_t)k * P.nt + i) * M;
  const uint32_t *pin = perm_all + ((size_t)k * P.nt + i + 1) * L;
  const uint32_t *pout = perm_all + ((size_t)k * P.nt + i) * L;

  // ---- sources: Ψ_j = Φ_{i+1}[j, c'] = S_{i+1}[c' - b̃_j(i+1)][pos_{i+1}(j)], read position-coalesced ----
  uint32_t ein[8], eout[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    ein[q] = pin[tid + T * q];
    eout[q] = pout[tid + T * q];
  }
  double v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int row = cp - (int)(ein[q] >> 16);
    v[q] = row >= 0 ? Sin[(size_t)row * L + tid + T * q] : INFINITY;
  }
  if (tid == 0) nlist = 0;
  double pmn = INFINITY, pmx = -INFINITY;
  int nv = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    psi[ein[q] & 0xFFFFu] = v[q];
    if (v[q] < INFINITY) {
      pmn = fmin(pmn, v[q]);
      pmx = fmax(pmx, v[q]);
    }
    nv += (int)(eout[q] >> 16) <= B - cp;  // target inside the trust region: c' + b̃_l(i) <= B
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    pmn = fmin(pmn, __shfl_xor(pmn, off));
    pmx = fmax(pmx, __shfl_xor(pmx, off));
    nv += __shfl_xor(nv, off);
  }
  if (lane == 0) {
    rmn[w] = pmn;
    rmx[w] = pmx;
    rnv[w] = nv;
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    pmn = fmin(pmn, rmn[q]);
    pmx = fmax(pmx, rmx[q]);
  }
  nv = 0;
#pragma unroll
  for (int q = 0; q < NW; ++q) nv += rnv[q];
  if (nv == 0 || !(pmn < INFINITY)) {  // no target in the trust region, or nothing reachable
#pragma unroll
    for (int q = 0; q < 8; ++q) Sout[tid + T * q] = INFINITY;
    return;
  }

  // ---- the binade: values base + (Ψ - Ψmin)/β + d lie in [base, 2·base), grid g = 2^13 ulp ----------
  double a[M];
  int lb[M], uo[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    a[m] = P.dt * dfi[m];
    lb[m] = G.base[m];
    uo[m] = (int)uoi[m];
  }
  const double inv = 1.0 / beta;
  const double rs = (pmx - pmn) * inv + (double)Smax;  // scaled range of every transform value
  const bool scale_ok = rs < 0x1p36;                   // else unit steps are not on the grid: exact scans
  const int E = ilogb(fmin(rs, 0x1p36) * (1.0 + 0x1p-20) + 1.0) + 2;  // 2^E >= 2·rs
  const double base = ldexp(1.0, E), g = ldexp(1.0, E - 39);
  double qmax = beta * (double)Smax + fmax(fabs(pmn), fabs(pmx));  // >= |T1 + β·d + Ψ| for every candidate
#pragma unroll
  for (int m = 0; m < M; ++m) qmax += fabs(a[m]) * (double)max(abs(lb[m]), abs(lb[m] + 7));
  // 2 × stamping error (< g) + 2 × the reference's rounding (<= 4u·qmax per candidate), in units of β
  const double tol = 3.0 * g + 0x1p-49 * qmax * inv;
  const bool direct = nv <= SD_FEW || !scale_ok || !(tol < base * 0x1p-20);

  if (!direct) {
    // ---- stamp: V_j = trunc_g(base + (Ψ_j - Ψmin)/β) | j --------------------------------------------
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int j = (int)(ein[q] & 0xFFFFu);
      double V = INFINITY;
      if (v[q] < INFINITY) {
        const double y = (v[q] - pmn) * inv + base;
        V = __hiloint2double(__double2hiint(y), (__double2loint(y) & ~SD_PAY) | j);
      }
      dtv[sd_swz(j)] = V;
    }
    __syncthreads();
  }

  // ---- M passes: forward and backward sweep along the 8 levels of one dimension, unit step 1.0 -------
  double o[8];
  if (!direct) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      int pos[8];
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        pos[x] = sd_swz(sd_rank(tid, m, x));
        o[x] = dtv[pos[x]];
      }
      double lf[8], rb[8];
      lf[0] = o[0];
#pragma unroll
      for (int x = 1; x < 8; ++x) lf[x] = sd_merge(o[x], lf[x - 1] + 1.0, tol);
      rb[7] = o[7];
#pragma unroll
      for (int x = 6; x >= 1; --x) rb[x] = sd_merge(o[x], rb[x + 1] + 1.0, tol);
      o[7] = lf[7];
#pragma unroll
      for (int x = 0; x < 7; ++x) o[x] = sd_merge(lf[x], rb[x + 1] + 1.0, tol);
      if (m + 1 < M) {
#pragma unroll
        for (int x = 0; x < 8; ++x) dtv[pos[x]] = o[x];
      }
      __syncthreads();  // last pass: every read of dtv is done before it becomes the output buffer
    }
  }

  // ---- targets of this thread: ranks tid | x << 3(M-1) ----------------------------------------------
  double pre = 0.0;
  int bpre = 0;
  int xt[M];
#pragma unroll
  for (int m = 0; m < M - 1; ++m) {
    xt[m] = (tid >> (3 * m)) & 7;
    const int nu = lb[m] + xt[m];
    pre = pre + a[m] * (double)nu;
    bpre += abs(nu - uo[m]);
  }
  unsigned listed = 0;
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    const int r = tid | (x << (3 * (M - 1)));
    const int nu = lb[M - 1] + x;
    const bool valid = bpre + abs(nu - uo[M - 1]) <= B - cp;
    double ov = INFINITY;
    if (direct) {
      listed |= (unsigned)valid << x;
    } else if (valid && o[x] < INFINITY) {
      const int pl = __double2loint(o[x]);
      if (pl & SD_FLAG) {
        listed |= 1u << x;
      } else {
        const int j = pl & (SD_FLAG - 1);
        unsigned d = __sad(x, (j >> (3 * (M - 1))) & 7, 0u);
#pragma unroll
        for (int m = 0; m < M - 1; ++m) d = __sad((j >> (3 * m)) & 7, xt[m], d);
        const double t1 = pre + a[M - 1] * (double)nu;
        ov = (t1 + beta * (double)d) + psi[j];  // R(l, j*), HelpFunctions.jl:63-71
        UU[r] = (uint16_t)j;
      }
    }
    dtv[r] = ov;
  }
  if (listed) {
    const int at = atomicAdd(&nlist, __popc(listed));
    int e = at;
#pragma unroll
    for (int x = 0; x < 8; ++x)
      if (listed >> x & 1) list[e++] = (uint16_t)(tid | (x << (3 * (M - 1))));
  }
  __syncthreads();
  const int nl = nlist;
  if (nl) {
    if (nl <= SD_COOP)
      sd_scan<M, true>(list, nl, psi, a, lb, beta, UU, dtv, redv, redj);
    else
      sd_scan<M, false>(list, nl, psi, a, lb, beta, UU, dtv, redv, redj);
    __syncthreads();
    if (tid == 0) atomicAdd(&counters[direct ? 1 : 0], nl);
  }
  // ---- Φ_i row c' in the sphere order of u_old(i), position-coalesced -----------------------------
#pragma unroll
  for (int q = 0; q < 8; ++q) Sout[tid + T * q] = dtv[eout[q] & 0xFFFFu];
}

size_t sdt_lds_bytes(const PyrGeom &G) {
  const size_t L = (size_t)1 << (3 * G.M);
  return L * (2 * sizeof(double) + sizeof(uint16_t));
}

bool sdt_supported(const PyrGeom &G) {
  if (G.M != 3 && G.M != 4) return false;
  for (int m = 0; m < G.M; ++m)
    if (G.n[m] != 8) return false;
  return true;
}

hipError_t launch_sdt_step(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G, int i,
                           const uint32_t *perm, const double *Sin, double *Sout, uint16_t *UU, size_t s_stride,
                           size_t uu_stride_k, int32_t *counters) {
  if (!sdt_supported(G)) return hipErrorInvalidValue;
  const dim3 grid(P.B + 1, P.K);
  const size_t lds = sdt_lds_bytes(G);
  if (G.M == 4)
    hipLaunchKernelGGL(k_sdt_step<4>, grid, dim3(512), lds, s, P, Lv, G, i, perm, Sin, Sout, UU, s_stride,
                       uu_stride_k, counters);
  else
    hipLaunchKernelGGL(k_sdt_step<3>, grid, dim3(64), lds, s, P, Lv, G, i, perm, Sin, Sout, UU, s_stride,
                       uu_stride_k, counters);
  return hipGetLastError();
}

}  // namespace mioc
