// mioc_pyramid.hip -- exact L1-ball pyramid sweep of bellman_TRM! for p = 1 on product grids (gfx950).
//
// For p = 1 the switching weight is the L1 distance d(l, j) = sum_m |ν_lm - ν_jm| (HelpFunctions.jl:63-67),
// so for one source budget row c' with values Ψ_j = Φ_{i+1}[j, c'] and one target level l
//     out(l) = min_j fl(K_l(d(l,j)) + Ψ_j),        K_l(S) = fl(T1_l + fl(β·S)),
// and because fl(K + x) is monotone in both arguments this equals
//     out(l) = min_S fl(K_l(S) + BM_S(l)),         BM_S(l) = min over the L1 ball of radius S around l of Ψ.
// BM_{S+1} is BM_S dilated by the unit cross (levels are consecutive integers, so value distance = index
// distance): 2M neighbour minima per grid point per level instead of L candidates per target.
//
// Argmin (the reference's strict `>` over iterator order, HelpFunctions.jl:73): in a "clean" row -- every
// pair of finite Ψ values more than δ apart, δ >= ulp of any candidate value -- the only j with
// fl(K_l(d) + Ψ_j) == out(l) is the unique j holding BM at the first winning level (a value hash maps it
// back to its rank).  A target whose minimum is reached at two levels, and every dirty row, is resolved by
// the exact brute-force scan instead, so results are bit-identical to the reference in every case.
//
// Layout ("staging"): S_i[c'][l] = Φ_i[l, c' + b̃_l(i)] (source row major, +Inf where c'+b̃_l > B);
// UU_i[c'][l] = U_i[l, c' + b̃_l(i)] (uint16 rank).  One workgroup per source row; rows are dispatched
// from c' = B downwards so the cheap high rows (few valid targets) never delay a full pyramid row.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "mioc_internal.h"

namespace mioc {

constexpr int PY_T = 512;          // threads per workgroup: one grid column (dim-0 run) per thread
constexpr int PY_CPT = 1;          // grid columns per thread
constexpr int PY_HBITS = 13;
constexpr int PY_HSIZE = 1 << PY_HBITS;
constexpr long long PY_EMPTY = 0x7FFFFFFFFFFFFFFFLL;

// v_min_f64 without the sNaN-quieting v_max_f64 x,x that llvm.minnum puts in front of every operand
// not known to be canonical (inputs here are finite or +Inf, never NaN)
__device__ __forceinline__ double vmin(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Diagnostic build only (make stamps -> libmioc_stamps.so): per-workgroup phase clocks of the last launch.
#ifdef MIOC_STAMPS
__device__ unsigned long long g_pyr_stamps[4096][8];
#define PY_STAMP(k)                                                                          \
  do {                                                                                       \
    if (threadIdx.x == 0) g_pyr_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memtime();         \
  } while (0)
#else
#define PY_STAMP(k) \
  do {              \
  } while (0)
#endif

struct PyrView {
  double *lvl;        // [2][ncol][8]
  long long *hkey;    // [PY_HSIZE]
  uint16_t *hval;     // [PY_HSIZE]
};

__device__ __forceinline__ unsigned py_hash(long long q) {
  return (unsigned)(((unsigned long long)q * 0x9E3779B97F4A7C15ull) >> (64 - PY_HBITS));
}

// returns true if q was already present (a duplicate bucket)
__device__ __forceinline__ bool py_insert(PyrView V, long long q, int rank) {
  unsigned s = py_hash(q);
  for (;;) {
    unsigned long long old = atomicCAS(reinterpret_cast<unsigned long long *>(&V.hkey[s]),
                                       (unsigned long long)PY_EMPTY, (unsigned long long)q);
    if (old == (unsigned long long)PY_EMPTY) {
      V.hval[s] = (uint16_t)rank;
      return false;
    }
    if ((long long)old == q) return true;
    s = (s + 1) & (PY_HSIZE - 1);
  }
}

__device__ __forceinline__ int py_find(PyrView V, long long q) {
  unsigned s = py_hash(q);
  for (;;) {
    const long long k = V.hkey[s];
    if (k == q) return V.hval[s];
    if (k == PY_EMPTY) return -1;
    s = (s + 1) & (PY_HSIZE - 1);
  }
}

__device__ __forceinline__ double py_block_max(double v, double *red) {
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = red[0];
  for (int w = 1; w < PY_T / 64; ++w) r = fmax(r, red[w]);
  __syncthreads();
  return r;
}
__device__ __forceinline__ double py_block_min(double v, double *red) {
  for (int off = 32; off > 0; off >>= 1) v = fmin(v, __shfl_xor(v, off));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double r = red[0];
  for (int w = 1; w < PY_T / 64; ++w) r = fmin(r, red[w]);
  __syncthreads();
  return r;
}

struct PyrDims {  // geometry copied by value into registers (never escapes to memory)
  int n[kMaxM];
  int base[kMaxM];
};

template <int M>
__device__ __forceinline__ int py_dist(const PyrDims &D, int a, int b) {
  int d = 0;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int xa = a % D.n[m], xb = b % D.n[m];
    d += xa > xb ? xa - xb : xb - xa;
    a /= D.n[m];
    b /= D.n[m];
  }
  return d;
}

// Ψ_j = Φ_{i+1}[j, c'] read back from the staging buffer of step i+1
template <int M>
__device__ __forceinline__ double py_psi(const PyrDims &D, const double *Sin, const double *uo1, int L, int cp,
                                         int j) {
  int b = 0, g = j;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int x = g % D.n[m];
    g /= D.n[m];
    b += (int)fabs((double)(D.base[m] + x) - uo1[m]);
  }
  return cp >= b ? Sin[(size_t)(cp - b) * L + j] : INFINITY;
}

// exact first-index argmin for one target: the reference loop (HelpFunctions.jl:60-77) for one cell
template <int M>
__device__ __forceinline__ void py_brute_target(const PyrDims &D, const double *costlut, double T1l, int l,
                                                const double *psi_lds, const double *Sin, const double *uo1, int L,
                                                int cp, double *best, int *arg) {
  double bv = INFINITY;
  int ba = -1;
  for (int j = 0; j < L; ++j) {
    const double v = psi_lds ? psi_lds[j] : py_psi<M>(D, Sin, uo1, L, cp, j);
    if (!(v < INFINITY)) continue;
    const double val = (T1l + costlut[py_dist<M>(D, l, j)]) + v;
    if (val < bv) {
      bv = val;
      ba = j;
    }
  }
  *best = bv;
  *arg = ba;
}

// A column (N0 doubles = N0/2 16-byte chunks) is stored with its chunks XOR-swizzled by the column's
// position inside a 256-byte LDS row, so the 16 lanes of every ds_read_b128 / ds_write_b128 lane group
// (consecutive columns) hit 16 distinct 4-bank slots: conflict-free (64-byte stride alone is 4-way).
template <int N0>
__device__ __forceinline__ int col_swz(int col) {
  return (col / (32 / N0)) & (N0 / 2 - 1);
}
template <int N0>
__device__ __forceinline__ void col_store(double *buf, int col, const double *v) {
  double2 *base = reinterpret_cast<double2 *>(buf + (size_t)col * N0);
  const int sw = col_swz<N0>(col);
#pragma unroll
  for (int c = 0; c < N0 / 2; ++c) base[c ^ sw] = make_double2(v[2 * c], v[2 * c + 1]);
}
template <int N0>
__device__ __forceinline__ void col_min(const double *buf, int col, double *acc) {
  const double2 *base = reinterpret_cast<const double2 *>(buf + (size_t)col * N0);
  const int sw = col_swz<N0>(col);
#pragma unroll
  for (int c = 0; c < N0 / 2; ++c) {
    const double2 t = base[c ^ sw];
    acc[2 * c] = vmin(acc[2 * c], t.x);
    acc[2 * c + 1] = vmin(acc[2 * c + 1], t.y);
  }
}

template <int M, int N0>
__global__ __launch_bounds__(PY_T) void k_pyr_step(ProblemDev P, LevelsDev Lv, PyrGeom G, int i,
                                                   const double *__restrict__ Sin_all, double *__restrict__ Sout_all,
                                                   uint16_t *__restrict__ UU_all, size_t s_stride, size_t uu_stride_k,
                                                   int32_t *__restrict__ counters) {
  static_assert(N0 == 4 || N0 == 8, "column length");
  constexpr int CW = N0;                 // doubles per column in LDS
  constexpr int NP = PY_CPT * N0;        // points per thread
  extern __shared__ __attribute__((aligned(16))) unsigned char pys[];
  __shared__ double red[PY_T / 64];
  __shared__ double sc[64];              // costlut (β·S), S <= Smax < 64
  __shared__ int vote[2][PY_T / 64];     // per-wave early-exit votes, double-buffered by level parity
  __shared__ int nlist;
  PyrDims D;
#pragma unroll
  for (int m = 0; m < kMaxM; ++m) {
    D.n[m] = G.n[m];
    D.base[m] = G.base[m];
  }
  const int k = blockIdx.y;
  const int L = Lv.L, B = P.B, tid = threadIdx.x, ncol = G.ncol, Smax = G.Smax;
  const int cp = B - (int)blockIdx.x;  // source row: high rows first
  const double *Sin = Sin_all + (size_t)k * s_stride;
  double *Sout = Sout_all + (size_t)k * s_stride + (size_t)cp * L;
  uint16_t *UU = UU_all + (size_t)k * uu_stride_k + (size_t)i * ((size_t)(B + 1) * L) + (size_t)cp * L;
  const double *dfi = P.df + ((size_t)k * P.nt + i) * M;
  const double *uoi = P.uold + ((size_t)k * P.nt + i) * M;
  const double *uo1 = P.uold + ((size_t)k * P.nt + i + 1) * M;
  PyrView V;
  V.lvl = reinterpret_cast<double *>(pys);
  V.hkey = reinterpret_cast<long long *>(pys + (size_t)2 * ncol * CW * sizeof(double));
  V.hval = reinterpret_cast<uint16_t *>(V.hkey + PY_HSIZE);
  const double *costlut = Lv.costlut;
  PY_STAMP(0);
  if (tid <= Smax) sc[tid] = costlut[tid];
  double a[M], uo0[M], uo1v[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    a[m] = P.dt * dfi[m];
    uo0[m] = uoi[m];
    uo1v[m] = uo1[m];
  }

  // ---- own points: targets (T1, validity) and sources (Ψ) -------------------------------------
  // invalid targets carry T1 = +Inf and best = -Inf, so the level loop needs no branches
  double cur[NP], T1[NP], best[NP], bmb[NP];
  unsigned valid = 0, multi = 0;
  int nbm[PY_CPT];                       // per column: has lower / upper neighbour in dim m (bits 2m, 2m+1)
  double psimax = 0.0, psimin = INFINITY;
#pragma unroll
  for (int c2 = 0; c2 < PY_CPT; ++c2) {
    const int col = tid + PY_T * c2;
    int msk = 0, cc = col;
#pragma unroll
    for (int m = 1; m < M; ++m) {
      const int xm = cc % D.n[m];
      cc /= D.n[m];
      msk |= (xm > 0 ? 1 : 0) << (2 * m);
      msk |= (xm + 1 < D.n[m] ? 1 : 0) << (2 * m + 1);
    }
    nbm[c2] = col < ncol ? msk : 0;
  }
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int col = tid + PY_T * (q / N0), x0 = q % N0;
    cur[q] = INFINITY;
    T1[q] = INFINITY;
    best[q] = -INFINITY;
    bmb[q] = INFINITY;
    if (col < ncol) {
      int g = x0 + N0 * col;
      double t = 0.0;
      int bl = 0, bs = 0;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int x = g % D.n[m];
        g /= D.n[m];
        const double nu = (double)(D.base[m] + x);
        t = t + a[m] * nu;  // ((0 + (Δt*df_1)*ν_1) + ...), HelpFunctions.jl:52-57
        bl += (int)fabs(nu - uo0[m]);
        bs += (int)fabs(nu - uo1v[m]);
      }
      if (bl <= B - cp) {
        valid |= 1u << q;
        T1[q] = t;
        best[q] = INFINITY;
      }
      const double v = cp >= bs ? Sin[(size_t)(cp - bs) * L + x0 + N0 * col] : INFINITY;
      cur[q] = v;
      if (v < INFINITY) {
        psimax = fmax(psimax, fabs(v));
        psimin = fmin(psimin, v);
      }
    }
  }
  const int any_valid = __syncthreads_or(valid != 0);
  if (!any_valid) {  // no target of this row lies inside the trust region
    for (int g = tid; g < L; g += PY_T) Sout[g] = INFINITY;
    return;
  }
  PY_STAMP(1);
  const double Pmax = py_block_max(psimax, red);
  const double Rmin = py_block_min(psimin, red);
  if (!(Rmin < INFINITY)) {  // nothing is reachable from this source row
    for (int g = tid; g < L; g += PY_T) Sout[g] = INFINITY;
    return;
  }
  // δ >= 2 ulp of any candidate fl(K + Ψ):  |K| <= sum_m |Δt·df_m|·max|ν_m| + β·Smax
  double kb = sc[Smax];
#pragma unroll
  for (int m = 0; m < M; ++m)
    kb += fabs(a[m]) * fmax(fabs((double)D.base[m]), fabs((double)(D.base[m] + D.n[m] - 1)));
  const double Y = (Pmax + kb) * (1.0 + 0x1p-40) + 0x1p-1000;
  const int E = ilogb(Y) + 1;                   // |y| < 2^E for every candidate y
  const double inv_delta = ldexp(1.0, 52 - E);  // δ = 2^(E-52)

  // ---- clean-row test: no two finite Ψ within δ (bucket hash: same or adjacent bucket) ---------
  PY_STAMP(2);
  for (int s2 = tid; s2 < PY_HSIZE; s2 += PY_T) V.hkey[s2] = PY_EMPTY;
  if (tid == 0) nlist = 0;
  __syncthreads();
  bool dirty = false;
#pragma unroll
  for (int q = 0; q < NP; ++q)
    if (cur[q] < INFINITY)
      dirty |= py_insert(V, (long long)floor(cur[q] * inv_delta), q % N0 + N0 * (tid + PY_T * (q / N0)));
  __syncthreads();
#pragma unroll
  for (int q = 0; q < NP; ++q)
    if (cur[q] < INFINITY) {
      const long long b = (long long)floor(cur[q] * inv_delta);
      dirty |= py_find(V, b - 1) >= 0 || py_find(V, b + 1) >= 0;
    }
  const int row_dirty = __syncthreads_or(dirty);
  PY_STAMP(3);

  double *lvl = V.lvl;
  if (row_dirty) {
    // exact scan of every (target, j) pair, Ψ and the target data staged in LDS
    double *psi = lvl;                                 // [L]
    double *t1s = reinterpret_cast<double *>(V.hkey);  // [L]  (the hash is no longer needed)
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const int col = tid + PY_T * (q / N0);
      if (col < ncol) {
        const int g = q % N0 + N0 * col;
        psi[g] = cur[q];
        t1s[g] = T1[q];  // +Inf marks a target outside the trust region
      }
    }
    __syncthreads();
    for (int g = tid; g < L; g += PY_T) {
      double bv = INFINITY;
      int ba = -1;
      const double t = t1s[g];
      if (t < INFINITY) py_brute_target<M>(D, sc, t, g, psi, nullptr, nullptr, L, cp, &bv, &ba);
      Sout[g] = bv;
      if (ba >= 0) UU[g] = (uint16_t)ba;
    }
    if (tid == 0) atomicAdd(&counters[0], 1);
    return;
  }

  // ---- the pyramid (branch-free level loop) ------------------------------------------------------
  int S = 0;
  for (;; ++S) {
    const double cS = sc[S];
    unsigned mlt = 0, meq = 0;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const double cand = (T1[q] + cS) + cur[q];
      const bool lt = cand < best[q];
      const bool eq = (cand == best[q]) & (cand < INFINITY);
      best[q] = lt ? cand : best[q];
      bmb[q] = lt ? cur[q] : bmb[q];
      mlt |= (unsigned)lt << q;
      meq |= (unsigned)eq << q;
    }
    multi = (multi & ~mlt) | meq;
    if (S == Smax) break;
    // can a deeper level still reach (or tie) the minimum of some target of this workgroup?
    const double cN = sc[S + 1];
    bool more = false;
#pragma unroll
    for (int q = 0; q < NP; ++q) more |= ((T1[q] + cN) + Rmin) <= best[q];
    if ((tid & 63) == 0) vote[S & 1][tid >> 6] = 0;
    double *buf = lvl + (size_t)(S & 1) * ncol * CW;
#pragma unroll
    for (int c2 = 0; c2 < PY_CPT; ++c2) {
      const int col = tid + PY_T * c2;
      if (col < ncol) col_store<N0>(buf, col, &cur[N0 * c2]);
    }
    if (__ballot(more) && (tid & 63) == 0) vote[S & 1][tid >> 6] = 1;
    __syncthreads();
    int go = 0;
#pragma unroll
    for (int w = 0; w < PY_T / 64; ++w) go |= vote[S & 1][w];
    if (!go) break;
    // dilate by the unit cross: BM_{S+1}(x) = min(BM_S(x), BM_S(x ± e_m)); a missing neighbour
    // reads the own column (min with itself is a no-op), so there is no divergence
#pragma unroll
    for (int c2 = 0; c2 < PY_CPT; ++c2) {
      const int col = tid + PY_T * c2;
      const int colc = col < ncol ? col : 0;
      double nw[N0];
#pragma unroll
      for (int x0 = 0; x0 < N0; ++x0) {
        double v = cur[N0 * c2 + x0];
        if (x0 > 0) v = vmin(v, cur[N0 * c2 + x0 - 1]);
        if (x0 + 1 < N0) v = vmin(v, cur[N0 * c2 + x0 + 1]);
        nw[x0] = v;
      }
#pragma unroll
      for (int m = 1; m < M; ++m) {
        const int st = G.cstride[m];
        col_min<N0>(buf, colc - (((nbm[c2] >> (2 * m)) & 1) ? st : 0), nw);
        col_min<N0>(buf, colc + (((nbm[c2] >> (2 * m + 1)) & 1) ? st : 0), nw);
      }
#pragma unroll
      for (int x0 = 0; x0 < N0; ++x0) cur[N0 * c2 + x0] = nw[x0];
    }
  }

  // ---- argmin by value lookup; targets whose minimum is reached at two levels go to a list --------
  __syncthreads();
  PY_STAMP(4);
#ifdef MIOC_STAMPS
  if (tid == 0) g_pyr_stamps[blockIdx.x][6] = S;
#endif
  int *list = reinterpret_cast<int *>(lvl);  // the level buffers are free now
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const int col = tid + PY_T * (q / N0);
    if (col >= ncol) continue;
    const int g = q % N0 + N0 * col;
    if ((valid >> q & 1) && (multi >> q & 1)) {
      list[atomicAdd(&nlist, 1)] = g;
      continue;
    }
    double bv = INFINITY;
    int ba = -1;
    if ((valid >> q & 1) && best[q] < INFINITY) {
      bv = best[q];
      ba = py_find(V, (long long)floor(bmb[q] * inv_delta));
    }
    Sout[g] = bv;
    if (ba >= 0) UU[g] = (uint16_t)ba;
  }
  __syncthreads();
  const int nl = nlist;
  for (int e = tid; e < nl; e += PY_T) {
    const int g = list[e];
    int gg = g;
    double t = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const int x = gg % D.n[m];
      gg /= D.n[m];
      t = t + a[m] * (double)(D.base[m] + x);
    }
    double bv = INFINITY;
    int ba = -1;
    py_brute_target<M>(D, sc, t, g, nullptr, Sin, uo1v, L, cp, &bv, &ba);
    Sout[g] = bv;
    if (ba >= 0) UU[g] = (uint16_t)ba;
  }
  PY_STAMP(5);
  if (tid == 0 && nl) atomicAdd(&counters[1], nl);
}

// terminal staging row: S_{n-1}[0][l] = T1(l, n-1) if b̃(l, n-1) <= B (HelpFunctions.jl:27-43), rows > 0 Inf
__global__ void k_pyr_terminal(ProblemDev P, LevelsDev Lv, double *S_all, size_t s_stride) {
  const int k = blockIdx.y;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t n = (size_t)(P.B + 1) * Lv.L;
  if (idx >= n) return;
  const int cp = (int)(idx / Lv.L), l = (int)(idx % Lv.L);
  const int i = P.nt - 1, M = P.M;
  double v = INFINITY;
  if (cp == 0) {
    const double *nuv = Lv.nuval + (size_t)l * M;
    const double *dfi = P.df + ((size_t)k * P.nt + i) * M;
    const double *uoi = P.uold + ((size_t)k * P.nt + i) * M;
    double t = 0.0;
    int b = 0;
    for (int m = 0; m < M; ++m) {
      t = t + (P.dt * dfi[m]) * nuv[m];
      b += (int)fabs(nuv[m] - uoi[m]);
    }
    if (b <= P.B) v = t;
  }
  S_all[(size_t)k * s_stride + idx] = v;
}

hipError_t launch_pyr_terminal(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, double *S, size_t s_stride) {
  const size_t n = (size_t)(P.B + 1) * Lv.L;
  hipLaunchKernelGGL(k_pyr_terminal, dim3((unsigned)((n + 255) / 256), P.K), dim3(256), 0, s, P, Lv, S, s_stride);
  return hipGetLastError();
}

size_t pyr_lds_bytes(const PyrGeom &G) {
  return (size_t)2 * G.ncol * G.n[0] * sizeof(double) + (size_t)PY_HSIZE * (sizeof(long long) + sizeof(uint16_t));
}

hipError_t launch_pyr_step(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G, int i,
                           const double *Sin, double *Sout, uint16_t *UU, size_t s_stride, size_t uu_stride_k,
                           int32_t *counters) {
  const dim3 grid(P.B + 1, P.K), blk(PY_T);
  const size_t lds = pyr_lds_bytes(G);
#define PYR_CASE(MM, NN)                                                                                   \
  if (G.M == MM && G.n[0] == NN) {                                                                         \
    hipLaunchKernelGGL((k_pyr_step<MM, NN>), grid, blk, lds, s, P, Lv, G, i, Sin, Sout, UU, s_stride,      \
                       uu_stride_k, counters);                                                             \
    return hipGetLastError();                                                                              \
  }
  PYR_CASE(2, 8) PYR_CASE(3, 8) PYR_CASE(4, 8) PYR_CASE(5, 8) PYR_CASE(6, 8)
  PYR_CASE(2, 4) PYR_CASE(3, 4) PYR_CASE(4, 4) PYR_CASE(5, 4) PYR_CASE(6, 4)
#undef PYR_CASE
  return hipErrorInvalidValue;
  return hipGetLastError();
}

#ifdef MIOC_STAMPS
extern "C" int32_t mioc_debug_pyr_stamps(unsigned long long *out, int64_t nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pyr_stamps), (size_t)nblocks * 8 * sizeof(unsigned long long)) ==
                 hipSuccess
             ? 0
             : -4;
}
#endif

}  // namespace mioc
