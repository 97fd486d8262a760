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
// Argmin (the reference's strict `>` over iterator order, HelpFunctions.jl:73): the winner of a target is
// the source holding BM at its first winning level.  It is the unique j with fl(K_l(d) + Ψ_j) == out(l)
// unless another source's Ψ lies within δ >= ulp of any candidate value (rounding could tie), or the
// minimum is reached at two levels.  Both cases are detected exactly -- a bucket hash over the row's Ψ
// (same bucket, or close across a bucket border) and per-level tie tracking -- and those targets are
// resolved by a workgroup-parallel exact scan, so results are bit-identical to the reference always.
//
// Layout ("staging"): S_i[c'][pos_i(l)] = Φ_i[l, c' + b̃_l(i)] (+Inf where c'+b̃_l > B), each row in the
// sphere order pos_i of u_old(i) (levels grouped by b̃_l(i)), so the sources a row of step i-1 needs
// from row c'-s of S_i (the sphere s) are one contiguous run; UU_i[c'][l] = U_i[l, c' + b̃_l(i)] (uint16
// rank, natural order).  One workgroup per source row, rows in ascending order (longest first).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <type_traits>

#include "mioc_internal.h"

namespace mioc {

constexpr int PY_T = 1024;         // threads per workgroup: 16 waves, 4 per SIMD
constexpr int PY_TPC = 2;          // threads per grid column (dim-0 run): each owns N0 / PY_TPC points
constexpr int PY_NW = PY_T / 64;   // waves per workgroup
constexpr int PY_HS = 12288;       // hash slots (uint32): <= 4096 sources, load <= 1/3
constexpr int PY_NB = PY_HS / 4;   // 16-byte buckets of 4 slots, each with a 16-bit arrival count
constexpr int PY_OVF = 256;        // keys that found both of their buckets full
constexpr int PY_G = 14;           // bucket width = 2^PY_G · δ (wide: few border checks; false collisions only cost exact scans)
constexpr int PY_CMAX = 512;       // grid columns per row at most (level-buffer chunk stride)
constexpr int PY_CS2 = PY_CMAX + 4;    // level-buffer chunk stride in 16-byte slots (64-byte pad: bank groups)
constexpr int PY_LVLB = PY_CS2 * 16;   // level-buffer bytes per point of a column: 2 parities x 8 B x PY_CS2
constexpr int PY_FEW = 48;         // rows with at most this many targets in the trust region: exact scans
constexpr unsigned PY_RB = 13;     // hash entry = tag << PY_RB | (rank + 1); 0 = empty

// v_min_f64 without the sNaN-quieting v_max_f64 x,x that llvm.minnum puts in front of every operand
// not known to be canonical (inputs here are finite or +Inf, never NaN)
__device__ __forceinline__ double vmin(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Diagnostic build only (make stamps -> libmioc_stamps.so): per-workgroup phase clocks of the last launch.
#ifdef MIOC_STAMPS
__device__ unsigned long long g_pyr_stamps[4096][16];
#define PY_STAMP(k)                                                                          \
  do {                                                                                       \
    if (threadIdx.x == 0) g_pyr_stamps[blockIdx.x][k] = __builtin_amdgcn_s_memtime();         \
  } while (0)
#else
#define PY_STAMP(k) \
  do {              \
  } while (0)
#endif

// Bucket hash.  A bucket of Ψ values is an integer-valued double fq = floor(Ψ·2^k) (+0.0, so -0 and +0
// agree).  Its key has two 16-byte hash buckets of 4 slots; a slot holds tag << PY_RB | (rank + 1).
// Insertion is first-fit without races: an atomicAdd on bucket b1's arrival count hands out slot
// `count` (< 4), arrivals beyond 4 spill to b2 the same way, and beyond that to a small overflow list.
// A count above 4 therefore says "also look at the next place".  Reads are one ds_read_b128 plus the
// count; a tag match is confirmed against the exact Ψ of that rank (psiarr).
struct PyKey {
  unsigned b1, b2, tag;
};
__device__ __forceinline__ PyKey py_key(double fq) {
  unsigned long long x = (unsigned long long)__double_as_longlong(fq);  // splitmix64 finaliser
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  x ^= x >> 31;
  const unsigned lo = (unsigned)x, hi = (unsigned)(x >> 32);
  PyKey k;
  k.b1 = __umulhi(lo, (unsigned)PY_NB);
  k.b2 = __umulhi(hi, (unsigned)PY_NB);
  if (k.b2 == k.b1) k.b2 = k.b1 + 1 == (unsigned)PY_NB ? 0u : k.b1 + 1;
  k.tag = (lo ^ (hi >> 7)) & ((1u << (32 - PY_RB)) - 1);
  return k;
}
__device__ __forceinline__ int py_erank(unsigned e) { return (int)(e & ((1u << PY_RB) - 1)) - 1; }
__device__ __forceinline__ unsigned py_slot(const uint4 &b, int s) {
  return s == 0 ? b.x : s == 1 ? b.y : s == 2 ? b.z : b.w;
}
__device__ __forceinline__ unsigned py_count(const unsigned *hcnt, unsigned b) {
  return (hcnt[b >> 1] >> ((b & 1) * 16)) & 0xFFFFu;
}
__device__ __forceinline__ double py_bucket(double v, double inv_w) { return floor(v * inv_w) + 0.0; }

struct PyHash {
  const uint4 *tab4;     // [PY_NB] buckets
  const unsigned *hcnt;  // [PY_NB / 2] arrival counts, two 16-bit counts per word
  const uint2 *hovf;     // [PY_OVF] {bucket b1, entry}
  int novf;              // entries in hovf (<= PY_OVF; more means the row is resolved by exact scans)
};

// Every entry of `key` beyond bucket b1: bucket b2 when b1 spilled, then the overflow list when b2 did
// too.  Cold path, out of line.  Calls visit(e) as f(e) through a small state machine: returns the
// first rank r != self whose entry carries key.tag and whose Ψ lies in bucket fq (mode 0, also marks
// every such rank in coll), or whose Ψ equals v (mode 1).
__device__ __forceinline__ int py_spill(PyHash H, const double *psiarr, unsigned char *coll, PyKey key, double fq,
                                     double inv_w, double v, int self, int mode) {
  int found = -1;
  auto visit = [&](unsigned e) {
    if ((e >> PY_RB) != key.tag) return;
    const int r = py_erank(e);
    if (r == self) return;
    if (mode == 0) {
      if (py_bucket(psiarr[r], inv_w) == fq) {
        coll[r] = 1;
        if (found < 0) found = r;
      }
    } else if (found < 0 && psiarr[r] == v) {
      found = r;
    }
  };
  const unsigned c2 = py_count(H.hcnt, key.b2);
  const uint4 t = H.tab4[key.b2];
  for (int s2 = 0; s2 < 4 && s2 < (int)c2; ++s2) visit(py_slot(t, s2));
  if (c2 > 4)
    for (int o = 0; o < H.novf; ++o)
      if (H.hovf[o].x == key.b1) visit(H.hovf[o].y);
  return found;
}

// All entries of `key` (bucket b1, then the spill places): mode 0 marks every other source whose Ψ lies
// in bucket fq and returns one of them, mode 1 returns the first source whose Ψ equals v.  Out of line.
__device__ __forceinline__ int py_search(PyHash H, const double *psiarr, unsigned char *coll, PyKey key, double fq,
                                      double inv_w, double v, int self, int mode) {
  int found = -1;
  const unsigned c1 = py_count(H.hcnt, key.b1);
  const uint4 t = H.tab4[key.b1];
  for (int s2 = 0; s2 < 4 && s2 < (int)c1; ++s2) {
    const unsigned e = py_slot(t, s2);
    const int r = py_erank(e);
    if ((e >> PY_RB) != key.tag || r == self) continue;
    if (mode == 0) {
      if (py_bucket(psiarr[r], inv_w) == fq) {
        coll[r] = 1;
        if (found < 0) found = r;
      }
    } else if (found < 0 && psiarr[r] == v) {
      found = r;
    }
  }
  if (c1 > 4 && (mode == 0 || found < 0)) {
    const int f2 = py_spill(H, psiarr, coll, key, fq, inv_w, v, self, mode);
    if (found < 0) found = f2;
  }
  return found;
}

struct PyrDims {  // geometry copied by value into registers (never escapes to memory)
  int n[kMaxM];
  int base[kMaxM];
};

// PT consecutive uint32 (PT = 2 or 4) with one vector load
template <int PT>
__device__ __forceinline__ void py_load_u32(const uint32_t *p, uint32_t *e) {
  if constexpr (PT == 4) {
    const uint4 t = *reinterpret_cast<const uint4 *>(p);
    e[0] = t.x, e[1] = t.y, e[2] = t.z, e[3] = t.w;
  } else {
    const uint2 t = *reinterpret_cast<const uint2 *>(p);
    e[0] = t.x, e[1] = t.y;
  }
}

// value of lane ^ 1 (DPP quad_perm [1,0,3,2]): the other half of the thread pair's grid column
__device__ __forceinline__ double py_swap_pair(double x) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// workgroup-wide OR of one flag per thread: wave ballot, one LDS word per wave, one barrier
__device__ __forceinline__ bool py_any(bool f, int *slots) {
  const unsigned long long bal = __ballot(f);
  if ((threadIdx.x & 63) == 0) slots[threadIdx.x >> 6] = bal != 0ull;
  __syncthreads();
  int r = 0;
#pragma unroll
  for (int w = 0; w < PY_NW; ++w) r |= slots[w];
  return r != 0;
}

// Exact scan of listed targets, the reference loop (HelpFunctions.jl:60-77) for one cell: one wave per
// target.  Lane k evaluates the sources of columns k, k+64, ... (N0 points each, Ψ by rank in LDS) in
// increasing rank, then a (value, rank) minimum over the wave.  Writes UU[l] for a finite minimum, and
// outv[l] (the minimum, +Inf if none) when outv is given.  No barriers; waves take targets round-robin.
template <int M, int N0>
__device__ __forceinline__ void py_scan_list(const int *list, int nl, const double *psiarr, const PyrDims &D,
                                             int ncol, const double *dfi, double dt, double beta, uint16_t *UU,
                                             double *outv) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (w >= nl) return;
  // this lane's columns, coordinates 1..M-1 packed 10 bits each (n_m <= ncol <= 512)
  unsigned long long pk[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    int cc = lane + 64 * t;
    unsigned long long v = 0;
#pragma unroll
    for (int m = 1; m < M; ++m) {
      v |= (unsigned long long)(cc % D.n[m]) << (10 * (m - 1));
      cc /= D.n[m];
    }
    pk[t] = v;
  }
  double a[M];
#pragma unroll
  for (int m = 0; m < M; ++m) a[m] = dt * dfi[m];
  for (int e = w; e < nl; e += PY_NW) {
    const int l = list[e];
    int xl[M];
    {
      int gg = l;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        xl[m] = gg % D.n[m];
        gg /= D.n[m];
      }
    }
    double t1 = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) t1 = t1 + a[m] * (double)(D.base[m] + xl[m]);
    double bv = INFINITY;
    int bj = -1;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int c = lane + 64 * t;
      if (c >= ncol) break;
      int dcol = 0;
#pragma unroll
      for (int m = 1; m < M; ++m) dcol += abs((int)((pk[t] >> (10 * (m - 1))) & 1023u) - xl[m]);
      const double2 *p2 = reinterpret_cast<const double2 *>(psiarr + N0 * c);
#pragma unroll
      for (int q = 0; q < N0 / 2; ++q) {
        const double2 ps = p2[q];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int x0 = 2 * q + h;
          const double val = (t1 + beta * (double)(abs(x0 - xl[0]) + dcol)) + (h ? ps.y : ps.x);
          if (val < bv) {
            bv = val;
            bj = x0 + N0 * c;
          }
        }
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double ov = __shfl_xor(bv, off);
      const int oj = __shfl_xor(bj, off);
      if (oj >= 0 && (bj < 0 || ov < bv || (ov == bv && oj < bj))) {
        bv = ov;
        bj = oj;
      }
    }
    if (lane == 0) {
      if (bj >= 0) UU[l] = (uint16_t)bj;
      if (outv) outv[l] = bj >= 0 ? bv : INFINITY;
    }
  }
}

template <int M, int N0>
__global__ __launch_bounds__(PY_T) void k_pyr_step(ProblemDev P, LevelsDev Lv, PyrGeom G, int i,
                                                   const uint32_t *__restrict__ perm_all,
                                                   const double *__restrict__ Sin_all, double *__restrict__ Sout_all,
                                                   uint16_t *__restrict__ UU_all, size_t s_stride, size_t uu_stride_k,
                                                   int32_t *__restrict__ counters) {
  static_assert(N0 == 4 || N0 == 8, "column length");
  static_assert(M >= 2, "product grid");
  constexpr int PT = N0 / PY_TPC;  // points per thread: thread pairs share a grid column
  extern __shared__ __attribute__((aligned(16))) unsigned char pys[];
  __shared__ double red[2][PY_NW];
  __shared__ int anyv[PY_NW];
  __shared__ int vote[2][PY_NW];        // per-wave early-exit votes, double-buffered by level parity
  __shared__ int nlist, nmulti, novf, nvalid;
#ifdef MIOC_STAMPS
  __shared__ int dbg_lv[2];
  if (threadIdx.x == 0) dbg_lv[0] = dbg_lv[1] = 0;
#endif
  PyrDims D;
#pragma unroll
  for (int m = 0; m < kMaxM; ++m) {
    D.n[m] = G.n[m];
    D.base[m] = G.base[m];
  }
  const int k = blockIdx.y;
  const int L = Lv.L, B = P.B, tid = threadIdx.x, ncol = G.ncol, Smax = G.Smax;
  const double beta = Lv.beta;
  // source row, ascending: rows near B have few targets inside the trust region and are the cheapest,
  // so with B+1 > #CUs the rows that wait for a free CU are the short ones (longest-first order)
  const int cp = (int)blockIdx.x;
  const double *Sin = Sin_all + (size_t)k * s_stride;
  double *Sout = Sout_all + (size_t)k * s_stride + (size_t)cp * L;
  uint16_t *UU = UU_all + (size_t)k * uu_stride_k + (size_t)i * ((size_t)(B + 1) * L) + (size_t)cp * L;
  const double *dfi = P.df + ((size_t)k * P.nt + i) * M;
  const double *uoi = P.uold + ((size_t)k * P.nt + i) * M;
  double *lvl = reinterpret_cast<double *>(pys);                             // level buffers (below)
  double *psiarr = reinterpret_cast<double *>(pys + PY_LVLB * N0);           // [L] Ψ_j by rank j
  unsigned *htab = reinterpret_cast<unsigned *>(psiarr + L);                 // [PY_HS] hash buckets
  unsigned *hcnt = htab + PY_HS;                                             // [PY_NB / 2] arrival counts
  uint2 *hovf = reinterpret_cast<uint2 *>(hcnt + PY_NB / 2);                 // [PY_OVF] overflow list
  unsigned char *coll = reinterpret_cast<unsigned char *>(hovf + PY_OVF);    // [L] Ψ_j has a close value
  PY_STAMP(0);
#ifdef MIOC_STAMPS
  if (tid == 0) g_pyr_stamps[blockIdx.x][13] = __builtin_amdgcn_s_memrealtime();
#endif

  // ---- this thread's half column: coordinates 1..M-1 are shared by the column's N0 points; thread h of
  // the pair owns x0 = PT*h .. PT*h + PT-1, ranks pbase .. pbase + PT-1 -----------------------------
  const int h = tid & (PY_TPC - 1);
  const bool colok = (tid / PY_TPC) < ncol;
  const int col = colok ? tid / PY_TPC : 0;
  const int pbase = N0 * col + PT * h;
  double a[M], pc[M];
#pragma unroll
  for (int m = 0; m < M; ++m) a[m] = P.dt * dfi[m];
  int bcl = 0, nbm = 0;
  {
    int cc = col;
#pragma unroll
    for (int m = 1; m < M; ++m) {
      const int xm = cc % D.n[m];
      cc /= D.n[m];
      const double nu = (double)(D.base[m] + xm);
      pc[m] = a[m] * nu;
      bcl += (int)fabs(nu - uoi[m]);
      nbm |= (xm > 0 ? 1 : 0) << (2 * m);
      nbm |= (xm + 1 < D.n[m] ? 1 : 0) << (2 * m + 1);
    }
  }
  const double u00 = uoi[0];
  // δ >= 2 ulp of any candidate fl(K + Ψ):  |K| <= sum_m |Δt·df_m|·max|ν_m| + β·Smax (so a[] dies early)
  double kb = beta * (double)Smax;
#pragma unroll
  for (int m = 0; m < M; ++m)
    kb += fabs(a[m]) * fmax(fabs((double)D.base[m]), fabs((double)(D.base[m] + D.n[m] - 1)));

  // ---- sources: Ψ_j = Φ_{i+1}[j, c'] = S_{i+1}[c' - b̃_j(i+1)][pos(j)].  Rows are stored in the sphere
  // order of u_old(i+1), so thread t reads positions PT·t .. PT·t+PT-1 -- one contiguous run of a
  // row for all positions of one sphere -- and scatters them into Ψ-by-rank (psiarr) in LDS ----------
  const uint32_t *pin = perm_all + ((size_t)k * P.nt + i + 1) * L;
  const uint32_t *pout = perm_all + ((size_t)k * P.nt + i) * L;
  if (tid == 0) nvalid = 0;
  if (colok) {
    uint32_t e[PT];
    py_load_u32<PT>(pin + pbase, e);
    double v[PT];
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      const int row = cp - (int)(e[q] >> 16);
      v[q] = Sin[(size_t)(row >= 0 ? row : 0) * L + pbase + q];
      if (row < 0) v[q] = INFINITY;
    }
#pragma unroll
    for (int q = 0; q < PT; ++q) psiarr[e[q] & 0xFFFFu] = v[q];
  }
  __syncthreads();
  // ---- own points: targets (T1, validity) and sources (Ψ) -----------------------------------------
  // invalid targets carry T1 = +Inf and best = -Inf, so the level loop needs no branches
  double cur[PT], T1[PT];
  unsigned valid = 0, fin = 0;
  if (colok) {
    const double2 *p2 = reinterpret_cast<const double2 *>(psiarr + pbase);
#pragma unroll
    for (int c = 0; c < PT / 2; ++c) {
      const double2 t = p2[c];
      cur[2 * c] = t.x;
      cur[2 * c + 1] = t.y;
    }
  } else {
#pragma unroll
    for (int x0 = 0; x0 < PT; ++x0) cur[x0] = INFINITY;
  }
#pragma unroll
  for (int x0 = 0; x0 < PT; ++x0) {
    const double nu0 = (double)(D.base[0] + PT * h + x0);
    double t = 0.0;
    t = t + a[0] * nu0;  // ((0 + (Δt*df_1)*ν_1) + ...), HelpFunctions.jl:52-57
#pragma unroll
    for (int m = 1; m < M; ++m) t = t + pc[m];
    const int bl = (int)fabs(nu0 - u00) + bcl;
    const bool v = colok && bl <= B - cp;
    valid |= (unsigned)v << x0;
    T1[x0] = v ? t : INFINITY;
    fin |= (unsigned)(cur[x0] < INFINITY) << x0;
  }
  double psimax = 0.0, psimin = INFINITY;
#pragma unroll
  for (int x0 = 0; x0 < PT; ++x0) {
    const bool f = fin >> x0 & 1;
    psimax = fmax(psimax, f ? fabs(cur[x0]) : 0.0);
    psimin = fmin(psimin, cur[x0]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    psimax = fmax(psimax, __shfl_xor(psimax, off));
    psimin = fmin(psimin, __shfl_xor(psimin, off));
  }
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = psimax;
    red[1][tid >> 6] = psimin;
  }
  if (valid) atomicAdd(&nvalid, __popc(valid));
  const bool any_valid = py_any(valid != 0, anyv);  // its barrier also publishes red[][] and nvalid
  double Pmax = red[0][0], Rmin = red[1][0];
#pragma unroll
  for (int w = 1; w < PY_NW; ++w) {
    Pmax = fmax(Pmax, red[0][w]);
    Rmin = fmin(Rmin, red[1][w]);
  }
  PY_STAMP(1);
  if (!any_valid || !(Rmin < INFINITY)) {  // no target in the trust region, or nothing reachable
    if (colok) {
#pragma unroll
      for (int x0 = 0; x0 < PT; ++x0) Sout[pbase + x0] = INFINITY;
    }
    return;
  }
  if (nvalid <= PY_FEW) {
    // few targets inside the trust region (rows near B): exact scans instead of hash + pyramid
    int *list = reinterpret_cast<int *>(lvl);
    double *outnat = lvl + L;
    if (tid == 0) nlist = 0;
    __syncthreads();
    if (colok) {
#pragma unroll
      for (int x0 = 0; x0 < PT; ++x0) {
        outnat[pbase + x0] = INFINITY;
        if (valid >> x0 & 1) list[atomicAdd(&nlist, 1)] = pbase + x0;
      }
    }
    __syncthreads();
    py_scan_list<M, N0>(list, nlist, psiarr, D, ncol, dfi, P.dt, beta, UU, outnat);
    __syncthreads();
    if (colok) {
      uint32_t e[PT];
      py_load_u32<PT>(pout + pbase, e);
      double o[PT];
#pragma unroll
      for (int q = 0; q < PT; ++q) o[q] = outnat[e[q] & 0xFFFFu];
      double2 *s2 = reinterpret_cast<double2 *>(Sout + pbase);
#pragma unroll
      for (int c = 0; c < PT / 2; ++c) s2[c] = make_double2(o[2 * c], o[2 * c + 1]);
    }
    return;
  }
  const double Y = (Pmax + kb) * (1.0 + 0x1p-40) + 0x1p-1000;
  const int E = ilogb(Y) + 1;                                  // |y| < 2^E for every candidate y
  const double inv_w = ldexp(1.0, min(52 - PY_G - E, 1000));  // bucket width 2^(E-52+G) >= δ = 2^(E-52)
  constexpr double FR = 1.0 / (double)(1 << PY_G);             // δ / bucket width

  // ---- collision flags: coll[j] = 1 iff some other finite Ψ lies within δ of Ψ_j (it shares Ψ_j's
  // bucket, or sits across a bucket border close to it).  Inserts advance in lock-step so their LDS
  // atomics overlap; duplicates are inserted too. -----------------------------------------------------
  double fq[PT], fr[PT];
#pragma unroll
  for (int x0 = 0; x0 < PT; ++x0) {
    const double x = (fin >> x0 & 1) ? cur[x0] * inv_w : 0.0;
    fq[x0] = floor(x) + 0.0;
    fr[x0] = x - fq[x0];
  }
  {
    uint4 *c4 = reinterpret_cast<uint4 *>(hcnt);
    for (int s2 = tid; s2 < PY_NB / 8; s2 += PY_T) c4[s2] = make_uint4(0u, 0u, 0u, 0u);
    for (int s2 = tid; s2 < L; s2 += PY_T) coll[s2] = 0;
  }
  if (tid == 0) {
    nlist = 0;
    nmulti = 0;
    novf = 0;
  }
  PY_STAMP(2);
  __syncthreads();
  PY_STAMP(7);
  PyHash H;
  H.tab4 = reinterpret_cast<const uint4 *>(htab);
  H.hcnt = hcnt;
  H.hovf = hovf;
  {
    PyKey key[PT];
    unsigned ent[PT], cnt[PT];
#pragma unroll
    for (int x0 = 0; x0 < PT; ++x0) {
      key[x0] = py_key(fq[x0]);
      ent[x0] = key[x0].tag << PY_RB | (unsigned)(pbase + x0 + 1);
    }
    // first fit: slot `count` of b1, else of b2, else the overflow list (one atomic round each)
#pragma unroll
    for (int x0 = 0; x0 < PT; ++x0)
      cnt[x0] = (fin >> x0 & 1) ? atomicAdd(&hcnt[key[x0].b1 >> 1], 1u << ((key[x0].b1 & 1) * 16)) : 0u;
    unsigned spill = 0;
#pragma unroll
    for (int x0 = 0; x0 < PT; ++x0) {
      if (!(fin >> x0 & 1)) continue;
      const unsigned c = (cnt[x0] >> ((key[x0].b1 & 1) * 16)) & 0xFFFFu;
      if (c < 4)
        htab[key[x0].b1 * 4 + c] = ent[x0];
      else
        spill |= 1u << x0;
    }
    if (spill) {
#pragma unroll
      for (int x0 = 0; x0 < PT; ++x0)
        cnt[x0] = (spill >> x0 & 1) ? atomicAdd(&hcnt[key[x0].b2 >> 1], 1u << ((key[x0].b2 & 1) * 16)) : 0u;
#pragma unroll
      for (int x0 = 0; x0 < PT; ++x0) {
        if (!(spill >> x0 & 1)) continue;
        const unsigned c = (cnt[x0] >> ((key[x0].b2 & 1) * 16)) & 0xFFFFu;
        if (c < 4) {
          htab[key[x0].b2 * 4 + c] = ent[x0];
        } else {
          const int o = atomicAdd(&novf, 1);
          if (o < PY_OVF) hovf[o] = make_uint2(key[x0].b1, ent[x0]);
        }
      }
    }
    PY_STAMP(8);
    __syncthreads();  // every value is in the table
    PY_STAMP(9);
    H.novf = min(novf, PY_OVF);
    // close across a bucket border (same-bucket pairs are caught by the lookups below)
    unsigned hit = 0, need = 0;
#pragma unroll
    for (int x0 = 0; x0 < PT; ++x0) {
      if (!(fin >> x0 & 1)) continue;
      need |= (unsigned)(fr[x0] <= FR) << (x0 + 8);
      need |= (unsigned)(fr[x0] >= 1.0 - FR) << (x0 + 16);
    }
    // cold: full searches (bucket b1, spill places) -- one copy of the code, operands from LDS
#pragma unroll 1
    for (int q = 0; q < 3 * PT; ++q) {
      const int x0 = q % PT, kind = q / PT;
      if (!(need >> (x0 + 8 * kind) & 1)) continue;
      const int me = pbase + x0;
      const double fqs = py_bucket(psiarr[me], inv_w) + (kind == 1 ? -1.0 : kind == 2 ? 1.0 : 0.0);
      if (py_search(H, psiarr, coll, py_key(fqs), fqs, inv_w, 0.0, me, 0) >= 0) hit |= 1u << x0;
    }
#pragma unroll
    for (int x0 = 0; x0 < PT; ++x0)
      if (hit >> x0 & 1) coll[pbase + x0] = 1;
    if (hit) atomicAdd(&counters[6], __popc(hit));
  }
  PY_STAMP(3);

  // ---- the pyramid (branch-free level loop) ------------------------------------------------------
  double best[PT], bmb[PT];
#pragma unroll
  for (int x0 = 0; x0 < PT; ++x0) {
    best[x0] = (valid >> x0 & 1) ? INFINITY : -INFINITY;
    bmb[x0] = INFINITY;
  }
  // per point: the wave's lanes whose minimum was tied at a later level (wave-uniform 64-bit masks, so
  // the bookkeeping is scalar and issues beside the vector work)
  unsigned long long mm[PT];
#pragma unroll
  for (int x0 = 0; x0 < PT; ++x0) mm[x0] = 0ull;
  int S = 0;
  // Level buffers, chunk-major: [parity][N0/2 chunks][PY_CS2 columns] of 16-byte chunks.  Consecutive
  // columns are consecutive 16-byte slots and the chunk stride is padded by 64 bytes, so the two
  // halves of a column (chunks 0..PT/2-1 and PT/2..) fall in different bank groups: conflict-free
  // ds_read_b128 / ds_write_b128 lane groups.  Chunk and parity are immediate offsets: every neighbour
  // column needs one loop-invariant address register, and the loop is unrolled by two for the parity.
  double2 *lv2 = reinterpret_cast<double2 *>(pys);
  const int hoff = h * (PT / 2) * PY_CS2;  // this thread's half column: its first chunk
  int ncl[M - 1][2];  // neighbour half columns (the own column where the grid ends)
#pragma unroll
  for (int m = 1; m < M; ++m) {
    const int st = G.cstride[m];
    ncl[m - 1][0] = hoff + col - (((nbm >> (2 * m)) & 1) ? st : 0);
    ncl[m - 1][1] = hoff + col + (((nbm >> (2 * m + 1)) & 1) ? st : 0);
  }
  const int own = hoff + col;
  auto level = [&](auto par_tag) -> bool {  // one level; true when the loop is over
    constexpr int PAR = decltype(par_tag)::value;
    constexpr int HALF = (N0 / 2) * PY_CS2;
    const double cS = beta * (double)S;
#pragma unroll
    for (int x0 = 0; x0 < PT; ++x0) {
      const double cand = (T1[x0] + cS) + cur[x0];  // fl(K_l(S) + BM_S), K_l(S) = fl(T1 + fl(β·S))
      const bool lt = cand < best[x0];
      const bool eq = cand == best[x0];  // Inf == Inf ties only mark targets left at +Inf (never listed)
      best[x0] = vmin(cand, best[x0]);
      bmb[x0] = lt ? cur[x0] : bmb[x0];
      mm[x0] = (mm[x0] & ~__ballot(lt)) | __ballot(eq);
    }
    if (S == Smax) return true;
    // can a deeper level still reach (or tie) the minimum of some target of this workgroup?
    // (K_l(S) is non-decreasing in S: the pyramid is only selected for β >= 0)
    const double cN = beta * (double)(S + 1);
    bool more = false;
#pragma unroll
    for (int x0 = 0; x0 < PT; ++x0) {
      more |= ((T1[x0] + cN) + Rmin) <= best[x0];
    }
    if (colok) {
#pragma unroll
      for (int c = 0; c < PT / 2; ++c) lv2[PAR * HALF + c * PY_CS2 + own] = make_double2(cur[2 * c], cur[2 * c + 1]);
    }
    {
      const unsigned long long bal = __ballot(more);
      if ((tid & 63) == 0) vote[PAR][tid >> 6] = bal != 0ull;
    }
    __syncthreads();
    // every LDS read of this level is issued before the first use
    int go = 0;
#pragma unroll
    for (int w = 0; w < PY_NW; ++w) go |= vote[PAR][w];
    double2 nb[M - 1][2][PT / 2];
#pragma unroll
    for (int m = 0; m < M - 1; ++m)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int c = 0; c < PT / 2; ++c) nb[m][s2][c] = lv2[PAR * HALF + c * PY_CS2 + ncl[m][s2]];
    // dilate by the unit cross: BM_{S+1}(x) = min(BM_S(x), BM_S(x ± e_m)); a missing neighbour
    // reads the own column (min with itself is a no-op), so there is no divergence.  The dilation
    // runs before the exit test so the neighbour reads are issued together with the vote reads.
    double nw[PT];
#pragma unroll
    for (int x0 = 0; x0 < PT; ++x0) {
      double v = cur[x0];
      if (x0 > 0) v = vmin(v, cur[x0 - 1]);
      if (x0 + 1 < PT) v = vmin(v, cur[x0 + 1]);
      nw[x0] = v;
    }
    {  // across the half-column boundary: the partner lane (lane ^ 1) holds the other half
      const double r = py_swap_pair(h ? cur[0] : cur[PT - 1]);
      nw[0] = vmin(nw[0], h ? r : INFINITY);
      nw[PT - 1] = vmin(nw[PT - 1], h ? INFINITY : r);
    }
#pragma unroll
    for (int m = 0; m < M - 1; ++m)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int c = 0; c < PT / 2; ++c) {
          nw[2 * c] = vmin(nw[2 * c], nb[m][s2][c].x);
          nw[2 * c + 1] = vmin(nw[2 * c + 1], nb[m][s2][c].y);
        }
#ifdef MIOC_STAMPS
    {
      bool ch = false;
#pragma unroll
      for (int x0 = 0; x0 < PT; ++x0) ch |= nw[x0] < cur[x0];
      const unsigned long long bc = __ballot(ch);
      if ((tid & 63) == 0) {
        atomicAdd(&dbg_lv[0], 1);
        if (bc) atomicAdd(&dbg_lv[1], 1);
      }
    }
#endif
#pragma unroll
    for (int x0 = 0; x0 < PT; ++x0) cur[x0] = nw[x0];
    ++S;
    return !go;
  };
  for (;;) {
    if (level(std::integral_constant<int, 0>{})) break;
    if (level(std::integral_constant<int, 1>{})) break;
  }
  PY_STAMP(4);
#ifdef MIOC_STAMPS
  __syncthreads();
  if (tid == 0) g_pyr_stamps[blockIdx.x][15] = ((unsigned long long)dbg_lv[0] << 32) | (unsigned)dbg_lv[1];
  if (tid == 0) g_pyr_stamps[blockIdx.x][6] = S;
#endif

  // ---- argmin.  A target whose minimum is reached at one level only, by a value with no close
  // neighbour, has a unique minimiser: the source holding that value (one bucket-pair read).  Every
  // other target with a finite minimum goes to the exact scan below. --------------------------------
  unsigned multi = 0;
#pragma unroll
  for (int x0 = 0; x0 < PT; ++x0) multi |= (unsigned)((mm[x0] >> (tid & 63)) & 1ull) << x0;
  int rk[PT];
  unsigned want = 0;
#pragma unroll
  for (int x0 = 0; x0 < PT; ++x0) want |= (unsigned)((valid >> x0 & 1) && !(multi >> x0 & 1) && best[x0] < INFINITY) << x0;
  {
    PyKey key[PT];
    uint4 bk[PT][2];
    unsigned cc[PT][2];
#pragma unroll
    for (int x0 = 0; x0 < PT; ++x0) {
      rk[x0] = -1;
      if (want >> x0 & 1) {
        key[x0] = py_key(py_bucket(bmb[x0], inv_w));
        bk[x0][0] = H.tab4[key[x0].b1];
        bk[x0][1] = H.tab4[key[x0].b2];
        cc[x0][0] = py_count(hcnt, key[x0].b1);
        cc[x0][1] = py_count(hcnt, key[x0].b2);
      }
    }
    // the tag's entries in b1 (and b2 if b1 spilled): exactly one, holding bmb, is the clean case;
    // a second one may be another source in the same bucket, and a double spill may hide more
    unsigned redo = 0;
#pragma unroll
    for (int x0 = 0; x0 < PT; ++x0) {
      if (!(want >> x0 & 1)) continue;
      int nm = 0;
#pragma unroll
      for (int h = 1; h >= 0; --h)
#pragma unroll
        for (int s2 = 3; s2 >= 0; --s2) {
          const unsigned e = py_slot(bk[x0][h], s2);
          if ((h == 0 || cc[x0][0] > 4) && s2 < (int)cc[x0][h] && (e >> PY_RB) == key[x0].tag) {
            rk[x0] = py_erank(e);
            ++nm;
          }
        }
      redo |= (unsigned)(nm != 1 || (cc[x0][0] > 4 && cc[x0][1] > 4)) << x0;
    }
#pragma unroll
    for (int x0 = 0; x0 < PT; ++x0)  // confirm the single match (one batch of reads)
      redo |= (unsigned)((want >> x0 & 1) && !(redo >> x0 & 1) && psiarr[rk[x0]] != bmb[x0]) << x0;
    // cold: find the holder of bmb among all entries of the key, and whether another source shares
    // its bucket -- one copy of the search code
#pragma unroll 1
    for (int x0 = 0; x0 < PT; ++x0) {
      if (!(redo >> x0 & 1)) continue;
      double v = bmb[0];
#pragma unroll
      for (int q = 1; q < PT; ++q) v = q == x0 ? bmb[q] : v;
      const double fqv = py_bucket(v, inv_w);
      const PyKey kv = py_key(fqv);
      int r = py_search(H, psiarr, coll, kv, 0.0, inv_w, v, -1, 1);
      if (r >= 0 && py_search(H, psiarr, coll, kv, fqv, inv_w, 0.0, r, 0) >= 0) coll[r] = 1;  // not unique
#pragma unroll
      for (int q = 0; q < PT; ++q) rk[q] = q == x0 ? r : rk[q];
    }
  }
  unsigned finb = 0;
#pragma unroll
  for (int x0 = 0; x0 < PT; ++x0) finb |= (unsigned)(best[x0] < INFINITY) << x0;
  multi &= valid & finb;
  unsigned tolist = multi, lost = 0;
#pragma unroll
  for (int x0 = 0; x0 < PT; ++x0) {
    if ((want >> x0 & 1) && (rk[x0] < 0 || coll[rk[x0]])) tolist |= 1u << x0;
    if ((want >> x0 & 1) && rk[x0] < 0) lost |= 1u << x0;
  }
  if (lost) atomicAdd(&counters[5], __popc(lost));
  if (novf > PY_OVF) tolist |= want;  // the overflow list itself overflowed: exact scans for this row
  if (tid == 0 && novf) atomicAdd(&counters[4], 1);
  PY_STAMP(10);
  uint32_t po[PT];  // sphere order of step i for the output row, fetched before the barrier
  if (colok) py_load_u32<PT>(pout + pbase, po);
  __syncthreads();  // the level buffers are free: the list and the natural-order outputs live there
  int *list = reinterpret_cast<int *>(lvl);
  double *outnat = lvl + L;
  if (colok) {
    double2 *o2 = reinterpret_cast<double2 *>(outnat + pbase);
#pragma unroll
    for (int c = 0; c < PT / 2; ++c)
      o2[c] = make_double2((valid >> (2 * c) & 1) ? best[2 * c] : INFINITY,
                           (valid >> (2 * c + 1) & 1) ? best[2 * c + 1] : INFINITY);
    if (!tolist) {  // U in natural order: one PT·2-byte store (cells with Φ = +Inf are unspecified)
      uint32_t w[PT / 2];
#pragma unroll
      for (int c = 0; c < PT / 2; ++c)
        w[c] = (uint32_t)(uint16_t)rk[2 * c] | ((uint32_t)(uint16_t)rk[2 * c + 1] << 16);
      if constexpr (PT == 4)
        *reinterpret_cast<uint2 *>(UU + pbase) = make_uint2(w[0], w[1]);
      else
        *reinterpret_cast<uint32_t *>(UU + pbase) = w[0];
    } else {
#pragma unroll
      for (int x0 = 0; x0 < PT; ++x0) {
        const int g = pbase + x0;
        if (tolist >> x0 & 1)
          list[atomicAdd(&nlist, 1)] = g;
        else if (rk[x0] >= 0)
          UU[g] = (uint16_t)rk[x0];
      }
    }
  }
  if (multi) atomicAdd(&nmulti, __popc(multi));
  __syncthreads();
  PY_STAMP(11);
  // Φ_i row c' in the sphere order of u_old(i): gathered from LDS, written as one contiguous run
  if (colok) {
    double o[PT];
#pragma unroll
    for (int q = 0; q < PT; ++q) o[q] = outnat[po[q] & 0xFFFFu];
    double2 *s2 = reinterpret_cast<double2 *>(Sout + pbase);
#pragma unroll
    for (int c = 0; c < PT / 2; ++c) s2[c] = make_double2(o[2 * c], o[2 * c + 1]);
  }
  PY_STAMP(12);
  const int nl = nlist;
  // exact scan of the listed targets (UU only: their values came out of the pyramid)
  py_scan_list<M, N0>(list, nl, psiarr, D, ncol, dfi, P.dt, beta, UU, nullptr);
  PY_STAMP(5);
#ifdef MIOC_STAMPS
  if (tid == 0) g_pyr_stamps[blockIdx.x][14] = __builtin_amdgcn_s_memrealtime();
#endif
  if (tid == 0 && nl) {
    atomicAdd(&counters[0], nl - nmulti);
    if (nmulti) atomicAdd(&counters[1], nmulti);
  }
}

// Sphere order of u_old(i) for every step (one workgroup per (step, subproblem)): the ranks j grouped by
// their L1 distance b̃_j(i) = Σ_m |ν_jm - u_old[m,i]| (HelpFunctions.jl:53-57), perm[p] = j | b̃_j << 16.
// Staging rows of step i are stored in this order, so the L sources a workgroup of step i-1 reads from
// row c' - s of S_i (the sphere s) form one contiguous run per sphere.  Inside a sphere the ranks ascend (a
// stable counting sort), so the order is a function of u_old(i) alone: steps with equal u_old share one table,
// which the persistent separable-transform driver uses to skip reloading it.
constexpr int kOrderMaxL = 4096;
__global__ __launch_bounds__(256) void k_pyr_order(ProblemDev P, PyrGeom G, uint32_t *perm_all, int32_t *same2,
                                                   uint16_t *strad, int32_t *counters) {
  constexpr int NK = 64;            // bucket keys: min(distance, 63)
  __shared__ int start[NK];         // the next free position of each bucket
  __shared__ int wcnt[4][NK + 1];   // ranks of the current chunk per wave and bucket (NK: the inactive lanes)
  // the order is built here and stored coalesced at the end: scattered 4-byte stores straight to HBM cost a
  // read-modify-write of every 128-byte line at the memory side (the launch checks L <= kOrderMaxL)
  __shared__ uint32_t sperm[kOrderMaxL];
  __shared__ uint16_t sdist[kOrderMaxL];  // each rank's distance (computed once)
  const int i = blockIdx.x, k = blockIdx.y, L = G.ncol * G.n[0], M = G.M;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const double *uo = P.uold + ((size_t)k * P.nt + i) * M;
  uint32_t *perm = perm_all + ((size_t)k * P.nt + i) * L;
  int u[kMaxM];
#pragma unroll
  for (int m = 0; m < kMaxM; ++m) u[m] = m < M ? (int)uo[m] : 0;
  if (same2 && tid == 0) {  // u_old(i) == u_old(i+2) bit for bit: equal sphere orders (the persistent driver's reuse)
    bool eq = i + 2 < P.nt;
    for (int m = 0; eq && m < M; ++m) eq = __double_as_longlong(uo[m]) == __double_as_longlong(uo[2 * M + m]);
    same2[(size_t)k * P.nt + i] = eq ? 1 : 0;
  }
  for (int e = tid; e < NK; e += blockDim.x) start[e] = 0;
  for (int e = tid; e < 4 * (NK + 1); e += blockDim.x) (&wcnt[0][0])[e] = 0;
  __syncthreads();
  // every dimension of 8 levels (the 8^M grids of the separable paths): coordinates by shifts, not divisions
  bool oct = true;
  for (int m = 0; m < M; ++m) oct = oct && G.n[m] == 8;
  auto dist = [&](int j) {
    int d = 0;
    if (oct) {
      for (int m = 0; m < M; ++m) d += abs(G.base[m] + ((j >> (3 * m)) & 7) - u[m]);
    } else {
      for (int m = 0; m < M; ++m) {
        const int x = j % G.n[m];
        j /= G.n[m];
        d += abs(G.base[m] + x - u[m]);
      }
    }
    return min(d, 0xFFFF);
  };
  auto key = [&](int j, int d) { return min(d, 63); };
  // each rank's distance, computed once (the placement below reads it back)
  for (int j = tid; j < L; j += blockDim.x) {
    const int d = dist(j);
    sdist[j] = (uint16_t)d;
    atomicAdd(&start[key(j, d)], 1);
  }
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int b = 0; b < NK; ++b) {
      const int c = start[b];
      start[b] = run;
      run += c;
    }
  }
  __syncthreads();
  // chunks of 256 consecutive ranks in order; inside a chunk, a rank's place among its bucket's ranks is the number of
  // lower lanes of its wave with the same key (7 ballots) plus those of the lower waves
  for (int c = 0; c < L; c += 256) {
    const int j = c + tid;
    const bool act = j < L;
    const int d = act ? (int)sdist[j] : 0, b = act ? key(j, d) : NK;
    unsigned long long same = ~0ull;
#pragma unroll
    for (int q = 0; q < 7; ++q) {
      const unsigned long long m = __ballot((b >> q) & 1);
      same &= ((b >> q) & 1) ? m : ~m;
    }
    const int below = __popcll(same & ((1ull << lane) - 1ull));
    if (below == 0) wcnt[w][b] = __popcll(same);
    __syncthreads();
    if (act) {
      int pos = start[b] + below;
      for (int q = 0; q < w; ++q) pos += wcnt[q][b];
      sperm[pos] = (uint32_t)j | ((uint32_t)d << 16);
    }
    __syncthreads();
    for (int e = tid; e < NK; e += blockDim.x) {
      start[e] += wcnt[0][e] + wcnt[1][e] + wcnt[2][e] + wcnt[3][e];
      wcnt[0][e] = wcnt[1][e] = wcnt[2][e] = wcnt[3][e] = 0;
    }
    if (tid == 0) wcnt[0][NK] = wcnt[1][NK] = wcnt[2][NK] = wcnt[3][NK] = 0;
    __syncthreads();
  }
  if ((L & 3) == 0) {  // 16 bytes per lane (perm rows are 16-byte aligned when L is a multiple of 4)
    for (int e = 4 * tid; e < L; e += 4 * blockDim.x)
      *reinterpret_cast<uint4 *>(perm + e) = *reinterpret_cast<const uint4 *>(sperm + e);
  } else {
    for (int e = tid; e < L; e += blockDim.x) perm[e] = sperm[e];
  }
  // strad (the persistent separable driver at 8^4, 8 waves of 512 positions): per wave, the in-wave offsets of the odd
  // positions whose distance differs from position p-1's -- the second elements of the 16-byte position pairs that
  // straddle a sphere seam -- 0xFFFF-padded to 32.  A wave's positions (sd_seam_pos, mioc_sdt.hip): positions
  // 2(64w + l + (L/8)·q) + {0, 1} at offset 128q + 2l + {0, 1} (at most 28 seams in the whole order: 29 distances)
  if (strad) {
    uint16_t *st = strad + ((size_t)k * P.nt + i) * 8 * 32;
    const int T = L / 8;
    for (int e = tid; e < 8 * 32; e += blockDim.x) st[e] = 0xFFFFu;
    if (tid < 8) start[tid] = 0;  // per-wave counts
    __syncthreads();
    for (int p = 2 * tid + 1; p < L; p += 2 * blockDim.x)
      if ((sperm[p] >> 16) != (sperm[p - 1] >> 16)) {
        const int u = (p - 1) >> 1, t = u % T;
        const int wv = t >> 6;
        const int o = 128 * (u / T) + 2 * (t & 63) + 1;
        const int e = atomicAdd(&start[wv], 1);
        if (e < 32)
          st[wv * 32 + e] = (uint16_t)o;
        else if (counters)  // the list cannot hold this seam: a loud internal-consistency failure (diagnostics [3])
          atomicAdd(&counters[3], 1);
      }
  }
}

hipError_t launch_pyr_order(hipStream_t s, const ProblemDev &P, const PyrGeom &G, uint32_t *perm, int32_t *same2,
                            uint16_t *strad, int32_t *counters) {
  if (G.ncol * G.n[0] > kOrderMaxL) return hipErrorInvalidValue;  // (the pyramid paths need L <= 4096 anyway)
  hipLaunchKernelGGL(k_pyr_order, dim3(P.nt, P.K), dim3(256), 0, s, P, G, perm, same2, strad, counters);
  return hipGetLastError();
}

// terminal staging row: S_{n-1}[0][pos(l)] = T1(l, n-1) if b̃(l, n-1) <= B (HelpFunctions.jl:27-43),
// rows > 0 Inf
__global__ void k_pyr_terminal(ProblemDev P, LevelsDev Lv, const uint32_t *perm_all, double *S_all,
                               size_t s_stride) {
  const int k = blockIdx.y;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t n = (size_t)(P.B + 1) * Lv.L;
  if (idx >= n) return;
  const int cp = (int)(idx / Lv.L), p = (int)(idx % Lv.L);
  const int i = P.nt - 1, M = P.M;
  double v = INFINITY;
  if (cp == 0) {
    const uint32_t e = perm_all[((size_t)k * P.nt + i) * Lv.L + p];
    const int l = (int)(e & 0xFFFFu), b = (int)(e >> 16);
    const double *nuv = Lv.nuval + (size_t)l * M;
    const double *dfi = P.df + ((size_t)k * P.nt + i) * M;
    double t = 0.0;
    for (int m = 0; m < M; ++m) t = t + (P.dt * dfi[m]) * nuv[m];
    if (b <= P.B) v = t;
  }
  S_all[(size_t)k * s_stride + idx] = v;
}

hipError_t launch_pyr_terminal(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const uint32_t *perm, double *S,
                               size_t s_stride) {
  const size_t n = (size_t)(P.B + 1) * Lv.L;
  hipLaunchKernelGGL(k_pyr_terminal, dim3((unsigned)((n + 255) / 256), P.K), dim3(256), 0, s, P, Lv, perm, S,
                     s_stride);
  return hipGetLastError();
}

size_t pyr_lds_bytes(const PyrGeom &G) {
  return (size_t)PY_LVLB * G.n[0] + (size_t)G.ncol * G.n[0] * sizeof(double) + (size_t)PY_HS * sizeof(unsigned) +
         (size_t)(PY_NB / 2) * sizeof(unsigned) + (size_t)PY_OVF * sizeof(uint2) + (size_t)G.ncol * G.n[0];
}

hipError_t launch_pyr_step(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G, int i,
                           const uint32_t *perm, const double *Sin, double *Sout, uint16_t *UU, size_t s_stride,
                           size_t uu_stride_k, int32_t *counters) {
  const dim3 grid(P.B + 1, P.K), blk(PY_T);
  const size_t lds = pyr_lds_bytes(G);
#define PYR_CASE(MM, NN)                                                                                   \
  if (G.M == MM && G.n[0] == NN) {                                                                         \
    hipLaunchKernelGGL((k_pyr_step<MM, NN>), grid, blk, lds, s, P, Lv, G, i, perm, Sin, Sout, UU, s_stride,      \
                       uu_stride_k, counters);                                                             \
    return hipGetLastError();                                                                              \
  }
  PYR_CASE(2, 8) PYR_CASE(3, 8) PYR_CASE(4, 8) PYR_CASE(5, 8) PYR_CASE(6, 8)
  PYR_CASE(2, 4) PYR_CASE(3, 4) PYR_CASE(4, 4) PYR_CASE(5, 4) PYR_CASE(6, 4)
#undef PYR_CASE
  return hipErrorInvalidValue;
}

#ifdef MIOC_STAMPS
extern "C" int32_t mioc_debug_pyr_stamps(unsigned long long *out, int64_t nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pyr_stamps), (size_t)nblocks * 16 * sizeof(unsigned long long)) ==
                 hipSuccess
             ? 0
             : -4;
}
#endif

}  // namespace mioc
