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
// Tables per subproblem k:  kmin/k2/kfirst [nt][BWP] (terminal row i = nt-1 holds T1 minima, no β)
//                           R              [nt][RP]
#include <hip/hip_runtime.h>

#include <climits>
#include <algorithm>
#include <cstdint>

#include "mioc_internal.h"

namespace mioc {
#ifndef PINF_RECUR_SPLIT
#define PINF_RECUR_SPLIT 1  // few subproblems: G lanes per row pair (A/B builds: 0)
#endif
#ifndef PINF_RECUR_MC
#define PINF_RECUR_MC 1     // few subproblems: row segments on several CUs (k_pinf_recur_mc)
#endif
#ifndef PINF_MC_CHUNK
#define PINF_MC_CHUNK 64       // k_pinf_recur_mc: steps per segment hand-off (C4, 8-row segments: 16: 23.3 ms, 32: 19.9 ms, 64: 19.6 ms)
#endif
#ifndef PINF_RECUR_MC_LANES
#define PINF_RECUR_MC_LANES 8  // k_pinf_recur_mc: lanes per budget row (8: 8 rows per segment; 16: 4 rows, 8 % slower at C4; 4: 16 rows, 11 % slower with the one-step loop; 2: 32)
#endif
#ifndef PINF_MC_SPLIT
#define PINF_MC_SPLIT 1  // k_pinf_recur_mc, 8 lanes per row: classes >= 8 (rows below the segment) off the step chain
#endif
#ifndef PINF_MC_HELPERS
#define PINF_MC_HELPERS 1  // k_pinf_recur_mcw: the off-chain minima of a chunk by three helper waves (A/B builds: 0)
#endif
#ifndef PINF_RECUR_XR
#define PINF_RECUR_XR 1     // C4's B = 256: eight waves and the extra row split by classes (k_pinf_recur_xr)
#endif
#ifndef PINF_PREP_REGS
#define PINF_PREP_REGS 1    // class tables: M a template constant, a thread's levels in registers (A/B builds: 0)
#endif
#ifndef PINF_RECUR_G
#define PINF_RECUR_G 4      // lanes per row pair when split (2 or 4)
#endif
#ifndef PINF_RECUR_WS
#define PINF_RECUR_WS 1     // few subproblems, classes <= 8: 64-row segments, the chain by DPP wave shifts (k_pinf_recur_ws)
#endif
#ifndef PINF_WS_CHUNK
#define PINF_WS_CHUNK 64    // k_pinf_recur_ws: steps per segment hand-off
#endif

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
  __shared__ unsigned long long s_kab;  // max |K| as the bits of a non-negative double (ordered as integers)
  if (threadIdx.x == 0) s_kab = 0ull;
  __syncthreads();
  unsigned long long kab = 0ull;
  for (int r = threadIdx.x; r < Lv.L; r += blockDim.x) {
    const double *nuv = Lv.nuval + (size_t)r * M;
    const int b = p_bt(nuv, uoi, M);
    if (b >= BW) continue;
    const double t1 = p_t1(nuv, dfi, M, P.dt);
    const double v = term ? t1 : t1 + Lv.beta;  // fl(T1 + β·1.0)
    atomicMin(reinterpret_cast<unsigned long long *>(&skmin[b]), (unsigned long long)okey(v));
    const unsigned long long av = (unsigned long long)__double_as_longlong(fabs(v));
    kab = av > kab ? av : kab;
  }
  atomicMax(&s_kab, kab);
  __syncthreads();
  if (threadIdx.x == 0) D.kabs[(size_t)k * P.nt + i] = __longlong_as_double((long long)s_kab);
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
  const size_t row = ((size_t)k * P.nt + i) * D.BWP;
  for (int b = threadIdx.x; b < D.BWP; b += blockDim.x) {
    const bool in = b < BW;
    D.kmin[row + b] = in ? from_okey(skmin[b]) : INFINITY;
    D.k2[row + b] = in ? from_okey(sk2[b]) : INFINITY;
    D.kfirst[row + b] = (!in || sfirst[b] == INT_MAX) ? -1 : sfirst[b];
  }
}

// The same tables with M a compile-time constant and each thread's (at most PREP_PR) levels kept in registers between
// the two passes: a level's values are loaded and its K and class computed once, with Δt·df(:, i) and u_old(:, i) in
// registers (the loop above reloads both per level and per pass).  Same keys, same atomics, same three tables.
constexpr int PREP_PR = 16;
template <int M>
__global__ __launch_bounds__(256) void k_pinf_prep_m(ProblemDev P, LevelsDev Lv, PinfDev D) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int BW = D.BW;
  uint64_t *skmin = reinterpret_cast<uint64_t *>(smem);
  uint64_t *sk2 = skmin + BW;
  int32_t *sfirst = reinterpret_cast<int32_t *>(sk2 + BW);
  const int i = blockIdx.x, k = blockIdx.y, tid = threadIdx.x;
  for (int b = tid; b < BW; b += blockDim.x) {
    skmin[b] = ~0ull;
    sk2[b] = ~0ull;
    sfirst[b] = INT_MAX;
  }
  const double *dfi = P.df + ((size_t)k * P.nt + i) * M;
  const double *uoi = P.uold + ((size_t)k * P.nt + i) * M;
  const bool term = (i == P.nt - 1);
  __shared__ unsigned long long s_kab;
  if (tid == 0) s_kab = 0ull;
  double a[M], uo[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    a[m] = P.dt * dfi[m];  // the factor p_t1 forms per level: the same rounding
    uo[m] = uoi[m];
  }
  __syncthreads();
  uint64_t key[PREP_PR];
  int bb[PREP_PR];
  unsigned long long kab = 0ull;
#pragma unroll
  for (int j = 0; j < PREP_PR; ++j) {
    const int r = tid + 256 * j;
    key[j] = ~0ull;
    bb[j] = BW;  // no class (outside the tracked budgets, or past the level set)
    if (r < Lv.L) {
      const double *nuv = Lv.nuval + (size_t)r * M;
      double nv[M];
#pragma unroll
      for (int m = 0; m < M; ++m) nv[m] = nuv[m];
      int b = 0;
#pragma unroll
      for (int m = 0; m < M; ++m) b += (int)fabs(nv[m] - uo[m]);  // p_bt
      if (b < BW) {
        double t = 0.0;
#pragma unroll
        for (int m = 0; m < M; ++m) t = t + a[m] * nv[m];  // p_t1
        const double v = term ? t : t + Lv.beta;           // fl(T1 + β·1.0)
        key[j] = okey(v);
        bb[j] = b;
        atomicMin(reinterpret_cast<unsigned long long *>(&skmin[b]), (unsigned long long)key[j]);
        const unsigned long long av = (unsigned long long)__double_as_longlong(fabs(v));
        kab = av > kab ? av : kab;
      }
    }
  }
  atomicMax(&s_kab, kab);
  __syncthreads();
  if (tid == 0) D.kabs[(size_t)k * P.nt + i] = __longlong_as_double((long long)s_kab);
#pragma unroll
  for (int j = 0; j < PREP_PR; ++j) {
    const int b = bb[j];
    if (b < BW) {
      if (key[j] == skmin[b])
        atomicMin(&sfirst[b], tid + 256 * j);
      else
        atomicMin(reinterpret_cast<unsigned long long *>(&sk2[b]), (unsigned long long)key[j]);
    }
  }
  __syncthreads();
  const size_t row = ((size_t)k * P.nt + i) * D.BWP;
  for (int b = tid; b < D.BWP; b += blockDim.x) {
    const bool in = b < BW;
    D.kmin[row + b] = in ? from_okey(skmin[b]) : INFINITY;
    D.k2[row + b] = in ? from_okey(sk2[b]) : INFINITY;
    D.kfirst[row + b] = (!in || sfirst[b] == INT_MAX) ? -1 : sfirst[b];
  }
}

// Small level sets (L <= 64, BWP <= 16: the SOS1 shapes of C1-C3): one THREAD per (step, subproblem) walks the L
// levels in rank order and keeps the class keys in registers -- the same three quantities as k_pinf_prep (first
// minimum key, smallest other key, first rank at the minimum; keys compare as okey, so -0.0 < +0.0 as there).
template <int BWP>
__global__ __launch_bounds__(256) void k_pinf_prep_small(ProblemDev P, LevelsDev Lv, PinfDev D) {
  const long long gi = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gi >= (long long)P.K * P.nt) return;
  const int k = (int)(gi / P.nt), i = (int)(gi % P.nt), M = P.M, BW = D.BW;
  const double *dfi = P.df + ((size_t)k * P.nt + i) * M;
  const double *uoi = P.uold + ((size_t)k * P.nt + i) * M;
  const bool term = (i == P.nt - 1);
  double dfv[kMaxM], uov[kMaxM];
  for (int m = 0; m < M; ++m) dfv[m] = dfi[m], uov[m] = uoi[m];
  uint64_t km[BWP], k2[BWP];
  int kf[BWP];
#pragma unroll
  for (int b = 0; b < BWP; ++b) km[b] = ~0ull, k2[b] = ~0ull, kf[b] = -1;
  double kab = 0.0;
  for (int r = 0; r < Lv.L; ++r) {
    const double *nuv = Lv.nuval + (size_t)r * M;
    const int b = p_bt(nuv, uov, M);
    if (b >= BW) continue;
    const double t1 = p_t1(nuv, dfv, M, P.dt);
    const double v = term ? t1 : t1 + Lv.beta;
    kab = fmax(kab, fabs(v));
    const uint64_t key = okey(v);
#pragma unroll
    for (int q = 0; q < BWP; ++q) {
      if (q != b) continue;
      if (key < km[q]) {
        k2[q] = km[q];  // every key seen so far is >= the old minimum, which is not the new one
        km[q] = key;
        kf[q] = r;
      } else if (key != km[q] && key < k2[q]) {
        k2[q] = key;
      }
    }
  }
  const size_t row = ((size_t)k * P.nt + i) * BWP;
  D.kabs[(size_t)k * P.nt + i] = kab;
#pragma unroll
  for (int q = 0; q < BWP; ++q) {
    D.kmin[row + q] = from_okey(km[q]);
    D.k2[row + q] = from_okey(k2[q]);
    D.kfirst[row + q] = kf[q];
  }
}

hipError_t launch_pinf_prep(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PinfDev &D) {
  if (Lv.L <= 64 && D.BWP <= 16) {
    const long long n = (long long)P.K * P.nt;
    const dim3 grid((unsigned)((n + 255) / 256));
    if (D.BWP == 8)
      hipLaunchKernelGGL(k_pinf_prep_small<8>, grid, dim3(256), 0, s, P, Lv, D);
    else
      hipLaunchKernelGGL(k_pinf_prep_small<16>, grid, dim3(256), 0, s, P, Lv, D);
    return hipGetLastError();
  }
  dim3 grid(P.nt, P.K);
  size_t lds = (size_t)D.BW * 20 + 16;
  if (PINF_PREP_REGS && Lv.L <= 256 * PREP_PR && P.M >= 2 && P.M <= 4) {
    if (P.M == 4)
      hipLaunchKernelGGL(k_pinf_prep_m<4>, grid, dim3(256), lds, s, P, Lv, D);
    else if (P.M == 3)
      hipLaunchKernelGGL(k_pinf_prep_m<3>, grid, dim3(256), lds, s, P, Lv, D);
    else
      hipLaunchKernelGGL(k_pinf_prep_m<2>, grid, dim3(256), lds, s, P, Lv, D);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_pinf_prep, grid, dim3(256), lds, s, P, Lv, D);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA staging helpers (global_load_lds_dwordx4: 1 KiB per wave-instruction, no VGPRs).  The
// LDS destination is wave-uniform base + lane*16, so a linear copy maps lane i to bytes [16i, 16i+16).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void glds_copy(const void *gsrc, void *ldst, int bytes, int tid, int nthreads) {
  const int wave = tid >> 6, lane = tid & 63, nw = (nthreads + 63) >> 6;
  for (int off = wave * 1024; off < bytes; off += nw * 1024) {
    if (off + lane * 16 < bytes)
      __builtin_amdgcn_global_load_lds(
          (const __attribute__((address_space(1))) void *)((const char *)gsrc + off + lane * 16),
          (__attribute__((address_space(3))) void *)((char *)ldst + off), 16, 0, 0);
  }
}
// a wave-uniform pointer as an SGPR pair (the "s" operand of an LDS-DMA needs it provably)
__device__ __forceinline__ const void *pi_uniform(const void *p) {
  const unsigned long long x = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)x), hi = __builtin_amdgcn_readfirstlane((unsigned)(x >> 32));
  return (const void *)(((unsigned long long)hi << 32) | lo);
}
typedef unsigned int pi_u32x2 __attribute__((ext_vector_type(2)));

// glds_copy as inline asm (M0 saved and restored): the compiler does not see these LDS writes, so it does not make
// every later LDS read wait for ALL outstanding vector-memory operations (the recursions' streamed R stores among
// them: a store round trip per step); the callers complete them explicitly (vm_drain, then a barrier or, in one
// wave, program order) before the first read of the copy
__device__ __forceinline__ void glds_copy_asm(const void *gsrc_, void *ldst, int bytes, int tid, int nthreads) {
  const int wave = tid >> 6, lane = tid & 63, nw = (nthreads + 63) >> 6;
  const void *gsrc = pi_uniform(gsrc_);
  const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char *)ldst);
  for (int off = wave * 1024; off < bytes; off += nw * 1024) {
    if (off + lane * 16 < bytes) {
      const unsigned m0 = __builtin_amdgcn_readfirstlane(lds0 + (unsigned)off), voff = (unsigned)(off + lane * 16);
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(voff), "s"(gsrc), "s"(m0)
                   : "memory");
    }
  }
}
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ double dpp_swap_pair(double x) {  // value of lane ^ 1 (quad_perm [1,0,3,2])
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

// v_min_f64 without llvm.minnum's operand canonicalisation (inputs are finite or +Inf, never NaN)
__device__ __forceinline__ double pvmin(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// ---------------------------------------------------------------------------------------------
// sequential recursion over steps, one workgroup per subproblem.
//   R_i[c] = min_{b < BWP} fl(Kmin_i[b] + R_{i+1}[c - b])      (padding: Kmin = +Inf, R[<0] = +Inf)
// Thread t computes the budget rows c = 2t and 2t+1: its window R_{i+1}[2t-BWP+1 .. 2t+1] is BWP+1
// consecutive values.  R is kept in LDS shifted by one (A[k] = R[k + 1 - BWP]), so every window
// starts 16-byte aligned and is read with BWP/2 + 1 ds_read_b128; the class row Kmin_i is a broadcast
// read.  Class rows for CH steps at a time are staged into LDS by LDS-DMA one chunk ahead; the barrier
// per step waits only on LDS (lgkmcnt), so the streamed R_i stores and the next chunk's DMA stay in
// flight.  Four independent min accumulators per output keep the dependency chain short.
// G > 1 (few subproblems, so one workgroup per subproblem leaves most of the CU idle): G adjacent lanes share a row
// pair, each taking BWP/G of the classes over a window of BWP/G + 1 values; their partial minima combine by DPP
// (min is exact, so the result is the same whatever the grouping, and every candidate fl(Kmin_i[b] + R_{i+1}[c-b])
// is the same expression).  C4 at p = Inf: 10 waves instead of 3, each with a quarter of the chain.
// ---------------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double pv_dpp(double x) {
  return __hiloint2double(__builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xF, 0xF, true),
                          __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xF, 0xF, true));
}
#ifdef MIOC_STAMPS
// diagnostic build: per-wave phase cycles of workgroup 0 (s_memtime): [0] window + class reads waited,
// [1] min-plus VALU + stores, [2] barrier, [3] steps, [4] total
__device__ unsigned long long g_pinf_stamps[16][8];
#define PI_T(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define PI_T(v)
#endif

template <int BWP, int G>
__global__ __launch_bounds__(G == 1 ? 512 : 1024) void k_pinf_recur(ProblemDev P, PinfDev D, int CH) {
  if (redo_skip(P)) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  constexpr int CB = BWP / G;     // classes per lane
  constexpr int NP = CB / 2 + 1;  // 16-byte pieces of a lane's window
  static_assert(G == 1 || ((G == 2 || G == 4) && CB % 2 == 0), "k_pinf_recur: G = 1, 2 or 4");
  const int RP = P.RP, B = P.B, nt = P.nt, k = blockIdx.x, nthr = blockDim.x / G;
  const int tid = (int)threadIdx.x / G, h = (int)threadIdx.x % G;  // row pair slot, class quarter
  const int AW = RP + BWP;                     // even: RP is a multiple of 64
  double *A = sm, *Kbuf = sm + 2 * AW;         // A: [2 parities][AW]; Kbuf: [2][CH][BWP]
  const double *kmin = D.kmin + (size_t)k * nt * BWP;
  double *R = D.R + (size_t)k * nt * RP;
  {
    const int pt = (nt - 1) & 1;  // terminal row R_{n-1}[c] = Kmin_{n-1}[c] (class minima of T1, no β)
    for (int q = (int)threadIdx.x; q < 2 * AW; q += (int)blockDim.x) {
      const int par = q / AW, kk = q % AW, c = kk + 1 - BWP;
      double v = INFINITY;
      if (par == pt && c >= 0 && c < BWP) v = kmin[(size_t)(nt - 1) * BWP + c];
      A[q] = v;
      if (par == pt && c >= 0 && c < RP) R[(size_t)(nt - 1) * RP + c] = c <= B ? v : INFINITY;
    }
  }
  if (nt < 2) return;
  int hi = nt - 2, lo = hi - CH + 1 < 0 ? 0 : hi - CH + 1;
  glds_copy_asm(kmin + (size_t)lo * BWP, Kbuf, (hi - lo + 1) * BWP * 8, (int)threadIdx.x, (int)blockDim.x);
  vm_drain();
  lds_barrier();
  for (int q = 0; hi >= 0; ++q) {
    const double *Kc = Kbuf + (size_t)(q & 1) * CH * BWP;
    const int nhi = lo - 1, nlo = nhi - CH + 1 < 0 ? 0 : nhi - CH + 1;
    if (nhi >= 0)
      glds_copy_asm(kmin + (size_t)nlo * BWP, Kbuf + (size_t)((q + 1) & 1) * CH * BWP, (nhi - nlo + 1) * BWP * 8,
                (int)threadIdx.x, (int)blockDim.x);
    for (int i = hi; i >= lo; --i) {
      PI_T(t0);
      for (int c0 = 2 * tid; c0 < RP; c0 += 2 * nthr) {
        // this lane's classes b = h·CB + bb: row 2t reads R_{i+1}[c0 - b] = A[c0 + BWP - 1 - b], a window of CB + 1
        // values from A[c0 + BWP - (h + 1)·CB] (even: 16-byte aligned)
        const double2 *win = reinterpret_cast<const double2 *>(A + (size_t)((i + 1) & 1) * AW + c0 + BWP - (h + 1) * CB);
        const double2 *kr = reinterpret_cast<const double2 *>(Kc + (size_t)(i - lo) * BWP + h * CB);
        double w[2 * NP], kv[CB];
#pragma unroll
        for (int p2 = 0; p2 < NP; ++p2) {
          const double2 x = win[p2];
          w[2 * p2] = x.x;
          w[2 * p2 + 1] = x.y;
        }
#pragma unroll
        for (int p2 = 0; p2 < CB / 2; ++p2) {
          const double2 y = kr[p2];
          kv[2 * p2] = y.x;
          kv[2 * p2 + 1] = y.y;
        }
#ifdef MIOC_STAMPS
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        PI_T(t1);
        if (blockIdx.x == 0 && (threadIdx.x & 63) == 0 && c0 == 2 * tid) g_pinf_stamps[threadIdx.x >> 6][0] += t1 - t0;
#endif
        // row 2t:   R_{i+1}[2t - b]   = w[CB - 1 - bb];   row 2t+1: R_{i+1}[2t + 1 - b] = w[CB - bb]
        // four accumulators per row, each started by its first candidate
        double m0[4], m1[4];
#pragma unroll
        for (int b2 = 0; b2 < CB; ++b2) {
          const double c0 = kv[b2] + w[CB - 1 - b2], c1 = kv[b2] + w[CB - b2];
          m0[b2 & 3] = b2 < 4 ? c0 : pvmin(m0[b2 & 3], c0);
          m1[b2 & 3] = b2 < 4 ? c1 : pvmin(m1[b2 & 3], c1);
        }
        double r0, r1;
        if constexpr (CB >= 4) {
          r0 = pvmin(pvmin(m0[0], m0[1]), pvmin(m0[2], m0[3]));
          r1 = pvmin(pvmin(m1[0], m1[1]), pvmin(m1[2], m1[3]));
        } else {
          r0 = pvmin(m0[0], m0[1]);
          r1 = pvmin(m1[0], m1[1]);
        }
        if constexpr (G >= 2) {  // the class parts of the lane group (quad_perm xor 1, then xor 2)
          r0 = pvmin(r0, pv_dpp<0xB1>(r0));
          r1 = pvmin(r1, pv_dpp<0xB1>(r1));
        }
        if constexpr (G == 4) {
          r0 = pvmin(r0, pv_dpp<0x4E>(r0));
          r1 = pvmin(r1, pv_dpp<0x4E>(r1));
        }
        double *Aout = A + (size_t)(i & 1) * AW;
        if (G == 1 || h == 0) {
          Aout[c0 + BWP - 1] = r0;
          R[(size_t)i * RP + c0] = c0 <= B ? r0 : INFINITY;
        }
        if (G == 1 || h == 1) {
          Aout[c0 + BWP] = r1;
          R[(size_t)i * RP + c0 + 1] = c0 + 1 <= B ? r1 : INFINITY;
        }
      }
      PI_T(t2);
      lds_barrier();
#ifdef MIOC_STAMPS
      PI_T(t3);
      if (blockIdx.x == 0 && (threadIdx.x & 63) == 0) {
        unsigned long long *g = g_pinf_stamps[threadIdx.x >> 6];
        g[1] += t2 - t0;  // minus slot 0 afterwards
        g[2] += t3 - t2;
        g[3] += 1;
        g[4] += t3 - t0;
      }
#endif
    }
    vm_drain();
    lds_barrier();
    hi = nhi;
    lo = nlo;
  }
}

// Budget rows 0 .. 32·NW (one more than NW full waves of lane quads, C4: B = 256, NW = 8): k_pinf_recur<BWP, 4> would
// take a ninth wave (three waves on one SIMD, which bounds the step) for the one extra row E = 32·NW.  Here NW waves
// of row pairs (two per SIMD) and the extra row split by classes: wave w's lane 0 takes classes [w·CW, (w+1)·CW) of
// row E (CW = BWP / NW) and leaves its partial minimum in the LDS; after the step's barrier, wave 0 folds the NW
// partials into R_i[E] (min is exact: the same value as one lane's fold over all classes) while the next step runs.
template <int BWP, int NW>
__global__ __launch_bounds__(NW * 64) void k_pinf_recur_xr(ProblemDev P, PinfDev D, int CH) {
  if (redo_skip(P)) return;
  extern __shared__ __attribute__((aligned(16))) double sm[];
  constexpr int G = 4, CB = BWP / G, NP = CB / 2 + 1, CW = BWP / NW, E = 32 * NW;
  static_assert(CB % 2 == 0 && CW * NW == BWP, "k_pinf_recur_xr shape");
  const int RP = P.RP, B = P.B, nt = P.nt, k = blockIdx.x;
  const int tid = (int)threadIdx.x / G, h = (int)threadIdx.x % G, w = (int)threadIdx.x >> 6, lane = (int)threadIdx.x & 63;
  const int AW = RP + BWP;
  double *A = sm, *Kbuf = sm + 2 * AW, *part = Kbuf + 2 * CH * BWP;  // part: [2 parities][NW]
  const double *kmin = D.kmin + (size_t)k * nt * BWP;
  double *R = D.R + (size_t)k * nt * RP;
  const int c0 = 2 * tid;
  {
    const int pt = (nt - 1) & 1;
    for (int q = (int)threadIdx.x; q < 2 * AW; q += (int)blockDim.x) {
      const int par = q / AW, kk = q % AW, c = kk + 1 - BWP;
      double v = INFINITY;
      if (par == pt && c >= 0 && c < BWP) v = kmin[(size_t)(nt - 1) * BWP + c];
      A[q] = v;
      if (par == pt && c >= 0 && c < RP) R[(size_t)(nt - 1) * RP + c] = c <= B ? v : INFINITY;
    }
  }
  if (nt < 2) return;
  // R_{i+1}[E] for wave 0's classes (b = 0 reads row E itself): the terminal value first
  double rE = E < BWP ? kmin[(size_t)(nt - 1) * BWP + E] : INFINITY;
  int hi = nt - 2, lo = hi - CH + 1 < 0 ? 0 : hi - CH + 1;
  glds_copy_asm(kmin + (size_t)lo * BWP, Kbuf, (hi - lo + 1) * BWP * 8, (int)threadIdx.x, (int)blockDim.x);
  vm_drain();
  lds_barrier();
  for (int q = 0; hi >= 0; ++q) {
    const double *Kc = Kbuf + (size_t)(q & 1) * CH * BWP;
    const int nhi = lo - 1, nlo = nhi - CH + 1 < 0 ? 0 : nhi - CH + 1;
    if (nhi >= 0)
      glds_copy_asm(kmin + (size_t)nlo * BWP, Kbuf + (size_t)((q + 1) & 1) * CH * BWP, (nhi - nlo + 1) * BWP * 8,
                (int)threadIdx.x, (int)blockDim.x);
    for (int i = hi; i >= lo; --i) {
      const double *Ain = A + (size_t)((i + 1) & 1) * AW;
      // wave 0: R_{i+1}[E] from the partials of step i+1 (written before the last barrier)
      if (w == 0 && i + 1 <= nt - 2) {
        const double *pp = part + ((i + 1) & 1) * NW;
        double m = pp[0];
#pragma unroll
        for (int u = 1; u < NW; ++u) m = pvmin(m, pp[u]);
        rE = m;
        if (lane == 0) R[(size_t)(i + 1) * RP + E] = E <= B ? m : INFINITY;
      }
      const double2 *win = reinterpret_cast<const double2 *>(Ain + c0 + BWP - (h + 1) * CB);
      const double2 *kr = reinterpret_cast<const double2 *>(Kc + (size_t)(i - lo) * BWP + h * CB);
      double wv[2 * NP], kv[CB];
#pragma unroll
      for (int p2 = 0; p2 < NP; ++p2) {
        const double2 x = win[p2];
        wv[2 * p2] = x.x;
        wv[2 * p2 + 1] = x.y;
      }
#pragma unroll
      for (int p2 = 0; p2 < CB / 2; ++p2) {
        const double2 y = kr[p2];
        kv[2 * p2] = y.x;
        kv[2 * p2 + 1] = y.y;
      }
      // row E, classes [w·CW, (w+1)·CW): R_{i+1}[E - b] (row E itself from rE)
      double pe = INFINITY;
      {
        const double *ke = Kc + (size_t)(i - lo) * BWP + w * CW;
#pragma unroll
        for (int bb = 0; bb < CW; ++bb) {
          const int b = w * CW + bb;
          const double rv = b == 0 ? rE : Ain[E - b + BWP - 1];
          pe = pvmin(pe, ke[bb] + rv);
        }
      }
      double m0[4] = {INFINITY, INFINITY, INFINITY, INFINITY}, m1[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
#pragma unroll
      for (int b2 = 0; b2 < CB; ++b2) {
        m0[b2 & 3] = pvmin(m0[b2 & 3], kv[b2] + wv[CB - 1 - b2]);
        m1[b2 & 3] = pvmin(m1[b2 & 3], kv[b2] + wv[CB - b2]);
      }
      double r0 = pvmin(pvmin(m0[0], m0[1]), pvmin(m0[2], m0[3]));
      double r1 = pvmin(pvmin(m1[0], m1[1]), pvmin(m1[2], m1[3]));
      r0 = pvmin(r0, pv_dpp<0xB1>(r0));
      r1 = pvmin(r1, pv_dpp<0xB1>(r1));
      r0 = pvmin(r0, pv_dpp<0x4E>(r0));
      r1 = pvmin(r1, pv_dpp<0x4E>(r1));
      double *Aout = A + (size_t)(i & 1) * AW;
      if (h == 0) {
        Aout[c0 + BWP - 1] = r0;
        R[(size_t)i * RP + c0] = c0 <= B ? r0 : INFINITY;
      }
      if (h == 1) {
        Aout[c0 + BWP] = r1;
        R[(size_t)i * RP + c0 + 1] = c0 + 1 <= B ? r1 : INFINITY;
      }
      if (lane == 0) part[(i & 1) * NW + w] = pe;
      lds_barrier();
    }
    vm_drain();
    lds_barrier();
    hi = nhi;
    lo = nlo;
  }
  // R_0[E]
  if (threadIdx.x == 0) {
    double m = part[0];
    for (int u = 1; u < NW; ++u) m = pvmin(m, part[u]);
    R[E] = E <= B ? m : INFINITY;
  }
}

// Row segments on several CUs (few subproblems, classes <= 32): R_i[c] needs R_{i+1}[c - b] for b < BWP <= 32, i.e.
// rows c-31 .. c only, so rows split into segments of 32 (one wave, one workgroup each: lane pair per row, each lane
// half the classes) form a pipeline like k_sdt_run's: segment q runs a step once segment q-1 has published that
// step's rows below it.  Segments hand over in chunks of CH steps: q-1 stores its rows of R (sc1 buffer stores, the
// R array the walk reads anyway), drains, and publishes the chunk's last step (relaxed agent flag); q polls that flag
// one chunk ahead and copies the 32 rows below its own for the next chunk's steps into its LDS ring by LDS-DMA (sc1),
// then computes the chunk with no further waits (MI355X_MICROARCH.md, the measured-valid hand-off).  A wave needs no
// barrier: its LDS accesses execute in order.  Every candidate is the same expression and min is exact, so R is
// bit-identical to k_pinf_recur's.  A wait past the spin limit sets the error word and the host redoes the DP with
// the one-workgroup kernel (check_run).
template <int BWP, int LPR>
__global__ __launch_bounds__(64) void k_pinf_recur_mc(ProblemDev P, PinfDev D, int nseg, int32_t *flags,
                                                      unsigned spin_limit) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  constexpr int CB = BWP / LPR;      // classes per lane
  constexpr int RPS = 64 / LPR;      // rows per segment (one wave)
  constexpr int AS = 32 + RPS;       // step array: the 32 rows below the segment, then its own
  constexpr int CH = PINF_MC_CHUNK;  // steps per hand-off
  static_assert(BWP >= 8 && BWP <= 32 && CB >= 2 && CB % 2 == 0 && (LPR == 2 || LPR == 4 || LPR == 8 || LPR == 16),
                "k_pinf_recur_mc shape");
  const int RP = P.RP, B = P.B, nt = P.nt, K = P.K;
  const int k = (int)blockIdx.x / nseg, q = (int)blockIdx.x - k * nseg;
  const int lane = (int)threadIdx.x, r = lane / LPR, h = lane % LPR, c = RPS * q + r, u = r + 32;
  constexpr int NS = 2 * CH;                     // ring of step arrays
  double *A = sm, *Kbuf = sm + (size_t)NS * AS;  // Kbuf: [2][CH][BWP]
  const double *kmin = D.kmin + (size_t)k * nt * BWP;
  double *R = D.R + (size_t)k * nt * RP;
  // segments' flags packed; the error word where every segmented p = Inf kernel keeps it
  constexpr int FS = 1;
  int32_t *done = flags + (size_t)k * nseg * FS, *err = flags + (size_t)K * nseg * PINF_WS_FLAG_STRIDE;
  const __amdgpu_buffer_rsrc_t Rr = __builtin_amdgcn_make_buffer_rsrc(R, 0, (int)((size_t)nt * RP * 8), 0x00020000);
  auto slot = [&](int s) { return A + (size_t)(s % NS) * AS; };
  // terminal row R_{n-1}[c'] = Kmin_{n-1}[c'] (c' < BWP), the rows below included (a function of kmin: no hand-off)
  for (int e = lane; e < NS * AS; e += 64) A[e] = INFINITY;
  for (int e = lane; e < AS; e += 64) {
    const int cc = RPS * q - 32 + e;
    slot(nt - 1)[e] = cc >= 0 && cc < BWP ? kmin[(size_t)(nt - 1) * BWP + cc] : INFINITY;
  }
  if (h == 0) R[(size_t)(nt - 1) * RP + c] = c <= B && c < BWP ? kmin[(size_t)(nt - 1) * BWP + c] : INFINITY;
  if (nt < 2) return;
  bool stop = false;
  // the segments whose rows lie within 32 below this one (q-1, and q-2 for 16-row segments) have published step s
  // (token nt-1-s); false past the spin limit (err set)
  auto wait_below = [&](int s) {
    const int need = nt - 1 - s;
    for (int d = 1; d * RPS <= 32 && q - d >= 0; ++d) {
      unsigned spins = 0;
      while (__hip_atomic_load(done + (q - d) * FS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || ++spins > spin_limit) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return false;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    return true;
  };
  // the 32 rows below the segment (R_s[RPS·q-32 .. RPS·q-1], rows < 0 stay +Inf) for steps s in [s0, s1] into their
  // ring slots: lane l moves rows RPS·q-32+2l, +1 (16 bytes, LDS-DMA, sc1)
  auto halo = [&](int s0, int s1) {
    if (q == 0) return;
    const int row = RPS * q - 32 + 2 * lane;
    for (int s = s0; s <= s1; ++s) {
      if (lane < 16 && row >= 0) {
        const void *g = pi_uniform(R + (size_t)s * RP);
        const unsigned m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)((__attribute__((address_space(3))) char *)slot(s)));
        const unsigned voff = 8u * (unsigned)row;
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 sc1\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(voff), "s"(g), "s"(m0)
                     : "memory");
      }
    }
  };
  int hi = nt - 2, lo = hi - CH + 1 < 0 ? 0 : hi - CH + 1;
  glds_copy_asm(kmin + (size_t)lo * BWP, Kbuf, (hi - lo + 1) * BWP * 8, lane, 64);
  if (lo + 1 <= nt - 2) {  // the first chunk's rows below (step nt-1's are computed above)
    stop = !wait_below(lo + 1);
    halo(lo + 1, nt - 2);
  }
  vm_drain();
  for (int qq = 0; hi >= 0 && !stop; ++qq) {
    const double *Kc = Kbuf + (size_t)(qq & 1) * CH * BWP;
    const int nhi = lo - 1, nlo = nhi - CH + 1 < 0 ? 0 : nhi - CH + 1;
    if (nhi >= 0) {  // the next chunk: its class rows, and (once the segments below have them) its rows below
      glds_copy_asm(kmin + (size_t)nlo * BWP, Kbuf + (size_t)((qq + 1) & 1) * CH * BWP, (nhi - nlo + 1) * BWP * 8, lane, 64);
      if (!wait_below(nlo + 1)) {
        stop = true;
        break;
      }
      halo(nlo + 1, nhi + 1);
    }
    // this lane's class values of a step (read one step ahead: they are not on the recursion's chain)
    auto kload = [&](double (&kv)[CB], int i) {
      const double2 *kr = reinterpret_cast<const double2 *>(Kc + (size_t)(i - lo) * BWP + CB * h);
#pragma unroll
      for (int t = 0; t < CB / 2; ++t) {
        const double2 y = kr[t];
        kv[2 * t] = y.x;
        kv[2 * t + 1] = y.y;
      }
    };
    // one step: the class values kv of step i (loaded a step earlier), kn <- those of step i-1
    auto step = [&](int i, const double (&kv)[CB], double (&kn)[CB]) {
      asm volatile("" ::: "memory");
      if (i > lo) kload(kn, i - 1);
      const double *Ain = slot(i + 1) + u - CB * h - (CB - 1);  // R_{i+1}[c - CB·h - (CB-1) .. c - CB·h]
      double wv[CB];
#pragma unroll
      for (int t = 0; t < CB; ++t) wv[t] = Ain[t];
      double m[4];  // four accumulators, each started by its first candidate
#pragma unroll
      for (int bb = 0; bb < CB; ++bb) {
        const double cand = kv[bb] + wv[CB - 1 - bb];
        m[bb & 3] = bb < 4 ? cand : pvmin(m[bb & 3], cand);
      }
      double rv;
      if constexpr (CB >= 4)
        rv = pvmin(pvmin(m[0], m[1]), pvmin(m[2], m[3]));
      else
        rv = pvmin(m[0], m[1]);
      rv = pvmin(rv, pv_dpp<0xB1>(rv));                      // the lane group's other class parts
      if constexpr (LPR >= 4) rv = pvmin(rv, pv_dpp<0x4E>(rv));
      if constexpr (LPR >= 8) rv = pvmin(rv, pv_dpp<0x141>(rv));  // row_half_mirror: lane i <-> 7 - i, the other quad
      if constexpr (LPR == 16) rv = pvmin(rv, pv_dpp<0x140>(rv));  // row_mirror: lane i <-> 15 - i, the other half
      // every lane of the row group holds rv: all of them store it (one address per group, so the same lines and
      // bytes move), with no exec-mask switch on the chain (one lane storing: 16.1 ms at C4, all of them: 15.1 ms)
      // (rows above B of the top segment store their finite value too: k_pinf_rfill sets them to +Inf after the
      // launch, and no segment's window reads them)
      slot(i)[u] = rv;
      __builtin_amdgcn_raw_buffer_store_b64((pi_u32x2){(unsigned)__double2loint(rv), (unsigned)__double2hiint(rv)},
                                            Rr, (unsigned)(((size_t)i * RP + c) * 8), 0, 16);
    };
    if constexpr (PINF_MC_SPLIT && LPR == 8) {
      // The chain split in two.  Row c = 8q + r reads R_{i+1}[c - b]: a class b < 8 may read one of the segment's
      // own rows, which the previous step wrote (the step-to-step chain); a class b >= 8 reads only rows below the
      // segment, staged for the whole chunk, so their minimum P_i is computed one step ahead, off the chain.  On the
      // chain, lane h of a row group takes classes 2(h&3) and 2(h&3)+1 (lanes h and h+4 the same two): two DPP
      // steps and the min with P_i, where the one-part form above has three DPP steps after the class sums.  min is
      // exact, so the grouping changes no bit.
      constexpr int CO = (BWP - 8) / 8;  // off-chain classes per lane: 8 + CO·h .. 8 + CO·h + CO - 1
      const int b0 = 2 * (h & 3);
      // class values of step i (reads below the chunk's first step land in the LDS in front of Kc, unused)
      auto kl = [&](double (&kc)[2], double (&kf)[CO], int i) {
        const double *kr = Kc + (i - lo) * BWP;
        const double2 y = *reinterpret_cast<const double2 *>(kr + b0);
        kc[0] = y.x;
        kc[1] = y.y;
#pragma unroll
        for (int t = 0; t < CO; ++t) kf[t] = kr[8 + CO * h + t];
      };
      // the off-chain part from the window R_{i+1}[c - 8 - CO·h - (CO-1) .. c - 8 - CO·h] (wf) and K_i (kf)
      auto offc = [&](const double (&kf)[CO], const double (&wf)[CO]) {
        double p = kf[0] + wf[CO - 1];
#pragma unroll
        for (int t = 1; t < CO; ++t) p = pvmin(p, kf[t] + wf[CO - 1 - t]);
        p = pvmin(p, pv_dpp<0xB1>(p));
        p = pvmin(p, pv_dpp<0x4E>(p));
        return pvmin(p, pv_dpp<0x141>(p));
      };
      auto wload = [&](double (&wf)[CO], int i) {  // R_{i+1} below the segment, for step i's off-chain part
        const double *Af = slot(i + 1) + u - 8 - CO * h - (CO - 1);
#pragma unroll
        for (int t = 0; t < CO; ++t) wf[t] = Af[t];
      };
      // one step: the chain's reads of step i issued first, then the off-chain reads and class values of step i-1
      // (at the chunk's last step they read rows and values the chunk does not use), then P_i from the registers
      // the previous step loaded -- its VALU work fills the wait for the chain's reads -- then the chain
      auto st = [&](int i, const double (&kc)[2], const double (&kf)[CO], const double (&wf)[CO], double (&kcn)[2],
                    double (&kfn)[CO], double (&wfn)[CO]) {
        asm volatile("" ::: "memory");
        const double *Ain = slot(i + 1) + u - b0 - 1;  // R_{i+1}[c - b0 - 1], R_{i+1}[c - b0]
        const double w0 = Ain[0], w1 = Ain[1];
        wload(wfn, i - 1);
        kl(kcn, kfn, i - 1);
        const double P = offc(kf, wf);
        double rv = pvmin(kc[0] + w1, kc[1] + w0);
        rv = pvmin(rv, pv_dpp<0xB1>(rv));
        rv = pvmin(rv, pv_dpp<0x4E>(rv));
        rv = pvmin(rv, P);
        slot(i)[u] = rv;
        __builtin_amdgcn_raw_buffer_store_b64((pi_u32x2){(unsigned)__double2loint(rv), (unsigned)__double2hiint(rv)},
                                              Rr, (unsigned)(((size_t)i * RP + c) * 8), 0, 16);
      };
      double kca[2], kcb[2], kfa[CO], kfb[CO], wa[CO], wb[CO];
      kl(kca, kfa, hi);
      wload(wa, hi);
      for (int i = hi; i >= lo; i -= 2) {
        st(i, kca, kfa, wa, kcb, kfb, wb);
        if (i - 1 >= lo) st(i - 1, kcb, kfb, wb, kca, kfa, wa);
      }
    } else {
      // two steps per trip, the class-value registers alternating (no copies between steps)
      double ka[CB], kb[CB];
      kload(ka, hi);
      for (int i = hi; i >= lo; i -= 2) {
        step(i, ka, kb);
        if (i - 1 >= lo) step(i - 1, kb, ka);
      }
    }
    // this chunk's rows have landed: publish its last step for the segments above
    vm_drain();
    if (lane == 0) __hip_atomic_store(done + q * FS, nt - 1 - lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    hi = nhi;
    lo = nlo;
  }
}

// k_pinf_recur_mc with helper waves (8 lanes per row, 8-row segments, classes 16 or 32): the chain of a step only
// involves the classes b < 8 -- rows of the segment itself, which the previous step wrote; every class b >= 8 reads a
// row below the segment, staged for the whole chunk before the chunk starts.  So the off-chain minima
//   P_i[c] = min_{8 <= b < BWP} fl(Kmin_i[b] + R_{i+1}[c - b])
// of a whole chunk are computed ahead, by three helper waves, while wave 0 runs the previous chunk's chain; they also
// wait for the segments below, copy the chunk's rows below (LDS-DMA, sc1) and its class rows.  Wave 0's step is then
// the on-chain part only (lane h of a row group: classes 2(h&3), 2(h&3)+1, two DPP steps) and one min with P_i from
// the LDS.  min is exact, so R is bit-identical to k_pinf_recur's.  A workgroup barrier per chunk; a failed wait (spin
// limit) stops every wave after it.
template <int BWP>
__global__ __launch_bounds__(256) void k_pinf_recur_mcw(ProblemDev P, PinfDev D, int nseg, int32_t *flags,
                                                       unsigned spin_limit) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  __shared__ int s_stop, s_hsync;
  constexpr int RPS = 8, AS = 32 + RPS, CH = PINF_MC_CHUNK, NS = 2 * CH;
  static_assert(BWP == 16 || BWP == 32, "k_pinf_recur_mcw: classes 16 or 32");
  const int RP = P.RP, B = P.B, nt = P.nt, K = P.K;
  const int k = (int)blockIdx.x / nseg, q = (int)blockIdx.x - k * nseg;
  const int tid = (int)threadIdx.x, w = tid >> 6, lane = tid & 63;
  double *A = sm, *Kbuf = sm + (size_t)NS * AS, *Pbuf = Kbuf + (size_t)2 * CH * BWP;  // Pbuf: [2][CH][RPS]
  const double *kmin = D.kmin + (size_t)k * nt * BWP;
  double *R = D.R + (size_t)k * nt * RP;
  // segments' flags packed; the error word where every segmented p = Inf kernel keeps it
  constexpr int FS = 1;
  int32_t *done = flags + (size_t)k * nseg * FS, *err = flags + (size_t)K * nseg * PINF_WS_FLAG_STRIDE;
  const __amdgpu_buffer_rsrc_t Rr = __builtin_amdgcn_make_buffer_rsrc(R, 0, (int)((size_t)nt * RP * 8), 0x00020000);
  auto slot = [&](int s) { return A + (size_t)(s % NS) * AS; };
  // terminal row R_{n-1}[c'] = Kmin_{n-1}[c'] (c' < BWP), the rows below included (a function of kmin: no hand-off)
  for (int e = tid; e < NS * AS; e += 256) A[e] = INFINITY;
  if (tid == 0) {
    s_stop = 0;
    s_hsync = 0;
  }
  lds_barrier();
  for (int e = tid; e < AS; e += 256) {
    const int cc = RPS * q - 32 + e;
    slot(nt - 1)[e] = cc >= 0 && cc < BWP ? kmin[(size_t)(nt - 1) * BWP + cc] : INFINITY;
  }
  if (tid < RPS) {
    const int c = RPS * q + tid;
    R[(size_t)(nt - 1) * RP + c] = c <= B && c < BWP ? kmin[(size_t)(nt - 1) * BWP + c] : INFINITY;
  }
  lds_barrier();
  if (nt < 2) return;
  // ---- the helpers (waves 1..3, ht = 0..191): chunk [clo, chi] into buffer b ----------------------------------------
  int hgen = 0;  // helper-only syncs so far
  auto hsync = [&]() {  // the three helper waves (an LDS counter: wave 0 does not take part)
    ++hgen;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(&s_hsync, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(&s_hsync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < 3 * hgen)
      __builtin_amdgcn_s_sleep(1);
  };
  auto prepare = [&](int clo, int chi, int b) {
    const int ht = tid - 64;
    glds_copy_asm(kmin + (size_t)clo * BWP, Kbuf + (size_t)b * CH * BWP, (chi - clo + 1) * BWP * 8, ht, 192);
    const int s1 = min(chi + 1, nt - 2);  // the rows below of steps clo+1 .. chi+1 (step nt-1's are the terminal's)
    bool ok = true;
    if (q > 0 && clo + 1 <= s1) {
      // the segments within 32 rows below (q-1 .. q-4) have published step clo+1 (token nt-2-clo)
      const int need = nt - 1 - (clo + 1);
      for (int d = 1; d * RPS <= 32 && q - d >= 0 && ok; ++d) {
        unsigned spins = 0;
        while (__hip_atomic_load(done + (q - d) * FS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
          if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || ++spins > spin_limit) {
            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (lane == 0) s_stop = 1;
            ok = false;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      if (ok) {  // lane l of a helper wave moves rows RPS·q-32+2l, +1 of one step (16 bytes, LDS-DMA, sc1)
        const int row = RPS * q - 32 + 2 * lane;
        for (int s = clo + 1 + (w - 1); s <= s1; s += 3) {
          if (lane < 16 && row >= 0) {
            const void *g = pi_uniform(R + (size_t)s * RP);
            const unsigned m0 =
                __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)((__attribute__((address_space(3))) char *)slot(s)));
            const unsigned voff = 8u * (unsigned)row;
            unsigned keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 sc1\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep)
                         : "v"(voff), "s"(g), "s"(m0)
                         : "memory");
          }
        }
      }
    }
    vm_drain();  // this wave's copies are in the LDS
    hsync();     // ... and every helper wave's
    // P_i[c] for every step of the chunk and row of the segment: (step, row) pairs over the 192 helper lanes
    const double *Kc = Kbuf + (size_t)b * CH * BWP;
    double *Pc = Pbuf + (size_t)b * CH * RPS;
    for (int e = ht; e < (chi - clo + 1) * RPS; e += 192) {
      const int ii = e / RPS, r = e - ii * RPS, i = clo + ii;
      const double *kr = Kc + (size_t)ii * BWP;
      const double *Ab = slot(i + 1) + r + 32;  // R_{i+1}[c - b] = Ab[-b]
      double m[4];
#pragma unroll
      for (int bb = 8; bb < BWP; ++bb) {
        const double cand = kr[bb] + Ab[-bb];
        m[bb & 3] = bb < 12 ? cand : pvmin(m[bb & 3], cand);
      }
      Pc[e] = pvmin(pvmin(m[0], m[1]), pvmin(m[2], m[3]));
    }
  };
  int hi = nt - 2, lo = hi - CH + 1 < 0 ? 0 : hi - CH + 1;
  if (w > 0) prepare(lo, hi, 0);
  lds_barrier();
  bool stop = s_stop != 0;
  // ---- wave 0's lanes: row r = lane / 8 of the segment, h = lane % 8; classes 2(h&3), 2(h&3)+1 ---------------------
  const int r = lane >> 3, h = lane & 7, c = RPS * q + r, u = r + 32, b0 = 2 * (h & 3);
  for (int qq = 0; hi >= 0 && !stop; ++qq) {
    const int nhi = lo - 1, nlo = nhi - CH + 1 < 0 ? 0 : nhi - CH + 1;
    if (w == 0) {
      const double *Kc = Kbuf + (size_t)(qq & 1) * CH * BWP;
      const double *Pc = Pbuf + (size_t)(qq & 1) * CH * RPS;
      // step i's on-chain class values and P (read one step ahead: not on the chain)
      auto ld = [&](double (&kc)[2], double &pv, int i) {
        const double2 y = *reinterpret_cast<const double2 *>(Kc + (size_t)(i - lo) * BWP + b0);
        kc[0] = y.x;
        kc[1] = y.y;
        pv = Pc[(i - lo) * RPS + r];
      };
      auto st = [&](int i, const double (&kc)[2], double pv, double (&kcn)[2], double &pvn) {
        asm volatile("" ::: "memory");
        const double *Ain = slot(i + 1) + u - b0 - 1;  // R_{i+1}[c - b0 - 1], R_{i+1}[c - b0]
        const double w0 = Ain[0], w1 = Ain[1];
        if (i > lo) ld(kcn, pvn, i - 1);
        double rv = pvmin(kc[0] + w1, kc[1] + w0);
        rv = pvmin(rv, pv_dpp<0xB1>(rv));
        rv = pvmin(rv, pv_dpp<0x4E>(rv));
        rv = pvmin(rv, pv);
        slot(i)[u] = rv;
        __builtin_amdgcn_raw_buffer_store_b64((pi_u32x2){(unsigned)__double2loint(rv), (unsigned)__double2hiint(rv)},
                                              Rr, (unsigned)(((size_t)i * RP + c) * 8), 0, 16);
      };
      double ka[2], kb[2], pa, pb;
      ld(ka, pa, hi);
      for (int i = hi; i >= lo; i -= 2) {
        st(i, ka, pa, kb, pb);
        if (i - 1 >= lo) st(i - 1, kb, pb, ka, pa);
      }
      // this chunk's rows have landed: publish its last step for the segments above
      vm_drain();
      if (lane == 0) __hip_atomic_store(done + q * FS, nt - 1 - lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (nhi >= 0) {
      prepare(nlo, nhi, (qq + 1) & 1);
    }
    lds_barrier();
    stop = s_stop != 0;
    hi = nhi;
    lo = nlo;
  }
}

// Narrow class windows (BW <= 8 classes: the SOS1 shapes C1-C3, where k_pinf_recur's per-step LDS round trip and
// barrier are the whole step): row segments of 64 rows, one lane per row, one wave per workgroup, on as many CUs.
// Row c = 64q + l needs R_{i+1}[c - b] for b < CB <= 8 only: inside the segment that is lane l - b's register, reached
// by b chained DPP `wave_shr:1` moves whose lane 0 is filled from the segment below (rows 64q - b, staged for the step
// in the LDS); so a step is CB-1 shifts, CB sums and CB-1 minima on registers, and one R store, with no LDS round trip
// and no barrier on the chain.  The hand-off between segments is k_pinf_recur_mc's (chunks of CH steps: the segment
// below stores its rows, drains, publishes the chunk's last step; this one polls a chunk ahead and copies the 8 rows
// below it for the chunk's steps by LDS-DMA).  Same candidates fl(Kmin_i[b] + R_{i+1}[c - b]), and min is exact: R is
// bit-identical to k_pinf_recur's.  A wait past the spin limit sets the error word (flags[errw]) and the host redoes
// the DP in one workgroup (check_run).
template <int CB>
__device__ __forceinline__ double ws_shr1(double x, double fill) {  // lane l <- lane l-1, lane 0 <- fill
  return __hiloint2double(__builtin_amdgcn_update_dpp(__double2hiint(fill), __double2hiint(x), 0x138, 0xF, 0xF, false),
                          __builtin_amdgcn_update_dpp(__double2loint(fill), __double2loint(x), 0x138, 0xF, 0xF, false));
}
template <int CB>
__global__ __launch_bounds__(64) void k_pinf_recur_ws(ProblemDev P, PinfDev D, int nseg, int32_t *flags, int errw,
                                                      unsigned spin_limit) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  // steps per chunk; rows below the segment kept per step; padding entries in front of a chunk's operands (the reads
  // three steps ahead run up to three steps past the chunk's last step: junk there, never used)
  constexpr int CH = PINF_WS_CHUNK, HB = 8, EP = 4, CE = CH + EP;
  static_assert(CB >= 2 && CB <= HB && CH % 16 == 0, "k_pinf_recur_ws shape");
  const int RP = P.RP, nt = P.nt, BWP = D.BWP;
  const int k = (int)blockIdx.x / nseg, q = (int)blockIdx.x - k * nseg;
  const int lane = (int)threadIdx.x, c = 64 * q + lane;
  // per chunk parity, entry EP + (i - lo) for step i of the chunk [lo, hi]: Hbuf [2][CE][HB] rows 64q-8 .. 64q-1 of
  // step i+1; Kbuf [2][CE][BWP] Kmin_i
  double *Hbuf = sm, *Kbuf = sm + (size_t)2 * CE * HB;
  const double *kmin = D.kmin + (size_t)k * nt * BWP;
  double *R = D.R + (size_t)k * nt * RP;
  // segments' flags PINF_WS_FLAG_STRIDE words apart (mioc_internal.h)
  constexpr int FS = PINF_WS_FLAG_STRIDE;
  int32_t *done = flags + (size_t)k * nseg * FS, *err = flags + errw;
  const __amdgpu_buffer_rsrc_t Rr = __builtin_amdgcn_make_buffer_rsrc(R, 0, (int)((size_t)nt * RP * 8), 0x00020000);
  for (int e = lane; e < 2 * CE * HB; e += 64) Hbuf[e] = INFINITY;  // (segment 0: rows below 0 stay +Inf)
  for (int e = lane; e < 2 * CE * BWP; e += 64) Kbuf[e] = INFINITY;
  double r = c < BWP ? kmin[(size_t)(nt - 1) * BWP + c] : INFINITY;  // this lane's row of R_{i+1}: terminal first
  R[(size_t)(nt - 1) * RP + c] = c <= P.B ? r : INFINITY;
  if (nt < 2) return;
  bool stop = false;
  auto wait_below = [&](int s) {  // segment q-1 has published step s (token nt-1-s); false past the spin limit
    if (q == 0) return true;
    const int need = nt - 1 - s;
    unsigned spins = 0;
    while (__hip_atomic_load(done + (q - 1) * FS, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || ++spins > spin_limit) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    return true;
  };
  // rows 64q-8 .. 64q-1 of R_s for steps s in [s0, s1] into entries s - s0 of `dst` (LDS-DMA, sc1): lane j of
  // instruction t moves 16 bytes of step s0 + 16t + j/4, so one instruction covers 16 steps
  const void *Rg = pi_uniform(R);
  auto halo = [&](int s0, int s1, double *dst) {
    if (q == 0) return;
    for (int t = 0; s0 + 16 * t <= s1; ++t) {
      const int s = s0 + 16 * t + (lane >> 2);
      if (s <= s1) {
        const unsigned m0 = __builtin_amdgcn_readfirstlane(
            (unsigned)(uintptr_t)((__attribute__((address_space(3))) char *)(dst + (size_t)16 * HB * t)));
        const unsigned voff = 8u * (unsigned)((size_t)s * RP + 64 * q - HB + 2 * (lane & 3));
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 sc1\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(voff), "s"(Rg), "s"(m0)
                     : "memory");
      }
    }
  };
  auto kdst = [&](int par) { return Kbuf + (size_t)par * CE * BWP + EP * BWP; };
  auto hdst = [&](int par) { return Hbuf + (size_t)par * CE * HB + EP * HB; };
  // chunks aligned to multiples of CH from step 0: the first (top) one may be short, every later one is full
  int lo = ((nt - 2) / CH) * CH, hi = nt - 2;
  glds_copy_asm(kmin + (size_t)lo * BWP, kdst(0), (hi - lo + 1) * BWP * 8, lane, 64);
  if (lane < HB) {  // the terminal step's rows below, read by step nt-2 (a function of kmin: no hand-off)
    const int cc = 64 * q - HB + lane;
    hdst(0)[(size_t)(hi - lo) * HB + lane] = cc >= 0 && cc < BWP ? kmin[(size_t)(nt - 1) * BWP + cc] : INFINITY;
  }
  if (lo + 1 <= nt - 2) {  // the first chunk's rows below
    stop = !wait_below(lo + 1);
    halo(lo + 1, nt - 2, hdst(0));
  }
  vm_drain();
  // The hand-off without a drain stall: chunk [lo, hi]'s stores are published S steps into the next chunk, after a
  // counted wait that leaves only the S newest stores in flight; the next chunk's DMAs are issued after that publish
  // and completed at the chunk's end by a counted wait that leaves only the stores issued after them in flight.
  constexpr int S = 8;
  static_assert(S == 8 && (CH == 64 || CH == 32), "k_pinf_recur_ws: the counted waits");
  int prev_lo = -1;  // the previous chunk (published S steps into this one)
  for (int qq = 0; hi >= 0 && !stop; ++qq) {
    const double *Kc = Kbuf + (size_t)(qq & 1) * CE * BWP, *Hc = Hbuf + (size_t)(qq & 1) * CE * HB;
    const int nhi = lo - 1, nlo = nhi - CH + 1 < 0 ? 0 : nhi - CH + 1, n = hi - lo + 1;
    // publish the previous chunk, then the next chunk's class rows and (once the segment below has them) its rows below
    auto mid = [&](bool counted) {
      if (prev_lo >= 0) {
        if (counted)
          asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // S: every store but this chunk's first S
        else
          vm_drain();
        if (lane == 0) __hip_atomic_store(done + q * FS, nt - 1 - prev_lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (nhi >= 0) {  // (the poll first: its wait would otherwise also wait for the DMAs)
        if (!wait_below(nlo + 1)) {
          stop = true;
          return;
        }
        glds_copy_asm(kmin + (size_t)nlo * BWP, kdst((qq + 1) & 1), (nhi - nlo + 1) * BWP * 8, lane, 64);
        halo(nlo + 1, nhi + 1, hdst((qq + 1) & 1));
      }
    };
    // a step's operands (broadcast LDS reads, three steps ahead: off the chain): class values Kmin_i[0 .. CB-1] and the
    // fills R_{i+1}[64q - b] (hv[CB - b], b = 1 .. CB-1); i >= lo - 3 (the padding entries)
    struct Op {
      double kv[CB], hv[CB];
    };
    auto opnd = [&](Op &o, int i) {
      const double *kr = Kc + (size_t)(i - lo + EP) * BWP, *hr = Hc + (size_t)(i - lo + EP) * HB + HB - CB;
#pragma unroll
      for (int b = 0; b < CB; ++b) {
        o.kv[b] = kr[b];
        o.hv[b] = hr[b];
      }
    };
    // step i with its operands `o`; `pre` (the previous step's, consumed) takes step i-3's -- unconditionally: a
    // conditional read would leave the compiler's LDS count unknown, and its wait for this step's operands would then
    // also wait for the reads just issued
    auto step = [&](int i, const Op &o, Op &pre) {
      asm volatile("" ::: "memory");
      opnd(pre, i - 3);
      double sft = r, m = o.kv[0] + r;
#pragma unroll
      for (int b = 1; b < CB; ++b) {
        sft = ws_shr1<CB>(sft, o.hv[CB - b]);  // lane l: R_{i+1}[c - b]
        m = pvmin(m, o.kv[b] + sft);
      }
      r = m;
      __builtin_amdgcn_raw_buffer_store_b64((pi_u32x2){(unsigned)__double2loint(r), (unsigned)__double2hiint(r)}, Rr,
                                            (unsigned)(((size_t)i * RP + c) * 8), 0, 16);
    };
    Op o0, o1, o2, o3;
    opnd(o0, hi);
    opnd(o1, hi - 1);
    opnd(o2, hi - 2);
    if (n == CH) {  // a full chunk: groups of four steps, no guards
      // fully unrolled, so that the vector-memory operations between the counted waits are one straight line of
      // stores (tests/test_isa_guard.py checks the counts on the compiled code)
      auto group = [&](int i) {
        step(i, o0, o3);
        step(i - 1, o1, o0);
        step(i - 2, o2, o1);
        step(i - 3, o3, o2);
      };
#pragma unroll
      for (int g = 0; g < S / 4; ++g) group(hi - 4 * g);
      mid(true);  // S steps done
      if (stop) break;
#pragma unroll
      for (int g = S / 4; g < CH / 4; ++g) group(hi - 4 * g);
      if constexpr (CH == 64)
        asm volatile("s_waitcnt vmcnt(56)" ::: "memory");  // CH - S: the next chunk's DMAs have landed
      else
        asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    } else {  // the first chunk, short
      for (int i = hi; i >= lo; i -= 4) {
        step(i, o0, o3);
        if (i - 1 >= lo) step(i - 1, o1, o0);
        if (i - 2 >= lo) step(i - 2, o2, o1);
        if (i - 3 >= lo) step(i - 3, o3, o2);
      }
      mid(false);
      if (stop) break;
      vm_drain();
    }
    prev_lo = lo;
    hi = nhi;
    lo = nlo;
  }
  // the last chunk's rows have landed: publish it (segments above wait for it)
  vm_drain();
  if (!stop && prev_lo >= 0 && lane == 0)
    __hip_atomic_store(done + q * FS, nt - 1 - prev_lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// rows c_from .. RP-1 of R (beyond the rows k_pinf_recur_xr / _mc compute, all above B): +Inf for every step
__global__ void k_pinf_rfill(ProblemDev P, PinfDev D, int c_from) {
  if (P.redo_gate && *P.redo_gate == 0) return;
  const int k = blockIdx.y, RP = P.RP, nt = P.nt, n = RP - c_from;
  double *R = D.R + (size_t)k * nt * RP;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < (size_t)nt * n; e += (size_t)gridDim.x * blockDim.x)
    R[(e / n) * RP + c_from + e % n] = INFINITY;
}

int pinf_chunk_recur(int BWP) { return BWP <= 16 ? 64 : 32; }

namespace {
// k_pinf_recur_mc for one class width: false where the width leaves a lane fewer than two classes
template <int BWP, int LPR>
bool launch_pinf_mc(hipStream_t s, const ProblemDev &P, const PinfDev &D, int nseg, int32_t *flags,
                    unsigned spin_limit, size_t lds) {
  if constexpr (BWP >= 2 * LPR) {
    hipLaunchKernelGGL((k_pinf_recur_mc<BWP, LPR>), dim3(P.K * nseg), dim3(64), lds, s, P, D, nseg, flags, spin_limit);
    return true;
  } else {
    return false;
  }
}
}  // namespace

int pinf_recur_segments(const ProblemDev &P) { return (P.B + 1 + 64 / PINF_RECUR_MC_LANES - 1) / (64 / PINF_RECUR_MC_LANES); }

hipError_t launch_pinf_recur(hipStream_t s, const ProblemDev &P, const PinfDev &D, int ncu, int32_t *flags,
                             unsigned spin_limit, bool *segmented, const char **variant) {
  if (segmented) *segmented = false;
  if (variant) *variant = "k_pinf_recur";
  // few subproblems, classes <= 8, two or more 64-row segments: k_pinf_recur_ws (its error word where the host reads
  // k_pinf_recur_mc's: flags[K·pinf_recur_segments])
  {
    const int nseg = (P.B + 1 + 63) / 64;
    if (PINF_RECUR_WS && flags && segmented && D.BW >= 1 && D.BW <= 8 && D.BWP == 8 && nseg >= 2 &&
        P.K * nseg <= ncu && 64 * nseg <= P.RP && (size_t)P.nt * P.RP * 8 < (1ull << 31)) {
      const int errw = P.K * pinf_recur_segments(P) * PINF_WS_FLAG_STRIDE;
      const size_t lds = (size_t)2 * (PINF_WS_CHUNK + 4) * (8 + D.BWP) * sizeof(double);  // Hbuf, Kbuf
      const dim3 grid(P.K * nseg);
      switch (D.BW < 2 ? 2 : D.BW) {
        case 2: hipLaunchKernelGGL(k_pinf_recur_ws<2>, grid, dim3(64), lds, s, P, D, nseg, flags, errw, spin_limit); break;
        case 3: hipLaunchKernelGGL(k_pinf_recur_ws<3>, grid, dim3(64), lds, s, P, D, nseg, flags, errw, spin_limit); break;
        case 4: hipLaunchKernelGGL(k_pinf_recur_ws<4>, grid, dim3(64), lds, s, P, D, nseg, flags, errw, spin_limit); break;
        case 5: hipLaunchKernelGGL(k_pinf_recur_ws<5>, grid, dim3(64), lds, s, P, D, nseg, flags, errw, spin_limit); break;
        case 6: hipLaunchKernelGGL(k_pinf_recur_ws<6>, grid, dim3(64), lds, s, P, D, nseg, flags, errw, spin_limit); break;
        case 7: hipLaunchKernelGGL(k_pinf_recur_ws<7>, grid, dim3(64), lds, s, P, D, nseg, flags, errw, spin_limit); break;
        default: hipLaunchKernelGGL(k_pinf_recur_ws<8>, grid, dim3(64), lds, s, P, D, nseg, flags, errw, spin_limit); break;
      }
      // rows above B (the top segment's finite values, and the rows no segment computes): +Inf, after the launch
      if (P.B + 1 < P.RP) hipLaunchKernelGGL(k_pinf_rfill, dim3(64, P.K), dim3(256), 0, s, P, D, P.B + 1);
      *segmented = true;
      if (variant) *variant = "k_pinf_recur_ws";
      return hipGetLastError();
    }
  }
  // few subproblems, classes <= 32, tall enough: row segments of 32 on several CUs (k_pinf_recur_mc); the flags
  // (K·nseg·PINF_WS_FLAG_STRIDE + 1 words, zeroed by the caller) carry the hand-off (packed) and, last, the error word
  {
    constexpr int LPR = PINF_RECUR_MC_LANES, RPS = 64 / LPR;  // lanes per row, rows per segment
    const int nseg = (P.B + 1 + RPS - 1) / RPS;
    if (PINF_RECUR_MC && flags && segmented && D.BWP >= 2 * LPR && D.BWP <= 32 && nseg >= 3 && P.K * nseg <= ncu &&
        RPS * nseg <= P.RP && (size_t)P.nt * P.RP * 8 < (1ull << 31)) {
      constexpr int CH = PINF_MC_CHUNK;
      const bool helpers = PINF_MC_HELPERS && LPR == 8 && (D.BWP == 16 || D.BWP == 32);
      const size_t lds = (size_t)(2 * CH * (32 + RPS) + 2 * CH * D.BWP + (helpers ? 2 * CH * RPS : 0)) * sizeof(double);
      bool ok = true;
      if (helpers) {
        if (D.BWP == 16)
          hipLaunchKernelGGL((k_pinf_recur_mcw<16>), dim3(P.K * nseg), dim3(256), lds, s, P, D, nseg, flags, spin_limit);
        else
          hipLaunchKernelGGL((k_pinf_recur_mcw<32>), dim3(P.K * nseg), dim3(256), lds, s, P, D, nseg, flags, spin_limit);
      } else {
        ok = D.BWP == 8    ? launch_pinf_mc<8, LPR>(s, P, D, nseg, flags, spin_limit, lds)
             : D.BWP == 16 ? launch_pinf_mc<16, LPR>(s, P, D, nseg, flags, spin_limit, lds)
                           : launch_pinf_mc<32, LPR>(s, P, D, nseg, flags, spin_limit, lds);
      }
      if (ok) {
        // rows above B (the top segment's finite values, and the rows no segment computes): +Inf, after the launch
        if (P.B + 1 < P.RP) hipLaunchKernelGGL(k_pinf_rfill, dim3(64, P.K), dim3(256), 0, s, P, D, P.B + 1);
        *segmented = true;
        if (variant) *variant = helpers ? "k_pinf_recur_mcw" : "k_pinf_recur_mc";
        return hipGetLastError();
      }
    }
  }
  int pairs = ((P.RP / 2 + 63) / 64) * 64;  // one thread (G = 1) or lane quad (G = 4) per two budget rows
  if (pairs > 512) pairs = 512;
  // few subproblems (fewer workgroups than a quarter of the CUs): four lanes per row pair; a batch keeps one lane
  // (its workgroups already fill the CUs, and the recursion is then bound by the R stores)
  const int G = PINF_RECUR_SPLIT && P.K * 4 <= ncu && D.BWP >= 8 ? PINF_RECUR_G : 1;
  const int CH = pinf_chunk_recur(D.BWP);
  // ... and with B + 1 = 32·8 + 1 (C4), eight waves of row pairs and the extra row split by classes (k_pinf_recur_xr)
  if (PINF_RECUR_XR && G == 4 && D.BWP == 32 && P.B + 1 == 32 * 8 + 1 && 32 * 8 + 1 <= P.RP) {
    const size_t lds = (size_t)(2 * (D.BWP + P.RP) + 2 * CH * D.BWP + 2 * 8) * sizeof(double);
    if (32 * 8 + 1 < P.RP) hipLaunchKernelGGL(k_pinf_rfill, dim3(64, P.K), dim3(256), 0, s, P, D, 32 * 8 + 1);
    hipLaunchKernelGGL((k_pinf_recur_xr<32, 8>), dim3(P.K), dim3(512), lds, s, P, D, CH);
    if (variant) *variant = "k_pinf_recur_xr";
    return hipGetLastError();
  }
  if (G * pairs > 1024) pairs = 1024 / G;
  const int threads = pairs * G;
  size_t lds = (size_t)(2 * (D.BWP + P.RP) + 2 * CH * D.BWP) * sizeof(double);
#define PINF_RECUR(BW)                                                                                    \
  if (G == 4)                                                                                             \
    hipLaunchKernelGGL((k_pinf_recur<BW, 4>), dim3(P.K), dim3(threads), lds, s, P, D, CH);                \
  else if (G == 2)                                                                                        \
    hipLaunchKernelGGL((k_pinf_recur<BW, 2>), dim3(P.K), dim3(threads), lds, s, P, D, CH);                \
  else                                                                                                    \
    hipLaunchKernelGGL((k_pinf_recur<BW, 1>), dim3(P.K), dim3(threads), lds, s, P, D, CH);
  switch (D.BWP) {
    case 8: PINF_RECUR(8) break;
    case 16: PINF_RECUR(16) break;
    case 32: PINF_RECUR(32) break;
    case 64: PINF_RECUR(64) break;
    default: return hipErrorInvalidValue;
  }
#undef PINF_RECUR
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

// zero2 (nullable): two words zeroed by block 0 (the walk's fallback counters); fneed (nullable): the segmented walk's
// flags, fneed[k] by block k and the count fneed[K] by block 0 (fills folded into this launch)
__global__ __launch_bounds__(1024) void k_pinf_start(ProblemDev P, LevelsDev Lv, PinfDev D, int Bu, Start *start,
                                                     int32_t *zero2, int32_t *fneed) {
  if (threadIdx.x == 0) {
    if (fneed) fneed[blockIdx.x] = 0;
    if (blockIdx.x == 0) {
      if (fneed) fneed[P.K] = 0;
      if (zero2) zero2[0] = zero2[1] = 0;
    }
  }
  if (gate_closed(P.gate)) return;
  extern __shared__ __attribute__((aligned(16))) double sR1[];
  __shared__ PKey red[16];
  const int k = blockIdx.x, M = P.M, nt = P.nt;
  Bu = start_budget(P, k, Bu, start);  // <= the launch's Bu, which sized sR1
  if (Bu < 0) return;                  // uniform: an out-of-range B'_k (status MIOC_ESTATE)
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
  // work items (level r, chunk q of the budget range 0..Bu): with few levels (the SOS1 shapes: 2-3 levels, B' ~ 800)
  // one thread per level would scan the whole range alone.  Per level the reference takes the first minimum over c
  // (strict <), then compares (value, grid index, c) across levels: one lexicographic minimum of (key, grid index, c)
  // over every (r, c) is the same cell, so the chunks of a level need no order among themselves.
  const int nq = nt == 1 ? 1 : max(1, min(Bu + 1, (int)blockDim.x / max(1, Lv.L)));
  const int span = (Bu + nq) / nq;  // ceil((Bu + 1) / nq)
  for (int w = threadIdx.x; w < Lv.L * nq; w += blockDim.x) {
    const int r = w / nq, q = w - r * nq;
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
    // first minimum over this chunk's c for this l (strict), then compare (value, grid index, c)
    double bv = INFINITY;
    uint64_t bkey = ~0ull;
    int bc = -1;
    const int c0 = max(b, q * span), c1 = min(Bu, q * span + span - 1);
    for (int c = c0; c <= c1; ++c) {
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
                             Start *start, int32_t *zero2, int32_t *fneed) {
  size_t lds = (size_t)(Bu + 1) * sizeof(double);
  hipLaunchKernelGGL(k_pinf_start, dim3(P.K), dim3(1024), lds, s, P, Lv, D, Bu, start, zero2, fneed);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// forward walk, one workgroup per subproblem: wave 0 walks, all four waves stage.  State at step i:
// (c, l, K_l(i), b̃_l(i), Φ_i[c, l]).
// Lane b examines budget class b of step j = i+1: the levels of the class with K == Kmin give
// Φ_j[c', ·] = V_b = fl(Kmin + R_{j+1}[c' - b]) and the first of them is kfirst; a level with a
// larger K gives at least fl(K2 + R_{j+1}[c' - b]).  If that second value could still satisfy
// fl(K_l + ·) == Φ_i[c, l], the step is resolved by an exact scan over all levels instead.
// Class rows and R rows for CH steps are staged into LDS by LDS-DMA one chunk ahead, and the winner
// is selected with a ballot + readlane (scalar).  Only the window read R_{j+1}[c' - b] depends on the
// walk; the three class-row reads of a step are independent of it and issue beside it.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double readlane_f64(double x, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
  return __hiloint2double(hi, lo);
}

__global__ __launch_bounds__(256) void k_pinf_walk(ProblemDev P, LevelsDev Lv, PinfDev D, const Start *start,
                                                   int32_t *ranks, int32_t *nfallback, const int32_t *need) {
  if (gate_closed(P.gate)) return;
  if (need && need[blockIdx.x] == 0) return;  // walked by the segmented walk
  extern __shared__ __attribute__((aligned(16))) double wsm[];
  const int k = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nthr = blockDim.x;
  const int M = P.M, nt = P.nt, RP = P.RP, BWP = D.BWP, CH = D.CH, W = D.W;
  const bool walker = __builtin_amdgcn_readfirstlane(tid) < 64;  // wave 0 walks (wave-uniform); the others stage
  const Start st = start[k];
  if (st.status != MIOC_OK) return;
  int32_t *rk = ranks + (size_t)k * nt;
  if (tid == 0) rk[0] = st.r;
  if (nt == 1) return;
  // LDS: Rb[2][CH][W], Km[2][CH][BWP], K2[2][CH][BWP] (doubles), Kf[2][CH][BWP] (int32), s_lo[2], s_c[2].
  // Row `row` of a staged chunk holds R_{i0+2+row}[lo, lo + W): whole rows (lo = 0, W = RP), or, when the class
  // window is narrow (SOS1 shapes), a band: the walk's budget only decreases, by at most BW - 1 per step, so a
  // chunk staged while the walk is at budget c (one chunk ahead) reads R_{j+1}[c' - b] with
  // c - 2 CH (BW - 1) - (BWP - 1) <= c' - b <= c.
  double *Rb = wsm;
  double *Km = Rb + 2 * (size_t)CH * W;
  double *K2 = Km + 2 * (size_t)CH * BWP;
  int32_t *Kf = reinterpret_cast<int32_t *>(K2 + 2 * (size_t)CH * BWP);
  int *s_lo = reinterpret_cast<int *>(Kf + 2 * (size_t)CH * BWP);  // [2] band start of each staging buffer
  const double *R = D.R + (size_t)k * nt * RP;
  const size_t crow0 = (size_t)k * nt * BWP;
  const double *dfk = P.df + (size_t)k * nt * M;
  const double *uok = P.uold + (size_t)k * nt * M;
  const double beta = Lv.beta;
  const int nsteps = nt - 1;  // walk steps i = 0 .. nt-2

  auto stage = [&](int q, int buf, int cnow) {
    const int i0 = q * CH;
    const int ni = (i0 + CH <= nsteps ? CH : nsteps - i0);
    // class rows j = i0+1 .. i0+ni
    glds_copy(D.kmin + crow0 + (size_t)(i0 + 1) * BWP, Km + (size_t)buf * CH * BWP, ni * BWP * 8, tid, nthr);
    glds_copy(D.k2 + crow0 + (size_t)(i0 + 1) * BWP, K2 + (size_t)buf * CH * BWP, ni * BWP * 8, tid, nthr);
    glds_copy(D.kfirst + crow0 + (size_t)(i0 + 1) * BWP, Kf + (size_t)buf * CH * BWP, ni * BWP * 4, tid, nthr);
    // R bands of rows j+1 = i0+2 .. i0+ni+1 (row nt does not exist: the terminal step needs none); lo even, so
    // every band starts 16-byte aligned (RP is a multiple of 64)
    int lo = 0;
    if (W < RP) {
      lo = cnow - (W - 2);
      lo = lo < 0 ? 0 : (lo & ~1);
      if (lo + W > RP) lo = RP - W;
    }
    if (tid == 0) s_lo[buf] = lo;
    int nr = ni;
    if (i0 + 1 + nr > nt - 1) nr = nt - 1 - (i0 + 1);
    const int per = (W * 8 + 1023) >> 10;  // 1 KiB pieces per band; a wave copies one piece per instruction
    for (int pc = wave; pc < nr * per; pc += (nthr + 63) >> 6) {
      const int row = pc / per, off = (pc - row * per) * 1024;
      if (off + lane * 16 < W * 8)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void *)((const char *)(R + (size_t)(i0 + 2 + row) * RP + lo) +
                                                             off + lane * 16),
            (__attribute__((address_space(3))) void *)((char *)(Rb + ((size_t)buf * CH + row) * W) + off), 16, 0, 0);
    }
  };

  int r = st.r, c = st.c, br;
  double target = st.phi, Kr;
  {
    const double *nuv = Lv.nuval + (size_t)r * M;
    Kr = p_t1(nuv, dfk, M, P.dt) + beta;
    br = p_bt(nuv, uok, M);
  }
  int fallbacks = 0;
  bool dead = false;
  // s_c[q & 1]: the walk's budget at the start of chunk q, written by the walker at the end of chunk q - 1 and
  // read by every wave when it stages chunk q + 1 (two slots: a wave that stages late cannot see the next value)
  int *s_c = s_lo + 2;
  stage(0, 0, st.c);
  if (tid == 0) s_c[0] = st.c;
  vm_drain();
  lds_barrier();
  const int nq = (nsteps + CH - 1) / CH;
  for (int q = 0; q < nq; ++q) {
    const int buf = q & 1;
    PI_T(w0);
    if (q + 1 < nq) stage(q + 1, buf ^ 1, s_c[q & 1]);
    const int i0 = q * CH, i1 = (i0 + CH <= nsteps ? i0 + CH : nsteps);
    const double *KmB = Km + (size_t)buf * CH * BWP;
    const double *K2B = K2 + (size_t)buf * CH * BWP;
    const int32_t *KfB = Kf + (size_t)buf * CH * BWP;
    const double *RbB = Rb + (size_t)buf * CH * W;
    const int blo = s_lo[buf];
    const unsigned long long clsm = BWP >= 64 ? ~0ull : (1ull << BWP) - 1;  // the lanes that are classes
    // one walk step; TERM: the terminal step j = nt - 1 (compiled apart, so the other steps carry no term selects)
    auto step = [&](int i, auto TERM) {
      const int row = i - i0, j = i + 1, cp = c - br;
      constexpr bool term = decltype(TERM)::value;  // the last step (j = nt - 1): its own instance
      // Branch-free: every lane reads an in-bounds slot and masks afterwards.  The class row does not
      // depend on the walk, so its three reads issue beside the window read.
      const int lb = lane & (BWP - 1), xi = cp - lane;
      const double kmr = KmB[row * BWP + lb];
      const double k2r = K2B[row * BWP + lb];
      const int kfr = KfB[row * BWP + lb];
      const int xo = xi - blo;
      const double xr = RbB[(size_t)row * W + (xo > 0 ? (xo < W ? xo : W - 1) : 0)];
      // lanes >= BWP compute on wrapped class slots; their bits leave the ballots (clsm) instead of masked values
      const double km = kmr, k2 = k2r;
      const int kf = kfr;
      const double x = term ? (lane == cp ? 0.0 : INFINITY) : (xi >= 0 ? xr : INFINITY);
      const bool ok = km < INFINITY && x < INFINITY;
      const double V = term ? km : km + x;
      const double V2 = term ? k2 : k2 + x;
      const bool match = ok && (Kr + V == target);
      const bool amb = match && k2 < INFINITY && (Kr + V2 == target);
      const unsigned long long mm = __ballot(match) & clsm;
      const unsigned long long am = __ballot(amb) & clsm;
      int win, winb;
      double winV, winK;
      if (mm != 0 && am == 0) {
        winb = __builtin_ffsll((long long)mm) - 1;
        win = __builtin_amdgcn_readlane(kf, winb);
        for (unsigned long long rest = mm & (mm - 1); rest; rest &= rest - 1) {
          const int l2 = __builtin_ffsll((long long)rest) - 1;
          const int f2 = __builtin_amdgcn_readlane(kf, l2);
          if (f2 < win) {
            win = f2;
            winb = l2;
          }
        }
        winV = readlane_f64(V, winb);
        winK = readlane_f64(km, winb);
      } else {
        // exact scan of row c' of Φ_j: first rank s with fl(K_l + Φ_j[c', s]) == Φ_i[c, l]
        // (kf used on this path too: otherwise the compiler sinks its LDS read into the branch above, one more LDS
        // round trip on the walk's chain every step)
        asm volatile("" ::"v"(kf));
        ++fallbacks;
        const double *dfj = dfk + (size_t)j * M;
        const double *uoj = uok + (size_t)j * M;
        int sbest = INT_MAX, sb = -1;
        double sV = INFINITY, sK = INFINITY;
        for (int s = lane; s < Lv.L; s += 64) {
          const double *nuv = Lv.nuval + (size_t)s * M;
          const int bs = p_bt(nuv, uoj, M);
          const double t1 = p_t1(nuv, dfj, M, P.dt);
          double val = INFINITY, Ks = t1;
          if (term) {
            if (bs == cp) val = t1;
          } else {
            Ks = t1 + beta;
            if (cp >= bs && bs < BWP) val = Ks + RbB[(size_t)row * W + cp - bs - blo];
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
        if (bal == 0) {  // inconsistent tables: cannot happen for a consistent DP
          if (lane == 0) atomicAdd(nfallback + 1, 1);
          dead = true;  // stop walking, but keep joining the staging barriers
          return;
        }
        const int src = __builtin_ffsll((long long)bal) - 1;
        win = m2;
        winV = readlane_f64(sV, src);
        winK = readlane_f64(sK, src);
        winb = __builtin_amdgcn_readlane(sb, src);
      }
      if (lane == 0) rk[j] = win;
      r = win;
      c = cp;
      target = winV;
      Kr = winK;
      br = winb;
    };
    for (int i = i0; walker && !dead && i < i1; ++i) {
      if (i == nt - 2)
        step(i, std::true_type{});
      else
        step(i, std::false_type{});
    }
    PI_T(w1);
    if (tid == 0) s_c[(q + 1) & 1] = c;  // the walker's budget for the next staging decision
    vm_drain();
    lds_barrier();
#ifdef MIOC_STAMPS
    PI_T(w2);
    if (blockIdx.x == 0 && tid == 0) {  // walker: [8][0] staging issue + steps, [8][1] chunk-end wait
      g_pinf_stamps[8][0] += w1 - w0;
      g_pinf_stamps[8][1] += w2 - w1;
      g_pinf_stamps[8][2] += 1;
      g_pinf_stamps[8][3] += i1 - i0;
    }
#endif
  }
  (void)r;
  if (tid == 0 && fallbacks) atomicAdd(nfallback, fallbacks);
}

// ---------------------------------------------------------------------------------------------
// Segmented walk (many CUs for one subproblem).  The walker's decision at step j depends on its state
// (K_l of the level it stands on, Φ_i[c, l]) only through rounding: the target is Φ_i[c, l] =
// fl(K_l + R_j[c']) with c' = c - b̃_l, so a class b matches iff fl(K_l + V_b) == fl(K_l + R_j[c']) with
// V_b = fl(Kmin_j[b] + R_{j+1}[c' - b]) and R_j[c'] = min_b V_b.  Every class with V_b == R_j[c'] matches for
// any K_l; a class with V_b > R_j[c'] matches for none once V_b - R_j[c'] exceeds the rounding unit of
// |K_l| + max(|V_b|, |R|) (bounded with kabs_{j-1} >= |K_l|), and the same bound on the class's second value
// V2_b excludes the exact-scan case.  Where all classes of row c' are that clear, the winner -- the first
// rank among the classes at the minimum -- is a function of (j, c') alone: the class table ftab.  The path
// then is the chain c'_{j+1} = c'_j - b*(j, c'_j), which composes over segments of G steps in parallel
// (k_pinf_fseg: every entry row of every segment), is chained serially over the nseg segments, and is
// expanded per segment (k_pinf_fexpand).  A chain that meets a state-dependent row leaves its subproblem to
// the serial walk (k_pinf_walk gated by fneed), so the ranks equal the serial walk's always.
// ---------------------------------------------------------------------------------------------
// fts steps per workgroup (ftab_steps): rows R_j .. R_{j+fts} staged once (consecutive steps share them).  The row
// minimum R_j[c'] = min_b fl(Kmin_j[b] + R_{j+1}[c' - b]) is the recursion's own output, read instead of recomputed
// (the same candidates and an exact min: the same double).
int ftab_steps(int RP) { return std::max(1, std::min(8, 65536 / (RP * 8) - 1)); }
size_t ftab_lds(int RP, int BWP) {
  const int f = ftab_steps(RP);
  return ((size_t)(f + 1) * RP + 2 * (size_t)f * BWP) * sizeof(double) + (size_t)f * BWP * sizeof(int);
}
__global__ __launch_bounds__(256) void k_pinf_ftab(ProblemDev P, PinfDev D, int fts) {
  if (gate_closed(P.gate)) return;
  extern __shared__ __attribute__((aligned(16))) double fsm[];
  const int k = blockIdx.y, nt = P.nt, RP = P.RP, B = P.B, BWP = D.BWP, BW = D.BW;
  const int j0 = 1 + (int)blockIdx.x * fts, n = min(fts, nt - j0);  // steps j0 .. j0 + n - 1
  double *Rs = fsm;                                                // rows j0 .. j0 + n (the last if < nt)
  double *km = Rs + (size_t)(fts + 1) * RP, *k2 = km + fts * BWP;
  int *kf = reinterpret_cast<int *>(k2 + fts * BWP);
  const int nrow = j0 + n <= nt - 1 ? n + 1 : n;
  const double *Rk = D.R + (size_t)k * nt * RP;
  for (int e = threadIdx.x; e < nrow * RP; e += blockDim.x) Rs[e] = Rk[(size_t)j0 * RP + e];
  const size_t crow = ((size_t)k * nt + j0) * BWP;
  for (int e = threadIdx.x; e < n * BWP; e += blockDim.x) {
    km[e] = D.kmin[crow + e];
    k2[e] = D.k2[crow + e];
    kf[e] = D.kfirst[crow + e];
  }
  __syncthreads();
  for (int s = 0; s < n; ++s) {
    const int j = j0 + s;
    const bool term = (j == nt - 1);
    const double *Rj = Rs + (size_t)s * RP, *Rn = Rj + RP, *kmj = km + s * BWP, *k2j = k2 + s * BWP;
    const int *kfj = kf + s * BWP;
    const double kab = D.kabs[(size_t)k * nt + j - 1];
    uint8_t *out = D.ftab + ((size_t)k * nt + j) * RP;
    for (int cp = threadIdx.x; cp < RP; cp += blockDim.x) {
      unsigned res = 0xFFu;
      const double R = cp <= B ? Rj[cp] : INFINITY;
      if (R < INFINITY) {
        bool safe = true;
        int best = INT_MAX, bb = -1;
        for (int b = 0; b < BW; ++b) {
          const double x = term ? (b == cp ? 0.0 : INFINITY) : (cp - b >= 0 ? Rn[cp - b] : INFINITY);
          if (!(kmj[b] < INFINITY && x < INFINITY)) continue;
          const double V = term ? kmj[b] : kmj[b] + x;
          if (V == R) {
            if (kfj[b] < best) best = kfj[b], bb = b;
            if (k2j[b] < INFINITY) {  // a level of the class with a larger K must not round onto the target
              const double V2 = term ? k2j[b] : k2j[b] + x;
              if (!(V2 - R > (kab + fmax(fabs(R), fabs(V2))) * 0x1p-50)) safe = false;
            }
          } else if (!(V - R > (kab + fmax(fabs(R), fabs(V))) * 0x1p-50)) {
            safe = false;
          }
        }
        if (safe && bb >= 0 && best >= 0) res = (unsigned)bb;
      }
      out[cp] = (uint8_t)res;
    }
  }
}

// The chains of the segmented walk are dependent reads of ftab, one byte per step; read from global memory each step is
// a round trip (≈0.3 µs).  So a segment's class rows are staged into the LDS, FCH rows at a time (coalesced 16-byte
// copies), and the chains step through the LDS.
constexpr int kFwalkLds = 64 * 1024;  // LDS bytes of staged class rows per workgroup
__device__ __forceinline__ int fwalk_rows(int RP) { return kFwalkLds / RP; }
// rows j0 .. j0 + n - 1 of subproblem k's class table into `dst` (RP bytes each; RP is a multiple of 64)
__device__ __forceinline__ void fwalk_stage(const uint8_t *tab, int RP, int j0, int n, uint8_t *dst) {
  const uint4 *src = reinterpret_cast<const uint4 *>(tab + (size_t)j0 * RP);
  uint4 *d = reinterpret_cast<uint4 *>(dst);
  const int n16 = n * RP / 16;
  for (int e = threadIdx.x; e < n16; e += blockDim.x) d[e] = src[e];
}

// composed map of segment g: the row after steps j0 .. j1 for every entry row (one thread per entry row; B + 1 <= 8192)
__global__ __launch_bounds__(1024) void k_pinf_fseg(ProblemDev P, PinfDev D, int G, int nseg) {
  if (gate_closed(P.gate)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t frow[];
  const int g = blockIdx.x, k = blockIdx.y, nt = P.nt, RP = P.RP, B = P.B, FCH = fwalk_rows(RP);
  const int j0 = 1 + g * G, j1 = (j0 + G - 1 < nt - 1 ? j0 + G - 1 : nt - 1);
  const uint8_t *tab = D.ftab + (size_t)k * nt * RP;
  constexpr int PER = 8;
  int cs[PER];
#pragma unroll
  for (int e = 0; e < PER; ++e) cs[e] = (int)threadIdx.x + e * (int)blockDim.x;
  for (int jb = j0; jb <= j1; jb += FCH) {
    const int n = min(FCH, j1 - jb + 1);
    __syncthreads();  // every chain is past the previous chunk
    fwalk_stage(tab, RP, jb, n, frow);
    __syncthreads();
#pragma unroll
    for (int e = 0; e < PER; ++e) {
      int cc = cs[e];
      if ((int)threadIdx.x + e * (int)blockDim.x > B || cc < 0) continue;
      for (int j = jb; j < jb + n; ++j) {
        const unsigned bb = frow[(size_t)(j - jb) * RP + cc];
        if (bb == 0xFFu) {
          cc = -1;
          break;
        }
        if (j < nt - 1) cc -= (int)bb;
      }
      cs[e] = cc;
    }
  }
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int cp0 = (int)threadIdx.x + e * (int)blockDim.x;
    if (cp0 <= B) D.fseg[((size_t)k * nseg + g) * RP + cp0] = cs[e];
  }
}

// one workgroup per (segment g, subproblem): thread 0 chains the segment maps from the start cell through segment g
// (the chain must exist through this segment's own steps; the last segment's workgroup thereby checks the whole chain
// and owns the verdict: fneed[k] = 1 hands the subproblem to the serial walk), then walks the segment's steps through
// its staged class rows, and every thread writes the ranks of the steps
constexpr int kFexpandSteps = 512;  // steps staged per round (the classes of a round in s_b)
__global__ __launch_bounds__(256) void k_pinf_fexpand(ProblemDev P, LevelsDev Lv, PinfDev D, const Start *start,
                                                      int32_t *ranks, int G, int nseg) {
  if (gate_closed(P.gate)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t frow[];
  __shared__ int s_ok, s_c;
  __shared__ uint8_t s_b[kFexpandSteps];
  const int g = blockIdx.x, k = blockIdx.y, nt = P.nt, RP = P.RP, M = P.M;
  const int FCH = min(fwalk_rows(RP), kFexpandSteps);
  const Start st = start[k];
  if (st.status != MIOC_OK || nt == 1) {  // nothing to walk: the serial walk returns at once as well
    if (threadIdx.x == 0 && g == nseg - 1) {
      D.fneed[k] = 0;
      if (st.status == MIOC_OK) ranks[(size_t)k * nt] = st.r;
    }
    return;
  }
  if (threadIdx.x == 0) {
    int cp = st.c - p_bt(Lv.nuval + (size_t)st.r * M, P.uold + (size_t)k * nt * M, M);
    int ok = cp >= 0 && cp <= P.B, entry = -1;
    for (int h = 0; ok && h <= g; ++h) {
      if (h == g) entry = cp;
      cp = D.fseg[((size_t)k * nseg + h) * RP + cp];
      ok = cp >= 0;
    }
    if (g == nseg - 1) {
      D.fneed[k] = !ok;
      if (!ok) atomicAdd(D.fneed + P.K, 1);
      else ranks[(size_t)k * nt] = st.r;
    }
    s_ok = ok;
    s_c = entry;
  }
  __syncthreads();
  if (!s_ok) return;
  const int j0 = 1 + g * G, j1 = (j0 + G - 1 < nt - 1 ? j0 + G - 1 : nt - 1);
  const uint8_t *tab = D.ftab + (size_t)k * nt * RP;
  const int32_t *kfk = D.kfirst + (size_t)k * nt * D.BWP;
  int32_t *rk = ranks + (size_t)k * nt;
  int c = s_c;
  for (int jb = j0; jb <= j1; jb += FCH) {
    const int n = min(FCH, j1 - jb + 1);
    __syncthreads();
    fwalk_stage(tab, RP, jb, n, frow);
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int j = jb; j < jb + n; ++j) {
        const int b = (int)frow[(size_t)(j - jb) * RP + c];  // not 0xFF: the chain through this segment exists
        s_b[j - jb] = (uint8_t)b;
        c -= b;
      }
    }
    __syncthreads();
    for (int j = jb + (int)threadIdx.x; j < jb + n; j += blockDim.x) rk[j] = kfk[(size_t)j * D.BWP + s_b[j - jb]];
  }
}

// G: steps per segment, about 2·sqrt(nt) (the chain over the segment maps is a global read per segment, a segment's
// own steps are LDS reads), a power of two in [64, 4096], and at most 4096 segments
void pinf_fplan(int nt, int *G, int *nseg) {
  const int steps = nt > 1 ? nt - 1 : 1;
  int g = 64;
  while (g < 4096 && (double)g * g < 4.0 * steps) g *= 2;
  while ((steps + g - 1) / g > 4096) g *= 2;
  *G = g;
  *nseg = (steps + g - 1) / g;
}

hipError_t launch_pinf_fwalk(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PinfDev &D,
                             const Start *start, int32_t *ranks) {
  if (D.BWP > 64 || P.B + 1 > P.RP) return hipErrorInvalidValue;
  int G, nseg;
  pinf_fplan(P.nt, &G, &nseg);
  if (P.nt > 1) {
    const int fts = ftab_steps(P.RP);
    hipLaunchKernelGGL(k_pinf_ftab, dim3((P.nt - 1 + fts - 1) / fts, P.K), dim3(256), ftab_lds(P.RP, D.BWP), s, P, D,
                       fts);
    const size_t flds = (size_t)(kFwalkLds / P.RP) * P.RP;  // fwalk_rows(RP) staged class rows
    hipLaunchKernelGGL(k_pinf_fseg, dim3(nseg, P.K), dim3(1024), flds, s, P, D, G, nseg);
    hipLaunchKernelGGL(k_pinf_fexpand, dim3(nseg, P.K), dim3(256), flds, s, P, Lv, D, start, ranks, G, nseg);
  } else {
    hipLaunchKernelGGL(k_pinf_fexpand, dim3(1, P.K), dim3(256), 0, s, P, Lv, D, start, ranks, G, nseg);
  }
  return hipGetLastError();
}

// The walk's chunk and LDS row width: a band covering two chunks of budget descent plus one class window when that
// is at most half a row (the narrow class windows of SOS1 problems: C1-C3 have BW = 4, W = 106 of RP = 832), else
// whole rows with the largest chunk that fits 96 KB.
void pinf_plan(int RP, int nt, PinfDev &D) {
  (void)nt;
  const int ch = 16, w = (2 * ch * (D.BW - 1) + D.BWP + 2 + 1) & ~1;
  if (2 * w <= RP) {
    D.CH = ch;
    D.W = w;
    return;
  }
  const int per = RP * 8 + D.BWP * 20;  // bytes per staged step
  int c = (96 * 1024) / (2 * per);
  D.CH = c < 1 ? 1 : (c > 32 ? 32 : c);
  D.W = RP;
}

hipError_t launch_pinf_walk(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PinfDev &D,
                            const Start *start, int32_t *ranks, int32_t *nfallback, const int32_t *need) {
  if (D.BWP > 64 || D.CH < 1 || D.W < 2) return hipErrorInvalidValue;
  size_t lds = (size_t)2 * D.CH * ((size_t)D.W * 8 + (size_t)D.BWP * 20) + 32;
  hipLaunchKernelGGL(k_pinf_walk, dim3(P.K), dim3(256), lds, s, P, Lv, D, start, ranks, nfallback, need);
  return hipGetLastError();
}

#ifdef MIOC_STAMPS
extern "C" int32_t mioc_debug_pinf_stamps(unsigned long long *out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pinf_stamps), sizeof(g_pinf_stamps)) == hipSuccess ? 0 : -4;
}
#endif

}  // namespace mioc
