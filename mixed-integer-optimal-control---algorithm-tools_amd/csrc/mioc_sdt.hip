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
// Two drivers: one launch per step (k_sdt_step), or the whole DP as one persistent launch (k_sdt_run) whose
// workgroups hand rows to each other through per-row flags.
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
constexpr int SD_SPARSE = 4;             // rows with at most this many finite sources: direct minimum over them
constexpr int SD_LCAP = 512;             // listed targets kept in LDS; beyond, the scan sweeps every rank
constexpr int SD_BLAG = 2;               // persistent kernel: row B runs this many steps behind row 0
#ifndef SDT_RUN_MINW
#define SDT_RUN_MINW 2                   // persistent kernel: waves per SIMD the registers must allow (4: two workgroups per CU, but the row code then spills)
#endif
#ifndef SDT_PREFETCH
#define SDT_PREFETCH 1                   // load the sphere orders ahead of the dependency wait
#endif

// Diagnostic build only (make stamps -> libmioc_stamps.so): per-workgroup phase clocks of the last launch.
#if defined(MIOC_STAMPS) && !defined(MIOC_STAMPS_TL)
// phase clocks are kept in LDS (a global store would join the vmcnt queue and delay the row's own
// loads) and copied out once per row: g_sdt_stamps[workgroup] = the last row it processed
__device__ unsigned long long g_sdt_stamps[4096][16];
#define SD_STAMP(k)                                                                          \
  do {                                                                                       \
    if (threadIdx.x == 0) sh.stamp[k] = __builtin_amdgcn_s_memtime();                         \
  } while (0)
#define SD_RSTAMP(k)                                                                         \
  do {                                                                                       \
    if (threadIdx.x == 0) sh.stamp[k] = __builtin_amdgcn_s_memrealtime();                     \
  } while (0)
#define SD_FLUSH()                                                                           \
  do {                                                                                       \
    if (threadIdx.x == 0)                                                                    \
      for (int _q = 0; _q < 16; ++_q) g_sdt_stamps[blockIdx.x][_q] = sh.stamp[_q];           \
  } while (0)
#define SD_TL(k) \
  do {           \
  } while (0)
#elif defined(MIOC_STAMPS)
// persistent-kernel timeline (diagnostic build, make stamps_tl): per row, for steps i < 64: wait begin, wait
// end (after the barrier), row body end, done published -- s_memrealtime (100 MHz); no in-row stamps
__device__ unsigned long long g_sdt_tl[4096][64][4];
#define SD_TL(k)                                                                                          \
  do {                                                                                                    \
    if (threadIdx.x == 0 && g < 4096 && (unsigned)i < 64u) g_sdt_tl[g][i][k] = __builtin_amdgcn_s_memrealtime();    \
  } while (0)
#define SD_STAMP(k) \
  do {              \
  } while (0)
#define SD_RSTAMP(k) \
  do {               \
  } while (0)
#define SD_FLUSH() \
  do {             \
  } while (0)
#else
#define SD_TL(k) \
  do {           \
  } while (0)
#define SD_STAMP(k) \
  do {              \
  } while (0)
#define SD_RSTAMP(k) \
  do {               \
  } while (0)
#define SD_FLUSH() \
  do {             \
  } while (0)
#endif

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

// L1 distance between two ranks of the 8^M grid with one v_sad_u8: a rank spread to one byte per dimension
__device__ __forceinline__ unsigned sd_bytes(unsigned r) {
  return (r & 7u) | ((r & 0x38u) << 5) | ((r & 0x1C0u) << 10) | ((r & 0xE00u) << 15);
}
__device__ __forceinline__ unsigned sd_l1(unsigned pa, unsigned pb) { return __builtin_amdgcn_sad_u8(pa, pb, 0u); }

// Exact scan of the listed targets: the reference loop (HelpFunctions.jl:60-77) for one cell each.
// COOP: the whole workgroup scans one target at a time (thread t: sources t + T·s, ascending), then a
// (value, rank) minimum, ties to the lower rank.  Otherwise one wave per target (lane: sources
// lane + 64·t); list == nullptr scans every rank whose outnat slot is NaN.  Writes U (finite minimum, into the
// LDS U row) and the value (+Inf if none) into outnat.
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
      const unsigned dpre = sd_l1(sd_bytes(tid), sd_bytes(r & ((1 << (3 * (M - 1))) - 1)));
      double bv = INFINITY;
      int bj = -1;
#pragma unroll
      for (int s = 0; s < 8; ++s) {
        const int j = tid + T * s;
        const double val = (t1 + beta * (double)(dpre + (unsigned)abs(s - xl[M - 1]))) + psi[j];
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
      const int r = list ? (int)list[e] : e;
      if (!list && !__builtin_isnan(outnat[r])) continue;  // overflowed list: every NaN-marked rank
      int xl[M];
      const double t1 = target(r, xl);
      const unsigned pr = sd_bytes(r);
      double bv = INFINITY;
      int bj = -1;
      for (int t = 0; t < L / 64; ++t) {
        const int j = lane + 64 * t;
        const unsigned d = sd_l1(sd_bytes(j), pr);
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

// Global traffic of a row.  The per-step kernel uses plain loads and stores (kernel boundaries order the
// steps).  The persistent kernel hands rows between workgroups inside one launch (MI355X_MICROARCH.md,
// visibility: payload stored write-through `sc1` and drained, flag stored `sc1`, every load of handed-off
// bytes an `sc1` load), so there its staging loads and stores are `sc1` buffer loads / stores (aux 16),
// 16 bytes per lane where the layout allows (narrow `sc1` stores cost 2-3x per byte and write partial lines).
// `base` is wave-uniform (a subproblem's staging block or one row of it), `bytes` its extent (< 2^31).
typedef unsigned int sd_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int sd_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sd_rsrc(const double *base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(base), 0, bytes, 0x00020000);
}
template <bool SC1>
__device__ __forceinline__ double sd_load8(const double *base, int bytes, int e) {
  if constexpr (SC1) {
    const sd_u32x2 w = __builtin_amdgcn_raw_buffer_load_b64(sd_rsrc(base, bytes), e * 8, 0, 16);
    return __hiloint2double((int)w.y, (int)w.x);
  } else {
    return base[e];
  }
}
// Ψ at elements ea (even) and eb of a staging block: eb = ea + 1 (one 16-byte load) unless the pair straddles
// a sphere boundary, i.e. its two positions come from different rows (then a second, 8-byte load)
template <bool SC1>
__device__ __forceinline__ void sd_load_pair(const double *base, int bytes, int ea, int eb, double &va, double &vb) {
  if constexpr (SC1) {
    const sd_u32x4 t = __builtin_amdgcn_raw_buffer_load_b128(sd_rsrc(base, bytes), ea * 8, 0, 16);
    va = __hiloint2double((int)t.y, (int)t.x);
    vb = __hiloint2double((int)t.w, (int)t.z);
  } else {
    const double2 t = *reinterpret_cast<const double2 *>(base + ea);
    va = t.x;
    vb = t.y;
  }
  if (eb != ea + 1) vb = sd_load8<SC1>(base, bytes, eb);
}
template <bool SC1>
__device__ __forceinline__ void sd_store16(double *base, int bytes, int e, unsigned long long lo,
                                           unsigned long long hi) {
  if constexpr (SC1) {
    const sd_u32x4 d = {(unsigned)lo, (unsigned)(lo >> 32), (unsigned)hi, (unsigned)(hi >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(d, sd_rsrc(base, bytes), e * 8, 0, 16);
  } else {
    *reinterpret_cast<ulonglong2 *>(base + e) = make_ulonglong2(lo, hi);
  }
}

template <int NW>
struct SdtShared {
  double redv[SD_COOP * NW];
  int redj[SD_COOP * NW];
  double rmn[NW], rmx[NW];
  int rnv[NW];
  int nlist;
  int stop;  // persistent kernel: a dependency wait timed out
  unsigned long long stamp[16];  // diagnostic build: phase clocks of the current row
  int nsp;   // sparse rows: the finite sources (rank, Ψ)
  int spj[SD_SPARSE];
  double spv[SD_SPARSE];
};

// The sphere orders a step reads (step i+1, for the sources) and writes (step i, for the output row), as the
// position pairs 2(tid + T·q) + {0, 1} of this thread, plus both heads (position 0).  Loaded at the start of
// a row (per-step kernel) or ahead of the dependency wait (persistent kernel): they are static, so their
// latency never sits behind a barrier.
struct SdPerm {
  uint2 in[4], out[4];
  uint32_t hin, hout;
};
template <int M>
__device__ __forceinline__ void sd_perm_load(SdPerm &pm, const uint32_t *__restrict__ perm_all, int nt, int k,
                                             int i) {
  constexpr int T = 1 << (3 * M - 3);
  const uint32_t *pin = perm_all + ((size_t)k * nt + i + 1) * ((size_t)T * 8);
  const uint32_t *pout = perm_all + ((size_t)k * nt + i) * ((size_t)T * 8);
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    pm.in[q] = *reinterpret_cast<const uint2 *>(pin + 2 * (tid + T * q));
    pm.out[q] = *reinterpret_cast<const uint2 *>(pout + 2 * (tid + T * q));
  }
  pm.hin = pin[0];
  pm.hout = pout[0];
}

// One source row c' of step i for subproblem k: reads S_{i+1} (Sin), writes row c' of S_i (Sout) and of
// UU_i.  `loaded` (persistent kernel): flag stored once this row's reads of S_{i+1} are complete.
template <int M, bool PERSIST>
__device__ __forceinline__ void sdt_row(const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G, int k, int cp,
                                        int i, const SdPerm &pm, const double *Sin_all,
                                        double *Sout_all, uint16_t *__restrict__ UU_all, size_t s_stride,
                                        size_t uu_stride_k, int32_t *__restrict__ counters,
                                        SdtShared<(1 << (3 * M - 3)) / 64> &sh, unsigned char *sds, int32_t *loaded,
                                        int token) {
  constexpr int L = 1 << (3 * M), T = L / 8, NW = T / 64, Smax = 7 * M;
  double *psi = reinterpret_cast<double *>(sds);        // [L] Ψ_j by rank
  double *dtv = psi + L;                                // [L] transform values (swizzled), then outputs (natural)
  uint16_t *uu = reinterpret_cast<uint16_t *>(dtv + L);  // [L] the U row (natural order)
  uint16_t *list = uu + L;                              // [SD_LCAP] targets for the exact scan
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int B = P.B;
  const double beta = Lv.beta;
  const double *Sin = Sin_all + (size_t)k * s_stride;
  double *Sout = Sout_all + (size_t)k * s_stride + (size_t)cp * L;
  uint16_t *UU = UU_all + (size_t)k * uu_stride_k + (size_t)i * ((size_t)(B + 1) * L) + (size_t)cp * L;
  const double *dfi = P.df + ((size_t)k * P.nt + i) * M;
  const double *uoi = P.uold + ((size_t)k * P.nt + i) * M;
  const uint2 *ein = pm.in, *eout = pm.out;
  SD_RSTAMP(13);
  SD_STAMP(0);

  // ---- sources: Ψ_j = Φ_{i+1}[j, c'] = S_{i+1}[c' - b̃_j(i+1)][pos_{i+1}(j)]; thread: position pairs
  // 2(tid + T·q) + {0, 1}, so each wave instruction covers 512 contiguous bytes ----------------------
  // all loads issue back to back: a row below 0 (no such budget) reads row 0 and is masked after
  const int sbytes = (B + 1) * L * (int)sizeof(double);
  double v[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p2 = 2 * (tid + T * q);
    const int ra = max(cp - (int)(ein[q].x >> 16), 0), rb = max(cp - (int)(ein[q].y >> 16), 0);
    sd_load_pair<PERSIST>(Sin, sbytes, ra * L + p2, rb * L + p2 + 1, v[2 * q], v[2 * q + 1]);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if ((int)((h ? ein[q].y : ein[q].x) >> 16) > cp) v[2 * q + h] = INFINITY;
  // ---- this thread's targets: ranks tid | x << 3(M-1) (the lines of the last pass) -----------------
  double a[M];
  int lb[M], uo[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    a[m] = P.dt * dfi[m];
    lb[m] = G.base[m];
    uo[m] = (int)uoi[m];
  }
  double pre = 0.0;
  int bpre = 0;
  int xt[M];
#pragma unroll
  for (int m = 0; m < M - 1; ++m) {
    xt[m] = (tid >> (3 * m)) & 7;
    const int nu = lb[m] + xt[m];
    pre = pre + a[m] * (double)nu;  // ((0 + (Δt·df_1)·ν_1) + ...), HelpFunctions.jl:52-57
    bpre += abs(nu - uo[m]);
  }
  const unsigned ptid = sd_bytes((unsigned)tid);  // the thread's first M-1 coordinates, one byte each
  unsigned valid = 0;  // target inside the trust region: c' + b̃_l(i) <= B
#pragma unroll
  for (int x = 0; x < 8; ++x) valid |= (unsigned)(bpre + abs(lb[M - 1] + x - uo[M - 1]) <= B - cp) << x;

  if (tid == 0) sh.nlist = 0;
  double pmn = INFINITY, pmx = -INFINITY;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const double x = v[2 * q + h];
      psi[(h ? ein[q].y : ein[q].x) & 0xFFFFu] = x;
      if (x < INFINITY) {
        pmn = fmin(pmn, x);
        pmx = fmax(pmx, x);
      }
    }
  int nv = __popc(valid);  // targets in the trust region (low 16 bits) + finite sources (high 16 bits)
#pragma unroll
  for (int q = 0; q < 8; ++q) nv += (v[q] < INFINITY) << 16;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    pmn = fmin(pmn, __shfl_xor(pmn, off));
    pmx = fmax(pmx, __shfl_xor(pmx, off));
    nv += __shfl_xor(nv, off);
  }
  if (lane == 0) {
    sh.rmn[w] = pmn;
    sh.rmx[w] = pmx;
    sh.rnv[w] = nv;
  }
  __syncthreads();  // every load of S_{i+1} has returned (its value is in LDS)
  if (PERSIST && tid == 0) __hip_atomic_store(loaded, token, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    pmn = fmin(pmn, sh.rmn[q]);
    pmx = fmax(pmx, sh.rmx[q]);
  }
  nv = 0;
#pragma unroll
  for (int q = 0; q < NW; ++q) nv += sh.rnv[q];
  const int nf = nv >> 16;
  nv &= 0xFFFF;
  SD_STAMP(1);
  if (nv == 0 || !(pmn < INFINITY)) {  // no target in the trust region, or nothing reachable
#pragma unroll
    for (int q = 0; q < 4; ++q)
      sd_store16<PERSIST>(Sout, L * 8, 2 * (tid + T * q), 0x7FF0000000000000ull, 0x7FF0000000000000ull);
    // and the U row: no cell written (0xFFFF), as in the reference, where U keeps nothing for Φ_i = +Inf
    *reinterpret_cast<ulonglong2 *>(UU + 8 * tid) = make_ulonglong2(~0ull, ~0ull);
    return;
  }

  // ---- the binade: values base + (Ψ - Ψmin)/β + d lie in [base, 2·base), grid g = 2^13 ulp ----------
  const double inv = Lv.inv_beta;                      // fl(1/β), host-computed
  const double rs = (pmx - pmn) * inv + (double)Smax;  // scaled range of every transform value
  const bool scale_ok = rs < 0x1p36;                   // else unit steps are not on the grid: exact scans
  const int E = ilogb(fmin(rs, 0x1p36) * (1.0 + 0x1p-20) + 1.0) + 2;  // 2^E >= 2·rs
  const double base = ldexp(1.0, E), g = ldexp(1.0, E - 39);
  double qmax = beta * (double)Smax + fmax(fabs(pmn), fabs(pmx));  // >= |T1 + β·d + Ψ| for every candidate
#pragma unroll
  for (int m = 0; m < M; ++m) qmax += fabs(a[m]) * (double)max(abs(lb[m]), abs(lb[m] + 7));
  // 2 × stamping error (< g) + 2 × the reference's rounding (<= 4u·qmax per candidate), in units of β
  const double tol = 3.0 * g + 0x1p-49 * qmax * inv;
  // few finite sources (rows near c' = 0): every target's minimum over them, directly
  const bool sparse = nf <= SD_SPARSE;
  const bool direct = !sparse && (nv <= SD_FEW || !scale_ok || !(tol < base * 0x1p-20));

  double o[8];
  int spj[SD_SPARSE];
  double spv[SD_SPARSE];
  if (sparse) {
    if (tid == 0) sh.nsp = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (v[2 * q + h] < INFINITY) {
          const int e = atomicAdd(&sh.nsp, 1);
          sh.spj[e] = (int)((h ? ein[q].y : ein[q].x) & 0xFFFFu);
          sh.spv[e] = v[2 * q + h];
        }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < SD_SPARSE; ++e) {  // uniform: broadcast reads into registers
      spj[e] = sh.spj[e];
      spv[e] = sh.spv[e];
    }
  } else if (!direct) {
    // ---- stamp: V_j = trunc_g(base + (Ψ_j - Ψmin)/β) | j --------------------------------------------
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = (int)((h ? ein[q].y : ein[q].x) & 0xFFFFu);
        const double x = v[2 * q + h];
        double V = INFINITY;
        if (x < INFINITY) {
          const double y = (x - pmn) * inv + base;
          V = __hiloint2double(__double2hiint(y), (__double2loint(y) & ~SD_PAY) | j);
        }
        dtv[sd_swz(j)] = V;
      }
    __syncthreads();
    SD_STAMP(2);
    // ---- M passes: forward and backward sweep along the 8 levels of one dimension, unit step 1.0 -----
#pragma unroll
    for (int m = 0; m < M; ++m) {
      int pos[8];
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        pos[x] = sd_swz(sd_rank(tid, m, x));
        o[x] = dtv[pos[x]];
      }
      // in place: after the forward sweep o[x] covers the sources at <= x; a backward merge of o[x] with
      // o[x+1] + 1 compares a source at <= x with itself shifted by >= 2, never within tol, so every
      // flagged tie is between two distinct sources (as in a merge of disjoint sets)
#pragma unroll
      for (int x = 1; x < 8; ++x) o[x] = sd_merge(o[x], o[x - 1] + 1.0, tol);
#pragma unroll
      for (int x = 6; x >= 0; --x) o[x] = sd_merge(o[x], o[x + 1] + 1.0, tol);
      if (m + 1 < M) {
#pragma unroll
        for (int x = 0; x < 8; ++x) dtv[pos[x]] = o[x];
      }
      __syncthreads();  // last pass: every read of dtv is done before it becomes the output buffer
      SD_STAMP(3 + m);
    }
  }

  // ---- targets: R(l, j*) for a certified winner; the others are listed for the exact scan (their
  // output slot holds NaN until the scan fills it) ----------------------------------------------------
  unsigned listed = 0;
  if (!direct && !sparse) {  // branch-free: the eight winners' Ψ reads issue together
    int jx[8];
    double pv[8];
#pragma unroll
    for (int x = 0; x < 8; ++x) jx[x] = __double2loint(o[x]) & (SD_FLAG - 1);  // +Inf carries payload 0
#pragma unroll
    for (int x = 0; x < 8; ++x) pv[x] = psi[jx[x]];
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      const int r = tid | (x << (3 * (M - 1))), j = jx[x];
      const bool fin = (valid >> x & 1) && o[x] < INFINITY;
      const bool flg = (__double2loint(o[x]) & SD_FLAG) != 0;
      const unsigned d = sd_l1(sd_bytes(j), ptid | (unsigned)x << (8 * (M - 1)));
      const double t1 = pre + a[M - 1] * (double)(lb[M - 1] + x);
      const double val = (t1 + beta * (double)d) + pv[x];  // R(l, j*), HelpFunctions.jl:63-71
      listed |= (unsigned)(fin && flg) << x;
      uu[r] = (uint16_t)(fin && !flg ? j : 0xFFFF);  // 0xFFFF: unwritten (Φ = +Inf) or not yet known (listed)
      dtv[r] = fin ? (flg ? __longlong_as_double(0x7FF8000000000000ll) : val) : INFINITY;
    }
  } else {
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      const int r = tid | (x << (3 * (M - 1)));
      double ov = INFINITY;
      int uj = 0xFFFF;  // U cell not written by the reference (Φ = +Inf) or not yet known (listed)
      if (direct) {
        listed |= valid & (1u << x);
      } else if (sparse) {
        if (valid >> x & 1) {  // the reference loop over the finite sources, ties to the lower rank
          const double t1 = pre + a[M - 1] * (double)(lb[M - 1] + x);
          double bv = INFINITY;
          int bj = 0xFFFF;
#pragma unroll
          for (int e = 0; e < SD_SPARSE; ++e) {
            if (e < nf) {
              const int j = spj[e];
              const unsigned d = sd_l1(sd_bytes(j), ptid | (unsigned)x << (8 * (M - 1)));
              const double val = (t1 + beta * (double)d) + spv[e];
              if (val < bv || (val == bv && j < bj)) {
                bv = val;
                bj = j;
              }
            }
          }
          ov = bv;
          uj = bj;
        }
      }
      uu[r] = (uint16_t)uj;
      dtv[r] = (listed >> x & 1) ? __longlong_as_double(0x7FF8000000000000ll) : ov;
    }
  }
  if (listed) {
    int e = atomicAdd(&sh.nlist, __popc(listed));
#pragma unroll
    for (int x = 0; x < 8; ++x)
      if (listed >> x & 1) {
        if (e < SD_LCAP) list[e] = (uint16_t)(tid | (x << (3 * (M - 1))));
        ++e;
      }
  }
  __syncthreads();
  SD_STAMP(7);
  const int nl = sh.nlist;
  if (nl) {
    if (nl <= SD_COOP)
      sd_scan<M, true>(list, nl, psi, a, lb, beta, uu, dtv, sh.redv, sh.redj);
    else if (nl <= SD_LCAP)
      sd_scan<M, false>(list, nl, psi, a, lb, beta, uu, dtv, sh.redv, sh.redj);
    else
      sd_scan<M, false>(nullptr, L, psi, a, lb, beta, uu, dtv, sh.redv, sh.redj);  // every NaN-marked rank
    __syncthreads();
    if (tid == 0) atomicAdd(&counters[direct ? 1 : 0], nl);
  }
  SD_STAMP(8);
  // ---- Φ_i row c' in the sphere order of u_old(i), and the U row, both 16 bytes per lane ------------
#pragma unroll
  for (int q = 0; q < 4; ++q)
    sd_store16<PERSIST>(Sout, L * 8, 2 * (tid + T * q), __double_as_longlong(dtv[eout[q].x & 0xFFFFu]),
                        __double_as_longlong(dtv[eout[q].y & 0xFFFFu]));
  {
    const ulonglong2 t = reinterpret_cast<const ulonglong2 *>(uu)[tid];
    *reinterpret_cast<ulonglong2 *>(UU + 8 * tid) = t;  // read by later launches only (backtrack)
  }
  SD_STAMP(9);
  SD_RSTAMP(14);
}

// The two rows that need no transform (B >= 1):
//  * row 0 has at most one finite source, j0 = the level at L1 distance 0 from u_old(i+1) (sphere position 0
//    of step i+1): Φ_i[l, b̃_l] = fl(fl(T1(l) + β·d(l, j0)) + Φ_{i+1}[j0, 0]) and U = j0 for every target;
//  * row B has at most one target, l0 = the level at distance 0 from u_old(i) (sphere position 0 of step i):
//    Φ_i[l0, B] = min_j fl(fl(T1(l0) + β·d(l0, j)) + Φ_{i+1}[j, B]), the first minimum in rank order
//    (HelpFunctions.jl:60-77); every other cell of row B is +Inf and unwritten.
// Both run in one workgroup (block 0 of the per-step kernel, workgroup 0 of the persistent one, which runs
// row B a few steps behind row 0).  `loaded` (persistent kernel): the row's flag, stored once every read of
// S_{i+1} has returned.
template <int M>
struct SdEdge {
  double a[M];
  int lb[M], uo[M];
  __device__ __forceinline__ SdEdge(const ProblemDev &P, const int *lb_g, int k, int i) {
    const double *dfi = P.df + ((size_t)k * P.nt + i) * M;
    const double *uoi = P.uold + ((size_t)k * P.nt + i) * M;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      a[m] = P.dt * dfi[m];
      lb[m] = lb_g[m];
      uo[m] = (int)uoi[m];
    }
  }
  __device__ __forceinline__ double t1(int r) const {  // ((0 + (Δt·df_1)·ν_1) + ...), HelpFunctions.jl:52-57
    double t = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) t = t + a[m] * (double)(lb[m] + ((r >> (3 * m)) & 7));
    return t;
  }
  __device__ __forceinline__ int bt(int r) const {  // b̃_r(i) = Σ_m |ν_rm - u_old[m, i]|
    int b = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) b += abs(lb[m] + ((r >> (3 * m)) & 7) - uo[m]);
    return b;
  }
  static __device__ __forceinline__ unsigned dist(int r, int j) { return sd_l1(sd_bytes(r), sd_bytes(j)); }
};
__device__ __forceinline__ unsigned long long sd_pack4(const unsigned short *u) {
  return (unsigned long long)u[0] | (unsigned long long)u[1] << 16 | (unsigned long long)u[2] << 32 |
         (unsigned long long)u[3] << 48;
}

template <int M, bool PERSIST>
__device__ __forceinline__ void sdt_row0(const ProblemDev &P, const LevelsDev &Lv, int k, int i, const SdPerm &pm,
                                         const double *Sin_all, double *Sout_all, uint16_t *__restrict__ UU_all,
                                         size_t s_stride, size_t uu_stride_k, const int *lb_g, int32_t *loaded,
                                         int token) {
  constexpr int L = 1 << (3 * M), T = L / 8;
  const int tid = threadIdx.x, B = P.B;
  const double beta = Lv.beta;
  const double *Sin = Sin_all + (size_t)k * s_stride;
  double *S0 = Sout_all + (size_t)k * s_stride;
  uint16_t *U0 = UU_all + (size_t)k * uu_stride_k + (size_t)i * ((size_t)(B + 1) * L);
  const double psi0 = sd_load8<PERSIST>(Sin, (B + 1) * L * (int)sizeof(double), 0);  // Φ_{i+1}[j0, 0]
  const SdEdge<M> E(P, lb_g, k, i);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave's read of S_{i+1} has returned
  if (PERSIST && tid == 0) __hip_atomic_store(loaded, token, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int j0 = (int)(pm.hin & 0xFFFFu);
  const bool src0 = (pm.hin >> 16) == 0 && psi0 < INFINITY;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    double o[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t e = h ? pm.out[q].y : pm.out[q].x;
      const int r = (int)(e & 0xFFFFu);
      const double val = (E.t1(r) + beta * (double)SdEdge<M>::dist(r, j0)) + psi0;
      o[h] = src0 && (int)(e >> 16) <= B && val < INFINITY ? val : INFINITY;
    }
    sd_store16<PERSIST>(S0, L * 8, 2 * (tid + T * q), __double_as_longlong(o[0]), __double_as_longlong(o[1]));
  }
  // U row in natural order: ranks 8·tid .. 8·tid + 7, one 16-byte store
  unsigned short u0[8];
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    const int r = 8 * tid + x;
    const double val = (E.t1(r) + beta * (double)SdEdge<M>::dist(r, j0)) + psi0;
    u0[x] = src0 && E.bt(r) <= B && val < INFINITY ? (unsigned short)j0 : (unsigned short)0xFFFF;
  }
  *reinterpret_cast<ulonglong2 *>(U0 + 8 * tid) = make_ulonglong2(sd_pack4(u0), sd_pack4(u0 + 4));
}

template <int M, bool PERSIST>
__device__ __forceinline__ void sdt_rowB(const ProblemDev &P, const LevelsDev &Lv, int k, int i, const SdPerm &pm,
                                         const double *Sin_all, double *Sout_all, uint16_t *__restrict__ UU_all,
                                         size_t s_stride, size_t uu_stride_k, const int *lb_g,
                                         int32_t *__restrict__ counters, SdtShared<(1 << (3 * M - 3)) / 64> &sh,
                                         int32_t *loaded, int token) {
  constexpr int L = 1 << (3 * M), T = L / 8, NW = T / 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, B = P.B;
  const double beta = Lv.beta;
  const double *Sin = Sin_all + (size_t)k * s_stride;
  double *SB = Sout_all + (size_t)k * s_stride + (size_t)B * L;
  uint16_t *UB = UU_all + (size_t)k * uu_stride_k + (size_t)i * ((size_t)(B + 1) * L) + (size_t)B * L;
  // ---- every source: Ψ_j = S_{i+1}[B - b̃_j(i+1)][pos(j)] (position pairs as in sdt_row) ------------------
  const int sbytes = (B + 1) * L * (int)sizeof(double);
  double v[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p2 = 2 * (tid + T * q);
    const int ra = max(B - (int)(pm.in[q].x >> 16), 0), rb = max(B - (int)(pm.in[q].y >> 16), 0);
    sd_load_pair<PERSIST>(Sin, sbytes, ra * L + p2, rb * L + p2 + 1, v[2 * q], v[2 * q + 1]);
  }
  const SdEdge<M> E(P, lb_g, k, i);
  // ---- the one target's minimum over every source ------------------------------------------------------
  const int r0 = (int)(pm.hout & 0xFFFFu);
  const bool has0 = (pm.hout >> 16) == 0;  // u_old(i) is a level of the table
  const double t1b = E.t1(r0);
  double bv = INFINITY;
  int bj = -1;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t e = h ? pm.in[q].y : pm.in[q].x;
      const int j = (int)(e & 0xFFFFu);
      const double x = (int)(e >> 16) > B ? INFINITY : v[2 * q + h];
      const double val = (t1b + beta * (double)SdEdge<M>::dist(r0, j)) + x;
      if (val < bv || (val == bv && bj >= 0 && j < bj)) {
        bv = val;
        bj = j;
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
    sh.redv[w] = bv;
    sh.redj[w] = bj;
  }
  __syncthreads();  // every read of S_{i+1} has returned (its values are consumed above)
  if (PERSIST && tid == 0) __hip_atomic_store(loaded, token, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  bv = INFINITY;
  bj = -1;
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const double ov = sh.redv[q];
    const int oj = sh.redj[q];
    if (oj >= 0 && (bj < 0 || ov < bv || (ov == bv && oj < bj))) {
      bv = ov;
      bj = oj;
    }
  }
  __syncthreads();  // sh.redv / redj are free again
  const bool wb = has0 && bj >= 0;  // the reference writes U[l0, B] (finite minimum)
  if (has0 && tid == 0) atomicAdd(&counters[1], 1);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const bool p0 = wb && tid == 0 && q == 0;  // only sphere position 0 (= l0) can be finite
    sd_store16<PERSIST>(SB, L * 8, 2 * (tid + T * q), p0 ? __double_as_longlong(bv) : 0x7FF0000000000000ull,
                        0x7FF0000000000000ull);
  }
  unsigned short ub[8];
#pragma unroll
  for (int x = 0; x < 8; ++x) ub[x] = wb && 8 * tid + x == r0 ? (unsigned short)bj : (unsigned short)0xFFFF;
  *reinterpret_cast<ulonglong2 *>(UB + 8 * tid) = make_ulonglong2(sd_pack4(ub), sd_pack4(ub + 4));
}

// One launch per step: one workgroup per (source row c', subproblem k).
template <int M>
__global__ __launch_bounds__(1 << (3 * M - 3)) void k_sdt_step(ProblemDev P, LevelsDev Lv, PyrGeom G, int i,
                                                           const uint32_t *__restrict__ perm_all,
                                                           const double *__restrict__ Sin_all,
                                                           double *__restrict__ Sout_all,
                                                           uint16_t *__restrict__ UU_all, size_t s_stride,
                                                           size_t uu_stride_k, int32_t *__restrict__ counters) {
  extern __shared__ __attribute__((aligned(16))) unsigned char sds[];
  __shared__ SdtShared<(1 << (3 * M - 3)) / 64> sh;
  SdPerm pm;
  sd_perm_load<M>(pm, perm_all, P.nt, (int)blockIdx.y, i);
  // B >= 1: block 0 takes rows 0 and B together, block x the row x (B workgroups, one per CU at B = 256)
  if (blockIdx.x == 0 && P.B >= 1) {
    sdt_row0<M, false>(P, Lv, (int)blockIdx.y, i, pm, Sin_all, Sout_all, UU_all, s_stride, uu_stride_k, G.base,
                       nullptr, 0);
    sdt_rowB<M, false>(P, Lv, (int)blockIdx.y, i, pm, Sin_all, Sout_all, UU_all, s_stride, uu_stride_k, G.base,
                       counters, sh, nullptr, 0);
  } else
    sdt_row<M, false>(P, Lv, G, (int)blockIdx.y, (int)blockIdx.x, i, pm, Sin_all, Sout_all, UU_all,
                      s_stride, uu_stride_k, counters, sh, sds, nullptr, 0);
  SD_FLUSH();
}

// Persistent: the whole DP in one launch.  Each subproblem's rows 0..B are split into chunks, one per resident
// workgroup (nwg / K workgroups per subproblem, one per CU; chunks differ by at most one row).  With W = B
// workgroups (257 rows on 256 CUs), workgroup w >= 1 takes row w and workgroup 0 the two rows that need no
// transform: row 0 of step i and row B of step i + SD_BLAG.  Row B lags because it reads rows B - Smax .. B
// of the step before: run in lockstep with row 0 it would close a dependency cycle through every row
// (row 0 -> row 1 -> ... -> row B -> row 0 of the next step) and hold the whole DP to the hand-off latency
// of every step; a lag of SD_BLAG steps leaves each row bound by its own body.
//
// Row c' of step i reads rows c' - s (s <= Smax) of S_{i+1} and overwrites row c' of the staging buffer
// i % NB, which held S_{i+NB}, read by rows c' .. c' + Smax at step i+NB-1.  So before a chunk [lo, hi)
// starts a step, one wave polls (relaxed agent loads, s_sleep)
//   done[k][lo - s]        >= token(i+1)      for 1 <= s <= min(lo, Smax)           (its inputs are published)
//   loaded[k][hi - 1 + s]  >= token(i+NB-1)   for 1 <= s <= min(B + 1 - hi, Smax)   (nobody still reads S_{i+NB})
// with token(i) = nt - 1 - i (0 = nothing yet; the terminal row comes from the previous launch); rows inside
// the chunk are the workgroup's own, already done in order.  Every wait points at a strictly earlier item in
// the order (step descending, row ascending; workgroup 0's iteration i between steps i + 1 and i), so with
// every workgroup resident there is no deadlock; a wait that exceeds its spin bound sets *err and every
// workgroup leaves.
template <int M>
__global__ __launch_bounds__(1 << (3 * M - 3), SDT_RUN_MINW) void k_sdt_run(ProblemDev P, LevelsDev Lv, PyrGeom G,
                                                          const uint32_t *__restrict__ perm_all, double *S_all,
                                                          size_t buf_stride, uint16_t *__restrict__ UU_all,
                                                          size_t s_stride, size_t uu_stride_k,
                                                          int32_t *__restrict__ counters, int32_t *flags, int nwg,
                                                          int kint) {
  constexpr int Smax = 7 * M, NB = kSdtBuffers;
  extern __shared__ __attribute__((aligned(16))) unsigned char sds[];
  __shared__ SdtShared<(1 << (3 * M - 3)) / 64> sh;
  const int R = P.B + 1, nrows = P.K * R, tid = threadIdx.x;
  int32_t *done = flags, *loaded = flags + nrows, *err = flags + 2 * nrows;
  // this workgroup's chunk of rows, in every one of its group's kint subproblems (interleaved: while one
  // subproblem's row hand-off is in flight, the workgroup computes the same row of the next one)
  const int W = nwg / (P.K / kint);  // workgroups per group of kint subproblems (the host guarantees >= 1)
  const int kg = (int)blockIdx.x / W, wl = (int)blockIdx.x - kg * W;
  if (kg * kint >= P.K) return;
  const int base = R / W, extra = R - base * W;
  const bool split = W == R - 1 && R >= 2, edges = split && wl == 0;
  int lo, hi;  // rows [lo, hi), contiguous, the longer chunks highest
  if (split) {
    lo = wl;
    hi = lo + 1;
  } else {
    lo = wl * base + max(0, wl - (W - extra));
    hi = lo + base + (wl >= W - extra ? 1 : 0);
  }
  if (tid == 0) sh.stop = 0;
  auto tok_of = [&](int step) { return P.nt - 1 - step; };
  auto buf = [&](int step) { return S_all + (size_t)(step % NB) * buf_stride; };
#pragma nounroll
  for (int i = P.nt - 2; i >= (edges ? -SD_BLAG : 0); --i) {
#pragma nounroll
    for (int kk = 0; kk < kint; ++kk) {
      const int k = kg * kint + kk;
      const int iB = i + SD_BLAG;                   // workgroup 0: the step of its row B
      const bool do0 = i >= 0, doB = edges && iB <= P.nt - 2;
      const int g = k * R + lo;  // timeline stamps: the chunk's first row
      (void)g;
      SdPerm pm, pmB;  // static; SDT_PREFETCH: in flight during the wait (costs VGPRs)
#if SDT_PREFETCH
      if (do0) sd_perm_load<M>(pm, perm_all, P.nt, k, i);
      if (doB) sd_perm_load<M>(pmB, perm_all, P.nt, k, iB);
#endif
      SD_TL(0);
      if (tid < 64) {  // wave 0: dependency wait
        const int lane = tid;
        const int s = lane < 32 ? lane + 1 : lane - 31;
        int32_t *fp = nullptr;
        int need = 0;
        // RAW: inputs of row lo at step i (workgroup 0: of row B at step iB)
        const int rlo = edges ? R - 1 : lo, sraw = edges ? iB : i;
        // WAR: readers of the buffer row lo .. hi-1 overwrites at step i (workgroup 0: row 0 at step i)
        const int whi = edges ? 1 : hi;
        if (lane < 32 && s <= Smax && s <= rlo && (!edges || doB)) {
          fp = done + k * R + rlo - s;
          need = tok_of(sraw + 1);
        } else if (lane >= 32 && s <= Smax && whi - 1 + s < R && do0) {
          fp = loaded + k * R + whi - 1 + s;
          need = tok_of(i + NB - 1);
        }
        unsigned spins = 0;
        for (;;) {
          const bool ok =
              !fp || need <= 0 || __hip_atomic_load(fp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need;
          if (__all(ok)) break;
          if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || ++spins > (1u << 24)) {
            if (lane == 0) {
              __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              sh.stop = 1;
            }
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __syncthreads();
      SD_TL(1);
      if (sh.stop) return;
#if !SDT_PREFETCH
      if (do0) sd_perm_load<M>(pm, perm_all, P.nt, k, i);
      if (doB) sd_perm_load<M>(pmB, perm_all, P.nt, k, iB);
#endif
      if (edges) {
        if (do0)
          sdt_row0<M, true>(P, Lv, k, i, pm, buf(i + 1), buf(i), UU_all, s_stride, uu_stride_k, G.base,
                            loaded + k * R, tok_of(i));
        if (doB)
          sdt_rowB<M, true>(P, Lv, k, iB, pmB, buf(iB + 1), buf(iB), UU_all, s_stride, uu_stride_k, G.base,
                            counters, sh, loaded + k * R + R - 1, tok_of(iB));
        SD_TL(2);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its write-through stores have landed
        __syncthreads();
        if (tid == 0) {
          if (do0) __hip_atomic_store(done + k * R, tok_of(i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (doB)
            __hip_atomic_store(done + k * R + R - 1, tok_of(iB), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        SD_TL(3);
      }
#pragma nounroll
      for (int cp = lo; cp < hi && !edges; ++cp) {
        sdt_row<M, true>(P, Lv, G, k, cp, i, pm, buf(i + 1), buf(i), UU_all, s_stride, uu_stride_k, counters,
                         sh, sds, loaded + k * R + cp, tok_of(i));
        SD_TL(2);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its write-through stores have landed
        __syncthreads();
        if (tid == 0) __hip_atomic_store(done + k * R + cp, tok_of(i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        SD_TL(3);
      }
    }
    if (i == 0) SD_FLUSH();
  }
}

size_t sdt_lds_bytes(const PyrGeom &G) {
  const size_t L = (size_t)1 << (3 * G.M);
  return L * (2 * sizeof(double) + sizeof(uint16_t)) + SD_LCAP * sizeof(uint16_t);
}

bool sdt_supported(const PyrGeom &G) {
  if (G.M != 3 && G.M != 4) return false;
  for (int m = 0; m < G.M; ++m)
    if (G.n[m] != 8) return false;
  return true;
}

hipError_t launch_sdt_run(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G,
                          const uint32_t *perm, double *S, size_t buf_stride, uint16_t *UU, size_t s_stride,
                          size_t uu_stride_k, int32_t *counters, int32_t *flags, int nwg, int kint, size_t lds) {
  if (!sdt_supported(G)) return hipErrorInvalidValue;
  // cooperative launch: the runtime checks at launch time that every workgroup can be resident at once (the
  // row hand-off spins on other workgroups), and refuses the launch otherwise (hipErrorCooperativeLaunchTooLarge)
  void *args[] = {(void *)&P, (void *)&Lv, (void *)&G, (void *)&perm, (void *)&S, (void *)&buf_stride, (void *)&UU,
                  (void *)&s_stride, (void *)&uu_stride_k, (void *)&counters, (void *)&flags, (void *)&nwg,
                  (void *)&kint};
  if (G.M == 4)
    return hipLaunchCooperativeKernel((const void *)k_sdt_run<4>, dim3(nwg), dim3(512), args, (unsigned)lds, s);
  return hipLaunchCooperativeKernel((const void *)k_sdt_run<3>, dim3(nwg), dim3(64), args, (unsigned)lds, s);
}

int sdt_run_blocks_per_cu(const PyrGeom &G, size_t lds) {
  int n = 0;
  hipError_t e = G.M == 4 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_sdt_run<4>, 512, lds)
                          : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_sdt_run<3>, 64, lds);
  return e == hipSuccess ? n : 0;
}

hipError_t launch_sdt_step(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G, int i,
                           const uint32_t *perm, const double *Sin, double *Sout, uint16_t *UU, size_t s_stride,
                           size_t uu_stride_k, int32_t *counters) {
  if (!sdt_supported(G)) return hipErrorInvalidValue;
  const dim3 grid(P.B >= 1 ? P.B : 1, P.K);  // rows 0 and B share block 0
  const size_t lds = sdt_lds_bytes(G);
  if (G.M == 4)
    hipLaunchKernelGGL(k_sdt_step<4>, grid, dim3(512), lds, s, P, Lv, G, i, perm, Sin, Sout, UU, s_stride,
                       uu_stride_k, counters);
  else
    hipLaunchKernelGGL(k_sdt_step<3>, grid, dim3(64), lds, s, P, Lv, G, i, perm, Sin, Sout, UU, s_stride,
                       uu_stride_k, counters);
  return hipGetLastError();
}

#if defined(MIOC_STAMPS) && defined(MIOC_STAMPS_TL)
extern "C" int32_t mioc_debug_sdt_timeline(unsigned long long *out, int64_t nrows) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sdt_tl), (size_t)nrows * 64 * 4 * sizeof(unsigned long long)) ==
                 hipSuccess
             ? 0
             : -4;
}
#elif defined(MIOC_STAMPS)
extern "C" int32_t mioc_debug_sdt_stamps(unsigned long long *out, int64_t nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sdt_stamps), (size_t)nblocks * 16 * sizeof(unsigned long long)) ==
                 hipSuccess
             ? 0
             : -4;
}
#endif

}  // namespace mioc
