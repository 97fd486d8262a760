// mioc_sdt2.hip -- the C4 headline path (8^4 = 4096 levels, p = 1): the persistent separable-transform DP with TWO
// workgroups per budget row, so that two row items are in flight on every CU.
//
// The row item (c', i) is the certified L1 distance transform of source row c' of step i+1 (mioc_sdt.hip, header):
//   Φ_i[c' + b̃_l(i), l] = min_j fl(fl(T1(l, i) + β·d(l, j)) + Ψ_j),   Ψ_j = Φ_{i+1}[c', j]
// (HelpFunctions.jl:49-77).  In the staging layout S_{i+1}[c' - b̃_j(i+1)][pos_{i+1}(j)] = Φ_{i+1}[c', j], item (c', i)
// reads rows c' - 28 .. c' of step i+1 -- and of its own row c' exactly one value: the head j = h(i+1), the level at
// L1 distance 0 from u_old(i+1), at position 0.  That value, Φ_{i+1}[c', h(i+1)], is the output of item (c', i+1) at
// the target h(i+1), i.e. one 4096-candidate reduction of the item before it:
//   Φ_{i+1}[c', h(i+1)] = min_j fl(fl(T1(h(i+1), i+1) + β·d(h(i+1), j)) + Φ_{i+2}[c', j])          (*)
// with the head term j = h(i+2) of (*) again the output of the item before.  So a row's items do not depend on each
// other as a whole: item (c', i) needs only rows below (steps i+1 and i+2) and the scalar chain (*).
//
// Design (one process, one GPU; MI355X: 256 CUs, 160 KB LDS per CU):
//  * two workgroups of 256 threads (four waves, one per SIMD) per budget row c' = 1..B: workgroup p takes the steps
//    i with (nt - 2 - i) % 2 == p; with 74 KB of LDS each, the two share a CU and the SIMDs interleave their waves,
//    so one item's barrier-separated phases (LDS round trips, waits) are covered by the other's instruction stream;
//  * no hand-off between the two: each computes the chain (*) itself -- at item (c', i) it also loads the rows below
//    of step i+2 (the other workgroup's item's sources) and reduces them for the one target h(i+1); the head term
//    j = h(i+2) of that reduction is its own previous item's output at h(i+2) (kept in LDS), folded in after the
//    first barrier.  The exact reduction is bit-identical to the certified transform's value there (both are the
//    reference's minimum of the same candidates);
//  * rows and steps hand over through the measured-valid flag protocol of the one-workgroup driver (mioc_sdt.hip:
//    16-byte `sc1` stores drained by every storing wave, ONE lane's `sc1` flag store behind a barrier; every wave
//    polls its own flags, `sc1` loads after the poll matched), with one flag pair per (row, step parity):
//      done[k][r][p]   = token(i): row r's stores of step i have landed (token(i) = nt - 1 - i)
//      loaded[k][r][p] = token(i): row r's loads for its item at step i (steps i+1 and i+2) have returned
//    item (c', i) issues its loads (during item (c', i+2)) once done[c' - s][par(i+1)] >= token(i+1) and
//    done[c' - s][par(i+2)] >= token(i+2), 1 <= s <= 28; it stores into buffer i % NB once
//    loaded[c' + s][par(i+NB-1)] >= token(i+NB-1) and loaded[c' + s][par(i+NB-2)] >= token(i+NB-2) (the readers of
//    the step it overwrites).  Every wait points at a lower row or an earlier step, so with every workgroup resident
//    nothing deadlocks; a wait beyond the spin limit sets the error word and every workgroup leaves (the host redoes
//    the DP per step, check_run);
//  * per lane 16 values: eight position pairs 2(t + 256·q) + {0, 1} (16-byte loads and stores, a wave's 1 KB
//    contiguous); the sphere orders are packed per position pair (k_sdt2_pack: both ranks and the first element's
//    distance in one word, the second elements that straddle a sphere seam listed per wave), loaded into registers
//    two items ahead instead of being copied into LDS;
//  * the transform's lines of passes 0..2 keep the top coordinate x3 in {w, w+4} for wave w (wave-local, no
//    barrier), the last pass needs every wave; its outputs go back to the swizzled positions the lane read (no
//    separate output buffer: 74 KB of LDS per workgroup).
//
// Parity: identical cells (u, Φ*, every U cell) to the reference loop: the same certified transform and exact scans
// as mioc_sdt.hip, and (*) is the reference's own expression.  Tested against the oracle's U hashes on the C4 nt=64
// fixture (tests/test_gpu_c4.py) like the one-workgroup driver.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mioc_internal.h"
#include "mioc_sdt_common.h"

namespace mioc {
namespace {

constexpr int S2_L = 4096;         // levels
constexpr int S2_SEAMS = 32;        // seam words per wave (<= 28 seams in a sphere order)
constexpr int S2_PACK = S2_L / 2;   // pair words per step

// LDS (dynamic): Ψ by rank | transform values (swizzled; the outputs after the last pass) | U row | scan list |
// per wave df(:, i..i+1), u_old(:, i..i+2)
constexpr size_t S2_PSI = 0, S2_DTV = S2_PSI + S2_L * 8, S2_UU = S2_DTV + S2_L * 8, S2_LIST = S2_UU + S2_L * 2,
                 S2_DFUO = S2_LIST + SD_LCAP * 2, S2_DFUO_WAVE = 256;

// the workgroup shape: T = 256 threads (16 values per lane, two last-pass lines, 4 waves: two workgroups per CU at
// 256 VGPRs) or 512 (8 values per lane, one line, 8 waves: two workgroups per CU -- four waves per SIMD -- at 128)
template <int T>
struct S2C {
  static constexpr int NW = T / 64;                // waves
  static constexpr int Q = S2_L / 2 / T;           // position pairs per lane
  static constexpr int LN = S2_L / 8 / T;          // last-pass lines per lane
  static constexpr int UB = S2_L * 2 / T / 16;     // 16-byte stores per lane of the U row
  static constexpr int NST = Q + UB;               // an item's stores (the counted wait at the next item's start)
  static constexpr size_t LDS = S2_DFUO + NW * S2_DFUO_WAVE;
  static_assert(Q % 4 == 0 && LN >= 1 && UB >= 1, "k_sdt_pair shape");
};

template <int NW>
struct S2Shared {
  double redv[SD_COOP * NW];
  int redj[SD_COOP * NW];
  double rmn[NW], rmx[NW], pmin[NW];  // pmin: this item's head value (*) over each wave's values
  int rnv[NW];
  int nlist;
  int stop;  // a dependency wait timed out: the launch is abandoned
  int nsp;   // sparse rows: the finite sources (rank, Ψ)
  int spj[SD_SPARSE];
  double spv[SD_SPARSE];
  int cnt[2];     // targets sent to the exact scan (near ties, direct rows); flushed to the counters [0], [1]
};

// pair word: rank_a | rank_b << 12 | b̃_a << 24 | (b̃_b != b̃_a) << 29; seam word: o | b̃ << 10 | rank << 16 for the
// in-wave offset o (0..1023) of a straddling pair's second element, 0xFFFFFFFF none
__device__ __forceinline__ int s2_ra(uint32_t w) { return (int)(w & 0xFFFu); }
__device__ __forceinline__ int s2_rb(uint32_t w) { return (int)((w >> 12) & 0xFFFu); }
__device__ __forceinline__ int s2_bt(uint32_t w) { return (int)((w >> 24) & 31u); }
__device__ __forceinline__ bool s2_strad(uint32_t w) { return (w >> 29) & 1u; }
// the position of in-wave offset o of wave w: o = 128q + 2l + h <-> position 2(64w + l + T·q) + h
template <int T>
__device__ __forceinline__ int s2_seam_pos(int w, int o) { return 2 * T * (o >> 7) + 128 * w + (o & 127); }

// One step's sphere order (perm: rank | b̃ << 16 by position, k_pyr_order) packed for k_sdt_pair: thread t's Q pair
// words contiguous (16-byte loads), and per wave the second elements of the pairs that straddle a seam.
template <int T>
__global__ __launch_bounds__(T) void k_sdt2_pack(const uint32_t *__restrict__ perm_all, int nt,
                                                   uint32_t *__restrict__ pack_all, uint32_t *__restrict__ seam_all,
                                                   int32_t *__restrict__ counters) {
  const int i = (int)blockIdx.x, k = (int)blockIdx.y, t = threadIdx.x, lane = t & 63, w = t >> 6;
  constexpr int NW = S2C<T>::NW, Q = S2C<T>::Q;
  const uint32_t *perm = perm_all + ((size_t)k * nt + i) * S2_L;
  __shared__ int cnt[NW];
  __shared__ uint32_t sl[NW * S2_SEAMS];
  if (t < NW) cnt[t] = 0;
  for (int e = t; e < NW * S2_SEAMS; e += T) sl[e] = 0xFFFFFFFFu;
  __syncthreads();
  uint32_t wd[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int u = t + T * q;
    const uint32_t ea = perm[2 * u], eb = perm[2 * u + 1];
    const uint32_t ba = min(ea >> 16, 31u), bb = min(eb >> 16, 31u);
    const bool st = ba != bb;
    wd[q] = (ea & 0xFFFu) | (eb & 0xFFFu) << 12 | ba << 24 | (uint32_t)st << 29;
    if (st) {
      const int e = atomicAdd(&cnt[w], 1);
      if (e < S2_SEAMS)
        sl[w * S2_SEAMS + e] = (uint32_t)(128 * q + 2 * lane + 1) | bb << 10 | (eb & 0xFFFu) << 16;
      else if (counters)
        atomicAdd(&counters[3], 1);  // the list cannot hold this seam: a loud internal-consistency failure
    }
  }
  uint4 *dst = reinterpret_cast<uint4 *>(pack_all + ((size_t)k * nt + i) * S2_PACK + (size_t)t * Q);
#pragma unroll
  for (int q4 = 0; q4 < Q / 4; ++q4) dst[q4] = make_uint4(wd[4 * q4], wd[4 * q4 + 1], wd[4 * q4 + 2], wd[4 * q4 + 3]);
  __syncthreads();
  for (int e = t; e < NW * S2_SEAMS; e += T) seam_all[((size_t)k * nt + i) * (NW * S2_SEAMS) + e] = sl[e];
}

// this lane's pair words and seam word of one step (registers)
template <int Q>
struct S2Ent {
  uint32_t w[Q];
  uint32_t seam;
};
// the loads of one step's values at this lane's positions (registers, in flight across an item)
template <int Q>
struct S2Raw {
  sd_u32x4 a[Q];
  sd_u32x2 sv;
  unsigned mask;  // per pair q: bit 2q the first element has no value here (row below 0, or the head), 2q+1 the second
  int srow;       // the seam element's source row (< 0: none / below row 0)
};

template <int Q>
__device__ __forceinline__ void s2_ent_issue(S2Ent<Q> &e, const uint32_t *pack, const uint32_t *seam) {
  const int t = threadIdx.x;
  const uint4 *src = reinterpret_cast<const uint4 *>(pack + (size_t)t * Q);
#pragma unroll
  for (int q4 = 0; q4 < Q / 4; ++q4) {
    const uint4 x = src[q4];
    e.w[4 * q4] = x.x, e.w[4 * q4 + 1] = x.y, e.w[4 * q4 + 2] = x.z, e.w[4 * q4 + 3] = x.w;
  }
  e.seam = seam[(t >> 6) * S2_SEAMS + (t & 31)];  // lanes 32..63 repeat lanes 0..31 (masked in s2_issue)
}

// The loads of one step's values for source row cp: position pair q from row cp - b̃_a (one 16-byte `sc1` load), the
// straddling second elements by the wave's seam list (one 8-byte load per lane); out-of-range offsets (dropped by the
// hardware) for rows below 0, for the head (b̃ = 0: the caller supplies it) and when `live` is false.  Always
// exactly Q + 1 vector-memory instructions.
template <int T, int Q>
__device__ __forceinline__ void s2_issue(S2Raw<Q> &r, __amdgpu_buffer_rsrc_t rs, const S2Ent<Q> &e, int cp,
                                         unsigned boff, unsigned r0, unsigned rowb, bool live) {
  constexpr unsigned OOB = 0xFFFFFFF0u;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  unsigned mask = 0;
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int p2 = 2 * (t + T * q);
    const int ra = cp - s2_bt(e.w[q]);
    const bool bad = !live || ra < 0 || ra == cp;  // (ra == cp: the head, position 0 -- its pair always straddles)
    unsigned oa = bad ? OOB : ra >= 1 ? boff + (unsigned)ra * rowb + (unsigned)p2 * 8u : r0 + (unsigned)p2 * 8u;
    // (the offset as an opaque value: otherwise the select became a branch with a load on each side, which the
    // compiler's wait counts then treat as possibly not issued -- later waits on older loads became waits on these)
    asm volatile("" : "+v"(oa));
    r.a[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, oa, 0, 16);
    mask |= ((unsigned)bad | (unsigned)(bad || s2_strad(e.w[q])) << 1) << (2 * q);
  }
  const uint32_t sw = lane < 32 ? e.seam : 0xFFFFFFFFu;
  const int srow = sw == 0xFFFFFFFFu || !live ? -1 : cp - (int)((sw >> 10) & 31u);
  const int P = s2_seam_pos<T>(w, (int)(sw & 1023u));
  const unsigned os = srow < 0 ? OOB : srow >= 1 ? boff + (unsigned)srow * rowb + (unsigned)P * 8u : r0 + (unsigned)P * 8u;
  r.sv = __builtin_amdgcn_raw_buffer_load_b64(rs, os, 0, 16);
  r.mask = mask;
  r.srow = srow;
}
// the 2Q values (+Inf where this lane has none) and the seam element (+Inf if none)
template <int Q>
__device__ __forceinline__ void s2_take(double (&v)[2 * Q], double &xs, const S2Raw<Q> &r) {
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const unsigned m = r.mask >> (2 * q);
    v[2 * q] = (m & 1) ? INFINITY : __hiloint2double((int)r.a[q].y, (int)r.a[q].x);
    v[2 * q + 1] = (m & 2) ? INFINITY : __hiloint2double((int)r.a[q].w, (int)r.a[q].z);
  }
  xs = r.srow < 0 ? INFINITY : __hiloint2double((int)r.sv.y, (int)r.sv.x);
}

// df(:, s .. s+1) and u_old(:, s .. s+2) of one subproblem (M = 4: 16 + 24 dwords) into this wave's LDS words, one
// dword per lane (LDS-DMA, inline asm: the compiler would otherwise make later LDS accesses wait for it); exactly one
// vector-memory instruction per wave.  s <= nt - 2; u_old(:, nt) does not exist: those lanes read u_old(:, nt - 1)
// (the caller never uses u_old(:, s+2) at s = nt - 2)
__device__ __forceinline__ void s2_dfuo_dma(const double *dfk, const double *uok, int s, int nt, unsigned char *sds) {
  // (the lane's offsets from an opaque thread index, recomputed per call: held across the loop they were spilled, and
  // the reload's vmcnt(0) waited for the values A issued just before)
  const int t = sd_tid(), wave = t >> 6, lane = t & 63;
  if (lane < 40) {
    const int e = min(4 * 2 * s + (lane - 16), 4 * 2 * nt - 1);  // dword index into u_old(:, :) (8 dwords per step)
    const char *g = lane < 16 ? (const char *)(dfk + (size_t)s * 4) + 4 * lane : (const char *)uok + 4 * (size_t)e;
    const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char *)(sds + S2_DFUO)) +
                          wave * (unsigned)S2_DFUO_WAVE;
    const unsigned m0 = __builtin_amdgcn_readfirstlane(lds0);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(m0)
                 : "memory");
  }
}

__device__ __forceinline__ double s2_wave_min(double x) {
  x = sd_min(x, sd_dpp_d<0xB1>(x));
  x = sd_min(x, sd_dpp_d<0x4E>(x));
  x = sd_min(x, sd_dpp_d<0x141>(x));
  x = sd_min(x, sd_dpp_d<0x140>(x));
  return sd_min(sd_min(sd_rdl(x, 0), sd_rdl(x, 16)), sd_min(sd_rdl(x, 32), sd_rdl(x, 48)));
}

// the rank of a level-value tuple on the 8^4 grid (u on the grid)
__device__ __forceinline__ int s2_rank(const double *u, const int *lb) {
  int r = 0;
#pragma unroll
  for (int m = 0; m < 4; ++m) r |= ((int)u[m] - lb[m]) << (3 * m);
  return r;
}

// Exact scan of the listed targets (the reference loop, HelpFunctions.jl:60-77): as sd_scan (mioc_sdt.hip) for T
// threads; outputs at the swizzled positions
template <int T, bool COOP>
__device__ __forceinline__ void s2_scan(const uint16_t *list, int nl, const double *psi, const double *a,
                                        const int *base, double beta, uint16_t *UU, double *outs, double *redv,
                                        int *redj) {
  constexpr int NW = T / 64;
  const int tid = sd_tid(), lane = tid & 63, w = tid >> 6;
  auto target = [&](int r, int *xl) {
    double t1 = 0.0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      xl[m] = (r >> (3 * m)) & 7;
      t1 = t1 + a[m] * (double)(base[m] + xl[m]);  // ((0 + (Δt·df_1)·ν_1) + ...), HelpFunctions.jl:52-57
    }
    return t1;
  };
  auto better = [](double ov, int oj, double bv, int bj) {
    return oj >= 0 && (bj < 0 || ov < bv || (ov == bv && oj < bj));
  };
  auto wave_min = [&](double &bv, int &bj) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const double ov = __shfl_xor(bv, off);
      const int oj = __shfl_xor(bj, off);
      if (better(ov, oj, bv, bj)) {
        bv = ov;
        bj = oj;
      }
    }
  };
  if constexpr (COOP) {
    for (int e = 0; e < nl; ++e) {
      const int r = list[e];
      int xl[4];
      const double t1 = target(r, xl);
      const unsigned pr = sd_bytes((unsigned)r);
      double bv = INFINITY;
      int bj = -1;
#pragma unroll
      for (int s = 0; s < S2_L / T; ++s) {  // sources tid + T·s, ascending for this thread
        const int j = tid + T * s;
        const double val = (t1 + beta * (double)sd_l1(sd_bytes((unsigned)j), pr)) + psi[j];
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
    sd_bar();
    if (tid < nl) {
      double bv = INFINITY;
      int bj = -1;
      for (int q = 0; q < NW; ++q) {
        const double ov = redv[tid * NW + q];
        const int oj = redj[tid * NW + q];
        if (better(ov, oj, bv, bj)) {
          bv = ov;
          bj = oj;
        }
      }
      const int r = list[tid];
      if (bj >= 0) UU[r] = (uint16_t)bj;
      outs[sd_swz(r)] = bj >= 0 ? bv : INFINITY;
    }
  } else {
    for (int e = w; e < nl; e += NW) {
      const int r = list ? (int)list[e] : e;
      if (!list && !__builtin_isnan(outs[sd_swz(r)])) continue;  // overflowed list: every NaN-marked rank
      int xl[4];
      const double t1 = target(r, xl);
      const unsigned pr = sd_bytes((unsigned)r);
      double bv = INFINITY;
      int bj = -1;
      for (int t = 0; t < S2_L / 64; ++t) {
        const int j = lane + 64 * t;
        const double val = (t1 + beta * (double)sd_l1(sd_bytes((unsigned)j), pr)) + psi[j];
        if (val < bv) {
          bv = val;
          bj = j;
        }
      }
      wave_min(bv, bj);
      if (lane == 0) {
        if (bj >= 0) UU[r] = (uint16_t)bj;
        outs[sd_swz(r)] = bj >= 0 ? bv : INFINITY;
      }
    }
  }
}

#if defined(MIOC_STAMPS) && defined(MIOC_STAMPS_TL)
// timeline (diagnostic build): per workgroup and for 32 of its items from the middle of the run, s_memrealtime
// (100 MHz) at 8 points of an item; kept in LDS during the launch (a global store would join the vector-memory queue
// the item's counted waits rely on) and copied out at the end
__device__ unsigned long long g_sdt2_tl[1024][32][8];
__shared__ unsigned long long s2_tl_lds[32][8];
__device__ unsigned long long g_sdt2_tlx[1024][32][4];  // extra points: 0 item-start wait done, 1 head parts in, 2 spins
__shared__ unsigned long long s2_tlx_lds[32][4];
#define S2_TLX(k, v)                                                            \
  do {                                                                          \
    if (threadIdx.x == 0 && tl_on) s2_tlx_lds[item - tl_item0][k] = (v);       \
  } while (0)
#define S2_TL(k)                                                                                                \
  do {                                                                                                          \
    if (threadIdx.x == 0 && tl_on) s2_tl_lds[item - tl_item0][k] = __builtin_amdgcn_s_memrealtime();          \
  } while (0)
#else
#define S2_TL(k) \
  do {           \
  } while (0)
#define S2_TLX(k, v) \
  do {               \
  } while (0)
#endif

}  // namespace

// The persistent DP, two workgroups per budget row (see the file header).  Grid: 2·K·B workgroups of 256 threads,
// two resident per CU (the host checks); flags: done [K][B+1][2], loaded [K][B+1][2], then the error word (zeroed);
// heads [K][B+1][nt][4]: item (c', i)'s four waves' parts of the head minimum (*), all-ones (a NaN) until written.
template <int T>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(T == 512 ? 4 : 2))) void k_sdt_pair(ProblemDev P, LevelsDev Lv, PyrGeom G,
                                                     const uint32_t *__restrict__ pack_all,
                                                     const uint32_t *__restrict__ seam_all, double *S_all,
                                                     size_t kstride, int NB, uint16_t *__restrict__ UU_all,
                                                     size_t uu_stride_k, int32_t *__restrict__ counters,
                                                     int32_t *flags, double *heads, unsigned spin_limit,
                                                     const double *__restrict__ df_all,
                                                     const double *__restrict__ uo_all) {
  constexpr int M = 4, L = S2_L, Smax = 7 * M;
  using C = S2C<T>;
  constexpr int NW = C::NW, Q = C::Q, LN = C::LN, UB = C::UB;
  constexpr unsigned OOB = 0xFFFFFFF0u;
  extern __shared__ __attribute__((aligned(16))) unsigned char sds[];
  __shared__ S2Shared<NW> sh;
  double *psi = reinterpret_cast<double *>(sds + S2_PSI);
  double *dtv = reinterpret_cast<double *>(sds + S2_DTV);
  uint16_t *uu = reinterpret_cast<uint16_t *>(sds + S2_UU);
  uint16_t *list = reinterpret_cast<uint16_t *>(sds + S2_LIST);
  const double *dfuo = reinterpret_cast<const double *>(sds + S2_DFUO) + (threadIdx.x >> 6) * (S2_DFUO_WAVE / 8);
  const int B = P.B, R = B + 1, nt = P.nt, NR = P.K * B;
  if ((int)blockIdx.x >= 2 * NR) return;
  const int par = (int)blockIdx.x / NR, rid0 = (int)blockIdx.x - par * NR;
  // rows by XCD (blocks b and b + 8 share one under round-robin dispatch; speed only): consecutive rows -- which read
  // each other -- on one XCD; the two workgroups of a row (b, b + NR) too when NR % 8 == 0
  // and the second workgroups shifted by half the rows: under that dispatch blocks b and b + NR share a CU, and the two
  // workgroups of one row, which hand each other the head parts, fall into step and compete for the same SIMDs
  const int rid1 = NR % 8 == 0 ? (rid0 & 7) * (NR >> 3) + (rid0 >> 3) : rid0;
  const int rid = par ? (rid1 + NR / 2) % NR : rid1;
  const int k = rid / B, cp = 1 + rid % B;
  const int i0 = nt - 2 - par;  // this workgroup's first step; then i0 - 2, i0 - 4, ...
  if (i0 < 0) return;
  const int tid = threadIdx.x, lane = tid & 63;
  int32_t *done = flags + (size_t)k * R * 2, *loaded = flags + ((size_t)P.K + k) * R * 2;
  int32_t *err = flags + (size_t)P.K * R * 4;
  // the flag words and this row's head values through buffer resources: every wave issues the same stores, with
  // out-of-range offsets in all lanes but one (a fixed vector-memory sequence per wave, for the counted waits)
  const __amdgpu_buffer_rsrc_t frs = __builtin_amdgcn_make_buffer_rsrc(flags, 0, (int)(((size_t)P.K * R * 4 + 1) * 4), 0x00020000);
  double *hk = heads + ((size_t)k * R + cp) * nt * NW;  // item (cp, s)'s wave parts at hk[NW·s .. NW·s + NW-1]
  const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(hk, 0, nt * NW * 8, 0x00020000);
  const unsigned rowb = (unsigned)L * 8u, bufb = (unsigned)R * rowb, r0b = (unsigned)NB * bufb;
  double *reg = S_all + (size_t)k * kstride;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(reg, 0, (int)(r0b + (unsigned)nt * rowb), 0x00020000);
  const uint32_t *pk = pack_all + (size_t)k * nt * S2_PACK;
  const uint32_t *sk = seam_all + (size_t)k * nt * (NW * S2_SEAMS);
  const double *dfk = df_all + (size_t)k * nt * M, *uok = uo_all + (size_t)k * nt * M;
  auto tok = [&](int s) { return nt - 1 - s; };
  auto parof = [&](int s) { return (nt - 2 - s) & 1; };
  auto pstep = [&](int s) { return min(max(s, 0), nt - 1); };
  auto boffs = [&](int s) { return (unsigned)(s % NB) * bufb; };
  const int lb[M] = {G.base[0], G.base[1], G.base[2], G.base[3]};
  const double beta = Lv.beta, inv = Lv.inv_beta;
#if defined(MIOC_STAMPS) && defined(MIOC_STAMPS_TL)
  const int tl_item0 = (nt / 2 - par) / 2;  // items from the middle of the run
  bool tl_on = false;
#endif
  if (tid == 0) {
    sh.stop = 0;
    sh.cnt[0] = sh.cnt[1] = 0;
  }
  // a wave-uniform wait for one flag word per lane (lanes with nothing to wait for point at row 0's words, never
  // written, with need 0); false (and the launch abandoned) past the spin limit
  auto spin = [&](const int32_t *fp, int need, int &val) {
    unsigned spins = 0;
    while (!__all(val >= need)) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || ++spins > spin_limit) {
        if (lane == 0) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          sh.stop = 1;  // read after the next barrier: the launch is abandoned
        }
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
      val = __hip_atomic_load(fp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return true;
  };
  // The words item ii's go() checks: lanes 0..27 rows cp - s of step ii-1 (RAW, the values of the item after it) and
  // rows cp + s of step ii+NB-1 (WAR: the readers of the step that buffer ii % NB held before item ii's stores)
  struct Deps {
    int32_t *fp1, *fp2;
    int need1, need2;
  };
  auto deps = [&](int ii, int ln) {
    Deps d{done, done, 0, 0};  // row 0's words: never written, needed 0
    const int s = ln + 1;
    if (ln < Smax) {
      const int rd = cp - s, ru = cp + s, sw = ii + NB - 1;
      if (ii - 2 >= 0 && rd >= 1) {
        d.fp1 = done + 2 * rd + parof(ii - 1);
        d.need1 = tok(ii - 1);
      }
      if (ru <= B && sw <= nt - 2) {
        d.fp2 = loaded + 2 * ru + parof(sw);
        d.need2 = tok(sw);
      }
    }
    return d;
  };
  // The partner's head parts of step ii+1 (lanes 0..3; all-ones until that item has stored them), which item ii reads
  // before its first wait: loaded one item ahead, before the stores, so that the wait on them does not wait for the
  // stores
  auto parts_load = [&](int ii, int ln) {
    const unsigned long long *src =
        reinterpret_cast<const unsigned long long *>(hk + NW * min(max(ii + 1, 0), nt - 1) + (ln & (NW - 1)));
    return __longlong_as_double((long long)__hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  };
  double pp;  // the partner's head parts (lanes 0 .. NW-1)
  double Hprev = INFINITY;  // Φ_{i+2}[cp, h(i+2)]: the previous item's head value (+Inf: the terminal row at cp >= 1)
  // ---- prologue: the first item's sphere orders and values; the next item's A orders ----------------------------
  // orders of steps i+1 (values A: the previous item's eAn across the back edge), i-1 (the next item's A: loaded at
  // the item start) and i (outputs: loaded at go(), read at the item's end) -- eO and eAn are not held across the
  // transform and the scan together (the 512-thread variant's register cap)
  S2Ent<Q> eA;
  s2_ent_issue(eA, pk + (size_t)pstep(i0 + 1) * S2_PACK, sk + (size_t)pstep(i0 + 1) * (NW * S2_SEAMS));
  s2_dfuo_dma(dfk, uok, i0, nt, sds);
  // the second workgroup's first item reads step nt-2, which the first workgroups of the rows below produce
  if (par == 1) {
    const int s = lane + 1, r = cp - s;
    int32_t *fp = done;  // row 0's flag word: never written, needed 0
    int need = 0;
    if (lane < Smax && r >= 1) {
      fp = done + 2 * r + parof(nt - 2);
      need = tok(nt - 2);
    }
    int val = __hip_atomic_load(fp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    spin(fp, need, val);
  }
  pp = parts_load(i0, lane);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the orders are in
  sd_bar();
  S2Raw<Q> rA;
  s2_issue<T>(rA, rs, eA, cp, boffs(i0 + 1), r0b + (unsigned)(i0 + 1) * rowb, rowb, sh.stop == 0);
  __builtin_amdgcn_s_waitcnt(0x0F70);
  sd_bar();
  bool stop = sh.stop != 0;
  int prev_i = -1;  // the previous item (its `done` is published in this one)
  int item = 0;
#pragma nounroll
  for (int i = i0; i >= 0 && !stop; i -= 2, ++item) {
#if defined(MIOC_STAMPS) && defined(MIOC_STAMPS_TL)
    tl_on = item >= tl_item0 && item < tl_item0 + 32;
#endif
    S2_TL(0);
    // the thread index as an opaque value (sd_tid): the lane's LDS addresses are recomputed per item instead of being
    // hoisted out of the loop into registers held across every item
    const int tid = sd_tid(), lane = tid & 63, w = tid >> 6;
    const bool has_next = i - 2 >= 0;
    // everything but the previous item's ten stores has landed: this item's values, orders, df / u_old, the partner's
    // head parts and the go() words
    if constexpr (C::NST == 10)
      asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    static_assert(C::NST == 10 || C::NST == 5, "the item start's count");
    S2_TLX(0, __builtin_amdgcn_s_memrealtime());
    S2Ent<Q> eAn;  // the order of step i-1 (the values the go() below issues)
    s2_ent_issue(eAn, pk + (size_t)pstep(i - 1) * S2_PACK, sk + (size_t)pstep(i - 1) * (NW * S2_SEAMS));
    asm volatile("" ::: "memory");
    // ---- the step's scalars (this wave's LDS copy): df(:, i .. i+1), u_old(:, i .. i+2) -----------------------------
    // (the same in every lane: read into scalars)
    auto sread = [&](int e) {
      const double x = dfuo[e];
      return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(x)),
                              __builtin_amdgcn_readfirstlane(__double2loint(x)));
    };
    double a[M], an[M], u0[M], u1[M], u2[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      a[m] = P.dt * sread(m);        // Δt·df(m, i)
      an[m] = P.dt * sread(M + m);   // Δt·df(m, i+1)
      u0[m] = sread(2 * M + m);
      u1[m] = sread(3 * M + m);
      u2[m] = sread(4 * M + m);
    }
    const int h0 = s2_rank(u0, lb), h1 = s2_rank(u1, lb);
    const bool sameH = h0 == h1;  // d(h(i), j) = b̃_j(i+1) (the sphere index of step i+1) for every j
    // T1(h(i), i), left to right (HelpFunctions.jl:52-57): the level values of h(i) are u_old(:, i)
    double T1H = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) T1H = T1H + a[m] * u0[m];
    int d01 = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) d01 += abs((int)u0[m] - (int)u1[m]);
    const unsigned hb0 = sd_bytes((unsigned)h0);
    // ---- this item's values A: Ψ by rank, raw into the transform buffer, the row's statistics -------------------
    double v[2 * Q], xs;
    s2_take(v, xs, rA);
    const int srank = (int)(eA.seam >> 16);
    const bool shas = lane < 32 && eA.seam != 0xFFFFFFFFu;
    // ---- this item's part of its own head value Φ_i[c', h(i)] (b̃ = 0, row c'), the chain (*): the minimum over the
    // values of this wave, stored at once for the partner's next item (one lane per wave; every wave issues the store)
    double hp = INFINITY;
    {
      auto cand = [&](double x, unsigned d) { return (T1H + beta * (double)d) + x; };  // HelpFunctions.jl:67,71
      if (sameH) {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          const unsigned d = (unsigned)s2_bt(eA.w[q]);
          hp = sd_min(hp, sd_min(cand(v[2 * q], d), cand(v[2 * q + 1], d)));
        }
        hp = sd_min(hp, cand(xs, (eA.seam >> 10) & 31u));
      } else {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
          hp = sd_min(hp, sd_min(cand(v[2 * q], sd_l1(sd_bytes((unsigned)s2_ra(eA.w[q])), hb0)),
                                 cand(v[2 * q + 1], sd_l1(sd_bytes((unsigned)s2_rb(eA.w[q])), hb0))));
        }
        hp = sd_min(hp, cand(xs, sd_l1(sd_bytes(eA.seam >> 16), hb0)));
      }
      hp = s2_wave_min(hp);
      __builtin_amdgcn_raw_buffer_store_b64((sd_u32x2){(unsigned)__double2loint(hp), (unsigned)__double2hiint(hp)},
                                            hrs, lane == 0 ? (unsigned)(NW * i + w) * 8u : OOB, 0, 16);
    }
    // ---- the value at this item's head position, Φ_{i+1}[c', h(i+1)] = min(the partner's parts over the values of its
    // item (c', i+1), the term j = h(i+2): fl(fl(T1(h(i+1), i+1) + β·d(h(i+1), h(i+2))) + Φ_{i+2}[c', h(i+2)])); +Inf at
    // the terminal step (Φ_{nt-1} is finite at budget b̃ only) -------------------------------------------------------
    double l0v = INFINITY;
    if (i < nt - 2) {
      {  // the parts were loaded one item ahead; a part still all-ones (not yet stored) is polled here
        // (the first test outside the loop: its operand is the tail load, which the item start's count covers)
        bool okp = !__any(lane < NW && __double_as_longlong(pp) == -1ll);
        unsigned spins = 0;
        while (!okp) {
          if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || ++spins > spin_limit) {
            if (lane == 0) {
              __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              sh.stop = 1;
            }
            pp = INFINITY;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          pp = __longlong_as_double((long long)__hip_atomic_load(
              reinterpret_cast<const unsigned long long *>(hk + NW * (i + 1) + (lane & (NW - 1))), __ATOMIC_RELAXED,
              __HIP_MEMORY_SCOPE_AGENT));
          okp = !__any(lane < NW && __double_as_longlong(pp) == -1ll);
        }
        S2_TLX(2, spins);
      }
      double T1P = 0.0;  // T1(h(i+1), i+1), left to right (HelpFunctions.jl:52-57)
#pragma unroll
      for (int m = 0; m < M; ++m) T1P = T1P + an[m] * u1[m];
      int d12 = 0;
#pragma unroll
      for (int m = 0; m < M; ++m) d12 += abs((int)u1[m] - (int)u2[m]);
      l0v = (T1P + beta * (double)d12) + Hprev;  // HelpFunctions.jl:67,71
#pragma unroll
      for (int q = 0; q < NW; ++q) l0v = sd_min(l0v, sd_rdl(pp, q));
    }
    S2_TLX(1, __builtin_amdgcn_s_memrealtime());
    // this lane's targets: the lines q = tid and tid + 256 of the last pass, ranks q | x << 9
    int uo[M];
#pragma unroll
    for (int m = 0; m < M; ++m) uo[m] = __builtin_amdgcn_readfirstlane((int)u0[m]);
    double pre[LN];
    unsigned valid = 0;
    int nv = 0;
#pragma unroll
    for (int ln = 0; ln < LN; ++ln) {
      const int q = tid + T * ln;
      double t = 0.0;
      int bp = 0;
#pragma unroll
      for (int m = 0; m < M - 1; ++m) {
        const int nu = lb[m] + ((q >> (3 * m)) & 7);
        t = t + a[m] * (double)nu;  // ((0 + (Δt·df_1)·ν_1) + ...), HelpFunctions.jl:52-57
        bp += abs(nu - uo[m]);
      }
      pre[ln] = t;
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        const bool in = bp <= B - cp - abs(lb[M - 1] + x - uo[M - 1]);  // c' + b̃_l(i) <= B
        valid |= (unsigned)in << (8 * ln + x);
        nv += __popcll(__ballot(in));
      }
    }
    if (tid == 0) sh.nlist = 0;
    double pmn = INFINITY, pmx = -INFINITY;
#pragma unroll
    for (int q = 0; q < Q; ++q)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const double x = v[2 * q + hh];
        const int j = hh ? s2_rb(eA.w[q]) : s2_ra(eA.w[q]);
        // written anyway (+Inf where this lane has no value): a straddling second element is written after this by
        // its seam lane of the same wave (in-wave LDS order); the head after the barrier
        psi[j] = x;
        dtv[sd_swz(j)] = x;
        const bool fin = x < INFINITY;
        nv += __popcll(__ballot(fin)) << 16;
        pmn = sd_min(pmn, x);
        pmx = sd_max(pmx, __hiloint2double(fin ? __double2hiint(x) : (int)0xFFF00000, __double2loint(x)));
      }
    {
      const bool fin = shas && xs < INFINITY;
      nv += __popcll(__ballot(fin)) << 16;
      if (shas) {
        psi[srank] = xs;
        dtv[sd_swz(srank)] = xs;
      }
      pmn = sd_min(pmn, fin ? xs : INFINITY);
      pmx = sd_max(pmx, fin ? xs : -INFINITY);
    }
    sd_wave_stats(pmn, pmx);
    if (lane == 0) {
      sh.rmn[w] = pmn;
      sh.rmx[w] = pmx;
      sh.rnv[w] = nv;
      sh.pmin[w] = hp;
    }
    S2_TL(1);
    // every wave's stores of the previous item have landed (all but this item's head part, younger)
    asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    sd_bar();  // (1) every wave has consumed its values (in LDS now): `loaded`; the statistics are in; the previous
               // item is complete: `done`
    // ---- this item's head value (the next item's head term) and `loaded` (one lane; every wave issues the store) ------
    {
      double hm = (T1H + beta * (double)d01) + l0v;  // the term j = h(i+1) of (*)
#pragma unroll
      for (int q = 0; q < NW; ++q) hm = sd_min(hm, sh.pmin[q]);
      Hprev = hm;
    }
    // go()'s words, checked after the winners
    const Deps dp = deps(i, lane);
    int val1 = __hip_atomic_load(dp.fp1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int val2 = __hip_atomic_load(dp.fp2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    {
      __builtin_amdgcn_raw_buffer_store_b32((unsigned)tok(i), frs,
                                            tid == T - 64 ? (unsigned)((size_t)(loaded + 2 * cp + par) - (size_t)flags)
                                                             : OOB,
                                            0, 16);
      __builtin_amdgcn_raw_buffer_store_b32((unsigned)tok(prev_i), frs,
                                            tid == T - 64 && prev_i >= 0
                                                ? (unsigned)((size_t)(done + 2 * cp + par) - (size_t)flags)
                                                : OOB,
                                            0, 16);
    }
    // ---- the row's statistics, the A head h(i+1) -------------------------------------------------------------------
    double pmn2 = INFINITY, pmx2 = -INFINITY;
    nv = 0;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      pmn2 = sd_min(pmn2, sh.rmn[q]);
      pmx2 = sd_max(pmx2, sh.rmx[q]);
      nv += sh.rnv[q];
    }
    int nf = (nv >> 16) + (l0v < INFINITY ? 1 : 0);
    nv &= 0xFFFF;
    pmn2 = sd_min(pmn2, l0v);
    pmx2 = sd_max(pmx2, l0v < INFINITY ? l0v : -INFINITY);
    if (lane == 0 && w == ((h1 >> 9) & 3)) {  // the wave whose pass 0 reads rank h(i+1) (in-wave order)
      psi[h1] = l0v;
      dtv[sd_swz(h1)] = l0v;
    }
    // no target in the trust region, or nothing reachable: the row is +Inf and U unwritten (0xFFFF)
    const bool empty = __builtin_amdgcn_readfirstlane((int)(nv == 0 || !(pmn2 < INFINITY))) != 0;
    // ---- the binade: values base + (Ψ - ref)/β + d lie in [base, 2·base), grid g = 2^18 ulp ------------------------
    double qa = beta * (double)Smax;  // |T1 + β·d + Ψ| <= qa + max(|lo|, |hi|) for every candidate
#pragma unroll
    for (int m = 0; m < M; ++m) qa += fabs(a[m]) * (double)max(abs(lb[m]), abs(lb[m] + 7));
    double ref, base, tol;
    bool scale_ok;
    {
      const double lo = pmn2, hi = pmx2;
      const double rs_ = (hi - lo) * inv + (double)Smax;
      scale_ok = rs_ < 0x1p31;
      const int E = ilogb(fmin(rs_, 0x1p31) * (1.0 + 0x1p-20) + 1.0) + 2;
      base = ldexp(1.0, E);
      const double g = ldexp(1.0, E - SD_GRID);
      tol = 3.0 * g + 0x1p-49 * (qa + fmax(fabs(lo), fabs(hi))) * inv;
      ref = lo;
    }
    auto stamp = [&](double x, int j) {
      const double y = (x - ref) * inv + base;
      return __hiloint2double(__double2hiint(y), (__double2loint(y) & ~SD_PAY) | (j << SD_CB));
    };
    auto stamp_inf = [&](double x, int j) {
      const double y = stamp(x, j);
      const unsigned mk = x < INFINITY ? ~0u : 0u;
      return __hiloint2double((int)(((unsigned)__double2hiint(y) & mk) | (0x7FF00000u & ~mk)),
                              (int)((unsigned)__double2loint(y) & mk));
    };
    const bool sparse = !empty && nf <= SD_SPARSE;
    const bool direct = !empty && !sparse && (nv <= SD_FEW || !scale_ok || !(tol < base * 0x1p-20));
    if (sparse) {  // few finite sources (rows near c' = 0): every target's minimum over them, directly
      if (tid == 0) sh.nsp = 0;
      sd_bar();
#pragma unroll
      for (int q = 0; q < Q; ++q)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh)
          if (v[2 * q + hh] < INFINITY) {
            const int e = atomicAdd(&sh.nsp, 1);
            sh.spj[e] = hh ? s2_rb(eA.w[q]) : s2_ra(eA.w[q]);
            sh.spv[e] = v[2 * q + hh];
          }
      if (shas && xs < INFINITY) {
        const int e = atomicAdd(&sh.nsp, 1);
        sh.spj[e] = srank;
        sh.spv[e] = xs;
      }
      if (tid == 0 && l0v < INFINITY) {
        const int e = atomicAdd(&sh.nsp, 1);
        sh.spj[e] = h1;
        sh.spv[e] = l0v;
      }
      sd_bar();  // (the sources are read from LDS below: broadcast reads)
    }
    const bool transform = !direct && !empty && !sparse;
    S2_TL(2);
    // ---- the transform -------------------------------------------------------------------------------------------
    auto pos3 = [&](int e) { return sd_swz((sd_tid() + T * (e >> 3)) | ((e & 7) << 9)); };
    // an opaque zero: the targets' T1 terms a_3·ν_3 are recomputed per target (two VALU) instead of being hoisted into
    // registers that would be spilled
    int zop = 0;
    asm volatile("" : "+v"(zop));
    if (transform) {
      double o[8 * LN];
      auto pass = [&](int m) {
        int pos[8 * LN];
#pragma unroll
        for (int ln = 0; ln < LN; ++ln)
#pragma unroll
          for (int x = 0; x < 8; ++x) {
            pos[8 * ln + x] = sd_swz(sd_rank(tid + T * ln, m, x));
            o[8 * ln + x] = dtv[pos[8 * ln + x]];
          }
        if (m == 0) {  // the raw Ψ of ranks 8q + x: stamp them here
#pragma unroll
          for (int ln = 0; ln < LN; ++ln)
#pragma unroll
            for (int x = 0; x < 8; ++x) o[8 * ln + x] = stamp_inf(o[8 * ln + x], sd_rank(tid + T * ln, 0, x));
        }
        // forward then backward sweep of both lines, interleaved (two independent chains)
#pragma unroll
        for (int x = 1; x < 8; ++x) {
          o[x] = sd_merge(o[x], o[x - 1] + 1.0, tol);
          o[8 + x] = sd_merge(o[8 + x], o[7 + x] + 1.0, tol);
        }
#pragma unroll
        for (int x = 6; x >= 0; --x) {
          o[x] = sd_merge(o[x], o[x + 1] + 1.0, tol);
          o[8 + x] = sd_merge(o[8 + x], o[9 + x] + 1.0, tol);
        }
        if (m + 1 < M) {
#pragma unroll
          for (int x = 0; x < 8 * LN; ++x) dtv[pos[x]] = o[x];
        }
      };
      pass(0);
      sd_wave_sync();
      pass(1);
      sd_wave_sync();
      pass(2);
    }
    if (transform) sd_bar();  // (2) the last pass runs along x3: every wave's values
    S2_TL(3);
    // ---- targets: R(l, j*) for a certified winner, the others listed for the exact scan ---------------------------
    // (outputs at the swizzled positions the last pass read: each lane writes only its own)
    unsigned listed = 0;
    if (empty) {
#pragma unroll
      for (int x = 0; x < 8 * LN; ++x) dtv[pos3(x)] = INFINITY;
#pragma unroll
      for (int ub = 0; ub < UB; ++ub) reinterpret_cast<ulonglong2 *>(uu)[UB * tid + ub] = make_ulonglong2(~0ull, ~0ull);
    } else if (transform) {
#pragma unroll
      for (int ln = 0; ln < LN; ++ln) {
        // the last pass (along x3) on this line, then its eight winners (their Ψ reads issue together)
        double o[8];
#pragma unroll
        for (int x = 0; x < 8; ++x) o[x] = dtv[pos3(8 * ln + x)];
#pragma unroll
        for (int x = 1; x < 8; ++x) o[x] = sd_merge(o[x], o[x - 1] + 1.0, tol);
#pragma unroll
        for (int x = 6; x >= 0; --x) o[x] = sd_merge(o[x], o[x + 1] + 1.0, tol);
        int jx[8];
        double pv[8];
#pragma unroll
        for (int x = 0; x < 8; ++x) jx[x] = (__double2loint(o[x]) >> SD_CB) & ((1 << SD_RB) - 1);
#pragma unroll
        for (int x = 0; x < 8; ++x) pv[x] = psi[jx[x]];
#pragma unroll
        for (int x = 0; x < 8; ++x) {
          const int e = 8 * ln + x, r = (tid + T * ln) | (x << 9), j = jx[x];
          const bool fin = (valid >> e & 1) && o[x] < INFINITY;
          const bool flg = (__double2loint(o[x]) & SD_CNT) != 0;
          // d(l, j*) exactly: an unflagged finite o is V_j* + d with V_j* the stamp of Ψ_j*
          const double dd = o[x] - stamp(pv[x], j);
          const double t1 = pre[ln] + a[M - 1] * (double)(lb[M - 1] + x + zop);
          const double val = (t1 + beta * dd) + pv[x];  // R(l, j*), HelpFunctions.jl:63-71
          listed |= (unsigned)(fin && flg) << e;
          uu[r] = (uint16_t)(fin && !flg ? j : 0xFFFF);
          dtv[pos3(e)] = fin ? (flg ? __longlong_as_double(0x7FF8000000000000ll) : val) : INFINITY;
        }
      }
    } else {
#pragma unroll
      for (int ln = 0; ln < LN; ++ln)
#pragma unroll
        for (int x = 0; x < 8; ++x) {
          const int e = 8 * ln + x, r = (tid + T * ln) | (x << 9);
          double ov = INFINITY;
          int uj = 0xFFFF;
          if (direct) {
            listed |= valid & (1u << e);
          } else if (valid >> e & 1) {  // sparse: the reference loop over the finite sources, ties to the lower rank
            const double t1 = pre[ln] + a[M - 1] * (double)(lb[M - 1] + x + zop);
            double bv = INFINITY;
            int bj = 0xFFFF;
            for (int q = 0; q < nf; ++q) {
              {
                const int j = sh.spj[q];
                const double val = (t1 + beta * (double)sd_l1(sd_bytes((unsigned)j), sd_bytes((unsigned)r))) + sh.spv[q];
                if (val < bv || (val == bv && j < bj)) {
                  bv = val;
                  bj = j;
                }
              }
            }
            ov = bv;
            uj = bj;
          }
          uu[r] = (uint16_t)uj;
          dtv[pos3(e)] = (listed >> e & 1) ? __longlong_as_double(0x7FF8000000000000ll) : ov;
        }
    }
    if (listed) {
      int e = atomicAdd(&sh.nlist, __popc(listed));
#pragma unroll
      for (int x = 0; x < 8 * LN; ++x)
        if (listed >> x & 1) {
          if (e < SD_LCAP) list[e] = (uint16_t)((tid + T * (x >> 3)) | ((x & 7) << 9));
          ++e;
        }
    }
    S2_TL(4);
    // the order of step i (this item's outputs, read after the scan): issued before the next item's loads, so that the
    // gather waits for it alone
    S2Ent<Q> eO;
    s2_ent_issue(eO, pk + (size_t)i * S2_PACK, sk + (size_t)i * (NW * S2_SEAMS));
    asm volatile("" ::: "memory");  // (issued here, not sunk below the next item's loads)
#if defined(MIOC_STAMPS) && defined(MIOC_STAMPS_TL)
    unsigned long long tl_bits = 0;
#endif
    // ---- go(): this wave's polls matched (RAW: the rows below have published step i-1; WAR: the rows above have
    // loaded the step this item's stores overwrite) -> the next item's loads (values A of step i-1, its df / u_old) --
    {
      int32_t *const fp1 = dp.fp1, *const fp2 = dp.fp2;
      const int need1 = dp.need1, need2 = dp.need2;
      bool ready = __all(val1 >= need1 && val2 >= need2);
#if defined(MIOC_STAMPS) && defined(MIOC_STAMPS_TL)
      // the first test's outcome in the stamp's top bits: 62 RAW unmet, 61 WAR unmet
      tl_bits = (__all(val1 >= need1) ? 0ull : 1ull << 62) | (__all(val2 >= need2) ? 0ull : 1ull << 61);
#endif
      unsigned spins = 0;
      while (!ready) {
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || ++spins > spin_limit) {
          if (lane == 0) {
            __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sh.stop = 1;  // read after the next barrier: the launch is abandoned
          }
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        val1 = __hip_atomic_load(fp1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        val2 = __hip_atomic_load(fp2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ready = __all(val1 >= need1 && val2 >= need2);
      }
      const int ni = i - 2;
      s2_issue<T>(rA, rs, eAn, cp, boffs(pstep(ni + 1)), r0b + (unsigned)pstep(ni + 1) * rowb, rowb, has_next);
      s2_dfuo_dma(dfk, uok, pstep(ni), nt, sds);
    }
    S2_TL(5);
#if defined(MIOC_STAMPS) && defined(MIOC_STAMPS_TL)
    if (threadIdx.x == 0 && tl_on) s2_tl_lds[item - tl_item0][5] |= tl_bits;
#endif
    S2_TL(6);
    sd_bar();  // (3) the list is complete
    const int nl = sh.nlist;
    if (nl) {
      if (nl <= SD_COOP)
        s2_scan<T, true>(list, nl, psi, a, lb, beta, uu, dtv, sh.redv, sh.redj);
      else if (nl <= SD_LCAP)
        s2_scan<T, false>(list, nl, psi, a, lb, beta, uu, dtv, sh.redv, sh.redj);
      else
        s2_scan<T, false>(nullptr, L, psi, a, lb, beta, uu, dtv, sh.redv, sh.redj);  // every NaN-marked rank
      sd_bar();
      if (tid == 0) sh.cnt[direct ? 1 : 0] += nl;
    }
    // ---- row c' of S_i in the sphere order of u_old(i), the U row ---------------------------------------------------
    unsigned long long so[2 * Q];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      so[2 * q] = __double_as_longlong(dtv[sd_swz(s2_ra(eO.w[q]))]);
      so[2 * q + 1] = __double_as_longlong(dtv[sd_swz(s2_rb(eO.w[q]))]);
    }
    // (two named values, not an array: an array of them went to scratch)
    const ulonglong2 ua = reinterpret_cast<const ulonglong2 *>(uu)[UB * tid];
    const ulonglong2 ub = UB > 1 ? reinterpret_cast<const ulonglong2 *>(uu)[UB * tid + 1] : ua;
    eA = eAn;  // the next item's values A
    sd_bar();  // (4) every wave has read the outputs: the next item may overwrite the buffers
    stop = sh.stop != 0;
    pp = parts_load(i - 2, lane);  // before the stores (the next item's first wait does not wait for them)
    {
      const __amdgpu_buffer_rsrc_t rso = sd_rsrc(reg + (size_t)(i % NB) * R * L + (size_t)cp * L, L * 8);
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        const sd_u32x4 d = {(unsigned)so[2 * q], (unsigned)(so[2 * q] >> 32), (unsigned)so[2 * q + 1],
                            (unsigned)(so[2 * q + 1] >> 32)};
        __builtin_amdgcn_raw_buffer_store_b128(d, rso, 2 * (tid + T * q) * 8, 0, 16);
      }
      ulonglong2 *Ur = reinterpret_cast<ulonglong2 *>(UU_all + (size_t)k * uu_stride_k + (size_t)i * ((size_t)R * L) +
                                                      (size_t)cp * L) + UB * tid;
      Ur[0] = ua;  // read by later launches only (backtrack)
      if constexpr (UB > 1) Ur[1] = ub;
    }
    S2_TL(7);
    prev_i = i;
  }
  // the last item: its stores drained, then published (the other workgroups of the rows above read step i_last)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  sd_bar();
  if (tid == 0) {
    if (!stop && prev_i >= 0)
      __hip_atomic_store(done + 2 * cp + par, tok(prev_i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (sh.cnt[0]) atomicAdd(&counters[0], sh.cnt[0]);
    if (sh.cnt[1]) atomicAdd(&counters[1], sh.cnt[1]);
#if defined(MIOC_STAMPS) && defined(MIOC_STAMPS_TL)
    if (blockIdx.x < 1024)
      for (int j = 0; j < 32; ++j)
        for (int q = 0; q < 8; ++q) g_sdt2_tl[blockIdx.x][j][q] = s2_tl_lds[j][q];
    if (blockIdx.x < 1024)
      for (int j = 0; j < 32; ++j)
        for (int q = 0; q < 4; ++q) g_sdt2_tlx[blockIdx.x][j][q] = s2_tlx_lds[j][q];
#endif
  }
}

bool sdt_pair_supported(const PyrGeom &G, int K, int B, int ncu, int bpc) {
  if (G.M != 4) return false;
  for (int m = 0; m < 4; ++m)
    if (G.n[m] != 8) return false;
  return B >= 1 && bpc >= 2 && (size_t)K * (size_t)B <= (size_t)ncu * (size_t)(bpc / 2);
}

size_t sdt_pair_lds_bytes(int threads) { return threads == 512 ? S2C<512>::LDS : S2C<256>::LDS; }

int sdt_pair_blocks_per_cu(int threads) {
  int n = 0;
  const hipError_t e =
      threads == 512
          ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_sdt_pair<512>, 512, S2C<512>::LDS)
          : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_sdt_pair<256>, 256, S2C<256>::LDS);
  return e == hipSuccess ? n : 0;
}

int sdt_pair_seam_words(int threads) { return threads / 64 * S2_SEAMS; }

hipError_t launch_sdt_pack(hipStream_t s, const ProblemDev &P, const uint32_t *perm, uint32_t *pack, uint32_t *seams,
                           int32_t *counters, int threads) {
  if (threads == 512)
    hipLaunchKernelGGL(k_sdt2_pack<512>, dim3(P.nt, P.K), dim3(512), 0, s, perm, P.nt, pack, seams, counters);
  else
    hipLaunchKernelGGL(k_sdt2_pack<256>, dim3(P.nt, P.K), dim3(256), 0, s, perm, P.nt, pack, seams, counters);
  return hipGetLastError();
}

hipError_t launch_sdt_pair(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G,
                           const uint32_t *pack, const uint32_t *seams, double *S, size_t kstride, int NB, uint16_t *UU,
                           size_t uu_stride_k, int32_t *counters, int32_t *flags, double *heads, unsigned spin_limit,
                           int threads) {
  // every workgroup must be resident (the caller checked 2·K·B <= CUs x resident workgroups per CU); an ordinary
  // launch (mioc_sdt.hip, launch_sdt_run: a cooperative launch crashed the profiler at exit)
  const double *df = P.df, *uo = P.uold;
  void *args[] = {(void *)&P,     (void *)&Lv,         (void *)&G,     (void *)&pack,       (void *)&seams,
                  (void *)&S,     (void *)&kstride,    (void *)&NB,    (void *)&UU,         (void *)&uu_stride_k,
                  (void *)&counters, (void *)&flags,   (void *)&heads, (void *)&spin_limit, (void *)&df,
                  (void *)&uo};
  if (threads == 512)
    return hipLaunchKernel((const void *)k_sdt_pair<512>, dim3(2 * P.K * P.B), dim3(512), args, S2C<512>::LDS, s);
  return hipLaunchKernel((const void *)k_sdt_pair<256>, dim3(2 * P.K * P.B), dim3(256), args, S2C<256>::LDS, s);
}

#if defined(MIOC_STAMPS) && defined(MIOC_STAMPS_TL)
extern "C" int32_t mioc_debug_sdt2_timeline_x(unsigned long long *out, int64_t nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sdt2_tlx), (size_t)nblocks * 32 * 4 * sizeof(unsigned long long)) ==
                 hipSuccess
             ? 0
             : -4;
}
extern "C" int32_t mioc_debug_sdt2_timeline(unsigned long long *out, int64_t nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sdt2_tl), (size_t)nblocks * 32 * 8 * sizeof(unsigned long long)) ==
                 hipSuccess
             ? 0
             : -4;
}
#endif

}  // namespace mioc
