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
//   - each finite Ψ_j becomes V_j = base + (Ψ_j - Ψmin)/β, truncated to the grid g = 2^18 ulp(base), with
//     the source rank j in mantissa bits 6..17 and a near-tie count in bits 0..5 (the payload);
//   - a unit step costs exactly 1.0 (a multiple of g), so every sum is exact and keeps its payload, and
//     v_min_f64 carries the winner's rank through every pass for free;
//   - every merge of two disjoint candidate sets whose values differ by <= tol adds one to the count of its result
//     (one v_addc on the low word: a value passes at most 14 merges per pass, 56 in all, so the count never reaches
//     the rank bits); a nonzero count is the "near tie" flag.
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
#include "mioc_sdt_common.h"

namespace mioc {

constexpr int SD_STRAD_N = 32;           // seam list entries per wave (<= 28 seams in a sphere order)
// the persistent driver at M = 4: the position pairs that straddle a sphere seam get their second element from one
// straddle load per lane (a per-wave list of the wave's seams, k_pyr_order) instead of one masked 8-byte load per pair
// and lane (SdRaw)
template <int M>
__host__ __device__ constexpr bool sd_strad() {
  return M == 4;
}

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
#define SD_TL_AT(gg, ii, ntt, k) \
  do {                           \
  } while (0)
#define SD_TL_FLUSH(gg) \
  do {                  \
  } while (0)
#elif defined(MIOC_STAMPS)
// persistent-kernel timeline (diagnostic build, make stamps_tl): per workgroup (its chunk's first row) and for the 64
// steps from nt/2 down, s_memrealtime (100 MHz) at 7 points of a row: 0 start, 1 loads consumed (h.early), 2 drain
// point, 3 after the drain barrier, 4 polls matched, 5 the next row's loads and DMAs issued, 6 stores issued.  Kept
// in LDS during the launch (a global store would join the vector-memory queue the driver counts) and copied out at
// the end.
__device__ unsigned long long g_sdt_tl[4096][64][8];
__shared__ unsigned long long sd_tl_lds[64][8];
#define SD_TL_AT(gg, ii, ntt, k)                                                                          \
  do {                                                                                                    \
    if (threadIdx.x == 0 && (gg) < 4096 && (unsigned)((ii) - ((ntt) >> 1)) < 64u)                          \
      sd_tl_lds[(ii) - ((ntt) >> 1)][k] = __builtin_amdgcn_s_memrealtime();                                \
  } while (0)
#define SD_TL(k) SD_TL_AT(g, i, P.nt, k)
#define SD_TL_FLUSH(gg)                                                                                   \
  do {                                                                                                    \
    if (threadIdx.x == 0 && (gg) < 4096)                                                                  \
      for (int _j = 0; _j < 64; ++_j)                                                                     \
        for (int _q = 0; _q < 8; ++_q) g_sdt_tl[gg][_j][_q] = sd_tl_lds[_j][_q];                           \
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
#define SD_TL_AT(gg, ii, ntt, k) \
  do {                           \
  } while (0)
#define SD_TL_FLUSH(gg) \
  do {                  \
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


// The first position of thread tid's q-th position pair (q < 4) in a staging row / sphere order: 2(tid + T·q), so a
// wave's pairs are 128 consecutive positions per q (16 bytes per lane: coalesced).
template <int M>
__device__ __forceinline__ int sd_p2(int tid, int q) {
  constexpr int L = 1 << (3 * M), T = L / 8;
  return 2 * (tid + T * q);
}
// (sd_strad) the position of in-wave offset o (0 .. 511) of wave w: the wave's four runs of 128 positions
// 2(64w + l + T·q) + {0, 1} (o = 128q + 2l + {0, 1}); k_pyr_order builds the seam lists with the same map
template <int M>
__device__ __forceinline__ int sd_seam_pos(int w, int o) {
  constexpr int L = 1 << (3 * M), T = L / 8;
  return 2 * T * (o >> 7) + 128 * w + (o & 127);
}
// The position of the level at distance 0 from u_old (when u_old is on the grid): the head of the first sphere,
// position 0 of the sphere order.  Callers check b̃ == 0 there.
constexpr int kSdHeadPos = 0;


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
  const int tid = sd_tid(), lane = tid & 63, w = tid >> 6;
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
    sd_bar();
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
  // by row parity (sdt_body's `par`): targets listed for the exact scan, and whether a near tie was met anywhere in
  // the row's first (non-counting) transform.  Each row resets the other parity's slots after its first barrier: the
  // row before has read them before that barrier, the row after writes them after its own first barrier.
  int nlist[2];
  int redo[2];
  int stop;  // persistent kernel: a dependency wait timed out
  unsigned long long stamp[16];  // diagnostic build: phase clocks of the current row
  int nsp;   // sparse rows: the finite sources (rank, Ψ)
  int spj[SD_SPARSE];
  double spv[SD_SPARSE];
  // targets sent to the exact scan (near ties, direct rows), flushed to the global counters [0], [1]; (persistent
  // driver) rows whose write-after-read wait on the rows above was armed (staging-buffer reuse), flushed to [4]; rows
  // whose transform met a near tie and was redone counting them, flushed to [5]
  int cnt[4];
};

template <int M>
__host__ __device__ constexpr size_t sd_slot_offset() {  // the two sphere-order slots follow the row body's arrays
  return ((size_t)1 << (3 * M)) * (2 * sizeof(double) + sizeof(uint16_t)) + SD_LCAP * sizeof(uint16_t);
}
// per wave: df(:, i) and u_old(:, i) (2M doubles), then one int32 flag (sphere-order reuse, SdPipe::go), padded to 16 B
template <int M>
__host__ __device__ constexpr size_t sd_dfuo_stride() {
  return (2 * M + 2) * sizeof(double);
}
template <int M>
__host__ __device__ constexpr size_t sd_strad_offset() {  // then the two slots' straddle lists (8 slabs x SD_STRAD_N)
  return sd_slot_offset<M>() + 2 * ((size_t)1 << (3 * M)) * sizeof(uint32_t);
}
template <int M>
__host__ __device__ constexpr size_t sd_dfuo_offset() {  // then df(:, i), u_old(:, i), a flag word per wave (persistent)
  return sd_strad_offset<M>() + 2 * 8 * SD_STRAD_N * sizeof(uint16_t);
}
template <int M>
__host__ __device__ constexpr size_t sd_out_offset() {  // then the row's outputs (natural order)
  return sd_dfuo_offset<M>() + ((sd_dfuo_stride<M>() * (((size_t)1 << (3 * M - 3)) / 64) + 255) & ~(size_t)255);
}
template <int M>
__host__ __device__ constexpr size_t sd_lds_total() {
  return sd_out_offset<M>() + ((size_t)1 << (3 * M)) * sizeof(double);
}


// The sphere orders a step reads (step i+1, for the sources) and writes (step i, for the output row), as the
// position pairs 2(tid + T·q) + {0, 1} of this thread, plus both heads (position 0).  Loaded at the start of
// a row (per-step kernel) or ahead of the dependency wait (persistent kernel): they are static, so their
// latency never sits behind a barrier.
struct SdPerm {
  uint2 in[4], out[4];
  uint32_t hin, hout;  // the sphere-order entries at the head positions pin_h (step i+1) and pout_h (step i)
  int pin_h, pout_h;
};
template <int M>
__device__ __forceinline__ void sd_perm_load(SdPerm &pm, const uint32_t *__restrict__ perm_all, const ProblemDev &P,
                                             const PyrGeom &G, int k, int i) {
  constexpr int T = 1 << (3 * M - 3);
  const int nt = P.nt;
  const uint32_t *pin = perm_all + ((size_t)k * nt + i + 1) * ((size_t)T * 8);
  const uint32_t *pout = perm_all + ((size_t)k * nt + i) * ((size_t)T * 8);
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    pm.in[q] = *reinterpret_cast<const uint2 *>(pin + sd_p2<M>(tid, q));
    pm.out[q] = *reinterpret_cast<const uint2 *>(pout + sd_p2<M>(tid, q));
  }
  pm.pin_h = kSdHeadPos;
  pm.pout_h = kSdHeadPos;
  pm.hin = pin[pm.pin_h];
  pm.hout = pout[pm.pout_h];
}

// The first phase of row c' of step i: its loaded Ψ (v: this thread's eight positions, + the straddle element srank / xs)
// into the LDS by rank (psi, for the winners and exact scans) and raw into the transform buffer (stamped by pass 0); the
// wave's min and max of Ψ and its counts (targets in the trust region, low 16 bits; finite sources, high 16 bits) into
// sh.rmn / rmx / rnv[w].  Returns this lane's trust-region targets (bit x: target tid | x << 3(M-1) has c' + b̃ <= B).
// The persistent driver runs it for the NEXT row at the end of a row (the next row's loads have landed by then: the
// row's late drain waited for them), where the row's stores leave the SIMDs idle; the row body then starts at the
// barrier that publishes these statistics.
template <int M, bool PERSIST>
__device__ __forceinline__ unsigned sdt_stats(const ProblemDev &P, const PyrGeom &G, int k, int cp, int i,
                                              const double (&v)[8], const uint2 (&ein)[4],
                                              SdtShared<(1 << (3 * M - 3)) / 64> &sh, unsigned char *sds,
                                              const double *__restrict__ df_all, const double *__restrict__ uo_all,
                                              int srank = -1, double xs = 0.0) {
  constexpr int L = 1 << (3 * M);
  double *psi = reinterpret_cast<double *>(sds);  // [L] Ψ_j by rank
  double *dtv = psi + L;                          // [L] transform values (swizzled)
  const int tid = sd_tid(), lane = tid & 63, w = tid >> 6;
  const int B = P.B;
  const double *uoi = PERSIST ? reinterpret_cast<const double *>(sds + sd_dfuo_offset<M>()) +
                                    (2 * M + 2) * (threadIdx.x >> 6) + M
                              : uo_all + ((size_t)k * P.nt + i) * M;
  (void)df_all;
  int lb[M], uo[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    lb[m] = G.base[m];
    // u_old(:, i) is the same for every lane: as a scalar, the trust-region thresholds below are scalar arithmetic
    uo[m] = __builtin_amdgcn_readfirstlane((int)uoi[m]);
  }
  int bpre = 0;
#pragma unroll
  for (int m = 0; m < M - 1; ++m) bpre += abs(lb[m] + ((tid >> (3 * m)) & 7) - uo[m]);
  unsigned valid = 0;  // target inside the trust region: c' + b̃_l(i) <= B
  // targets in the trust region (low 16 bits) + finite sources (high 16 bits) of the wave: ballots counted on the
  // scalar unit
  int nv = 0;
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    const bool in = bpre <= B - cp - abs(lb[M - 1] + x - uo[M - 1]);  // right side wave-uniform
    valid |= (unsigned)in << x;
    nv += __popcll(__ballot(in));
  }
  double pmn = INFINITY, pmx = -INFINITY;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const double x = v[2 * q + hh];  // (sd_strad: +Inf for a straddling second element, written by its loader)
      // written anyway: the straddle lane is in this wave and writes after it (in-wave LDS order)
      const int j = (int)((hh ? ein[q].y : ein[q].x) & 0xFFFFu);
      psi[j] = x;
      dtv[sd_swz(j)] = x;  // raw, stamped by pass 0
      const bool fin = x < INFINITY;
      nv += __popcll(__ballot(fin)) << 16;
      pmn = sd_min(pmn, x);  // +Inf is neutral
      pmx = sd_max(pmx, __hiloint2double(fin ? __double2hiint(x) : (int)0xFFF00000, __double2loint(x)));  // +Inf -> -Inf
    }
  if constexpr (sd_strad<M>()) {  // this lane's straddle element
    const double x = (srank & 0x10000) ? INFINITY : xs;
    const bool fin = srank >= 0 && x < INFINITY;
    nv += __popcll(__ballot(fin)) << 16;
    if (srank >= 0) {
      psi[srank & 0xFFFF] = x;
      dtv[sd_swz(srank & 0xFFFF)] = x;
    }
    pmn = sd_min(pmn, fin ? x : INFINITY);
    pmx = sd_max(pmx, fin ? x : -INFINITY);
  }
  sd_wave_stats(pmn, pmx);
  if (lane == 0) {
    sh.rmn[w] = pmn;
    sh.rmx[w] = pmx;
    sh.rnv[w] = nv;
  }
  return valid;
}

// One source row c' of step i for subproblem k (the row body shared by both drivers), after its statistics phase
// (sdt_stats: Ψ in the LDS, each wave's statistics in sh):
//   valid  : sdt_stats' result for this row (this lane's targets inside the trust region).
//   ein_in : this thread's sphere-order entries of step i+1 at its eight positions (rank | b̃ << 16).
//   pin    : LDS copy of the sphere order of step i+1 (rank | b̃ << 16 by position), pout: of step i.
//   h      : the driver's pipeline hooks (no-ops for one launch per step): h.early() once every wave has consumed its Ψ
//            (publish `loaded`, issue the polls); h.go() after the first barrier (check the polls, issue the next row's
//            loads, the next step's sphere order and df / u_old); h.late_drain() before the barrier after the winners
//            (this wave's stores of the previous row have landed), h.publish() after it (the previous row is done).  A
//            timed-out wait sets sh.stop, which the driver reads after the row; h.tail(empty, outv) once the row's
//            outputs are final, before its stores (the persistent driver runs the next row's sdt_stats there).
//   smask, srank: (sd_strad) the pairs q whose second element straddles a sphere seam (bit 3q+2 of smask: not
//            this lane's to store), and the rank of this lane's straddle element (srank < 0: none)
// Returns 1 if the row is all +Inf (no target in the trust region or no finite source), else 0.
// Writes row c' of S_i (sphere order of u_old(i)) and of UU_i: exactly five 16-byte vector-memory stores per
// thread on every path, the last vector-memory instructions of the row (the persistent driver's counted wait
// for the next row's loads relies on it).  Every barrier is LDS-only (sd_bar): nothing here waits for the
// caller's outstanding loads or stores.
template <int M, bool PERSIST, class Hooks>
__device__ __forceinline__ int sdt_body(const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G, int k, int cp,
                                         int i, unsigned valid, const uint2 (&ein_in)[4], const uint32_t *pin,
                                         const uint32_t *pout,
                                         double *Sout, uint16_t *UU, SdtShared<(1 << (3 * M - 3)) / 64> &sh,
                                         unsigned char *sds, Hooks &h, const double *__restrict__ df_all,
                                         const double *__restrict__ uo_all, int par, unsigned smask = 0,
                                         int srank = -1) {
  constexpr int L = 1 << (3 * M), T = L / 8, NW = T / 64, Smax = 7 * M;
  double *psi = reinterpret_cast<double *>(sds);        // [L] Ψ_j by rank
  double *dtv = psi + L;                                // [L] transform values (swizzled)
  uint16_t *uu = reinterpret_cast<uint16_t *>(dtv + L);  // [L] the U row (natural order)
  // [L] the outputs (natural order): a buffer of their own, so that the winners of one wave need not wait for every
  // other wave's last pass
  double *outv = reinterpret_cast<double *>(sds + sd_out_offset<M>());
  uint16_t *list = uu + L;                              // [SD_LCAP] targets for the exact scan
  const int tid = sd_tid(), lane = tid & 63;
  const double beta = Lv.beta;
  // df / u_old of this step: the persistent driver has copied them into this wave's LDS words (LDS-DMA issued one
  // row ahead: a global load here would cost a memory round trip per row); the per-step driver reads them directly
  const double *dfi = PERSIST ? reinterpret_cast<const double *>(sds + sd_dfuo_offset<M>()) + (2 * M + 2) * (threadIdx.x >> 6)
                              : df_all + ((size_t)k * P.nt + i) * M;
  (void)uo_all;
  SD_RSTAMP(13);
  SD_STAMP(0);
  // this thread's sphere-order entries (rank | b̃ << 16 at its eight positions of step i+1): read by the caller (the
  // persistent driver kept them from issuing this row's loads, so no LDS round trip starts the row)
  uint2 ein[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) ein[q] = ein_in[q];
  // ---- this thread's targets: ranks tid | x << 3(M-1) (the lines of the last pass) -----------------
  double a[M];
  int lb[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    a[m] = P.dt * dfi[m];
    lb[m] = G.base[m];
  }
  double pre = 0.0;
#pragma unroll
  for (int m = 0; m < M - 1; ++m) {
    const int nu = lb[m] + ((tid >> (3 * m)) & 7);
    pre = pre + a[m] * (double)nu;  // ((0 + (Δt·df_1)·ν_1) + ...), HelpFunctions.jl:52-57
  }

  // ---- the binade: values base + (Ψ - ref)/β + d lie in [base, 2·base), grid g = 2^18 ulp ----------------
  // for Ψ in [lo, hi] (ref = lo): every quantity of the certified transform follows from the range alone
  const double inv = Lv.inv_beta;  // fl(1/β), host-computed
  double qa = beta * (double)Smax;  // |T1 + β·d + Ψ| <= qa + max(|lo|, |hi|) for every candidate
#pragma unroll
  for (int m = 0; m < M; ++m) qa += fabs(a[m]) * (double)max(abs(lb[m]), abs(lb[m] + 7));
  double ref, base, g, tol;
  bool scale_ok;
  auto scale = [&](double lo, double hi) {
    const double rs = (hi - lo) * inv + (double)Smax;              // scaled range of every transform value
    scale_ok = rs < 0x1p31;                                        // else unit steps are not on the grid: exact scans
    const int E = ilogb(fmin(rs, 0x1p31) * (1.0 + 0x1p-20) + 1.0) + 2;  // 2^E >= 2·rs (E <= SD_GRID: g <= 1)
    base = ldexp(1.0, E);
    g = ldexp(1.0, E - SD_GRID);
    // 2 × stamping error (< g) + 2 × the reference's rounding (<= 4u·qmax per candidate), in units of β
    tol = 3.0 * g + 0x1p-49 * (qa + fmax(fabs(lo), fabs(hi))) * inv;
    ref = lo;
  };
  // V_j = trunc_g(base + (Ψ_j - ref)/β) | j
  auto stamp = [&](double x, int j) {
    const double y = (x - ref) * inv + base;
    return __hiloint2double(__double2hiint(y), (__double2loint(y) & ~SD_PAY) | (j << SD_CB));
  };
  // the stamp, +Inf kept +Inf, without a branch
  auto stamp_inf = [&](double x, int j) {
    const double y = stamp(x, j);
    const unsigned m = x < INFINITY ? ~0u : 0u;
    return __hiloint2double((int)(((unsigned)__double2hiint(y) & m) | (0x7FF00000u & ~m)),
                            (int)((unsigned)__double2loint(y) & m));
  };
  // ---- one pass of the transform: forward and backward sweep along the 8 levels of dimension m, unit step 1.0;
  // this thread's line is read from and (but for the last pass) written back to the swizzled LDS values ---------
  double o[8];
  // the smallest |a - b| over every merge of the row's first transform (per lane): a near tie anywhere (<= tol) sends
  // the whole row through the counting transform again (below); +Inf - +Inf is NaN, which v_min_f64 ignores
  double dmin = INFINITY;
  // COUNT = false: each merge is add, min, and the |a - b| folded into dmin off the value chain (the first transform);
  // COUNT = true: the certified merge with the near-tie count in the payload (sd_merge), pass 0 reading the raw Ψ by
  // rank (the redo: dtv holds the first transform's values by then)
  auto pass = [&](int m, auto count_tag) {
    constexpr bool COUNT = decltype(count_tag)::value;
    int pos[8];
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      pos[x] = sd_swz(sd_rank((int)threadIdx.x, m, x));  // tid-only: hoisted out of the row loop
      o[x] = (COUNT && m == 0) ? psi[sd_rank((int)threadIdx.x, 0, x)] : dtv[pos[x]];
    }
    if (m == 0) {  // the raw Ψ of ranks 8·tid + x (written with Ψ by rank): stamp them here
#pragma unroll
      for (int x = 0; x < 8; ++x) o[x] = stamp_inf(o[x], sd_rank((int)threadIdx.x, 0, x));
    }
    // in place: after the forward sweep o[x] covers the sources at <= x; a backward merge of o[x] with
    // o[x+1] + 1 compares a source at <= x with itself shifted by >= 2, never within tol, so every
    // flagged tie is between two distinct sources (as in a merge of disjoint sets)
    auto merge = [&](double a, double b) {
      if constexpr (COUNT) {
        return sd_merge(a, b, tol);
      } else {
        dmin = sd_min_abs(dmin, a - b);
        return sd_min(a, b);
      }
    };
#pragma unroll
    for (int x = 1; x < 8; ++x) o[x] = merge(o[x], o[x - 1] + 1.0);
#pragma unroll
    for (int x = 6; x >= 0; --x) o[x] = merge(o[x], o[x + 1] + 1.0);
    if (m + 1 < M) {
#pragma unroll
      for (int x = 0; x < 8; ++x) dtv[pos[x]] = o[x];
    }
  };
  auto passes = [&](auto count_tag) {
    // the lines of passes 0 .. M-2 keep the top grid coordinate (rank bits 3(M-1)..), which is the wave index (the
    // swizzle leaves those bits alone), so a wave reads only what it wrote itself; only the last pass, which runs
    // along the top coordinate, needs every wave's values
#pragma unroll
    for (int m = 0; m < M; ++m) {
      pass(m, count_tag);
      if (m + 2 < M)
        sd_wave_sync();
      else if (m + 1 < M)
        sd_bar();
      SD_STAMP(3 + m);
    }
  };
  // the certified winners of the transform in o[] (FLAG: the counting transform, near ties listed for the exact scan)
  auto winners = [&](auto flag_tag) {
    constexpr bool FLAG = decltype(flag_tag)::value;
    unsigned listed = 0;
    int jx[8];
    double pv[8];
#pragma unroll
    for (int x = 0; x < 8; ++x) jx[x] = (__double2loint(o[x]) >> SD_CB) & ((1 << SD_RB) - 1);  // +Inf: payload 0
#pragma unroll
    for (int x = 0; x < 8; ++x) pv[x] = psi[jx[x]];  // branch-free: the eight winners' Ψ reads issue together
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      const int r = tid | (x << (3 * (M - 1))), j = jx[x];
      const bool fin = (valid >> x & 1) && o[x] < INFINITY;
      const bool flg = FLAG && (__double2loint(o[x]) & SD_CNT) != 0;
      // d(l, j*) exactly: an unflagged finite o[x] is V_j* + d with V_j* = the stamp of Ψ_j* (the same expression
      // as the stamping above, payload j*), every term exact in the binade (garbage, unused, otherwise)
      const double dd = o[x] - stamp(pv[x], j);
      const double t1 = pre + a[M - 1] * (double)(lb[M - 1] + x);
      const double val = (t1 + beta * dd) + pv[x];  // R(l, j*), HelpFunctions.jl:63-71
      if constexpr (FLAG) {
        listed |= (unsigned)(fin && flg) << x;
        uu[r] = (uint16_t)(fin && !flg ? j : 0xFFFF);  // 0xFFFF: unwritten (Φ = +Inf) or not yet known (listed)
        outv[r] = fin ? (flg ? __longlong_as_double(0x7FF8000000000000ll) : val) : INFINITY;
      } else {
        uu[r] = (uint16_t)(fin ? j : 0xFFFF);  // 0xFFFF: unwritten (Φ = +Inf)
        outv[r] = fin ? val : INFINITY;
      }
    }
    return listed;
  };
  auto list_targets = [&](unsigned listed) {
    if (listed) {
      int e = atomicAdd(&sh.nlist[par], __popc(listed));
#pragma unroll
      for (int x = 0; x < 8; ++x)
        if (listed >> x & 1) {
          if (e < SD_LCAP) list[e] = (uint16_t)(tid | (x << (3 * (M - 1))));
          ++e;
        }
    }
  };
  int nf, nv;
  bool empty;
  {
    double pmn, pmx;
    sd_bar();  // every wave's row statistics (sdt_stats) are in sh, its Ψ in the LDS: the loads of S_{i+1} are consumed
    if (tid == 0) sh.nlist[par ^ 1] = sh.redo[par ^ 1] = 0;  // the next row's slots
    h.early();
    {
      // every wave's statistics in one batch of LDS reads and one wait (the compiler interleaved them with the
      // reduction: six dependent LDS round trips), then a tree
      double mn[NW], mx[NW];
      int cn[NW];
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        mn[q] = sh.rmn[q];
        mx[q] = sh.rmx[q];
        cn[q] = sh.rnv[q];
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int h = NW / 2; h >= 1; h >>= 1)
#pragma unroll
        for (int q = 0; q < h; ++q) {
          mn[q] = sd_min(mn[q], mn[q + h]);
          mx[q] = sd_max(mx[q], mx[q + h]);
          cn[q] += cn[q + h];
        }
      pmn = mn[0];
      pmx = mx[0];
      nv = cn[0];
    }
    nf = nv >> 16;
    nv &= 0xFFFF;
    SD_STAMP(1);
    // no target in the trust region, or nothing reachable: the row is +Inf and U unwritten (0xFFFF)
    empty = __builtin_amdgcn_readfirstlane((int)(nv == 0 || !(pmn < INFINITY))) != 0;  // uniform
    scale(pmn, pmx);
  }
  // few finite sources (rows near c' = 0): every target's minimum over them, directly
  const bool sparse = !empty && nf <= SD_SPARSE;
  const bool direct = !empty && !sparse && (nv <= SD_FEW || !scale_ok || !(tol < base * 0x1p-20));

  int spj[SD_SPARSE];
  double spv[SD_SPARSE];
  if (sparse) {
    if (tid == 0) sh.nsp = 0;
    sd_bar();
    // this lane's finite sources, from Ψ by rank (sd_strad: a straddling second element is its straddle lane's to add;
    // otherwise this lane loaded it itself)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int j = (int)((hh ? ein[q].y : ein[q].x) & 0xFFFFu);
        const double x = psi[j];
        if (x < INFINITY && !(sd_strad<M>() && hh && (smask >> (3 * q + 2) & 1))) {
          const int e = atomicAdd(&sh.nsp, 1);
          sh.spj[e] = j;
          sh.spv[e] = x;
        }
      }
    if (sd_strad<M>() && srank >= 0 && !(srank & 0x10000) && psi[srank & 0xFFFF] < INFINITY) {
      const int e = atomicAdd(&sh.nsp, 1);
      sh.spj[e] = srank & 0xFFFF;
      sh.spv[e] = psi[srank & 0xFFFF];
    }
    sd_bar();
#pragma unroll
    for (int e = 0; e < SD_SPARSE; ++e) {  // uniform: broadcast reads into registers
      spj[e] = sh.spj[e];
      spv[e] = sh.spv[e];
    }
  }
  const bool transform = !direct && !empty && !sparse;  // uniform
  // no stamp phase (pass 0 stamps): every wave is past its last read of `pin` (the first barrier)
  h.go();
  if (transform) passes(std::false_type{});  // the M passes, near ties folded into dmin

  if (!empty) {
    // ---- targets: R(l, j*) for a certified winner (no merge of the row's transform came within tol: every winner beats
    // every other source by more than tol); a row that met a near tie anywhere is redone below, counting them
    unsigned listed = 0;
    if (!direct && !sparse) {
      winners(std::false_type{});
      if (__any(dmin <= tol) && lane == 0) sh.redo[par] = 1;
    } else {
#pragma unroll
      for (int x = 0; x < 8; ++x) {
        const int r = tid | (x << (3 * (M - 1)));
        double ov = INFINITY;
        int uj = 0xFFFF;  // U cell not written by the reference (Φ = +Inf) or not yet known (listed)
        if (direct) {
          listed |= valid & (1u << x);
        } else {  // sparse: the reference loop over the finite sources, ties to the lower rank
          if (valid >> x & 1) {
            const double t1 = pre + a[M - 1] * (double)(lb[M - 1] + x);
            double bv = INFINITY;
            int bj = 0xFFFF;
#pragma unroll
            for (int e = 0; e < SD_SPARSE; ++e) {
              if (e < nf) {
                const int j = spj[e];
                const unsigned d = sd_l1(sd_bytes(j), sd_bytes((unsigned)tid) | (unsigned)x << (8 * (M - 1)));
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
        outv[r] = (listed >> x & 1) ? __longlong_as_double(0x7FF8000000000000ll) : ov;
      }
    }
    list_targets(listed);
    h.late_drain();  // this wave's stores of the previous row have landed (late: they have had the whole row)
    sd_bar();
    h.publish();     // ... so have every wave's: the previous row is done
    SD_STAMP(7);
    if (transform && sh.redo[par]) {  // uniform, rare: a near tie somewhere in the row -- the certified transform
      passes(std::true_type{});
      list_targets(winners(std::true_type{}));
      sd_bar();
      if (tid == 0) ++sh.cnt[3];
    }
    const int nl = sh.nlist[par];
    if (nl) {
      if (nl <= SD_COOP)
        sd_scan<M, true>(list, nl, psi, a, lb, beta, uu, outv, sh.redv, sh.redj);
      else if (nl <= SD_LCAP)
        sd_scan<M, false>(list, nl, psi, a, lb, beta, uu, outv, sh.redv, sh.redj);
      else
        sd_scan<M, false>(nullptr, L, psi, a, lb, beta, uu, outv, sh.redv, sh.redj);  // every NaN-marked rank
      sd_bar();
      if (tid == 0) sh.cnt[direct ? 1 : 0] += nl;
    }
  }
  if (empty) {  // uniform: the row is +Inf, U unwritten -- through LDS, so that the stores below take one path
#pragma unroll
    for (int x = 0; x < 8; ++x) outv[tid | (x << (3 * (M - 1)))] = INFINITY;
    reinterpret_cast<ulonglong2 *>(uu)[tid] = make_ulonglong2(~0ull, ~0ull);
    h.late_drain();
    sd_bar();
    h.publish();
  }
  SD_STAMP(8);
  // ---- Φ_i row c' in the sphere order of u_old(i), and the U row, both 16 bytes per lane: gathered from the LDS
  // before the tail, so that the two dependent LDS round trips (order entries, then values) run under its VALU work
  uint2 eo[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) eo[q] = *reinterpret_cast<const uint2 *>(pout + sd_p2<M>(tid, q));
  double go[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    go[2 * q] = outv[eo[q].x & 0xFFFFu];
    go[2 * q + 1] = outv[eo[q].y & 0xFFFFu];
  }
  const ulonglong2 ut = reinterpret_cast<const ulonglong2 *>(uu)[tid];
  // the persistent driver's next row: its statistics phase (LDS writes and VALU only), with this row's outputs final
  h.tail(empty, outv);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    sd_store16<PERSIST>(Sout, L * 8, sd_p2<M>(tid, q), __double_as_longlong(go[2 * q]),
                        __double_as_longlong(go[2 * q + 1]));
  *reinterpret_cast<ulonglong2 *>(UU + 8 * tid) = ut;  // read by later launches only (backtrack)
  SD_STAMP(9);
  SD_RSTAMP(14);
  return empty ? 1 : 0;
}

// Ψ of row c' at step i: S_{i+1}[c' - b̃_j(i+1)][pos] for this thread's eight positions (sphere order `pin` of step
// i+1, in LDS), +Inf where that row is below 0.  Row 0 comes from `r0` (the persistent driver keeps row 0 of every
// step in its own array, written before the launch) or, when r0 is null, from the staging block itself.
// SC1: the persistent driver's hand-off loads (`sc1` buffer loads to registers, MI355X_MICROARCH.md Valid forms).
template <int M, bool SC1>
__device__ __forceinline__ void sd_issue_loads(double (&v)[8], const uint32_t *pin, int cp, const double *Sin,
                                               int sbytes, const double *r0) {
  constexpr int L = 1 << (3 * M);
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p2 = sd_p2<M>(tid, q);
    const uint2 e = *reinterpret_cast<const uint2 *>(pin + p2);
    const int ra = cp - (int)(e.x >> 16), rb = cp - (int)(e.y >> 16);
    double va = INFINITY, vb = INFINITY;
    if (ra == rb && (ra >= 1 || (ra == 0 && !r0))) {  // one 16-byte load (the common case)
      sd_load_pair<SC1>(Sin, sbytes, ra * L + p2, ra * L + p2 + 1, va, vb);
    } else {
      if (ra >= 1 || (ra == 0 && !r0))
        va = sd_load8<SC1>(Sin, sbytes, ra * L + p2);
      else if (ra == 0)
        va = r0[p2];
      if (rb >= 1 || (rb == 0 && !r0))
        vb = sd_load8<SC1>(Sin, sbytes, rb * L + p2 + 1);
      else if (rb == 0)
        vb = r0[p2 + 1];
    }
    v[2 * q] = va;
    v[2 * q + 1] = vb;
  }
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
  constexpr int L = 1 << (3 * M);
  const int tid = threadIdx.x, B = P.B;
  const double beta = Lv.beta;
  const double *Sin = Sin_all + (size_t)k * s_stride;
  double *S0 = Sout_all + (size_t)k * s_stride;
  uint16_t *U0 = UU_all + (size_t)k * uu_stride_k + (size_t)i * ((size_t)(B + 1) * L);
  const double psi0 = sd_load8<PERSIST>(Sin, (B + 1) * L * (int)sizeof(double), pm.pin_h);  // Φ_{i+1}[j0, 0]
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
    sd_store16<PERSIST>(S0, L * 8, sd_p2<M>(tid, q), __double_as_longlong(o[0]), __double_as_longlong(o[1]));
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
    const int p2 = sd_p2<M>(tid, q);
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
    const bool p0 = wb && sd_p2<M>(tid, q) == pm.pout_h;  // only the head position (= l0) can be finite
    sd_store16<PERSIST>(SB, L * 8, sd_p2<M>(tid, q), p0 ? __double_as_longlong(bv) : 0x7FF0000000000000ull,
                        0x7FF0000000000000ull);
  }
  unsigned short ub[8];
#pragma unroll
  for (int x = 0; x < 8; ++x) ub[x] = wb && 8 * tid + x == r0 ? (unsigned short)bj : (unsigned short)0xFFFF;
  *reinterpret_cast<ulonglong2 *>(UB + 8 * tid) = make_ulonglong2(sd_pack4(ub), sd_pack4(ub + 4));
}

// per-step driver: no pipeline hooks
struct SdHooksNone {
  __device__ __forceinline__ void early() {}
  __device__ __forceinline__ void go() {}
  __device__ __forceinline__ void late_drain() {}
  __device__ __forceinline__ void publish() {}
  __device__ __forceinline__ void tail(bool, const double *) {}
};

// LDS bytes of the row body: Ψ by rank, the transform / output values, the U row, the scan list, and two
// sphere-order slots (steps i+1 and i)
size_t sdt_lds_bytes(const PyrGeom &G) { return G.M == 4 ? sd_lds_total<4>() : sd_lds_total<3>(); }

// copy one step's sphere order (L uint32) into an LDS slot with LDS-DMA (1 KiB per wave-instruction, no VGPRs);
// lands asynchronously (vmcnt), visible to the other waves after their wait and a barrier
template <int M>
__device__ __forceinline__ void sd_perm_dma(const uint32_t *src, uint32_t *slot) {
  constexpr int L = 1 << (3 * M), T = L / 8, NW = T / 64;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int c = wave; c < L * 4 / 1024; c += NW)
    __builtin_amdgcn_global_load_lds(
        (const __attribute__((address_space(1))) void *)((const char *)src + c * 1024 + lane * 16),
        (__attribute__((address_space(3))) void *)((char *)slot + c * 1024), 16, 0, 0);
}

// The same copy for the persistent driver, as inline asm: the compiler then does not know these instructions
// write LDS, and does not make every later LDS atomic wait (vmcnt(0)) for them -- and for the row loads queued
// behind.  The driver orders them itself: they are issued before the next row's loads and complete under the
// counted wait at that row's start, and every reader of the slot reads it after a later vmcnt(0) and a barrier.
template <int M>
__device__ __forceinline__ void sd_perm_dma_asm(const uint32_t *src, uint32_t *slot) {
  constexpr int L = 1 << (3 * M), T = L / 8, NW = T / 64, NC = L * 4 / 1024;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char *)slot);
#pragma unroll
  for (int c = wave; c < NC; c += NW) {
    const char *g = (const char *)src + c * 1024 + lane * 16;
    const unsigned m0 = __builtin_amdgcn_readfirstlane(lds0 + (unsigned)c * 1024u);
    unsigned keep;  // M0 is reserved to the compiler: saved and restored around the copy
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(m0)
                 : "memory");
  }
}

// df(:, s) and u_old(:, s) (M doubles each) into this wave's LDS words, and the flag same2[s - 1] (u_old(s-1) ==
// u_old(s+1): the sphere order of step s-1 equals the one its slot holds, k_pyr_order) after them: lanes 0..4M move
// one dword each (global_load_lds_dword, LDS-DMA, inline asm for the same reason as sd_perm_dma_asm)
template <int M>
__device__ __forceinline__ void sd_dfuo_dma(const double *df, const double *uo, const int32_t *flag, unsigned char *sds) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane < 4 * M + (flag ? 1 : 0)) {
    const char *g = lane < 2 * M   ? (const char *)df + 4 * lane
                    : lane < 4 * M ? (const char *)uo + 4 * (lane - 2 * M)
                                   : (const char *)flag;
    const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char *)(sds + sd_dfuo_offset<M>())) +
                          wave * (unsigned)sd_dfuo_stride<M>();
    const unsigned m0 = __builtin_amdgcn_readfirstlane(lds0);
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(m0)
                 : "memory");
  }
}

// (sd_strad) this wave's slab of a step's seam list (SD_STRAD_N uint16 = 64 bytes) into the slot's list in LDS:
// lanes 0..15 move one dword each (LDS-DMA, inline asm as sd_perm_dma_asm); only this wave reads its slab's list
__device__ __forceinline__ void sd_strad_dma(const uint16_t *src, uint16_t *slot) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane < SD_STRAD_N / 2) {
    const char *g = (const char *)(src + wave * SD_STRAD_N) + 4 * lane;
    const unsigned m0 = __builtin_amdgcn_readfirstlane(
        (unsigned)(uintptr_t)((__attribute__((address_space(3))) char *)(slot + wave * SD_STRAD_N)));
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(m0)
                 : "memory");
  }
}

// One launch per step: one workgroup per (source row c', subproblem k).
template <int M>
__global__ __launch_bounds__(1 << (3 * M - 3)) void k_sdt_step(ProblemDev P, LevelsDev Lv, PyrGeom G, int i,
                                                           const uint32_t *__restrict__ perm_all,
                                                           const double *__restrict__ Sin_all,
                                                           double *__restrict__ Sout_all,
                                                           uint16_t *__restrict__ UU_all, size_t s_stride,
                                                           size_t uu_stride_k, int32_t *__restrict__ counters) {
  constexpr int L = 1 << (3 * M);
  extern __shared__ __attribute__((aligned(16))) unsigned char sds[];
  __shared__ SdtShared<(1 << (3 * M - 3)) / 64> sh;
  const int k = (int)blockIdx.y, tid = threadIdx.x;
  if (tid == 0) {
    sh.cnt[0] = sh.cnt[1] = sh.cnt[3] = 0;
    sh.nlist[0] = sh.redo[0] = 0;
  }
  // B >= 1: block 0 takes rows 0 and B together, block x the row x (B workgroups, one per CU at B = 256)
  if (blockIdx.x == 0 && P.B >= 1) {
    SdPerm pm;
    sd_perm_load<M>(pm, perm_all, P, G, k, i);
    sdt_row0<M, false>(P, Lv, k, i, pm, Sin_all, Sout_all, UU_all, s_stride, uu_stride_k, G.base, nullptr, 0);
    sdt_rowB<M, false>(P, Lv, k, i, pm, Sin_all, Sout_all, UU_all, s_stride, uu_stride_k, G.base, counters, sh,
                       nullptr, 0);
  } else {
    const int cp = (int)blockIdx.x;
    uint32_t *slot = reinterpret_cast<uint32_t *>(sds + sd_slot_offset<M>());
    sd_perm_dma<M>(perm_all + ((size_t)k * P.nt + i + 1) * L, slot);
    sd_perm_dma<M>(perm_all + ((size_t)k * P.nt + i) * L, slot + L);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sd_bar();
    double v[8];
    sd_issue_loads<M, false>(v, slot, cp, Sin_all + (size_t)k * s_stride, (P.B + 1) * L * (int)sizeof(double),
                             nullptr);
    SdHooksNone hooks;
    uint2 ein[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) ein[q] = *reinterpret_cast<const uint2 *>(slot + sd_p2<M>(tid, q));
    const unsigned valid = sdt_stats<M, false>(P, G, k, cp, i, v, ein, sh, sds, P.df, P.uold);
    sdt_body<M, false>(P, Lv, G, k, cp, i, valid, ein, slot, slot + L, Sout_all + (size_t)k * s_stride + (size_t)cp * L,
                       UU_all + (size_t)k * uu_stride_k + (size_t)i * ((size_t)(P.B + 1) * L) + (size_t)cp * L, sh,
                       sds, hooks, P.df, P.uold, 0);
    if (tid == 0) {
      if (sh.cnt[0]) atomicAdd(&counters[0], sh.cnt[0]);
      if (sh.cnt[1]) atomicAdd(&counters[1], sh.cnt[1]);
      if (sh.cnt[3]) atomicAdd(&counters[5], sh.cnt[3]);
    }
  }
  SD_FLUSH();
}

// ---- the persistent driver's row 0 ---------------------------------------------------------------------------
// Row 0 of every step has at most one finite source, j0(i+1) = the level at L1 distance 0 from u_old(i+1), so
//   S_i[0][pos_i(l)] = Φ_i[l, b̃_l(i)] = fl(fl(T1(l, i) + β·d(l, j0(i+1))) + V(i+1))   (+Inf where b̃_l(i) > B),
//   V(i) = S_i[0][0] = Φ_i[j0(i), 0], V(nt-1) = T1(j0(nt-1), nt-1), U_i[l, b̃_l(i)] = j0(i+1),
// with V(i) = +Inf where u_old(i) is off the level grid (no level at distance 0),
// (HelpFunctions.jl:29-43, 45-77 restricted to budget row 0).  V is a scalar chain in time: k_sdt_chain folds it
// once (its additions in the reference's order), k_sdt_row0 expands every step's row 0 into R0[k][i][pos] and its
// U row, and the persistent kernel's rows 1..28 read row 0 from there instead of waiting for a workgroup.
template <int M>
__global__ __launch_bounds__(256) void k_sdt_chain(ProblemDev P, PyrGeom G, double beta,
                                                  const uint32_t *__restrict__ perm_all, double *__restrict__ V) {
  constexpr int L = 1 << (3 * M), CH = 2048;
  __shared__ double av[CH];
  const int k = (int)blockIdx.x, tid = threadIdx.x, nt = P.nt;
  const uint32_t *pk = perm_all + (size_t)k * nt * L;
  double *Vk = V + (size_t)k * nt;
  // the head of step i's sphere order (the level at distance 0 from u_old(i), if u_old(i) is on the grid)
  auto head = [&](int i) { return pk[(size_t)i * L + kSdHeadPos]; };
  auto j0 = [&](int i) { return (int)(head(i) & 0xFFFFu); };
  // Φ_i[j0(i), 0] exists only where u_old(i) is a level (the head at distance 0); an off-grid u_old(i) leaves
  // budget row 0 empty at step i, and then at every earlier step (+Inf propagates through the additions)
  auto on_grid = [&](int i) { return (head(i) >> 16) == 0u; };
  auto t1 = [&](int r, int i) {  // ((0 + (Δt·df_1)·ν_1) + ...), HelpFunctions.jl:52-57
    const double *dfi = P.df + ((size_t)k * nt + i) * M;
    double t = 0.0;
#pragma unroll
    for (int m = 0; m < M; ++m) t = t + (P.dt * dfi[m]) * (double)(G.base[m] + ((r >> (3 * m)) & 7));
    return t;
  };
  double run = on_grid(nt - 1) ? t1(j0(nt - 1), nt - 1) : INFINITY;  // the terminal row (no switching term)
  if (tid == 0) Vk[nt - 1] = run;
  for (int hi = nt - 2; hi >= 0; hi -= CH) {  // steps hi, hi-1, ..., lo
    const int lo = max(0, hi - CH + 1), n = hi - lo + 1;
    for (int q = tid; q < n; q += blockDim.x) {
      const int i = hi - q, r = j0(i);
      const unsigned d = sd_l1(sd_bytes((unsigned)r), sd_bytes((unsigned)j0(i + 1)));
      av[q] = on_grid(i) ? t1(r, i) + beta * (double)d : INFINITY;  // temp_val_2, HelpFunctions.jl:67
    }
    __syncthreads();
    if (tid == 0) {
      int q = 0;
      for (; q + 8 <= n; q += 8) {
        double x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = av[q + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          run = x[u] + run;  // val = temp_val_2 + Φ_{i+1}, HelpFunctions.jl:71
          av[q + u] = run;
        }
      }
      for (; q < n; ++q) {
        run = av[q] + run;
        av[q] = run;
      }
    }
    __syncthreads();
    for (int q = tid; q < n; q += blockDim.x) Vk[hi - q] = av[q];
    __syncthreads();
  }
}

template <int M>
__global__ __launch_bounds__(1 << (3 * M - 3)) void k_sdt_row0(ProblemDev P, LevelsDev Lv, PyrGeom G,
                                                            const uint32_t *__restrict__ perm_all,
                                                            const double *__restrict__ V, double *__restrict__ S_all,
                                                            size_t kstride, size_t r0off, uint16_t *__restrict__ UU_all,
                                                            size_t uu_stride_k) {
  constexpr int L = 1 << (3 * M);
  const int i = (int)blockIdx.x, k = (int)blockIdx.y, tid = threadIdx.x, nt = P.nt, B = P.B;
  const uint32_t *pi = perm_all + ((size_t)k * nt + i) * L;
  const bool term = i == nt - 1;
  const int jn = term ? 0
                      : (int)(perm_all[((size_t)k * nt + i + 1) * L +
                                       kSdHeadPos] &
                              0xFFFFu);  // j0(i+1)
  const double vn = term ? 0.0 : V[(size_t)k * nt + i + 1];
  const SdEdge<M> E(P, G.base, k, i);
  double *reg = S_all + (size_t)k * kstride;
  double *r0 = reg + r0off + (size_t)i * L;
  auto val = [&](int r) {
    const double t = E.t1(r);
    return term ? t : (t + Lv.beta * (double)SdEdge<M>::dist(r, jn)) + vn;
  };
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint2 e = *reinterpret_cast<const uint2 *>(pi + sd_p2<M>(tid, q));
    const double o0 = (int)(e.x >> 16) > B ? INFINITY : val((int)(e.x & 0xFFFFu));
    const double o1 = (int)(e.y >> 16) > B ? INFINITY : val((int)(e.y & 0xFFFFu));
    *reinterpret_cast<double2 *>(r0 + sd_p2<M>(tid, q)) = make_double2(o0, o1);
    if (i == 0) *reinterpret_cast<double2 *>(reg + sd_p2<M>(tid, q)) = make_double2(o0, o1);  // S_0 row 0 (buffer 0)
  }
  if (!term) {  // U row 0 of step i, natural order: ranks 8·tid .. 8·tid + 7 (written where Φ_i is finite)
    unsigned short u0[8];
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      const int r = 8 * tid + x;
      u0[x] = E.bt(r) <= B && val(r) < INFINITY ? (unsigned short)jn : (unsigned short)0xFFFF;
    }
    uint16_t *U0 = UU_all + (size_t)k * uu_stride_k + (size_t)i * ((size_t)(B + 1) * L);
    *reinterpret_cast<ulonglong2 *>(U0 + 8 * tid) = make_ulonglong2(sd_pack4(u0), sd_pack4(u0 + 4));
  }
}

// The persistent driver's hand-off loads, branch-free (a divergent load makes the compiler wait for it before
// the branches join): per position pair one 16-byte `sc1` load at the row of its first element; at M = 4 (sd_strad)
// the second elements of the pairs that straddle a sphere seam come with one straddle load per lane (the wave's seam
// list), else one 8-byte `sc1` load per pair at the row of its second element where the pair straddles; all through
// ONE buffer resource spanning the subproblem's staging buffers and its row-0 array; out-of-range offsets (dropped by
// the hardware) where a row is below 0 or no second load is needed.  `sd_take` selects once the data is in (at the
// next row's start).
struct SdRaw {
  sd_u32x4 a[4];
  sd_u32x2 b[4];  // (not sd_strad) the second elements of straddling pairs
  sd_u32x2 sv;    // (sd_strad) this lane's straddle element, at position sp of its wave: rank srank
  int srank;      // -1: no straddle element for this lane; bit 16: its source row is below 0 (+Inf)
  uint2 e[4];     // the sphere-order entries the offsets came from (the row body's `ein`)
  unsigned mask;  // per pair q: bit 3q the first element has no source row, 3q+1 the second, 3q+2 it straddles
};
// the LDS side of a row's loads: this thread's sphere-order entries of the slot `pin` and (sd_strad) its seam, from
// the slot's seam list `sl` (SD_STRAD_N in-wave offsets per wave, 0xFFFF: none)
struct SdNext {
  uint2 e[4];
  unsigned sp;  // (sd_strad) in-wave offset of this lane's seam (0xFFFF: none)
  uint32_t se;  // its sphere-order entry
};
template <int M>
__device__ __forceinline__ void sd_read_next(SdNext &n, const uint32_t *pin, const uint16_t *sl) {
  constexpr int L = 1 << (3 * M), T = L / 8, NW = T / 64;
  const int tid = threadIdx.x;
#pragma unroll
  for (int q = 0; q < 4; ++q) n.e[q] = *reinterpret_cast<const uint2 *>(pin + sd_p2<M>(tid, q));
  // sd_strad: lane l < SD_STRAD_N of wave w takes the l-th seam of the wave's positions (its rank and distance)
  n.sp = 0xFFFFu;
  n.se = 0;
  if constexpr (sd_strad<M>()) {
    const int lane = tid & 63, wv = tid >> 6;
    n.sp = lane < SD_STRAD_N ? sl[wv * SD_STRAD_N + lane] : 0xFFFFu;
    n.se = pin[sd_seam_pos<M>(wv, (int)(n.sp & (L / NW - 1)))];
  }
}
template <int M>
__device__ __forceinline__ void sd_issue_pipe(SdRaw &w, __amdgpu_buffer_rsrc_t rs, const SdNext &n, int cp,
                                              unsigned boff, unsigned r0, const unsigned rowb) {
  constexpr int L = 1 << (3 * M), T = L / 8, NW = T / 64;
  const int tid = threadIdx.x;
  uint2 e[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) e[q] = n.e[q];
  const unsigned sp = n.sp;
  const uint32_t se = n.se;
  (void)se;
#pragma unroll
  for (int q = 0; q < 4; ++q) w.e[q] = e[q];
  // an offset beyond the resource's range drops the access (the load returns 0 without touching memory): rows
  // below 0, and the second element wherever the pair does not straddle (it came with the first)
  constexpr unsigned OOB = 0xFFFFFFF0u;
  unsigned oa[4], ob[4], mask = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p2 = sd_p2<M>(tid, q);
    const int ra = cp - (int)(e[q].x >> 16), rb = cp - (int)(e[q].y >> 16);
    oa[q] = ra >= 1 ? boff + (unsigned)ra * rowb + (unsigned)p2 * 8u : ra == 0 ? r0 + (unsigned)p2 * 8u : OOB;
    ob[q] = rb == ra ? OOB
            : rb >= 1 ? boff + (unsigned)rb * rowb + (unsigned)(p2 + 1) * 8u
            : rb == 0 ? r0 + (unsigned)(p2 + 1) * 8u
                      : OOB;
    mask |= ((unsigned)(ra < 0) | (unsigned)(rb < 0) << 1 | (unsigned)(ra != rb) << 2) << (3 * q);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    w.a[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, oa[q], 0, 16);
    if constexpr (!sd_strad<M>()) w.b[q] = __builtin_amdgcn_raw_buffer_load_b64(rs, ob[q], 0, 16);
  }
  if constexpr (sd_strad<M>()) {
    const int P = sd_seam_pos<M>(tid >> 6, (int)(sp & (L / NW - 1)));
    const int rsr = cp - (int)(se >> 16);
    const bool has = sp != 0xFFFFu;
    const unsigned osv =
        !has || rsr < 0 ? OOB : rsr >= 1 ? boff + (unsigned)rsr * rowb + (unsigned)P * 8u : r0 + (unsigned)P * 8u;
    w.sv = __builtin_amdgcn_raw_buffer_load_b64(rs, osv, 0, 16);
    w.srank = has ? (int)(se & 0xFFFFu) | (rsr < 0 ? 0x10000 : 0) : -1;
  }
  w.mask = mask;
}
// this lane's eight values; (sd_strad) the second element of a straddling pair is +Inf here -- its value comes with
// the lane that loaded it as a straddle element, which writes it after this lane (in-wave LDS order)
template <int M>
__device__ __forceinline__ void sd_take(double (&v)[8], const SdRaw &w) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const unsigned m = w.mask >> (3 * q);
    const double a0 = __hiloint2double((int)w.a[q].y, (int)w.a[q].x);
    const double a1 = __hiloint2double((int)w.a[q].w, (int)w.a[q].z);
    v[2 * q] = (m & 1) ? INFINITY : a0;
    if constexpr (sd_strad<M>()) {
      v[2 * q + 1] = (m & 6) ? INFINITY : a1;
    } else {
      const double b1 = __hiloint2double((int)w.b[q].y, (int)w.b[q].x);
      v[2 * q + 1] = (m & 2) ? INFINITY : (m & 4) ? b1 : a1;
    }
  }
}

// ---- the persistent driver --------------------------------------------------------------------------------
// The whole DP in one launch.  Rows 1..B of subproblem k are split into contiguous chunks [lo, hi), one per
// resident workgroup (nwg / K per subproblem, one per CU); row 0 comes from R0 (k_sdt_row0).  A workgroup works
// through its items (row, step) in the order step descending, row ascending, and runs one item ahead:
//   item n:  wait for its Ψ (issued during item n-1) -> reductions, `loaded` published -> stamp, passes
//            -> MID: wait until item n+1's inputs are published (RAW) and nobody still reads what item n overwrites
//               (WAR); issue item n+1's Ψ loads (and the next step's sphere order, LDS-DMA)
//            -> certified winners; drain item n-1's stores, publish item n-1 `done`; exact scans -> item n's stores.
// So the load latency of a row hides behind the second half of the previous row, the store drain behind the
// next row, and the row hand-off latency becomes pipeline skew: a row runs behind the rows below it, which the NB
// staging buffers absorb (step i lives in buffer i % NB).
//
// Flags (relaxed agent-scope atomics, the measured-valid hand-off of MI355X_MICROARCH.md, Valid forms, row 1 of
// its table: sc1 stores drained by every storing wave, then ONE lane's sc1 flag store behind a workgroup barrier;
// one polling wave, sc1 loads of the bytes after the poll matched and a barrier):
//   done[k][r]   = token(i): row r's stores of step i have landed   (token(i) = nt - 1 - i; 0 = nothing yet)
//   loaded[k][r] = token(i): row r's loads of S_{i+1} have returned (its WAR guard)
// Item (r, i) needs done[k][r - s] >= token(i+1) for 1 <= s <= 28, r - s >= 1, outside the chunk, and before
// writing buffer i % NB, loaded[k][r + s] >= token(i + NB - 1) for 1 <= s <= 28, r + s <= B, outside the chunk.
// Every wait points at an item of an earlier step, or of the same step and a lower row, so with every workgroup
// resident nothing deadlocks; a wait beyond spin_limit polls sets *err and every workgroup leaves (the host then
// redoes the DP with per-step launches: check_run).
// The pipeline hooks of the persistent driver (the row body calls them, see sdt_body).
template <int M>
struct SdPipe {
  static constexpr int L = 1 << (3 * M);
  // the current row (cp, step i) and the next one (ncp, step ni)
  int cp, i, ncp, ni;
  bool has_next;
  // constants of the launch
  int lo, hi, B, NB, nt, k, g0;
  unsigned spin_limit, rowb, bufb, r0b;
  int32_t *dk, *lk, *err;
  const uint32_t *pk;
  uint32_t *slot;
  __amdgpu_buffer_rsrc_t rs;
  const double *dfa, *uoa;
  const int32_t *sm;  // same2 (k_pyr_order): u_old(s) == u_old(s + 2) per step s
  const uint16_t *sk;  // (sd_strad) this subproblem's seam lists, [nt][8][SD_STRAD_N]
  uint16_t *sslot;     // (sd_strad) the two slots' seam lists in LDS
  unsigned char *sds;
  SdtShared<(1 << (3 * M - 3)) / 64> *sh;
  // carried from row to row: the previous row (its `done` is published at this row's publish()), this wave's polls,
  // the next row's loads in flight
  int pcp, pi;
  int32_t *fp;
  int need, val;
  SdRaw raw;
  SdNext nx;  // the next row's sphere-order entries and seam (sd_read_next)
  // the next row's statistics phase, run at the end of this row (tail): its result for the next sdt_body
  const ProblemDev *Pp;
  const PyrGeom *Gp;
  unsigned valid_next;
  int whole;  // one row per workgroup (hi - lo == 1)
  unsigned nbo;     // byte offset of the next row's input buffer, (ni + 1) % NB (kept by the driver: no division)
  bool stop_seen;   // sh.stop as read after the row's barrier 3 (publish)

  // every wave polls its own dependency flags (lanes 0-31 RAW for the next row, 32-63 WAR for this row's stores; a
  // lane without one polls a flag that always passes -- every lane loads, no branch), once every wave has consumed
  // this row's loads (early()); checked in go()
  __device__ __forceinline__ void early() {
    SD_TL_AT(g0, i, nt, 1);
    const int tid = threadIdx.x, lane = tid & 63, s = lane < 32 ? lane + 1 : lane - 31;
    fp = lk + cp * SDT_FLAG_STRIDE;
    need = INT32_MIN;
    if (lane < 32) {
      const int r = ncp - s;
      if (has_next && s <= 7 * M && r >= 1 && r < lo && nt - 2 - ni > 0) {
        fp = dk + r * SDT_FLAG_STRIDE;
        need = nt - 2 - ni;  // token(ni + 1)
      }
    } else {
      const int r = cp + s;
      if (s <= 7 * M && r <= B && r >= hi && nt - i - NB > 0) {
        fp = lk + r * SDT_FLAG_STRIDE;
        need = nt - i - NB;  // token(i + NB - 1)
      }
    }
    val = __hip_atomic_load(fp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // diagnostics [4]: this row reuses a staging buffer that a row above may still read (some WAR lane armed above)
    if (tid == 0 && nt - i - NB > 0 && min(cp + 7 * M, B) >= max(cp + 1, hi)) ++sh->cnt[2];
  }
  // after the row's first barrier (every wave has consumed this row's loads): publish `loaded`; this wave waits until
  // its polls match (re-polling), then issues the next row's loads -- the measured-valid consumer form: the polling
  // wave loads only after its own poll matched
  __device__ __forceinline__ void go() {
    SD_TL_AT(g0, i, nt, 2);
    const int tid = threadIdx.x;
    // evaluated before the flag store below: the compiler's wait for `val` would otherwise cover that store
    bool ready = __all(val >= need);
    if (tid == 0) __hip_atomic_store(lk + cp * SDT_FLAG_STRIDE, nt - 1 - i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (!ready) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || ++spins > spin_limit) {
        if ((tid & 63) == 0) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          sh->stop = 1;  // read by the driver after the row's next barrier: the launch is abandoned
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      val = __hip_atomic_load(fp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ready = __all(val >= need);
    }
    SD_TL_AT(g0, i, nt, 3);
    // the next row's loads; then (LDS-DMA, after them so that they do not wait for it) the next step's sphere order
    // into the slot of step i+1 (every wave is past its last read of it: the barrier before go()) and the next row's
    // df / u_old; all of it is older than this row's five stores, so the counted wait at the next row's start covers it
    if (has_next) {
      // the reuse flag of the slot: same2[i-1] = (u_old(i-1) == u_old(i+1)), copied with this step's df / u_old (the
      // slot of step i+1 already holds the order of step ni = i-1 then: the order is a function of u_old alone,
      // k_pyr_order, and by induction every slot holds the order of the last step assigned to it)
      // (an LDS load: through the generic pointer it was a flat load, whose vmcnt(0) wait made wave 0 wait for its own
      // `loaded` flag store above to complete before issuing the next row's loads)
      const int same = *(const volatile __attribute__((address_space(3))) int32_t *)(
          sds + sd_dfuo_offset<M>() + (threadIdx.x >> 6) * sd_dfuo_stride<M>() + 16 * M);
      sd_read_next<M>(nx, slot + ((ni + 1) & 1) * L, sslot + ((ni + 1) & 1) * 8 * SD_STRAD_N);
      sd_issue_pipe<M>(raw, rs, nx, ncp, nbo, r0b + (unsigned)(ni + 1) * rowb, rowb);
      if (ni != i && !same) {
        sd_perm_dma_asm<M>(pk + (size_t)ni * L, slot + (ni & 1) * L);
        if constexpr (sd_strad<M>()) sd_strad_dma(sk + (size_t)ni * 8 * SD_STRAD_N, sslot + (ni & 1) * 8 * SD_STRAD_N);
      }
      sd_dfuo_dma<M>(dfa + ((size_t)k * nt + ni) * M, uoa + ((size_t)k * nt + ni) * M,
                     ni >= 1 ? sm + (size_t)k * nt + ni - 1 : nullptr, sds);
    }
    SD_TL_AT(g0, i, nt, 4);
  }
  // late in the row, before the barrier after the winners: this wave's stores of the previous row have landed (they
  // have had the whole row: no wait), so after that barrier the previous row can be published
  __device__ __forceinline__ void late_drain() {
#ifdef SD_TL_DRAIN  // timeline builds: stamp 7 = the drain's start (instead of "loads taken" at the row start)
    SD_TL_AT(g0, i, nt, 7);
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    SD_TL_AT(g0, i, nt, 5);
  }
  __device__ __forceinline__ void publish() {
    if (threadIdx.x == 0 && pcp >= 0)
      __hip_atomic_store(dk + pcp * SDT_FLAG_STRIDE, nt - 1 - pi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // a timed-out wait of this row (go(), before this barrier) set sh.stop: read here, where every wave reads the same
    // value, so that the driver's exit test after the row needs no LDS round trip of its own
    stop_seen = sh->stop != 0;
    pcp = cp;
    pi = i;
  }
  // the next row's statistics phase (its loads landed at this row's late drain): after this row's outputs are final,
  // before its stores.  A one-row workgroup's next row reads its own row of this step, whose stores are not issued yet:
  // the sphere-0 source at distance 0 (u_old(i) on the level grid: position 0 with b̃ = 0, lane 0 of wave 0) is this
  // row's output, from the LDS (an off-grid u_old has b̃ >= 1 everywhere and no such source).
  __device__ __forceinline__ void tail(bool empty, const double *outv) {
    if (!has_next) return;
    double v[8];
    sd_take<M>(v, raw);
    if (whole && (threadIdx.x & 63) == 0 && (raw.e[0].x >> 16) == 0) v[0] = empty ? INFINITY : outv[raw.e[0].x & 0xFFFFu];
    const double xs = __hiloint2double((int)raw.sv.y, (int)raw.sv.x);
    valid_next = sdt_stats<M, true>(*Pp, *Gp, k, ncp, ni, v, raw.e, *sh, sds, dfa, uoa, raw.srank, xs);
  }
};

template <int M>
__global__ __launch_bounds__(1 << (3 * M - 3), 2) void k_sdt_run(ProblemDev P, LevelsDev Lv, PyrGeom G,
                                                              const uint32_t *__restrict__ perm_all, double *S_all,
                                                              size_t kstride, int NB, uint16_t *__restrict__ UU_all,
                                                              size_t uu_stride_k, int32_t *__restrict__ counters,
                                                              int32_t *flags, int nwg, unsigned spin_limit,
                                                              const double *__restrict__ df_all,
                                                              const double *__restrict__ uo_all,
                                                              const int32_t *__restrict__ same2,
                                                              const uint16_t *__restrict__ strad) {
  constexpr int L = 1 << (3 * M);
  extern __shared__ __attribute__((aligned(16))) unsigned char sds[];
  __shared__ SdtShared<(1 << (3 * M - 3)) / 64> sh;
  const int B = P.B, R = B + 1, nt = P.nt, tid = threadIdx.x;
  // (each flag SDT_FLAG_STRIDE words apart)
  const int FR = R * SDT_FLAG_STRIDE;
  int32_t *done = flags, *loaded = flags + P.K * FR, *err = flags + 2 * P.K * FR;
  const int W = nwg / P.K;  // workgroups per subproblem (the host guarantees 1 <= W <= B)
  const int k = (int)blockIdx.x / W, wl = (int)blockIdx.x - k * W;
  if (k >= P.K) return;
  const int base = B / W, extra = B - base * W;  // rows 1..B, the longer chunks highest
  const int lo = 1 + wl * base + max(0, wl - (W - extra)), hi = lo + base + (wl >= W - extra ? 1 : 0);
  uint32_t *slot = reinterpret_cast<uint32_t *>(sds + sd_slot_offset<M>());
  auto pslot = [&](int step) { return slot + (step & 1) * L; };  // sphere order of `step`
  // this subproblem's region: NB staging buffers of R rows, then row 0 of every step (k_sdt_row0); one buffer
  // resource over all of it (the host checks it is below 4 GiB)
  double *reg = S_all + (size_t)k * kstride;
  SdPipe<M> h;
  h.lo = lo, h.hi = hi, h.B = B, h.NB = NB, h.nt = nt, h.k = k, h.g0 = k * R + lo;
  h.spin_limit = spin_limit, h.rowb = (unsigned)L * 8u, h.bufb = (unsigned)R * h.rowb, h.r0b = (unsigned)NB * h.bufb;
  h.dk = done + (size_t)k * FR, h.lk = loaded + (size_t)k * FR, h.err = err;
  h.pk = perm_all + (size_t)k * nt * L, h.slot = slot;
  h.rs = __builtin_amdgcn_make_buffer_rsrc(reg, 0, (int)(h.r0b + (unsigned)nt * h.rowb), 0x00020000);
  h.dfa = df_all, h.uoa = uo_all, h.sm = same2, h.sds = sds, h.sh = &sh;
  h.sk = strad ? strad + (size_t)k * nt * 8 * SD_STRAD_N : nullptr;
  h.sslot = reinterpret_cast<uint16_t *>(sds + sd_strad_offset<M>());
  h.pcp = -1, h.pi = 0;
  if (tid == 0) {
    sh.stop = 0;
    sh.cnt[0] = sh.cnt[1] = sh.cnt[2] = sh.cnt[3] = 0;
    sh.nlist[0] = sh.nlist[1] = sh.redo[0] = sh.redo[1] = 0;
  }
  // prologue: both sphere orders of the first step, df / u_old, and the first row's loads (the terminal row was
  // written by an earlier launch)
  sd_perm_dma_asm<M>(h.pk + (size_t)(nt - 1) * L, pslot(nt - 1));
  sd_perm_dma_asm<M>(h.pk + (size_t)(nt - 2) * L, pslot(nt - 2));
  if constexpr (sd_strad<M>()) {
    sd_strad_dma(h.sk + (size_t)(nt - 1) * 8 * SD_STRAD_N, h.sslot + ((nt - 1) & 1) * 8 * SD_STRAD_N);
    sd_strad_dma(h.sk + (size_t)(nt - 2) * 8 * SD_STRAD_N, h.sslot + ((nt - 2) & 1) * 8 * SD_STRAD_N);
  }
  sd_dfuo_dma<M>(df_all + ((size_t)k * nt + nt - 2) * M, uo_all + ((size_t)k * nt + nt - 2) * M,
                 nt >= 3 ? same2 + (size_t)k * nt + nt - 3 : nullptr, sds);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  sd_bar();
  sd_read_next<M>(h.nx, pslot(nt - 1), h.sslot + ((nt - 1) & 1) * 8 * SD_STRAD_N);
  sd_issue_pipe<M>(h.raw, h.rs, h.nx, lo, (unsigned)((nt - 1) % NB) * h.bufb, h.r0b + (unsigned)(nt - 1) * h.rowb,
                   h.rowb);
  // a wait the compiler sees (vmcnt(0), other counters untouched): entering the loop with these loads pending would
  // make it assume, at the loop head, that nothing younger can be outstanding, and wait for every store there
  __builtin_amdgcn_s_waitcnt(0x0F70);
  h.Pp = &P, h.Gp = &G, h.whole = hi - lo == 1;
  {  // the first row's statistics phase (later rows': the previous row's tail)
    double v[8];
    sd_take<M>(v, h.raw);
    const double xs = __hiloint2double((int)h.raw.sv.y, (int)h.raw.sv.x);
    h.valid_next = sdt_stats<M, true>(P, G, k, lo, nt - 2, v, h.raw.e, sh, sds, df_all, uo_all, h.raw.srank, xs);
  }
  int par = 0;     // the row's parity (sdt_body's LDS slots)
  bool stop = false;
  // the staging buffers of steps i and i + 1 (i % NB, (i + 1) % NB), stepped down with i instead of divided per row
  int bi = (nt - 2) % NB, bi1 = (nt - 1) % NB;
#pragma nounroll
  for (int i = nt - 2; i >= 0 && !stop; --i) {
#pragma nounroll
    for (int cp = lo; cp < hi && !stop; ++cp) {
      const bool last_row = cp + 1 == hi;
      h.cp = cp, h.i = i;
      h.ncp = last_row ? lo : cp + 1, h.ni = last_row ? i - 1 : i;  // the next row
      h.has_next = h.ni >= 0;
      h.nbo = (unsigned)(last_row ? bi : bi1) * h.bufb;  // buffer (ni + 1) % NB
      const int g = cp == lo ? h.g0 : 1 << 30;  // timeline stamps: the chunk's first row
      (void)g;
      SD_TL(0);
      // this row's loads, sphere order and df / u_old (everything but the previous row's five stores) have landed (at
      // the previous row's late drain already: its tail ran this row's statistics phase); the memory clobber keeps the
      // LDS reads of what the DMA wrote below this point
      asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
#ifndef SD_TL_DRAIN
      SD_TL(7);
#endif
      uint2 ein[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) ein[q] = h.raw.e[q];
      sdt_body<M, true>(P, Lv, G, k, cp, i, h.valid_next, ein, pslot(i + 1), pslot(i),
                        reg + (size_t)bi * R * L + (size_t)cp * L,
                        UU_all + (size_t)k * uu_stride_k + (size_t)i * ((size_t)R * L) + (size_t)cp * L, sh, sds, h,
                        df_all, uo_all, par, h.raw.mask, h.raw.srank);
      par ^= 1;
      SD_TL(6);
      stop = h.stop_seen;  // read after the row's barrier 3 (every path has one)
    }
    bi1 = bi;
    bi = bi == 0 ? NB - 1 : bi - 1;
  }
  if (tid == 0) {
    if (sh.cnt[0]) atomicAdd(&counters[0], sh.cnt[0]);
    if (sh.cnt[1]) atomicAdd(&counters[1], sh.cnt[1]);
    if (sh.cnt[2]) atomicAdd(&counters[4], sh.cnt[2]);
    if (sh.cnt[3]) atomicAdd(&counters[5], sh.cnt[3]);
  }
  SD_FLUSH();
  SD_TL_FLUSH(h.g0);
}

bool sdt_seam_lists(const PyrGeom &G) { return G.M == 4 && sd_strad<4>(); }

bool sdt_supported(const PyrGeom &G) {
  if (G.M != 3 && G.M != 4) return false;
  for (int m = 0; m < G.M; ++m)
    if (G.n[m] != 8) return false;
  return true;
}

hipError_t launch_sdt_prep(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G,
                           const uint32_t *perm, double *V, double *S, size_t kstride, size_t r0off, uint16_t *UU,
                           size_t uu_stride_k) {
  if (!sdt_supported(G)) return hipErrorInvalidValue;
  if (G.M == 4) {
    hipLaunchKernelGGL(k_sdt_chain<4>, dim3(P.K), dim3(256), 0, s, P, G, Lv.beta, perm, V);
    hipLaunchKernelGGL(k_sdt_row0<4>, dim3(P.nt, P.K), dim3(512), 0, s, P, Lv, G, perm, (const double *)V, S, kstride,
                       r0off, UU, uu_stride_k);
  } else {
    hipLaunchKernelGGL(k_sdt_chain<3>, dim3(P.K), dim3(256), 0, s, P, G, Lv.beta, perm, V);
    hipLaunchKernelGGL(k_sdt_row0<3>, dim3(P.nt, P.K), dim3(64), 0, s, P, Lv, G, perm, (const double *)V, S, kstride,
                       r0off, UU, uu_stride_k);
  }
  return hipGetLastError();
}

hipError_t launch_sdt_run(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G,
                          const uint32_t *perm, const int32_t *same2, const uint16_t *strad, double *S, size_t kstride,
                          int NB, uint16_t *UU,
                          size_t uu_stride_k, int32_t *counters, int32_t *flags, int nwg, unsigned spin_limit,
                          size_t lds) {
  if (!sdt_supported(G)) return hipErrorInvalidValue;
  // every workgroup must be resident at once (the row hand-off spins on other workgroups): the caller sizes the grid
  // to the CUs x resident workgroups per CU (sdt_run_blocks_per_cu); a dependency wait that times out anyway (another
  // process's kernels holding CUs) sets the error word and the host redoes the DP per step.  An ordinary launch, not a
  // cooperative one: a cooperative launch leaves the HIP runtime cooperative-queue state that it tears down at process
  // exit, which crashed every rocprofv3 run of round 3 (profiles/round4_exit_probe.txt)
  void *args[] = {(void *)&P,     (void *)&Lv,       (void *)&G,         (void *)&perm,
                  (void *)&S,     (void *)&kstride,  (void *)&NB,        (void *)&UU,
                  (void *)&uu_stride_k, (void *)&counters, (void *)&flags, (void *)&nwg, (void *)&spin_limit,
                  (void *)&P.df,  (void *)&P.uold, (void *)&same2, (void *)&strad};
  if (G.M == 4) return hipLaunchKernel((const void *)k_sdt_run<4>, dim3(nwg), dim3(512), args, lds, s);
  return hipLaunchKernel((const void *)k_sdt_run<3>, dim3(nwg), dim3(64), args, lds, s);
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
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sdt_tl), (size_t)nrows * 64 * 8 * sizeof(unsigned long long)) ==
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
