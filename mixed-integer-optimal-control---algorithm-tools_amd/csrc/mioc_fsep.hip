// mioc_fsep.hip -- the fused separable DP of a small 2-D product grid (p = 1, the batch path):
// bellman_TRM! (HelpFunctions.jl:20-83) for one subproblem entirely on chip, round-3 layout.
//
//   * Two lanes per source row c': lane pair (2r, 2r+1) splits the N0 x N1 grid into its x1 halves, so one
//     wave carries 32 rows and a row's separable transform is half as long.  Lane 2r holds x1 = 0..H-1 in its
//     slots s = 0..H-1, lane 2r+1 holds x1 = N1-1..H in the same slots (mirrored), which makes the cross-half
//     step of the x1 pass the same instruction on both lanes: take the partner's slot H-1 (DPP swap) and merge
//     it into slot H-1-t at cost t+1.
//   * Four lanes per row (LN = 4, the row-segment launches of small batches): the lane quad also splits x0 into
//     mirrored halves, with the same cross-half step in the x0 pass (partner lane ^ 2).  A wave then carries 16
//     rows, so a segment of 128 rows fills 8 waves, two per SIMD, where two lanes per row leave one wave per SIMD
//     with nothing to hide its dependency chains behind.
//   * The front Φ is updated IN PLACE: read phase (every lane reads its row, runs the transform, gathers its
//     results into registers), barrier, write phase (results, the inbox of the segment below, +Inf cells, the
//     next step's K table), barrier.  One copy of the front (~79 KB at C5) lets two subproblems share a CU.
//   * A subproblem may be split into S row segments on S workgroups (strong scaling: 128 restarts still fill
//     256 CUs).  Segment q owns rows [lo_q, hi_q); the targets its rows send above hi_q (at most SMAX rows) go
//     to an outbox ring in HBM that segment q+1 reads one step later.  The hand-off is one-directional, so
//     segment q never waits for q+1 except to reuse a ring slot (NB steps back).  Flags are relaxed agent-scope
//     atomics in the measured-valid form of MI355X_MICROARCH.md (sc1 stores drained by every storing wave,
//     then one lane's flag store behind a barrier; the consumer loads the bytes only after its own poll
//     matched).  S > 1 needs every workgroup resident: the host launches it only when K·S fits the CUs x resident
//     workgroups per CU (an ordinary launch, not a cooperative one); a wait past the spin limit sets *err and every
//     workgroup leaves, and the host redoes the DP with S = 1 (check_run).
//
// Certified argmin, as in mioc_fused.hip's k_fsep_run: V_j = trunc_g(base + (Ψ_j - Ψmin)/β) with the source
// coordinates x0 | x1 << 3 in the 6 low mantissa bits and bit 6 as the near-tie flag; an unflagged winner is the
// reference's unique argmin and its value is recomputed with the reference's expression
// fl(fl(T1_l + fl(β·d)) + Ψ_j*) from the per-step table K_l[d].  Flagged targets and rows outside the binade run
// the reference loop (HelpFunctions.jl:60-77) exactly, one lane per target.  The merge order of a separable pass
// does not matter for the certificate: any binary merge tree compares the eventual winner's candidate set with
// every other set's minimum, so a candidate within tol of the winner always sets the flag.
//
// HBM traffic per subproblem: df, u_old once, U = (nt-1)·L·(B+1) bytes, Φ_0 = L·RP·8 bytes at the end, plus
// (S > 1) the outbox rows: (nt-1)·SMAX·L·8 bytes per segment boundary, written once and read once.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <climits>
#include <cstdint>

#include "mioc_internal.h"

namespace mioc {

namespace {

constexpr int FS2_FLAG = 64;  // near-tie flag (payload bit 6)
constexpr int FS2_MAXT = 512;  // threads per workgroup: 256 budget rows + row B (larger B: mioc_fused.hip)
#ifndef FSEP_LANES4
#define FSEP_LANES4 1  // row segments with four lanes per row where they fit (A/B builds: 0)
#endif

__device__ __forceinline__ void fs_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ double fs_min(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// merge of two candidate sets in 32-bit fixed point (finite candidates < 2^30, +Inf = 2^30, so every operand and
// sum stays below 2^31): the smaller, flagged (bit 6) when the two are within tolerance.  ntol = -(tolq + 1):
// |a - t| + ntol has bit 31 set exactly when |a - t| <= tolq.  Five VALU ops.
__device__ __forceinline__ unsigned fs_qmerge(unsigned a, unsigned nb, unsigned d, unsigned ntol) {
  const unsigned t = nb + d;
  const unsigned m = min(a, t);
  unsigned x;
  asm("v_sad_u32 %0, %1, %2, %3" : "=v"(x) : "v"(a), "v"(t), "v"(ntol));
  return m | ((x >> 25) & (unsigned)FS2_FLAG);
}

__device__ __forceinline__ double fs_max(double a, double b) {  // v_max_f64 without the canonicalising operands
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

template <int CTRL>
__device__ __forceinline__ double fs_dpp(double x) {
  return __hiloint2double(__builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xF, 0xF, true),
                          __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ double fs_rdl(double x, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l), __builtin_amdgcn_readlane(__double2loint(x), l));
}
// minimum over the wave: DPP within each row of 16 lanes (quad swaps, half-row and row mirrors), then the four
// rows' lane 0, 16, 32, 48
__device__ __forceinline__ double fs_wave_min(double v) {
  v = fs_min(v, fs_dpp<0xB1>(v));
  v = fs_min(v, fs_dpp<0x4E>(v));
  v = fs_min(v, fs_dpp<0x141>(v));
  v = fs_min(v, fs_dpp<0x140>(v));
  return fs_min(fs_min(fs_rdl(v, 0), fs_rdl(v, 16)), fs_min(fs_rdl(v, 32), fs_rdl(v, 48)));
}

typedef unsigned fs_u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned fs_swap_u(unsigned x) {
  return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);
}

// the partner lane's (tid ^ 1) value: DPP quad_perm [1, 0, 3, 2], no LDS round trip
__device__ __forceinline__ double fs_swap(double x) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), 0xB1, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), 0xB1, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ int fs_uint(double u) { return (int)fmin(fmax(u, -1.0e8), 1.0e8); }

}  // namespace

// diagnostic build (make stamps): per-wave phase cycles (s_memtime), summed over the steps
#if defined(MIOC_STAMPS)
__device__ unsigned long long g_fs_stamps[4096][8];
#define FS_T(v) [[maybe_unused]] unsigned long long v = __builtin_amdgcn_s_memtime()
#define FS_ACC(q, a, b) acc[q] += (b) - (a)
#else
#define FS_T(v)
#define FS_ACC(q, a, b)
#endif

struct FsepArgs {
  double *front0;
  size_t front_stride;
  uint8_t *U;
  size_t u_stride_k;
  int32_t *counters;
  double *ring;    // [K][S][NB][SMAX][L]: segment q's outbox (rows hi_q .. hi_q + SMAX - 1), read by q + 1
  int32_t *flags;  // [K][S][2] {outbox token, consumed token}, then the error flag at [2·K·S]
  int S, RS, NB;   // segments, rows per segment (a multiple of 32), ring depth
  int koff;        // K table offset in the LDS (doubles)
  int stg;         // S > 1: the inbox staging rows in the LDS (doubles)
  int slot_bytes;  // S > 1: bytes per ring slot (SMAX·L doubles, rounded up to 1 KiB: whole LDS-DMA chunks)
  unsigned spin_limit;
  int base0, base1;
};

// the partner lane's (tid ^ 2) value: DPP quad_perm [2, 3, 0, 1]
__device__ __forceinline__ unsigned fs_swap2_u(unsigned x) {
  return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);
}
__device__ __forceinline__ double fs_swap2(double x) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), 0x4E, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), 0x4E, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

// LN lanes per source row (2: x1 halves; 4: x1 and x0 halves).  A lane's slot t = s·H0 + u holds the level
// x0 = h0 ? N0-1-u : u, x1 = h1 ? N1-1-s : s (h1 = lane bit 0, h0 = lane bit 1 for LN = 4, else 0).
template <int N0, int N1, bool SEG, int LN>
__global__ __launch_bounds__(FS2_MAXT) __attribute__((amdgpu_waves_per_eu(!SEG && N0 * N1 <= 36 ? 4 : 2))) void k_fsep2(
    ProblemDev P, LevelsDev Lv, FsepArgs A) {
  constexpr int L = N0 * N1, H = N1 / 2, H0 = LN == 4 ? N0 / 2 : N0, V = H0 * H, SMAX = N0 + N1 - 2, ND = SMAX + 1;
  constexpr int LSH = LN == 4 ? 2 : 1, RPW = 64 / LN;  // lanes per row (log2), rows per wave
  constexpr int FS = (L + 1) | 1;  // odd row stride (8-byte words)
  static_assert(N1 % 2 == 0 && (LN == 2 || N0 % 2 == 0) && N0 <= 8 && N1 <= 8 && V <= 32, "grid shape");
  extern __shared__ __attribute__((aligned(16))) unsigned char fsm[];
  __shared__ int s_stop;
  const int S = SEG ? A.S : 1, k = (int)blockIdx.x / S, q = (int)blockIdx.x - k * S;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nthr = blockDim.x, nw = nthr >> 6;
  const int B = P.B, R = B + 1, nt = P.nt, NB = A.NB;
  const int lo = min(R, q * A.RS), hi = q == S - 1 ? R : min(R, (q + 1) * A.RS);
  const int nloc = min(R, hi + SMAX) - lo;  // LDS rows: own rows, then the outbox halo
  double *const F = reinterpret_cast<double *>(fsm);
  double *const Kt = F + A.koff;
  // d(l, j), the L1 distance of two levels, one byte each (static: built once)
  unsigned char *const Dt = reinterpret_cast<unsigned char *>(Kt + L * ND);
  const int cx = lo + (nthr >> LSH);  // past the lane groups: the extra row (row B) when cx < hi
  const double beta = Lv.beta, inv = Lv.inv_beta;
  const double numx0 = (double)max(abs(A.base0), abs(A.base0 + N0 - 1)),
               numx1 = (double)max(abs(A.base1), abs(A.base1 + N1 - 1));
  // this segment's record {outbox token, consumed token}, FSEP_FLAG_STRIDE words apart from its neighbours'
  constexpr int FW = FSEP_FLAG_STRIDE;
  int32_t *const fl = A.flags + FW * ((size_t)k * S + q);
  int32_t *const err = A.flags + FW * (size_t)P.K * S;
  // rings through buffer resources (32-bit offsets, sc1 accesses); the inbox slot is copied into the LDS staging
  // rows by LDS-DMA (no registers held across the read phase)
  const size_t ring_seg = SEG ? (size_t)NB * A.slot_bytes : 0;
  const __amdgpu_buffer_rsrc_t ring_out =
      __builtin_amdgcn_make_buffer_rsrc((char *)A.ring + ((size_t)k * S + q) * ring_seg, 0, (int)ring_seg, 0x00020000);
  const char *const ring_in = (const char *)A.ring + ((size_t)k * S + (q > 0 ? q - 1 : 0)) * ring_seg;

  auto inputs = [&](int s, double &a0, double &a1, double &u0, double &u1) {
    const double *dfs = P.df + ((size_t)k * nt + s) * 2;
    const double *uos = P.uold + ((size_t)k * nt + s) * 2;
    a0 = P.dt * dfs[0];
    a1 = P.dt * dfs[1];
    u0 = uos[0];
    u1 = uos[1];
  };
  // per-step table, HelpFunctions.jl:52-67: K_l[d] = fl(T1(l) + fl(β·d))
  auto prepare = [&](double a0, double a1) {
    for (int e = tid; e < L * ND; e += nthr) {
      const int l = e / ND, d = e - l * ND;
      const double t1 = (0.0 + a0 * (double)(A.base0 + l % N0)) + a1 * (double)(A.base1 + l / N0);
      Kt[e] = t1 + beta * (double)d;
    }
  };
  // a wave-uniform wait for a flag to reach `need`; false (and the launch abandoned) past the spin limit
  auto wait_flag = [&](const int32_t *f, int &val, int need) {
    unsigned spins = 0;
    while (!__all(val >= need)) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) || ++spins > A.spin_limit) {
        if (lane == 0) {
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_stop = 1;
        }
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
      val = __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return true;
  };

  // ---- terminal step (HelpFunctions.jl:27-43): Φ_{nt-1}[c][l] = T1 where b̃_l(nt-1) = c --------------------
  double ca0 = 0.0, ca1 = 0.0;
  int cu0 = 0, cu1 = 0;
  {
    double a0, a1, u0, u1;
    inputs(nt - 1, a0, a1, u0, u1);
    const int iu0 = fs_uint(u0), iu1 = fs_uint(u1);
    for (int e = tid; e < nloc * FS; e += nthr) {
      const int c = lo + e / FS, l = e % FS;
      double v = INFINITY;
      if (l < L && abs(A.base0 + l % N0 - iu0) + abs(A.base1 + l / N0 - iu1) == c)
        v = (0.0 + a0 * (double)(A.base0 + l % N0)) + a1 * (double)(A.base1 + l / N0);
      F[e] = v;
    }
    if (nt >= 2) {
      inputs(nt - 2, a0, a1, u0, u1);
      prepare(a0, a1);
      ca0 = a0;
      ca1 = a1;
      cu0 = fs_uint(u0);
      cu1 = fs_uint(u1);
    }
    if (tid == 0) s_stop = 0;
    for (int e = tid; e < L * L; e += nthr) {
      const int l = e / L, j = e - l * L;
      Dt[e] = (unsigned char)(abs(l % N0 - j % N0) + abs(l / N0 - j / N0));
    }
  }
  __syncthreads();
  uint8_t *Uk = A.U + (size_t)k * A.u_stride_k;
  int nflag = 0, nscan = 0;
  // the inbox flag of the segment below, polled one step ahead: the value a step checks was loaded during the step
  // before, so the inbox copy issues at the start of the read phase and its latency hides behind the transform
  int vin_next = 0;
  if (SEG && q > 0) vin_next = __hip_atomic_load(fl - FW, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if defined(MIOC_STAMPS)
  unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
#pragma nounroll
  for (int i = nt - 2; i >= 0; --i) {
    // this lane's row and slots, derived from an opaque copy of the thread index every step: hoisted out of the
    // step loop, the per-target constants (LDS offsets, U offsets) would take more registers than the row itself
    int tido = tid;
    asm volatile("" : "+v"(tido));
    const int hf = tido & 1, h0 = LN == 4 ? (tido >> 1) & 1 : 0;
    const int cp = lo + (tido >> LSH);  // this lane group's source row
    const bool act = cp < hi;
    const int room = act ? B - cp : -1;  // target l of this row is inside the trust region iff b̃_l <= room
    const int cl = act ? cp - lo : 0;
    // slot (s, u) at F[lb + ls·s + lu·u]
    const int lb = cl * FS + (hf ? N0 * (N1 - 1) : 0) + (h0 ? N0 - 1 : 0), ls = hf ? -N0 : N0, lu = h0 ? -1 : 1;
    int x1v[H], x0v[H0];
#pragma unroll
    for (int s = 0; s < H; ++s) x1v[s] = hf ? N1 - 1 - s : s;
#pragma unroll
    for (int u = 0; u < H0; ++u) x0v[u] = h0 ? N0 - 1 - u : u;
    const int su0 = __builtin_amdgcn_readfirstlane(cu0), su1 = __builtin_amdgcn_readfirstlane(cu1);
    auto btl = [&](int x0, int x1) { return abs(A.base0 + x0 - su0) + abs(A.base1 + x1 - su1); };
    // U_i[l][c] through a buffer resource (bounds-checked to the step's L·R bytes: a store past them is dropped)
    const __amdgpu_buffer_rsrc_t Ur =
        __builtin_amdgcn_make_buffer_rsrc(Uk + (size_t)i * ((size_t)L * R), 0, L * R, 0x00020000);
    double na0 = 0.0, na1 = 0.0, nu0 = 0.0, nu1 = 0.0;
    if (i >= 1) inputs(i - 1, na0, na1, nu0, nu1);
    // polls, issued now and checked later: the outbox of the segment below for this step (RAW), and whether
    // the segment above has consumed the ring slot this step's outbox overwrites (WAR)
    const int need_in = SEG && q > 0 ? nt - 1 - i : INT_MIN;
    const int need_cons = SEG && q < S - 1 && i + NB <= nt - 2 ? nt - 1 - (i + NB) : INT_MIN;
    int vin = vin_next, vcons = 0;
    if (SEG && need_cons != INT_MIN) vcons = __hip_atomic_load(fl + FW + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    // ================= read phase: Φ_{i+1} rows into registers, the transform, results into registers ========
    FS_T(q0);
    // ---- the segment below has published this step's outbox: load it (consumed in the write phase) --------
    if (SEG && q > 0 && wait_flag(fl - FW, vin, need_in)) {
      if (i >= 1) vin_next = vin >= need_in + 1 ? vin : __hip_atomic_load(fl - FW, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // LDS-DMA of the slot, 1 KiB chunks by wave (inline asm: the compiler does not make later LDS accesses
      // wait for it; the drain before barrier 1 completes it, the barrier publishes it)
      const char *slot = ring_in + (size_t)(i % NB) * A.slot_bytes;
      const unsigned lds0 = (unsigned)(uintptr_t)((__attribute__((address_space(3))) char *)(fsm)) + A.stg * 8u;
      for (int c = w; c < A.slot_bytes / 1024; c += nw) {
        const char *gsrc = slot + c * 1024 + lane * 16;
        const unsigned m0 = __builtin_amdgcn_readfirstlane(lds0 + (unsigned)c * 1024u);
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc1\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(gsrc), "s"(m0)
                     : "memory");
      }
    }
    double o[V];
#pragma unroll
    for (int s = 0; s < H; ++s)
#pragma unroll
      for (int u = 0; u < H0; ++u) o[u + H0 * s] = F[lb + ls * s + lu * u];
    const double a0 = ca0, a1 = ca1;
    // ---- row statistics over the finite sources (every lane of the group) ---------------------------------
    double pmn = o[0], pmx = o[0];
#pragma unroll
    for (int j = 1; j < V; ++j) {
      pmn = fs_min(pmn, o[j]);
      pmx = fs_max(pmx, o[j]);
    }
    pmn = fs_min(pmn, fs_swap(pmn));
    pmx = fs_max(pmx, fs_swap(pmx));
    if constexpr (LN == 4) {
      pmn = fs_min(pmn, fs_swap2(pmn));
      pmx = fs_max(pmx, fs_swap2(pmx));
    }
    const bool infrow = !(pmx < INFINITY);
    if (__ballot(infrow && pmn < INFINITY)) {  // some sources unreachable: the maximum over the finite ones
      double m2 = pmn;
#pragma unroll
      for (int j = 0; j < V; ++j) m2 = fs_max(m2, o[j] < INFINITY ? o[j] : pmn);
      m2 = fs_max(m2, fs_swap(m2));
      if constexpr (LN == 4) m2 = fs_max(m2, fs_swap2(m2));
      pmx = m2;
    }
    // ---- 32-bit fixed point: A_j = trunc((Ψ_j - Ψmin)/β · 2^Fb) << 7 | j (rank), +Inf = 2^30 -----------------
    // (β units, grid g = 2^-Fb with 2^(Fb+7) · rs < 2^30: every finite candidate value A + d·2^(Fb+7) stays below
    // 2^30, so unit steps are exact integer additions; +Inf plus any distance stays in [2^30, 2^31))
    const double rs = (pmx - pmn) * inv + (double)SMAX;  // scaled range of every candidate value
    const bool scale_ok = rs < 0x1p17;
    const int E = ilogb(fmin(rs, 0x1p17) * (1.0 + 0x1p-20) + 1.0) + 1;  // 2^E > rs
    const int Fb = 23 - E;
    const double g = ldexp(1.0, -Fb);
    const double qmax = beta * (double)SMAX + fmax(fabs(pmn), fabs(pmx)) + fabs(a0) * numx0 + fabs(a1) * numx1;
    // 2 x stamping error (< g, the fma's rounding included) + 2 x the reference's rounding (<= 4u·qmax per
    // candidate), in units of β
    const double tol = 3.0 * g + 0x1p-49 * qmax * inv;
    const bool none = !(pmn < INFINITY);
    const bool direct = !none && !(scale_ok && tol < 0.25);
    const double sc = ldexp(inv, Fb);
    const unsigned U1 = 1u << (Fb + 7);  // one unit of distance
    const unsigned ntol = direct ? ~0u : ~(unsigned)(tol * ldexp(1.0, Fb + 7));  // -(tolq + 1)
    if (none) pmn = 0.0;
    const double c0 = -pmn * sc;
    unsigned a[V];
#pragma unroll
    for (int s = 0; s < H; ++s)
#pragma unroll
      for (int u = 0; u < H0; ++u) {
        const int t = u + H0 * s;
        // +Inf converts to 0xFFFFFFFF (clamped), which the min turns into 2^30
        const unsigned q0 = (unsigned)__builtin_fma(o[t], sc, c0) << 7 | (unsigned)(x0v[u] + N0 * x1v[s]);
        a[t] = min(q0, 0x40000000u);
      }
    __builtin_amdgcn_sched_barrier(0);
    FS_T(q1);
    // ---- pass along x0: this lane's H line pieces (orientation-free), then (LN = 4) the partner's boundary ----
#pragma unroll
    for (int s = 0; s < H; ++s) {
#pragma unroll
      for (int u = 1; u < H0; ++u) a[s * H0 + u] = fs_qmerge(a[s * H0 + u], a[s * H0 + u - 1], U1, ntol);
#pragma unroll
      for (int u = H0 - 2; u >= 0; --u) a[s * H0 + u] = fs_qmerge(a[s * H0 + u], a[s * H0 + u + 1], U1, ntol);
    }
    if constexpr (LN == 4) {
#pragma unroll
      for (int s = 0; s < H; ++s) {
        const unsigned pb = fs_swap2_u(a[s * H0 + H0 - 1]);
#pragma unroll
        for (int t = 0; t < H0; ++t)
          a[s * H0 + H0 - 1 - t] = fs_qmerge(a[s * H0 + H0 - 1 - t], pb, (t + 1) * U1, ntol);
      }
    }
    // ---- pass along x1: this lane's H slots (orientation-free), then the partner's boundary slot ------------
#pragma unroll
    for (int u = 0; u < H0; ++u) {
#pragma unroll
      for (int s = 1; s < H; ++s) a[s * H0 + u] = fs_qmerge(a[s * H0 + u], a[(s - 1) * H0 + u], U1, ntol);
#pragma unroll
      for (int s = H - 2; s >= 0; --s) a[s * H0 + u] = fs_qmerge(a[s * H0 + u], a[(s + 1) * H0 + u], U1, ntol);
    }
#pragma unroll
    for (int u = 0; u < H0; ++u) {
      const unsigned pb = fs_swap_u(a[(H - 1) * H0 + u]);
#pragma unroll
      for (int t = 0; t < H; ++t) a[(H - 1 - t) * H0 + u] = fs_qmerge(a[(H - 1 - t) * H0 + u], pb, (t + 1) * U1, ntol);
    }
    __builtin_amdgcn_sched_barrier(0);
    FS_T(q2);
    // ---- winners: R(l, j*) = fl(K_l[d(l, j*)] + Ψ_j*) for the certified winner j* ----------------------------
    // b̃_l = |ν0 - u0| + |ν1 - u1| splits into a wave-uniform x0 part (SGPRs) and this lane's x1 part per slot
    unsigned vmask = 0, smask = 0;
    const unsigned dirb = direct ? 1u : 0u;
    uint32_t jw[(V + 3) / 4];
#pragma unroll
    for (int u = 0; u < (V + 3) / 4; ++u) jw[u] = 0;
    const double *const Frow = F + cl * FS;
#pragma unroll
    for (int s = 0; s < H; ++s) {
      const int x1 = x1v[s];
      const int rr = abs(A.base1 + x1 - su1) - room - 1;  // + |ν0 - u0| < 0  <=>  b̃_l <= room
      const double *const Ks = Kt + N0 * x1 * ND;         // K_l[·] of l = x0 + N0·x1 at Ks + x0·ND
      const unsigned char *const Ds = Dt + N0 * x1 * L;   // d(l, ·) at Ds + x0·L
      double kv[H0], pv[H0];
#pragma unroll
      for (int u = 0; u < H0; ++u) {
        const unsigned jx = a[u + H0 * s] & 63u;
        kv[u] = Ks[x0v[u] * ND + Ds[x0v[u] * L + jx]];
        pv[u] = Frow[jx];
      }
      // targets of this line inside the trust region: |ν0 - u0| <= room - |ν1 - u1| = -1 - rr is an interval of
      // x0 around u0 - base0 (wave-uniform), so the line's mask is a bit range
      {
        const int thr = -1 - rr, uc = su0 - A.base0;
        const int x0lo = max(uc - thr, 0), x0hi = min(uc + thr, N0 - 1);
        if constexpr (LN == 4) {  // this lane's half of the line, slot u = x0 (h0 = 0) or N0-1-x0 (mirrored)
          const int ulo = h0 ? N0 - 1 - x0hi : x0lo, uhi = h0 ? N0 - 1 - x0lo : x0hi;
          const int a0s = max(ulo, 0), a1s = min(uhi, H0 - 1);
          const unsigned lm = thr >= 0 && a0s <= a1s ? ((2u << a1s) - (1u << a0s)) : 0u;
          vmask |= lm << (H0 * s);
        } else {
          const unsigned lm = thr >= 0 && x0lo <= x0hi ? ((2u << x0hi) - (1u << x0lo)) : 0u;
          vmask |= lm << (N0 * s);
        }
      }
#pragma unroll
      for (int u = 0; u < H0; ++u) {
        const int t = u + H0 * s;
        const unsigned av = a[t];
        // flagged and finite (below 2^30): bit 6 set, bit 30 clear -- integer arithmetic, a shift-or per target
        // (a condition would become a select between 0 and a materialised 1 << t per bit)
        const unsigned sb = ((av >> 6) & ~(av >> 30)) & 1u;
        smask |= sb << t;
        const bool fin = av < 0x40000000u;
        const double sum = kv[u] + pv[u];
        o[t] = fin ? sum : INFINITY;
        jw[t >> 2] |= (av & 63u) << (8 * (t & 3));
      }
      __builtin_amdgcn_sched_barrier(0);  // one line's gathers at a time (all in flight would need 4·V VGPRs)
    }
    FS_T(q3);
    // flagged targets count only inside the trust region; a row outside the fixed-point range scans them all
    smask = dirb ? vmask : smask & vmask;
    // the masks stay VGPR words: seen through, the compiler keeps one 64-bit lane mask per target in SGPRs
    // through the barrier (and spills them)
    asm volatile("" : "+v"(vmask), "+v"(smask));
    // ---- exact scans (near ties, rows outside the binade): the reference loop, one lane per target ---------
    if (__ballot(smask != 0)) {
#pragma unroll
      for (int s = 0; s < H; ++s)
#pragma unroll
        for (int u = 0; u < H0; ++u) {
          const int t = u + H0 * s;
          if ((smask >> t) & 1u) {
            const int x0 = x0v[u], x1 = x1v[s], l = x0 + N0 * x1;
            double best = INFINITY;
            int bj = 0;
#pragma unroll 4
            for (int j = 0; j < L; ++j) {
              const int dj = abs(x0 - j % N0) + abs(x1 - j / N0);
              const double v = Kt[l * ND + dj] + F[cl * FS + j];
              if (v < best) {  // strict: the first j in iterator order wins ties (HelpFunctions.jl:71-76)
                best = v;
                bj = j;
              }
            }
            o[t] = best;
            jw[t >> 2] = (jw[t >> 2] & ~(0xFFu << (8 * (t & 3)))) | ((uint32_t)bj << (8 * (t & 3)));
          }
        }
      nscan += __popc(smask);
      nflag += direct ? 0 : __popc(smask);
    }
    // ---- the extra row (row B, past the lane pairs): its one target, u_old(i) itself, by an exact scan -------
    double xv = INFINITY;
    int xj = 0, xl = -1;
    if (w == nw - 1 && cx < hi) {
      const int x0t = su0 - A.base0, x1t = su1 - A.base1;
      if (x0t >= 0 && x0t < N0 && x1t >= 0 && x1t < N1) {
        xl = x0t + N0 * x1t;
        double v = INFINITY;
        if (lane < L)
          v = Kt[xl * ND + abs(x0t - lane % N0) + abs(x1t - lane / N0)] + F[(cx - lo) * FS + lane];
        xv = fs_wave_min(v);
        const unsigned long long at = __ballot(v == xv);  // the first source attaining it (iterator order)
        xj = at ? (int)__builtin_ctzll(at) : 0;
        if (lane == 0) nscan += 1;
      }
    }
    FS_T(q4);
    // every wave's outstanding global accesses (the previous write phase's U / outbox stores, this step's
    // inbox loads) complete before the barrier: the flags published after it cover them
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    fs_bar();  // ---- every lane has read Φ_{i+1}: the front may be overwritten ---------------------------------
    FS_T(q5);
    if (SEG && tid == 0) {
      if (q < S - 1 && i + 1 <= nt - 2)
        __hip_atomic_store(fl, nt - 1 - (i + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // outbox of i+1
      if (q > 0) __hip_atomic_store(fl + 1, nt - 1 - i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // inbox i read
    }
    // ================= write phase: Φ_i ======================================================================
    if (SEG && need_cons != INT_MIN) wait_flag(fl + FW + 1, vcons, need_cons);
    // the write offsets from a second opaque copy of the thread index, taken after the barrier: computed before
    // it, they would stay live through the whole read phase
    int tidw = tid;
    asm volatile("" : "+v"(tidw));
    const int hfw = tidw & 1, h0w = LN == 4 ? (tidw >> 1) & 1 : 0, cpw = lo + (tidw >> LSH);
    double *const padw = F + (cpw < hi ? cpw - lo : 0) * FS + L;  // this lane group's pad word (never read)
#pragma unroll
    for (int s = 0; s < H; ++s) {
      const int x1 = hfw ? N1 - 1 - s : s;
      const int cb = cpw + abs(A.base1 + x1 - su1);  // target row minus the wave-uniform |ν0 - u0|
      double *const Fw = F + (int)__umul24((unsigned)(cb - lo), (unsigned)FS) + N0 * x1;
      // U offset l·R + c, less x0·R + |ν0 - u0| (kept opaque: re-associated, the x0·R terms become a v_mul_lo
      // per target)
      int ub = (int)__umul24((unsigned)(N0 * x1), (unsigned)R) + cb;
      asm volatile("" : "+v"(ub));
#pragma unroll
      for (int u = 0; u < H0; ++u) {
        const int x0 = h0w ? N0 - 1 - u : u, t = u + H0 * s, bx0 = abs(A.base0 + x0 - su0);
        const bool v = (vmask >> t) & 1u;
        // branch-free: a target outside the trust region writes this row's pad word (column L) instead
        double *const dst = v ? Fw + (bx0 * FS + x0) : padw;
        *dst = o[t];
        __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(jw[t >> 2] >> (8 * (t & 3))), Ur,
                                             v && o[t] < INFINITY ? ub + x0 * R + bx0 : 0x40000000, 0, 0);
      }
    }
    FS_T(w1);
    // the outbox: targets above hi (only waves whose rows reach within SMAX of hi), sc1 stores into the ring
    if (SEG && q < S - 1 && lo + RPW * (w + 1) + SMAX > hi) {
      const unsigned slot0 = (unsigned)(i % NB) * (unsigned)A.slot_bytes;
#pragma unroll
      for (int s = 0; s < H; ++s) {
        const int x1 = hfw ? N1 - 1 - s : s;
        const int cb = cpw + abs(A.base1 + x1 - su1);
#pragma unroll
        for (int u = 0; u < H0; ++u) {
          const int x0 = h0w ? N0 - 1 - u : u, t = u + H0 * s, c = cb + abs(A.base0 + x0 - su0);
          const bool v = ((vmask >> t) & 1u) && c >= hi;
          const double ov = o[t];
          __builtin_amdgcn_raw_buffer_store_b64(
              (fs_u32x2){(unsigned)__double2loint(ov), (unsigned)__double2hiint(ov)}, ring_out,
              v ? slot0 + (unsigned)(((c - hi) * L + N0 * x1 + x0) * 8) : 0x80000000u, 0, 16);
        }
      }
    }
    if (xl >= 0 && lane == 0) {
      F[(cx - lo) * FS + xl] = xv;
      __builtin_amdgcn_raw_buffer_store_b8((unsigned char)xj, Ur, xv < INFINITY ? xl * R + cx : 0x40000000, 0, 0);
    }
    FS_T(w2);
    if (SEG && q > 0 && lane < L) {  // the inbox: cells of rows lo .. lo+SMAX-1 whose source row is below lo
      const int bl = abs(A.base0 + lane % N0 - su0) + abs(A.base1 + lane / N0 - su1);
      const double *stg = F + A.stg;
      for (int r = w; r < SMAX; r += nw) {
        const int c = lo + r;
        if (c < hi && c >= bl && c - bl < lo) F[r * FS + lane] = stg[r * L + lane];
      }
    }
    FS_T(w3);
    // cells below the target's own budget class (c < b̃_l: no source row): +Inf.  On the level grid b̃ <= SMAX, so
    // these are rows < SMAX, one pass of the workgroup over SMAX·L cells (the first segment only); an off-grid
    // u_old (wave-uniform test) takes the general loop
    if (abs(A.base0 - su0) + abs(A.base0 + N0 - 1 - su0) <= N0 - 1 &&
        abs(A.base1 - su1) + abs(A.base1 + N1 - 1 - su1) <= N1 - 1) {  // u_old(i) inside the grid's box
      if (lo < SMAX)
        for (int e = tid; e < SMAX * L; e += nthr) {
          const int c = e / L, l = e - c * L;
          if (c >= lo && c < hi && c < btl(l % N0, l / N0)) F[(c - lo) * FS + l] = INFINITY;
        }
    } else {
      const int ws = __builtin_amdgcn_readfirstlane(w);
#pragma unroll 1
      for (int l = ws; l < L; l += nw) {
        const int b = min(btl(l % N0, l / N0), hi);
        for (int c = lo + lane; c < b; c += 64) F[(c - lo) * FS + l] = INFINITY;
      }
    }
    FS_T(w4);
    if (i >= 1) prepare(na0, na1);
    ca0 = na0;
    ca1 = na1;
    cu0 = fs_uint(nu0);
    cu1 = fs_uint(nu1);
    FS_T(q6);
    fs_bar();  // ---- Φ_i complete -------------------------------------------------------------------------------
    FS_T(q7);
#if defined(MIOC_STAMPS_WRITE)  // the write phase in detail
    FS_ACC(0, q0, q5);
    FS_ACC(1, q5, w1);
    FS_ACC(2, w1, w2);
    FS_ACC(3, w2, w3);
    FS_ACC(4, w3, w4);
    FS_ACC(5, w4, q6);
    FS_ACC(6, q6, q7);
    FS_ACC(7, q0, q7);
#else
    FS_ACC(0, q0, q1);
    FS_ACC(1, q1, q2);
    FS_ACC(2, q2, q3);
    FS_ACC(3, q3, q4);
    FS_ACC(4, q4, q5);
    FS_ACC(5, q5, q6);
    FS_ACC(6, q6, q7);
    FS_ACC(7, q0, q7);
#endif
    if (s_stop) break;
  }
#if defined(MIOC_STAMPS)
  if (lane == 0)
    for (int u = 0; u < 8; ++u) g_fs_stamps[((int)blockIdx.x * nw + w) & 4095][u] = acc[u];
#endif
  // the last step's outbox
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (SEG && tid == 0 && q < S - 1 && !s_stop)
    __hip_atomic_store(fl, nt - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    nflag += __shfl_xor(nflag, off);
    nscan += __shfl_xor(nscan, off);
  }
  if (lane == 0 && (nflag | nscan)) {  // diagnostics: [0] near-tie targets, [1] other exact-scan targets
    atomicAdd(&A.counters[0], nflag);
    atomicAdd(&A.counters[1], nscan - nflag);
  }
  // ---- Φ_0 to HBM in the generic layout [L][RP] (the backtrack's argmin reads it): this segment's rows -----
  double *f0 = A.front0 + (size_t)k * A.front_stride;
  const int chi = q == S - 1 ? P.RP : hi;
  for (int e = tid; e < L * (chi - lo); e += nthr) {
    const int l = e / (chi - lo), c = lo + e % (chi - lo);
    f0[(size_t)l * P.RP + c] = c < R ? F[(c - lo) * FS + l] : INFINITY;
  }
}

// ---- host side ---------------------------------------------------------------------------------------------
namespace {
bool fsep2_shape(const PyrGeom &G) {
  const int n0 = G.n[0], n1 = G.n[1];
  return G.M == 2 && ((n0 == 6 && n1 == 6) || (n0 == 4 && n1 == 4) || (n0 == 8 && n1 == 8) || (n0 == 8 && n1 == 4));
}
template <bool SEG, int LN>
const void *fsep2_fn_t(const PyrGeom &G) {
  return G.n[0] == 6 ? (const void *)k_fsep2<6, 6, SEG, LN>
         : G.n[0] == 4 ? (const void *)k_fsep2<4, 4, SEG, LN>
         : G.n[1] == 8 ? (const void *)k_fsep2<8, 8, SEG, LN>
                       : (const void *)k_fsep2<8, 4, SEG, LN>;
}
const void *fsep2_fn(const PyrGeom &G, const FsepPlan &p) {
  return p.S == 1 ? fsep2_fn_t<false, 2>(G) : p.lanes == 4 ? fsep2_fn_t<true, 4>(G) : fsep2_fn_t<true, 2>(G);
}
}  // namespace

bool fsep2_plan(const PyrGeom &G, int B, int S, FsepPlan *out) {
  if (!fsep2_shape(G) || B < 0 || S < 1) return false;
  const int L = G.n[0] * G.n[1], SMAX = G.n[0] + G.n[1] - 2, ND = SMAX + 1, FS = (L + 1) | 1, R = B + 1;
  FsepPlan p;
  p.S = S;
  if (S == 1) {
    p.lanes = 2;
    p.W = std::max(1, (R - 1 + 31) / 32);  // lane pairs for rows 0 .. 32W-1; row B beyond them is the extra row
    p.RS = 32 * p.W;
    p.rows = R;
  } else {
    // segments: four lanes per row (16 rows per wave) where the segment still fits one workgroup, else two
    p.lanes = 2;
    if (FSEP_LANES4 && G.n[0] % 2 == 0) {
      const int rs4 = 16 * std::max(1, (R - 1 + 16 * S - 1) / (16 * S));
      if (64 * (rs4 / 16) <= FS2_MAXT) p.lanes = 4;
    }
    const int rpw = 64 / p.lanes;
    p.RS = rpw * std::max(1, (R - 1 + rpw * S - 1) / (rpw * S));
    p.W = p.RS / rpw;
    if ((S - 1) * p.RS >= R || p.RS < SMAX + 1) return false;  // an empty last segment / a halo past the next one
    p.rows = std::min(R, p.RS + 1 + SMAX);
  }
  if (64 * p.W > FS2_MAXT) return false;
  p.koff = (p.rows * FS + 1) / 2 * 2;
  p.slot_bytes = (SMAX * L * 8 + 1023) / 1024 * 1024;
  const int dend = p.koff + L * ND + (L * L + 7) / 8;  // K table, then the distance bytes
  p.stg = (dend + 1) / 2 * 2;
  p.lds = (size_t)(S > 1 ? p.stg * 8 + p.slot_bytes : dend * 8);
  if (p.lds > 160 * 1024) return false;
  p.threads = 64 * p.W;
  if (out) *out = p;
  return true;
}

int fsep2_blocks_per_cu(const PyrGeom &G, const FsepPlan &p) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fsep2_fn(G, p), p.threads, p.lds) != hipSuccess) return 0;
  return n;
}

hipError_t launch_fsep2(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G, const FsepPlan &p,
                        double *front0, size_t front_stride, uint8_t *U, size_t u_stride_k, int32_t *counters,
                        double *ring, int NB, int32_t *flags, unsigned spin_limit) {
  if (P.M != 2 || !fsep2_shape(G)) return hipErrorInvalidValue;
  FsepArgs A;
  A.front0 = front0;
  A.front_stride = front_stride;
  A.U = U;
  A.u_stride_k = u_stride_k;
  A.counters = counters;
  A.ring = ring;
  A.flags = flags;
  A.S = p.S;
  A.RS = p.RS;
  A.NB = NB;
  A.koff = p.koff;
  A.stg = p.stg;
  A.slot_bytes = p.slot_bytes;
  A.spin_limit = spin_limit;
  A.base0 = G.base[0];
  A.base1 = G.base[1];
  ProblemDev Pc = P;
  LevelsDev Lc = Lv;
  const dim3 grid((unsigned)(P.K * p.S)), block((unsigned)p.threads);
  // S > 1: the segments of a subproblem wait for each other, so every workgroup must be resident -- the caller checks
  // the grid against the CUs x resident workgroups per CU (launch_fsep2 is not a cooperative launch: a cooperative
  // launch makes the HIP runtime tear down its cooperative-queue state at process exit, which crashed every
  // rocprofv3 run of round 3), and a dependency wait that times out makes the host redo the DP unsegmented
  void *args[] = {&Pc, &Lc, &A};
  return hipLaunchKernel(fsep2_fn(G, p), grid, block, args, p.lds, s);
}

#if defined(MIOC_STAMPS)
extern "C" int32_t mioc_debug_fsep_stamps(unsigned long long *out, int64_t nwaves) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fs_stamps), (size_t)nwaves * 8 * sizeof(unsigned long long)) ==
                 hipSuccess
             ? 0
             : -4;
}
#endif

}  // namespace mioc
