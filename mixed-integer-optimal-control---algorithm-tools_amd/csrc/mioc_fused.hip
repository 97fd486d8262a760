// mioc_fused.hip -- the fused small-state bellman_TRM! for gfx950: one workgroup per subproblem runs the whole
// DP (all nt - 1 recursion steps) in one launch, with the value front resident in LDS.  This is the batch
// path: 1024 random restarts of a 36-level problem are 1024 independent workgroups, four per
// CU in turn, and only the argmin table U (one byte per cell) and the final front leave the CU.
//
// Reference: HelpFunctions.jl:20-83 (bellman_TRM!).  Indices are 0-based.  Rounding order is the reference's
// (build with -ffp-contract=off):
//   T1  = ((0.0 + (Δt*df_1)*ν_1) + (Δt*df_2)*ν_2) + ...          HelpFunctions.jl:52-57
//   K   = T1 + β*w(l, j)                                             :60-67
//   val = K + Φ_{i+1}[c - b̃, j];  update iff Φ_i[c, l] > val         :69-76 (strict: the first j wins)
//
// LDS layout (one subproblem):
//   front  Φ[c][j]      (B+1) rows x FS doubles, FS = LP + 2 (odd count of 16-byte units: a wave's
//                       ds_read_b128 of 64 consecutive rows is conflict-free); updated IN PLACE each step
//   K[2][L][LP]         per-step K(l, j) = fl(T1(l) + β·w(l, j)) (+Inf for padding j >= L), double-buffered
//   bt[2][LP]           b̃(l, i), double-buffered
//   task[2][W*MAXT]     (row block, target) pairs with at least one target row inside the trust region
//
// Step i: every wave takes a contiguous share of the task list.  A task (rb, l) is one wave-uniform target l
// for the 64 source rows c' = 64·rb + lane: Ψ_j = Φ_{i+1}[c', j] sits in VGPRs (re-read only when the row
// block changes), K(l, ·) is broadcast from LDS, and the lane feeds target row c = c' + b̃(l).  Per candidate
// one v_add_f64 and one v_min_f64; the first minimising j is tracked per group of 4 and resolved exactly by
// re-reading the winning group.  The outputs stay in VGPRs until every wave has read its rows; then they are
// written into the front in place (Φ_i), and the U bytes to HBM.  Two barriers per step.
//
// HBM traffic per subproblem: df, u_old once, U = (nt-1)·L·(B+1) bytes, Φ_0 = L·(B+1)·8 bytes at the end.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mioc_internal.h"

namespace mioc {

constexpr int FU_W = 8;      // waves per workgroup (two per SIMD)
constexpr int FU_MAXT = 24;  // tasks per wave per step (host checks ceil(R/64)·L <= FU_W·FU_MAXT)
constexpr int FU_G = 4;      // argmin group

// Workgroup barrier for LDS hand-offs only: every wave drains its own LDS operations, then s_barrier.  A
// __syncthreads() would also wait for the wave's outstanding global stores (the U bytes, which nothing in the
// launch reads back), i.e. pay their full latency at every step.  The "memory" clobber keeps the compiler from
// moving LDS accesses across it.
__device__ __forceinline__ void fu_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// v_min_f64 without llvm.minnum's canonicalising v_max_f64 x,x on every operand (operands are finite or +Inf)
__device__ __forceinline__ double fu_min(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

struct FuLayout {
  int FS, R, nrb;
  size_t off_K, off_bt, off_task, off_cnt, off_nu, bytes;
};

__host__ __device__ inline FuLayout fu_layout(int LP, int L, int B) {
  FuLayout f;
  f.FS = LP + 2;
  f.R = B + 1;
  f.nrb = (f.R + 63) / 64;
  size_t o = (size_t)f.R * f.FS * sizeof(double);
  o = (o + 15) / 16 * 16;
  f.off_K = o;
  o += 2 * (size_t)L * LP * sizeof(double);
  f.off_bt = o;
  o += 2 * (size_t)LP * sizeof(int);
  f.off_task = o;
  o += 2 * (size_t)FU_W * FU_MAXT * sizeof(uint16_t);
  o = (o + 15) / 16 * 16;
  f.off_cnt = o;
  o += 16;
  f.off_nu = o;
  o += (size_t)L * kMaxM * sizeof(double);
  f.bytes = o;
  return f;
}

// b̃(l, i) and T1(l, i) from a[m] = Δt·df[m, i] and u_old[:, i] (HelpFunctions.jl:52-57)
__device__ __forceinline__ double fu_t1(const LevelsDev &Lv, int l, const double *a) {
  double t = 0.0;
  for (int m = 0; m < Lv.M; ++m) t = t + a[m] * Lv.nuval[l * Lv.M + m];
  return t;
}
__device__ __forceinline__ int fu_bt(const LevelsDev &Lv, int l, const double *uo) {
  int b = 0;  // saturated: far off-grid u_old entries only ever mean "beyond every budget"
  for (int m = 0; m < Lv.M; ++m) b += (int)fmin(fabs(Lv.nuval[l * Lv.M + m] - uo[m]), 1.0e8);
  return b;
}

// integer switching key of (l, j) (mioc_generic.hip) -> costlut; P_TABLE: the pair table
__device__ __forceinline__ double fu_cost(const LevelsDev &Lv, int l, int j) {
  if (Lv.p_kind == MIOC_P_TABLE) return Lv.costtab[(size_t)l * Lv.L + j];
  if (Lv.p_kind == MIOC_P_INF) return Lv.costlut[0];
  int key = 0;
  for (int m = 0; m < Lv.M; ++m) {
    int d = Lv.nuint[l * Lv.M + m] - Lv.nuint[j * Lv.M + m];
    d = d < 0 ? -d : d;
    if (Lv.p_kind == MIOC_P_ONE) {
      key += d;
    } else {
      int t = 1;
      for (int q = 0; q < Lv.p_int; ++q) t *= d;
      key += t;
    }
  }
  return Lv.costlut[key];
}

// Per-step tables for step s (K, b̃, task list) into buffer `buf`, from the step's Δt·df and u_old, which lane
// m of every wave holds (dfv, uov: loaded a step ahead).  Every thread recomputes the T1 / b̃ it needs, so no
// barrier separates the pieces.  cst: this thread's cached β·w(l, j) for the pairs e = tid + 512·q; nul: the
// level values [L][M] in LDS.
template <int LP, int NQ>
__device__ __forceinline__ void fu_prepare(const ProblemDev &P, const LevelsDev &Lv, double dfv, double uov,
                                           int buf, const double (&cst)[NQ], const double *nul, double *Kb,
                                           int *btb, uint16_t *taskb, int *cnt, const FuLayout &F) {
  const int tid = threadIdx.x, L = Lv.L, M = P.M;
  double a[kMaxM], uo[kMaxM];
  for (int m = 0; m < M; ++m) {
    a[m] = __shfl(dfv, m);
    uo[m] = __shfl(uov, m);
  }
  double *K = Kb + (size_t)buf * L * LP;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int e = tid + 512 * q;
    if (e < L * LP) {
      const int l = e / LP, j = e - l * LP;
      double t = 0.0;  // T1(l) = ((0 + (Δt·df_1)·ν_1) + ...), HelpFunctions.jl:52-57
      for (int m = 0; m < M; ++m) t = t + a[m] * nul[l * M + m];
      K[e] = j < L ? t + cst[q] : INFINITY;
    }
  }
  if (tid < 64) {  // wave 0: b̃ and the compacted task list (row block major, target ascending)
    const int lane = tid;
    int b = 1 << 29;
    if (lane < L) {
      b = 0;  // saturated: far off-grid u_old entries only ever mean "beyond every budget"
      for (int m = 0; m < M; ++m) b += (int)fmin(fabs(nul[lane * M + m] - uo[m]), 1.0e8);
    }
    if (lane < LP) btb[buf * LP + lane] = b;
    int n = 0;
    uint16_t *tl = taskb + buf * (FU_W * FU_MAXT);
    for (int rb = 0; rb < F.nrb; ++rb) {
      const bool v = lane < L && 64 * rb + b <= P.B;
      const unsigned long long mk = __ballot(v);
      if (v) tl[n + __popcll(mk & ((1ull << lane) - 1))] = (uint16_t)(rb << 8 | lane);
      n += __popcll(mk);
    }
    if (lane == 0) cnt[buf] = n;
  }
}

// lane m < M: Δt·df[m, s] and u_old[m, s] (one load each, in flight until fu_prepare)
__device__ __forceinline__ void fu_fetch(const ProblemDev &P, int k, int s, double &dfv, double &uov) {
  const int lane = threadIdx.x & 63;
  dfv = 0.0;
  uov = 0.0;
  if (lane < P.M) {
    dfv = P.dt * P.df[((size_t)k * P.nt + s) * P.M + lane];
    uov = P.uold[((size_t)k * P.nt + s) * P.M + lane];
  }
}

#if defined(MIOC_STAMPS)
// diagnostic build: cycles per phase summed over the steps, per workgroup (wave 0's view)
__device__ unsigned long long g_fu_stamps[4096][8];
#define FU_T(v) unsigned long long v = ((threadIdx.x & 63) == 0) ? __builtin_amdgcn_s_memtime() : 0ull
#define FU_ACC(q, a, b) \
  if ((threadIdx.x & 63) == 0) acc[q] += (b) - (a)
#else
#define FU_T(v) \
  do {          \
  } while (0)
#define FU_ACC(q, a, b) \
  do {                  \
  } while (0)
#endif

template <int LP>
__global__ __launch_bounds__(512) void k_fused_run(ProblemDev P, LevelsDev Lv, double *__restrict__ front0_all,
                                                   size_t front_stride, uint8_t *__restrict__ U_all,
                                                   size_t u_stride_k) {
  extern __shared__ __attribute__((aligned(16))) unsigned char fsm[];
  constexpr int NQ = (LP * LP + 511) / 512;  // cached cost pairs per thread (L <= LP)
  const int k = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int L = Lv.L, B = P.B, nt = P.nt;
  const FuLayout F = fu_layout(LP, L, B);
  const int FS = F.FS, R = F.R;
  double *front = reinterpret_cast<double *>(fsm);
  double *Kb = reinterpret_cast<double *>(fsm + F.off_K);
  int *btb = reinterpret_cast<int *>(fsm + F.off_bt);
  uint16_t *taskb = reinterpret_cast<uint16_t *>(fsm + F.off_task);
  int *cnt = reinterpret_cast<int *>(fsm + F.off_cnt);
  double *nul = reinterpret_cast<double *>(fsm + F.off_nu);
  for (int e = tid; e < L * P.M; e += 512) nul[e] = Lv.nuval[e];
#if defined(MIOC_STAMPS)
  unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif

  double cst[NQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int e = tid + 512 * q, l = e / LP, j = e - l * LP;
    cst[q] = (e < L * LP && j < L) ? fu_cost(Lv, l, j) : 0.0;
  }
  // ---- terminal step (HelpFunctions.jl:27-43): Φ_{n-1}[c, l] = T1(l, n-1) at c = b̃(l, n-1) <= B, else +Inf
  {
    const double *dfs = P.df + ((size_t)k * nt + nt - 1) * P.M;
    const double *uos = P.uold + ((size_t)k * nt + nt - 1) * P.M;
    double a[kMaxM], uo[kMaxM];
    for (int m = 0; m < P.M; ++m) {
      a[m] = P.dt * dfs[m];
      uo[m] = uos[m];
    }
    for (int e = tid; e < R * LP; e += 512) {
      const int c = e / LP, l = e - c * LP;
      double v = INFINITY;
      if (l < L && fu_bt(Lv, l, uo) == c) v = fu_t1(Lv, l, a);
      front[c * FS + l] = v;
    }
  }
  double dfv, uov;
  __syncthreads();  // nul
  if (nt >= 2) {
    fu_fetch(P, k, nt - 2, dfv, uov);
    fu_prepare<LP, NQ>(P, Lv, dfv, uov, (nt - 2) & 1, cst, nul, Kb, btb, taskb, cnt, F);
  }
  __syncthreads();

  uint8_t *Uk = U_all + (size_t)k * u_stride_k;
#pragma nounroll
  for (int i = nt - 2; i >= 0; --i) {
    const int cur = i & 1;
    const double *K = Kb + (size_t)cur * L * LP;
    const uint16_t *tl = taskb + cur * (FU_W * FU_MAXT);
    const int V = __builtin_amdgcn_readfirstlane(cnt[cur]);
    const int t0 = (w * V) / FU_W, t1 = ((w + 1) * V) / FU_W;
    const int *bt = btb + cur * LP;
    uint8_t *Ui = Uk + (size_t)i * ((size_t)L * R);
    if (i >= 1) fu_fetch(P, k, i - 1, dfv, uov);  // the next step's inputs, consumed after this step's tasks
    FU_T(s0);
    double ov[FU_MAXT];
    double psi[LP];
    int cur_rb = -1;
    // ---- compute: every task of this wave, outputs kept in registers -----------------------------------
#pragma unroll
    for (int t = 0; t < FU_MAXT; ++t) {
      ov[t] = INFINITY;
      if (t0 + t < t1) {
        const int task = __builtin_amdgcn_readfirstlane((int)tl[t0 + t]);
        const int rb = task >> 8, l = task & 255;
        const int cp = 64 * rb + lane;
        if (rb != cur_rb) {
          cur_rb = rb;
          if (cp < R) {
            const double2 *row = reinterpret_cast<const double2 *>(front + cp * FS);
#pragma unroll
            for (int q = 0; q < LP / 2; ++q) {
              const double2 x = row[q];
              psi[2 * q] = x.x;
              psi[2 * q + 1] = x.y;
            }
          } else {
#pragma unroll
            for (int q = 0; q < LP; ++q) psi[q] = INFINITY;
          }
        }
        const double2 *Kl = reinterpret_cast<const double2 *>(K + l * LP);
        double best = INFINITY;
        int bg = -1;
#pragma unroll
        for (int g = 0; g < LP / FU_G; ++g) {
          const double2 k0 = Kl[2 * g], k1 = Kl[2 * g + 1];
          const double gm = fu_min(fu_min(k0.x + psi[4 * g], k0.y + psi[4 * g + 1]),
                                   fu_min(k1.x + psi[4 * g + 2], k1.y + psi[4 * g + 3]));
          if (gm < best) bg = g;
          best = fu_min(best, gm);
        }
        int arg = 0xFF;
        if (bg >= 0) {  // the first j of the winning group attaining the minimum (exact re-evaluation)
          const double2 *row = reinterpret_cast<const double2 *>(front + cp * FS + FU_G * bg);
          const double2 p0 = row[0], p1 = row[1], q0 = Kl[2 * bg], q1 = Kl[2 * bg + 1];
          const int j0 = FU_G * bg;
          arg = q1.y + p1.y == best ? j0 + 3 : arg;
          arg = q1.x + p1.x == best ? j0 + 2 : arg;
          arg = q0.y + p0.y == best ? j0 + 1 : arg;
          arg = q0.x + p0.x == best ? j0 : arg;
        }
        ov[t] = best;
        const int c = cp + bt[l];  // U goes to HBM at once; the value waits for the barrier
        if (c <= B && best < INFINITY) Ui[(size_t)l * R + c] = (uint8_t)arg;
      }
    }
    FU_T(s1);
    if (i >= 1) fu_prepare<LP, NQ>(P, Lv, dfv, uov, (i - 1) & 1, cst, nul, Kb, btb, taskb, cnt, F);
    FU_T(s2);
    fu_lds_barrier();  // every wave has read its rows of Φ_{i+1}: the front may be overwritten
    FU_T(s3);
    // ---- write Φ_i in place --------------------------------------------------------------------------------
#pragma unroll
    for (int t = 0; t < FU_MAXT; ++t) {
      if (t0 + t < t1) {
        const int task = __builtin_amdgcn_readfirstlane((int)tl[t0 + t]);
        const int rb = task >> 8, l = task & 255;
        const int c = 64 * rb + lane + bt[l];
        if (c <= B) front[c * FS + l] = ov[t];
      }
    }
    // cells below the target's own budget class are unreachable: Φ_i[c, l] = +Inf for c < b̃(l, i)
    for (int l = w; l < L; l += FU_W) {
      const int b = min(bt[l], R);
      for (int c = lane; c < b; c += 64) front[c * FS + l] = INFINITY;
    }
    FU_T(s4);
    fu_lds_barrier();
    FU_T(s5);
    FU_ACC(0, s0, s1);
    FU_ACC(1, s1, s2);
    FU_ACC(2, s2, s3);
    FU_ACC(3, s3, s4);
    FU_ACC(4, s4, s5);
  }
#if defined(MIOC_STAMPS)
  if (tid == 0)
    for (int q = 0; q < 8; ++q) g_fu_stamps[k & 4095][q] = acc[q];
#endif
  // ---- Φ_0 to HBM in the generic layout [L][RP] (the backtrack's argmin reads it) ------------------------
  double *f0 = front0_all + (size_t)k * front_stride;
  for (int e = tid; e < L * P.RP; e += 512) {
    const int l = e / P.RP, c = e - l * P.RP;
    f0[e] = c < R ? front[c * FS + l] : INFINITY;
  }
}

// ==============================================================================================================
// p = 1 on a 2-D product grid of consecutive integer levels (N0 x N1 <= 8 x 8): the same fused DP with the
// separable L1 transform of mioc_sdt.hip in place of the min-plus sweep, entirely in registers.
//
// Lane = source row c' (one wave per 64 rows, the whole workgroup one subproblem).  The lane's row Ψ_j =
// Φ_{i+1}[c', j] (all L sources) sits in VGPRs, so the two passes of the transform (forward and backward along
// x0, then along x1) are register-to-register: 2·(N1·2(N0-1) + N0·2(N1-1)) merges per row.  Exact fixed point as
// in mioc_sdt.hip: V_j = trunc_g(base + (Ψ_j - Ψmin)/β) with the source coordinates x0 | x1 << 3 in the 6 low
// mantissa bits and bit 6 as the near-tie flag (g = 2^7 ulp(base)); a unit step costs exactly 1.0; a merge of two
// candidate sets whose values differ by <= tol sets the flag.  An unflagged winner j* beats every other source by
// more than tol, so it is the reference's unique argmin and the output is R(l, j*) = fl(fl(T1_l + fl(β·d)) + Ψ_j*)
// evaluated with the reference's expression (K_l[d] = fl(T1_l + fl(β·d)) is a per-step table).  Flagged targets,
// rows whose value range leaves the binade, and waves whose rows have at most FSP_FEW targets each run the
// reference loop (HelpFunctions.jl:60-77) exactly.  Results are bit-identical to the reference in every case.
// ==============================================================================================================
constexpr int FSP_FLAG = 64;       // near-tie flag (payload bit 6)
constexpr int FSP_FEW_PAIRS = 8;   // a wave with at most this many (row, target) pairs scans them exactly



__device__ __forceinline__ double fsp_merge(double a, double t, double tol) {
  const double m = fu_min(a, t);
  const bool close = fabs(a - t) <= tol;
  return __hiloint2double(__double2hiint(m), __double2loint(m) | (close ? FSP_FLAG : 0));
}

struct FspLayout {
  int FS, ND;
  size_t off_f1, off_K, bytes;
};
__host__ __device__ inline FspLayout fsp_layout(int N0, int N1, int B) {
  FspLayout f;
  const int L = N0 * N1;
  f.FS = (L + 1) | 1;  // odd row stride (8-byte words, a pad column at index L): a wave's ds_read_b64 /
                       // ds_write_b64 of 64 rows is conflict-free
  f.ND = N0 + N1 - 1;
  size_t o = (size_t)(B + 1) * f.FS * sizeof(double);
  o = (o + 15) / 16 * 16;
  f.off_f1 = o;  // the second front buffer
  o += (size_t)(B + 1) * f.FS * sizeof(double);
  o = (o + 15) / 16 * 16;
  f.off_K = o;  // K_l[d], double-buffered by step parity
  o += 2 * (size_t)L * f.ND * sizeof(double);
  f.bytes = (o + 15) / 16 * 16;
  return f;
}

// b̃(l) = |ν0(l) - u0| + |ν1(l) - u1| for the integer u_old coordinates of the step (clamped: a far off-grid
// entry only ever means "beyond every budget"); wave-uniform, so it lives in SGPRs
__device__ __forceinline__ int fsp_uint(double u) { return (int)fmin(fmax(u, -1.0e8), 1.0e8); }

// Double-buffered front (Φ_{i+1} read, Φ_i written), so every output goes to LDS the moment it is known and
// a step needs one barrier; one workgroup per CU (the two fronts fill its LDS).
template <int N0, int N1>
__global__ __launch_bounds__(512, 2) void k_fsep_run(ProblemDev P, LevelsDev Lv, int base0, int base1,
                                                     double *__restrict__ front0_all, size_t front_stride,
                                                     uint8_t *__restrict__ U_all, size_t u_stride_k,
                                                     int32_t *__restrict__ counters) {
  constexpr int L = N0 * N1, SMAX = N0 + N1 - 2;
  constexpr int FS = (L + 1) | 1, ND = SMAX + 1;  // odd row stride with a pad column (index L)
  extern __shared__ __attribute__((aligned(16))) unsigned char fsm[];
  const int k = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6, nthr = blockDim.x;
  const int nw = nthr >> 6;
  const int B = P.B, R = B + 1, nt = P.nt;
  const FspLayout F = fsp_layout(N0, N1, B);
  // (pointer arithmetic on the LDS array itself -- a pointer picked from a private array would lose the LDS
  // address space and turn every front access into a flat load / store)
  double *const fbase = reinterpret_cast<double *>(fsm);
  const int f1off = (int)(F.off_f1 / sizeof(double));
  double *Ktb = reinterpret_cast<double *>(fsm + F.off_K);
  const int cp = 64 * w + lane;
  const bool act = cp < R;
  const int room = act ? B - cp : -1;   // target l is inside the trust region iff b̃_l <= room
  const int cps = act ? cp : 0;         // rows past B read row 0: they have no targets
  const int padw = (act ? cp : cp % R) * FS + L;  // this lane's pad slot: the target of a masked-off write
  const double beta = Lv.beta, inv = Lv.inv_beta;
  // |T1| bound over the step's targets is folded into qmax per step: Σ_m |a_m|·max|ν_m|
  const double numx0 = (double)max(abs(base0), abs(base0 + N0 - 1)),
               numx1 = (double)max(abs(base1), abs(base1 + N1 - 1));
  const bool prep_wave = w == nw - 1;  // the last wave (the fewest rows) builds the per-step table

  // per-step table, HelpFunctions.jl:52-67: K_l[d] = fl(T1(l) + fl(β·d)), double-buffered by step parity
  auto prepare = [&](double a0, double a1, int buf) {
    double *K = Ktb + buf * (L * ND);
    for (int e = lane; e < L * ND; e += 64) {
      const int l = e / ND, d = e - l * ND;
      const double t1 = (0.0 + a0 * (double)(base0 + l % N0)) + a1 * (double)(base1 + l / N0);
      K[e] = t1 + beta * (double)d;
    }
  };
  auto inputs = [&](int s, double &a0, double &a1, double &u0, double &u1) {
    const double *dfs = P.df + ((size_t)k * nt + s) * 2;
    const double *uos = P.uold + ((size_t)k * nt + s) * 2;
    a0 = P.dt * dfs[0];
    a1 = P.dt * dfs[1];
    u0 = uos[0];
    u1 = uos[1];
  };
  // ---- terminal step (HelpFunctions.jl:27-43) into the buffer step nt-2 reads ------------------------------
  double ca0 = 0.0, ca1 = 0.0;  // Δt·df of the current step (the tolerance's |T1| bound)
  int cu0 = 0, cu1 = 0;         // u_old of the current step (integer coordinates, b̃)
  {
    double a0, a1, u0, u1;
    inputs(nt - 1, a0, a1, u0, u1);
    const int iu0 = fsp_uint(u0), iu1 = fsp_uint(u1);
    double *ft = fbase + ((nt - 1) & 1) * f1off;
    for (int e = tid; e < R * FS; e += nthr) {
      const int c = e / FS, l = e - c * FS;
      double v = INFINITY;
      if (l < L && abs(base0 + l % N0 - iu0) + abs(base1 + l / N0 - iu1) == c)
        v = (0.0 + a0 * (double)(base0 + l % N0)) + a1 * (double)(base1 + l / N0);
      ft[e] = v;
    }
    if (nt >= 2) {
      inputs(nt - 2, a0, a1, u0, u1);
      if (prep_wave) prepare(a0, a1, (nt - 2) & 1);
      ca0 = a0;
      ca1 = a1;
      cu0 = fsp_uint(u0);
      cu1 = fsp_uint(u1);
    }
  }
  __syncthreads();
  uint8_t *Uk = U_all + (size_t)k * u_stride_k;
  int nflag = 0, nscan = 0;
#if defined(MIOC_STAMPS)
  unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
#pragma nounroll
  for (int i = nt - 2; i >= 0; --i) {
    const double *fin_ = fbase + ((i + 1) & 1) * f1off;  // Φ_{i+1}
    double *fout = fbase + (i & 1) * f1off;               // Φ_i
    const double *Kt = Ktb + (i & 1) * (L * ND);
    // b̃ of every target, in SGPRs for the whole step
    const int su0 = __builtin_amdgcn_readfirstlane(cu0), su1 = __builtin_amdgcn_readfirstlane(cu1);
    auto btof = [&](int l) { return abs(base0 + l % N0 - su0) + abs(base1 + l / N0 - su1); };
    // U_i[l][c] through a buffer resource: 32-bit offsets (no per-target 64-bit address arithmetic for the
    // compiler to hoist into VGPRs), bounds-checked to the step's L·R bytes: a store at an offset past them is
    // dropped, which makes every U store branch-free
    const __amdgpu_buffer_rsrc_t Ur =
        __builtin_amdgcn_make_buffer_rsrc(Uk + (size_t)i * ((size_t)L * R), 0, L * R, 0x00020000);
    double na0 = 0.0, na1 = 0.0, nu0 = 0.0, nu1 = 0.0;
    if (i >= 1) inputs(i - 1, na0, na1, nu0, nu1);  // the next step's inputs
    FU_T(q0);
    unsigned long long scan = 0;  // targets resolved by the exact scan
    // (row, target) pairs of this wave inside the trust region: a wave with very few (the rows next to B)
    // resolves them all by exact scans instead of running the transform
    int npairs = 0;
#pragma unroll
    for (int l = 0; l < L; ++l) npairs += min(max(B - 64 * w - btof(l) + 1, 0), 64);
    if (npairs <= FSP_FEW_PAIRS) {
#pragma unroll
      for (int l = 0; l < L; ++l) scan |= (unsigned long long)((unsigned)(btof(l) - room - 1) >> 31) << l;
    } else {
    // ---- this lane's row of Φ_{i+1} -----------------------------------------------------------------------
    double o[L];
#pragma unroll
    for (int j = 0; j < L; ++j) o[j] = fin_[cps * FS + j];
    const double a0 = ca0, a1 = ca1;
    // ---- row statistics over the finite sources ------------------------------------------------------------
    double pmn = o[0], pmx = o[0];
#pragma unroll
    for (int j = 1; j < L; ++j) {
      pmn = fu_min(pmn, o[j]);
      pmx = fmax(pmx, o[j]);
    }
    const bool infrow = !(pmx < INFINITY);
    if (__ballot(infrow && pmn < INFINITY)) {  // some sources unreachable: the maximum over the finite ones
      pmx = pmn;
#pragma unroll
      for (int j = 0; j < L; ++j) pmx = fmax(pmx, o[j] < INFINITY ? o[j] : pmn);
    }
    // ---- the binade: values base + (Ψ - Ψmin)/β + d lie in [base, 2·base), grid g = 2^7 ulp(base) ---------
    const double rs = (pmx - pmn) * inv + (double)SMAX;
    const bool scale_ok = rs < 0x1p36;
    const int E = ilogb(fmin(rs, 0x1p36) * (1.0 + 0x1p-20) + 1.0) + 2;
    const double base = ldexp(1.0, E), g = ldexp(1.0, E - 45);
    const double qmax = beta * (double)SMAX + fmax(fabs(pmn), fabs(pmx)) + fabs(a0) * numx0 + fabs(a1) * numx1;
    // 2 x stamping error (< g) + 2 x the reference's rounding (<= 4u·qmax per candidate), in units of β
    const double tol = 3.0 * g + 0x1p-49 * qmax * inv;
    const bool none = !(pmn < INFINITY);
    const bool direct = !none && !(scale_ok && tol < 0.25);
    if (none) pmn = 0.0;  // every source +Inf: stamps stay +Inf (no NaN), payload 0
    // ---- stamp: V_j = trunc_g(base + (Ψ_j - Ψmin)/β) | x0 | x1 << 3 -------------------------------------------
    const bool anyinf = __ballot(infrow) != 0;
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const double y = (o[j] - pmn) * inv + base;
      const int hi = __double2hiint(y);
      int lo = (__double2loint(y) & ~(2 * FSP_FLAG - 1)) | ((j % N0) | (j / N0) << 3);
      if (anyinf) lo = hi == 0x7FF00000 ? 0 : lo;  // +Inf stays +Inf (payload bits would make it a NaN)
      o[j] = __hiloint2double(hi, lo);
    }
    FU_T(q1);
    FU_ACC(0, q0, q1);
    // ---- pass over x0 (lines of N0 along each x1), then over x1 --------------------------------------------
#pragma unroll
    for (int x1 = 0; x1 < N1; ++x1) {
#pragma unroll
      for (int x0 = 1; x0 < N0; ++x0)
        o[x1 * N0 + x0] = fsp_merge(o[x1 * N0 + x0], o[x1 * N0 + x0 - 1] + 1.0, tol);
#pragma unroll
      for (int x0 = N0 - 2; x0 >= 0; --x0)
        o[x1 * N0 + x0] = fsp_merge(o[x1 * N0 + x0], o[x1 * N0 + x0 + 1] + 1.0, tol);
    }
#pragma unroll
    for (int x0 = 0; x0 < N0; ++x0) {
#pragma unroll
      for (int x1 = 1; x1 < N1; ++x1)
        o[x1 * N0 + x0] = fsp_merge(o[x1 * N0 + x0], o[(x1 - 1) * N0 + x0] + 1.0, tol);
#pragma unroll
      for (int x1 = N1 - 2; x1 >= 0; --x1)
        o[x1 * N0 + x0] = fsp_merge(o[x1 * N0 + x0], o[(x1 + 1) * N0 + x0] + 1.0, tol);
    }
    FU_T(q2);
    FU_ACC(1, q1, q2);
    // ---- targets: Φ_i[c' + b̃_l, l] = R(l, j*) = fl(fl(T1_l + fl(β·d)) + Ψ_j*) for the winner j*, written at once
    // with U (a target outside the trust region writes the lane's pad slot).  Flags are only OR-ed here; a
    // flagged target, or any target of a row outside the binade, is rewritten by the exact scan below (same
    // wave, program order, for the LDS cell and for the U byte) -----------------------------------------------
    int flagacc = 0;
    const int cpFS = cp * FS;
#pragma unroll
    for (int x1 = 0; x1 < N1; ++x1) {  // one grid line of N0 targets: its 2·N0 LDS gathers issue together
      double kv[N0], pv[N0];
      int jv[N0];
#pragma unroll
      for (int x0 = 0; x0 < N0; ++x0) {
        const int l = x1 * N0 + x0;
        const int lo = __double2loint(o[l]);
        const unsigned pb = (unsigned)(lo & 7) | ((unsigned)(lo & 0x38) << 5);  // x0, x1 one byte each
        jv[x0] = (lo & 7) + N0 * ((unsigned)(lo >> 3) & 7u);
        const int d = (int)__builtin_amdgcn_sad_u8(pb, (unsigned)(x0 | x1 << 8), 0u);
        kv[x0] = Kt[l * ND + d];
        pv[x0] = fin_[cps * FS + jv[x0]];
      }
#pragma unroll
      for (int x0 = 0; x0 < N0; ++x0) {
        const int l = x1 * N0 + x0;
        const int b = btof(l);
        const bool valid = b <= room;
        const bool ok = valid && o[l] < INFINITY;
        flagacc |= __double2loint(o[l]);
        fout[valid ? cpFS + (b * FS + l) : padw] = ok ? kv[x0] + pv[x0] : INFINITY;
        __builtin_amdgcn_raw_buffer_store_b8((unsigned char)jv[x0], Ur, ok ? cp + b : 0x40000000, l * R, 0);
      }
    }
    if (__ballot(!none && (direct || (flagacc & FSP_FLAG)))) {  // rare: list the targets for the exact scan
      const unsigned lanemode = none ? 0u : (direct ? 1u : 2u);
#pragma unroll
      for (int l = 0; l < L; ++l) {
        const unsigned valid = (unsigned)(btof(l) - room - 1) >> 31;
        const int lo = __double2loint(o[l]);
        const unsigned fin = valid & (lanemode >> 1) & (unsigned)(o[l] < INFINITY);
        const unsigned flg = ((unsigned)lo >> 6) & 1u;
        scan |= (unsigned long long)((valid & (lanemode & 1u)) | (fin & flg)) << l;
      }
      nflag += lanemode == 2u ? __popcll(scan) : 0;
    }
    FU_T(q3i);
    FU_ACC(2, q2, q3i);
    }
    FU_T(q3);
    nscan += __popcll(scan);
    // ---- exact scans, one (row, target) pair at a time across the wave: lane j evaluates source j with the
    // reference's expression (HelpFunctions.jl:60-77), then a (value, rank) minimum over the lanes, ties to the
    // lower rank -----------------------------------------------------------------------------------------------
    if (__ballot(scan != 0)) {
#pragma unroll 1
      for (int l = 0; l < L; ++l) {
        unsigned long long rows = __ballot((scan >> l) & 1);
        if (rows) {
          const int dj = abs(lane % N0 - l % N0) + abs(lane / N0 - l / N0);
          const double kl = lane < L ? Kt[l * ND + min(dj, SMAX)] : INFINITY;
          const int bl = abs(base0 + l % N0 - su0) + abs(base1 + l / N0 - su1);
          while (rows) {
            const int r = __builtin_ctzll(rows);
            rows &= rows - 1;
            const int rowr = 64 * w + r;  // the source row of lane r
            double bv = lane < L ? kl + fin_[rowr * FS + min(lane, L - 1)] : INFINITY;
            int bj = lane < L && bv < INFINITY ? lane : 0xFF;
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) {
              const double ov = __shfl_xor(bv, off);
              const int oj = __shfl_xor(bj, off);
              if (ov < bv || (ov == bv && oj < bj)) {
                bv = ov;
                bj = oj;
              }
            }
            if (lane == 0) {
              fout[(rowr + bl) * FS + l] = bv;
              __builtin_amdgcn_raw_buffer_store_b8((unsigned char)bj, Ur, bv < INFINITY ? rowr + bl : 0x40000000,
                                                   l * R, 0);
            }
          }
        }
      }
    }
    // ---- cells below the target's own budget class: +Inf (target l by wave l % nw) ------------------------
#pragma unroll 1
    for (int l = w; l < L; l += nw) {
      const int b = min(btof(l), R);
      for (int c = lane; c < b; c += 64) fout[c * FS + l] = INFINITY;
    }
    if (i >= 1 && prep_wave) prepare(na0, na1, (i - 1) & 1);
    ca0 = na0;
    ca1 = na1;
    cu0 = fsp_uint(nu0);
    cu1 = fsp_uint(nu1);
    FU_T(q5);
    FU_ACC(3, q3, q5);
    fu_lds_barrier();  // Φ_i complete: the next step reads it
    FU_T(q6);
    FU_ACC(4, q5, q6);
    FU_ACC(7, q0, q6);
  }
#if defined(MIOC_STAMPS)
  if (lane == 0)  // per wave: block k, wave w at (8k + w) mod 4096
    for (int q = 0; q < 8; ++q) g_fu_stamps[(8 * k + w) & 4095][q] = acc[q];
#endif
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    nflag += __shfl_xor(nflag, off);
    nscan += __shfl_xor(nscan, off);
  }
  if (lane == 0 && (nflag | nscan)) {  // diagnostics: [0] near-tie targets, [1] targets of rows out of the binade
    atomicAdd(&counters[0], nflag);
    atomicAdd(&counters[1], nscan - nflag);
  }
  // ---- Φ_0 to HBM in the generic layout [L][RP] (the backtrack's argmin reads it) --------------------------
  const double *f0s = fbase;
  double *f0 = front0_all + (size_t)k * front_stride;
  for (int e = tid; e < L * P.RP; e += nthr) {
    const int l = e / P.RP, c = e - l * P.RP;
    f0[e] = c < R ? f0s[c * FS + l] : INFINITY;
  }
}

bool fsep_supported(const PyrGeom &G, int B, size_t *lds_out, int *threads_out) {
  if (G.M != 2 || B < 0 || B + 1 > 512) return false;
  const int n0 = G.n[0], n1 = G.n[1];
  const bool shape = (n0 == 6 && n1 == 6) || (n0 == 4 && n1 == 4) || (n0 == 8 && n1 == 8) || (n0 == 8 && n1 == 4);
  if (!shape) return false;
  const FspLayout F = fsp_layout(n0, n1, B);
  if (F.bytes > 160 * 1024) return false;
  if (lds_out) *lds_out = F.bytes;
  if (threads_out) *threads_out = 64 * ((B + 1 + 63) / 64);
  return true;
}

int fused_blocks_per_cu(int algo_sep, const PyrGeom &G, int L, int B) {
  int n = 0;
  size_t lds = 0;
  int thr = 512;
  if (algo_sep) {
    if (!fsep_supported(G, B, &lds, &thr)) return 0;
    const void *f = G.n[0] == 6 ? (const void *)k_fsep_run<6, 6> : G.n[0] == 4 ? (const void *)k_fsep_run<4, 4>
                    : G.n[1] == 8 ? (const void *)k_fsep_run<8, 8> : (const void *)k_fsep_run<8, 4>;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, thr, lds) != hipSuccess) return 0;
  } else {
    if (!fused_supported(L, B, &lds)) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void *)k_fused_run<36>, 512, lds) != hipSuccess) return 0;
  }
  return n;
}

hipError_t launch_fsep_run(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G, double *front0,
                           size_t front_stride, uint8_t *U, size_t u_stride_k, int32_t *counters) {
  size_t lds = 0;
  int thr = 0;
  if (!fsep_supported(G, P.B, &lds, &thr)) return hipErrorInvalidValue;
  if (P.M != 2) return hipErrorInvalidValue;
#define FSP_LAUNCH(A, Bv)                                                                                          \
  hipLaunchKernelGGL((k_fsep_run<A, Bv>), dim3(P.K), dim3(thr), lds, s, P, Lv, G.base[0], G.base[1], front0,       \
                     front_stride, U, u_stride_k, counters)
  if (G.n[0] == 6)
    FSP_LAUNCH(6, 6);
  else if (G.n[0] == 4)
    FSP_LAUNCH(4, 4);
  else if (G.n[1] == 8)
    FSP_LAUNCH(8, 8);
  else
    FSP_LAUNCH(8, 4);
#undef FSP_LAUNCH
  return hipGetLastError();
}

bool fused_supported(int L, int B, size_t *lds_out) {
  if (L < 1 || L > 64 || B < 0) return false;
  const int LP = L <= 4 ? 4 : L <= 8 ? 8 : L <= 16 ? 16 : L <= 24 ? 24 : L <= 32 ? 32 : L <= 36 ? 36 : L <= 48 ? 48 : 64;
  const FuLayout F = fu_layout(LP, L, B);
  if ((size_t)F.nrb * L > (size_t)FU_W * FU_MAXT) return false;
  if (F.bytes > 160 * 1024) return false;
  if (lds_out) *lds_out = F.bytes;
  return true;
}

hipError_t launch_fused_run(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, double *front0,
                            size_t front_stride, uint8_t *U, size_t u_stride_k) {
  size_t lds = 0;
  if (!fused_supported(Lv.L, P.B, &lds)) return hipErrorInvalidValue;
  const int L = Lv.L;
#define FU_LAUNCH(LPV)                                                                                     \
  hipLaunchKernelGGL(k_fused_run<LPV>, dim3(P.K), dim3(512), lds, s, P, Lv, front0, front_stride, U, u_stride_k)
  if (L <= 4)
    FU_LAUNCH(4);
  else if (L <= 8)
    FU_LAUNCH(8);
  else if (L <= 16)
    FU_LAUNCH(16);
  else if (L <= 24)
    FU_LAUNCH(24);
  else if (L <= 32)
    FU_LAUNCH(32);
  else if (L <= 36)
    FU_LAUNCH(36);
  else if (L <= 48)
    FU_LAUNCH(48);
  else
    FU_LAUNCH(64);
#undef FU_LAUNCH
  return hipGetLastError();
}

#if defined(MIOC_STAMPS)
extern "C" int32_t mioc_debug_fused_stamps(unsigned long long *out, int64_t nblocks) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fu_stamps), (size_t)nblocks * 8 * sizeof(unsigned long long)) ==
                 hipSuccess
             ? 0
             : -4;
}
#endif

}  // namespace mioc
