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

// v_min_f64 without llvm.minnum's canonicalising v_max_f64 x,x on every operand (operands are finite or +Inf)
__device__ __forceinline__ double fu_min(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

struct FuLayout {
  int FS, R, nrb;
  size_t off_K, off_bt, off_task, off_cnt, bytes;
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

// Per-step tables for step s (K, b̃, task list) into buffer `buf`.  Every thread recomputes the T1 / b̃ it needs
// from the step's df / u_old (broadcast loads), so no barrier separates the pieces.  cst: this thread's cached
// β·w(l, j) for the pairs e = tid + 512·q.
template <int LP, int NQ>
__device__ __forceinline__ void fu_prepare(const ProblemDev &P, const LevelsDev &Lv, int k, int s, int buf,
                                           const double (&cst)[NQ], double *Kb, int *btb, uint16_t *taskb,
                                           int *cnt, const FuLayout &F) {
  const int tid = threadIdx.x, L = Lv.L, M = P.M;
  const double *dfs = P.df + ((size_t)k * P.nt + s) * M;
  const double *uos = P.uold + ((size_t)k * P.nt + s) * M;
  double a[kMaxM], uo[kMaxM];
  for (int m = 0; m < M; ++m) {
    a[m] = P.dt * dfs[m];
    uo[m] = uos[m];
  }
  double *K = Kb + (size_t)buf * L * LP;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int e = tid + 512 * q;
    if (e < L * LP) {
      const int l = e / LP, j = e - l * LP;
      K[e] = j < L ? fu_t1(Lv, l, a) + cst[q] : INFINITY;
    }
  }
  if (tid < 64) {  // wave 0: b̃ and the compacted task list (row block major, target ascending)
    const int lane = tid;
    int b = 1 << 29;
    if (lane < L) b = fu_bt(Lv, lane, uo);
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
  if (nt >= 2) fu_prepare<LP, NQ>(P, Lv, k, nt - 2, (nt - 2) & 1, cst, Kb, btb, taskb, cnt, F);
  __syncthreads();

  uint8_t *Uk = U_all + (size_t)k * u_stride_k;
#pragma nounroll
  for (int i = nt - 2; i >= 0; --i) {
    const int cur = i & 1;
    const double *K = Kb + (size_t)cur * L * LP;
    const uint16_t *tl = taskb + cur * (FU_W * FU_MAXT);
    const int V = __builtin_amdgcn_readfirstlane(cnt[cur]);
    const int t0 = (w * V) / FU_W, t1 = ((w + 1) * V) / FU_W;
    double ov[FU_MAXT];
    int oa[FU_MAXT];
    double psi[LP];
    int cur_rb = -1;
    // ---- compute: every task of this wave, outputs kept in registers -----------------------------------
#pragma unroll
    for (int t = 0; t < FU_MAXT; ++t) {
      ov[t] = INFINITY;
      oa[t] = 0xFF;
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
        oa[t] = arg;
      }
    }
    // prefetch-free: the next step's tables come from df / u_old, read after the barrier
    __syncthreads();  // every wave has read its rows of Φ_{i+1}: the front may be overwritten
    // ---- write Φ_i in place and the U bytes ---------------------------------------------------------------
    const int *bt = btb + cur * LP;
    uint8_t *Ui = Uk + (size_t)i * ((size_t)L * R);
#pragma unroll
    for (int t = 0; t < FU_MAXT; ++t) {
      if (t0 + t < t1) {
        const int task = __builtin_amdgcn_readfirstlane((int)tl[t0 + t]);
        const int rb = task >> 8, l = task & 255;
        const int c = 64 * rb + lane + bt[l];
        if (c <= B) {
          front[c * FS + l] = ov[t];
          if (ov[t] < INFINITY) Ui[(size_t)l * R + c] = (uint8_t)oa[t];
        }
      }
    }
    // cells below the target's own budget class are unreachable: Φ_i[c, l] = +Inf for c < b̃(l, i)
    for (int l = w; l < L; l += FU_W) {
      const int b = min(bt[l], R);
      for (int c = lane; c < b; c += 64) front[c * FS + l] = INFINITY;
    }
    if (i >= 1) fu_prepare<LP, NQ>(P, Lv, k, i - 1, (i - 1) & 1, cst, Kb, btb, taskb, cnt, F);
    __syncthreads();
  }
  // ---- Φ_0 to HBM in the generic layout [L][RP] (the backtrack's argmin reads it) ------------------------
  double *f0 = front0_all + (size_t)k * front_stride;
  for (int e = tid; e < L * P.RP; e += 512) {
    const int l = e / P.RP, c = e - l * P.RP;
    f0[e] = c < R ? front[c * FS + l] : INFINITY;
  }
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

}  // namespace mioc
