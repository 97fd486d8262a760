// mioc_generic.hip -- the generic per-step min-plus sweep of bellman_TRM! for gfx950 (any p).
//
// Reference: HelpFunctions.jl:20-83 (bellman_TRM!), :98-124 (eval_u_TRM!).  Indices are 0-based.
//
// HBM layouts (all per subproblem k of a batch):
//   front  Φ_i   : [L][RP] f64, budget row c fastest (the reference's Φ is (B+1) x grid, c fastest);
//                  rows B+1..RP-1 are +Inf padding so every 64-row tile is aligned and full.
//   U_i          : [L][B+1] uint8 (L <= 256) or uint16 -- the iterator RANK of the minimising j
//                  (the reference stores the M-tuple j: 2.21 TB at nt=65536/4096 levels/B=256).
//
// Rounding order is the reference's exactly (build with -ffp-contract=off, no fast-math):
//   T1  = ((0.0 + (Δt*df_1)*ν_1) + (Δt*df_2)*ν_2) + ...          HelpFunctions.jl:52-57
//   K   = T1 + β*w(l, j)                                             :63-67
//   val = K + Φ_{i+1}[c - b̃, j];  update iff Φ_i[c, l] > val         :71-76  (strict: first j wins)
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "mioc_internal.h"

namespace mioc {

// ---------------------------------------------------------------------------------------------
// shared device helpers
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double t1_of(const double *nuv, const double *dfi, int M, double dt) {
  double t = 0.0;
  for (int m = 0; m < M; ++m) t = t + (dt * dfi[m]) * nuv[m];
  return t;
}

__device__ __forceinline__ int bt_of(const double *nuv, const double *uoi, int M) {
  int b = 0;
  for (int m = 0; m < M; ++m) b += (int)fabs(nuv[m] - uoi[m]);
  return b;
}

// integer switching key of (l, j); the cost is costlut[key] = fl(β * w(key))
__device__ __forceinline__ int pair_key(const LevelsDev &Lv, int l, int j) {
  if (Lv.p_kind == MIOC_P_INF) return 0;
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
  return key;
}

__device__ __forceinline__ double pair_cost(const LevelsDev &Lv, int l, int j) {
  if (Lv.p_kind == MIOC_P_TABLE) return Lv.costtab[(size_t)l * Lv.L + j];
  return Lv.costlut[pair_key(Lv, l, j)];
}

// Julia findmin order on Float64 as an unsigned key: NaN first, then isless (-0.0 < +0.0).
__device__ __forceinline__ uint64_t jl_key(double v) {
  if (v != v) return 0ull;
  uint64_t u = (uint64_t)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}

// ---------------------------------------------------------------------------------------------
// input validation: finite df, integral u_old (the reference's InexactError), max budget class
// flags[0] |= 1 non-finite df, |= 2 non-integral u_old;  flags[1] = max_i max_l b̃(l, i) (capped)
// ---------------------------------------------------------------------------------------------
__global__ void k_validate(ProblemDev P, const double *__restrict__ numin, const double *__restrict__ numax,
                           int32_t *flags) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int k = blockIdx.y;
  int bad = 0, bm = 0;
  if (i < P.nt) {
    const double *dfi = P.df + ((size_t)k * P.nt + i) * P.M;
    const double *uoi = P.uold + ((size_t)k * P.nt + i) * P.M;
    long long bmax = 0;
    for (int m = 0; m < P.M; ++m) {
      double d = dfi[m];
      if (!(fabs(d) <= 1.7976931348623157e308)) bad |= 1;
      double u = uoi[m];
      if (!(u == floor(u)) || !(fabs(u) < 4.0e15)) bad |= 2;
      double e = fmax(fabs(numax[m] - u), fabs(numin[m] - u));
      bmax += (e > 1.0e9 || e != e) ? 1000000000LL : (long long)e;
    }
    bm = bmax > (long long)P.B ? P.B : (int)bmax;
  }
  // at most one pair of atomics per wave, and the maximum only when it raises the value already there: same-address
  // atomics serialise at the L2 (one per thread, or even one per wave, took 0.4-0.75 ms at 1024 x 4096 steps)
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    bad |= __shfl_xor(bad, off);
    bm = max(bm, __shfl_xor(bm, off));
  }
  if ((threadIdx.x & 63) == 0) {
    if (bad) atomicOr(&flags[0], bad);
    if (bm > 0 && bm > __hip_atomic_load(&flags[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(&flags[1], bm);
  }
}

hipError_t launch_validate(hipStream_t s, const ProblemDev &P, const double *numin, const double *numax,
                           int32_t *flags) {
  dim3 grid((P.nt + 255) / 256, P.K);
  hipLaunchKernelGGL(k_validate, grid, dim3(256), 0, s, P, numin, numax, flags);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// terminal step (HelpFunctions.jl:27-43): Φ_{n-1}[c, l] = T1(l, n-1) at c = b̃(l, n-1) <= B, else Inf
// ---------------------------------------------------------------------------------------------
__global__ void k_generic_terminal(ProblemDev P, LevelsDev Lv, double *front, size_t front_stride) {
  const int k = blockIdx.y;
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (size_t)Lv.L * P.RP) return;
  const int r = (int)(idx / P.RP);
  const int c = (int)(idx % P.RP);
  const int i = P.nt - 1;
  const double *nuv = Lv.nuval + (size_t)r * Lv.M;
  const double *dfi = P.df + ((size_t)k * P.nt + i) * P.M;
  const double *uoi = P.uold + ((size_t)k * P.nt + i) * P.M;
  const int b = bt_of(nuv, uoi, P.M);
  double v = INFINITY;
  if (c == b && b <= P.B) v = t1_of(nuv, dfi, P.M, P.dt);
  front[(size_t)k * front_stride + idx] = v;
}

hipError_t launch_generic_terminal(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, double *front,
                                   size_t front_stride) {
  size_t n = (size_t)Lv.L * P.RP;
  dim3 grid((unsigned)((n + 255) / 256), P.K);
  hipLaunchKernelGGL(k_generic_terminal, grid, dim3(256), 0, s, P, Lv, front, front_stride);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// one recursion step i (HelpFunctions.jl:45-81), any p.
//
// Work decomposition (64-wide waves): lane = SOURCE budget row c' of Φ_{i+1}; a wave owns RT
// target levels l (wave-uniform, so b̃(l) is uniform and lane c' feeds target row c' + b̃(l));
// the 4 waves of a workgroup share LDS tiles of Φ_{i+1}[j][c'] (64 rows x SCH levels j) and of
// K[l][j] = T1(l) + β·w(l, j).  Per candidate: one v_add_f64 + one v_min_f64; the strict
// first-index argmin is tracked per group of GRP consecutive j (the first group whose minimum
// improves), then resolved exactly by re-scanning that group once at the end.
// ---------------------------------------------------------------------------------------------
constexpr int GS_RT = 8;            // target levels per wave
constexpr int GS_WAVES = 4;
constexpr int GS_RPB = GS_RT * GS_WAVES;
constexpr int GS_SCH = 64;          // source levels per LDS chunk
constexpr int GS_GRP = 8;           // argmin group

template <typename UT>
__global__ __launch_bounds__(256) void k_generic_step(ProblemDev P, LevelsDev Lv, int i,
                                                      const double *__restrict__ psi_all,
                                                      double *__restrict__ phi_all, UT *__restrict__ U_all,
                                                      size_t front_stride, size_t u_stride_k) {
  __shared__ double sPsi[GS_SCH][64];
  __shared__ double sK[GS_RPB][GS_SCH];
  __shared__ double sT1[GS_RPB];
  __shared__ int sB[GS_RPB];

  const int k = blockIdx.z;
  const int L = Lv.L, RP = P.RP, B = P.B, M = P.M;
  const double *psi = psi_all + (size_t)k * front_stride;
  double *phi = phi_all + (size_t)k * front_stride;
  UT *Ui = U_all + (size_t)k * u_stride_k + (size_t)i * ((size_t)L * (B + 1));
  const double *dfi = P.df + ((size_t)k * P.nt + i) * M;
  const double *uoi = P.uold + ((size_t)k * P.nt + i) * M;
  const int c0 = blockIdx.x * 64;
  const int r0 = blockIdx.y * GS_RPB;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  if (threadIdx.x < GS_RPB) {
    const int r = r0 + threadIdx.x;
    double t1 = 0.0;
    int b = INT_MAX / 4;
    if (r < L) {
      const double *nuv = Lv.nuval + (size_t)r * M;
      t1 = t1_of(nuv, dfi, M, P.dt);
      b = bt_of(nuv, uoi, M);
    }
    sT1[threadIdx.x] = t1;
    sB[threadIdx.x] = b;
  }
  __syncthreads();

  const int cp = c0 + lane;  // source row c'
  double best[GS_RT];
  int bg[GS_RT];
  int bk[GS_RT];
  bool valid[GS_RT];
  bool any = false;
#pragma unroll
  for (int kk = 0; kk < GS_RT; ++kk) {
    bk[kk] = sB[w * GS_RT + kk];
    valid[kk] = (r0 + w * GS_RT + kk < L) && (cp <= B - bk[kk]);
    best[kk] = INFINITY;
    bg[kk] = -1;
    any |= valid[kk];
  }
  const int block_any = __syncthreads_or(any);

  if (block_any) {
    for (int s0 = 0; s0 < L; s0 += GS_SCH) {
      for (int e = threadIdx.x; e < GS_SCH * 64; e += 256) {
        const int s = e >> 6, c = e & 63;
        sPsi[s][c] = (s0 + s < L) ? psi[(size_t)(s0 + s) * RP + c0 + c] : INFINITY;
      }
      for (int e = threadIdx.x; e < GS_RPB * GS_SCH; e += 256) {
        const int rr = e / GS_SCH, s = e % GS_SCH;
        const int r = r0 + rr;
        sK[rr][s] = (r < L && s0 + s < L) ? sT1[rr] + pair_cost(Lv, r, s0 + s) : INFINITY;
      }
      __syncthreads();
#pragma unroll 1
      for (int g = 0; g < GS_SCH; g += GS_GRP) {
        double gm[GS_RT];
#pragma unroll
        for (int kk = 0; kk < GS_RT; ++kk) gm[kk] = INFINITY;
#pragma unroll
        for (int s = 0; s < GS_GRP; ++s) {
          const double v = sPsi[g + s][lane];
#pragma unroll
          for (int kk = 0; kk < GS_RT; ++kk) gm[kk] = fmin(gm[kk], sK[w * GS_RT + kk][g + s] + v);
        }
#pragma unroll
        for (int kk = 0; kk < GS_RT; ++kk) {
          if (gm[kk] < best[kk]) {
            best[kk] = gm[kk];
            bg[kk] = s0 + g;
          }
        }
      }
      __syncthreads();
    }
  }

#pragma unroll
  for (int kk = 0; kk < GS_RT; ++kk) {
    const int r = r0 + w * GS_RT + kk;
    if (r >= L) continue;
    const int b = bk[kk];
    if (valid[kk]) {
      int arg = -1;
      if (bg[kk] >= 0) {
        const double t1 = sT1[w * GS_RT + kk];
        for (int s = bg[kk]; s < bg[kk] + GS_GRP && s < L; ++s) {
          const double val = (t1 + pair_cost(Lv, r, s)) + psi[(size_t)s * RP + cp];
          if (val == best[kk]) {
            arg = s;
            break;
          }
        }
      }
      phi[(size_t)r * RP + cp + b] = best[kk];
      if (arg >= 0) Ui[(size_t)r * (B + 1) + cp + b] = (UT)arg;
    }
    if (cp < b || cp > B) phi[(size_t)r * RP + cp] = INFINITY;
  }
}

hipError_t launch_generic_step(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, int i,
                               const double *psi, double *phi, void *U, int ubytes, size_t front_stride,
                               size_t u_stride_k) {
  dim3 grid(P.RP / 64, (Lv.L + GS_RPB - 1) / GS_RPB, P.K);
  if (ubytes == 1)
    hipLaunchKernelGGL(k_generic_step<uint8_t>, grid, dim3(256), 0, s, P, Lv, i, psi, phi, (uint8_t *)U,
                       front_stride, u_stride_k);
  else
    hipLaunchKernelGGL(k_generic_step<uint16_t>, grid, dim3(256), 0, s, P, Lv, i, psi, phi, (uint16_t *)U,
                       front_stride, u_stride_k);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// argmin(@view Φ[1:B'+1, Inds, 1]) (HelpFunctions.jl:106): first minimum in column-major order,
// i.e. lexicographic (Julia order of the value, grid index of l, c).  One workgroup per subproblem.
// ---------------------------------------------------------------------------------------------
struct ArgKey {
  uint64_t v;    // jl_key of the value
  uint64_t pos;  // grid index * 2^32 + c
  double val;
  int32_t r;
  int32_t c;
};

__device__ __forceinline__ bool key_less(const ArgKey &a, const ArgKey &b) {
  return a.v < b.v || (a.v == b.v && a.pos < b.pos);
}

__device__ ArgKey block_argmin(ArgKey mine) {
  __shared__ ArgKey red[16];
  for (int off = 32; off > 0; off >>= 1) {
    ArgKey o;
    o.v = __shfl_xor(mine.v, off);
    o.pos = __shfl_xor(mine.pos, off);
    o.val = __shfl_xor(mine.val, off);
    o.r = __shfl_xor(mine.r, off);
    o.c = __shfl_xor(mine.c, off);
    if (key_less(o, mine)) mine = o;
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[wv] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    for (int q = 1; q < nw; ++q)
      if (key_less(red[q], mine)) mine = red[q];
    red[0] = mine;
  }
  __syncthreads();
  ArgKey res = red[0];
  __syncthreads();
  return res;
}

__global__ __launch_bounds__(1024) void k_generic_argmin0(ProblemDev P, LevelsDev Lv, const double *front0,
                                                          size_t front_stride, int Bu, Start *start) {
  if (gate_closed(P.gate)) return;
  const int k = blockIdx.x;
  Bu = start_budget(P, k, Bu, start);
  if (Bu < 0) return;  // uniform: an out-of-range B'_k (status MIOC_ESTATE)
  const double *f = front0 + (size_t)k * front_stride;
  ArgKey best;
  best.v = ~0ull;
  best.pos = ~0ull;
  best.val = INFINITY;
  best.r = -1;
  best.c = 0;
  const int ncol = Bu + 1;
  const size_t total = (size_t)Lv.L * ncol;
  for (size_t e = threadIdx.x; e < total; e += blockDim.x) {
    const int r = (int)(e / ncol), c = (int)(e % ncol);
    const double v = f[(size_t)r * P.RP + c];
    ArgKey a;
    a.v = jl_key(v);
    a.pos = ((uint64_t)(uint32_t)Lv.gidx[r] << 32) | (uint32_t)c;
    a.val = v;
    a.r = r;
    a.c = c;
    if (key_less(a, best)) best = a;
  }
  best = block_argmin(best);
  if (threadIdx.x == 0) {
    Start st;
    st.phi = best.val;
    st.c = best.c;
    st.r = best.r;
    st.status = (best.r >= 0 && best.val < INFINITY) ? MIOC_OK : MIOC_EINFEASIBLE;
    st.pad = 0;
    start[k] = st;
  }
}

hipError_t launch_generic_argmin0(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const double *front0,
                                  size_t front_stride, int Bu, Start *start) {
  hipLaunchKernelGGL(k_generic_argmin0, dim3(P.K), dim3(1024), 0, s, P, Lv, front0, front_stride, Bu, start);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// forward walk (HelpFunctions.jl:115-122): l <- U_i[c, l]; c <- c - ||ν(l_i) - u_old_i||_1.
//
// Sequentially that is one dependent HBM read per step (nt-1 reads ≈ 0.8 µs each).  One wave per
// subproblem runs the chain ahead instead: lanes t = 0..63 read the argmin cells of steps i..i+63
// along two guessed paths at once,
//   B: the level r of step i is kept (the budget drops by its distance to u_old at every step),
//   A: from step i+1 on, the level equal to u_old (distance 0, the budget stays),
// and a ballot finds the first step where the true path leaves the guess.  Lane 0's cell on path B is
// the true cell of step i, and a cell is accepted only when every earlier accepted cell put the walk
// into exactly the guessed state, so the result is the sequential walk's bit for bit.  A round costs
// one read latency and advances up to 64 steps: A covers the stretches where the solution follows
// u_old (the trust-region budget bounds the deviations), B the deviations themselves.
// ---------------------------------------------------------------------------------------------
__global__ void k_uold_rank(ProblemDev P, LevelsDev Lv, int32_t *urank) {
  if (gate_closed(P.gate)) return;
  const int k = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P.nt) return;
  const double *uo = P.uold + ((size_t)k * P.nt + i) * P.M;
  int g = 0, stride = 1;
  bool ok = Lv.g2r != nullptr;
  for (int m = 0; ok && m < P.M; ++m) {
    const double v = uo[m];
    const int q0 = Lv.voff[m], q1 = Lv.voff[m + 1];
    int q = q0;
    while (q < q1 && (double)Lv.vals[q] != v) ++q;
    ok = q < q1;
    g += (q - q0) * stride;
    stride *= q1 - q0;
  }
  urank[(size_t)k * P.nt + i] = ok ? Lv.g2r[g] : -1;
}

hipError_t launch_uold_rank(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, int32_t *urank) {
  dim3 grid((P.nt + 255) / 256, P.K);
  hipLaunchKernelGGL(k_uold_rank, grid, dim3(256), 0, s, P, Lv, urank);
  return hipGetLastError();
}

__device__ __forceinline__ int wave_incl_sum(int x, int lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(x, off);
    if (lane >= off) x += y;
  }
  return x;
}

// first lane t in [1, n) whose guess failed, else n
__device__ __forceinline__ int first_fail(bool ok, int lane, int n) {
  const unsigned long long bad = __ballot(!ok && lane >= 1 && lane < n);
  return bad ? __builtin_ffsll((long long)bad) - 1 : n;
}

// cell(s, c, b, r): the argmin rank stored for step s, budget c, level r (b = distance of r to u_old_s)
template <class Cell>
__device__ void spec_walk(const ProblemDev &P, const LevelsDev &Lv, int k, const Start &st, const int32_t *urk,
                          int32_t *rk, int32_t *counters, Cell cell) {
  const int lane = threadIdx.x & 63, M = P.M, nt = P.nt;
  const double *uok = P.uold + (size_t)k * nt * M;
  int i = 0, r = st.r, c = st.c, rounds = 0;
  if (lane == 0) rk[0] = r;
  while (i + 1 < nt) {
    ++rounds;
    const int n = min(64, nt - 1 - i);  // this round resolves the cells of steps i .. i+n-1
    const int s = i + lane;
    const bool act = lane < n;
    const int bB = act ? bt_of(Lv.nuval + (size_t)r * M, uok + (size_t)s * M, M) : 0;
    const int inc = wave_incl_sum(bB, lane);
    const int cB = c - (inc - bB);  // budget at step s on path B
    const int c1 = c - __shfl(bB, 0);
    const int g = (urk && act) ? urk[s] : -1;
    int vB = -1, vA = -1;
    if (act && cB >= bB) vB = cell(s, cB, bB, r);
    if (lane >= 1 && g >= 0 && c1 >= 0) vA = cell(s, c1, 0, g);
    if (__shfl(vB, 0) < 0) {  // the true cell of step i is unreachable: inconsistent tables
      if (lane == 0) atomicAdd(counters + 1, 1);
      return;
    }
    const int vAx = lane == 0 ? vB : vA;  // path A's cells (lane 0: the true cell of step i)
    const int fB = first_fail(__shfl_up(vB, 1) == r, lane, n);
    const int fA = first_fail(g >= 0 && __shfl_up(vAx, 1) == g, lane, n);
    const bool useA = fA > fB;
    const int f = useA ? fA : fB;        // steps i+1 .. i+f are now known
    const int v = useA ? vAx : vB;       // lane t < f: the level of step i+t+1
    if (lane < f) rk[i + lane + 1] = v;
    const int rn = __shfl(v, f - 1);
    const int cn = useA ? c1 : __shfl(c - inc, f - 1);
    if (rn < 0 || rn >= Lv.L || cn < 0) {
      if (lane == 0) atomicAdd(counters + 1, 1);
      return;
    }
    i += f;
    r = rn;
    c = cn;
  }
  if (lane == 0) atomicAdd(counters, rounds);
}

template <typename UT>
__global__ __launch_bounds__(64) void k_generic_walk(ProblemDev P, LevelsDev Lv, const UT *__restrict__ U,
                                                     size_t u_stride_k, const Start *start, const int32_t *urank,
                                                     int32_t *ranks, int32_t *counters) {
  if (gate_closed(P.gate)) return;
  const int k = blockIdx.x;
  const Start st = start[k];
  if (st.status != MIOC_OK) return;
  const UT *Uk = U + (size_t)k * u_stride_k;
  const size_t step = (size_t)Lv.L * (P.B + 1);
  const int R = P.B + 1;
  spec_walk(P, Lv, k, st, urank ? urank + (size_t)k * P.nt : nullptr, ranks + (size_t)k * P.nt, counters,
            [&](int s, int c, int, int r) { return (int)Uk[(size_t)s * step + (size_t)r * R + c]; });
}

hipError_t launch_generic_walk(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const void *U, int ubytes,
                               size_t u_stride_k, const Start *start, const int32_t *urank, int32_t *ranks,
                               int32_t *counters) {
  if (ubytes == 1)
    hipLaunchKernelGGL(k_generic_walk<uint8_t>, dim3(P.K), dim3(64), 0, s, P, Lv, (const uint8_t *)U, u_stride_k,
                       start, urank, ranks, counters);
  else
    hipLaunchKernelGGL(k_generic_walk<uint16_t>, dim3(P.K), dim3(64), 0, s, P, Lv, (const uint16_t *)U, u_stride_k,
                       start, urank, ranks, counters);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// ranks -> u (level values, nx x nt column-major per subproblem), Φ*, status
// ---------------------------------------------------------------------------------------------
__global__ void k_expand(ProblemDev P, LevelsDev Lv, const Start *start, const int32_t *ranks, double *u_out,
                         double *phi_star, int32_t *status) {
  if (gate_closed(P.gate)) return;
  const int k = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const Start st = start[k];
  if (i == 0) {
    if (phi_star) phi_star[k] = st.phi;
    if (status) status[k] = st.status;
  }
  if (i >= P.nt) return;
  double *uo = u_out + ((size_t)k * P.nt + i) * P.M;
  if (st.status != MIOC_OK) {
    for (int m = 0; m < P.M; ++m) uo[m] = NAN;
    return;
  }
  const int r = ranks[(size_t)k * P.nt + i];
  for (int m = 0; m < P.M; ++m) uo[m] = Lv.nuval[(size_t)r * P.M + m];
}

hipError_t launch_expand(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const Start *start,
                         const int32_t *ranks, double *u_out, double *phi_star, int32_t *status) {
  dim3 grid((P.nt + 255) / 256, P.K);
  hipLaunchKernelGGL(k_expand, grid, dim3(256), 0, s, P, Lv, start, ranks, u_out, phi_star, status);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// staging layout (pyramid path): Φ_0[l, c] = S_0[c - b̃_l(0)][pos_0(l)] (rows in sphere order of u_old(0)),
// U_i[l, c] = UU_i[c - b̃_l(i)][l]
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_stage_argmin0(ProblemDev P, LevelsDev Lv, const uint32_t *perm_all,
                                                        const double *S0_all, size_t s_stride, int Bu, Start *start) {
  if (gate_closed(P.gate)) return;
  const int k = blockIdx.x, L = Lv.L;
  Bu = start_budget(P, k, Bu, start);
  if (Bu < 0) return;  // uniform: an out-of-range B'_k (status MIOC_ESTATE)
  const double *S0 = S0_all + (size_t)k * s_stride;
  const uint32_t *perm = perm_all + (size_t)k * P.nt * L;  // sphere order of u_old(0): rank | b̃ << 16
  ArgKey best;
  best.v = ~0ull;
  best.pos = ~0ull;
  best.val = INFINITY;
  best.r = -1;
  best.c = 0;
  for (int p = threadIdx.x; p < L; p += blockDim.x) {
    const int r = (int)(perm[p] & 0xFFFFu), b = (int)(perm[p] >> 16);
    for (int c = b; c <= Bu; ++c) {  // first minimum over c for this l, then (value, grid index, c)
      const double v = S0[(size_t)(c - b) * L + p];
      ArgKey a;
      a.v = jl_key(v);
      a.pos = ((uint64_t)(uint32_t)Lv.gidx[r] << 32) | (uint32_t)c;
      a.val = v;
      a.r = r;
      a.c = c;
      if (key_less(a, best)) best = a;
    }
  }
  best = block_argmin(best);
  if (threadIdx.x == 0) {
    Start st;
    st.phi = best.val;
    st.c = best.c;
    st.r = best.r;
    st.status = (best.r >= 0 && best.val < INFINITY) ? MIOC_OK : MIOC_EINFEASIBLE;
    st.pad = 0;
    start[k] = st;
  }
}

hipError_t launch_stage_argmin0(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const uint32_t *perm,
                                const double *S0, size_t s_stride, int Bu, Start *start) {
  hipLaunchKernelGGL(k_stage_argmin0, dim3(P.K), dim3(1024), 0, s, P, Lv, perm, S0, s_stride, Bu, start);
  return hipGetLastError();
}

// the staging layout's argmin table: UU_i[c - b][r] (source row c - b̃, level rank r)
__global__ __launch_bounds__(64) void k_stage_walk(ProblemDev P, LevelsDev Lv, const uint16_t *__restrict__ UU,
                                                   size_t uu_stride_k, const Start *start, const int32_t *urank,
                                                   int32_t *ranks, int32_t *counters) {
  if (gate_closed(P.gate)) return;
  const int k = blockIdx.x;
  const Start st = start[k];
  if (st.status != MIOC_OK) return;
  const uint16_t *Uk = UU + (size_t)k * uu_stride_k;
  const size_t step = (size_t)(P.B + 1) * Lv.L;
  const int L = Lv.L;
  spec_walk(P, Lv, k, st, urank ? urank + (size_t)k * P.nt : nullptr, ranks + (size_t)k * P.nt, counters,
            [&](int s, int c, int b, int r) { return (int)Uk[(size_t)s * step + (size_t)(c - b) * L + r]; });
}

hipError_t launch_stage_walk(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const uint16_t *UU,
                             size_t uu_stride_k, const Start *start, const int32_t *urank, int32_t *ranks,
                             int32_t *counters) {
  hipLaunchKernelGGL(k_stage_walk, dim3(P.K), dim3(64), 0, s, P, Lv, UU, uu_stride_k, start, urank, ranks,
                     counters);
  return hipGetLastError();
}

}  // namespace mioc
