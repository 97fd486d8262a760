// mioc_ode.hip -- the ODE gradient producer of the reference's TRM examples, batched on gfx950.
//
// Reference: julia_opt/ODEObjective.jl:125-150 (eval_f_helper: explicit Euler, trapezoid cost), :153-184
// (eval_df_helper: explicit-Euler adjoint, df = Gu - Fu' λ), with the problem hooks F, Fy, Fu, G, Gy of
//   MIOC_ODE_FISHING     julia_opt/example_fishing.jl:14-92     (Lotka-Volterra fishing, SOS1 over 3 controls)
//   MIOC_ODE_DOUBLETANK  julia_opt/example_doubletank.jl:14-82  (double tank multimode)
//   MIOC_ODE_VANDERPOL   julia_opt/example_vanderpol.jl:14-81   (Van der Pol, binary variant)
// The host mirror is mioc/ode.py (the tests compare against it).
//
// One thread per restart k: the forward sweep (nt sequential Euler steps) and the backward adjoint sweep are
// inherently serial in time, and K independent restarts are the parallelism.  The forward states go to a scratch
// array [K][nt][2] that the backward sweep reads back; df[k][i][m] is written in the backward sweep as soon as
// λ_i is known (the reference's separate df loop, fused).  Layouts of x and df are the DP's input layout
// (K x nx x nt, each nx x nt column-major), so the gradient feeds mioc_bellman_batch_device directly.
// Built with -ffp-contract=off: every sum is a plain left-to-right sequence of rounded products and adds.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mioc_internal.h"

namespace mioc {

namespace {

constexpr int NY = 2, NX = 3;

struct OdePar {
  double p[14];
};

// ---- problem hooks (F: right-hand side, Fy: ∂F/∂y as [r][c], Fu: ∂F/∂u as [r][m], G: running cost, Gy) -----
template <int PROB>
struct Hooks;

template <>
struct Hooks<MIOC_ODE_FISHING> {  // p = alpha, beta, gamma, delta, c1, c2, v1[3], v2[3], y0[2]
  __device__ static double s1(const OdePar &P, const double *x) { return ((0.0 + x[0] * P.p[6]) + x[1] * P.p[7]) + x[2] * P.p[8]; }
  __device__ static double s2(const OdePar &P, const double *x) { return ((0.0 + x[0] * P.p[9]) + x[1] * P.p[10]) + x[2] * P.p[11]; }
  __device__ static void F(const OdePar &P, const double *y, const double *x, double *f) {
    f[0] = y[0] * ((P.p[0] - P.p[1] * y[1]) - P.p[4] * s1(P, x));
    f[1] = y[1] * ((-P.p[2] + P.p[3] * y[0]) - P.p[5] * s2(P, x));
  }
  __device__ static void Fy(const OdePar &P, const double *y, const double *x, double fy[2][2]) {
    fy[0][0] = (P.p[0] - P.p[1] * y[1]) - P.p[4] * s1(P, x);
    fy[0][1] = y[0] * -P.p[1];
    fy[1][0] = y[1] * P.p[3];
    fy[1][1] = (-P.p[2] + P.p[3] * y[0]) - P.p[5] * s2(P, x);
  }
  __device__ static void Fu(const OdePar &P, const double *y, const double *, double fu[2][3]) {
    for (int m = 0; m < 3; ++m) {
      fu[0][m] = (y[0] * -P.p[4]) * P.p[6 + m];
      fu[1][m] = (y[1] * -P.p[5]) * P.p[9 + m];
    }
  }
  __device__ static double G(const OdePar &, const double *y) {
    const double a = y[0] - 1.0, b = y[1] - 1.0;
    return 0.5 * (a * a) + 0.5 * (b * b);
  }
  __device__ static void Gy(const OdePar &, const double *y, double *g) {
    g[0] = y[0] - 1.0;
    g[1] = y[1] - 1.0;
  }
};

template <>
struct Hooks<MIOC_ODE_DOUBLETANK> {  // p = k1, k2, c[3], y0[2]
  __device__ static double cx(const OdePar &P, const double *x) { return ((0.0 + P.p[2] * x[0]) + P.p[3] * x[1]) + P.p[4] * x[2]; }
  __device__ static void F(const OdePar &P, const double *y, const double *x, double *f) {
    f[0] = cx(P, x) - sqrt(y[0]);
    f[1] = sqrt(y[0]) - sqrt(y[1]);
  }
  __device__ static void Fy(const OdePar &, const double *y, const double *, double fy[2][2]) {
    fy[0][0] = -1.0 / (2.0 * sqrt(y[0]));
    fy[0][1] = 0.0;
    fy[1][0] = 1.0 / (2.0 * sqrt(y[0]));
    fy[1][1] = -1.0 / (2.0 * sqrt(y[1]));
  }
  __device__ static void Fu(const OdePar &P, const double *, const double *, double fu[2][3]) {
    for (int m = 0; m < 3; ++m) {
      fu[0][m] = P.p[2 + m];
      fu[1][m] = 0.0;
    }
  }
  __device__ static double G(const OdePar &P, const double *y) {
    const double d = y[1] - P.p[1];
    return P.p[0] * (d * d);
  }
  __device__ static void Gy(const OdePar &P, const double *y, double *g) {
    g[0] = 0.0;
    g[1] = (2.0 * P.p[0]) * (y[1] - P.p[1]);
  }
};

template <>
struct Hooks<MIOC_ODE_VANDERPOL> {  // p = c[3], y0[2]
  __device__ static double cx(const OdePar &P, const double *x) { return ((0.0 + P.p[0] * x[0]) + P.p[1] * x[1]) + P.p[2] * x[2]; }
  __device__ static void F(const OdePar &P, const double *y, const double *x, double *f) {
    f[0] = y[1];
    f[1] = ((1.0 - y[0] * y[0]) * y[1]) * cx(P, x) - y[0];
  }
  __device__ static void Fy(const OdePar &P, const double *y, const double *x, double fy[2][2]) {
    const double s = cx(P, x);
    fy[0][0] = 0.0;
    fy[0][1] = 1.0;
    fy[1][0] = ((-2.0 * y[0]) * y[1]) * s - 1.0;
    fy[1][1] = (1.0 - y[0] * y[0]) * s;
  }
  __device__ static void Fu(const OdePar &P, const double *y, const double *, double fu[2][3]) {
    for (int m = 0; m < 3; ++m) {
      fu[0][m] = 0.0;
      fu[1][m] = (P.p[m] * (1.0 - y[0] * y[0])) * y[1];
    }
  }
  __device__ static double G(const OdePar &, const double *y) { return y[0] * y[0] + y[1] * y[1]; }
  __device__ static void Gy(const OdePar &, const double *y, double *g) {
    g[0] = 2.0 * y[0];
    g[1] = 2.0 * y[1];
  }
};

template <int PROB>
__global__ __launch_bounds__(64) void k_ode_eval(int K, int nt, double tau, OdePar P, int y0off, const double *X,
                                                  double *J, double *DF, double *ST, const int32_t *gate) {
  if (gate_closed(gate)) return;
  using H = Hooks<PROB>;
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  const double *x = X + (size_t)k * nt * NX;
  double *st = ST + (size_t)k * nt * NY;
  const double y0[2] = {P.p[y0off], P.p[y0off + 1]};
  // ---- forward: explicit Euler, trapezoid cost (ODEObjective.jl:125-150) ----
  double y[2] = {y0[0], y0[1]}, f[2];
  double fval = 0.5 * H::G(P, y0);
  for (int i = 0; i < nt; ++i) {
    H::F(P, y, x + (size_t)i * NX, f);
    y[0] = y[0] + tau * f[0];
    y[1] = y[1] + tau * f[1];
    st[(size_t)i * NY] = y[0];
    st[(size_t)i * NY + 1] = y[1];
    fval = fval + (i < nt - 1 ? H::G(P, y) : 0.5 * H::G(P, y));
  }
  if (J) J[k] = fval * tau;
  if (!DF) return;
  // ---- backward: adjoint and df = Gu - Fu' λ (ODEObjective.jl:153-184; Gu = 0 for these problems) ----
  double *df = DF + (size_t)k * nt * NX;
  double g[2], fy[2][2], fu[2][3], lam[2];
  H::Gy(P, st + (size_t)(nt - 1) * NY, g);
  lam[0] = (-0.5 * tau) * g[0];
  lam[1] = (-0.5 * tau) * g[1];
  for (int i = nt - 1; i >= 0; --i) {
    // df[:, i] needs λ_i and the state before step i (state0 for i = 0)
    const double *sprev = i == 0 ? y0 : st + (size_t)(i - 1) * NY;
    H::Fu(P, sprev, x + (size_t)i * NX, fu);
    for (int m = 0; m < NX; ++m) df[(size_t)i * NX + m] = (0.0 - (fu[0][m] * lam[0] + fu[1][m] * lam[1])) + 0.0;
    if (i == 0) break;
    // λ_{i-1} = λ_i + τ (Fy' λ_i - Gy), Fy and Gy at (state_{i-1}, x_i)
    const double *si = st + (size_t)(i - 1) * NY;
    H::Gy(P, si, g);
    H::Fy(P, si, x + (size_t)i * NX, fy);
    const double a0 = fy[0][0] * lam[0] + fy[1][0] * lam[1];
    const double a1 = fy[0][1] * lam[0] + fy[1][1] * lam[1];
    lam[0] = lam[0] + tau * (a0 - g[0]);
    lam[1] = lam[1] + tau * (a1 - g[1]);
  }
}

}  // namespace

hipError_t launch_ode_eval(hipStream_t s, const int32_t *gate, int problem, int K, int nt, double tau, const double *params, int y0off,
                           const double *X, double *J, double *DF, double *ST) {
  OdePar P;
  for (int q = 0; q < 14; ++q) P.p[q] = params[q];
  const dim3 grid((K + 63) / 64), block(64);
  switch (problem) {
    case MIOC_ODE_FISHING:
      hipLaunchKernelGGL(k_ode_eval<MIOC_ODE_FISHING>, grid, block, 0, s, K, nt, tau, P, y0off, X, J, DF, ST, gate);
      break;
    case MIOC_ODE_DOUBLETANK:
      hipLaunchKernelGGL(k_ode_eval<MIOC_ODE_DOUBLETANK>, grid, block, 0, s, K, nt, tau, P, y0off, X, J, DF, ST, gate);
      break;
    case MIOC_ODE_VANDERPOL:
      hipLaunchKernelGGL(k_ode_eval<MIOC_ODE_VANDERPOL>, grid, block, 0, s, K, nt, tau, P, y0off, X, J, DF, ST, gate);
      break;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}


// ---------------------------------------------------------------------------------------------------------------
// Restart generator: rand_func_int (HelpFunctions.jl:204-225) on the device.  The reference draws `jumps` distinct
// jump times from 2..nt (1-based; here 1..nt-1) with MersenneTwister + StatsBase.sample and a random admissible
// level per segment.  Julia's stream cannot be reproduced outside Julia, so this generator keeps the algorithm and
// its distribution with a counter-based stream instead: value(seed, k, stream, idx) = mix(mix(seed + φ(k+1)) ^
// (stream << 56) ^ idx), mix = splitmix64's finaliser; a uniform draw in [0, n) is (v >> 32) * n >> 32.  Jump times:
// Robert Floyd's sampling without replacement (one lane, an LDS bitmap of the nt steps); segment s takes the level
// of rank uniform_L(stream 2, s).  The tests restate the same stream on the host bit for bit.
// ---------------------------------------------------------------------------------------------------------------
namespace {

__device__ __forceinline__ uint64_t rs_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint32_t rs_uniform(uint64_t key, uint64_t stream, uint64_t idx, uint32_t n) {
  const uint64_t v = rs_mix(key ^ (stream << 56) ^ idx);
  return (uint32_t)(((v >> 32) * (uint64_t)n) >> 32);
}

__global__ __launch_bounds__(256) void k_rand_start(int nt, int jumps, uint64_t seed, LevelsDev Lv, double *U) {
  extern __shared__ uint32_t bits[];  // [nw] jump-time bitmap, then [256] per-thread segment counts
  const int k = blockIdx.x, tid = threadIdx.x, nw = (nt + 31) >> 5, M = Lv.M;
  uint32_t *cnt = bits + nw;
  const uint64_t key = rs_mix(seed + 0x9E3779B97F4A7C15ull * (uint64_t)(k + 1));
  for (int w = tid; w < nw; w += 256) bits[w] = 0u;
  __syncthreads();
  if (tid == 0) {  // Floyd: a uniform `jumps`-subset of the N = nt - 1 candidate steps 1 .. nt-1
    const int N = nt - 1;
    for (int j = N - jumps + 1, q = 0; j <= N; ++j, ++q) {
      const int t = 1 + (int)rs_uniform(key, 1, (uint64_t)q, (uint32_t)j);  // in [1, j]
      const int pick = (bits[t >> 5] >> (t & 31)) & 1u ? j : t;
      bits[pick >> 5] |= 1u << (pick & 31);
    }
  }
  __syncthreads();
  // segment index of step i = number of jump times <= i: each thread owns a contiguous range of words
  const int wpt = (nw + 255) / 256, w0 = tid * wpt, w1 = min(nw, w0 + wpt);
  uint32_t c = 0;
  for (int w = w0; w < w1; ++w) c += __popc(bits[w]);
  cnt[tid] = c;
  __syncthreads();
  uint32_t seg = 0;
  for (int q = 0; q < tid; ++q) seg += cnt[q];
  double *u = U + (size_t)k * nt * M;
  int rank = -1;
  uint32_t rseg = 0xFFFFFFFFu;
  for (int i = w0 * 32; i < min(nt, w1 * 32); ++i) {
    seg += (bits[i >> 5] >> (i & 31)) & 1u;
    if (seg != rseg) {
      rseg = seg;
      rank = (int)rs_uniform(key, 2, (uint64_t)seg, (uint32_t)Lv.L);
    }
    for (int m = 0; m < M; ++m) u[(size_t)i * M + m] = Lv.nuval[(size_t)rank * M + m];
  }
}

}  // namespace

hipError_t launch_rand_start(hipStream_t s, int K, int nt, int jumps, uint64_t seed, const LevelsDev &Lv, double *U) {
  const size_t lds = ((size_t)(nt + 31) / 32 + 256) * sizeof(uint32_t);
  hipLaunchKernelGGL(k_rand_start, dim3(K), dim3(256), lds, s, nt, jumps, seed, Lv, U);
  return hipGetLastError();
}

}  // namespace mioc
