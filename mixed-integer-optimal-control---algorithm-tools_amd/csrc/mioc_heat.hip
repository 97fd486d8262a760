// mioc_heat.hip -- the PDE heat objective's value and gradient, batched over restarts on gfx950.
//
// Reference: julia_opt/PDEObjective.jl:129-139 (impleuler_state!: y_i = SMatLU \ (y_{i-1} + τ·M⁻¹F·x_{i-1})),
// :142-156 (eval_f_helper: trapezoid over G + G_t, x extended by its last column), :159-172 (impleuler_adjoint!:
// p_i = AMatLU \ (p_{i+1} + τ·Gy_i), AMatLU = lu(StateMat')), :174-199 (eval_df_helper: df_i = (M⁻¹F)ᵀ p_i, plus
// Gu = γ for i ≥ 2 only), with the hooks of julia_opt/example_heat.jl:135-161 (G = ½ vᵀMv, v = y_i − yd_i;
// G_t = γ·Σx; Gy = M·v; Gu = γ).  StateMat = I + τ·M⁻¹A (example_heat.jl:113-115).
//
// The matrices are the caller's: the Julia objective assembles A, M, F, state0 and yd with its FEM bundle
// (FEMBundle, julia_fem/) and hands them over once (mioc_heat_setup); only the time loops run here.
//
// Design.  The system is linear and time-invariant, so both triangular solves per step become one product with a
// precomputed inverse (S⁻¹ for the state, S⁻ᵀ for the adjoint), and the K restarts side by side turn every step
// into a dense (N × N) · (N × 16) product on the FP64 matrix cores: one workgroup (16 waves) per 16 restarts (one
// MFMA column tile), all nt forward and nt adjoint steps in one launch, the 16 state columns in LDS (N ≤ 512) or in
// a per-workgroup global scratch (N ≤ 2048).  A forward step is one pass over its right-hand side z computing
// y' = S⁻¹z and Gy' = (M·S⁻¹)z − M·yd' with two accumulators that share the B reads; an adjoint step one product
// with S⁻ᵀ.  Gy goes to an HBM scratch between the sweeps (written once, read once).  The operand matrices stream
// from L2 in the MFMA A-operand order, one 16-byte load per lane per two MFMAs.  Results agree with the
// reference's LU solves to rounding (the inverse and the MFMA sum order are not the reference's operation order):
// the tests hold them to 1e-9 relative.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "mioc_internal.h"

namespace mioc {

struct HeatState {
  bool ready = false;  // every device table matches N / Np / nx / nt (false after a failed setup)
  int64_t N = 0, Np = 0, nx = 0, nt = 0;
  double tau = 0.0, gamma = 0.0;
  double *d_sinv = nullptr, *d_sinvT = nullptr;                    // A-operand order, [Np/16][Np/8][64] double2
  double *d_minvF = nullptr;                                        // [Np][nx] row-major, zero-padded
  double *d_state0 = nullptr;                                       // [Np]
  double *d_yd = nullptr;                                           // [nt + 1][Np]
  double *d_gy = nullptr;                                           // [tiles][nt][Np][16] Gy_i between the sweeps
  size_t gy_cap = 0;
  double *d_io = nullptr;                                           // host entry staging: x, df, J
  size_t io_cap = 0;
  double *d_msinv = nullptr;                                        // M·S⁻¹ in the A-operand order
  double *d_myd = nullptr;                                          // [nt + 1][Np] M·yd_j
  double *d_gy0 = nullptr;                                          // [Np] M·(state0 − yd_0)
  double g0 = 0.0;                                                  // (state0 − yd_0)ᵀ M (state0 − yd_0)
  double *d_sc = nullptr;                                           // [tiles][2][Np][16] y, z for Np > 512
  size_t sc_cap = 0;
};

void heat_free(HeatState *h) {
  if (!h) return;
  for (double *p : {h->d_sinv, h->d_sinvT, h->d_minvF, h->d_state0, h->d_yd, h->d_gy, h->d_io, h->d_msinv, h->d_myd, h->d_gy0, h->d_sc})
    if (p) hipFree(p);
  delete h;
}

namespace {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

// Measured at N = 289, K = 4096 (scripts/probe_heat.py): 4 / 8 / 16 waves per workgroup 39.4 / 33.8 / 28.9 ms per
// launch with separate forward products; one fused forward pass 25.1 ms; A prefetched two k-blocks ahead instead
// of one 3-5 % slower; non-temporal Gy stores no change.
constexpr int HW = 16;          // waves per workgroup
constexpr int HMAXNX = 4;       // controls per step
constexpr int HMAXN_LDS = 496;  // y and z (2 x Np x 16 doubles), yd / M·yd rows and the reductions fit 160 KB of LDS
constexpr int HMAXN = 2048;     // beyond HMAXN_LDS the 16 state columns live in a global scratch (L2-served)

struct HeatArgs {
  const d2 *sinv, *sinvT, *msinv;   // A-operand order: S⁻¹, S⁻ᵀ, M·S⁻¹
  const double *minvF, *state0, *yd, *myd, *gy0;
  double g0;
  const double *X;
  double *J, *DF, *GY;
  double *SC;                       // [tiles][2][Np][16] y, z when they do not fit LDS
  int K, nx, nt, Np;
  double tau, gamma;
  const int32_t *gate;              // device TRM control gate (see ProblemDev::gate)
};

// acc1 = A1(tile t) · Bs (and acc2 = A2(t) · Bs when A2) for the two row tiles t0, t1 of this wave (a tile
// >= ntile is skipped); Bs is [Np][16].  A-operand lanes hold A[16t + (l & 15)][k + (l >> 4)] (MI355X_MICROARCH.md,
// v_mfma_f64_16x16x4_f64), two k-blocks per 16-byte load; the loads of block kb + 1 are in flight while block kb's
// MFMAs issue, and both products share the B reads.
template <bool TWO>
__device__ __forceinline__ void heat_gemm(const d2 *__restrict__ A1, const d2 *__restrict__ A2, const double *Bs,
                                          int Np, int t0, int t1, int lane, d4 (&acc1)[2], d4 (&acc2)[2]) {
  const int ntile = Np >> 4, KB = Np >> 3;
  const bool on[2] = {t0 < ntile, t1 < ntile};
  size_t off[2];
  off[0] = (size_t)min(t0, ntile - 1) * KB * 64 + lane;
  off[1] = (size_t)min(t1, ntile - 1) * KB * 64 + lane;
#pragma unroll
  for (int s = 0; s < 2; ++s) acc1[s] = acc2[s] = d4{0.0, 0.0, 0.0, 0.0};
  d2 n1[2], n2[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    n1[s] = A1[off[s]];
    if (TWO) n2[s] = A2[off[s]];
  }
  for (int kb = 0; kb < KB; ++kb) {
    d2 a1[2], a2[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) a1[s] = n1[s], a2[s] = n2[s];
    const size_t kn = (size_t)min(kb + 1, KB - 1) * 64;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      n1[s] = A1[off[s] + kn];
      if (TWO) n2[s] = A2[off[s] + kn];
    }
    const double b0 = Bs[kb * 128 + lane], b1 = Bs[kb * 128 + 64 + lane];
#pragma unroll
    for (int s = 0; s < 2; ++s)
      if (on[s]) {
        acc1[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[s].x, b0, acc1[s], 0, 0, 0);
        if (TWO) acc2[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[s].x, b0, acc2[s], 0, 0, 0);
        acc1[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[s].y, b1, acc1[s], 0, 0, 0);
        if (TWO) acc2[s] = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[s].y, b1, acc2[s], 0, 0, 0);
      }
  }
}

// y / z in LDS: LDS traffic only, so the barrier waits for LDS operations alone (the Gy stores to HBM stay in
// flight); in the global scratch the barrier must also drain the vector-memory stores
template <bool GM>
__device__ __forceinline__ void heat_barrier() {
  if (GM)
    __syncthreads();
  else
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <bool GM>
__global__ __launch_bounds__(HW * 64) void k_heat_run(HeatArgs H) {
  if (gate_closed(H.gate)) return;
  extern __shared__ __attribute__((aligned(16))) double hsm[];
  const int Np = H.Np, nx = H.nx, nt = H.nt, E = Np * 16;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, c = lane & 15, tile = blockIdx.x;
  const int ntile = Np >> 4;
  double *Ys = GM ? H.SC + (size_t)tile * 2 * E : hsm, *Zs = Ys + E;
  double *ydl = GM ? hsm : hsm + 2 * E, *mydl = ydl + Np;  // yd_{j+1}, M·yd_{j+1} of the running step
  double *red = mydl + Np;                                   // [HW][16], then [HW][HMAXNX][16]
  const double tau = H.tau;
  const size_t xs = (size_t)nt * nx;  // doubles per restart in X / DF
  // this thread's restart column in the elementwise phases (every e it visits has e & 15 == tid & 15)
  const int kcol = tile * 16 + (tid & 15);
  const double *xk = kcol < H.K ? H.X + (size_t)kcol * xs : nullptr;
  double *gyt = H.DF ? H.GY + (size_t)tile * nt * E : nullptr;
  d4 acc[2], acc2[2];

  // state column 0 = state0 (PDEObjective.jl:130); Gy_0 and v_0ᵀMv_0 do not depend on the control (setup)
  for (int e = tid; e < E; e += HW * 64) {
    Ys[e] = H.state0[e >> 4];
    if (gyt) gyt[e] = H.gy0[e >> 4];
  }
  __syncthreads();
  double gacc = 0.0;  // Σ_j w_j · v_jᵀ M v_j for column c (trapezoid weights of PDEObjective.jl:148-153)
  for (int j = 0; j < nt; ++j) {
    // z = y_j + τ·(M⁻¹F · x_j)  (PDEObjective.jl:136)
    {
      double xq[HMAXNX];
#pragma unroll
      for (int q = 0; q < HMAXNX; ++q) xq[q] = (xk && q < nx) ? xk[(size_t)j * nx + q] : 0.0;
      for (int e = tid; e < E; e += HW * 64) {
        const double *f = H.minvF + (size_t)(e >> 4) * nx;
        double sf = 0.0;
#pragma unroll
        for (int q = 0; q < HMAXNX; ++q)
          if (q < nx) sf += f[q] * xq[q];
        Zs[e] = Ys[e] + tau * sf;
      }
      // the epilogue's yd_{j+1} / M·yd_{j+1} through LDS: their global round trip overlaps this phase's
      for (int r = tid; r < Np; r += HW * 64) {
        ydl[r] = H.yd[(size_t)(j + 1) * Np + r];
        mydl[r] = H.myd[(size_t)(j + 1) * Np + r];
      }
    }
    heat_barrier<GM>();
    // y_{j+1} = S⁻¹·z; Gy_{j+1} = M·(y_{j+1} − yd_{j+1}) = (M·S⁻¹)·z − M·yd_{j+1}; G partial v·Gy
    const double wj = (j + 1 == nt) ? 0.5 : 1.0;
    for (int t0 = w; t0 < ntile; t0 += 2 * HW) {
      heat_gemm<true>(H.sinv, H.msinv, Zs, Np, t0, t0 + HW, lane, acc, acc2);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int t = t0 + HW * s;
        if (t < ntile) {
          double part = 0.0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int r = 16 * t + (lane >> 4) + 4 * q;
            const double y = acc[s][q], gy = acc2[s][q] - mydl[r];
            Ys[r * 16 + c] = y;
            part += (y - ydl[r]) * gy;
            if (gyt && j + 1 < nt) gyt[(size_t)(j + 1) * E + r * 16 + c] = gy;
          }
          gacc += wj * part;
        }
      }
    }
    heat_barrier<GM>();
  }
  // J = τ·(½·Σ w_j v_jᵀMv_j + Σ w_j γ·Σx_j), x extended by its last column (PDEObjective.jl:145-153)
  gacc += __shfl_xor(gacc, 16);
  gacc += __shfl_xor(gacc, 32);
  if (lane < 16) red[w * 16 + lane] = gacc;
  __syncthreads();
  if (tid < 16 && H.J && kcol < H.K) {
    double g = 0.5 * H.g0;  // the j = 0 term (weight ½)
    for (int v = 0; v < HW; ++v) g += red[v * 16 + tid];
    double gt = 0.0;
    for (int i = 0; i <= nt; ++i) {
      const int ic = i < nt ? i : nt - 1;
      double sx = 0.0;
      for (int q = 0; q < nx; ++q) sx += xk[(size_t)ic * nx + q];
      gt += (i == 0 || i == nt ? 0.5 : 1.0) * (H.gamma * sx);
    }
    H.J[kcol] = tau * (0.5 * g + gt);
  }
  if (!H.DF) return;
  // adjoint: p_nt = 0; p_i = S⁻ᵀ·(p_{i+1} + τ·Gy_i); df_i = (M⁻¹F)ᵀ p_i (+ γ for i ≥ 1)  (PDEObjective.jl:159-199)
  for (int e = tid; e < E; e += HW * 64) Ys[e] = 0.0;
  __syncthreads();
  double *redf = red + HW * 16;  // [HW][HMAXNX][16]
  // Gy_i of this thread's first GPF elements is loaded one step ahead, in flight across the barrier and the product
  constexpr int GPF = GM ? 2 : 8;  // the global-scratch variant has no registers to spare
  double gn[GPF];
#pragma unroll
  for (int u = 0; u < GPF; ++u) {
    const int e = tid + u * HW * 64;
    gn[u] = e < E ? gyt[(size_t)(nt - 1) * E + e] : 0.0;
  }
  for (int i = nt - 1; i >= 0; --i) {
    {
#pragma unroll
      for (int u = 0; u < GPF; ++u) {
        const int e = tid + u * HW * 64;
        if (e < E) Zs[e] = Ys[e] + tau * gn[u];
      }
      const double *g = gyt + (size_t)i * E;
      for (int e = tid + GPF * HW * 64; e < E; e += HW * 64) Zs[e] = Ys[e] + tau * g[e];
      if (i > 0) {
#pragma unroll
        for (int u = 0; u < GPF; ++u) {
          const int e = tid + u * HW * 64;
          if (e < E) gn[u] = g[e - E];
        }
      }
    }
    heat_barrier<GM>();
    double dq[HMAXNX] = {0.0, 0.0, 0.0, 0.0};
    for (int t0 = w; t0 < ntile; t0 += 2 * HW) {
      heat_gemm<false>(H.sinvT, nullptr, Zs, Np, t0, t0 + HW, lane, acc, acc2);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int t = t0 + HW * s;
        if (t < ntile) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int r = 16 * t + (lane >> 4) + 4 * q;
            const double p = acc[s][q];
            Ys[r * 16 + c] = p;
#pragma unroll
            for (int m = 0; m < HMAXNX; ++m)
              if (m < nx) dq[m] += H.minvF[(size_t)r * nx + m] * p;
          }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < HMAXNX; ++m) {
      double v = dq[m];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (lane < 16 && m < nx) redf[(w * HMAXNX + m) * 16 + lane] = v;
    }
    heat_barrier<GM>();
    if (tid < nx * 16) {
      const int m = tid >> 4, cc = tid & 15, k = tile * 16 + cc;
      if (k < H.K) {
        double v = 0.0;
        for (int u = 0; u < HW; ++u) v += redf[(u * HMAXNX + m) * 16 + cc];
        H.DF[(size_t)k * xs + (size_t)i * nx + m] = (0.0 + v) + (i >= 1 ? H.gamma : 0.0);
      }
    }
  }
}

hipError_t launch_heat(hipStream_t s, const HeatArgs &H, int tiles) {
  const bool gm = H.Np > HMAXN_LDS;
  const size_t lds = ((gm ? 0 : (size_t)2 * H.Np * 16) + 2 * (size_t)H.Np + HW * 16 + HW * HMAXNX * 16) * sizeof(double);
  const void *fn = gm ? reinterpret_cast<const void *>(&k_heat_run<true>)
                      : reinterpret_cast<const void *>(&k_heat_run<false>);
  (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (gm)
    hipLaunchKernelGGL(k_heat_run<true>, dim3(tiles), dim3(HW * 64), lds, s, H);
  else
    hipLaunchKernelGGL(k_heat_run<false>, dim3(tiles), dim3(HW * 64), lds, s, H);
  return hipGetLastError();
}

// A (N x N, element a(r, c)) into the MFMA A-operand order: [Np/16][Np/8][64] double2, lane l of block (t, kb)
// holding {a(16t + (l&15), 8kb + (l>>4)), a(16t + (l&15), 8kb + 4 + (l>>4))}, zero outside N.
template <class F>
std::vector<double> swizzle(int64_t N, int64_t Np, F a) {
  std::vector<double> out((size_t)Np * Np, 0.0);
  const int64_t KB = Np / 8;
  for (int64_t t = 0; t < Np / 16; ++t)
    for (int64_t kb = 0; kb < KB; ++kb)
      for (int l = 0; l < 64; ++l) {
        const int64_t r = 16 * t + (l & 15), k0 = 8 * kb + (l >> 4), k1 = k0 + 4;
        double *o = &out[(((size_t)t * KB + kb) * 64 + l) * 2];
        o[0] = (r < N && k0 < N) ? a(r, k0) : 0.0;
        o[1] = (r < N && k1 < N) ? a(r, k1) : 0.0;
      }
  return out;
}

// inverse of the dense N x N matrix S (column-major) by Gauss-Jordan with partial pivoting; false if singular
bool invert(int64_t N, std::vector<double> S, std::vector<double> &inv) {
  inv.assign((size_t)N * N, 0.0);
  for (int64_t i = 0; i < N; ++i) inv[(size_t)i * N + i] = 1.0;
  auto s = [&](int64_t r, int64_t c) -> double & { return S[(size_t)c * N + r]; };
  auto v = [&](int64_t r, int64_t c) -> double & { return inv[(size_t)c * N + r]; };
  std::vector<double> f(N);
  for (int64_t col = 0; col < N; ++col) {
    int64_t piv = col;
    for (int64_t r = col + 1; r < N; ++r)
      if (std::fabs(s(r, col)) > std::fabs(s(piv, col))) piv = r;
    if (!(std::fabs(s(piv, col)) > 0.0)) return false;
    if (piv != col)
      for (int64_t c = 0; c < N; ++c) std::swap(s(piv, c), s(col, c)), std::swap(v(piv, c), v(col, c));
    const double d = s(col, col);
    for (int64_t c = 0; c < N; ++c) s(col, c) /= d, v(col, c) /= d;
    for (int64_t r = 0; r < N; ++r) f[r] = r == col ? 0.0 : s(r, col);
    // column by column (contiguous in r): row r -= f[r] * pivot row
    for (int64_t c = 0; c < N; ++c) {
      const double ps = s(col, c), pv = v(col, c);
      if (ps != 0.0) {
        double *sc = &s(0, c);
        for (int64_t r = 0; r < N; ++r) sc[r] -= f[r] * ps;
      }
      if (pv != 0.0) {
        double *vc = &v(0, c);
        for (int64_t r = 0; r < N; ++r) vc[r] -= f[r] * pv;
      }
    }
  }
  return true;
}

int heat_fail(mioc_ctx *ctx, int code, const std::string &msg) {
  ctx->err = msg;
  return code;
}

int upload(mioc_ctx *ctx, double **dst, const std::vector<double> &src, const char *what) {
  if (*dst) hipFree(*dst), *dst = nullptr;
  if (hipMalloc(reinterpret_cast<void **>(dst), src.size() * sizeof(double)) != hipSuccess) {
    (void)hipGetLastError();
    *dst = nullptr;
    return heat_fail(ctx, MIOC_ENOMEM, std::string("cannot allocate the heat ") + what);
  }
  if (hipMemcpy(*dst, src.data(), src.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
    return heat_fail(ctx, MIOC_EHIP, std::string("heat upload failed: ") + what);
  return MIOC_OK;
}

}  // namespace
}  // namespace mioc

using namespace mioc;

extern "C" {

int32_t mioc_heat_setup(mioc_ctx *ctx, int64_t N, int64_t nx, int64_t nt, double T0, double T1, double gamma,
                        const double *M_invA, const double *M_invF, const double *mass, const double *state0,
                        const double *yd) {
  if (!ctx) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  if (N < 1 || N > HMAXN)
    return heat_fail(ctx, MIOC_EINVAL, "heat: need 1 <= Nglobal_dofs <= " + std::to_string(HMAXN));
  if (nx < 1 || nx > HMAXNX) return heat_fail(ctx, MIOC_EINVAL, "heat: need 1 <= nx <= 4 controls");
  if (nt < 1 || nt > (1 << 24)) return heat_fail(ctx, MIOC_EINVAL, "heat: bad nt");
  if (!(T1 > T0)) return heat_fail(ctx, MIOC_EINVAL, "heat: need T1 > T0");
  if (!M_invA || !M_invF || !mass || !state0 || !yd) return heat_fail(ctx, MIOC_EINVAL, "heat: null matrix");
  if (!std::isfinite(gamma)) return heat_fail(ctx, MIOC_EINVAL, "heat: gamma must be finite");
  const double tau = (T1 - T0) / (double)nt;  // example_heat.jl:90
  // StateMat = spdiagm(ones(N)) + τ·M⁻¹A (example_heat.jl:113)
  std::vector<double> S((size_t)N * N);
  for (int64_t c = 0; c < N; ++c)
    for (int64_t r = 0; r < N; ++r) {
      const double a = M_invA[(size_t)c * N + r];
      if (!std::isfinite(a)) return heat_fail(ctx, MIOC_EINVAL, "heat: M_invA has a non-finite entry");
      S[(size_t)c * N + r] = (r == c ? 1.0 : 0.0) + tau * a;
    }
  std::vector<double> Si;
  if (!invert(N, S, Si)) return heat_fail(ctx, MIOC_EINVAL, "heat: I + tau*M_invA is singular");
  const int64_t Np = (N + 15) / 16 * 16;
  HeatState *h = ctx->heat ? ctx->heat : new HeatState();
  ctx->heat = h;
  h->ready = false;  // until every table below is uploaded for the new sizes
  h->N = N, h->Np = Np, h->nx = nx, h->nt = nt, h->tau = tau, h->gamma = gamma;
  if (hipSetDevice(ctx->device) != hipSuccess) return heat_fail(ctx, MIOC_EHIP, "hipSetDevice failed");
  int rc;
  if ((rc = upload(ctx, &h->d_sinv, swizzle(N, Np, [&](int64_t r, int64_t c) { return Si[(size_t)c * N + r]; }),
                   "S^-1")))
    return rc;
  if ((rc = upload(ctx, &h->d_sinvT, swizzle(N, Np, [&](int64_t r, int64_t c) { return Si[(size_t)r * N + c]; }),
                   "S^-T")))
    return rc;
  // M·S⁻¹ (column-major), M·yd_j, Gy_0 = M·(state0 − yd_0) and g0 = (state0 − yd_0)ᵀ Gy_0 for the fused step
  std::vector<double> MS((size_t)N * N, 0.0), myd((size_t)(nt + 1) * Np, 0.0), gy0(Np, 0.0);
  for (int64_t c = 0; c < N; ++c)
    for (int64_t k = 0; k < N; ++k) {
      const double b = Si[(size_t)c * N + k];
      if (b == 0.0) continue;
      for (int64_t r = 0; r < N; ++r) MS[(size_t)c * N + r] += mass[(size_t)k * N + r] * b;
    }
  for (int64_t j = 0; j <= nt; ++j)
    for (int64_t k = 0; k < N; ++k) {
      const double y = yd[(size_t)j * N + k];
      if (y == 0.0) continue;
      for (int64_t r = 0; r < N; ++r) myd[(size_t)j * Np + r] += mass[(size_t)k * N + r] * y;
    }
  double g0 = 0.0;
  for (int64_t k = 0; k < N; ++k) {
    const double v0 = state0[k] - yd[k];
    for (int64_t r = 0; r < N; ++r) gy0[r] += mass[(size_t)k * N + r] * v0;
  }
  for (int64_t r = 0; r < N; ++r) g0 += (state0[r] - yd[r]) * gy0[r];
  h->g0 = g0;
  if ((rc = upload(ctx, &h->d_msinv, swizzle(N, Np, [&](int64_t r, int64_t c) { return MS[(size_t)c * N + r]; }),
                   "M S^-1")) ||
      (rc = upload(ctx, &h->d_myd, myd, "M yd")) || (rc = upload(ctx, &h->d_gy0, gy0, "Gy_0")))
    return rc;
  std::vector<double> f((size_t)Np * nx, 0.0), y0(Np, 0.0), ydp((size_t)(nt + 1) * Np, 0.0);
  for (int64_t r = 0; r < N; ++r) {
    for (int64_t q = 0; q < nx; ++q) f[(size_t)r * nx + q] = M_invF[(size_t)q * N + r];
    y0[r] = state0[r];
  }
  for (int64_t j = 0; j <= nt; ++j)
    for (int64_t r = 0; r < N; ++r) ydp[(size_t)j * Np + r] = yd[(size_t)j * N + r];
  if ((rc = upload(ctx, &h->d_minvF, f, "M_invF")) || (rc = upload(ctx, &h->d_state0, y0, "state0")) ||
      (rc = upload(ctx, &h->d_yd, ydp, "yd")))
    return rc;
  h->ready = true;
  return MIOC_OK;
}

int32_t mioc_heat_eval_device(mioc_ctx *ctx, int64_t K, const double *d_x, double *d_J, double *d_df) {
  if (!ctx) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  HeatState *h = ctx->heat;
  if (!h || !h->ready) return heat_fail(ctx, MIOC_ESTATE, "heat: no successful mioc_heat_setup");
  if (K < 1 || K > INT32_MAX || !d_x) return heat_fail(ctx, MIOC_EINVAL, "heat: bad K / x");
  if (hipSetDevice(ctx->device) != hipSuccess) return heat_fail(ctx, MIOC_EHIP, "hipSetDevice failed");
  const int64_t tiles = (K + 15) / 16;
  const size_t need = (size_t)tiles * h->nt * h->Np * 16 * sizeof(double);
  if (d_df && h->gy_cap < need) {
    if (h->d_gy) hipFree(h->d_gy), h->d_gy = nullptr, h->gy_cap = 0;
    if (hipMalloc(reinterpret_cast<void **>(&h->d_gy), need) != hipSuccess) {
      (void)hipGetLastError();
      h->d_gy = nullptr;
      return heat_fail(ctx, MIOC_ENOMEM, "heat: cannot allocate the Gy scratch");
    }
    h->gy_cap = need;
  }
  HeatArgs A;
  A.sinv = reinterpret_cast<const d2 *>(h->d_sinv);
  A.sinvT = reinterpret_cast<const d2 *>(h->d_sinvT);
  A.msinv = reinterpret_cast<const d2 *>(h->d_msinv);
  A.minvF = h->d_minvF, A.state0 = h->d_state0, A.yd = h->d_yd, A.myd = h->d_myd, A.gy0 = h->d_gy0, A.g0 = h->g0;
  A.X = d_x, A.J = d_J, A.DF = d_df;
  A.GY = h->d_gy;
  A.K = (int)K, A.nx = (int)h->nx, A.nt = (int)h->nt, A.Np = (int)h->Np;
  A.tau = h->tau, A.gamma = h->gamma;
  A.gate = ctx->gate;
  A.SC = nullptr;
  if (h->Np > HMAXN_LDS) {
    const size_t sneed = (size_t)tiles * 2 * h->Np * 16 * sizeof(double);
    if (h->sc_cap < sneed) {
      if (h->d_sc) hipFree(h->d_sc), h->d_sc = nullptr, h->sc_cap = 0;
      if (hipMalloc(reinterpret_cast<void **>(&h->d_sc), sneed) != hipSuccess) {
        (void)hipGetLastError();
        h->d_sc = nullptr;
        return heat_fail(ctx, MIOC_ENOMEM, "heat: cannot allocate the state scratch");
      }
      h->sc_cap = sneed;
    }
    A.SC = h->d_sc;
  }
  const hipError_t e = launch_heat(ctx->stream, A, (int)tiles);
  if (e != hipSuccess) return heat_fail(ctx, MIOC_EHIP, std::string("k_heat_run: ") + hipGetErrorString(e));
  return MIOC_OK;
}

int32_t mioc_heat_eval(mioc_ctx *ctx, int64_t K, const double *x, double *J, double *df) {
  if (!ctx) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  HeatState *h = ctx->heat;
  if (!h || !h->ready) return heat_fail(ctx, MIOC_ESTATE, "heat: no successful mioc_heat_setup");
  if (K < 1 || K > INT32_MAX || !x || (!J && !df)) return heat_fail(ctx, MIOC_EINVAL, "heat: bad K / x / outputs");
  if (hipSetDevice(ctx->device) != hipSuccess) return heat_fail(ctx, MIOC_EHIP, "hipSetDevice failed");
  const size_t nxt = (size_t)K * h->nx * h->nt, need = (2 * nxt + K) * sizeof(double);
  if (h->io_cap < need) {
    if (h->d_io) hipFree(h->d_io), h->d_io = nullptr, h->io_cap = 0;
    if (hipMalloc(reinterpret_cast<void **>(&h->d_io), need) != hipSuccess) {
      (void)hipGetLastError();
      h->d_io = nullptr;
      return heat_fail(ctx, MIOC_ENOMEM, "heat: cannot allocate the host-entry staging");
    }
    h->io_cap = need;
  }
  double *dx = h->d_io, *ddf = h->d_io + nxt, *dJ = h->d_io + 2 * nxt;
  if (hipMemcpyAsync(dx, x, nxt * sizeof(double), hipMemcpyHostToDevice, ctx->stream) != hipSuccess)
    return heat_fail(ctx, MIOC_EHIP, "heat: x copy-in failed");
  int rc = mioc_heat_eval_device(ctx, K, dx, J ? dJ : nullptr, df ? ddf : nullptr);
  if (rc) return rc;
  if (J && hipMemcpyAsync(J, dJ, K * sizeof(double), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
    return heat_fail(ctx, MIOC_EHIP, "heat: J copy-out failed");
  if (df && hipMemcpyAsync(df, ddf, nxt * sizeof(double), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
    return heat_fail(ctx, MIOC_EHIP, "heat: df copy-out failed");
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) return heat_fail(ctx, MIOC_EHIP, "hipStreamSynchronize failed");
  return MIOC_OK;
}

}  // extern "C"
