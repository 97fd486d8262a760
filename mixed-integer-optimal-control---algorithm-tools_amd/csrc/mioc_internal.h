// mioc_internal.h -- context and kernel-launch declarations shared by the C ABI (mioc_api.cpp)
// and the gfx950 kernels (mioc_generic.hip, mioc_pinf.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/mioc.h"

namespace mioc {

constexpr int kMaxM = 8;          // controls per tuple supported by the kernels
constexpr int kRowTile = 64;      // budget rows per lane-tile; fronts are padded to a multiple

// Device-side view of the flattened level table + switching cost, passed by value to kernels.
struct LevelsDev {
  int M = 0;
  int L = 0;
  const double *nuval = nullptr;   // [L][M] level values per iterator rank
  const int32_t *nuint = nullptr;  // [L][M] same, as int32 (distance keys)
  const int32_t *gidx = nullptr;   // [L] grid linear index per rank (argmin tie-break)
  const int32_t *vals = nullptr;   // [Σ counts] level values per dimension, concatenated
  const int32_t *voff = nullptr;   // [M+1] offsets of each dimension's values in vals
  const int32_t *g2r = nullptr;    // [Lgrid] rank of each grid tuple (-1: not admissible); null if too large
  int p_kind = MIOC_P_INF;
  int p_int = 1;
  double beta = 0.0;
  double inv_beta = 0.0;           // fl(1/beta) for beta > 0 (separable transform scale)
  const double *costlut = nullptr; // beta*weight by integer key (P_INF: [beta], P_ONE/P_INTLUT)
  const double *costtab = nullptr; // [L][L] beta*weight (P_TABLE only)
};

// One batch of K subproblems sharing levels, cost, nt, B.
struct ProblemDev {
  int K = 0;
  int M = 0;
  int nt = 0;
  int B = 0;
  int RP = 0;                      // padded rows per front column: roundup(B+1, 64)
  double dt = 0.0;
  const double *df = nullptr;      // [K][nt][M]  (each subproblem nx x nt column-major)
  const double *uold = nullptr;    // [K][nt][M]
  const int32_t *Bvec = nullptr;   // backtrack: per-subproblem budget B'_k (null: one B' for the batch)
  const int32_t *gate = nullptr;   // device TRM control (mioc_trm_attach): backtrack kernels return at once while *gate == 0
  // the one-workgroup p = Inf recursion as the device-side redo of a segmented one: it runs only if the segmented
  // launch's error word (a timed-out wait) is set, and then counts itself in *redo_count (null: an ordinary launch)
  const int32_t *redo_gate = nullptr;
  int32_t *redo_count = nullptr;
};
// the kernels of a gated call return at once (uniformly) while the device TRM control's gate word is 0
__device__ __forceinline__ bool gate_closed(const int32_t *gate) { return gate && *gate == 0; }
// a redo launch (ProblemDev::redo_gate) returns at once unless the launch it backs up timed out
__device__ __forceinline__ bool redo_skip(const ProblemDev &P) {
  if (!P.redo_gate) return false;
  if (*P.redo_gate == 0) return true;
  if (P.redo_count && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) atomicAdd(P.redo_count, 1);
  return false;
}

// Product grid with consecutive integer levels per dimension (the L1-ball pyramid's domain).
struct PyrGeom {
  int M = 0;
  int ncol = 0;                    // grid columns: L / n[0]
  int Smax = 0;                    // largest L1 distance: sum_m (n_m - 1)
  int n[kMaxM] = {};               // levels per dimension
  int base[kMaxM] = {};            // first level value per dimension
  int cstride[kMaxM] = {};         // column-index stride of dimension m >= 1
};

struct Start {                      // backtrack start cell per subproblem
  double phi;
  int32_t c;
  int32_t r;
  int32_t status;
  int32_t pad;
};

// The backtrack budget of subproblem k: the per-subproblem B'_k when the call passed a device vector
// (mioc_backtrack_batch_budgets_device), else the call's B'.  A B'_k outside [0, B] is checked here, on the device,
// so that the call needs no host read-back of the budgets: the start kernel records MIOC_ESTATE as the
// subproblem's status (its u row becomes NaN in k_expand, the walk skips it) and returns -1.
__device__ __forceinline__ int start_budget(const ProblemDev &P, int k, int Bu, Start *start) {
  if (!P.Bvec) return Bu;
  const int b = P.Bvec[k];
  if (b >= 0 && b <= P.B) return b;
  if (threadIdx.x == 0) {
    Start st;
    st.phi = __builtin_nan("");
    st.c = 0;
    st.r = -1;
    st.status = MIOC_ESTATE;
    st.pad = 0;
    start[k] = st;
  }
  return -1;
}

// ---- kernel launchers (mioc_generic.hip) ------------------------------------------------------
hipError_t launch_validate(hipStream_t s, const ProblemDev &P, const double *numin, const double *numax,
                           int32_t *flags);
hipError_t launch_generic_terminal(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, double *front,
                                   size_t front_stride);
hipError_t launch_generic_step(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, int i,
                               const double *psi, double *phi, void *U, int ubytes, size_t front_stride,
                               size_t u_stride_k);
hipError_t launch_generic_argmin0(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const double *front0,
                                  size_t front_stride, int Bu, Start *start);
hipError_t launch_uold_rank(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, int32_t *urank);
hipError_t launch_generic_walk(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const void *U, int ubytes,
                               size_t u_stride_k, const Start *start, const int32_t *urank, int32_t *ranks,
                               int32_t *counters);
hipError_t launch_expand(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const Start *start,
                         const int32_t *ranks, double *u_out, double *phi_star, int32_t *status);

// ---- L1-ball pyramid (mioc_pyramid.hip) + staging-layout backtrack (mioc_generic.hip) -------------
// same2 (nullable): [K][nt] int32, u_old(s) == u_old(s + 2) bit for bit (0 for s >= nt - 2); strad (nullable):
// [K][nt][8 waves][32] uint16, per wave of the persistent separable driver the in-wave offsets of the second elements
// of seam-straddling position pairs
// counters (nullable): [3] += seams a wave's list could not hold (an internal-consistency failure, must stay 0)
// k_pinf_recur_ws's segment flags: this many 32-bit words apart (packed, one line held all 13 segments' flags of
// C2 / C3; 128 bytes apart the single-subproblem recursion is 2-3 % faster, profiles/round6_flag_stride.txt); the
// segmented p = Inf kernels' error word sits at K · pinf_recur_segments · this (k_pinf_recur_mc / _mcw keep their
// flags packed: spaced out, _mcw was 6 % slower)
#ifndef PINF_WS_FLAG_STRIDE
#define PINF_WS_FLAG_STRIDE 32
#endif
// k_fsep2's segment records {outbox token, consumed token}: this many 32-bit words apart (>= 2)
#ifndef FSEP_FLAG_STRIDE
#define FSEP_FLAG_STRIDE 2
#endif
// k_sdt_run's row flags (done, loaded): this many 32-bit words apart.  Packed (1), one 128-byte line carried the flags
// of 32 rows, each stored every item by its own row and polled by the 28 rows around it; 32-byte spacing is 2 % faster
// at full C4 and cuts the run-to-run spread (7.02-7.28 -> 6.94-7.03 us per DP step, profiles/round6_flag_stride.txt)
#ifndef SDT_FLAG_STRIDE
#define SDT_FLAG_STRIDE 8
#endif
hipError_t launch_pyr_order(hipStream_t s, const ProblemDev &P, const PyrGeom &G, uint32_t *perm,
                            int32_t *same2 = nullptr, uint16_t *strad = nullptr, int32_t *counters = nullptr);
hipError_t launch_pyr_terminal(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const uint32_t *perm, double *S,
                               size_t s_stride);
hipError_t launch_pyr_step(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G, int i,
                           const uint32_t *perm, const double *Sin, double *Sout, uint16_t *UU, size_t s_stride,
                           size_t uu_stride_k, int32_t *counters);
size_t pyr_lds_bytes(const PyrGeom &G);
// separable L1 transform (mioc_sdt.hip): same staging layout, 8^M grids (M = 3, 4), beta > 0
bool sdt_supported(const PyrGeom &G);
bool sdt_seam_lists(const PyrGeom &G);  // the persistent driver loads straddling pair elements by seam lists (k_pyr_order)
size_t sdt_lds_bytes(const PyrGeom &G);
constexpr int kSdtMaxBuffers = 256;  // persistent separable transform: staging buffers S_i, step i in buffer i % NB
constexpr int kSdtDefaultBuffers = 256;  // at most (C4: 255 x 8.4 MB + the 2.1 GB row-0 array fit the 4 GiB buffer range)
hipError_t launch_sdt_step(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G, int i,
                           const uint32_t *perm, const double *Sin, double *Sout, uint16_t *UU, size_t s_stride,
                           size_t uu_stride_k, int32_t *counters);
// persistent driver: per subproblem one region of kstride doubles = NB staging buffers of (B+1)·L, then row 0 of
// every step (nt·L, at r0off); k_sdt_chain + k_sdt_row0 fill row 0, its U rows and S_0 row 0, then k_sdt_run
hipError_t launch_sdt_prep(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G,
                           const uint32_t *perm, double *V, double *S, size_t kstride, size_t r0off, uint16_t *UU,
                           size_t uu_stride_k);
// same2[k][s] = (u_old(s) == u_old(s + 2)), written by launch_pyr_order: the persistent driver's sphere-order reuse
hipError_t launch_sdt_run(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G,
                          const uint32_t *perm, const int32_t *same2, const uint16_t *strad, double *S, size_t kstride,
                          int NB, uint16_t *UU,
                          size_t uu_stride_k, int32_t *counters, int32_t *flags, int nwg, unsigned spin_limit,
                          size_t lds);
int sdt_run_blocks_per_cu(const PyrGeom &G, size_t lds);
hipError_t launch_stage_argmin0(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const uint32_t *perm,
                                const double *S0, size_t s_stride, int Bu, Start *start);
hipError_t launch_stage_walk(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const uint16_t *UU,
                             size_t uu_stride_k, const Start *start, const int32_t *urank, int32_t *ranks,
                             int32_t *counters);

// ---- fused small-state DP (mioc_fused.hip): one workgroup per subproblem, front in LDS -------------
bool fused_supported(int L, int B, size_t *lds_out);
hipError_t launch_fused_run(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, double *front0,
                            size_t front_stride, uint8_t *U, size_t u_stride_k);
// p = 1 on a 2-D product grid of consecutive levels: the fused DP with the separable L1 transform
bool fsep_supported(const PyrGeom &G, int B, size_t *lds_out, int *threads_out);
int fused_blocks_per_cu(int algo_sep, const PyrGeom &G, int L, int B);  // occupancy query (diagnostics [7])
hipError_t launch_fsep_run(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G, double *front0,
                           size_t front_stride, uint8_t *U, size_t u_stride_k, int32_t *counters);
// ... round-3 layout (mioc_fsep.hip): two lanes per row, the front updated in place, optionally S row segments per
// subproblem on S workgroups chained by an outbox ring (strong scaling)
struct FsepPlan {
  int S = 1, RS = 0, W = 0;  // segments, rows per segment (multiple of 32), waves per workgroup
  int rows = 0, koff = 0;    // LDS front rows, K table offset (doubles)
  int stg = 0, slot_bytes = 0;  // S > 1: inbox staging offset (doubles), ring slot bytes
  int threads = 0;
  int lanes = 2;  // lanes per budget row (4: row segments of small batches)
  size_t lds = 0;
};
bool fsep2_plan(const PyrGeom &G, int B, int S, FsepPlan *out);
int fsep2_blocks_per_cu(const PyrGeom &G, const FsepPlan &p);
hipError_t launch_fsep2(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PyrGeom &G, const FsepPlan &p,
                        double *front0, size_t front_stride, uint8_t *U, size_t u_stride_k, int32_t *counters,
                        double *ring, int NB, int32_t *flags, unsigned spin_limit);

// ---- p = Inf collapse (mioc_pinf.hip) -----------------------------------------------------------
struct PinfDev {
  int BW = 0;                      // budget classes tracked: bmax+1 <= B+1
  int BWP = 0;                     // padded class-row width: pow2 >= max(8, BW) (pad = +Inf / -1)
  double *kmin = nullptr;          // [K][nt][BWP] min over ranks of class b of K_r (T1 at terminal)
  double *k2 = nullptr;            // [K][nt][BWP] second-smallest distinct value in the class
  int32_t *kfirst = nullptr;       // [K][nt][BWP] first rank attaining kmin
  double *R = nullptr;             // [K][nt][RP] row minima R_i[c] = min_r Φ_i[c, r]
  double *kabs = nullptr;          // [K][nt] max |K_l(i)| over the levels of classes < BW (rounding bound)
  int CH = 0, W = 0;               // the walk's staged steps per chunk and LDS row width (pinf_plan)
  // segmented walk (mioc_pinf.hip): the step's winning class per row, when it does not depend on the state
  uint8_t *ftab = nullptr;         // [K][nt][RP] class b* of row c' at step j, 0xFF: state-dependent / +Inf
  int32_t *fseg = nullptr;         // [K][nseg][RP] row after the G steps of segment g entered at row c' (-1: none)
  int32_t *fneed = nullptr;        // [K + 1] 1: subproblem left to the serial walk; [K]: their count
};
// the walk's chunk and band for a p = Inf problem (mioc_pinf.hip)
void pinf_plan(int RP, int nt, PinfDev &D);
hipError_t launch_pinf_prep(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PinfDev &D);
// ncu: the device's CUs; flags (K·ceil((B+1)/32) + 1 zeroed words, or null): lets few subproblems run in row segments
// on several CUs, *segmented then says so (the caller checks the error word after it, check_run)
// variant (nullable): the name of the recursion kernel launched (k_pinf_recur_mc, k_pinf_recur_xr or k_pinf_recur),
// which names the timing window (mioc_kernel_stats)
hipError_t launch_pinf_recur(hipStream_t s, const ProblemDev &P, const PinfDev &D, int ncu, int32_t *flags,
                             unsigned spin_limit, bool *segmented, const char **variant = nullptr);
int pinf_recur_segments(const ProblemDev &P);  // row segments of k_pinf_recur_mc per subproblem (its error word's offset)
hipError_t launch_pinf_start(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PinfDev &D, int Bu,
                             Start *start, int32_t *zero2 = nullptr, int32_t *fneed = nullptr);
hipError_t launch_pinf_walk(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PinfDev &D,
                            const Start *start, int32_t *ranks, int32_t *nfallback, const int32_t *need);
// segmented walk: steps per segment and segment count for nt steps
void pinf_fplan(int nt, int *G, int *nseg);
hipError_t launch_pinf_fwalk(hipStream_t s, const ProblemDev &P, const LevelsDev &Lv, const PinfDev &D,
                             const Start *start, int32_t *ranks);


// ---- trust-region quantities around the DP (mioc_trm.hip) ---------------------------------------
struct TrmDev {
  int K = 0, M = 0, nt = 0, L = 0;
  double dt = 0.0, beta = 0.0;
  int p_kind = MIOC_P_ONE, p_int = 1;
  int mode = 0;                    // 1: int_val, 2: TV(u_old), 4: TV(u)
  int fma = 0;                     // int_val accumulated with fma (MIOC_OPT_PRED_FMA)
  const double *df = nullptr;      // [K][nt][M]
  const double *uold = nullptr;    // [K][nt][M]
  const double *u = nullptr;       // [K][nt][M] control values, or null: the levels of `ranks`
  const int32_t *ranks = nullptr;  // [K][nt] iterator ranks of u (u == null)
  const double *nuval = nullptr;   // [L][M]
  const int32_t *vals = nullptr, *voff = nullptr, *g2r = nullptr;  // grid lookup (MIOC_P_TABLE)
  const double *tvw = nullptr;     // unscaled weights: by key (MIOC_P_INTLUT) or [L][L] (MIOC_P_TABLE)
  long long tvw_len = 0;
  double *out_int = nullptr, *out_told = nullptr, *out_tnew = nullptr, *out_pred = nullptr;  // [K] each
  int32_t *err = nullptr;          // bit 0: a TV key / rank outside the weight table
  const int32_t *gate = nullptr;   // device TRM control gate (see ProblemDev::gate)
};
hipError_t launch_trm_pred(hipStream_t s, const TrmDev &T);
hipError_t launch_trm_decide(hipStream_t s, int K, const double *J_old, const double *J_new, const double *tv_old,
                             const double *tv_new, const double *pred, double beta, double sigma, double *ared,
                             int32_t *decision);

hipError_t launch_rand_start(hipStream_t s, int K, int nt, int jumps, uint64_t seed, const LevelsDev &Lv, double *U);
// device-resident TRM control (mioc_trm.hip)
size_t trm_state_bytes(int K);
hipError_t launch_trm_outer_begin(hipStream_t s, int K, void *state, const double *tv_u, double D0, int B,
                                  int32_t *budgets);
hipError_t launch_trm_inner_end(hipStream_t s, int K, void *state, double beta, double sigma, int kmax, double tau,
                                int B, const double *int_val, const double *tv_new, const double *J_new,
                                double *J_old, double *J, double *tv_u, int32_t *budgets, int32_t *decision,
                                size_t n, const double *trial, double *u, double *u_old);
hipError_t launch_ode_eval(hipStream_t s, const int32_t *gate, int problem, int K, int nt, double tau, const double *params, int y0off,
                           const double *X, double *J, double *DF, double *ST);

// orders the context's stream after its in-flight p = Inf backtracks (mioc_api.cpp); every C ABI call that is not a
// bellman or a backtrack calls it first
int join_bt(mioc_ctx *ctx);
#define MIOC_JOIN_BT(ctx)                         \
  do {                                            \
    const int rcj_ = mioc::join_bt(ctx);          \
    if (rcj_) return rcj_;                        \
  } while (0)

struct HeatState;  // mioc_heat.hip: the PDE heat objective's device matrices (mioc_heat_setup)
void heat_free(HeatState *h);

}  // namespace mioc

// ---- the context ----------------------------------------------------------------------------------
struct mioc_ctx {
  int device = 0;
  int ncu = 0;  // the device's compute units (cached on first use)
  hipStream_t stream = nullptr;
  std::string err;
  int64_t opt_algo = MIOC_ALGO_AUTO;
  bool timing = false;

  // levels (host copies + device tables)
  bool have_levels = false;
  int64_t M = 0, L = 0, Lgrid = 0;
  std::vector<int64_t> counts, values;
  std::vector<int32_t> tuples;     // [L][M] 1-based
  std::vector<double> nuval_h;     // [L][M]
  std::vector<int32_t> gidx_h;     // [L] grid-linear index of each admissible tuple
  std::vector<double> numin_h, numax_h;
  double *d_nuval = nullptr;
  int32_t *d_nuint = nullptr;
  int32_t *d_gidx = nullptr;
  int32_t *d_vals = nullptr, *d_voff = nullptr, *d_g2r = nullptr;
  double *d_numin = nullptr, *d_numax = nullptr;

  // cost
  bool have_cost = false;
  int32_t p_kind = MIOC_P_INF;
  int64_t p_int = 1;
  double beta = 0.0;
  std::vector<double> table;
  double *d_costlut = nullptr;
  double *d_costtab = nullptr;
  double *d_tvw = nullptr;         // unscaled weight table for TV_p (MIOC_P_INTLUT / MIOC_P_TABLE)
  int64_t tvw_len = 0;
  bool pred_fma = false;           // MIOC_OPT_PRED_FMA
  double *d_pred_own = nullptr;    // mioc_pred staging: 4 doubles, then the TV error flag (int32)
  bool trm_pending = false;
  const int32_t *Bvec = nullptr;   // per-subproblem B' of the running backtrack (mioc_backtrack_batch_budgets_device)
  double *d_ode_state = nullptr;   // [K][nt][2] forward states of mioc_ode_eval_device
  size_t ode_cap = 0;
  mioc::HeatState *heat = nullptr; // mioc_heat_setup / mioc_heat_eval_device
  int64_t costlut_len = 0;

  // owned problem inputs (device)
  double *d_df = nullptr, *d_uold = nullptr;
  size_t in_cap = 0;               // doubles per array

  // last DP
  bool have_dp = false;
  int algo = 0;
  int K = 0, nt = 0, B = 0, RP = 0;
  double dt = 0.0;

  // pyramid (p = 1, product grid, unit gaps)
  bool pyr_ok = false;
  bool grid_ok = false;            // product grid of consecutive integer levels in grid order (PyrGeom valid)
  mioc::PyrGeom pyr;
  double *d_stage = nullptr;       // [2][K][B+1][L] source-row-major fronts, each row in sphere order
  size_t stage_cap = 0;
  uint32_t *d_perm = nullptr;      // [K][nt][L] sphere order of u_old(i): rank | (L1 distance << 16)
  int32_t *d_same2 = nullptr;      // [K][nt] u_old(i) == u_old(i+2) (the persistent separable driver's order reuse)
  size_t same2_cap = 0;
  uint16_t *d_strad = nullptr;     // [K][nt][8][32] seam-straddling pairs per wave (k_sdt_run's 8-wave layout)
  size_t strad_cap = 0;
  size_t perm_cap = 0;
  bool opt_persist = true;         // separable transform: one persistent launch (MIOC_OPT_PERSIST)
  bool force_steps = false;        // redo of a persistent DP whose waits timed out: per-step launches
  int64_t n_persist_fallbacks = 0; // persistent DPs redone with per-step launches (mioc_diagnostics slot 6 after a separable DP)
  int32_t *d_runflags = nullptr;   // persistent DP: [K][B+1] done, [K][B+1] loaded, err
  double *d_chain = nullptr;       // persistent DP: V[k][i] = Φ_i[j0(i), 0], the row-0 chain (k_sdt_chain)
  size_t chain_cap = 0;
  unsigned spin_limit = 1u << 24;  // persistent DP: polls before a dependency wait gives up (MIOC_OPT_SPIN_LIMIT)
  size_t stage_kstride = 0;        // doubles between two subproblems' staging blocks in the last pyramid / sdt DP
  int opt_nb = mioc::kSdtDefaultBuffers;  // staging buffers of a persistent separable DP (MIOC_OPT_SDT_BUFFERS)
  const int32_t *gate = nullptr;   // device TRM control (mioc_trm_attach): the state block's gate word
  int32_t *h_trm_poll = nullptr;   // pinned: the gate and any-active words (mioc_trm_poll)
  int opt_fsep_seg = 0;            // fused separable DP: row segments (MIOC_OPT_FSEP_SEGMENTS)
  double *d_ring = nullptr;        // fused separable DP, S > 1: the segments' outbox rings
  size_t ring_cap = 0;
  int32_t *d_segflags = nullptr;   // ... and their flags (+ err)
  size_t segflag_cap = 0;
  int last_fsep_seg = 0;           // segments of the last fused separable launch (0: the mioc_fused.hip kernel)
  size_t runflag_cap = 0;
  int32_t *h_run_err = nullptr;    // pinned copy of err
  bool run_pending = false;
  int32_t *d_counters = nullptr;   // [8] diagnostics: value-collision targets, multi-level targets, ...
  int64_t occupancy = 0;           // diagnostics [7]: resident workgroups per CU of the last fused launch

  // generic buffers
  double *d_front = nullptr;       // [2][K][L][RP]
  size_t front_cap = 0;            // bytes
  void *d_U = nullptr;             // [K][nt-1][L][B+1] uint8 / uint16
  size_t U_cap = 0;                // bytes
  int ubytes = 1;

  // p = Inf buffers
  mioc::PinfDev pinf;
  size_t pinf_cap_k = 0, pinf_cap_R = 0, pinf_cap_kabs = 0, pinf_cap_ftab = 0, pinf_cap_fseg = 0, pinf_cap_fneed = 0;
  int opt_pinf_walk = 0;           // p = Inf backtrack: 0 auto, 1 segmented walk, -1 serial (MIOC_OPT_PINF_WALK)
  bool last_pinf_fwalk = false;    // the last p = Inf backtrack ran the segmented walk

  // backtrack scratch
  bool have_path = false;          // d_ranks holds the controls of the last backtrack
  mioc::Start *d_start = nullptr;
  int32_t *d_ranks = nullptr;      // [K][nt] level ranks of the path, then [K][nt] ranks of u_old
  size_t ranks_cap = 0;
  int32_t *d_flags = nullptr;      // [4] validation flags / counters
  int32_t *h_flags = nullptr;      // pinned mirror
  double *d_uout_own = nullptr;    // host-API backtrack output staging
  double *d_phistar_own = nullptr;
  int32_t *d_status_own = nullptr;
  size_t uout_cap = 0;

  // p = Inf backtrack overlapping the next DP: it runs on bstream (the next bellman's kernels on `stream` meanwhile),
  // so every DP owns one of two slots of its inputs and p = Inf tables (the backtrack of DP n reads slot n % 2 while
  // DP n + 1 writes the other).  ev_bt[s]: the last backtrack that read slot s (the bellman that reuses s waits on it);
  // join_bt orders `stream` after the backtracks before any other call reads their outputs.
  hipStream_t bstream = nullptr;
  hipEvent_t ev_dp = nullptr, ev_bt[2] = {nullptr, nullptr};
  bool bt_rec[2] = {false, false};
  bool bt_pending = false;
  int bt_last = 0;
  int slot = 0;  // the last bellman's slot
  struct Slot {
    double *df = nullptr, *uold = nullptr;
    size_t in_cap = 0;
    double *kmin = nullptr, *k2 = nullptr, *R = nullptr, *kabs = nullptr;
    int32_t *kfirst = nullptr;
    size_t cap_k = 0, cap_R = 0, cap_kabs = 0;
  } slots[2];

  // timing
  struct EvPair {
    hipEvent_t begin = nullptr, end = nullptr;
    int64_t launches = 0;
  };
  std::vector<EvPair> ev_pool, ev_pending[4];
  EvPair ev_open[4];
  double stat_ms[4] = {};
  int64_t stat_launches[4] = {};
  const char *stat_name[4] = {"", "", "", ""};
};
