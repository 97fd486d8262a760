/*
 * mioc.h -- C ABI of libmioc, the MI355X (gfx950) implementation of the reference's DP
 * trust-region subproblem.
 *
 * The reference (Julia, Jonas477/mixed-integer-optimal-control---algorithm-tools) has no FFI; the
 * entry points below are what a `ccall` glue for its hot path binds (INTEGRATION.md shows the Julia
 * stubs).  Each entry cites the reference interface it replaces.
 *
 * Conventions
 *   - every call returns an int32 status (MIOC_OK == 0, negative on error); no C++ exception
 *     crosses the ABI; mioc_last_error(ctx) returns a NUL-terminated description;
 *   - host arrays are borrowed for the duration of a synchronous call only, column-major
 *     (Julia layout): df[m + nx*i], u[m + nx*i], 0 <= m < nx, 0 <= i < nt;
 *   - a context owns all device memory (value fronts, the compact argmin table, level tables) and
 *     keeps the DP resident between mioc_bellman and mioc_backtrack, so the trust-region halving
 *     path (multi-trust.jl:108-110) costs only a backtrack;
 *   - a context is not thread-safe; distinct contexts may be used concurrently; every call first
 *     selects the context's device (HIP's current device is per host thread).
 */
#ifndef MIOC_H
#define MIOC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes --------------------------------------------------------------------------- */
#define MIOC_OK 0
#define MIOC_EINVAL -1      /* bad argument / shape */
#define MIOC_EINEXACT -2    /* |nu - u_old| not integral: the reference's InexactError,
                               HelpFunctions.jl:37,57 (convert(Int64, ...)) */
#define MIOC_ENOMEM -3      /* device allocation failed */
#define MIOC_EHIP -4        /* HIP runtime error */
#define MIOC_EINFEASIBLE -5 /* no finite value within the budget; the reference would read an
                               unwritten U cell at HelpFunctions.jl:116 */
#define MIOC_ESTATE -6      /* call order violated (e.g. backtrack before bellman, B_use > B) */
#define MIOC_ENONFINITE -7  /* non-finite gradient entry */

/* ---- switching-cost kinds: beta * (sum_m |nu_jm - nu_lm|^p)^(1/p), HelpFunctions.jl:63-67 ----- */
#define MIOC_P_INF 0    /* p = Inf: the reference evaluates (sum |d|^Inf)^(1/Inf) == x^0.0 == 1.0, so
                           every transition (including "no switch") costs beta.  Reproduced. */
#define MIOC_P_ONE 1    /* p = 1: weight = sum_m |d_m| (exact integer) */
#define MIOC_P_INTLUT 2 /* integer p >= 2: weight = table[sum_m |d_m|^p]; the host supplies Julia's
                           Float64(S)^(1/p) for S = 0..table_len-1 */
#define MIOC_P_TABLE 3  /* any p: weight = table[rank_l * L + rank_j] (L*L host-supplied weights) */

/* ---- algorithm selection (mioc_set_option(MIOC_OPT_ALGO, ...)) ----------------------------- */
#define MIOC_OPT_ALGO 1
#define MIOC_ALGO_AUTO 0    /* p=Inf -> class collapse; p=1, beta>0 on an 8^3 or 8^4 product grid ->
                               separable transform; small state (front fits one CU's LDS) -> fused;
                               other large product grids at p=1 -> pyramid; otherwise the generic
                               min-plus sweep */
#define MIOC_ALGO_GENERIC 1 /* per-step min-plus sweep over every (c, l, j): any p */
#define MIOC_ALGO_PINF 2    /* exact p=Inf collapse onto per-budget row minima */
#define MIOC_ALGO_PYRAMID 3 /* p=1 on product grids of consecutive levels: exact L1-ball pyramid */
#define MIOC_ALGO_SEPARABLE 4 /* p=1, beta>0, 8^3 / 8^4 product grid of consecutive levels: separable L1
                                 distance transform in exact fixed point with a certified argmin */
#define MIOC_ALGO_FUSED 5   /* whole DP of each subproblem in ONE workgroup with the value front in LDS
                               (any p; L <= 64, small B): the batch path for small-state problems */
#define MIOC_ALGO_FUSED_SEPARABLE 6 /* the fused DP with the separable L1 transform of MIOC_ALGO_SEPARABLE:
                                       p=1, beta>0, 2-D product grid of consecutive integer levels
                                       (6x6, 4x4, 8x8, 8x4), B < 512 */
#define MIOC_OPT_TIMING 2   /* 1: record HIP events around the dominant kernel (mioc_kernel_stats) */
#define MIOC_OPT_PERSIST 3  /* separable transform: 1 (default) runs the whole DP as one persistent launch
                               whose workgroups hand rows to each other; 0: one launch per step */
#define MIOC_OPT_PRED_FMA 4 /* mioc_pred*: 1 accumulates each ∇f[:,j]'(u_old[:,j] - u[:,j]) with fma, as an
                               FMA-contracted BLAS ddot does; 0 (default): products rounded, then added */
#define MIOC_OPT_SPIN_LIMIT 5 /* separable transform, persistent launch: polls a dependency wait may take
                                 before the launch is abandoned and the DP redone with per-step launches
                                 (default 2^24; a tiny value forces that fallback, for tests) */
#define MIOC_OPT_SDT_BUFFERS 6 /* persistent separable transform: staging buffers (4..256, default 256; more
                                  buffers let rows run further apart, which hides the row hand-off; cut to
                                  the most that keep a subproblem's staging region under 4 GiB; raised to
                                  7·M + 1 (29 on 8^4 grids): with fewer, a row's write-after-read wait can
                                  close a cycle with the one-row-ahead waits of the rows below it, so the DP
                                  would deadlock -- a problem where 7·M + 1 do not fit runs per step) */
#define MIOC_OPT_FSEP_SEGMENTS 7 /* fused separable DP: row segments per subproblem, each on its own workgroup
                                    (0, default: chosen from the batch size -- more than one only when the
                                    batch alone cannot fill the GPU; 1..8: forced; -1: the one-lane-per-row
                                    kernel of mioc_fused.hip) */
#define MIOC_OPT_PINF_WALK 8 /* p=Inf backtrack: 0 (default) the segmented walk -- one subproblem's path spread
                                over many workgroups -- for batches of at most 64 subproblems with >= 512 steps,
                                else one serial walk per subproblem; 1: segmented walk forced; -1: serial walk */
/* option 9 (a two-workgroups-per-row separable driver, opt-in and slower) was removed in round 6: MIOC_EINVAL */

typedef struct mioc_ctx mioc_ctx;

const char *mioc_version(void);

/* Create / destroy a context on HIP device `device`. */
int32_t mioc_create(int32_t device, mioc_ctx **out);
int32_t mioc_destroy(mioc_ctx *ctx);
const char *mioc_last_error(const mioc_ctx *ctx);
int32_t mioc_set_option(mioc_ctx *ctx, int32_t option, int64_t value);

/*
 * Flattened admissible-level iterator: replaces `obj.𝓥` + `obj.iterator`
 * (product_iterator / bounded_sum_iterator, julia_opt/AdmissibleIterators.jl:9-49) as consumed by
 * bellman_TRM! (HelpFunctions.jl:29,49,60) and eval_u_TRM! (HelpFunctions.jl:104-118).
 *   counts[M]          |V_m|
 *   values[sum counts] level values, V_1 then V_2 ...
 *   tuples[L*M]        admissible tuples in iterator order, tuple-major, 1-based level indices
 * The iterator order must be the grid's column-major order filtered (both reference iterators are).
 */
int32_t mioc_set_levels(mioc_ctx *ctx, int64_t M, const int64_t *counts, const int64_t *values, int64_t L,
                        const int32_t *tuples);

/*
 * Switching cost: the `β` and `p` arguments of bellman_TRM! (HelpFunctions.jl:20, :63-67),
 * TRM_parameters.β / .p (multi-trust.jl:27-28).  p_int is p for MIOC_P_INTLUT; `table` as above.
 */
int32_t mioc_set_cost(mioc_ctx *ctx, int32_t p_kind, int64_t p_int, double beta, int64_t table_len,
                      const double *table);

/*
 * bellman_TRM!(∇f, u_old, B, β, p, Δt, nu, U, Φ, iterator)  -- HelpFunctions.jl:20-83,
 * called at multi-trust.jl:112.  U and Φ live in the context (device memory), not on the host:
 * the reference layout would be 2.21 TB for nt=65536, 4096 levels, B=256.
 * Host buffers df (∇f) and u_old: nx x nt column-major.  B = floor(Δ⁰/Δt) (multi-trust.jl:69).
 */
int32_t mioc_bellman(mioc_ctx *ctx, const double *df, const double *u_old, int64_t nx, int64_t nt, int64_t B,
                     double dt);

/*
 * eval_u_TRM!(u, u_old, U, Φ, B, nu)  -- HelpFunctions.jl:98-124, called at multi-trust.jl:110,113.
 * B_use <= B of the last mioc_bellman (the halving path reuses the DP, multi-trust.jl:108-110).
 * u_out: nx x nt column-major level values (obj.x); phi_star: the minimal Φ value (nullable);
 * switch_mask: nt bytes, switch_mask[i] = (u[:,i] != u[:,i-1]), switch_mask[0] = 0 (nullable).
 */
int32_t mioc_backtrack(mioc_ctx *ctx, int64_t B_use, double *u_out, double *phi_star, uint8_t *switch_mask);

/*
 * Batched, device-resident variants (inputs already in HBM; the bench and the multi-GPU batch
 * runner use these).  K independent subproblems sharing levels, cost, nt and B (random restarts):
 *   d_df, d_u_old : K x nx x nt (subproblem-major, each nx x nt column-major), device pointers
 *   d_u_out       : K x nx x nt device pointer;  d_phi_star: K doubles (device, nullable)
 *   d_status      : K int32 (device, nullable): per-subproblem MIOC_OK / MIOC_EINFEASIBLE
 * Work is enqueued on the context's stream; call mioc_synchronize before reading results.
 */
int32_t mioc_bellman_batch_device(mioc_ctx *ctx, int64_t K, const double *d_df, const double *d_u_old,
                                  int64_t nx, int64_t nt, int64_t B, double dt);
int32_t mioc_backtrack_batch_device(mioc_ctx *ctx, int64_t B_use, double *d_u_out, double *d_phi_star,
                                    int32_t *d_status);
/* The same with one budget per subproblem: d_B_use[k] (device, K int32, each 0 <= B_use[k] <= B) -- the
 * per-restart trust-region radii after halving (multi-trust.jl:108-110, B_new = floor(Δᵏ/Δt) per restart).
 * The budgets are validated on the device (no host read-back): a B_use[k] outside [0, B] makes d_status[k] =
 * MIOC_ESTATE and leaves subproblem k's u row NaN; the call itself returns MIOC_OK.  The first backtrack after a DP
 * whose workgroups hand rows to each other inside one launch (persistent separable DP, segmented fused separable
 * DP, segmented p=Inf recursion: small batches) synchronises the stream once, to read that DP's timeout word and
 * redo the DP if a wait timed out; later backtracks of the same DP enqueue without a synchronisation. */
int32_t mioc_backtrack_batch_budgets_device(mioc_ctx *ctx, const int32_t *d_B_use, double *d_u_out, double *d_phi_star,
                                            int32_t *d_status);
int32_t mioc_synchronize(mioc_ctx *ctx);

/*
 * The controls of the last backtrack as 0-based level ranks in iterator order (obj.iterator of
 * eval_u_TRM!, HelpFunctions.jl:110-118: u[:, i] = ν(l_i)): d_ranks_out receives K x nt int32 (device
 * pointer), enqueued on the context's stream.  The multi-GPU batch gathers these (one 16-bit rank per step
 * instead of nx level values) without recovering them from u.
 */
int32_t mioc_get_ranks_device(mioc_ctx *ctx, int32_t *d_ranks_out);

/*
 * Trust-region quantities of the last backtrack, multi-trust.jl:117-127 (pred) with TV_p of
 * HelpFunctions.jl:251-268 (p = the context's cost; p = Inf is the true max norm here, unlike the DP's cost):
 *   int_val = Δt · Σ_j ∇f[:,j]'(u_old[:,j] − u[:,j]);   tv_old = TV_p(u_old, p);   tv_new = TV_p(u, p)
 *   pred    = int_val + β·(tv_old − tv_new)
 * u is the path of the last mioc_backtrack*, ∇f and u_old those of the last mioc_bellman*.  All sums are
 * accumulated in the reference's loop order, so TV_p is bit-identical for p = 1, Inf and MIOC_P_INTLUT (the
 * summand is the host table's Julia pow) and int_val differs from the reference's BLAS dot only by its FMA use
 * (MIOC_OPT_PRED_FMA).  MIOC_P_TABLE needs both controls on the level grid (else MIOC_EINVAL).
 * Outputs are nullable.  mioc_pred: the single-subproblem (host) API, synchronous.
 * mioc_pred_batch_device: K values per output (device pointers), enqueued; errors surface at mioc_synchronize.
 */
int32_t mioc_pred(mioc_ctx *ctx, double *int_val, double *tv_old, double *tv_new, double *pred);
int32_t mioc_pred_batch_device(mioc_ctx *ctx, double *d_int_val, double *d_tv_old, double *d_tv_new, double *d_pred);

/* TV_p(u, p) of K device controls d_u (K x nx x nt, each column-major) into d_tv[K]; enqueued. */
int32_t mioc_tv_device(mioc_ctx *ctx, int64_t K, const double *d_u, int64_t nx, int64_t nt, double *d_tv);

/*
 * The trust-region step decision of multi-trust.jl:127-158 per subproblem, on the device:
 *   ared = J_old − J_new + β·(tv_old − tv_new);   decision = 2 if pred <= 0 (stop: optimal),
 *   1 if ared < σ·pred (bad step: halve Δ), else 0 (good step: accept).  d_ared nullable; enqueued.
 */
/*
 * Device-resident TRM control (multi-trust.jl:92-163) for K restarts, so that the host reads back one flag per
 * inner-loop chunk instead of K decisions plus stream syncs per inner iteration:
 *   mioc_trm_state_bytes(K): bytes of the zero-initialised state block the caller allocates on the device
 *     (offset 0: gate word, 4: any-active word, 8: copy word; then K doubles Δᵏ, K doubles TV_old, K int32 k,
 *     K int32 flags (1 inner, 2 halved, 4 stopped), K int32 outer iterations per restart).
 *   mioc_trm_attach(ctx, d_state): while the gate word is 0, the kernels of mioc_backtrack_batch*_device,
 *     mioc_pred_batch_device, mioc_ode_eval_device and mioc_heat_eval_device return at once; NULL detaches.
 *   mioc_trm_outer_begin_device: multi-trust.jl:99-107 (TV_old = TV_p(u), Δᵏ = Δ⁰, k = 1, budgets = B, every
 *     restart not stopped enters its inner loop; the gate opens if any did).
 *   mioc_trm_inner_end_device: multi-trust.jl:117-158 for the restarts inside their inner loop: pred (with TV_old),
 *     ared, the decision (written to d_decision if not NULL: 0 accept, 1 halve, 2 stop, -1 not in the loop),
 *     obj.x = trial, accept / halve / stop, k += 1, the next budgets; the gate stays open while any restart is
 *     inside its inner loop.  n_per_restart = nt·nx doubles of u, u_old and trial per restart.
 *   mioc_trm_poll: synchronises the stream once and returns {gate, any-active}.
 */
int64_t mioc_trm_state_bytes(int64_t K);
int32_t mioc_trm_attach(mioc_ctx *ctx, void *d_state);
int32_t mioc_trm_outer_begin_device(mioc_ctx *ctx, int64_t K, void *d_state, const double *d_tv_u, double D0,
                                    int64_t B, int32_t *d_budgets);
int32_t mioc_trm_inner_end_device(mioc_ctx *ctx, int64_t K, void *d_state, double sigma, int64_t kmax, double tau,
                                  int64_t B, const double *d_int_val, const double *d_tv_new, const double *d_J_new,
                                  double *d_J_old, double *d_J, double *d_tv_u, int32_t *d_budgets,
                                  int32_t *d_decision, int64_t n_per_restart, const double *d_trial, double *d_u,
                                  double *d_u_old);
int32_t mioc_trm_poll(mioc_ctx *ctx, const void *d_state, int32_t *out);

int32_t mioc_trm_decide_device(mioc_ctx *ctx, int64_t K, const double *d_J_old, const double *d_J_new,
                               const double *d_tv_old, const double *d_tv_new, const double *d_pred, double sigma,
                               double *d_ared, int32_t *d_decision);

/*
 * Multi-device batch from one process (SURVEY §8 b, `mioc_batch_multi`): K subproblems in host arrays (K x nx x nt,
 * each nx x nt column-major) are split into contiguous blocks over the nctx contexts -- one per device, each with
 * the same levels and cost already set -- and every block is solved on its context's device from its own host
 * thread: bellman_TRM! at B, then eval_u_TRM! at B_use (<= B).  u_out: K x nx x nt; phi_star, status: K entries
 * (nullable).  Synchronous.  On error the return is the first failing context's status, and
 * mioc_last_error(ctxs[0]) names that context.  (For one process per GPU over RCCL see INTEGRATION.md.)
 */
int32_t mioc_batch_multi(mioc_ctx *const *ctxs, int32_t nctx, int64_t K, const double *df, const double *u_old,
                         int64_t nx, int64_t nt, int64_t B, double dt, int64_t B_use, double *u_out, double *phi_star,
                         int32_t *status);

/*
 * The ODE gradient producer of the reference's TRM examples, batched on the device:
 * eval_f! / eval_df! of julia_opt/ODEObjective.jl:125-184 (explicit Euler forward, trapezoid cost, explicit-Euler
 * adjoint, df = Gu - Fu'λ) with the hooks of example_fishing.jl / example_doubletank.jl / example_vanderpol.jl.
 * d_x: K x nx x nt controls (nx = 3, the DP's input layout); d_J: K objective values (nullable); d_df: K x nx x nt
 * gradients (nullable), ready for mioc_bellman_batch_device.  τ = (T1 - T0) / nt.  params (nullable: the examples'
 * values) holds, in order: fishing α, β, γ, δ, c1, c2, v1[3], v2[3], y0[2] (14); doubletank k1, k2, c[3], y0[2] (7);
 * vanderpol c[3], y0[2] (5).  Enqueued on the context's stream.
 */
#define MIOC_ODE_FISHING 1
#define MIOC_ODE_DOUBLETANK 2
#define MIOC_ODE_VANDERPOL 3
int32_t mioc_ode_eval_device(mioc_ctx *ctx, int32_t problem, int64_t K, const double *d_x, int64_t nx, int64_t nt,
                             double T0, double T1, const double *params, int32_t nparams, double *d_J, double *d_df);

/*
 * Random admissible starts, rand_func_int (HelpFunctions.jl:204-225) on the device: K piecewise-constant controls
 * d_u_out (K x nx x nt, nx = the levels' M) with `jumps` distinct jump times drawn uniformly from steps 1..nt-1
 * (the reference's 2..nt) and a uniformly random admissible level per segment.  jumps < 0: floor(nt / 10), the
 * reference's default.  The stream is counter-based (seed, restart, draw), so a seed reproduces its controls on
 * any device; it is not Julia's MersenneTwister stream (not reproducible outside Julia).  Enqueued.
 */
int32_t mioc_rand_start_device(mioc_ctx *ctx, int64_t K, int64_t nt, int64_t jumps, uint64_t seed, double *d_u_out);

/*
 * The PDE heat objective's gradient producer, batched on the device: eval_f / eval_df of
 * julia_opt/PDEObjective.jl:129-199 (implicit-Euler state with SMatLU, trapezoid cost, implicit-Euler adjoint with
 * AMatLU = lu(StateMat'), df_i = (M⁻¹F)ᵀ p_i + Gu) with the hooks of example_heat.jl:135-161 (G = ½(y−yd)ᵀM(y−yd),
 * G_t = γ·Σx, Gu = γ).  mioc_heat_setup takes the matrices the Julia objective already holds (example_heat.jl:101-115;
 * all column-major): M_invA (N x N), M_invF (N x nx), mass = M (N x N), state0 (N), yd (N x (nt+1)); τ = (T1−T0)/nt,
 * StateMat = I + τ·M_invA is factored once on the host.  1 <= N <= 2048, 1 <= nx <= 4.  mioc_heat_eval_device:
 * d_x = K x nx x nt controls (the DP's input layout), d_J (K, nullable), d_df (K x nx x nt, nullable).  Enqueued.
 */
int32_t mioc_heat_setup(mioc_ctx *ctx, int64_t N, int64_t nx, int64_t nt, double T0, double T1, double gamma,
                        const double *M_invA, const double *M_invF, const double *mass, const double *state0,
                        const double *yd);
int32_t mioc_heat_eval_device(mioc_ctx *ctx, int64_t K, const double *d_x, double *d_J, double *d_df);
/* The same from host arrays (the Julia objective's x / df, K x nx x nt column-major; J: K), synchronous. */
int32_t mioc_heat_eval(mioc_ctx *ctx, int64_t K, const double *x, double *J, double *df);

/* The HIP stream the context enqueues on (hipStream_t), for callers that order their own work. */
void *mioc_stream(mioc_ctx *ctx);

/*
 * Kernel timing (MIOC_OPT_TIMING=1): HIP events recorded on the context's stream around the
 * launches of each kernel class.  which: 0 = dominant DP kernel of the last bellman call (generic
 * step sweep or p=Inf recursion), 2 = p=Inf class-table prep,
 * 1 = backtrack.  Returns cumulative milliseconds, launch count and the kernel's name.
 */
int32_t mioc_kernel_stats(mioc_ctx *ctx, int32_t which, double *total_ms, int64_t *launches,
                          const char **name);
int32_t mioc_reset_stats(mioc_ctx *ctx);

/* Which algorithm served the last mioc_bellman* call (MIOC_ALGO_GENERIC / _PINF / _PYRAMID). */
int32_t mioc_last_algo(mioc_ctx *ctx);

/*
 * Diagnostics of the last bellman/backtrack: counters[0] pyramid / separable-transform targets resolved by
 * the exact scan because their winning value has another source value within rounding distance, [1] pyramid
 * targets resolved by the exact scan because their minimum is reached at two levels (separable transform:
 * targets of rows sent straight to the exact scan: few targets, or a value scale outside its binade), [2] backtrack: p=Inf walk steps resolved
 * by the exact scan, or for the U-table walks (generic, pyramid) the run-ahead rounds taken (each round
 * settles up to 64 steps), [3] internal consistency failures (must be 0); [4..7] pyramid internals: rows whose
 * value hash overflowed, targets whose value was not found, values flagged as colliding (after a separable-transform
 * DP, [4] instead counts the persistent driver's rows whose write-after-read wait on the rows above was armed (a staging buffer reused while later rows may still read it), and [6] counts this context's persistent DPs redone with per-step launches: the grid does not fit, or
 * a dependency wait timed out -- 0 on a healthy run; after a fused separable DP, the segmented launches redone with
 * one workgroup per subproblem); [7] fused DP: resident workgroups per CU (occupancy query); [8] fused separable DP:
 * row segments per subproblem (0: the one-lane-per-row kernel); [9] p=Inf segmented walk: subproblems whose path
 * met a state-dependent step and were walked serially (-1: the serial walk ran for all).  n may be up to 10.
 */
int32_t mioc_diagnostics(mioc_ctx *ctx, int64_t *counters, int32_t n);

/*
 * The argmin table `U` of the last bellman call, one step at a time, in the reference's layout
 * (HelpFunctions.jl:74, U[:, c+1, l..., i+1] of multi-trust.jl:76): for subproblem k and step i
 * (0 <= i < nt-1), U_out[c + (B+1)*g] = 0-based iterator rank of the source j minimising Φ_i at budget
 * c and the target level with grid-linear index g (levels in column-major grid order), as an int32.
 * Cells the reference never writes because Φ_i = +Inf there hold -1 when c < b̃(l, i) and are
 * unspecified otherwise (the reference leaves them at whatever `U` held before); the separable transform
 * (MIOC_ALGO_SEPARABLE) reports -1 for every such cell, so its tables equal the reference's.  U_out has
 * (B+1) * prod(counts) entries.  The p=Inf collapse stores class tables instead (MIOC_EINVAL).
 */
int32_t mioc_get_argmin_table(mioc_ctx *ctx, int64_t k, int64_t step, int32_t *U_out);

#ifdef __cplusplus
}
#endif
#endif /* MIOC_H */
