/*
 * mioc_oracle.c -- CPU restatement of the reference's DP trust-region subproblem.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (the HIP library, the Python host mirror)
 * links, loads or calls this file.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / CPU baseline.
 *
 * Parity status: the reference is Julia 1.10 (Manifest.toml:3); there is no Julia toolchain in
 * this image and the reference has no tests for this path, so this restatement is
 * "parity unpinned" by the reference itself.  It is pinned instead by
 *   (1) an exhaustive-enumeration known-answer test on dyadic inputs (tests/test_oracle.py),
 *   (2) an independent pure-Python scalar twin (oracle/oracle.py) cross-checked bit for bit,
 *   (3) the TV_p docstring vectors of HelpFunctions.jl:235-249.
 *
 * Every loop below follows the reference line by line (1-based Julia indices restated 0-based):
 *   bellman_TRM!   HelpFunctions.jl:20-83
 *   eval_u_TRM!    HelpFunctions.jl:98-124
 *   TV_p           HelpFunctions.jl:251-268
 * Compile with -ffp-contract=off: Julia emits no FMA for these expressions.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* switching-cost kinds, identical to include/mioc.h */
#define OR_P_INF 0   /* p = Inf:  (sum |d|^Inf)^(1/Inf) == 1.0 for every pair, HelpFunctions.jl:63-67 */
#define OR_P_ONE 1   /* p = 1:    sum |d| (exact integer) */
#define OR_P_INTLUT 2 /* integer p >= 2: weight = lut[sum |d|^p] (host supplies Julia's S^(1/p)) */
#define OR_P_TABLE 3 /* any p: weight = table[rank_l * L + rank_j] (host supplies the pair weights) */

#define OR_OK 0
#define OR_EINVAL -1
#define OR_EINEXACT -2 /* reference: InexactError from convert(Int64, ...) at HelpFunctions.jl:37,57 */
#define OR_EINFEASIBLE -5

typedef struct {
    int64_t M;
    const int64_t *counts; /* |V_m| */
    const int64_t *values; /* concatenated level values, V_1 then V_2 ... */
    int64_t L;             /* number of admissible tuples (iterator length) */
    const int32_t *tuples; /* L x M, tuple-major, 1-based level indices, iterator order */
} or_levels;

static int64_t level_off(const or_levels *lv, int64_t m) {
    int64_t o = 0;
    for (int64_t k = 0; k < m; ++k) o += lv->counts[k];
    return o;
}

/* grid linear index of a tuple (first index fastest, 0-based) -- Julia column-major order */
static int64_t grid_index(const or_levels *lv, const int32_t *t) {
    int64_t g = 0, stride = 1;
    for (int64_t m = 0; m < lv->M; ++m) {
        g += (int64_t)(t[m] - 1) * stride;
        stride *= lv->counts[m];
    }
    return g;
}

static int64_t grid_size(const or_levels *lv) {
    int64_t s = 1;
    for (int64_t m = 0; m < lv->M; ++m) s *= lv->counts[m];
    return s;
}

/* convert(Int64, abs(x)) with the InexactError of the reference */
static int to_int_exact(double x, int64_t *out) {
    double a = fabs(x);
    if (!(a == floor(a)) || a > 9.0e15) return OR_EINEXACT;
    *out = (int64_t)a;
    return OR_OK;
}

static int64_t ipow(int64_t a, int64_t p) {
    int64_t r = 1;
    for (int64_t k = 0; k < p; ++k) r *= a;
    return r;
}

/* beta * (sum_m |nu_jm - nu_lm|^p)^(1/p) evaluated the way HelpFunctions.jl:63-67 does */
static double switch_cost(const or_levels *lv, const int64_t *off, int32_t rl, int32_t rj, int p_kind,
                          int64_t p_int, double beta, const double *wtab, int64_t wtab_len, int *err) {
    const int32_t *l = lv->tuples + (int64_t)rl * lv->M;
    const int32_t *j = lv->tuples + (int64_t)rj * lv->M;
    double w;
    if (p_kind == OR_P_INF) {
        w = 1.0; /* x^(1/Inf) == x^0.0 == 1.0 for every x, including 0 and Inf */
    } else if (p_kind == OR_P_ONE) {
        double s = 0.0;
        for (int64_t m = 0; m < lv->M; ++m) {
            int64_t d = lv->values[off[m] + j[m] - 1] - lv->values[off[m] + l[m] - 1];
            s += (double)(d < 0 ? -d : d);
        }
        w = s; /* s^1.0 == s */
    } else if (p_kind == OR_P_INTLUT) {
        int64_t s = 0;
        for (int64_t m = 0; m < lv->M; ++m) {
            int64_t d = lv->values[off[m] + j[m] - 1] - lv->values[off[m] + l[m] - 1];
            s += ipow(d < 0 ? -d : d, p_int);
        }
        if (s < 0 || s >= wtab_len) { *err = OR_EINVAL; return 0.0; }
        w = wtab[s];
    } else {
        w = wtab[(int64_t)rl * lv->L + rj];
    }
    return beta * w;
}

/*
 * One target level rl of recursion step i (1-based, HelpFunctions.jl:49-77): reads the front r (buffer of step
 * i+1), writes column gidx[rl] of the front w and of U_i.  Different rl touch disjoint columns.
 */
static int bellman_target(const or_levels *lv, const int64_t *off, const int64_t *gidx, const double *df,
                          const double *u_old, int64_t i, int64_t B, int p_kind, int64_t p_int, double beta,
                          const double *wtab, int64_t wtab_len, double dt, const double *r, double *w, int32_t *Ui,
                          int64_t rl) {
    const int64_t M = lv->M, L = lv->L, R = B + 1;
    const int32_t *l = lv->tuples + rl * M;
    double t1 = 0.0;
    int64_t bt = 0;
    int rc;
    for (int64_t m = 0; m < M; ++m) {
        int64_t numl = lv->values[off[m] + l[m] - 1];
        t1 += dt * df[m + M * (i - 1)] * (double)numl;
        int64_t e;
        if ((rc = to_int_exact((double)numl - u_old[m + M * (i - 1)], &e)) != OR_OK) return rc;
        bt += e;
    }
    for (int64_t rj = 0; rj < L; ++rj) {
        int err = OR_OK;
        double t2 = t1 + switch_cost(lv, off, (int32_t)rl, (int32_t)rj, p_kind, p_int, beta, wtab, wtab_len, &err);
        if (err != OR_OK) return err;
        const double *rcol = r + R * gidx[rj];
        double *wcol = w + R * gidx[rl];
        int32_t *ucol = Ui + R * gidx[rl];
        for (int64_t b = 0; b <= B - bt; ++b) {
            double val = t2 + rcol[b];
            if (wcol[b + bt] > val) { /* strict: first j in iterator order wins ties */
                ucol[b + bt] = (int32_t)rj;
                wcol[b + bt] = val;
            }
        }
    }
    return OR_OK;
}

/*
 * bellman_TRM!(∇f, u_old, B, β, p, Δt, nu, U, Φ, iterator)        HelpFunctions.jl:20-83
 * phi : (B+1) x Lgrid x 2 column-major (c fastest), exactly the reference's Φ
 * U   : (B+1) x Lgrid x (n-1) column-major; stores the iterator RANK of j (the reference stores
 *       the tuple j itself; rank <-> tuple is the bijection given by `tuples`).  Cells the
 *       reference never writes keep their previous contents (callers pre-fill with -1).
 * threads > 1: the target levels of each step split over OpenMP threads (every target writes only its own columns,
 * so the result is bit-identical to threads = 1; used to generate the larger golden fixtures).
 */
static int bellman_impl(const or_levels *lv, const double *df, const double *u_old, int64_t n, int64_t B,
                        int p_kind, int64_t p_int, double beta, const double *wtab, int64_t wtab_len,
                        double dt, double *phi, int32_t *U, int threads) {
    const int64_t M = lv->M, L = lv->L, Lg = grid_size(lv), R = B + 1;
    if (n < 1 || B < 0 || M < 1 || L < 1) return OR_EINVAL;
    int64_t *off = (int64_t *)malloc(sizeof(int64_t) * M);
    int64_t *gidx = (int64_t *)malloc(sizeof(int64_t) * L);
    for (int64_t m = 0; m < M; ++m) off[m] = level_off(lv, m);
    for (int64_t k = 0; k < L; ++k) gidx[k] = grid_index(lv, lv->tuples + k * M);
    int rc = OR_OK;

    /* :27  Φ[Inds, (n+1)%2+1] .= Inf    (1-based buffer (n+1)%2+1 -> 0-based (n+1)%2) */
    {
        double *w = phi + R * Lg * ((n + 1) % 2);
        for (int64_t k = 0; k < R * Lg; ++k) w[k] = INFINITY;
        /* :29-43 terminal step i = n */
        for (int64_t rl = 0; rl < L; ++rl) {
            const int32_t *l = lv->tuples + rl * M;
            int64_t b = 0;
            double t1 = 0.0;
            for (int64_t m = 0; m < M; ++m) {
                int64_t numl = lv->values[off[m] + l[m] - 1];
                t1 += dt * df[m + M * (n - 1)] * (double)numl; /* (Δt*∇f)*numl, left to right */
                int64_t e;
                if ((rc = to_int_exact((double)numl - u_old[m + M * (n - 1)], &e)) != OR_OK) goto done;
                b += e;
            }
            if (b <= B) w[b + R * gidx[rl]] = t1;
        }
    }

    /* :45-82 recursion, i = n-1 down to 1 (1-based) */
    for (int64_t i = n - 1; i >= 1; --i) {
        double *w = phi + R * Lg * ((i + 1) % 2);  /* Φ[..., (i+1)%2+1] */
        const double *r = phi + R * Lg * (i % 2);  /* Φ[..., i%2+1]     */
        int32_t *Ui = U + R * Lg * (i - 1);
        for (int64_t k = 0; k < R * Lg; ++k) w[k] = INFINITY;
        if (threads <= 1) {
            for (int64_t rl = 0; rl < L; ++rl)
                if ((rc = bellman_target(lv, off, gidx, df, u_old, i, B, p_kind, p_int, beta, wtab, wtab_len, dt, r,
                                         w, Ui, rl)) != OR_OK)
                    goto done;
        } else {
            int bad = OR_OK; /* error codes are negative: the smallest one seen */
#pragma omp parallel for num_threads(threads) schedule(dynamic, 16) reduction(min : bad)
            for (int64_t rl = 0; rl < L; ++rl) {
                const int e = bellman_target(lv, off, gidx, df, u_old, i, B, p_kind, p_int, beta, wtab, wtab_len, dt,
                                             r, w, Ui, rl);
                if (e < bad) bad = e;
            }
            if ((rc = bad) != OR_OK) goto done;
        }
    }
done:
    free(off);
    free(gidx);
    return rc;
}

int oracle_bellman(const or_levels *lv, const double *df, const double *u_old, int64_t n, int64_t B,
                   int p_kind, int64_t p_int, double beta, const double *wtab, int64_t wtab_len,
                   double dt, double *phi, int32_t *U) {
    return bellman_impl(lv, df, u_old, n, B, p_kind, p_int, beta, wtab, wtab_len, dt, phi, U, 1);
}

int oracle_bellman_mt(const or_levels *lv, const double *df, const double *u_old, int64_t n, int64_t B,
                      int p_kind, int64_t p_int, double beta, const double *wtab, int64_t wtab_len,
                      double dt, double *phi, int32_t *U, int threads) {
    return bellman_impl(lv, df, u_old, n, B, p_kind, p_int, beta, wtab, wtab_len, dt, phi, U, threads);
}

/* Julia findmin/argmin order on Float64: NaN first (treated smallest), then isless (-0.0 < +0.0) */
static int jl_less(double a, double b) {
    int an = isnan(a), bn = isnan(b);
    if (an || bn) return an && !bn;
    if (a == b) return signbit(a) && !signbit(b);
    return a < b;
}

/*
 * eval_u_TRM!(u, u_old, U, Φ, B, nu)                               HelpFunctions.jl:98-124
 * Bp : budget used for the argmin (B' <= B allocated): the halving reuse of multi-trust.jl:108-110
 */
int oracle_backtrack(const or_levels *lv, const double *u_old, int64_t n, int64_t B, int64_t Bp,
                     const double *phi, const int32_t *U, double *u_out, double *phi_star,
                     int64_t *c_star, int64_t *g_star) {
    const int64_t M = lv->M, Lg = grid_size(lv), R = B + 1;
    if (Bp < 0 || Bp > B) return OR_EINVAL;
    int64_t *off = (int64_t *)malloc(sizeof(int64_t) * M);
    for (int64_t m = 0; m < M; ++m) off[m] = level_off(lv, m);
    /* :106 argmin(@view Φ[1:B+1, Inds, 1]): first minimum in column-major order (c fastest) */
    int64_t bc = 0, bg = 0;
    double bv = phi[0];
    for (int64_t g = 0; g < Lg; ++g)
        for (int64_t c = 0; c <= Bp; ++c) {
            double v = phi[c + R * g];
            if (jl_less(v, bv)) { bv = v; bc = c; bg = g; }
        }
    if (phi_star) *phi_star = bv;
    if (c_star) *c_star = bc;
    if (g_star) *g_star = bg;
    int rc = OR_OK;
    if (!(bv < INFINITY)) { rc = OR_EINFEASIBLE; goto out; } /* reference would read stale U */
    /* :108-112 decode the grid index into level indices */
    int32_t *lt = (int32_t *)malloc(sizeof(int32_t) * M);
    {
        int64_t g = bg;
        for (int64_t m = 0; m < M; ++m) { lt[m] = (int32_t)(g % lv->counts[m]) + 1; g /= lv->counts[m]; }
    }
    for (int64_t m = 0; m < M; ++m) u_out[m] = (double)lv->values[off[m] + lt[m] - 1];
    int64_t b = bc;
    /* :115-122 */
    for (int64_t i = 0; i + 1 < n; ++i) {
        int64_t g = grid_index(lv, lt);
        int32_t q = U[b + R * (g + Lg * i)];
        if (q < 0 || q >= lv->L) { rc = OR_EINFEASIBLE; break; }
        memcpy(lt, lv->tuples + (int64_t)q * M, sizeof(int32_t) * M);
        for (int64_t m = 0; m < M; ++m) u_out[m + M * (i + 1)] = (double)lv->values[off[m] + lt[m] - 1];
        double nrm = 0.0;
        for (int64_t m = 0; m < M; ++m) nrm += fabs(u_out[m + M * i] - u_old[m + M * i]);
        b = (int64_t)((double)b - nrm);
    }
    free(lt);
out:
    free(off);
    return rc;
}

/* TV_p(u, p)   HelpFunctions.jl:251-268.  p_kind OR_P_INF -> max-norm; otherwise p-norm via pow */
double oracle_tv_p(const double *u, int64_t M, int64_t n, int p_kind, double p) {
    double val = 0.0;
    for (int64_t i = 1; i < n; ++i) {
        if (p_kind == OR_P_INF) {
            double mx = -INFINITY; /* maximum(abs.(u[:,i] - u[:,i-1])) */
            for (int64_t m = 0; m < M; ++m) {
                double d = fabs(u[m + M * i] - u[m + M * (i - 1)]);
                if (d > mx || isnan(d)) mx = d;
            }
            val += mx;
        } else {
            double s = 0.0;
            for (int64_t m = 0; m < M; ++m) s += pow(fabs(u[m + M * i] - u[m + M * (i - 1)]), p);
            val += pow(s, 1.0 / p);
        }
    }
    return val;
}

/*
 * The reference's DP recurrence, timed as the CPU baseline: identical loop order to
 * oracle_bellman but over the admissible ranks only (non-admissible grid cells are Inf in the
 * reference and never read), with the U table kept as uint16 ranks -- the reference layout for
 * the bench config would be 2.21 TB.  Runs `steps` recursion steps after the terminal step
 * (steps < n-1 gives the truncated timing sample of BASELINE.md §2).  Returns a checksum.
 */
static double bellman_steps_impl(const or_levels *lv, const double *df, const double *u_old, int64_t n,
                                 int64_t B, int p_kind, double beta, double dt, int64_t steps,
                                 double *front_a, double *front_b, uint16_t *Ustep, int threads);

double oracle_bellman_steps(const or_levels *lv, const double *df, const double *u_old, int64_t n,
                            int64_t B, int p_kind, double beta, double dt, int64_t steps,
                            double *front_a, double *front_b, uint16_t *Ustep) {
    return bellman_steps_impl(lv, df, u_old, n, B, p_kind, beta, dt, steps, front_a, front_b, Ustep, 1);
}

/*
 * The same loop with the target levels rl of each step split over `threads` OpenMP threads (BASELINE.md §2:
 * "OpenMP over the level index l"): every rl writes only its own front column and U cells, so the result is
 * identical to the single-threaded loop.
 */
double oracle_bellman_steps_mt(const or_levels *lv, const double *df, const double *u_old, int64_t n,
                               int64_t B, int p_kind, double beta, double dt, int64_t steps,
                               double *front_a, double *front_b, uint16_t *Ustep, int threads) {
    return bellman_steps_impl(lv, df, u_old, n, B, p_kind, beta, dt, steps, front_a, front_b, Ustep,
                              threads < 1 ? 1 : threads);
}

static double bellman_steps_impl(const or_levels *lv, const double *df, const double *u_old, int64_t n,
                                 int64_t B, int p_kind, double beta, double dt, int64_t steps,
                                 double *front_a, double *front_b, uint16_t *Ustep, int threads) {
    const int64_t M = lv->M, L = lv->L, R = B + 1;
    int64_t off[16];
    for (int64_t m = 0; m < M; ++m) off[m] = level_off(lv, m);
    double *w = front_a, *r = front_b;
    for (int64_t k = 0; k < R * L; ++k) r[k] = INFINITY;
    for (int64_t rl = 0; rl < L; ++rl) {
        const int32_t *l = lv->tuples + rl * M;
        int64_t b = 0;
        double t1 = 0.0;
        for (int64_t m = 0; m < M; ++m) {
            int64_t numl = lv->values[off[m] + l[m] - 1];
            t1 += dt * df[m + M * (n - 1)] * (double)numl;
            b += (int64_t)fabs((double)numl - u_old[m + M * (n - 1)]);
        }
        if (b <= B) r[b + R * rl] = t1;
    }
    for (int64_t i = n - 1; i >= 1 && steps > 0; --i, --steps) {
        for (int64_t k = 0; k < R * L; ++k) w[k] = INFINITY;
#pragma omp parallel for num_threads(threads) schedule(static)
        for (int64_t rl = 0; rl < L; ++rl) {
            const int32_t *l = lv->tuples + rl * M;
            double t1 = 0.0;
            int64_t bt = 0;
            for (int64_t m = 0; m < M; ++m) {
                int64_t numl = lv->values[off[m] + l[m] - 1];
                t1 += dt * df[m + M * (i - 1)] * (double)numl;
                bt += (int64_t)fabs((double)numl - u_old[m + M * (i - 1)]);
            }
            for (int64_t rj = 0; rj < L; ++rj) {
                const int32_t *j = lv->tuples + rj * M;
                double wgt;
                if (p_kind == OR_P_INF) wgt = 1.0;
                else {
                    double s = 0.0;
                    for (int64_t m = 0; m < M; ++m) {
                        int64_t d = lv->values[off[m] + j[m] - 1] - lv->values[off[m] + l[m] - 1];
                        s += (double)(d < 0 ? -d : d);
                    }
                    wgt = s;
                }
                double t2 = t1 + beta * wgt;
                const double *rc = r + R * rj;
                double *wc = w + R * rl;
                uint16_t *uc = Ustep + R * rl;
                for (int64_t b = 0; b <= B - bt; ++b) {
                    double val = t2 + rc[b];
                    if (wc[b + bt] > val) { uc[b + bt] = (uint16_t)rj; wc[b + bt] = val; }
                }
            }
        }
        double *t = w; w = r; r = t;
    }
    double cs = 0.0;
    for (int64_t k = 0; k < R * L; ++k) if (r[k] < INFINITY) cs += r[k];
    return cs;
}
