// mioc_api.cpp -- the C ABI of libmioc (include/mioc.h): context, validation, buffer management
// and the orchestration of the gfx950 kernels.  No C++ exception crosses the ABI.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "mioc_internal.h"

using namespace mioc;

namespace {

constexpr int kStats = 4;  // 0 dominant DP kernel, 1 backtrack walk, 2 p=Inf prep, 3 argmin

int fail(mioc_ctx *ctx, int code, const std::string &msg) {
  if (ctx) ctx->err = msg;
  return code;
}

int hip_fail(mioc_ctx *ctx, hipError_t e, const char *where) {
  return fail(ctx, MIOC_EHIP, std::string(where) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(ctx, expr)                                      \
  do {                                                          \
    hipError_t _e = (expr);                                     \
    if (_e != hipSuccess) return hip_fail((ctx), _e, #expr);    \
  } while (0)

template <typename T>
int grow(mioc_ctx *ctx, T **p, size_t *cap_bytes, size_t need_bytes, const char *what) {
  if (*p && *cap_bytes >= need_bytes) return MIOC_OK;
  if (*p) {
    (void)hipDeviceSynchronize();  // the old buffer may still be read by a backtrack in flight on the other stream
    hipFree(*p);
    *p = nullptr;
    *cap_bytes = 0;
  }
  if (need_bytes == 0) need_bytes = 16;
  hipError_t e = hipMalloc(reinterpret_cast<void **>(p), need_bytes);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    *p = nullptr;
    char buf[160];
    std::snprintf(buf, sizeof buf, "cannot allocate %.3f GB for %s", need_bytes / 1e9, what);
    return fail(ctx, MIOC_ENOMEM, buf);
  }
  *cap_bytes = need_bytes;
  return MIOC_OK;
}

LevelsDev levels_dev(const mioc_ctx *ctx) {
  LevelsDev Lv;
  Lv.M = (int)ctx->M;
  Lv.L = (int)ctx->L;
  Lv.nuval = ctx->d_nuval;
  Lv.nuint = ctx->d_nuint;
  Lv.gidx = ctx->d_gidx;
  Lv.vals = ctx->d_vals;
  Lv.voff = ctx->d_voff;
  Lv.g2r = ctx->d_g2r;
  Lv.p_kind = ctx->p_kind;
  Lv.p_int = (int)ctx->p_int;
  Lv.beta = ctx->beta;
  Lv.inv_beta = ctx->beta > 0.0 ? 1.0 / ctx->beta : 0.0;
  Lv.costlut = ctx->d_costlut;
  Lv.costtab = ctx->d_costtab;
  return Lv;
}

ProblemDev problem_dev(const mioc_ctx *ctx) {
  ProblemDev P;
  P.K = ctx->K;
  P.M = (int)ctx->M;
  P.nt = ctx->nt;
  P.B = ctx->B;
  P.RP = ctx->RP;
  P.dt = ctx->dt;
  P.df = ctx->d_df;
  P.uold = ctx->d_uold;
  P.Bvec = ctx->Bvec;
  P.gate = ctx->gate;
  return P;
}

void ev_collect(mioc_ctx *ctx);

// the context's current inputs and p = Inf tables <-> its DP slots
void slot_save(mioc_ctx *ctx) {
  mioc_ctx::Slot &q = ctx->slots[ctx->slot];
  q.df = ctx->d_df, q.uold = ctx->d_uold, q.in_cap = ctx->in_cap;
  q.kmin = ctx->pinf.kmin, q.k2 = ctx->pinf.k2, q.kfirst = ctx->pinf.kfirst, q.R = ctx->pinf.R, q.kabs = ctx->pinf.kabs;
  q.cap_k = ctx->pinf_cap_k, q.cap_R = ctx->pinf_cap_R, q.cap_kabs = ctx->pinf_cap_kabs;
}
void slot_load(mioc_ctx *ctx) {
  const mioc_ctx::Slot &q = ctx->slots[ctx->slot];
  ctx->d_df = q.df, ctx->d_uold = q.uold, ctx->in_cap = q.in_cap;
  ctx->pinf.kmin = q.kmin, ctx->pinf.k2 = q.k2, ctx->pinf.kfirst = q.kfirst, ctx->pinf.R = q.R, ctx->pinf.kabs = q.kabs;
  ctx->pinf_cap_k = q.cap_k, ctx->pinf_cap_R = q.cap_R, ctx->pinf_cap_kabs = q.cap_kabs;
}
// a new DP: the other slot, once the backtracks that read it are done (on the device: the stream waits)
int begin_dp(mioc_ctx *ctx) {
  slot_save(ctx);
  ctx->slot ^= 1;
  slot_load(ctx);
  if (ctx->bt_rec[ctx->slot]) HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_bt[ctx->slot], 0));
  return MIOC_OK;
}

void free_all(mioc_ctx *ctx) {
  if (ctx->d_runflags) hipFree(ctx->d_runflags);
  if (ctx->d_chain) hipFree(ctx->d_chain);
  if (ctx->d_ring) hipFree(ctx->d_ring);
  if (ctx->d_segflags) hipFree(ctx->d_segflags);
  if (ctx->h_run_err) hipHostFree(ctx->h_run_err);
  if (ctx->h_trm_poll) hipHostFree(ctx->h_trm_poll);
  if (ctx->bstream) hipStreamSynchronize(ctx->bstream);
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  slot_save(ctx);  // the current inputs and p = Inf tables are one of the slots
  for (auto &q : ctx->slots) {
    void *sp[] = {q.df, q.uold, q.kmin, q.k2, q.kfirst, q.R, q.kabs};
    for (void *p : sp)
      if (p) hipFree(p);
  }
  void *ptrs[] = {ctx->d_nuval, ctx->d_nuint,  ctx->d_gidx,      ctx->d_numin,       ctx->d_numax,
                  ctx->d_costlut, ctx->d_costtab, ctx->d_front,
                  ctx->d_U,     ctx->pinf.ftab, ctx->pinf.fseg, ctx->pinf.fneed,
                  ctx->d_start, ctx->d_ranks,   ctx->d_flags,      ctx->d_uout_own,    ctx->d_phistar_own,
                  ctx->d_status_own, ctx->d_stage,    ctx->d_counters, ctx->d_perm, ctx->d_same2, ctx->d_strad,
                  ctx->d_vals,  ctx->d_voff,    ctx->d_g2r,   ctx->d_tvw,        ctx->d_pred_own, ctx->d_ode_state};
  for (void *p : ptrs)
    if (p) hipFree(p);
  if (ctx->h_flags) hipHostFree(ctx->h_flags);
  heat_free(ctx->heat);
  ctx->heat = nullptr;
  ev_collect(ctx);
  for (auto &pr : ctx->ev_pool) hipEventDestroy(pr.begin), hipEventDestroy(pr.end);
  if (ctx->ev_dp) hipEventDestroy(ctx->ev_dp);
  for (hipEvent_t e : ctx->ev_bt)
    if (e) hipEventDestroy(e);
  if (ctx->bstream) hipStreamDestroy(ctx->bstream);
  if (ctx->stream) hipStreamDestroy(ctx->stream);
}

// (re)build the device cost tables for the current levels + cost
int build_cost_tables(mioc_ctx *ctx) {
  if (!ctx->have_levels || !ctx->have_cost) return MIOC_OK;
  const int64_t M = ctx->M, L = ctx->L;
  std::vector<double> lut;
  if (ctx->p_kind == MIOC_P_INF) {
    lut.assign(1, ctx->beta * 1.0);
  } else if (ctx->p_kind == MIOC_P_ONE || ctx->p_kind == MIOC_P_INTLUT) {
    int64_t maxkey = 0;
    for (int64_t m = 0; m < M; ++m) {
      int64_t d = (int64_t)(ctx->numax_h[m] - ctx->numin_h[m]);
      int64_t t = 1;
      if (ctx->p_kind == MIOC_P_ONE)
        t = d;
      else
        for (int64_t q = 0; q < ctx->p_int; ++q) t *= d;
      maxkey += t;
    }
    if (maxkey > (1 << 24)) return fail(ctx, MIOC_EINVAL, "switching-cost key range too large");
    lut.resize(maxkey + 1);
    for (int64_t s = 0; s <= maxkey; ++s) {
      double w;
      if (ctx->p_kind == MIOC_P_ONE) {
        w = (double)s;  // sum of |d| accumulated in Float64 is exact; s^(1/1) == s
      } else {
        if (s >= (int64_t)ctx->table.size())
          return fail(ctx, MIOC_EINVAL, "MIOC_P_INTLUT table shorter than the largest key sum |d|^p");
        w = ctx->table[s];
      }
      lut[s] = ctx->beta * w;
    }
  } else {  // MIOC_P_TABLE
    if ((int64_t)ctx->table.size() != L * L)
      return fail(ctx, MIOC_EINVAL, "MIOC_P_TABLE needs table_len == L*L for the current levels");
    std::vector<double> tab(L * L);
    for (int64_t q = 0; q < L * L; ++q) tab[q] = ctx->beta * ctx->table[q];
    size_t cap = 0;
    if (ctx->d_costtab) hipFree(ctx->d_costtab), ctx->d_costtab = nullptr;
    int rc = grow(ctx, &ctx->d_costtab, &cap, tab.size() * sizeof(double), "pair cost table");
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(ctx->d_costtab, tab.data(), tab.size() * sizeof(double), hipMemcpyHostToDevice));
    lut.assign(1, 0.0);
  }
  // TV_p's summand uses the unscaled weights (HelpFunctions.jl:262): keep the host table on the device as is
  if (ctx->d_tvw) hipFree(ctx->d_tvw), ctx->d_tvw = nullptr;
  ctx->tvw_len = 0;
  if ((ctx->p_kind == MIOC_P_INTLUT || ctx->p_kind == MIOC_P_TABLE) && !ctx->table.empty()) {
    size_t wcap = 0;
    int rc = grow(ctx, &ctx->d_tvw, &wcap, ctx->table.size() * sizeof(double), "TV weight table");
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(ctx->d_tvw, ctx->table.data(), ctx->table.size() * sizeof(double), hipMemcpyHostToDevice));
    ctx->tvw_len = (int64_t)ctx->table.size();
  }
  size_t cap = 0;
  if (ctx->d_costlut) hipFree(ctx->d_costlut), ctx->d_costlut = nullptr;
  int rc = grow(ctx, &ctx->d_costlut, &cap, lut.size() * sizeof(double), "cost lut");
  if (rc) return rc;
  HIP_TRY(ctx, hipMemcpy(ctx->d_costlut, lut.data(), lut.size() * sizeof(double), hipMemcpyHostToDevice));
  ctx->costlut_len = (int64_t)lut.size();
  return MIOC_OK;
}

// Per-kernel timing (MIOC_OPT_TIMING): an event pair around each timed launch (or launch sequence),
// folded into the totals at the next synchronising call.  Pairs are pooled, so every launch between two
// collections is counted.
void ev_collect(mioc_ctx *ctx) {
  for (int w = 0; w < kStats; ++w) {
    for (auto &pr : ctx->ev_pending[w]) {
      hipEventSynchronize(pr.end);
      float ms = 0.f;
      if (hipEventElapsedTime(&ms, pr.begin, pr.end) == hipSuccess) {
        ctx->stat_ms[w] += ms;
        ctx->stat_launches[w] += pr.launches;
      }
      ctx->ev_pool.push_back(pr);
    }
    ctx->ev_pending[w].clear();
  }
}
void ev_begin(mioc_ctx *ctx, int which, const char *name, hipStream_t st = nullptr) {
  if (!ctx->timing) return;
  if (ctx->ev_pending[which].size() >= 256) ev_collect(ctx);
  mioc_ctx::EvPair pr;
  if (!ctx->ev_pool.empty()) {
    pr = ctx->ev_pool.back();
    ctx->ev_pool.pop_back();
  } else {
    hipEventCreate(&pr.begin);
    hipEventCreate(&pr.end);
  }
  hipEventRecord(pr.begin, st ? st : ctx->stream);
  ctx->ev_open[which] = pr;
  ctx->stat_name[which] = name;
}
void ev_end(mioc_ctx *ctx, int which, int64_t launches, hipStream_t st = nullptr) {
  if (!ctx->timing) return;
  mioc_ctx::EvPair pr = ctx->ev_open[which];
  hipEventRecord(pr.end, st ? st : ctx->stream);
  pr.launches = launches;
  ctx->ev_pending[which].push_back(pr);
}

// --------------------------------------------------------------------------------------------------
// the DP
// --------------------------------------------------------------------------------------------------
int run_bellman(mioc_ctx *ctx) {
  ProblemDev P = problem_dev(ctx);
  LevelsDev Lv = levels_dev(ctx);
  // fills queued before the validation's host sync below, so that they overlap the previous call's device work: the
  // DP counters, and (p = Inf, the likely algorithm) the segmented recursion's flags
  if (!ctx->d_counters) {
    size_t cc = 0;
    int rc0 = grow(ctx, &ctx->d_counters, &cc, 8 * sizeof(int32_t), "counters");
    if (rc0) return rc0;
  }
  HIP_TRY(ctx, hipMemsetAsync(ctx->d_counters, 0, 8 * sizeof(int32_t), ctx->stream));
  bool pinf_flags_zeroed = false;
  if (ctx->p_kind == MIOC_P_INF && !ctx->force_steps) {
    const size_t fbytes = ((size_t)ctx->K * pinf_recur_segments(P) * PINF_WS_FLAG_STRIDE + 1) * sizeof(int32_t);
    int rcf = grow(ctx, &ctx->d_runflags, &ctx->runflag_cap, fbytes, "p=Inf segment flags");
    if (rcf) return rcf;
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_runflags, 0, fbytes, ctx->stream));
    pinf_flags_zeroed = true;
  }
  // validation pass: finite df, integral u_old, max budget class
  // (words 0, 1 only: 2, 3 are a backtrack's, which may still run on the other stream)
  HIP_TRY(ctx, hipMemsetAsync(ctx->d_flags, 0, 2 * sizeof(int32_t), ctx->stream));
  HIP_TRY(ctx, launch_validate(ctx->stream, P, ctx->d_numin, ctx->d_numax, ctx->d_flags));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->h_flags, ctx->d_flags, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  if (ctx->h_flags[0] & 2)
    return fail(ctx, MIOC_EINEXACT, "u_old has a non-integral entry: convert(Int64, abs(nu - u_old)) "
                                    "would throw InexactError (HelpFunctions.jl:37,57)");
  if (ctx->h_flags[0] & 1) return fail(ctx, MIOC_ENONFINITE, "df has a non-finite entry");
  const int bmax = ctx->h_flags[1];

  int algo = (int)ctx->opt_algo;
  // the p=Inf recursion keeps two budget rows and the staged class rows in LDS
  const bool pinf_ok = ctx->p_kind == MIOC_P_INF && bmax + 1 <= 64 && ctx->RP <= 7936;
  // the L1-ball identity min_j fl(K(d(l,j)) + Ψ_j) = min_S fl(K(S) + BM_S(l)) needs K non-decreasing in S
  const bool pyr_ok = ctx->p_kind == MIOC_P_ONE && ctx->pyr_ok && ctx->beta >= 0.0;
  // the separable transform works in units of beta (exact unit steps): beta > 0, 8^3 / 8^4 grids
  const bool sdt_ok = pyr_ok && ctx->beta > 0.0 && sdt_supported(ctx->pyr);
  // the fused small-state DP keeps a subproblem's whole front (and the per-step K table) in one CU's LDS
  const bool fused_ok = fused_supported((int)ctx->L, ctx->B, nullptr) && ctx->nt >= 1;
  // ... and with the separable L1 transform (p = 1, β > 0, 2-D product grid of consecutive levels)
  const bool fsep_ok = ctx->p_kind == MIOC_P_ONE && ctx->grid_ok && ctx->beta > 0.0 &&
                       fsep_supported(ctx->pyr, ctx->B, nullptr, nullptr);
  if (algo == MIOC_ALGO_AUTO)
    algo = pinf_ok    ? MIOC_ALGO_PINF
           : sdt_ok   ? MIOC_ALGO_SEPARABLE
           : fsep_ok  ? MIOC_ALGO_FUSED_SEPARABLE
           : fused_ok ? MIOC_ALGO_FUSED
                      : (pyr_ok && ctx->L >= 256 ? MIOC_ALGO_PYRAMID : MIOC_ALGO_GENERIC);
  if (algo == MIOC_ALGO_FUSED_SEPARABLE && !fsep_ok)
    return fail(ctx, MIOC_EINVAL, "the fused separable DP needs p = 1, beta > 0, a 2-D product grid of consecutive "
                                  "integer levels (6x6, 4x4, 8x8 or 8x4) and B < 512");
  if (algo == MIOC_ALGO_FUSED && !fused_ok)
    return fail(ctx, MIOC_EINVAL, "the fused small-state DP needs L <= 64 and a front that fits one CU's LDS");
  if (algo == MIOC_ALGO_PINF && !pinf_ok)
    return fail(ctx, MIOC_EINVAL, "p=Inf collapse needs p_kind MIOC_P_INF, <= 64 budget classes and B < 7936");
  if (algo == MIOC_ALGO_PYRAMID && !pyr_ok)
    return fail(ctx, MIOC_EINVAL, "the L1-ball pyramid needs p = 1, beta >= 0 and a product grid of consecutive "
                                  "integer levels (first dimension 4 or 8 levels, <= 4096 tuples)");
  if (algo == MIOC_ALGO_SEPARABLE && !sdt_ok)
    return fail(ctx, MIOC_EINVAL, "the separable L1 transform needs p = 1, beta > 0 and an 8^3 or 8^4 product grid "
                                  "of consecutive integer levels");
  ctx->algo = algo;
  const size_t K = (size_t)ctx->K, nt = (size_t)ctx->nt, L = (size_t)ctx->L, RP = (size_t)ctx->RP;

  if (algo == MIOC_ALGO_PYRAMID || algo == MIOC_ALGO_SEPARABLE) {
    const size_t s_stride = (size_t)(ctx->B + 1) * L;
    // persistent separable transform: rows 1..B of every subproblem in contiguous chunks over resident workgroups
    // (one per CU: the row body needs 2 waves per SIMD of registers and ~106 KB of LDS), row 0 of every step
    // precomputed (k_sdt_chain, k_sdt_row0), NB staging buffers
    const size_t run_lds = sdt_lds_bytes(ctx->pyr);
    int nwg = 0;
    bool persist = false;
    // (B + 1)·L·8 < 2^31: the persistent kernel addresses a staging block with 32-bit buffer offsets
    // ... and every b̃ within the kernel's dependency window (7 per dimension: u_old on the level grid); a u_old
    // off the grid reaches rows further back than the window waits for, so those problems take per-step launches
    if (algo == MIOC_ALGO_SEPARABLE && ctx->opt_persist && nt >= 2 && ctx->B >= 1 &&
        s_stride * sizeof(double) < (1ull << 31) && bmax <= 7 * ctx->pyr.M && !ctx->force_steps) {
      int ncu = 0;
      HIP_TRY(ctx, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
      // one workgroup per CU over contiguous row chunks (k_sdt_run)
      const int bpc = std::min(sdt_run_blocks_per_cu(ctx->pyr, run_lds), 1);  // one row workgroup per CU
      const size_t slots = (size_t)ncu * (size_t)std::max(bpc, 0);
      const size_t per_k = std::min<size_t>((size_t)ctx->B, K ? slots / K : 0);  // workgroups per subproblem
      nwg = (int)(per_k * K);
      persist = per_k >= 1;
    }
    // persistent layout: per subproblem NB staging buffers of (B+1)·L, then row 0 of every step (nt·L), one region
    // addressed by one buffer resource (< 4 GiB); per-step layout: two buffers of K blocks of (B+1)·L
    // at least 7·M + 1 buffers: item (c', i) waits (write-after-read) for the rows up to 7·M above it to have loaded
    // S_{i+NB}, and (one item ahead) for the rows below it to have finished step i; with NB <= 7·M those waits close a
    // cycle -- (c', i) <- (c'-1, i-1) <- ... <- (c'-NB, i-NB), whose WAR wait needs row c' to have loaded S_i, i.e.
    // item (c', i-1) -- and the DP deadlocks until the spin limit (tests/test_gpu_c4.py runs 29, 32 and 37)
    const int nb_min = 7 * ctx->pyr.M + 1;
    int nbuf = persist ? std::max(ctx->opt_nb, nb_min) : 2;
    // one buffer resource addresses a subproblem's whole region (32-bit offsets): as many buffers as fit under 4 GiB
    if (persist) {
      const size_t cap = (1ull << 32) / sizeof(double);
      const size_t fit = cap > nt * L ? (cap - nt * L - 1) / s_stride : 0;
      if ((size_t)nbuf > fit) nbuf = (int)fit;
      if (nbuf < nb_min) persist = false, nbuf = 2;  // too few fit to be deadlock-free: per-step launches
    }
    const size_t kstride = persist ? (size_t)nbuf * s_stride + nt * L : s_stride;
    if (persist && kstride * sizeof(double) >= (1ull << 32)) persist = false;  // (then also kstride = s_stride)
    const size_t ks = persist ? kstride : s_stride;
    // flags: done and loaded per row, then the error word
    const size_t nflag = 2 * K * (size_t)(ctx->B + 1) * SDT_FLAG_STRIDE;
    const size_t runflag_bytes = ((nflag + 1) * sizeof(int32_t) + 15) / 16 * 16;
    if (persist) {
      int rcf = grow(ctx, &ctx->d_runflags, &ctx->runflag_cap, runflag_bytes, "persistent row flags");
      if (!rcf) rcf = grow(ctx, &ctx->d_chain, &ctx->chain_cap, K * nt * sizeof(double), "row 0 chain");
      if (rcf) return rcf;
      if (!ctx->h_run_err) HIP_TRY(ctx, hipHostMalloc(&ctx->h_run_err, 16, 0));
      *ctx->h_run_err = 0;
    }
    const size_t stage_doubles = persist ? K * ks : 2 * K * s_stride;
    int rc = grow(ctx, &ctx->d_stage, &ctx->stage_cap, stage_doubles * sizeof(double), "staging fronts");
    if (rc) return rc;
    ctx->stage_kstride = ks;
    const size_t uu_stride_k = (nt > 1 ? nt - 1 : 1) * s_stride;
    rc = grow(ctx, &ctx->d_U, &ctx->U_cap, K * uu_stride_k * sizeof(uint16_t), "argmin table U");
    if (rc) return rc;
    rc = grow(ctx, &ctx->d_perm, &ctx->perm_cap, K * nt * L * sizeof(uint32_t), "sphere orders");
    if (!rc) rc = grow(ctx, &ctx->d_same2, &ctx->same2_cap, K * nt * sizeof(int32_t), "sphere-order reuse flags");
    const bool seams = persist && sdt_seam_lists(ctx->pyr);
    if (!rc && seams) rc = grow(ctx, &ctx->d_strad, &ctx->strad_cap, K * nt * 8 * 32 * sizeof(uint16_t), "seam lists");
    if (rc) return rc;
    double *st[2] = {ctx->d_stage, ctx->d_stage + K * s_stride};
    double *term = persist ? ctx->d_stage + ((nt - 1) % nbuf) * s_stride : st[(nt - 1) & 1];
    HIP_TRY(ctx, launch_pyr_order(ctx->stream, P, ctx->pyr, ctx->d_perm, ctx->d_same2, seams ? ctx->d_strad : nullptr,
                                  ctx->d_counters));
    HIP_TRY(ctx, launch_pyr_terminal(ctx->stream, P, Lv, ctx->d_perm, term, ks));
    if (algo == MIOC_ALGO_SEPARABLE && persist) {
      // the whole DP as one persistent launch: rows handed between resident workgroups by flags
      HIP_TRY(ctx, launch_sdt_prep(ctx->stream, P, Lv, ctx->pyr, ctx->d_perm, ctx->d_chain, ctx->d_stage, ks,
                                   (size_t)nbuf * s_stride, (uint16_t *)ctx->d_U, uu_stride_k));
      HIP_TRY(ctx, hipMemsetAsync(ctx->d_runflags, 0, runflag_bytes, ctx->stream));
      ev_begin(ctx, 0, "k_sdt_run");
      // (the grid is nwg <= CUs x resident workgroups per CU by construction above; a wait that never ends anyway --
      // another process holding CUs -- is caught by the spin limit and redone per step by check_run)
      HIP_TRY(ctx, launch_sdt_run(ctx->stream, P, Lv, ctx->pyr, ctx->d_perm, ctx->d_same2, ctx->d_strad, ctx->d_stage,
                                  ks, nbuf, (uint16_t *)ctx->d_U, uu_stride_k, ctx->d_counters, ctx->d_runflags, nwg,
                                  ctx->spin_limit, run_lds));
      ev_end(ctx, 0, 1);
      HIP_TRY(ctx, hipMemcpyAsync(ctx->h_run_err, ctx->d_runflags + nflag, sizeof(int32_t),
                                  hipMemcpyDeviceToHost, ctx->stream));
      ctx->run_pending = true;
    } else if (algo == MIOC_ALGO_SEPARABLE) {
      ev_begin(ctx, 0, "k_sdt_step");
      for (int i = ctx->nt - 2; i >= 0; --i)
        HIP_TRY(ctx, launch_sdt_step(ctx->stream, P, Lv, ctx->pyr, i, ctx->d_perm, st[(i + 1) & 1], st[i & 1],
                                     (uint16_t *)ctx->d_U, s_stride, uu_stride_k, ctx->d_counters));
      ev_end(ctx, 0, ctx->nt - 1);
    } else {
      ev_begin(ctx, 0, "k_pyr_step");
      for (int i = ctx->nt - 2; i >= 0; --i)
        HIP_TRY(ctx, launch_pyr_step(ctx->stream, P, Lv, ctx->pyr, i, ctx->d_perm, st[(i + 1) & 1], st[i & 1],
                                     (uint16_t *)ctx->d_U, s_stride, uu_stride_k, ctx->d_counters));
      ev_end(ctx, 0, ctx->nt - 1);
    }
  } else if (algo == MIOC_ALGO_FUSED || algo == MIOC_ALGO_FUSED_SEPARABLE) {
    ctx->ubytes = 1;
    const size_t front_stride = L * RP;
    int rc = grow(ctx, &ctx->d_front, &ctx->front_cap, K * front_stride * sizeof(double), "value fronts");
    if (rc) return rc;
    const size_t u_stride_k = (nt > 1 ? nt - 1 : 1) * L * (size_t)(ctx->B + 1);
    rc = grow(ctx, &ctx->d_U, &ctx->U_cap, K * u_stride_k, "argmin table U");
    if (rc) return rc;
    ctx->occupancy = fused_blocks_per_cu(algo == MIOC_ALGO_FUSED_SEPARABLE, ctx->pyr, (int)ctx->L, ctx->B);
    if (algo == MIOC_ALGO_FUSED) {
      ev_begin(ctx, 0, "k_fused_run");
      HIP_TRY(ctx, launch_fused_run(ctx->stream, P, Lv, ctx->d_front, front_stride, (uint8_t *)ctx->d_U, u_stride_k));
    } else {
      // two lanes per row, the front in place (mioc_fsep.hip); S row segments per subproblem when the batch alone
      // would leave CUs idle (two resident subproblems per CU when the front is half the LDS)
      FsepPlan plan;
      int S = ctx->force_steps ? 1 : ctx->opt_fsep_seg;
      if (S == 0) {
        int ncu = 0;
        HIP_TRY(ctx, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
        S = 1;
        while (S < 8 && (size_t)K * (size_t)(2 * S) <= (size_t)ncu && fsep2_plan(ctx->pyr, ctx->B, 2 * S, nullptr))
          S *= 2;
      }
      // a u_old off the level grid can send a target further than SMAX rows up, past a segment's outbox rows
      if (S > 1 && bmax > ctx->pyr.n[0] + ctx->pyr.n[1] - 2) S = 1;
      const bool v2 = S >= 1 && fsep2_plan(ctx->pyr, ctx->B, S, &plan);
      ctx->last_fsep_seg = v2 ? S : 0;
      if (v2 && S > 1) {
        // segments with at most one workgroup per CU to go round: reserve more than half a CU's LDS, so that the
        // dispatcher cannot put two segments on one CU while another CU idles (the segments run as one pipeline,
        // and a shared CU slows all of them: the 128-restart shard ran 17 - 28 ms from run to run)
        int ncu = 0, cu_lds = 0, wg_lds = 0;
        HIP_TRY(ctx, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
        HIP_TRY(ctx, hipDeviceGetAttribute(&cu_lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, ctx->device));
        HIP_TRY(ctx, hipDeviceGetAttribute(&wg_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, ctx->device));
        // half a CU's LDS plus one 2 KiB allocation granule (gfx950: 82 KiB of 160), capped at a workgroup's maximum
        const size_t half = std::min<size_t>((size_t)cu_lds / 2 + 2048, (size_t)wg_lds);
        if ((size_t)K * (size_t)S <= (size_t)ncu) plan.lds = std::max<size_t>(plan.lds, half);
      }
      if (v2) ctx->occupancy = fsep2_blocks_per_cu(ctx->pyr, plan);
      if (v2 && S > 1) {
        const int NB = 8, SM = ctx->pyr.n[0] + ctx->pyr.n[1] - 2;
        (void)SM;
        rc = grow(ctx, &ctx->d_ring, &ctx->ring_cap, K * (size_t)S * NB * (size_t)plan.slot_bytes, "segment rings");
        if (!rc) rc = grow(ctx, &ctx->d_segflags, &ctx->segflag_cap, (FSEP_FLAG_STRIDE * K * (size_t)S + 1) * sizeof(int32_t),
                           "segment flags");
        if (rc) return rc;
        if (!ctx->h_run_err) HIP_TRY(ctx, hipHostMalloc(&ctx->h_run_err, 16, 0));
        *ctx->h_run_err = 0;
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_segflags, 0, (FSEP_FLAG_STRIDE * K * (size_t)S + 1) * sizeof(int32_t), ctx->stream));
        ev_begin(ctx, 0, "k_fsep2");
        int ncu = 0;
        HIP_TRY(ctx, hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
        // every segment must be resident at once (they wait for each other): else the unsegmented kernel below
        const hipError_t le =
            (size_t)K * (size_t)S > (size_t)ncu * (size_t)std::max<int64_t>(ctx->occupancy, 0)
                ? hipErrorCooperativeLaunchTooLarge
                : launch_fsep2(ctx->stream, P, Lv, ctx->pyr, plan, ctx->d_front, front_stride, (uint8_t *)ctx->d_U,
                               u_stride_k, ctx->d_counters, ctx->d_ring, NB, ctx->d_segflags, ctx->spin_limit);
        if (le == hipErrorCooperativeLaunchTooLarge) {  // not every segment resident: one workgroup per subproblem
          ev_end(ctx, 0, 0);
          ctx->n_persist_fallbacks += 1;
          ctx->force_steps = true;
          const int rcs = run_bellman(ctx);
          ctx->force_steps = false;
          return rcs;
        }
        HIP_TRY(ctx, le);
        ev_end(ctx, 0, 1);
        HIP_TRY(ctx, hipMemcpyAsync(ctx->h_run_err, ctx->d_segflags + FSEP_FLAG_STRIDE * K * (size_t)S, sizeof(int32_t),
                                    hipMemcpyDeviceToHost, ctx->stream));
        ctx->run_pending = true;
        ctx->have_dp = true;
        return MIOC_OK;
      }
      if (v2) {
        ev_begin(ctx, 0, "k_fsep2");
        HIP_TRY(ctx, launch_fsep2(ctx->stream, P, Lv, ctx->pyr, plan, ctx->d_front, front_stride, (uint8_t *)ctx->d_U,
                                  u_stride_k, ctx->d_counters, nullptr, 1, nullptr, ctx->spin_limit));
      } else {
        ev_begin(ctx, 0, "k_fsep_run");
        HIP_TRY(ctx, launch_fsep_run(ctx->stream, P, Lv, ctx->pyr, ctx->d_front, front_stride, (uint8_t *)ctx->d_U,
                                     u_stride_k, ctx->d_counters));
      }
    }
    ev_end(ctx, 0, 1);
  } else if (algo == MIOC_ALGO_GENERIC) {
    ctx->ubytes = L <= 256 ? 1 : 2;
    const size_t front_stride = L * RP;
    int rc = grow(ctx, &ctx->d_front, &ctx->front_cap, 2 * K * front_stride * sizeof(double), "value fronts");
    if (rc) return rc;
    const size_t u_stride_k = (nt > 1 ? nt - 1 : 1) * L * (size_t)(ctx->B + 1);
    rc = grow(ctx, &ctx->d_U, &ctx->U_cap, K * u_stride_k * ctx->ubytes, "argmin table U");
    if (rc) return rc;
    double *fr[2] = {ctx->d_front, ctx->d_front + K * front_stride};
    HIP_TRY(ctx, launch_generic_terminal(ctx->stream, P, Lv, fr[(nt - 1) & 1], front_stride));
    ev_begin(ctx, 0, "k_generic_step");
    for (int i = ctx->nt - 2; i >= 0; --i)
      HIP_TRY(ctx, launch_generic_step(ctx->stream, P, Lv, i, fr[(i + 1) & 1], fr[i & 1], ctx->d_U, ctx->ubytes,
                                       front_stride, u_stride_k));
    ev_end(ctx, 0, ctx->nt - 1);
  } else {
    PinfDev &D = ctx->pinf;
    D.BW = bmax + 1;
    D.BWP = 8;
    while (D.BWP < D.BW) D.BWP *= 2;
    const size_t kcells = K * nt * (size_t)D.BWP;
    size_t cap_km = ctx->pinf_cap_k, cap_k2 = ctx->pinf_cap_k, cap_kf = ctx->pinf_cap_k;
    int rc = grow(ctx, &D.kmin, &cap_km, kcells * sizeof(double), "class minima");
    if (!rc) rc = grow(ctx, &D.k2, &cap_k2, kcells * sizeof(double), "class second minima");
    if (!rc) rc = grow(ctx, &D.kfirst, &cap_kf, kcells * sizeof(double), "class first ranks");
    if (rc) return rc;
    ctx->pinf_cap_k = std::min(cap_km, std::min(cap_k2, cap_kf));
    pinf_plan((int)RP, (int)nt, D);
    rc = grow(ctx, &D.R, &ctx->pinf_cap_R, K * nt * RP * sizeof(double), "row minima R");
    if (!rc) rc = grow(ctx, &D.kabs, &ctx->pinf_cap_kabs, K * nt * sizeof(double), "level value bounds");
    if (rc) return rc;
    ev_begin(ctx, 2, "k_pinf_prep");
    HIP_TRY(ctx, launch_pinf_prep(ctx->stream, P, Lv, D));
    ev_end(ctx, 2, 1);
    ev_begin(ctx, 0, "k_pinf_recur");
    if (!ctx->ncu) HIP_TRY(ctx, hipDeviceGetAttribute(&ctx->ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
    // row segments on several CUs need their hand-off flags (and a timed-out wait redoes the DP in one workgroup)
    int32_t *pflags = nullptr;
    if (!ctx->force_steps) {
      if (!pinf_flags_zeroed) {
        const size_t fbytes = ((size_t)K * pinf_recur_segments(P) * PINF_WS_FLAG_STRIDE + 1) * sizeof(int32_t);
        rc = grow(ctx, &ctx->d_runflags, &ctx->runflag_cap, fbytes, "p=Inf segment flags");
        if (rc) return rc;
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_runflags, 0, fbytes, ctx->stream));
      }
      if (!ctx->h_run_err) HIP_TRY(ctx, hipHostMalloc(&ctx->h_run_err, 16, 0));
      *ctx->h_run_err = 0;
      pflags = ctx->d_runflags;
    }
    bool segmented = false;
    const char *variant = "k_pinf_recur";
    HIP_TRY(ctx, launch_pinf_recur(ctx->stream, P, D, ctx->ncu, pflags, ctx->spin_limit, &segmented, &variant));
    ev_end(ctx, 0, 1);
    ctx->stat_name[0] = variant;  // the timing window is named after the recursion kernel that ran
    if (segmented) {
      const int nseg = pinf_recur_segments(P);
      if (!P.gate) {
        // a wait past the spin limit: the one-workgroup recursion redoes the DP on the device, gated by the error word
        // (no host round trip between the DP and the backtrack); diagnostics [6] reads its count (d_counters[6])
        ProblemDev Pr = P;
        Pr.redo_gate = ctx->d_runflags + (size_t)K * nseg * PINF_WS_FLAG_STRIDE;
        Pr.redo_count = ctx->d_counters + 6;
        HIP_TRY(ctx, launch_pinf_recur(ctx->stream, Pr, D, ctx->ncu, nullptr, ctx->spin_limit, nullptr, nullptr));
      } else {
        // under the device TRM control the backtrack kernels are gated already: the host checks and redoes (check_run)
        HIP_TRY(ctx, hipMemcpyAsync(ctx->h_run_err, ctx->d_runflags + (size_t)K * nseg * PINF_WS_FLAG_STRIDE, sizeof(int32_t),
                                    hipMemcpyDeviceToHost, ctx->stream));
        ctx->run_pending = true;
      }
    }
  }
  ctx->have_dp = true;
  return MIOC_OK;
}

int check_run(mioc_ctx *ctx);

int run_backtrack(mioc_ctx *ctx, int64_t B_use, double *d_u_out, double *d_phi_star, int32_t *d_status) {
  // a persistent DP still in flight: learn whether its dependency waits timed out BEFORE anything reads its
  // tables, so that a redone DP (check_run) is what the backtrack walks
  if (ctx->run_pending) {
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const int rcr = check_run(ctx);
    if (rcr) return rcr;
  }
  if (!ctx->have_dp) return fail(ctx, MIOC_ESTATE, "backtrack called before bellman");
  if (B_use < 0 || B_use > ctx->B)
    return fail(ctx, MIOC_ESTATE, "B_use must satisfy 0 <= B_use <= B of the last bellman call");
  // p = Inf (outside the device TRM control): on the second stream, after this DP, so that the next bellman's kernels
  // overlap it; the other algorithms run on the context's stream after any such backtrack in flight
  const bool async_bt = ctx->algo == MIOC_ALGO_PINF && !ctx->gate;
  if (!async_bt) {
    const int rcj = join_bt(ctx);
    if (rcj) return rcj;
  }
  hipStream_t bs = async_bt ? ctx->bstream : ctx->stream;
  if (async_bt) {
    HIP_TRY(ctx, hipEventRecord(ctx->ev_dp, ctx->stream));
    HIP_TRY(ctx, hipStreamWaitEvent(bs, ctx->ev_dp, 0));
  }
  ProblemDev P = problem_dev(ctx);
  LevelsDev Lv = levels_dev(ctx);
  const size_t K = (size_t)ctx->K, nt = (size_t)ctx->nt;
  size_t cap = 0;
  if (!ctx->d_start) {
    int rc = grow(ctx, &ctx->d_start, &cap, 4096 * sizeof(Start), "start cells");
    if (rc) return rc;
  }
  if (K > 4096) return fail(ctx, MIOC_EINVAL, "batch larger than 4096 subproblems");
  int rc = grow(ctx, &ctx->d_ranks, &ctx->ranks_cap, 2 * K * nt * sizeof(int32_t), "rank path");
  if (rc) return rc;
  int32_t *d_urank = ctx->d_ranks + K * nt;
  if (ctx->algo != MIOC_ALGO_PINF) HIP_TRY(ctx, launch_uold_rank(ctx->stream, P, Lv, d_urank));
  // (p = Inf: k_pinf_start zeroes them, one fill fewer on the stream)
  if (ctx->algo != MIOC_ALGO_PINF) HIP_TRY(ctx, hipMemsetAsync(ctx->d_flags + 2, 0, 2 * sizeof(int32_t), ctx->stream));
  if (ctx->algo == MIOC_ALGO_PYRAMID || ctx->algo == MIOC_ALGO_SEPARABLE) {
    const size_t s_stride = (size_t)(ctx->B + 1) * ctx->L;
    const size_t uu_stride_k = (nt > 1 ? nt - 1 : 1) * s_stride;
    HIP_TRY(ctx, launch_stage_argmin0(ctx->stream, P, Lv, ctx->d_perm, ctx->d_stage, ctx->stage_kstride, (int)B_use,
                                      ctx->d_start));
    ev_begin(ctx, 1, "k_stage_walk");
    HIP_TRY(ctx, launch_stage_walk(ctx->stream, P, Lv, (const uint16_t *)ctx->d_U, uu_stride_k, ctx->d_start,
                                   d_urank, ctx->d_ranks, ctx->d_flags + 2));
    ev_end(ctx, 1, 1);
  } else if (ctx->algo == MIOC_ALGO_GENERIC || ctx->algo == MIOC_ALGO_FUSED ||
             ctx->algo == MIOC_ALGO_FUSED_SEPARABLE) {
    const size_t front_stride = (size_t)ctx->L * ctx->RP;
    const size_t u_stride_k = (nt > 1 ? nt - 1 : 1) * (size_t)ctx->L * (size_t)(ctx->B + 1);
    HIP_TRY(ctx, launch_generic_argmin0(ctx->stream, P, Lv, ctx->d_front, front_stride, (int)B_use, ctx->d_start));
    ev_begin(ctx, 1, "k_generic_walk");
    HIP_TRY(ctx, launch_generic_walk(ctx->stream, P, Lv, ctx->d_U, ctx->ubytes, u_stride_k, ctx->d_start,
                                     d_urank, ctx->d_ranks, ctx->d_flags + 2));
    ev_end(ctx, 1, 1);
  } else {
    // the segmented walk spreads one subproblem's path over many workgroups: for batches too small to fill the GPU
    // with one serial walk each (auto: K <= 64 and at least 512 steps)
    const bool fwalk = ctx->opt_pinf_walk > 0 || (ctx->opt_pinf_walk == 0 && K <= 64 && nt >= 512);
    ctx->last_pinf_fwalk = fwalk;
    PinfDev &D = ctx->pinf;
    if (fwalk) {
      int G, nseg;
      pinf_fplan((int)nt, &G, &nseg);
      rc = grow(ctx, &D.ftab, &ctx->pinf_cap_ftab, K * nt * (size_t)ctx->RP, "segmented walk class table");
      if (!rc) rc = grow(ctx, &D.fseg, &ctx->pinf_cap_fseg, K * (size_t)nseg * ctx->RP * sizeof(int32_t),
                         "segmented walk segment maps");
      if (!rc) rc = grow(ctx, &D.fneed, &ctx->pinf_cap_fneed, (K + 1) * sizeof(int32_t), "segmented walk flags");
      if (rc) return rc;
    }
    // k_pinf_start also zeroes the walk's fallback counters (d_flags[2..3]) and, for the segmented walk, fneed
    HIP_TRY(ctx, launch_pinf_start(bs, P, Lv, D, (int)B_use, ctx->d_start, ctx->d_flags + 2, fwalk ? D.fneed : nullptr));
    if (fwalk) {
      ev_begin(ctx, 1, "k_pinf_fwalk", bs);
      HIP_TRY(ctx, launch_pinf_fwalk(bs, P, Lv, D, ctx->d_start, ctx->d_ranks));
      // subproblems whose chain met a state-dependent row: the serial walk (the others return at once)
      HIP_TRY(ctx, launch_pinf_walk(bs, P, Lv, D, ctx->d_start, ctx->d_ranks, ctx->d_flags + 2, D.fneed));
      ev_end(ctx, 1, 1, bs);
    } else {
      ev_begin(ctx, 1, "k_pinf_walk", bs);
      HIP_TRY(ctx, launch_pinf_walk(bs, P, Lv, D, ctx->d_start, ctx->d_ranks, ctx->d_flags + 2, nullptr));
      ev_end(ctx, 1, 1, bs);
    }
  }
  HIP_TRY(ctx, launch_expand(bs, P, Lv, ctx->d_start, ctx->d_ranks, d_u_out, d_phi_star, d_status));
  if (async_bt) {
    HIP_TRY(ctx, hipEventRecord(ctx->ev_bt[ctx->slot], bs));
    ctx->bt_rec[ctx->slot] = true;
    ctx->bt_pending = true;
    ctx->bt_last = ctx->slot;
  }
  ctx->have_path = true;
  return MIOC_OK;
}

// after a synchronisation: did the persistent DP's dependency waits time out (workgroups not co-resident, e.g.
// another context's kernels holding CUs)?  Then the DP is redone from the terminal step with one launch per
// step, which needs no co-residency, and the caller sees only the extra time.
int check_run(mioc_ctx *ctx) {
  if (!ctx->run_pending) return MIOC_OK;
  ctx->run_pending = false;
  if (ctx->h_run_err && *ctx->h_run_err) {
    ctx->have_dp = false;
    ctx->n_persist_fallbacks += 1;
    ctx->force_steps = true;
    const int rc = run_bellman(ctx);
    ctx->force_steps = false;
    if (rc) return rc;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  }
  return MIOC_OK;
}

int check_ready(mioc_ctx *ctx) {
  if (!ctx) return MIOC_EINVAL;
  if (!ctx->have_levels) return fail(ctx, MIOC_ESTATE, "mioc_set_levels has not been called");
  if (!ctx->have_cost) return fail(ctx, MIOC_ESTATE, "mioc_set_cost has not been called");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  return MIOC_OK;
}

int set_problem(mioc_ctx *ctx, int64_t K, int64_t nx, int64_t nt, int64_t B, double dt) {
  if (nx != ctx->M) return fail(ctx, MIOC_EINVAL, "nx does not match the number of controls in the level table");
  if (K < 1 || K > 4096) return fail(ctx, MIOC_EINVAL, "batch size must be in [1, 4096]");
  if (nt < 1 || nt > (1 << 30)) return fail(ctx, MIOC_EINVAL, "nt out of range");
  if (B < 0 || B > (1 << 20)) return fail(ctx, MIOC_EINVAL, "B out of range");
  if (!std::isfinite(dt)) return fail(ctx, MIOC_EINVAL, "dt must be finite");
  ctx->K = (int)K;
  ctx->nt = (int)nt;
  ctx->B = (int)B;
  ctx->RP = (int)(((B + 1 + kRowTile - 1) / kRowTile) * kRowTile);
  ctx->dt = dt;
  ctx->have_dp = false;
  ctx->have_path = false;
  size_t need = (size_t)K * nx * nt * sizeof(double);
  size_t cap = ctx->in_cap, cap2 = ctx->in_cap;
  int rc = grow(ctx, &ctx->d_df, &cap, need, "df copy");
  if (!rc) rc = grow(ctx, &ctx->d_uold, &cap2, need, "u_old copy");
  if (rc) return rc;
  ctx->in_cap = std::min(cap, cap2);
  return MIOC_OK;
}

}  // namespace

int mioc::join_bt(mioc_ctx *ctx) {
  if (!ctx->bt_pending) return MIOC_OK;
  (void)hipSetDevice(ctx->device);
  ctx->bt_pending = false;
  if (hipStreamWaitEvent(ctx->stream, ctx->ev_bt[ctx->bt_last], 0) != hipSuccess)
    return fail(ctx, MIOC_EHIP, "hipStreamWaitEvent failed");
  return MIOC_OK;
}

// ==================================================================================================
// C ABI
// ==================================================================================================
extern "C" {

const char *mioc_version(void) { return "mioc 0.1.0 (gfx950)"; }

int32_t mioc_create(int32_t device, mioc_ctx **out) {
  if (!out) return MIOC_EINVAL;
  *out = nullptr;
  mioc_ctx *ctx = new (std::nothrow) mioc_ctx();
  if (!ctx) return MIOC_ENOMEM;
  ctx->device = device;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
    delete ctx;
    return MIOC_EHIP;
  }
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->bstream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_dp, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_bt[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_bt[1], hipEventDisableTiming) != hipSuccess ||
      hipMalloc(&ctx->d_flags, 16) != hipSuccess || hipMalloc(&ctx->d_pred_own, 64) != hipSuccess || hipHostMalloc(&ctx->h_flags, 16, 0) != hipSuccess) {
    free_all(ctx);
    delete ctx;
    return MIOC_EHIP;
  }
  *out = ctx;
  return MIOC_OK;
}

int32_t mioc_destroy(mioc_ctx *ctx) {
  if (!ctx) return MIOC_EINVAL;
  hipSetDevice(ctx->device);
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  free_all(ctx);
  delete ctx;
  return MIOC_OK;
}

const char *mioc_last_error(const mioc_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int32_t mioc_set_option(mioc_ctx *ctx, int32_t option, int64_t value) {
  if (!ctx) return MIOC_EINVAL;
  if (option == MIOC_OPT_ALGO) {
    if (value < MIOC_ALGO_AUTO || value > MIOC_ALGO_FUSED_SEPARABLE) return fail(ctx, MIOC_EINVAL, "unknown algorithm");
    ctx->opt_algo = value;
    return MIOC_OK;
  }
  if (option == MIOC_OPT_TIMING) {
    ctx->timing = value != 0;
    return MIOC_OK;
  }
  if (option == MIOC_OPT_PERSIST) {
    ctx->opt_persist = value != 0;
    return MIOC_OK;
  }
  if (option == MIOC_OPT_PRED_FMA) {
    ctx->pred_fma = value != 0;
    return MIOC_OK;
  }
  if (option == MIOC_OPT_SPIN_LIMIT) {
    if (value < 1 || value > (1ll << 30)) return fail(ctx, MIOC_EINVAL, "spin limit must be in [1, 2^30]");
    ctx->spin_limit = (unsigned)value;
    return MIOC_OK;
  }
  if (option == MIOC_OPT_SDT_BUFFERS) {
    if (value < 4 || value > kSdtMaxBuffers) return fail(ctx, MIOC_EINVAL, "staging buffers must be in [4, 256]");
    ctx->opt_nb = (int)value;
    return MIOC_OK;
  }
  if (option == MIOC_OPT_PINF_WALK) {
    if (value < -1 || value > 1) return fail(ctx, MIOC_EINVAL, "p=Inf walk option must be -1, 0 or 1");
    ctx->opt_pinf_walk = (int)value;
    return MIOC_OK;
  }
  if (option == MIOC_OPT_FSEP_SEGMENTS) {
    if (value < -1 || value > 8) return fail(ctx, MIOC_EINVAL, "fused separable segments must be in [-1, 8]");
    ctx->opt_fsep_seg = (int)value;
    return MIOC_OK;
  }
  return fail(ctx, MIOC_EINVAL, "unknown option");
}

int32_t mioc_set_levels(mioc_ctx *ctx, int64_t M, const int64_t *counts, const int64_t *values, int64_t L,
                        const int32_t *tuples) {
  if (!ctx) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  if (M < 1 || M > kMaxM) return fail(ctx, MIOC_EINVAL, "number of controls must be in [1, 8]");
  if (!counts || !values || !tuples) return fail(ctx, MIOC_EINVAL, "null level arrays");
  if (L < 1 || L > 65535) return fail(ctx, MIOC_EINVAL, "number of admissible tuples must be in [1, 65535]");
  std::vector<int64_t> off(M + 1, 0);
  int64_t Lgrid = 1;
  for (int64_t m = 0; m < M; ++m) {
    if (counts[m] < 1 || counts[m] > 4096) return fail(ctx, MIOC_EINVAL, "level count out of range");
    off[m + 1] = off[m] + counts[m];
    Lgrid *= counts[m];
    if (Lgrid > (int64_t)1 << 31) return fail(ctx, MIOC_EINVAL, "level grid too large");
  }
  for (int64_t q = 0; q < off[M]; ++q)
    if (values[q] < -(1 << 24) || values[q] > (1 << 24)) return fail(ctx, MIOC_EINVAL, "level value out of range");
  ctx->M = M;
  ctx->L = L;
  ctx->Lgrid = Lgrid;
  ctx->counts.assign(counts, counts + M);
  ctx->values.assign(values, values + off[M]);
  ctx->tuples.assign(tuples, tuples + L * M);
  ctx->nuval_h.assign(L * M, 0.0);
  std::vector<int32_t> nuint(L * M), gidx(L);
  for (int64_t r = 0; r < L; ++r) {
    int64_t g = 0, stride = 1;
    for (int64_t m = 0; m < M; ++m) {
      int32_t t = tuples[r * M + m];
      if (t < 1 || t > counts[m]) return fail(ctx, MIOC_EINVAL, "tuple level index out of range (1-based)");
      int64_t v = values[off[m] + t - 1];
      ctx->nuval_h[r * M + m] = (double)v;
      nuint[r * M + m] = (int32_t)v;
      g += (int64_t)(t - 1) * stride;
      stride *= counts[m];
    }
    gidx[r] = (int32_t)g;
  }
  ctx->gidx_h = gidx;
  ctx->numin_h.assign(M, 0.0);
  ctx->numax_h.assign(M, 0.0);
  for (int64_t m = 0; m < M; ++m) {
    int64_t lo = values[off[m]], hi = values[off[m]];
    for (int64_t q = off[m]; q < off[m + 1]; ++q) lo = std::min(lo, values[q]), hi = std::max(hi, values[q]);
    ctx->numin_h[m] = (double)lo;
    ctx->numax_h[m] = (double)hi;
  }
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  size_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, c4 = 0;
  void *olds[] = {ctx->d_nuval, ctx->d_nuint, ctx->d_gidx, ctx->d_numin, ctx->d_numax,
                  ctx->d_vals,  ctx->d_voff,  ctx->d_g2r};
  for (void *p : olds)
    if (p) hipFree(p);
  ctx->d_nuval = nullptr, ctx->d_nuint = nullptr, ctx->d_gidx = nullptr, ctx->d_numin = nullptr, ctx->d_numax = nullptr;
  ctx->d_vals = nullptr, ctx->d_voff = nullptr, ctx->d_g2r = nullptr;
  // grid tuple -> rank, for the backtrack's guess "the level equal to u_old" (only where it is small)
  const bool want_g2r = Lgrid <= ((int64_t)1 << 22);
  std::vector<int32_t> vals32(off[M]), voff32(M + 1), g2r;
  for (int64_t q = 0; q < off[M]; ++q) vals32[q] = (int32_t)values[q];
  for (int64_t m = 0; m <= M; ++m) voff32[m] = (int32_t)off[m];
  if (want_g2r) {
    g2r.assign(Lgrid, -1);
    for (int64_t r = L - 1; r >= 0; --r) g2r[gidx[r]] = (int32_t)r;
  }
  size_t c5 = 0, c6 = 0, c7 = 0;
  int rc = grow(ctx, &ctx->d_nuval, &c0, L * M * sizeof(double), "levels");
  if (!rc) rc = grow(ctx, &ctx->d_nuint, &c1, L * M * sizeof(int32_t), "levels");
  if (!rc) rc = grow(ctx, &ctx->d_gidx, &c2, L * sizeof(int32_t), "levels");
  if (!rc) rc = grow(ctx, &ctx->d_numin, &c3, M * sizeof(double), "levels");
  if (!rc) rc = grow(ctx, &ctx->d_numax, &c4, M * sizeof(double), "levels");
  if (!rc) rc = grow(ctx, &ctx->d_vals, &c5, off[M] * sizeof(int32_t), "levels");
  if (!rc) rc = grow(ctx, &ctx->d_voff, &c6, (M + 1) * sizeof(int32_t), "levels");
  if (!rc && want_g2r) rc = grow(ctx, &ctx->d_g2r, &c7, Lgrid * sizeof(int32_t), "levels");
  if (rc) return rc;
  HIP_TRY(ctx, hipMemcpy(ctx->d_vals, vals32.data(), off[M] * sizeof(int32_t), hipMemcpyHostToDevice));
  HIP_TRY(ctx, hipMemcpy(ctx->d_voff, voff32.data(), (M + 1) * sizeof(int32_t), hipMemcpyHostToDevice));
  if (want_g2r)
    HIP_TRY(ctx, hipMemcpy(ctx->d_g2r, g2r.data(), Lgrid * sizeof(int32_t), hipMemcpyHostToDevice));
  HIP_TRY(ctx, hipMemcpy(ctx->d_nuval, ctx->nuval_h.data(), L * M * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(ctx, hipMemcpy(ctx->d_nuint, nuint.data(), L * M * sizeof(int32_t), hipMemcpyHostToDevice));
  HIP_TRY(ctx, hipMemcpy(ctx->d_gidx, gidx.data(), L * sizeof(int32_t), hipMemcpyHostToDevice));
  HIP_TRY(ctx, hipMemcpy(ctx->d_numin, ctx->numin_h.data(), M * sizeof(double), hipMemcpyHostToDevice));
  HIP_TRY(ctx, hipMemcpy(ctx->d_numax, ctx->numax_h.data(), M * sizeof(double), hipMemcpyHostToDevice));
  // pyramid domain: product iterator in grid order, consecutive integer levels, dim 0 <= 8 levels
  {
    // a product grid of consecutive integer levels in iterator (grid) order
    bool grid = L == Lgrid && L <= 4096 && M >= 2 && M <= 6;
    for (int64_t r = 0; grid && r < L; ++r) grid = gidx[r] == r;
    for (int64_t m = 0; grid && m < M; ++m)
      for (int64_t q = 0; grid && q < counts[m]; ++q) grid = values[off[m] + q] == values[off[m]] + q;
    ctx->grid_ok = grid;
    ctx->pyr_ok = grid && (counts[0] == 8 || counts[0] == 4) && Lgrid / counts[0] <= 512;
    mioc::PyrGeom G;
    G.M = (int)M;
    G.ncol = (int)(Lgrid / counts[0]);
    int cs = 1;
    for (int64_t m = 0; m < M; ++m) {
      G.n[m] = (int)counts[m];
      G.base[m] = (int)values[off[m]];
      G.Smax += (int)counts[m] - 1;
      if (m >= 1) {
        G.cstride[m] = cs;
        cs *= (int)counts[m];
      }
    }
    ctx->pyr = G;
  }
  ctx->have_levels = true;
  ctx->have_dp = false;
  return build_cost_tables(ctx);
}

int32_t mioc_set_cost(mioc_ctx *ctx, int32_t p_kind, int64_t p_int, double beta, int64_t table_len,
                      const double *table) {
  if (!ctx) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  if (p_kind < MIOC_P_INF || p_kind > MIOC_P_TABLE) return fail(ctx, MIOC_EINVAL, "unknown p_kind");
  if (!std::isfinite(beta)) return fail(ctx, MIOC_EINVAL, "beta must be finite");
  if (p_kind == MIOC_P_INTLUT && (p_int < 2 || p_int > 8))
    return fail(ctx, MIOC_EINVAL, "MIOC_P_INTLUT needs 2 <= p_int <= 8");
  if ((p_kind == MIOC_P_INTLUT || p_kind == MIOC_P_TABLE) && (!table || table_len < 1))
    return fail(ctx, MIOC_EINVAL, "this p_kind needs a host-supplied weight table");
  ctx->p_kind = p_kind;
  ctx->p_int = p_kind == MIOC_P_INTLUT ? p_int : 1;
  ctx->beta = beta;
  if (table && table_len > 0)
    ctx->table.assign(table, table + table_len);
  else
    ctx->table.clear();
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  ctx->have_cost = true;
  ctx->have_dp = false;
  return build_cost_tables(ctx);
}

int32_t mioc_bellman_batch_device(mioc_ctx *ctx, int64_t K, const double *d_df, const double *d_u_old, int64_t nx,
                                  int64_t nt, int64_t B, double dt) {
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (!d_df || !d_u_old) return fail(ctx, MIOC_EINVAL, "null input pointer");
  rc = begin_dp(ctx);
  if (rc) return rc;
  rc = set_problem(ctx, K, nx, nt, B, dt);
  if (rc) return rc;
  const size_t bytes = (size_t)K * nx * nt * sizeof(double);
  HIP_TRY(ctx, hipMemcpyAsync(ctx->d_df, d_df, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->d_uold, d_u_old, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  return run_bellman(ctx);
}

int32_t mioc_bellman(mioc_ctx *ctx, const double *df, const double *u_old, int64_t nx, int64_t nt, int64_t B,
                     double dt) {
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (!df || !u_old) return fail(ctx, MIOC_EINVAL, "null input pointer");
  rc = begin_dp(ctx);
  if (rc) return rc;
  rc = set_problem(ctx, 1, nx, nt, B, dt);
  if (rc) return rc;
  const size_t bytes = (size_t)nx * nt * sizeof(double);
  HIP_TRY(ctx, hipMemcpyAsync(ctx->d_df, df, bytes, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->d_uold, u_old, bytes, hipMemcpyHostToDevice, ctx->stream));
  rc = run_bellman(ctx);
  if (rc) return rc;
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  rc = check_run(ctx);
  if (rc) return rc;
  ev_collect(ctx);
  return MIOC_OK;
}

int32_t mioc_backtrack_batch_device(mioc_ctx *ctx, int64_t B_use, double *d_u_out, double *d_phi_star,
                                    int32_t *d_status) {
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (!d_u_out) return fail(ctx, MIOC_EINVAL, "null output pointer");
  return run_backtrack(ctx, B_use, d_u_out, d_phi_star, d_status);
}

int32_t mioc_backtrack_batch_budgets_device(mioc_ctx *ctx, const int32_t *d_B_use, double *d_u_out, double *d_phi_star,
                                            int32_t *d_status) {
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (!d_u_out || !d_B_use) return fail(ctx, MIOC_EINVAL, "null pointer");
  if (!ctx->have_dp) return fail(ctx, MIOC_ESTATE, "backtrack called before bellman");
  // the per-subproblem budgets must lie in [0, B]: checked by the start kernels on the device (start_budget), which
  // report an out-of-range B_use[k] as status[k] = MIOC_ESTATE -- no host read-back of the budgets.  (The first
  // backtrack after a DP that spans several workgroups with in-launch hand-offs -- the persistent separable DP, the
  // segmented fused separable DP, the segmented p=Inf recursion -- still synchronises once to read that DP's
  // timeout word, run_backtrack/check_run; every later backtrack of the same DP enqueues without one.)
  ctx->Bvec = d_B_use;
  rc = run_backtrack(ctx, ctx->B, d_u_out, d_phi_star, d_status);
  ctx->Bvec = nullptr;
  return rc;
}

int32_t mioc_backtrack(mioc_ctx *ctx, int64_t B_use, double *u_out, double *phi_star, uint8_t *switch_mask) {
  int rc = check_ready(ctx);
  if (rc) return rc;
  if (!u_out) return fail(ctx, MIOC_EINVAL, "null output pointer");
  if (!ctx->have_dp) return fail(ctx, MIOC_ESTATE, "backtrack called before bellman");
  if (ctx->K != 1) return fail(ctx, MIOC_ESTATE, "host backtrack after a batched bellman: use the batch API");
  const size_t n = (size_t)ctx->M * ctx->nt;
  size_t c1 = 0, c2 = 0;
  rc = grow(ctx, &ctx->d_uout_own, &ctx->uout_cap, n * sizeof(double), "u staging");
  if (!rc && !ctx->d_phistar_own) rc = grow(ctx, &ctx->d_phistar_own, &c1, 16, "phi staging");
  if (!rc && !ctx->d_status_own) rc = grow(ctx, &ctx->d_status_own, &c2, 16, "status staging");
  if (rc) return rc;
  rc = run_backtrack(ctx, B_use, ctx->d_uout_own, ctx->d_phistar_own, ctx->d_status_own);
  if (!rc) rc = join_bt(ctx);  // the copies below run on the context's stream
  if (rc) return rc;
  double ps = 0.0;
  int32_t st = 0;
  HIP_TRY(ctx, hipMemcpyAsync(u_out, ctx->d_uout_own, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(&ps, ctx->d_phistar_own, sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(&st, ctx->d_status_own, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  ev_collect(ctx);
  if (phi_star) *phi_star = ps;
  if (st != MIOC_OK) return fail(ctx, MIOC_EINFEASIBLE, "no finite Φ value within the budget B_use");
  if (switch_mask) {
    const int64_t M = ctx->M;
    switch_mask[0] = 0;
    for (int64_t i = 1; i < ctx->nt; ++i) {
      uint8_t sw = 0;
      for (int64_t m = 0; m < M; ++m) sw |= u_out[m + M * i] != u_out[m + M * (i - 1)];
      switch_mask[i] = sw;
    }
  }
  return MIOC_OK;
}

// One context's share of mioc_batch_multi: host arrays in, host arrays out, synchronous.
static int32_t batch_host(mioc_ctx *ctx, int64_t K, const double *df, const double *u_old, int64_t nx, int64_t nt,
                          int64_t B, double dt, int64_t B_use, double *u_out, double *phi_star, int32_t *status) {
  int rc = check_ready(ctx);
  if (rc) return rc;
  rc = begin_dp(ctx);
  if (rc) return rc;
  rc = set_problem(ctx, K, nx, nt, B, dt);
  if (rc) return rc;
  const size_t n = (size_t)K * nx * nt;
  HIP_TRY(ctx, hipMemcpyAsync(ctx->d_df, df, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->d_uold, u_old, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  rc = run_bellman(ctx);
  if (rc) return rc;
  double *d_u = nullptr, *d_phi = nullptr;
  int32_t *d_st = nullptr;
  size_t c0 = 0, c1 = 0, c2 = 0;
  rc = grow(ctx, &d_u, &c0, n * sizeof(double), "multi-device u staging");
  if (!rc) rc = grow(ctx, &d_phi, &c1, (size_t)K * sizeof(double), "multi-device phi staging");
  if (!rc) rc = grow(ctx, &d_st, &c2, (size_t)K * sizeof(int32_t), "multi-device status staging");
  if (!rc) rc = run_backtrack(ctx, B_use, d_u, d_phi, d_st);
  if (!rc) rc = join_bt(ctx);  // the copies below run on the context's stream
  if (!rc && hipMemcpyAsync(u_out, d_u, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
    rc = fail(ctx, MIOC_EHIP, "u copy-out failed");
  if (!rc && phi_star &&
      hipMemcpyAsync(phi_star, d_phi, K * sizeof(double), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
    rc = fail(ctx, MIOC_EHIP, "phi copy-out failed");
  if (!rc && status &&
      hipMemcpyAsync(status, d_st, K * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)
    rc = fail(ctx, MIOC_EHIP, "status copy-out failed");
  if (hipStreamSynchronize(ctx->stream) != hipSuccess && !rc) rc = fail(ctx, MIOC_EHIP, "hipStreamSynchronize failed");
  if (!rc) rc = check_run(ctx);
  for (void *p : {(void *)d_u, (void *)d_phi, (void *)d_st})
    if (p) hipFree(p);
  ev_collect(ctx);
  return rc;
}

int32_t mioc_ode_eval_device(mioc_ctx *ctx, int32_t problem, int64_t K, const double *d_x, int64_t nx, int64_t nt,
                             double T0, double T1, const double *params, int32_t nparams, double *d_J, double *d_df) {
  if (!ctx) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  // the examples' constants (example_fishing.jl, example_doubletank.jl, example_vanderpol.jl)
  static const double fishing[14] = {1, 1, 1, 1, 1, 1, 0.2, 0.4, 0.01, 0.1, 0.2, 0.1, 0.5, 0.7};
  static const double tank[7] = {2, 3, 1, 0.5, 2, 2, 2};
  static const double vdp[5] = {-1, 0.75, -2, 1, 0};
  const double *def = problem == MIOC_ODE_FISHING ? fishing : problem == MIOC_ODE_DOUBLETANK ? tank : vdp;
  const int np = problem == MIOC_ODE_FISHING ? 14 : problem == MIOC_ODE_DOUBLETANK ? 7 : 5;
  if (problem < MIOC_ODE_FISHING || problem > MIOC_ODE_VANDERPOL) return fail(ctx, MIOC_EINVAL, "unknown ODE problem");
  if (nx != 3) return fail(ctx, MIOC_EINVAL, "the ODE examples have nx = 3 controls");
  if (K < 1 || nt < 1 || K > INT32_MAX || nt > INT32_MAX || !d_x) return fail(ctx, MIOC_EINVAL, "bad K / nt / x");
  if (params && nparams != np) return fail(ctx, MIOC_EINVAL, "wrong parameter count for this ODE problem");
  if (!(T1 > T0)) return fail(ctx, MIOC_EINVAL, "need T1 > T0");
  double par[14] = {};
  for (int q = 0; q < np; ++q) par[q] = params ? params[q] : def[q];
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  {  // k_ode_eval stores every restart's forward states, J-only calls included
    int rc = grow(ctx, &ctx->d_ode_state, &ctx->ode_cap, (size_t)K * nt * 2 * sizeof(double), "ODE states");
    if (rc) return rc;
  }
  const double tau = (T1 - T0) / (double)nt;  // ODEObjective.jl: τ = (T1 - T0) / nt
  HIP_TRY(ctx, launch_ode_eval(ctx->stream, ctx->gate, problem, (int)K, (int)nt, tau, par, np - 2, d_x, d_J, d_df,
                               ctx->d_ode_state));
  return MIOC_OK;
}

int32_t mioc_rand_start_device(mioc_ctx *ctx, int64_t K, int64_t nt, int64_t jumps, uint64_t seed, double *d_u_out) {
  if (!ctx) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  if (!ctx->have_levels) return fail(ctx, MIOC_ESTATE, "levels must be set first");
  if (K < 1 || K > INT32_MAX || nt < 1 || nt > (1 << 24) || !d_u_out) return fail(ctx, MIOC_EINVAL, "bad K / nt / u");
  if (jumps < 0) jumps = nt / 10;
  if (jumps > nt - 1) return fail(ctx, MIOC_EINVAL, "jumps > nt - 1 (the reference's sample would throw)");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, launch_rand_start(ctx->stream, (int)K, (int)nt, (int)jumps, seed, levels_dev(ctx), d_u_out));
  return MIOC_OK;
}

int32_t mioc_batch_multi(mioc_ctx *const *ctxs, int32_t nctx, int64_t K, const double *df, const double *u_old,
                         int64_t nx, int64_t nt, int64_t B, double dt, int64_t B_use, double *u_out, double *phi_star,
                         int32_t *status) {
  if (!ctxs || nctx < 1 || !ctxs[0]) return MIOC_EINVAL;
  for (int32_t d = 0; d < nctx; ++d) {
    if (!ctxs[d]) return fail(ctxs[0], MIOC_EINVAL, "null context in the list");
    for (int32_t e = 0; e < d; ++e)
      if (ctxs[e] == ctxs[d]) return fail(ctxs[0], MIOC_EINVAL, "a context appears twice (contexts are not thread-safe)");
  }
  if (K < 1 || nx < 1 || nt < 1 || !df || !u_old || !u_out) return fail(ctxs[0], MIOC_EINVAL, "bad batch arguments");
  std::vector<int32_t> rcs(nctx, MIOC_OK);
  std::vector<std::thread> th;
  const size_t per = (size_t)nx * nt;
  for (int32_t d = 0; d < nctx; ++d) {
    const int64_t lo = K * d / nctx, hi = K * (d + 1) / nctx;  // contiguous block, as mioc.batch.shard
    if (hi <= lo) continue;
    th.emplace_back([=, &rcs] {
      rcs[d] = batch_host(ctxs[d], hi - lo, df + lo * per, u_old + lo * per, nx, nt, B, dt, B_use, u_out + lo * per,
                          phi_star ? phi_star + lo : nullptr, status ? status + lo : nullptr);
    });
  }
  for (auto &t : th) t.join();
  for (int32_t d = 0; d < nctx; ++d)
    if (rcs[d] != MIOC_OK) {
      if (d > 0) ctxs[0]->err = "context " + std::to_string(d) + ": " + ctxs[d]->err;
      return rcs[d];
    }
  return MIOC_OK;
}

extern "C++" {
namespace {
int trm_check_err(mioc_ctx *ctx);
}  // namespace
}

int32_t mioc_synchronize(mioc_ctx *ctx) {
  if (!ctx) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  ev_collect(ctx);
  if (ctx->trm_pending) {
    ctx->trm_pending = false;
    int rc = trm_check_err(ctx);
    if (rc) return rc;
  }
  return check_run(ctx);
}

void *mioc_stream(mioc_ctx *ctx) {
  if (!ctx) return nullptr;
  (void)join_bt(ctx);  // ordered after the backtracks in flight on the second stream
  return (void *)ctx->stream;
}

int32_t mioc_get_ranks_device(mioc_ctx *ctx, int32_t *d_ranks_out) {
  if (!ctx || !d_ranks_out) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  if (!ctx->have_path) return fail(ctx, MIOC_ESTATE, "no backtrack result to read");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, hipMemcpyAsync(d_ranks_out, ctx->d_ranks, (size_t)ctx->K * ctx->nt * sizeof(int32_t),
                              hipMemcpyDeviceToDevice, ctx->stream));
  return MIOC_OK;
}

// ---- trust-region quantities (multi-trust.jl:117-158, HelpFunctions.jl:251-268) -------------------------
extern "C++" {
namespace {

TrmDev trm_dev(const mioc_ctx *ctx, int mode, int64_t K, int64_t nt) {
  TrmDev T;
  T.K = (int)K;
  T.M = (int)ctx->M;
  T.nt = (int)nt;
  T.L = (int)ctx->L;
  T.dt = ctx->dt;
  T.beta = ctx->beta;
  T.p_kind = ctx->p_kind;
  T.p_int = (int)ctx->p_int;
  T.mode = mode;
  T.gate = ctx->gate;
  T.fma = ctx->pred_fma ? 1 : 0;
  T.df = ctx->d_df;
  T.uold = ctx->d_uold;
  T.ranks = ctx->d_ranks;
  T.nuval = ctx->d_nuval;
  T.vals = ctx->d_vals;
  T.voff = ctx->d_voff;
  T.g2r = ctx->d_g2r;
  T.tvw = ctx->d_tvw;
  T.tvw_len = ctx->tvw_len;
  T.err = reinterpret_cast<int32_t *>(ctx->d_pred_own + 4);
  return T;
}

int trm_ready(mioc_ctx *ctx) {
  if (!ctx) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  if (!ctx->have_levels || !ctx->have_cost) return fail(ctx, MIOC_ESTATE, "levels and cost must be set first");
  if (ctx->p_kind == MIOC_P_TABLE && !ctx->d_g2r)
    return fail(ctx, MIOC_EINVAL, "TV_p with MIOC_P_TABLE needs the level grid lookup (grid too large)");
  if (hipSetDevice(ctx->device) != hipSuccess) return fail(ctx, MIOC_EHIP, "hipSetDevice failed");
  return MIOC_OK;
}

int trm_check_err(mioc_ctx *ctx) {
  int32_t e = 0;
  HIP_TRY(ctx, hipMemcpy(&e, ctx->d_pred_own + 4, sizeof(int32_t), hipMemcpyDeviceToHost));
  if (e) return fail(ctx, MIOC_EINVAL, "TV_p: a control difference is outside the weight table (MIOC_P_INTLUT key "
                                       "beyond table_len, or MIOC_P_TABLE control off the level grid)");
  return MIOC_OK;
}

}  // namespace
}  // extern "C++"

int32_t mioc_pred(mioc_ctx *ctx, double *int_val, double *tv_old, double *tv_new, double *pred) {
  int rc = trm_ready(ctx);
  if (rc) return rc;
  if (!ctx->have_path || !ctx->d_df || !ctx->d_uold || !ctx->d_ranks)
    return fail(ctx, MIOC_ESTATE, "pred needs a backtrack result (mioc_backtrack first)");
  if (ctx->K != 1) return fail(ctx, MIOC_ESTATE, "host pred after a batched bellman: use mioc_pred_batch_device");
  double *o = ctx->d_pred_own;
  TrmDev T = trm_dev(ctx, 7, 1, ctx->nt);
  T.out_int = o, T.out_told = o + 1, T.out_tnew = o + 2, T.out_pred = o + 3;
  if (!ctx->trm_pending) HIP_TRY(ctx, hipMemsetAsync(o + 4, 0, sizeof(double), ctx->stream));
  ctx->trm_pending = false;  // checked below, with this call's own flag
  HIP_TRY(ctx, launch_trm_pred(ctx->stream, T));
  double h[5];
  HIP_TRY(ctx, hipMemcpyAsync(h, o, 5 * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  int32_t e;
  std::memcpy(&e, &h[4], sizeof(e));
  if (e) return trm_check_err(ctx);
  if (int_val) *int_val = h[0];
  if (tv_old) *tv_old = h[1];
  if (tv_new) *tv_new = h[2];
  if (pred) *pred = h[3];
  return MIOC_OK;
}

int32_t mioc_pred_batch_device(mioc_ctx *ctx, double *d_int_val, double *d_tv_old, double *d_tv_new, double *d_pred) {
  int rc = trm_ready(ctx);
  if (rc) return rc;
  if (!ctx->have_path || !ctx->d_df || !ctx->d_uold || !ctx->d_ranks)
    return fail(ctx, MIOC_ESTATE, "pred needs a backtrack result");
  TrmDev T = trm_dev(ctx, 7, ctx->K, ctx->nt);
  T.out_int = d_int_val, T.out_told = d_tv_old, T.out_tnew = d_tv_new, T.out_pred = d_pred;
  // the error flag is cleared by the first enqueue after a check only: an error of an earlier, not yet synchronised
  // TV / pred call stays visible to the next mioc_synchronize
  if (!ctx->trm_pending) HIP_TRY(ctx, hipMemsetAsync(ctx->d_pred_own + 4, 0, sizeof(double), ctx->stream));
  HIP_TRY(ctx, launch_trm_pred(ctx->stream, T));
  ctx->trm_pending = true;
  return MIOC_OK;
}

int32_t mioc_tv_device(mioc_ctx *ctx, int64_t K, const double *d_u, int64_t nx, int64_t nt, double *d_tv) {
  int rc = trm_ready(ctx);
  if (rc) return rc;
  if (!d_u || !d_tv) return fail(ctx, MIOC_EINVAL, "null pointer");
  if (K < 1 || nt < 1 || nt > INT32_MAX || K > INT32_MAX) return fail(ctx, MIOC_EINVAL, "bad K / nt");
  if (nx != ctx->M) return fail(ctx, MIOC_EINVAL, "nx must equal the number of controls of the levels");
  TrmDev T = trm_dev(ctx, 4, K, nt);
  T.u = d_u;
  T.out_tnew = d_tv;
  // the error flag is cleared by the first enqueue after a check only: an error of an earlier, not yet synchronised
  // TV / pred call stays visible to the next mioc_synchronize
  if (!ctx->trm_pending) HIP_TRY(ctx, hipMemsetAsync(ctx->d_pred_own + 4, 0, sizeof(double), ctx->stream));
  HIP_TRY(ctx, launch_trm_pred(ctx->stream, T));
  ctx->trm_pending = true;
  return MIOC_OK;
}

int32_t mioc_trm_decide_device(mioc_ctx *ctx, int64_t K, const double *d_J_old, const double *d_J_new,
                               const double *d_tv_old, const double *d_tv_new, const double *d_pred, double sigma,
                               double *d_ared, int32_t *d_decision) {
  int rc = trm_ready(ctx);
  if (rc) return rc;
  if (K < 1 || K > INT32_MAX) return fail(ctx, MIOC_EINVAL, "bad K");
  if (!d_J_old || !d_J_new || !d_tv_old || !d_tv_new || !d_pred || !d_decision)
    return fail(ctx, MIOC_EINVAL, "null pointer");
  HIP_TRY(ctx, launch_trm_decide(ctx->stream, (int)K, d_J_old, d_J_new, d_tv_old, d_tv_new, d_pred, ctx->beta, sigma,
                                 d_ared, d_decision));
  return MIOC_OK;
}

// ---- device-resident TRM control (multi-trust.jl:92-163) ---------------------------------------------------
int64_t mioc_trm_state_bytes(int64_t K) { return K < 1 || K > 4096 ? -1 : (int64_t)trm_state_bytes((int)K); }

int32_t mioc_trm_attach(mioc_ctx *ctx, void *d_state) {
  if (!ctx) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  ctx->gate = static_cast<const int32_t *>(d_state);
  return MIOC_OK;
}

int32_t mioc_trm_outer_begin_device(mioc_ctx *ctx, int64_t K, void *d_state, const double *d_tv_u, double D0,
                                    int64_t B, int32_t *d_budgets) {
  if (!ctx) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  if (K < 1 || K > 4096 || !d_state || !d_tv_u || !d_budgets) return fail(ctx, MIOC_EINVAL, "bad TRM state arguments");
  if (B < 0 || B > (1 << 20) || !std::isfinite(D0)) return fail(ctx, MIOC_EINVAL, "bad budget");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, launch_trm_outer_begin(ctx->stream, (int)K, d_state, d_tv_u, D0, (int)B, d_budgets));
  return MIOC_OK;
}

int32_t mioc_trm_inner_end_device(mioc_ctx *ctx, int64_t K, void *d_state, double sigma, int64_t kmax, double tau,
                                  int64_t B, const double *d_int_val, const double *d_tv_new, const double *d_J_new,
                                  double *d_J_old, double *d_J, double *d_tv_u, int32_t *d_budgets,
                                  int32_t *d_decision, int64_t n_per_restart, const double *d_trial, double *d_u,
                                  double *d_u_old) {
  if (!ctx) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  if (!ctx->have_cost) return fail(ctx, MIOC_ESTATE, "mioc_set_cost has not been called");
  if (K < 1 || K > 4096 || !d_state || !d_int_val || !d_tv_new || !d_J_new || !d_J_old || !d_J || !d_tv_u ||
      !d_budgets || !d_trial || !d_u || !d_u_old || n_per_restart < 1)
    return fail(ctx, MIOC_EINVAL, "bad TRM state arguments");
  if (!(tau > 0.0) || kmax < 0 || B < 0 || B > (1 << 20)) return fail(ctx, MIOC_EINVAL, "bad TRM parameters");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, launch_trm_inner_end(ctx->stream, (int)K, d_state, ctx->beta, sigma, (int)std::min<int64_t>(kmax, INT32_MAX),
                                    tau, (int)B, d_int_val, d_tv_new, d_J_new, d_J_old, d_J, d_tv_u, d_budgets,
                                    d_decision, (size_t)n_per_restart, d_trial, d_u, d_u_old));
  return MIOC_OK;
}

int32_t mioc_trm_poll(mioc_ctx *ctx, const void *d_state, int32_t *out) {
  if (!ctx || !d_state || !out) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  if (!ctx->h_trm_poll) HIP_TRY(ctx, hipHostMalloc(&ctx->h_trm_poll, 16, 0));
  HIP_TRY(ctx, hipMemcpyAsync(ctx->h_trm_poll, d_state, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  out[0] = ctx->h_trm_poll[0];
  out[1] = ctx->h_trm_poll[1];
  return MIOC_OK;
}

int32_t mioc_kernel_stats(mioc_ctx *ctx, int32_t which, double *total_ms, int64_t *launches, const char **name) {
  if (!ctx || which < 0 || which >= kStats) return MIOC_EINVAL;
  ev_collect(ctx);
  if (total_ms) *total_ms = ctx->stat_ms[which];
  if (launches) *launches = ctx->stat_launches[which];
  if (name) *name = ctx->stat_name[which];
  return MIOC_OK;
}

int32_t mioc_reset_stats(mioc_ctx *ctx) {
  if (!ctx) return MIOC_EINVAL;
  ev_collect(ctx);
  for (int w = 0; w < kStats; ++w) ctx->stat_ms[w] = 0.0, ctx->stat_launches[w] = 0;
  return MIOC_OK;
}

int32_t mioc_last_algo(mioc_ctx *ctx) { return ctx ? ctx->algo : MIOC_EINVAL; }

int32_t mioc_diagnostics(mioc_ctx *ctx, int64_t *counters, int32_t n) {
  if (!ctx || !counters || n < 0) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  int32_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0}, f[4] = {0, 0, 0, 0};
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  if (ctx->d_counters) HIP_TRY(ctx, hipMemcpy(c, ctx->d_counters, sizeof c, hipMemcpyDeviceToHost));
  HIP_TRY(ctx, hipMemcpy(f, ctx->d_flags, sizeof f, hipMemcpyDeviceToHost));
  // slot 6: the separable transform's persistent DPs redone with per-step launches (cooperative launch refused or a
  // dependency wait timed out) -- its kernels write no c[6]; the pyramid's value-collision count otherwise
  // slot 8: row segments per subproblem of the last fused separable DP (0: the one-lane-per-row kernel)
  // (p = Inf: plus the device-side redo of the last DP, counted by the gated one-workgroup recursion in c[6])
  const int64_t c6 = ctx->algo == MIOC_ALGO_SEPARABLE || ctx->algo == MIOC_ALGO_FUSED_SEPARABLE
                         ? ctx->n_persist_fallbacks
                         : ctx->algo == MIOC_ALGO_PINF ? ctx->n_persist_fallbacks + c[6] : c[6];
  // slot 9: after a p=Inf segmented walk, its subproblems left to the serial walk (-1: the serial walk ran alone)
  int32_t fserial = -1;
  if (ctx->algo == MIOC_ALGO_PINF && ctx->last_pinf_fwalk && ctx->pinf.fneed)
    HIP_TRY(ctx, hipMemcpy(&fserial, ctx->pinf.fneed + ctx->K, sizeof fserial, hipMemcpyDeviceToHost));
  // slot 3: internal-consistency failures of the backtrack (f[3]) and of the DP's tables (c[3]: seam-list overflow)
  const int64_t all[10] = {c[0], c[1], f[2], (int64_t)f[3] + c[3], c[4], c[5], c6, ctx->occupancy,
                           ctx->algo == MIOC_ALGO_FUSED_SEPARABLE ? ctx->last_fsep_seg : 0, fserial};
  for (int32_t q = 0; q < n && q < 10; ++q) counters[q] = all[q];
  return MIOC_OK;
}

int32_t mioc_get_argmin_table(mioc_ctx *ctx, int64_t k, int64_t step, int32_t *U_out) {
  if (!ctx || !U_out) return MIOC_EINVAL;
  MIOC_JOIN_BT(ctx);
  if (!ctx->have_dp) return fail(ctx, MIOC_ESTATE, "no bellman result to read");
  if (k < 0 || k >= ctx->K || step < 0 || step + 1 >= ctx->nt)
    return fail(ctx, MIOC_EINVAL, "subproblem or step out of range (0 <= step < nt-1)");
  if (ctx->algo == MIOC_ALGO_PINF)
    return fail(ctx, MIOC_EINVAL, "the p=Inf collapse keeps per-budget class tables, not U");
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  {
    const int rcr = check_run(ctx);  // a timed-out persistent DP is redone before its table is read
    if (rcr) return rcr;
  }
  const int64_t R = ctx->B + 1, L = ctx->L, M = ctx->M, nt = ctx->nt;
  std::vector<double> uo(M);
  HIP_TRY(ctx, hipMemcpy(uo.data(), ctx->d_uold + ((size_t)k * nt + step) * M, M * sizeof(double),
                         hipMemcpyDeviceToHost));
  std::vector<int32_t> out((size_t)R * ctx->Lgrid, -1);
  auto bt = [&](int64_t r) {
    int64_t b = 0;
    for (int64_t m = 0; m < M; ++m) b += (int64_t)std::fabs(ctx->nuval_h[r * M + m] - uo[m]);
    return b;
  };
  const size_t step_cells = (size_t)R * L;
  if (ctx->algo == MIOC_ALGO_PYRAMID || ctx->algo == MIOC_ALGO_SEPARABLE) {  // staged: UU_i[c'][l] = U_i[l, c' + b̃_l(i)]
    std::vector<uint16_t> uu(step_cells);
    const uint16_t *src = (const uint16_t *)ctx->d_U + ((size_t)k * (nt - 1) + step) * step_cells;
    HIP_TRY(ctx, hipMemcpy(uu.data(), src, step_cells * sizeof(uint16_t), hipMemcpyDeviceToHost));
    for (int64_t r = 0; r < L; ++r) {
      const int64_t b = bt(r);
      for (int64_t c = b; c < R; ++c) {  // 0xFFFF: a cell the separable transform left unwritten (Φ = +Inf)
        const uint16_t x = uu[(c - b) * L + r];
        out[c + R * ctx->gidx_h[r]] = x == 0xFFFF ? -1 : (int32_t)x;
      }
    }
  } else {  // generic: U_i[l][c]
    std::vector<unsigned char> raw(step_cells * ctx->ubytes);
    const unsigned char *src = (const unsigned char *)ctx->d_U + ((size_t)k * (nt - 1) + step) * step_cells * ctx->ubytes;
    HIP_TRY(ctx, hipMemcpy(raw.data(), src, raw.size(), hipMemcpyDeviceToHost));
    for (int64_t r = 0; r < L; ++r) {
      const int64_t b = bt(r);
      for (int64_t c = b; c < R; ++c) {
        const size_t q = (size_t)r * R + c;
        out[c + R * ctx->gidx_h[r]] =
            ctx->ubytes == 1 ? (int32_t)raw[q] : (int32_t)reinterpret_cast<const uint16_t *>(raw.data())[q];
      }
    }
  }
  std::memcpy(U_out, out.data(), out.size() * sizeof(int32_t));
  return MIOC_OK;
}

}  // extern "C"
