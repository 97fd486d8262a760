// mioc_sdt_common.h -- device helpers shared by the separable L1 transform kernels (mioc_sdt.hip: the per-step
// kernel, the one-workgroup-per-row persistent driver; mioc_sdt2.hip: the two-workgroups-per-row persistent driver).
// See mioc_sdt.hip's header for the certified fixed-point transform these constants describe.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace mioc {

constexpr int SD_RB = 12;                // payload rank bits (L <= 4096)
constexpr int SD_CB = 6;                 // payload near-tie count bits, below the rank (at most 56 merges per value)
constexpr int SD_CNT = (1 << SD_CB) - 1; // near-tie count mask: nonzero = flagged
constexpr int SD_PAY = (1 << (SD_CB + SD_RB)) - 1;  // payload mask: 18 low mantissa bits
constexpr int SD_GRID = 52 - SD_CB - SD_RB;         // g = 2^(E - SD_GRID) for the binade [2^E, 2^(E+1))
constexpr int SD_COOP = 8;               // listed targets up to this many: whole-workgroup scans, else one wave each
constexpr int SD_FEW = 4;                // rows with at most this many targets go straight to the exact scan
constexpr int SD_SPARSE = 4;             // rows with at most this many finite sources: direct minimum over them
constexpr int SD_LCAP = 512;             // listed targets kept in LDS; beyond, the scan sweeps every rank

// v_min_f64 without llvm.minnum's canonicalising v_max_f64 x,x on every operand (inputs are finite or +Inf)
__device__ __forceinline__ double sd_min(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// min(a, |b|) in one instruction (the abs is an operand modifier; fabs() on an asm operand would cost a v_and)
__device__ __forceinline__ double sd_min_abs(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, |%2|" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double sd_max(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// The thread index as a value the compiler cannot hoist out of the persistent driver's row loop: everything the
// row body derives from it (LDS addresses of the passes, swizzles, store offsets) is recomputed per row instead of
// being kept live in VGPRs across the whole loop, which would leave the body no registers (spills to scratch join
// the vector-memory queue the driver keeps busy).
__device__ __forceinline__ int sd_tid() {
  int t = (int)threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

// LDS-only workgroup barrier: __syncthreads() would also wait for every outstanding global load and store of
// the wave, which the persistent driver keeps in flight across the row body on purpose
__device__ __forceinline__ void sd_bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// merge two disjoint candidate sets (their minima a, b): the smaller keeps its payload; a near tie counts
// one.  |a - b| is exact (one binade), +Inf - +Inf is NaN and never flags.
__device__ __forceinline__ double sd_merge(double a, double b, double tol) {
  const double m = sd_min(a, b);
  const bool close = fabs(a - b) <= tol;
  return __hiloint2double(__double2hiint(m), (int)((unsigned)__double2loint(m) + (close ? 1u : 0u)));  // v_addc
}

// Wave-wide reductions through DPP (no LDS round trip, unlike __shfl_xor's ds_bpermute): four steps leave every
// lane with its 16-lane row's result (quad_perm xor 1, xor 2, row_half_mirror, row_mirror), then the four row
// results are read as scalars.  bound_ctrl: every lane has a source under these controls, so no old value is
// needed (and no register initialised for it).
template <int CTRL>
__device__ __forceinline__ int sd_dpp_i(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ double sd_dpp_d(double x) {
  return __hiloint2double(sd_dpp_i<CTRL>(__double2hiint(x)), sd_dpp_i<CTRL>(__double2loint(x)));
}
__device__ __forceinline__ double sd_rdl(double x, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l), __builtin_amdgcn_readlane(__double2loint(x), l));
}
// (min and max without llvm.minnum's canonicalisation: the operands are finite or ±Inf, never NaN)
__device__ __forceinline__ void sd_wave_stats(double &mn, double &mx) {
#define SD_STEP(C)                             \
  mn = sd_min(mn, sd_dpp_d<C>(mn));            \
  mx = sd_max(mx, sd_dpp_d<C>(mx));
  SD_STEP(0xB1) SD_STEP(0x4E) SD_STEP(0x141) SD_STEP(0x140)
#undef SD_STEP
  mn = sd_min(sd_min(sd_rdl(mn, 0), sd_rdl(mn, 16)), sd_min(sd_rdl(mn, 32), sd_rdl(mn, 48)));
  mx = sd_max(sd_max(sd_rdl(mx, 0), sd_rdl(mx, 16)), sd_max(sd_rdl(mx, 32), sd_rdl(mx, 48)));
}

// LDS position of rank r (3 bits per dimension): XOR swizzle so that each 32-lane half of a pass reads
// 32 distinct 8-byte bank slots in every pass: slot = (x0 ^ x1) + 8·((x1 ^ x2) & 3)
__device__ __forceinline__ int sd_swz(int r) { return r ^ ((r >> 3) & 7) ^ (((r >> 6) & 3) << 3); }

// rank of element x of line q in the pass over dimension m (q enumerates the other coordinates, lowest
// dimension fastest)
__device__ __forceinline__ int sd_rank(int q, int m, int x) {
  const int lo = q & ((1 << (3 * m)) - 1);
  return lo | (x << (3 * m)) | ((q >> (3 * m)) << (3 * (m + 1)));
}

// L1 distance between two ranks of the 8^M grid with one v_sad_u8: a rank spread to one byte per dimension
__device__ __forceinline__ unsigned sd_bytes(unsigned r) {
  return (r & 7u) | ((r & 0x38u) << 5) | ((r & 0x1C0u) << 10) | ((r & 0xE00u) << 15);
}
__device__ __forceinline__ unsigned sd_l1(unsigned pa, unsigned pb) { return __builtin_amdgcn_sad_u8(pa, pb, 0u); }

typedef unsigned int sd_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int sd_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sd_rsrc(const double *base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double *>(base), 0, bytes, 0x00020000);
}

// Wave-local LDS ordering: this wave's LDS stores are complete before its next LDS reads (LDS instructions of one
// wave execute in order; the wait also keeps the compiler from moving accesses across)
__device__ __forceinline__ void sd_wave_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

}  // namespace mioc
