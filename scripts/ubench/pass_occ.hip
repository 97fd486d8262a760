// Micro-benchmark: one L1-transform pass of k_sdt_run's row body (4096 fixed-point f64 values in LDS, 8-point lines,
// 14 near-tie-counting merges per line) at 512 threads (one line per thread, 2 waves per SIMD) against 1024 threads
// (half a line per thread, the two halves mirrored on a lane pair, one DPP exchange: 4 waves per SIMD).  Cycles per
// pass (s_memtime, wave 0) for the whole 4096-value array, with a workgroup barrier after every pass as in the row
// body's last pass, and without it (wave-local passes).  Build: hipcc --offload-arch=gfx950 -O3 pass_occ.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int L = 4096, NPASS = 256;

__device__ __forceinline__ double vmin(double a, double b) {
  double r;
  asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double merge(double a, double b, double tol) {
  const double m = vmin(a, b);
  const bool close = fabs(a - b) <= tol;
  return __hiloint2double(__double2hiint(m), (int)((unsigned)__double2loint(m) + (close ? 1u : 0u)));
}
__device__ __forceinline__ int swz(int r) { return r ^ ((r >> 3) & 7) ^ (((r >> 6) & 3) << 3); }
__device__ __forceinline__ int rankof(int q, int m, int x) {
  const int lo = q & ((1 << (3 * m)) - 1);
  return lo | (x << (3 * m)) | ((q >> (3 * m)) << (3 * (m + 1)));
}
__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
__device__ __forceinline__ void wsync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <bool BAR>
__global__ __launch_bounds__(512) void k8(double *out, unsigned long long *cyc, double tol) {
  __shared__ double d[L];
  const int t = threadIdx.x;
  for (int e = t; e < L; e += 512) d[e] = 1024.0 + (double)((e * 2654435761u) % 997);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < NPASS; ++it) {
    const int m = it % 3;  // dims 0..2: the lines of a wave stay inside the wave (as passes 0..2)
    int pos[8];
    double o[8];
#pragma unroll
    for (int x = 0; x < 8; ++x) {
      pos[x] = swz(rankof(t, m, x));
      o[x] = d[pos[x]];
    }
#pragma unroll
    for (int x = 1; x < 8; ++x) o[x] = merge(o[x], o[x - 1] + 1.0, tol);
#pragma unroll
    for (int x = 6; x >= 0; --x) o[x] = merge(o[x], o[x + 1] + 1.0, tol);
#pragma unroll
    for (int x = 0; x < 8; ++x) d[pos[x]] = o[x];
    if (BAR) bar(); else wsync();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  out[blockIdx.x * 512 + t] = d[t] + d[t + 2048];
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

// 1024 threads: lane pair (2p, 2p+1) owns line p; lane 2p holds x = 0..3, lane 2p+1 holds x = 7..4 (mirrored), so
// both run the same instructions: a forward sweep over their four, the partner's end value + 1 merged into slot 3,
// then a backward sweep (7 merges per lane, 14 per line, chain depth 7)
template <bool BAR>
__global__ __launch_bounds__(1024) void k4(double *out, unsigned long long *cyc, double tol) {
  __shared__ double d[L];
  const int t = threadIdx.x;
  for (int e = t; e < L; e += 1024) d[e] = 1024.0 + (double)((e * 2654435761u) % 997);
  __syncthreads();
  const int line = t >> 1, h = t & 1;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < NPASS; ++it) {
    const int m = it % 3;
    int pos[4];
    double o[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int x = h ? 7 - s : s;
      pos[s] = swz(rankof(line, m, x));
      o[s] = d[pos[s]];
    }
#pragma unroll
    for (int s = 1; s < 4; ++s) o[s] = merge(o[s], o[s - 1] + 1.0, tol);
    // partner's slot 3 (its sweep end: min over its four sources of V + distance to its slot-3 point) via DPP
    const double p = __hiloint2double(__builtin_amdgcn_update_dpp(0, __double2hiint(o[3]), 0xB1, 0xF, 0xF, true),
                                      __builtin_amdgcn_update_dpp(0, __double2loint(o[3]), 0xB1, 0xF, 0xF, true));
    o[3] = merge(o[3], p + 1.0, tol);
#pragma unroll
    for (int s = 2; s >= 0; --s) o[s] = merge(o[s], o[s + 1] + 1.0, tol);
#pragma unroll
    for (int s = 0; s < 4; ++s) d[pos[s]] = o[s];
    if (BAR) bar(); else wsync();
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  __syncthreads();
  out[blockIdx.x * 1024 + t] = d[t] + d[t + 2048];
  if (t == 0) cyc[blockIdx.x] = t1 - t0;
}

template <class K>
static void run(const char *name, K kern, int threads, double *out, unsigned long long *cyc) {
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, out, cyc, 3.0);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, out, cyc, 3.0);
  hipEventRecord(e1, 0);
  hipDeviceSynchronize();
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[256];
  hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int b = 0; b < 256; ++b) avg += h[b];
  avg /= 256;
  printf("%-34s %4d thr: %7.1f cycles per pass (s_memtime), wall %.3f ms = %.3f us per pass\n", name, threads,
         avg / NPASS, ms, ms * 1e3 / NPASS);
}

int main() {
  double *out;
  unsigned long long *cyc;
  hipMalloc(&out, 256 * 1024 * sizeof(double));
  hipMalloc(&cyc, 256 * sizeof(unsigned long long));
  run("8 values/thread, barrier per pass", k8<true>, 512, out, cyc);
  run("8 values/thread, wave-local", k8<false>, 512, out, cyc);
  run("4 values/thread, barrier per pass", k4<true>, 1024, out, cyc);
  run("4 values/thread, wave-local", k4<false>, 1024, out, cyc);
  return 0;
}
