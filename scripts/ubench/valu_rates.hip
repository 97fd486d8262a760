// Micro-benchmark: issue cost of FP64 VALU instructions on gfx950 (cycles per wave64 instruction, s_memtime),
// 8 independent chains per wave, 1 or 2 waves per SIMD.  Build: hipcc --offload-arch=gfx950 -O3 valu_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 4096
template <int OP>
__global__ void kern(double *out, unsigned long long *cyc, double seed) {
  double x[8];
  for (int q = 0; q < 8; ++q) x[q] = seed + threadIdx.x + q;
  double y = seed * 0.5;
  int xi[8];
  for (int q = 0; q < 8; ++q) xi[q] = threadIdx.x + q;
  int yi = (int)seed;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < N; ++it) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      if (OP == 0) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x[q]) : "v"(y));
      if (OP == 1) asm volatile("v_min_f64 %0, %0, %1" : "+v"(x[q]) : "v"(y));
      if (OP == 2) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x[q]) : "v"(y));
      if (OP == 3) asm volatile("v_cmp_lt_f64 vcc, %1, %2\n v_cndmask_b32 %0, %0, %3, vcc" : "+v"(xi[q]) : "v"(x[q]), "v"(y), "v"(yi) : "vcc");
      if (OP == 4) asm volatile("v_max_f64 %0, %0, %1" : "+v"(x[q]) : "v"(y));
      if (OP == 5) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(x[q]) : "v"(y));
      if (OP == 6) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(xi[q]) : "v"(yi) : "vcc");
      if (OP == 7) asm volatile("v_cmp_lt_f64 vcc, %0, %1" : : "v"(x[q]), "v"(y) : "vcc");
      if (OP == 8) asm volatile("v_add_u32 %0, %0, %1" : "+v"(xi[q]) : "v"(yi));
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
  for (int q = 0; q < 8; ++q) s += x[q] + xi[q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
  double *out; unsigned long long *cyc;
  hipMalloc(&out, (size_t)1024 * 1024 * 8); hipMalloc(&cyc, 1024 * 8);
  const char *nm[] = {"v_add_f64", "v_min_f64", "v_fma_f64", "v_cmp_lt_f64+cndmask", "v_max_f64", "v_mul_f64",
                      "v_cndmask_b32", "v_cmp_lt_f64", "v_add_u32"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int threads : {256, 512, 1024}) {
    for (int op = 0; op < 9; ++op) {
      void (*k)(double *, unsigned long long *, double) = nullptr;
      switch (op) { case 0: k = kern<0>; break; case 1: k = kern<1>; break; case 2: k = kern<2>; break;
        case 3: k = kern<3>; break; case 4: k = kern<4>; break; case 5: k = kern<5>; break; case 6: k = kern<6>; break;
        case 7: k = kern<7>; break; default: k = kern<8>; }
      hipLaunchKernelGGL(k, dim3(256), dim3(threads), 0, 0, out, cyc, 1.0);
      hipDeviceSynchronize();
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(k, dim3(1024), dim3(threads), 0, 0, out, cyc, 1.0);
      hipEventRecord(e1, 0);
      hipDeviceSynchronize();
      float ms = 0; hipEventElapsedTime(&ms, e0, e1);
      double lane_ops = 1024.0 * threads * N * 8 * (op == 3 ? 2 : 1);
      printf("   wall %.3f ms: %.2f T lane-instr/s (1024 WGs)\n", ms, lane_ops / ms / 1e9);
      unsigned long long h[256];
      hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
      double avg = 0; for (int b = 0; b < 256; ++b) avg += h[b]; avg /= 256;
      printf("%4d thr/WG (%d waves/SIMD)  %-22s  %.2f cycles per wave-instruction (per wave)\n", threads, threads / 256, nm[op],
             avg / (N * 8));
    }
  }
  return 0;
}
