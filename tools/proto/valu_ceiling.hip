// fp32 VALU FMA ceiling on gfx950: what one CU's SIMDs sustain for the
// instruction mix of the symmetric contraction (accumulator += SGPR coefficient x VGPR operand).
//
// Variants (all: 16 independent accumulators per lane, coefficients preloaded into SGPRs from the
// kernel arguments so the loop issues no memory instruction, no literal operands):
//   fmac_s   acc[i] = fma(c_k, v[i], acc[i])   VOP2 v_fmac_f32 with an SGPR coefficient
//   fma_vvv  acc[i] = fma(v[i], w[i], acc[i])  all-VGPR VOP3 / VOP2 form
//   fma_lit  acc[i] = fma(c, acc[i], 1.0001f)  the round-4 pkfma_bench form (literal addend)
//   pk_s     acc2[i] = pk_fma((c_k, c_k), v2[i], acc2[i])   v_pk_fma_f32, coefficient pair in SGPRs
// at 1, 2, 3, 4 and 8 waves per SIMD (one 256-thread block = one wave per SIMD of a CU; the grid
// is 256 x W blocks).  Reports TFLOP/s (2 per FMA lane-op, 4 per packed) and cycles per
// wave-instruction per SIMD at the measured clock (s_memtime over the kernel in one lane).
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_ceiling valu_ceiling.hip
//        (ISA: add -save-temps, or llvm-objdump -d on the code object)
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));
#define NACC 16
#define UNR 8

struct Coefs { float c[UNR]; };

__global__ __launch_bounds__(256) void fmac_s(Coefs cf, float* __restrict__ out, int iters,
                                              long long* __restrict__ clk) {
  float acc[NACC], v[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) { acc[i] = 0.f; v[i] = (float)(threadIdx.x + i) * 1e-3f; }
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < UNR; ++k)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_fmaf(cf.c[k], v[i], acc[i]);
  }
  const long long t1 = clock64();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = t1 - t0;
}

__global__ __launch_bounds__(256) void fma_vvv(Coefs cf, float* __restrict__ out, int iters,
                                               long long* __restrict__ clk) {
  float acc[NACC], v[NACC], w[UNR];
#pragma unroll
  for (int i = 0; i < NACC; ++i) { acc[i] = 0.f; v[i] = (float)(threadIdx.x + i) * 1e-3f; }
#pragma unroll
  for (int k = 0; k < UNR; ++k) w[k] = cf.c[k] + (float)threadIdx.x * 1e-7f;   // per-lane VGPRs
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < UNR; ++k)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_fmaf(w[k], v[i], acc[i]);
  }
  const long long t1 = clock64();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = t1 - t0;
}

__global__ __launch_bounds__(256) void fma_lit(Coefs cf, float* __restrict__ out, int iters,
                                               long long* __restrict__ clk) {
  float acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = (float)(threadIdx.x + i) * 1e-3f;
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < UNR; ++k)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_fmaf(cf.c[k], acc[i], 1.0001f);
  }
  const long long t1 = clock64();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = t1 - t0;
}

__global__ __launch_bounds__(256) void pk_s(Coefs cf, float* __restrict__ out, int iters,
                                            long long* __restrict__ clk) {
  f2 acc[NACC / 2], v[NACC / 2];
#pragma unroll
  for (int i = 0; i < NACC / 2; ++i) {
    acc[i] = (f2){0.f, 0.f};
    v[i] = (f2){(float)(threadIdx.x + i) * 1e-3f, (float)(threadIdx.x - i) * 1e-3f};
  }
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const f2 c2 = (f2){cf.c[k], cf.c[k]};
#pragma unroll
      for (int i = 0; i < NACC / 2; ++i) acc[i] = __builtin_elementwise_fma(c2, v[i], acc[i]);
    }
  }
  const long long t1 = clock64();
  f2 s = acc[0];
#pragma unroll
  for (int i = 1; i < NACC / 2; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
  if (blockIdx.x == 0 && threadIdx.x == 0) clk[0] = t1 - t0;
}

typedef void (*kfn)(Coefs, float*, int, long long*);

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  long long* clk;
  hipMalloc(&out, (size_t)256 * ncu * 8 * 4);
  hipMalloc(&clk, 8);
  Coefs cf;
  for (int k = 0; k < UNR; ++k) cf.c[k] = 0.999f + 1e-4f * k;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 8192;
  struct { const char* name; kfn f; int lane_ops_per_fma; } ks[] = {
      {"fmac_s", fmac_s, 1}, {"fma_vvv", fma_vvv, 1}, {"fma_lit", fma_lit, 1}, {"pk_s", pk_s, 2}};
  printf("CUs %d; %d FMA wave-instructions per wave (16 acc x %d unroll x %d iters)\n", ncu,
         NACC * UNR * iters, UNR, iters);
  const int wps_list[] = {1, 2, 3, 4, 8};
  for (int wi = 0; wi < 5; ++wi) {
    const int wps = wps_list[wi];
    const int blocks = ncu * wps;      // 256 threads = one wave per SIMD of a CU
    for (auto& k : ks) {
      float best = 1e30f;
      long long cyc = 0;
      for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, cf, out, iters, clk);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (rep > 0 && ms < best) {
          best = ms;
          hipMemcpy(&cyc, clk, 8, hipMemcpyDeviceToHost);
        }
      }
      const int ninst = NACC * UNR * iters / k.lane_ops_per_fma;   // wave-instructions per wave
      const double flops = 2.0 * (double)blocks * 256.0 * NACC * UNR * iters;
      // cycles per wave-instruction per SIMD, from one wave's clock64 span (waves of a SIMD
      // share it): span / (instructions of all waves resident on the SIMD)
      const double cpi = (double)cyc / ((double)ninst * wps);
      printf("waves/SIMD %d  %-8s %8.3f ms  %6.1f TFLOP/s  %5.2f cyc per wave-instr per SIMD"
             "  (clock64 span %lld, %.2f GHz)\n", wps, k.name, best, flops / best / 1e9, cpi, cyc,
             cyc / (best * 1e6));
    }
  }
  return 0;
}
