// fp32 VALU FMA ceiling on gfx950: what one CU's SIMDs sustain for the
// instruction mix of the symmetric contraction (accumulator += SGPR coefficient x VGPR operand).
//
// Variants (all: 16 independent accumulators per lane, coefficients preloaded into SGPRs from the
// kernel arguments so the loop issues no memory instruction, no literal operands):
//   fmac_s   acc[i] = fma(c_k, v[i], acc[i])   VOP2 v_fmac_f32 with an SGPR coefficient
//   fma_vvv  acc[i] = fma(v[i], w[i], acc[i])  all-VGPR VOP3 / VOP2 form
//   fma_lit  acc[i] = fma(c, acc[i], 1.0001f)  the round-4 pkfma_bench form (literal addend)
//   pk_s     acc2[i] = pk_fma((c_k, c_k), v2[i], acc2[i])   v_pk_fma_f32, coefficient pair in SGPRs
//   fmac_v   as fmac_s with the coefficient moved to a VGPR first (one v_mov per 16 FMAs)
//   pk_sel   v_pk_fma_f32 broadcasting ONE half of an SGPR pair (op_sel / op_sel_hi, inline asm)
//   pk_v     v_pk_fma_f32, all-VGPR operands
// at 1, 2, 3, 4 and 8 waves per SIMD (one 256-thread block = one wave per SIMD of a CU; the grid
// is 256 x W blocks).  Reports TFLOP/s (2 per FMA lane-op), each block's loop span from the
// 100 MHz wall clock, how many blocks per CU actually ran at once, and ns per wave-instruction
// per SIMD.
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
  const long long t0 = wall_clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < UNR; ++k)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_fmaf(cf.c[k], v[i], acc[i]);
  }
  const long long t1 = wall_clock64();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t0; clk[2 * blockIdx.x + 1] = t1; }
}

__global__ __launch_bounds__(256) void fma_vvv(Coefs cf, float* __restrict__ out, int iters,
                                               long long* __restrict__ clk) {
  float acc[NACC], v[NACC], w[UNR];
#pragma unroll
  for (int i = 0; i < NACC; ++i) { acc[i] = 0.f; v[i] = (float)(threadIdx.x + i) * 1e-3f; }
#pragma unroll
  for (int k = 0; k < UNR; ++k) w[k] = cf.c[k] + (float)threadIdx.x * 1e-7f;   // per-lane VGPRs
  const long long t0 = wall_clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < UNR; ++k)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_fmaf(w[k], v[i], acc[i]);
  }
  const long long t1 = wall_clock64();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t0; clk[2 * blockIdx.x + 1] = t1; }
}

__global__ __launch_bounds__(256) void fma_lit(Coefs cf, float* __restrict__ out, int iters,
                                               long long* __restrict__ clk) {
  float acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = (float)(threadIdx.x + i) * 1e-3f;
  const long long t0 = wall_clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < UNR; ++k)
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_fmaf(cf.c[k], acc[i], 1.0001f);
  }
  const long long t1 = wall_clock64();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t0; clk[2 * blockIdx.x + 1] = t1; }
}

__global__ __launch_bounds__(256) void pk_s(Coefs cf, float* __restrict__ out, int iters,
                                            long long* __restrict__ clk) {
  f2 acc[NACC / 2], v[NACC / 2];
#pragma unroll
  for (int i = 0; i < NACC / 2; ++i) {
    acc[i] = (f2){0.f, 0.f};
    v[i] = (f2){(float)(threadIdx.x + i) * 1e-3f, (float)(threadIdx.x - i) * 1e-3f};
  }
  const long long t0 = wall_clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const f2 c2 = (f2){cf.c[k], cf.c[k]};
#pragma unroll
      for (int i = 0; i < NACC / 2; ++i) acc[i] = __builtin_elementwise_fma(c2, v[i], acc[i]);
    }
  }
  const long long t1 = wall_clock64();
  f2 s = acc[0];
#pragma unroll
  for (int i = 1; i < NACC / 2; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t0; clk[2 * blockIdx.x + 1] = t1; }
}


__global__ __launch_bounds__(256) void fmac_v(Coefs cf, float* __restrict__ out, int iters,
                                              long long* __restrict__ clk) {
  float acc[NACC], v[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) { acc[i] = 0.f; v[i] = (float)(threadIdx.x + i) * 1e-3f; }
  const long long t0 = wall_clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      float cv = cf.c[k];
      asm volatile("v_mov_b32 %0, %1" : "=v"(cv) : "s"(cf.c[k]));   // uniform coefficient in a VGPR
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_fmaf(cv, v[i], acc[i]);
    }
  }
  const long long t1 = wall_clock64();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t0; clk[2 * blockIdx.x + 1] = t1; }
}

__global__ __launch_bounds__(256) void pk_v(Coefs cf, float* __restrict__ out, int iters,
                                            long long* __restrict__ clk) {
  f2 acc[NACC / 2], v[NACC / 2], w[UNR];
#pragma unroll
  for (int i = 0; i < NACC / 2; ++i) {
    acc[i] = (f2){0.f, 0.f};
    v[i] = (f2){(float)(threadIdx.x + i) * 1e-3f, (float)(threadIdx.x - i) * 1e-3f};
  }
#pragma unroll
  for (int k = 0; k < UNR; ++k) w[k] = (f2){cf.c[k] + threadIdx.x * 1e-7f, cf.c[k] - threadIdx.x * 1e-7f};
  const long long t0 = wall_clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < UNR; ++k)
#pragma unroll
      for (int i = 0; i < NACC / 2; ++i) acc[i] = __builtin_elementwise_fma(w[k], v[i], acc[i]);
  }
  const long long t1 = wall_clock64();
  f2 s = acc[0];
#pragma unroll
  for (int i = 1; i < NACC / 2; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t0; clk[2 * blockIdx.x + 1] = t1; }
}

// the coefficient pair (c_2j, c_2j+1) sits in one aligned SGPR pair; each packed FMA broadcasts
// ONE half of it to both lanes of the pair through op_sel / op_sel_hi (no s_mov to build (c, c))
__global__ __launch_bounds__(256) void pk_sel(Coefs cf, float* __restrict__ out, int iters,
                                              long long* __restrict__ clk) {
  f2 acc[NACC / 2], v[NACC / 2];
#pragma unroll
  for (int i = 0; i < NACC / 2; ++i) {
    acc[i] = (f2){0.f, 0.f};
    v[i] = (f2){(float)(threadIdx.x + i) * 1e-3f, (float)(threadIdx.x - i) * 1e-3f};
  }
  const long long t0 = wall_clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < UNR; k += 2) {
      const f2 cp = (f2){cf.c[k], cf.c[k + 1]};
#pragma unroll
      for (int i = 0; i < NACC / 2; ++i)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel_hi:[0,1,1]" : "+v"(acc[i]) : "s"(cp), "v"(v[i]));
#pragma unroll
      for (int i = 0; i < NACC / 2; ++i)
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc[i]) : "s"(cp), "v"(v[i]));
    }
  }
  const long long t1 = wall_clock64();
  f2 s = acc[0];
#pragma unroll
  for (int i = 1; i < NACC / 2; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
  if (threadIdx.x == 0) { clk[2 * blockIdx.x] = t0; clk[2 * blockIdx.x + 1] = t1; }
}

typedef void (*kfn)(Coefs, float*, int, long long*);

int main() {
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  float* out;
  long long* clk;
  const int maxb = ncu * 8;
  hipMalloc(&out, (size_t)256 * maxb * 4);
  hipMalloc(&clk, (size_t)2 * maxb * 8);
  long long* hclk = (long long*)malloc((size_t)2 * maxb * 8);
  Coefs cf;
  for (int k = 0; k < UNR; ++k) cf.c[k] = 0.999f + 1e-4f * k;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 8192;
  struct { const char* name; kfn f; int lane_ops_per_inst; } ks[] = {
      {"fmac_s", fmac_s, 1}, {"fmac_v", fmac_v, 1}, {"fma_vvv", fma_vvv, 1}, {"fma_lit", fma_lit, 1},
      {"pk_s", pk_s, 2}, {"pk_sel", pk_sel, 2}, {"pk_v", pk_v, 2}};
  printf("CUs %d; %d FMA lane-ops per lane (16 acc x %d unroll x %d iters); wall_clock64 = 100 MHz\n",
         ncu, NACC * UNR * iters, UNR, iters);
  const int wps_list[] = {1, 2, 3, 4, 8};
  for (int wi = 0; wi < 5; ++wi) {
    const int wps = wps_list[wi];
    const int blocks = ncu * wps;      // 256 threads = one wave per SIMD of a CU
    for (auto& k : ks) {
      float best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, cf, out, iters, clk);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (rep > 0 && ms < best) {
          best = ms;
          hipMemcpy(hclk, clk, (size_t)2 * blocks * 8, hipMemcpyDeviceToHost);
        }
      }
      // per-block loop spans (100 MHz ticks): mean span, and the mean number of blocks whose
      // loop is running at an instant (sum of spans / union extent) = blocks resident per CU x CUs
      long long lo = hclk[0], hi = hclk[1];
      double sum = 0;
      for (int i = 0; i < blocks; ++i) {
        lo = hclk[2 * i] < lo ? hclk[2 * i] : lo;
        hi = hclk[2 * i + 1] > hi ? hclk[2 * i + 1] : hi;
        sum += (double)(hclk[2 * i + 1] - hclk[2 * i]);
      }
      const double span_us = sum / blocks / 100.0;
      const double conc = sum / (double)(hi - lo) / ncu;          // blocks running per CU
      const double flops = 2.0 * (double)blocks * 256.0 * NACC * UNR * iters;
      const double inst = (double)NACC * UNR * iters / k.lane_ops_per_inst;   // per wave
      // one wave's loop: instructions / span -> ns per wave-instruction; with `conc` waves
      // sharing a SIMD, per-SIMD ns per instruction = span / (inst * conc)
      printf("waves/SIMD %d  %-8s %8.3f ms  %6.1f TFLOP/s  loop span %8.1f us  %.2f waves/SIMD "
             "running  %.3f ns per wave-instr per SIMD\n", wps, k.name, best, flops / best / 1e9,
             span_us, conc, span_us * 1e3 / (inst * conc));
    }
  }
  return 0;
}
