// VALU f32 FMA throughput: v_fma_f32 vs v_pk_fma_f32 (SGPR-broadcast coefficient), at 1, 2 and
// 4 waves per SIMD.  Decides whether two nodes per lane on packed FMAs can lift the symmetric
// contraction, whose waves are often the only ready wave on their SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f2 __attribute__((ext_vector_type(2)));
#define NACC 8
template <bool PK>
__global__ __launch_bounds__(256) void fma_k(const float* __restrict__ c, float* __restrict__ out, int iters) {
  if (PK) {
    f2 acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = (f2){(float)threadIdx.x, (float)i};
    const f2 x = (f2){1.0001f, 0.9999f};
    for (int it = 0; it < iters; ++it) {
      const float cc = c[it & 15];
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_elementwise_fma((f2){cc, cc}, acc[i], x);
    }
    f2 s = acc[0];
    for (int i = 1; i < NACC; ++i) s += acc[i];
    out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
  } else {
    float acc[NACC];
    for (int i = 0; i < NACC; ++i) acc[i] = (float)threadIdx.x + i;
    for (int it = 0; it < iters; ++it) {
      const float cc = c[it & 15];
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = fmaf(cc, acc[i], 1.0001f);
    }
    float s = 0;
    for (int i = 0; i < NACC; ++i) s += acc[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
  }
}
int main() {
  float *c, *out;
  hipMalloc(&c, 64 * 4); hipMemset(c, 0, 64 * 4);
  hipMalloc(&out, 256 * 4096 * 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int iters = 4096;
  for (int wps = 1; wps <= 4; wps *= 2) {
    const int blocks = 256 * wps;   // 256 threads = 4 waves = one per SIMD of a CU
    for (int pk = 0; pk < 2; ++pk) {
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(a);
        if (pk) hipLaunchKernelGGL(fma_k<true>, dim3(blocks), dim3(256), 0, 0, c, out, iters);
        else hipLaunchKernelGGL(fma_k<false>, dim3(blocks), dim3(256), 0, 0, c, out, iters);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        const double fl = 2.0 * blocks * 256.0 * iters * 8 * NACC * (pk ? 2 : 1);
        if (rep == 2) printf("waves/SIMD %d %-10s %.3f ms  %.1f TFLOP/s\n", wps, pk ? "pk_fma" : "fma", ms, fl / ms / 1e9);
      }
    }
  }
  return 0;
}
