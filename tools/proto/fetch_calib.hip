// FETCH_SIZE calibration: each kernel reads one 1 GiB buffer exactly once with a given load
// width per lane (4 B coalesced as tp_fwd's weight rows; 8; 12 B unaligned-vector as the
// x / accumulator runs; 16 B as the SH rows), so rocprofv3 --pmc FETCH_SIZE reports the
// counter's bytes for a known HBM read volume.  Run: rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f3u __attribute__((ext_vector_type(3), aligned(4)));
typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));

__global__ void rd4(const float* __restrict__ p, size_t n, float* out) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc += p[i];
  if (acc == 12345.f) out[0] = acc;
}
__global__ void rd8(const float* __restrict__ p, size_t n, float* out) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; 2 * i < n; i += (size_t)gridDim.x * 256) {
    const f2u v = *reinterpret_cast<const f2u*>(p + 2 * i);
    acc += v.x + v.y;
  }
  if (acc == 12345.f) out[0] = acc;
}
__global__ void rd12(const float* __restrict__ p, size_t n, float* out) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; 3 * i + 2 < n; i += (size_t)gridDim.x * 256) {
    const f3u v = *reinterpret_cast<const f3u*>(p + 3 * i);
    acc += v.x + v.y + v.z;
  }
  if (acc == 12345.f) out[0] = acc;
}
__global__ void rd16(const float* __restrict__ p, size_t n, float* out) {
  float acc = 0.f;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; 4 * i < n; i += (size_t)gridDim.x * 256) {
    const float4 v = *reinterpret_cast<const float4*>(p + 4 * i);
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.f) out[0] = acc;
}
// write side: every byte written once, 4 and 16 B per lane
__global__ void wr4(float* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = (float)i;
}
__global__ void wr16(float* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; 4 * i < n; i += (size_t)gridDim.x * 256)
    reinterpret_cast<float4*>(p)[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

int main() {
  const size_t n = (size_t)1 << 28;   // 1 GiB of floats
  float *p, *o;
  hipMalloc(&p, n * 4);
  hipMalloc(&o, 4);
  hipMemset(p, 0, n * 4);
  const dim3 g(4096), b(256);
  hipLaunchKernelGGL(wr4, g, b, 0, 0, p, n);
  hipLaunchKernelGGL(wr16, g, b, 0, 0, p, n);
  hipLaunchKernelGGL(rd4, g, b, 0, 0, p, n, o);
  hipLaunchKernelGGL(rd8, g, b, 0, 0, p, n, o);
  hipLaunchKernelGGL(rd12, g, b, 0, 0, p, n, o);
  hipLaunchKernelGGL(rd16, g, b, 0, 0, p, n, o);
  hipDeviceSynchronize();
  printf("bytes per kernel: %zu\n", n * 4);
  hipFree(p);
  hipFree(o);
  return 0;
}
