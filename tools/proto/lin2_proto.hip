// Prototype: channel-mixing linear with row-per-lane direct loads (no LDS transpose of X).
// y[n, y_off + j*d + m] = sum_u x[n, x_off + u*d + m] * W[u, j]   per slot (d = 2l+1, K = mul_in)
// MFMA 32x32x2 f32: A[row][k] = X[(n,m)][u] (lane = row, lane half = K half), B[k][j] = W[u][j]
// (W slot staged once per workgroup in LDS).  Timing harness for the 7360->800 and 800->800
// shapes of BASELINE config 2 (N = 32768).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include <algorithm>

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct Slot { int x_off, k, y_off, d; };

#ifndef PF
#define PF 8
#endif
#ifndef RW
#define RW 1
#endif

template <int KMAX>
__global__ __launch_bounds__(256) void lin2_fwd(const float* __restrict__ x, int x_row,
                                                const float* __restrict__ w, int n_nodes,
                                                float* __restrict__ y, int y_row, const Slot* slots,
                                                const int* w_off) {
  __shared__ float ws[KMAX * 33];
  const Slot s = slots[blockIdx.y];
  const int d = s.d, K = s.k, KH = (K + 1) / 2;
  const int rows = n_nodes * d;
  const int r0 = blockIdx.x * 128 * RW;
  if (r0 >= rows) return;
  const float* __restrict__ wsl = w + w_off[blockIdx.y];
  for (int i = threadIdx.x; i < K * 32; i += 256) ws[(i >> 5) * 33 + (i & 31)] = wsl[i];
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 31, hf = lane >> 5;
#pragma unroll 1
  for (int rt = 0; rt < RW; ++rt) {
    const int row = r0 + (rt * 4 + wave) * 32 + i;
    const bool ok = row < rows;
    const int n = ok ? row / d : 0, m = ok ? row - (row / d) * d : 0;
    const float* __restrict__ xa = x + (size_t)n * x_row + s.x_off + m + (size_t)hf * KH * d;
    const int kend = hf ? K - KH : KH;     // valid k in this half
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    float pf[PF];
#pragma unroll
    for (int q = 0; q < PF; ++q) pf[q] = (q < kend) ? xa[(size_t)q * d] : 0.f;
    for (int st = 0; st < KH; st += PF) {
#pragma unroll
      for (int q = 0; q < PF; ++q) {
        if (st + q < KH) {   // wave-uniform
          const float a = pf[q];
          const int kn = st + PF + q;
          pf[q] = (kn < kend) ? xa[(size_t)kn * d] : 0.f;
          const int kk = hf * KH + st + q;
          const float b = kk < K ? ws[kk * 33 + i] : 0.f;
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ok ? a : 0.f, b, acc, 0, 0, 0);
        }
      }
    }
    // epilogue: acc[r] = row (r&3) + 8(r>>2) + 4hf of the tile, column j = i
    const int rb = r0 + (rt * 4 + wave) * 32;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = rb + (r & 3) + 8 * (r >> 2) + 4 * hf;
      if (rr < rows) {
        const int nn = rr / d, mm = rr - nn * d;
        y[(size_t)nn * y_row + s.y_off + i * d + mm] = acc[r];
      }
    }
  }
}

int main(int argc, char** argv) {
  const int N = 32768;
  struct Cfg { const char* name; int x_row, y_row; std::vector<Slot> slots; };
  std::vector<Cfg> cfgs = {
      {"7360->800", 7360, 800, {}}, {"800->800", 800, 800, {}}};
  {
    int ks[5] = {160, 256, 320, 320, 288};
    int xo = 0, yo = 0;
    for (int l = 0; l < 5; ++l) { int d = 2 * l + 1; cfgs[0].slots.push_back({xo, ks[l], yo, d}); xo += ks[l] * d; yo += 32 * d; }
    xo = yo = 0;
    for (int l = 0; l < 5; ++l) { int d = 2 * l + 1; cfgs[1].slots.push_back({xo, 32, yo, d}); xo += 32 * d; yo += 32 * d; }
  }
  for (auto& c : cfgs) {
    size_t nx = (size_t)N * c.x_row, ny = (size_t)N * c.y_row;
    std::vector<float> hx(nx), hw;
    std::vector<int> woff;
    for (auto& v : hx) v = (float)rand() / RAND_MAX - 0.5f;
    for (auto& s : c.slots) { woff.push_back((int)hw.size()); for (int q = 0; q < s.k * 32; ++q) hw.push_back((float)rand() / RAND_MAX - 0.5f); }
    float *dx, *dw, *dy; Slot* ds; int* dwo;
    hipMalloc(&dx, nx * 4); hipMalloc(&dy, ny * 4); hipMalloc(&dw, hw.size() * 4);
    hipMalloc(&ds, c.slots.size() * sizeof(Slot)); hipMalloc(&dwo, woff.size() * 4);
    hipMemcpy(dx, hx.data(), nx * 4, hipMemcpyHostToDevice);
    hipMemcpy(dw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(ds, c.slots.data(), c.slots.size() * sizeof(Slot), hipMemcpyHostToDevice);
    hipMemcpy(dwo, woff.data(), woff.size() * 4, hipMemcpyHostToDevice);
    hipMemset(dy, 0, ny * 4);
    dim3 grid((N * 9 + 128 * RW - 1) / (128 * RW), c.slots.size());
    auto run = [&]() { hipLaunchKernelGGL((lin2_fwd<320>), grid, dim3(256), 0, 0, dx, c.x_row, dw, N, dy, c.y_row, ds, dwo); };
    for (int it = 0; it < 3; ++it) run();
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    std::vector<float> ts;
    for (int it = 0; it < 20; ++it) { hipEventRecord(a); run(); hipEventRecord(b); hipEventSynchronize(b); float ms; hipEventElapsedTime(&ms, a, b); ts.push_back(ms); }
    std::sort(ts.begin(), ts.end());
    std::vector<float> hy(ny);
    hipMemcpy(hy.data(), dy, ny * 4, hipMemcpyDeviceToHost);
    double maxerr = 0, maxref = 0;
    for (int n : {0, 1, 777, N - 1}) {
      for (size_t si = 0; si < c.slots.size(); ++si) {
        auto& s = c.slots[si];
        for (int j = 0; j < 32; ++j) for (int m = 0; m < s.d; ++m) {
          double acc = 0;
          for (int u = 0; u < s.k; ++u) acc += (double)hx[(size_t)n * c.x_row + s.x_off + u * s.d + m] * hw[woff[si] + u * 32 + j];
          double got = hy[(size_t)n * c.y_row + s.y_off + j * s.d + m];
          maxerr = fmax(maxerr, fabs(got - acc)); maxref = fmax(maxref, fabs(acc));
        }
      }
    }
    double bytes = 4.0 * N * (c.x_row + c.y_row);
    printf("%-10s PF=%d RW=%d median %.4f ms  %.0f GB/s  rel err %.2e\n", c.name, PF, RW, ts[10], bytes / ts[10] / 1e6, maxerr / maxref);
    hipFree(dx); hipFree(dy); hipFree(dw); hipFree(ds); hipFree(dwo);
  }
  return 0;
}
