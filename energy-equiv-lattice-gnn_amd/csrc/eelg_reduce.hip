// Deterministic sums over the leading dimension of partial results:
//   out[c] = scale * sum_{r < rows} part[r * ld + c],  c < cols
// The step's partial-sum reductions (per-slice weight gradients of the linears, the radial MLP's
// per-workgroup gradients, the contraction's per-chunk coefficient gradients) and the bias
// gradients (column sums of grad_out over the nodes) go through here instead of torch's
// reduce_kernel (r04i torch profile: 33 sums, 0.95 ms/step of device time).
//
// A 256-thread block (4 waves) owns CB column quads (4 consecutive columns, a float4 when the
// layout allows; CB = 64, or the next power of two >= the quad count of a narrow matrix), so a
// wave-load covers P = 64 / CB rows: lane = (phase, quad).  Wave w, phase ph sums rows
// w*P + ph, + 4P, ... in ascending order with 8 row loads in flight; the 4 x P partial sums of a
// quad are then added in (wave, phase) order through LDS.  Fixed order everywhere: the result
// does not depend on the launch.  Small blocks, so a reduction launched beside the step's large
// kernels finds room on a CU.  Longer reductions (rows > RED_ROWS_1P: the radial partials, the bias sums over
// 32k nodes) first reduce row chunks of RED_CHUNK rows into a workspace (grid.y = chunk), then
// sum the chunk partials the same way.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/eelg.h"
#include "eelg_internal.h"

#define RED_WAVES 4
#define RED_CHUNK 256     // rows per first-pass chunk of a long reduction
#define RED_ROWS_1P 256   // longest reduction summed in one pass (a wave sums <= 64 rows)

__device__ __forceinline__ void red_add(float4& a, const float4& b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
}

template <bool VEC>
__device__ __forceinline__ float4 red_load(const float* __restrict__ p, long long c0, long long cols) {
  if (VEC) return *reinterpret_cast<const float4*>(p);
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c0 + 0 < cols) v.x = p[0];
  if (c0 + 1 < cols) v.y = p[1];
  if (c0 + 2 < cols) v.z = p[2];
  if (c0 + 3 < cols) v.w = p[3];
  return v;
}

// rows [y * rows_per_y, ...) of part (row stride ld) summed into out + blockIdx.y * out_ld;
// cb = column quads per block (a power of two <= 64)
template <bool VEC>
__global__ __launch_bounds__(64 * RED_WAVES) void sum_rows_kernel(const float* __restrict__ part, long long ld,
                                                                  int rows, int rows_per_y, long long cols,
                                                                  int cb, float scale, float* __restrict__ out,
                                                                  long long out_ld) {
  __shared__ float4 red[RED_WAVES][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int P = 64 / cb, ph = lane / cb, qd = lane - ph * cb;
  const long long c0 = ((long long)blockIdx.x * cb + qd) * 4;
  const int r_beg = blockIdx.y * rows_per_y, r_end = min(rows, r_beg + rows_per_y);
  const int step = RED_WAVES * P;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c0 < cols) {
    const float* __restrict__ p = part + c0;
    int r = r_beg + wave * P + ph;
    for (; r + 7 * step < r_end; r += 8 * step) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = red_load<VEC>(p + (size_t)(r + u * step) * ld, c0, cols);
#pragma unroll
      for (int u = 0; u < 8; ++u) red_add(acc, v[u]);
    }
    for (; r < r_end; r += step) red_add(acc, red_load<VEC>(p + (size_t)r * ld, c0, cols));
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (threadIdx.x < cb && ((long long)blockIdx.x * cb + threadIdx.x) * 4 < cols) {
    const long long c = ((long long)blockIdx.x * cb + threadIdx.x) * 4;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int w = 0; w < RED_WAVES; ++w)
      for (int q = 0; q < P; ++q) red_add(s, red[w][q * cb + threadIdx.x]);
    s.x *= scale; s.y *= scale; s.z *= scale; s.w *= scale;
    float* __restrict__ o = out + (size_t)blockIdx.y * out_ld + c;
    if (VEC) {
      *reinterpret_cast<float4*>(o) = s;
    } else {
      if (c + 0 < cols) o[0] = s.x;
      if (c + 1 < cols) o[1] = s.y;
      if (c + 2 < cols) o[2] = s.z;
      if (c + 3 < cols) o[3] = s.w;
    }
  }
}

static int red_launch(const float* part, long long ld, int rows, int rows_per_y, int ny, long long cols,
                      float scale, float* out, long long out_ld, hipStream_t s) {
  const bool vec = (ld % 4 == 0) && (cols % 4 == 0) && (out_ld % 4 == 0) &&
                   (reinterpret_cast<uintptr_t>(part) % 16 == 0) && (reinterpret_cast<uintptr_t>(out) % 16 == 0);
  const long long quads = (cols + 3) / 4;
  int cb = 1;
  while (cb < 64 && cb < quads) cb *= 2;
  const long long nb = (quads + cb - 1) / cb;
  if (nb > INT32_MAX) return eelg_fail(-2, "sum_rows: %lld columns", cols);
  dim3 grid((unsigned)nb, (unsigned)ny);
  if (vec)
    hipLaunchKernelGGL(sum_rows_kernel<true>, grid, dim3(64 * RED_WAVES), 0, s, part, ld, rows, rows_per_y,
                       cols, cb, scale, out, out_ld);
  else
    hipLaunchKernelGGL(sum_rows_kernel<false>, grid, dim3(64 * RED_WAVES), 0, s, part, ld, rows, rows_per_y,
                       cols, cb, scale, out, out_ld);
  return eelg_check_launch("sum_rows");
}

extern "C" {

long long eelg_sum_rows_work(int rows, long long cols) {
  return rows > RED_ROWS_1P ? (long long)((rows + RED_CHUNK - 1) / RED_CHUNK) * cols : 0;
}

int eelg_sum_rows(const float* part, long long ld, int rows, long long cols, float scale, float* out,
                  float* work, long long work_len, void* stream) {
  if (rows < 0 || cols < 0 || ld < cols) return eelg_fail(-2, "sum_rows: rows %d, cols %lld, ld %lld", rows, cols, ld);
  if (cols == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  if (rows == 0) {
    if (hipMemsetAsync(out, 0, (size_t)cols * sizeof(float), s) != hipSuccess)
      return eelg_fail(-3, "sum_rows: memset failed");
    return 0;
  }
  if (rows <= RED_ROWS_1P) return red_launch(part, ld, rows, rows, 1, cols, scale, out, cols, s);
  const int chunks = (rows + RED_CHUNK - 1) / RED_CHUNK;
  if (!work || work_len < (long long)chunks * cols)
    return eelg_fail(-2, "sum_rows: %d rows need a workspace of %lld floats (eelg_sum_rows_work)", rows,
                     (long long)chunks * cols);
  const int rc = red_launch(part, ld, rows, RED_CHUNK, chunks, cols, 1.0f, work, cols, s);
  if (rc) return rc;
  return red_launch(work, cols, chunks, chunks, 1, cols, scale, out, cols, s);
}

}  // extern "C"
