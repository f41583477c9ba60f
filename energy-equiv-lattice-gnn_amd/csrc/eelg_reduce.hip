// Deterministic sums over the leading dimension of partial results:
//   out[c] = scale * sum_{r < rows} part[r * ld + c],  c < cols
// The step's partial-sum reductions (per-slice weight gradients of the linears, the radial MLP's
// per-workgroup gradients, the contraction's per-chunk coefficient gradients) and the bias
// gradients (column sums of grad_out over the nodes) go through here instead of torch's
// reduce_kernel (r04i torch profile: 33 sums, 0.95 ms/step of device time).
//
// A 1024-thread block owns 256 columns (a lane 4 consecutive columns, a float4 when the layout
// allows); its 16 waves split the rows (wave w sums rows w, w + 16, ... in ascending order, 8 row
// loads in flight, each wave-load one coalesced 1 KB run of a row) and the 16 wave sums are added
// in wave order through LDS.  Fixed order everywhere: the result does not depend on the launch.
// Long reductions (rows > RED_ROWS_1P, e.g. the bias sums over 32k nodes) first reduce row chunks
// of RED_CHUNK rows into a workspace (grid.y = chunk), then sum the chunk partials the same way.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/eelg.h"
#include "eelg_internal.h"

#define RED_WAVES 16
#define RED_CHUNK 1024    // rows per first-pass chunk of a long reduction
#define RED_ROWS_1P 2048  // longest reduction summed in one pass

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

// rows [r_beg, r_end) of part (row stride ld) summed into out + blockIdx.y * out_ld
template <bool VEC>
__global__ __launch_bounds__(64 * RED_WAVES) void sum_rows_kernel(const float* __restrict__ part, long long ld,
                                                                  int rows, int rows_per_y, long long cols,
                                                                  float scale, float* __restrict__ out,
                                                                  long long out_ld) {
  __shared__ float4 red[RED_WAVES][64];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long c0 = ((long long)blockIdx.x * 64 + lane) * 4;
  const int r_beg = blockIdx.y * rows_per_y, r_end = min(rows, r_beg + rows_per_y);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (c0 < cols) {
    const float* __restrict__ p = part + c0;
    int r = r_beg + wave;
    for (; r + 7 * RED_WAVES < r_end; r += 8 * RED_WAVES) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = red_load<VEC>(p + (size_t)(r + u * RED_WAVES) * ld, c0, cols);
#pragma unroll
      for (int u = 0; u < 8; ++u) red_add(acc, v[u]);
    }
    for (; r < r_end; r += RED_WAVES) red_add(acc, red_load<VEC>(p + (size_t)r * ld, c0, cols));
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && c0 < cols) {
    float4 s = red[0][lane];
#pragma unroll
    for (int w = 1; w < RED_WAVES; ++w) red_add(s, red[w][lane]);
    s.x *= scale; s.y *= scale; s.z *= scale; s.w *= scale;
    float* __restrict__ o = out + (size_t)blockIdx.y * out_ld + c0;
    if (VEC) {
      *reinterpret_cast<float4*>(o) = s;
    } else {
      if (c0 + 0 < cols) o[0] = s.x;
      if (c0 + 1 < cols) o[1] = s.y;
      if (c0 + 2 < cols) o[2] = s.z;
      if (c0 + 3 < cols) o[3] = s.w;
    }
  }
}

static int red_launch(const float* part, long long ld, int rows, int rows_per_y, int ny, long long cols,
                      float scale, float* out, long long out_ld, hipStream_t s) {
  const bool vec = (ld % 4 == 0) && (cols % 4 == 0) && (out_ld % 4 == 0) &&
                   (reinterpret_cast<uintptr_t>(part) % 16 == 0) && (reinterpret_cast<uintptr_t>(out) % 16 == 0);
  const long long nb = (cols + 255) / 256;
  if (nb > INT32_MAX) return eelg_fail(-2, "sum_rows: %lld columns", cols);
  dim3 grid((unsigned)nb, (unsigned)ny);
  if (vec)
    hipLaunchKernelGGL(sum_rows_kernel<true>, grid, dim3(64 * RED_WAVES), 0, s, part, ld, rows, rows_per_y,
                       cols, scale, out, out_ld);
  else
    hipLaunchKernelGGL(sum_rows_kernel<false>, grid, dim3(64 * RED_WAVES), 0, s, part, ld, rows, rows_per_y,
                       cols, scale, out, out_ld);
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
