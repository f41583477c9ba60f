// Channel-mixing linear on e3nn mul-major irreps rows (o3.Linear,
// gnn/blocks.py:516-521,553-559,471-476; gnn/model.py:82-86), fp32 MFMA.
//
// For one output slot (mul_out copies of an irrep of dimension d):
//   y[n, j, m] = sum_src alpha_src * sum_u x[n, x_off + u*d + m] * W[u, j]   (+ bias[j] if d == 1)
// i.e. a GEMM whose rows are (node, component) pairs, K = mul_in, N = mul_out.
// One wave computes a 32-row x 32-column tile with v_mfma_f32_32x32x2_f32
// (exact f32: a k-ordered fmaf chain).  The same kernel serves grad-x with
// the transposed weight (ldk/ldj swapped).  grad-W reduces over rows with
// deterministic per-wave partials (summed on the host side).
#include <hip/hip_runtime.h>

typedef float eelg_f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void lin_fwd_kernel(const float* __restrict__ x, int x_row,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ bias, int n_nodes,
                                                      float* __restrict__ y, int y_row,
                                                      eelg_lin_desc desc) {
  const eelg_lin_slot& sl = desc.slot[blockIdx.y];
  const int d = sl.d;
  const int rows = n_nodes * d;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int tile0 = (blockIdx.x * 4 + wave) * 32;
  const int jt = blockIdx.z * 32;
  if (tile0 >= rows || jt >= sl.n_out) return;
  const int kh = lane >> 5;
  const int r = tile0 + (lane & 31);
  const bool rok = r < rows;
  const int n = rok ? r / d : 0;
  const int m = rok ? r - n * d : 0;
  const int j = jt + (lane & 31);
  const bool jok = j < sl.n_out;
  eelg_f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  for (int s = 0; s < sl.n_src; ++s) {
    const eelg_lin_src& src = sl.src[s];
    const float* __restrict__ xa = x + (size_t)n * x_row + src.x_off + m + kh * d;
    const float* __restrict__ wb = w + src.w_off + (size_t)j * src.ldj + kh * src.ldk;
    const float al = src.alpha;
    const int xs = 2 * d, ws = 2 * src.ldk;
    const int k_even = src.k & ~1;
#pragma unroll 8
    for (int kk = 0; kk < k_even; kk += 2) {
      const float a = rok ? xa[(kk >> 1) * xs] : 0.0f;
      const float b = jok ? wb[(kk >> 1) * ws] * al : 0.0f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    if (src.k & 1) {  // odd K: the upper half-wave (k index k_even+1) contributes zero
      const bool ok = kh == 0;
      const float a = (ok && rok) ? xa[(k_even >> 1) * xs] : 0.0f;
      const float b = (ok && jok) ? wb[(k_even >> 1) * ws] * al : 0.0f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
  }
  if (!jok) return;
  const float bj = (sl.bias_off >= 0) ? bias[sl.bias_off + j] : 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int rr = tile0 + (i & 3) + 8 * (i >> 2) + 4 * kh;
    if (rr < rows) {
      const int nn = rr / d, mm = rr - nn * d;
      y[(size_t)nn * y_row + sl.y_off + j * d + mm] = acc[i] + bj;
    }
  }
}

// grad W for each instruction: partial[p, w_off + u*n_out + j] =
//   alpha * sum_{rows of this wave's slice} x[n, x_off + u*d + m] * g[n, g_off + j*d + m]
__global__ __launch_bounds__(256) void lin_bwdw_kernel(const float* __restrict__ x, int x_row,
                                                       const float* __restrict__ g, int g_row,
                                                       int n_nodes, int rows_per_wave,
                                                       float* __restrict__ partial, int w_total,
                                                       eelg_linw_desc desc) {
  const eelg_linw_ins& in = desc.ins[blockIdx.y];
  const int d = in.d;
  const int rows = n_nodes * d;
  const int n_ut = (in.k + 31) / 32;
  const int uti = blockIdx.z / desc.max_jt, jti = blockIdx.z % desc.max_jt;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int slice = blockIdx.x * 4 + wave;
  float* __restrict__ dst = partial + (size_t)slice * w_total + in.w_off;
  if (uti >= n_ut || jti * 32 >= in.n_out) return;
  const int kh = lane >> 5;
  const int u = uti * 32 + (lane & 31);
  const int j = jti * 32 + (lane & 31);
  const bool uok = u < in.k, jok = j < in.n_out;
  eelg_f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  const int r0 = slice * rows_per_wave;
  const int r1 = min(rows, r0 + rows_per_wave);
  if (r0 < r1) {
    // this lane walks rows r0 + kh, r0 + kh + 2, ...
    int r = r0 + kh;
    int n = r / d, m = r - n * d;
    const float* __restrict__ xb = x + in.x_off + (size_t)u * d;
    const float* __restrict__ gb = g + in.g_off + (size_t)j * d;
    for (; r - kh < r1; r += 2) {
      const bool ok = r < r1;
      const float a = (ok && uok) ? xb[(size_t)n * x_row + m] : 0.0f;
      const float b = (ok && jok) ? gb[(size_t)n * g_row + m] : 0.0f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
      m += 2;
      if (m >= d) { m -= d; ++n; if (m >= d) { m -= d; ++n; } }
    }
  }
  if (!jok) return;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int uu = uti * 32 + (i & 3) + 8 * (i >> 2) + 4 * kh;
    if (uu < in.k) dst[uu * in.n_out + j] = acc[i] * in.alpha;
  }
}
