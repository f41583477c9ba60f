// Symmetric contraction of degree <= 4 from a term table: correlation 4 (gnn/mace.py:180-280
// with U_matrix_real's filter_ir_mid, gnn/mace.py:435-477).  The generated kernels
// (gen_kernels.py: sc_fwd / sc_bwd_x / sc_bwd_coef) cover correlation 1..3 with straight-line
// code per irreps structure; correlation 4 has ~6.7k degree-4 monomial terms already at lmax 3,
// so it runs here from a table instead:
//
//   out[n, c, q] = sum_{t in q} coef[c, t] * x_i0 x_i1 x_i2 x_i3      (i = D: the constant 1)
//
// terms[t] packs the four component indices (8 bits each; unused slots = D, a row of ones in
// LDS, so every term is four reads and three multiplies with no branch), sorted by output
// component q; desc.orow[q] .. orow[q+1] is q's term range.  Layouts as the generated kernels:
// node rows of mul-major irreps blocks, component a of channel c at x[n*ldx + xb[a] + c*xs[a]].
//
// Forward and grad-x: one thread per (node, channel), its components in an LDS column (no barrier:
// a thread reads only its own column), grad-x's accumulators in registers indexed by the
// wave-uniform table entries (s_set_gpr_idx); the term loops are wave-uniform (scalar loads of
// the table and the channel's coefficients).  Coefficient gradient: as sc_bwd_coef, one
// workgroup = one channel x EELG_SCG_CHUNK LDS-resident nodes, each wave sweeps 64-term batches
// over the chunk with per-lane accumulators, reduced over the 64 lanes (eelg_lane_reduce64);
// deterministic partials [chunk, mul, ldc], summed by the caller.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/eelg.h"
#include "eelg_internal.h"

#define SCG_T 256   // threads per workgroup

__device__ __forceinline__ int scg_i(unsigned tm, int k) { return (int)((tm >> (8 * k)) & 0xffu); }

// Forward: the thread's components in an LDS column (row D = the constant 1), four terms per
// iteration with their table entries, coefficients and LDS reads independent.
__global__ __launch_bounds__(SCG_T) void scg_fwd_kernel(eelg_scg_desc d, const unsigned* __restrict__ terms,
                                                       const float* __restrict__ x, int ldx,
                                                       const float* __restrict__ coef, int ldc, int n_nodes,
                                                       float* __restrict__ out, int ldo) {
  extern __shared__ float sx[];   // (D + 1) rows of SCG_T
  const int c = blockIdx.y, tid = threadIdx.x;
  const int n = blockIdx.x * SCG_T + tid;
  const bool ok = n < n_nodes;
  const size_t row = (size_t)(ok ? n : 0) * ldx;
  for (int a = 0; a < d.D; ++a) sx[a * SCG_T + tid] = ok ? x[row + d.xb[a] + c * d.xs[a]] : 0.0f;
  sx[d.D * SCG_T + tid] = 1.0f;
  const float* __restrict__ cr = coef + (size_t)c * ldc;
  const float* __restrict__ col = sx + tid;
  for (int q = 0; q < d.Dout; ++q) {
    float acc = 0.0f, acc2 = 0.0f;
    int t = d.orow[q];
    const int te = d.orow[q + 1];
    for (; t + 4 <= te; t += 4) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const unsigned tm = terms[t + u];
        v[u] = (col[scg_i(tm, 0) * SCG_T] * col[scg_i(tm, 1) * SCG_T]) *
               (col[scg_i(tm, 2) * SCG_T] * col[scg_i(tm, 3) * SCG_T]);
      }
      acc = fmaf(cr[t], v[0], acc);
      acc2 = fmaf(cr[t + 1], v[1], acc2);
      acc = fmaf(cr[t + 2], v[2], acc);
      acc2 = fmaf(cr[t + 3], v[3], acc2);
    }
    for (; t < te; ++t) {
      const unsigned tm = terms[t];
      acc = fmaf(cr[t], (col[scg_i(tm, 0) * SCG_T] * col[scg_i(tm, 1) * SCG_T]) *
                            (col[scg_i(tm, 2) * SCG_T] * col[scg_i(tm, 3) * SCG_T]), acc);
    }
    if (ok) out[(size_t)n * ldo + d.ob[q] + c * d.os[q]] = acc + acc2;
  }
}

// grad_x[a] = sum_t coef_t g_q(t) d(x_i0 x_i1 x_i2 x_i3)/dx_a: each factor slot k adds the
// product of the other three to slot i_k's accumulator (a repeated index collects one
// contribution per occurrence, the product rule).  The components are read from the thread's LDS
// column; the accumulators live in registers indexed by the wave-uniform table entries
// (s_set_gpr_idx; slot D, the constant, collects and is dropped), so the updates form no LDS
// read-modify-write chains.
template <int DM>
__global__ __launch_bounds__(SCG_T) void scg_bwd_x_kernel(eelg_scg_desc d, const unsigned* __restrict__ terms,
                                                         const float* __restrict__ x, int ldx,
                                                         const float* __restrict__ coef, int ldc,
                                                         const float* __restrict__ gout, int ldg, int n_nodes,
                                                         float* __restrict__ gx) {
  const int c = blockIdx.y;
  const int n = blockIdx.x * SCG_T + threadIdx.x;
  const bool ok = n < n_nodes;
  const size_t row = (size_t)(ok ? n : 0) * ldx, grow = (size_t)(ok ? n : 0) * ldg;
  extern __shared__ float sx[];   // (D + 1) rows of SCG_T: the components, row D = 1
  float gr[DM];
#pragma unroll
  for (int a = 0; a < DM; ++a) gr[a] = 0.0f;
  for (int a = 0; a < d.D; ++a) sx[a * SCG_T + threadIdx.x] = ok ? x[row + d.xb[a] + c * d.xs[a]] : 0.0f;
  sx[d.D * SCG_T + threadIdx.x] = 1.0f;
  const float* __restrict__ col = sx + threadIdx.x;
  const float* __restrict__ cr = coef + (size_t)c * ldc;
  for (int q = 0; q < d.Dout; ++q) {
    if (d.orow[q] == d.orow[q + 1]) continue;   // uniform
    const float go = ok ? gout[grow + d.ob[q] + c * d.os[q]] : 0.0f;
#pragma unroll 4
    for (int t = d.orow[q]; t < d.orow[q + 1]; ++t) {
      const unsigned tm = terms[t];
      const int i0 = scg_i(tm, 0), i1 = scg_i(tm, 1), i2 = scg_i(tm, 2), i3 = scg_i(tm, 3);
      const float x0 = col[i0 * SCG_T], x1 = col[i1 * SCG_T], x2 = col[i2 * SCG_T], x3 = col[i3 * SCG_T];
      const float cg = cr[t] * go;
      const float p01 = x0 * x1, p23 = x2 * x3;
      gr[i0] = fmaf(cg * x1, p23, gr[i0]);
      gr[i1] = fmaf(cg * x0, p23, gr[i1]);
      gr[i2] = fmaf(cg * x3, p01, gr[i2]);
      gr[i3] = fmaf(cg * x2, p01, gr[i3]);
    }
  }
#pragma unroll
  for (int a = 0; a < DM; ++a)
    if (ok && a < d.D) gx[row + d.xb[a] + c * d.xs[a]] = gr[a];
}

// partial[ch, c, t] = sum over chunk ch's nodes of g_{out[t]} * x_i0 x_i1 x_i2 x_i3.  LDS:
// rows sx[0..D] (row D = 1) and sg[0..Dout] (row Dout = 0, the padding terms' output) of
// EELG_SCG_CHUNK nodes each.
__global__ __launch_bounds__(SCG_T) void scg_bwd_coef_kernel(eelg_scg_desc d, const unsigned* __restrict__ terms,
                                                            const int* __restrict__ tout, int ldc,
                                                            const float* __restrict__ x, int ldx,
                                                            const float* __restrict__ gout, int ldg,
                                                            int n_nodes, float* __restrict__ part) {
  extern __shared__ float sm[];
  constexpr int CH = EELG_SCG_CHUNK;
  float* __restrict__ sx = sm;
  float* __restrict__ sg = sm + (d.D + 1) * CH;
  const int ch = blockIdx.x, c = blockIdx.y, tid = threadIdx.x;
  for (int j = tid; j < CH; j += SCG_T) {
    const int n = ch * CH + j;
    const bool ok = n < n_nodes;
    const size_t xr = (size_t)(ok ? n : 0) * ldx, gr = (size_t)(ok ? n : 0) * ldg;
    for (int a = 0; a < d.D; ++a) sx[a * CH + j] = ok ? x[xr + d.xb[a] + c * d.xs[a]] : 0.0f;
    sx[d.D * CH + j] = 1.0f;
    for (int q = 0; q < d.Dout; ++q) sg[q * CH + j] = ok ? gout[gr + d.ob[q] + c * d.os[q]] : 0.0f;
    sg[d.Dout * CH + j] = 0.0f;
  }
  __syncthreads();
  const int wv = tid >> 6, lane = tid & 63;
  float* __restrict__ dst = part + ((size_t)ch * d.mul + c) * ldc;
  for (int b = wv; b * 64 < ldc; b += SCG_T / 64) {
    const int t0 = __builtin_amdgcn_readfirstlane(b * 64);
    float acc[64];
#pragma unroll
    for (int i = 0; i < 64; ++i) acc[i] = 0.0f;
#pragma unroll 1
    for (int s = 0; s < CH / 64; ++s) {
      const float* __restrict__ xc = sx + s * 64 + lane;
      const float* __restrict__ gc = sg + s * 64 + lane;
      // the batch's table is re-read (scalar cache) per sub-tile: hoisted out of the loop, its
      // 128 words would not fit the SGPRs and spill into VGPR lanes
      const unsigned* tp = terms + t0;
      const int* op = tout + t0;
      asm volatile("" : "+s"(tp), "+s"(op));
#pragma unroll
      for (int i = 0; i < 64; ++i) {
        const unsigned tm = tp[i];
        const float v = (xc[scg_i(tm, 0) * CH] * xc[scg_i(tm, 1) * CH]) *
                        (xc[scg_i(tm, 2) * CH] * xc[scg_i(tm, 3) * CH]);
        acc[i] = fmaf(gc[op[i] * CH], v, acc[i]);
      }
    }
    eelg_lane_reduce64(acc);
    dst[t0 + lane] = acc[0];
  }
}

static int scg_check(const eelg_scg_desc* d, int ldc) {
  if (!d) return eelg_fail(-2, "scg: null descriptor");
  if (d->D < 1 || d->D > EELG_SCG_MAXD || d->Dout < 1 || d->Dout > EELG_SCG_MAXD)
    return eelg_fail(-2, "scg: D %d / Dout %d outside 1..%d", d->D, d->Dout, EELG_SCG_MAXD);
  if (d->mul < 1 || d->mul > 65535) return eelg_fail(-2, "scg: mul %d", d->mul);
  if (d->orow[0] != 0 || d->orow[d->Dout] != d->nterms)
    return eelg_fail(-2, "scg: term ranges must cover 0..nterms (%d)", d->nterms);
  for (int q = 0; q < d->Dout; ++q)
    if (d->orow[q + 1] < d->orow[q]) return eelg_fail(-2, "scg: term ranges not ascending");
  if (ldc < d->nterms || ldc % 64) return eelg_fail(-2, "scg: ldc %d must be a multiple of 64 >= nterms %d",
                                                    ldc, d->nterms);
  return 0;
}

extern "C" {

int eelg_scg_fwd(const eelg_scg_desc* d, const unsigned* terms, const float* x, int ldx, const float* coef,
                 int ldc, int n_nodes, float* out, int ldo, void* stream) {
  if (int rc = scg_check(d, ldc)) return rc;
  if (n_nodes < 0) return eelg_fail(-2, "scg_fwd: negative node count");
  if (n_nodes == 0) return 0;
  const dim3 grid((n_nodes + SCG_T - 1) / SCG_T, d->mul);
  hipLaunchKernelGGL(scg_fwd_kernel, grid, dim3(SCG_T), (d->D + 1) * SCG_T * sizeof(float), (hipStream_t)stream,
                     *d, terms, x, ldx, coef, ldc, n_nodes, out, ldo);
  return eelg_check_launch("scg_fwd");
}

int eelg_scg_bwd_x(const eelg_scg_desc* d, const unsigned* terms, const float* x, int ldx, const float* coef,
                   int ldc, const float* grad_out, int ldg, int n_nodes, float* grad_x, void* stream) {
  if (int rc = scg_check(d, ldc)) return rc;
  if (n_nodes < 0) return eelg_fail(-2, "scg_bwd_x: negative node count");
  if (n_nodes == 0) return 0;
  const dim3 grid((n_nodes + SCG_T - 1) / SCG_T, d->mul);
  if (d->D <= 16)
    hipLaunchKernelGGL(scg_bwd_x_kernel<17>, grid, dim3(SCG_T), (d->D + 1) * SCG_T * sizeof(float),
                       (hipStream_t)stream, *d, terms, x, ldx, coef, ldc, grad_out, ldg, n_nodes, grad_x);
  else
    hipLaunchKernelGGL(scg_bwd_x_kernel<EELG_SCG_MAXD + 1>, grid, dim3(SCG_T), (d->D + 1) * SCG_T * sizeof(float),
                       (hipStream_t)stream, *d, terms, x, ldx, coef, ldc, grad_out, ldg, n_nodes, grad_x);
  return eelg_check_launch("scg_bwd_x");
}

int eelg_scg_bwd_coef(const eelg_scg_desc* d, const unsigned* terms, const int* term_out, int ldc, const float* x,
                      int ldx, const float* grad_out, int ldg, int n_nodes, float* partial, void* stream) {
  if (int rc = scg_check(d, ldc)) return rc;
  if (n_nodes < 0) return eelg_fail(-2, "scg_bwd_coef: negative node count");
  if (n_nodes == 0) return 0;
  const dim3 grid((n_nodes + EELG_SCG_CHUNK - 1) / EELG_SCG_CHUNK, d->mul);
  const size_t lds = (size_t)(d->D + 1 + d->Dout + 1) * EELG_SCG_CHUNK * sizeof(float);
  static bool lds_attr = false;   // > 64 KB of dynamic LDS must be allowed explicitly
  if (!lds_attr) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&scg_bwd_coef_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
      return eelg_fail(-3, "scg_bwd_coef: cannot raise the dynamic LDS limit");
    lds_attr = true;
  }
  hipLaunchKernelGGL(scg_bwd_coef_kernel, grid, dim3(SCG_T), lds, (hipStream_t)stream, *d, terms, term_out, ldc,
                     x, ldx, grad_out, ldg, n_nodes, partial);
  return eelg_check_launch("scg_bwd_coef");
}

}  // extern "C"
