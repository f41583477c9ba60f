// Crystal-graph edge convolution (CGC / mCGC benchmark models,
// scripts/benchmark_models/cgc_modified.py:11-25, cgc_vanilla.py:11-25, gnn/blocks.py:949-966):
//
//   z_e   = [x_s | x_r | f_e] @ W^T + b            (W = [W_values; W_multip], 2D outputs)
//   msg_e = softplus(z_e[:D]) * sigmoid(z_e[D:])
//   agg_n = sum_{e: recv(e) = n} msg_e  (* row_scale[n] for 'mean')
//
// The linear map is split by input block: z_e = Ps[s] + Pr[r] + Ep[e] with node-level
// projections Ps = x W_s^T, Pr = x W_r^T + b (N rows instead of E) and the edge-level
// Ep = f W_e^T; so the kernels never materialise the [E, 3D] concatenation nor the
// [E, D] messages.  Edges are receiver-sorted (rowptr = receiver CSR): one wave per
// receiver sums its in-edges in registers (no atomics).  softplus follows torch's
// default (beta 1, threshold 20).
//
// Factored edge features (EF, the model path): in both reference models the edge features are
// themselves a Linear of 5 per-edge inputs, f = e5 W5^T + b5 (cgc_modified.py:71-74), so
// Ep = f W_e^T = [e5 | 1] A with A = [W5^T W_e^T ; b5 W_e^T] ([6, 2D], formed on the host per
// layer).  With EF the kernels read the 8-float rows ef = [e5 | 1 | 0 | 0] (32 B per edge) and
// the [8, 2D] A instead of the [E, 2D] Ep (1 KiB per edge at D = 128), and form Ep in registers.
#include <hip/hip_runtime.h>

#ifndef CGC_FAST_MATH
#define CGC_FAST_MATH 1
#endif
#if CGC_FAST_MATH
// hardware exp2 / log2 / reciprocal (v_exp_f32, v_log_f32, v_rcp_f32: about 1 ulp each):
// softplus(z) = max(z, 0) + log1p(exp(-|z|)) never overflows and keeps torch's threshold.
// log1p(t) with the rounding of u = 1 + t corrected (log(u) * t / (u - 1); t itself once
// u rounds to 1), so that softplus keeps its relative accuracy for negative z, where it is
// about exp(z) (log(1 + t) alone loses ~0.3 % at z = -10 and is 0 below -16.6)
__device__ __forceinline__ float cgc_softplus(float z) {
  if (z > 20.0f) return z;
  const float t = __builtin_amdgcn_exp2f(-fabsf(z) * 1.4426950408889634f);
  const float u = 1.0f + t;
  const float lp = u == 1.0f ? t
      : __builtin_amdgcn_logf(u) * 0.6931471805599453f * t * __builtin_amdgcn_rcpf(u - 1.0f);
  return fmaxf(z, 0.0f) + lp;
}
__device__ __forceinline__ float cgc_sigmoid(float z) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(-z * 1.4426950408889634f));
}
#else
__device__ __forceinline__ float cgc_softplus(float z) { return z > 20.0f ? z : log1pf(expf(z)); }
__device__ __forceinline__ float cgc_sigmoid(float z) { return 1.0f / (1.0f + expf(-z)); }
#endif

// Block order (CGC_XCD, round 6): hardware block b runs on XCD b % 8.  With the grid padded to
// a multiple of 8, logical block (b % 8) * (gridDim.x / 8) + b / 8 hands XCD k one contiguous
// range of receivers, i.e. whole lattices in order, so a lattice's gathered Ps rows (1 KiB per
// node at D = 128, 1 MiB per 1024-node lattice) are fetched into one L2 and re-read there by
// the node's other out-edges, instead of being fetched by all eight L2s.
// Measured (r08d, cgc_modified, batch 256): cgc_fwd reads 1,328 -> 704 MB per launch and the
// streaming backward 1,433 -> 916 MB, but every CGC kernel ran ~1 % slower and the step 1.8 %
// slower (32,446 vs 33,033 graphs/s over three alternating pairs): the re-fetches it removes
// were served by the Infinity Cache, so the default keeps the round-robin order (0)
#ifndef CGC_XCD
#define CGC_XCD 0
#endif
__device__ __forceinline__ int cgc_block() {
#if CGC_XCD
  return (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
#else
  return blockIdx.x;
#endif
}
static inline unsigned cgc_grid(unsigned blocks) { return CGC_XCD ? (blocks + 7) / 8 * 8 : blocks; }

// Forward: a receiver's in-edges are taken CGC_EB at a time: their sender indices are
// wave-uniform (one scalar load batch), and every lane issues the batch's gathers of Ps[s] and
// Ep[e] before it evaluates any of them, so a receiver costs about three memory round trips
// instead of two per edge.  A lane owns channels lane + 64 k, k < CPL (CPL = ceil(D / 64)).
#ifndef CGC_EB
#define CGC_EB 4
#endif
#define CGC_EFW 8   // floats per factored edge-feature row: e5, 1, two zeros
#define CGC_EFN 6   // rows of A used
template <int CPL, bool EF>
__device__ __forceinline__ void cgc_edge_proj(const float* __restrict__ ep, const float* __restrict__ ef,
                                              const float (&av)[CGC_EFN][CPL], const float (&am)[CGC_EFN][CPL],
                                              int e, int D2, int D, int lane, float (&pv)[CPL], float (&pm)[CPL]) {
  if (EF) {
    float f[CGC_EFN];
#pragma unroll
    for (int i = 0; i < CGC_EFN; ++i) f[i] = ef[(size_t)e * CGC_EFW + i];   // wave-uniform
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      float v = 0.0f, m = 0.0f;
#pragma unroll
      for (int i = 0; i < CGC_EFN; ++i) { v = fmaf(f[i], av[i][k], v); m = fmaf(f[i], am[i][k], m); }
      pv[k] = v;
      pm[k] = m;
    }
  } else {
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int c = min(lane + 64 * k, D - 1);
      pv[k] = ep[(size_t)e * D2 + c];
      pm[k] = ep[(size_t)e * D2 + D + c];
    }
  }
}

template <int CPL, bool EF>
__device__ __forceinline__ void cgc_load_a(const float* __restrict__ ea, int D, int lane,
                                           float (&av)[CGC_EFN][CPL], float (&am)[CGC_EFN][CPL]) {
#pragma unroll
  for (int i = 0; i < CGC_EFN; ++i)
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int c = min(lane + 64 * k, D - 1);
      av[i][k] = EF ? ea[(size_t)i * 2 * D + c] : 0.0f;
      am[i][k] = EF ? ea[(size_t)i * 2 * D + D + c] : 0.0f;
    }
}

template <int CPL, bool EF>
__global__ __launch_bounds__(256) void cgc_fwd_kernel(
    const float* __restrict__ ps, const float* __restrict__ pr, const float* __restrict__ ep,
    const float* __restrict__ ef, const float* __restrict__ ea,
    const int* __restrict__ sender, const int* __restrict__ rowptr, const float* __restrict__ row_scale,
    int n_nodes, int D, float* __restrict__ agg, const float* __restrict__ res) {
  const int node = __builtin_amdgcn_readfirstlane(cgc_block() * 4 + (threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  if (node >= n_nodes) return;
  const int beg = rowptr[node], end = rowptr[node + 1];
  const int D2 = 2 * D;
  const float sc = row_scale ? row_scale[node] : 1.0f;
  const float* __restrict__ prn = pr + (size_t)node * D2;
  float rv[CPL], rm[CPL], acc[CPL];
  float av[CGC_EFN][CPL], am[CGC_EFN][CPL];
  cgc_load_a<CPL, EF>(ea, D, lane, av, am);
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int c = min(lane + 64 * k, D - 1);
    rv[k] = prn[c];
    rm[k] = prn[D + c];
    acc[k] = 0.0f;
  }
  for (int e0 = beg; e0 < end; e0 += CGC_EB) {
    int s[CGC_EB];
#pragma unroll
    for (int j = 0; j < CGC_EB; ++j) s[j] = sender[min(e0 + j, end - 1)];
    float zv[CGC_EB][CPL], zm[CGC_EB][CPL], pv[CGC_EB][CPL], pm[CGC_EB][CPL];
#pragma unroll
    for (int j = 0; j < CGC_EB; ++j) {
      const int e = min(e0 + j, end - 1);
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int c = min(lane + 64 * k, D - 1);
        zv[j][k] = ps[(size_t)s[j] * D2 + c];
        zm[j][k] = ps[(size_t)s[j] * D2 + D + c];
      }
      cgc_edge_proj<CPL, EF>(ep, ef, av, am, e, D2, D, lane, pv[j], pm[j]);
    }
#pragma unroll
    for (int j = 0; j < CGC_EB; ++j)
      if (e0 + j < end)   // uniform
#pragma unroll
        for (int k = 0; k < CPL; ++k)
          acc[k] += cgc_softplus((zv[j][k] + pv[j][k]) + rv[k]) * cgc_sigmoid((zm[j][k] + pm[j][k]) + rm[k]);
  }
  // the layer residual (h + conv(h), cgc_modified.py:77) added in the store (res may be NULL)
#pragma unroll
  for (int k = 0; k < CPL; ++k)
    if (lane + 64 * k < D) {
      const size_t o = (size_t)node * D + lane + 64 * k;
      // two roundings, as h + (sc * sum) in torch: no contraction into one fma
      agg[o] = res ? __fadd_rn(__fmul_rn(acc[k], sc), res[o]) : acc[k] * sc;
    }
}

// Backward: per receiver, recompute z_e and write dz_e = d msg / d z_e (.) g_n for every
// in-edge, and the receiver sums Gr[n] = sum_e dz_e in the same pass.  The sender sums
// Gs (for dW_s and dx) are a segmented sum of dz over the sender CSR.  Edges are taken CGC_EB
// at a time like the forward: the batch's sender indices are read together and every gather
// of Ps[s] / Ep[e] is issued before any of them is used.
template <int CPL, bool EF>
__global__ __launch_bounds__(256) void cgc_bwd_kernel(
    const float* __restrict__ ps, const float* __restrict__ pr, const float* __restrict__ ep,
    const float* __restrict__ ef, const float* __restrict__ ea, const int* __restrict__ sender, const int* __restrict__ rowptr, const float* __restrict__ row_scale,
    int n_nodes, int D, const float* __restrict__ gagg, float* __restrict__ dz, float* __restrict__ gr) {
  const int node = __builtin_amdgcn_readfirstlane(cgc_block() * 4 + (threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  if (node >= n_nodes) return;
  const int beg = rowptr[node], end = rowptr[node + 1];
  const int D2 = 2 * D;
  const float sc = row_scale ? row_scale[node] : 1.0f;
  const float* __restrict__ prn = pr + (size_t)node * D2;
  float rv[CPL], rm[CPL], g[CPL], av[CPL], am[CPL];
  float aav[CGC_EFN][CPL], aam[CGC_EFN][CPL];
  cgc_load_a<CPL, EF>(ea, D, lane, aav, aam);
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    const int c = min(lane + 64 * k, D - 1);
    rv[k] = prn[c];
    rm[k] = prn[D + c];
    g[k] = gagg[(size_t)node * D + c] * sc;
    av[k] = 0.0f;
    am[k] = 0.0f;
  }
  for (int e0 = beg; e0 < end; e0 += CGC_EB) {
    int s[CGC_EB];
#pragma unroll
    for (int j = 0; j < CGC_EB; ++j) s[j] = sender[min(e0 + j, end - 1)];
    float zv[CGC_EB][CPL], zm[CGC_EB][CPL], pv[CGC_EB][CPL], pm[CGC_EB][CPL];
#pragma unroll
    for (int j = 0; j < CGC_EB; ++j) {
      const int e = min(e0 + j, end - 1);
#pragma unroll
      for (int k = 0; k < CPL; ++k) {
        const int c = min(lane + 64 * k, D - 1);
        zv[j][k] = ps[(size_t)s[j] * D2 + c];
        zm[j][k] = ps[(size_t)s[j] * D2 + D + c];
      }
      cgc_edge_proj<CPL, EF>(ep, ef, aav, aam, e, D2, D, lane, pv[j], pm[j]);
    }
#pragma unroll
    for (int j = 0; j < CGC_EB; ++j)
      if (e0 + j < end)   // uniform
#pragma unroll
        for (int k = 0; k < CPL; ++k) {
          const float z1 = (zv[j][k] + pv[j][k]) + rv[k], z2 = (zm[j][k] + pm[j][k]) + rm[k];
          const float sv = z1 > 20.0f ? 1.0f : cgc_sigmoid(z1);   // softplus' (torch: 1 above threshold)
          const float sm = cgc_sigmoid(z2);
          const float dv = g[k] * sv * sm;
          const float dm = g[k] * cgc_softplus(z1) * sm * (1.0f - sm);
          if (lane + 64 * k < D) {
            dz[(size_t)(e0 + j) * D2 + lane + 64 * k] = dv;
            dz[(size_t)(e0 + j) * D2 + D + lane + 64 * k] = dm;
          }
          av[k] += dv;
          am[k] += dm;
        }
  }
#pragma unroll
  for (int k = 0; k < CPL; ++k)
    if (lane + 64 * k < D) {
      gr[(size_t)node * D2 + lane + 64 * k] = av[k];
      gr[(size_t)node * D2 + D + lane + 64 * k] = am[k];
    }
}

// ---------------------------------------------------------------------------------------------
// Receiver-streaming form (round 5, the models' factored-edge path): a wave owns CGC_RPW
// consecutive receivers and walks their edges (one contiguous CSR range) in batches of CGC_SB,
// the next batch's sender ids, edge-feature rows and Ps gathers in flight while the current one
// computes; the receivers' Pr rows (and grad rows in the backward) are loaded once up front.  A
// receiver's sum is flushed when the walk crosses its end (wave-uniform), receivers without
// edges get 0.  Per receiver the one-wave form paid three dependent memory round trips (row
// pointer, senders, gathers) for about four edges; here a wave pays about one per batch.
// ---------------------------------------------------------------------------------------------
#ifndef CGC_RPW
#define CGC_RPW 8
#endif
#ifndef CGC_SB
#define CGC_SB 8
#endif
static_assert(CGC_SB * CGC_EFW <= 64, "a batch's edge-feature rows are one vector load");

template <int CPL>
struct CgcBatch {
  float zv[CGC_SB][CPL], zm[CGC_SB][CPL];   // Ps[s] gathers
  float efv;                                 // lane l: ef row (l / 8) of the batch, column l % 8
  int rc[CGC_SB];                            // receivers of the batch's edges (wave-uniform)
};

template <int CPL>
__device__ __forceinline__ void cgc_batch_load(CgcBatch<CPL>& b, const float* __restrict__ ps,
                                               const float* __restrict__ ef, const int* __restrict__ sender,
                                               const int* __restrict__ receiver, int eb, int e1, int D,
                                               int lane) {
  const int D2 = 2 * D;
#pragma unroll
  for (int j = 0; j < CGC_SB; ++j) {
    const int e = min(eb + j, e1 - 1);
    const int s = sender[e];                 // wave-uniform (scalar load)
    b.rc[j] = receiver[e];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int c = min(lane + 64 * k, D - 1);
      b.zv[j][k] = ps[(size_t)s * D2 + c];
      b.zm[j][k] = ps[(size_t)s * D2 + D + c];
    }
  }
  b.efv = ef[(size_t)min(eb + (lane >> 3), e1 - 1) * CGC_EFW + (lane & 7)];
}

template <int CPL>
__device__ __forceinline__ void cgc_batch_feat(const CgcBatch<CPL>& b, int j, float (&f)[CGC_EFN]) {
#pragma unroll
  for (int i = 0; i < CGC_EFN; ++i)
    f[i] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, b.efv), j * CGC_EFW + i));
}

template <int CPL>
__device__ __forceinline__ void cgc_batch_proj(const float (&f)[CGC_EFN],
                                               const float (&av)[CGC_EFN][CPL], const float (&am)[CGC_EFN][CPL],
                                               float (&pv)[CPL], float (&pm)[CPL]) {
#pragma unroll
  for (int k = 0; k < CPL; ++k) {
    float v = 0.0f, m = 0.0f;
#pragma unroll
    for (int i = 0; i < CGC_EFN; ++i) { v = fmaf(f[i], av[i][k], v); m = fmaf(f[i], am[i][k], m); }
    pv[k] = v;
    pm[k] = m;
  }
}

template <int CPL, bool BWD>
__global__ __launch_bounds__(256) void cgc_stream_kernel(
    const float* __restrict__ ps, const float* __restrict__ pr, const float* __restrict__ ef,
    const float* __restrict__ ea, const int* __restrict__ sender, const int* __restrict__ receiver,
    const int* __restrict__ rowptr, const float* __restrict__ row_scale, int n_nodes, int D,
    float* __restrict__ agg, const float* __restrict__ gagg, float* __restrict__ dz,
    float* __restrict__ gr, float* __restrict__ dea_part) {
  const int bx = cgc_block();
  // a padding block of the XCD-ordered grid (past the last receiver group) leaves before the
  // workgroup reduction and writes no partial
  if (bx >= ((n_nodes + CGC_RPW - 1) / CGC_RPW + 3) / 4) return;
  const int wid = __builtin_amdgcn_readfirstlane(bx * 4 + (threadIdx.x >> 6));
  const int lane = threadIdx.x & 63;
  const int r0 = wid * CGC_RPW;
  // a wave past the last receiver still takes part in the workgroup's reduction of the
  // edge-factor gradient at the end (with zeros)
  const int nr = max(0, min(CGC_RPW, n_nodes - r0));
  const int D2 = 2 * D;
  const int e0 = nr > 0 ? rowptr[r0] : 0, e1 = nr > 0 ? rowptr[r0 + nr] : 0;
  float av[CGC_EFN][CPL], am[CGC_EFN][CPL];
  cgc_load_a<CPL, true>(ea, D, lane, av, am);
  // backward: d ea[i][k] = sum over the wave's edges of ef[e][i] * dz[e][k] (rows 0..5)
  float dav[CGC_EFN][CPL], dam[CGC_EFN][CPL];
#pragma unroll
  for (int i = 0; i < CGC_EFN; ++i)
#pragma unroll
    for (int q = 0; q < CPL; ++q) { dav[i][q] = 0.0f; dam[i][q] = 0.0f; }
  // the receivers' Pr rows (and grad rows, pre-scaled; the row scale in the forward), loaded once
  float rvs[CGC_RPW][CPL], rms[CGC_RPW][CPL], gs[CGC_RPW][CPL];
#pragma unroll
  for (int k = 0; k < CGC_RPW; ++k) {
    const int r = min(r0 + min(k, nr - 1), n_nodes - 1);
    const float sc = row_scale ? row_scale[r] : 1.0f;
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int c = min(lane + 64 * q, D - 1);
      rvs[k][q] = pr[(size_t)r * D2 + c];
      rms[k][q] = pr[(size_t)r * D2 + D + c];
      gs[k][q] = BWD ? gagg[(size_t)r * D + c] * sc : sc;
    }
  }
  int cur = 0;                                   // receiver being summed (relative to r0)
  float a1[CPL], a2[CPL];                        // fwd: message sum; bwd: sums of dz (v, m)
  float rvc[CPL], rmc[CPL], gc[CPL];             // the current receiver's rows
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    a1[q] = 0.0f; a2[q] = 0.0f;
    rvc[q] = rvs[0][q]; rmc[q] = rms[0][q]; gc[q] = gs[0][q];
  }
#define CGC_FLUSH_AND_NEXT()                                                                    \
  {                                                                                             \
    if (cur < nr) {                                                                             \
      _Pragma("unroll") for (int q = 0; q < CPL; ++q) if (lane + 64 * q < D) {                  \
        if (BWD) {                                                                              \
          gr[(size_t)(r0 + cur) * D2 + lane + 64 * q] = a1[q];                                  \
          gr[(size_t)(r0 + cur) * D2 + D + lane + 64 * q] = a2[q];                              \
        } else {                                                                                \
          agg[(size_t)(r0 + cur) * D + lane + 64 * q] = a1[q] * gc[q];                          \
        }                                                                                       \
      }                                                                                         \
    }                                                                                           \
    ++cur;                                                                                      \
    _Pragma("unroll") for (int q = 0; q < CPL; ++q) {                                           \
      a1[q] = 0.0f; a2[q] = 0.0f;                                                               \
      _Pragma("unroll") for (int kk = 1; kk < CGC_RPW; ++kk) if (cur == kk) {                   \
        rvc[q] = rvs[kk][q]; rmc[q] = rms[kk][q]; gc[q] = gs[kk][q];                            \
      }                                                                                         \
    }                                                                                           \
  }
#define CGC_PROCESS(B, EB)                                                                      \
  _Pragma("unroll") for (int j = 0; j < CGC_SB; ++j) {                                          \
    const int e = (EB) + j;                                                                     \
    if (e < e1) {                                                                               \
      const int k = B.rc[j] - r0;                                                               \
      while (cur < k) CGC_FLUSH_AND_NEXT();                                                     \
      float pv[CPL], pm[CPL], f_[CGC_EFN];                                                      \
      cgc_batch_feat<CPL>(B, j, f_);                                                            \
      cgc_batch_proj<CPL>(f_, av, am, pv, pm);                                                  \
      _Pragma("unroll") for (int q = 0; q < CPL; ++q) {                                         \
        const float z1 = (B.zv[j][q] + pv[q]) + rvc[q];                                         \
        const float z2 = (B.zm[j][q] + pm[q]) + rmc[q];                                         \
        if (!BWD) {                                                                             \
          a1[q] += cgc_softplus(z1) * cgc_sigmoid(z2);                                          \
        } else {                                                                                \
          const float sv = z1 > 20.0f ? 1.0f : cgc_sigmoid(z1);                                 \
          const float sm = cgc_sigmoid(z2);                                                     \
          const float dv = gc[q] * sv * sm;                                                     \
          const float dm = gc[q] * cgc_softplus(z1) * sm * (1.0f - sm);                         \
          if (lane + 64 * q < D) {                                                              \
            dz[(size_t)e * D2 + lane + 64 * q] = dv;                                            \
            dz[(size_t)e * D2 + D + lane + 64 * q] = dm;                                        \
          }                                                                                     \
          a1[q] += dv;                                                                          \
          a2[q] += dm;                                                                          \
          _Pragma("unroll") for (int i = 0; i < CGC_EFN; ++i) {                                 \
            dav[i][q] = fmaf(f_[i], dv, dav[i][q]);                                             \
            dam[i][q] = fmaf(f_[i], dm, dam[i][q]);                                             \
          }                                                                                     \
        }                                                                                       \
      }                                                                                         \
    }                                                                                           \
  }
  // two batch buffers, named (not indexed by a runtime slot: that would live in scratch)
  CgcBatch<CPL> b0, b1;
  if (e0 < e1) cgc_batch_load<CPL>(b0, ps, ef, sender, receiver, e0, e1, D, lane);
  for (int eb = e0; eb < e1; eb += 2 * CGC_SB) {
    if (eb + CGC_SB < e1) cgc_batch_load<CPL>(b1, ps, ef, sender, receiver, eb + CGC_SB, e1, D, lane);
    CGC_PROCESS(b0, eb);
    if (eb + CGC_SB >= e1) break;
    if (eb + 2 * CGC_SB < e1) cgc_batch_load<CPL>(b0, ps, ef, sender, receiver, eb + 2 * CGC_SB, e1, D, lane);
    CGC_PROCESS(b1, eb + CGC_SB);
  }
  // the last receiver with edges and every trailing receiver without
  while (cur < CGC_RPW) CGC_FLUSH_AND_NEXT();
#undef CGC_PROCESS
#undef CGC_FLUSH_AND_NEXT
  if (BWD && dea_part) {
    // the workgroup's partial of d ea: the 4 waves' sums added through LDS in wave order
    __shared__ float red[4 * CGC_EFN * 2 * 64 * CPL];
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < CGC_EFN; ++i)
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        red[((w * CGC_EFN + i) * 2 + 0) * 64 * CPL + q * 64 + lane] = dav[i][q];
        red[((w * CGC_EFN + i) * 2 + 1) * 64 * CPL + q * 64 + lane] = dam[i][q];
      }
    __syncthreads();
    float* __restrict__ dst = dea_part + (size_t)bx * CGC_EFN * D2;
    for (int t = threadIdx.x; t < CGC_EFN * 2 * 64 * CPL; t += 256) {
      const int i = t / (2 * 64 * CPL), rem = t - i * 2 * 64 * CPL;
      const int half = rem / (64 * CPL), c = rem - half * 64 * CPL;   // c = q * 64 + lane
      float v = 0.0f;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) v += red[((ww * CGC_EFN + i) * 2 + half) * 64 * CPL + c];
      const int ch = (c & 63) + 64 * (c >> 6);                         // channel lane + 64 q
      if (ch < D) dst[i * D2 + half * D + ch] = v;
    }
  }
}
