// Radial MLP of the interaction block (gnn/blocks.py:537-549, applied at :590):
//   z_0 = feats W_0^T + b_0,  h_1 = SiLU(z_0), ...,  z_n = h_n W_n^T + b_n,  h_{n+1} = SiLU(z_n),
//   w = h_NH W_o^T              (no bias on the output layer; W_o: [n_out, hidden])
// with w[E, n_out] the per-edge tensor-product weights (n_out = 1344 for the l>=1 layers of
// BASELINE config 2).  The reference runs this as torch.nn.Sequential of Linear + SiLU.
//
// Every GEMM here is on v_mfma_f32_32x32x2_f32 (exact f32 products, fmaf-chain numerics).
// Fragment convention (32x32x2): lane l = 32*hf + i supplies A[row i][k] and B[k][col i] for
// the step's k; the two lane halves take k = hf*KH + st over a K block of 2*KH, i.e. the K
// order is permuted (a sum, so any bijection shared by A and B is exact up to rounding
// order).  C/D: acc[r] is row (r&3) + 8*(r>>2) + 4*hf, column i.
//
// Masked accesses are branch-free: loads of small operands read a clamped valid element and
// select 0; the large streams go through buffer descriptors whose range check turns an
// out-of-range offset (past the end, or RAD_OOB for a masked lane) into a zero load / a
// dropped store.
//
// Forward (radial_fwd): one wave owns 32 edges end to end; the output layer's W_o tiles are
// shared by the workgroup's 4 waves through LDS.  Hidden activations stay in a
// wave-private LDS tile; only the pre-activations z_n (the backward's operand,
// [NH, E, H]) and w reach HBM.
// Backward (deterministic: per-wave / per-split partials, summed by the caller in a fixed
// order):
//   radial_bwd_gh   : grad_h = grad_w W_o  [E, H]  (the one long-K GEMM; W_o chunks staged in
//                     LDS and shared by the workgroup's 4 waves, grad_w rows prefetched)
//   radial_bwd_small: back through SiLU' and the hidden layers; weight / bias gradients
//                     accumulated in registers across the wave's edge tiles
//   radial_bwd_wo   : grad W_o = grad_w^T h_NH per (128-column block, edge split),
//                     h_NH = SiLU(z) staged once per workgroup in LDS for its 4 waves
#include <hip/hip_runtime.h>
#include <cstdlib>
#include <stdint.h>

#include "../../include/eelg.h"
#include "eelg_internal.h"

typedef float rad_f32x16 __attribute__((ext_vector_type(16)));
typedef __amdgpu_buffer_rsrc_t rad_rsrc_t;

#define RAD_MFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x2f32((a), (b), (c), 0, 0, 0)

__device__ __forceinline__ rad_rsrc_t rad_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ float rad_bld(rad_rsrc_t r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, (int)off, 0, 0));
}
__device__ __forceinline__ void rad_bst(rad_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, (int)off, 0, 0);
}
__device__ __forceinline__ void rad_bst16(rad_rsrc_t r, uint32_t off, unsigned short v) {
  __builtin_amdgcn_raw_buffer_store_b16(v, r, (int)off, 0, 0);
}
// a masked lane's offset gets bit 31 (past every buffer): arithmetic, so the compiler keeps
// one unconditional buffer access instead of branching around two
__device__ __forceinline__ uint32_t rad_off(uint32_t off, bool ok) {
  return off | ((uint32_t)(!ok) << 31);
}
// clamped load + select: no branch around the load
__device__ __forceinline__ float rad_ld(const float* __restrict__ p, size_t idx, bool ok) {
  const float v = p[ok ? idx : 0];
  return ok ? v : 0.0f;
}

// fast exp / reciprocal (a few ulp; the parity bound is 1e-5 of max)
__device__ __forceinline__ float rad_sigmoid(float z) { return __builtin_amdgcn_rcpf(1.0f + __expf(-z)); }
__device__ __forceinline__ float rad_silu(float z) { return z * rad_sigmoid(z); }
// torch silu_backward: g * s * (1 + z * (1 - s)), s = sigmoid(z)
__device__ __forceinline__ float rad_silu_grad(float z, float g) {
  const float s = rad_sigmoid(z);
  return g * s * (1.0f + z * (1.0f - s));
}
__device__ __forceinline__ int rad_row(int r, int hf) { return (r & 3) + 8 * (r >> 2) + 4 * hf; }

// ---------------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------------
#ifndef RAD_FWD_RT
#define RAD_FWD_RT 1   // 32-edge row tiles per wave (each W_o fragment read from LDS feeds RT MFMAs)
#endif
template <int H, int NH, bool BF>
__global__ __launch_bounds__(256) void radial_fwd_kernel(const float* __restrict__ feats,
                                                         int n_edges, eelg_radial_desc d,
                                                         const float* __restrict__ woT,
                                                         float* __restrict__ zsave,
                                                         void* __restrict__ out) {
  constexpr int HS = H + 1, NT = H / 32, KH = H / 2, ES = BF ? 2 : 4, RT = RAD_FWD_RT;
  __shared__ float hb[4 * RT * 32 * HS];
  __shared__ float bt[2][H * 32];   // W_o^T column tile [k][j], double-buffered, shared by 4 waves
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 31, hf = l >> 5;
  const int e00 = (blockIdx.x * 4 + wave) * 32 * RT;
  const int F = d.n_feat, W = d.n_out;
  const uint32_t E = (uint32_t)n_edges;
  const rad_rsrc_t rz = rad_rsrc(zsave, (uint32_t)NH * E * H * 4u);
  const rad_rsrc_t ro = rad_rsrc(out, E * (uint32_t)W * ES);
  const int KF = (F + 1) >> 1;  // layer 0: K = F (<= 32) split over the two lane halves
#pragma unroll 1
  for (int rt = 0; rt < RT; ++rt) {
  const int e0 = e00 + 32 * rt;
  // waves / tiles past the last edge skip the hidden layers but join the output layer's
  // barriers (their stores fall outside the buffer range)
  const bool active = e0 < n_edges;
  float* __restrict__ hw = hb + (wave * RT + rt) * 32 * HS;
  const bool rok = e0 + i < n_edges;

  float a[KH];
#pragma unroll
  for (int st = 0; st < 16; ++st) {
    const int k = hf * KF + st;
    a[st] = rad_ld(feats, (size_t)(e0 + i) * F + k, rok && st < KF && k < F);
  }
#pragma unroll
  for (int n = 0; n < NH; ++n) {
    if (!active) break;   // wave-uniform
    const float* __restrict__ wn = d.w[n];
    const float* __restrict__ bn = d.b[n];
    const int din = n == 0 ? F : H;
    const int kh = n == 0 ? KF : KH;
    if (n > 0) {
#pragma unroll
      for (int st = 0; st < KH; ++st) a[st] = hw[i * HS + hf * KH + st];
    }
    rad_f32x16 acc[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct) {
      const float bj = bn[ct * 32 + i];
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[ct][r] = bj;
#pragma unroll
      for (int st = 0; st < KH; ++st) {
        if (st < kh) {   // wave-uniform
          const int k = hf * kh + st;
          acc[ct] = RAD_MFMA(a[st], rad_ld(wn, (size_t)(ct * 32 + i) * din + k, k < din), acc[ct]);
        }
      }
    }
    // epilogue: z_n to HBM (backward operand), SiLU(z_n) into the wave's LDS tile.  All of
    // this layer's A reads of the tile were issued above (in-order LDS within the wave).
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = rad_row(r, hf), col = ct * 32 + i;
        const float z = acc[ct][r];
        // rows >= E must be masked: past the end of z_n lies z_{n+1}
        rad_bst(rz, rad_off((((uint32_t)n * E + e0 + row) * H + col) * 4u, e0 + row < n_edges), z);
        hw[row * HS + col] = rad_silu(z);
      }
  }
  }
  // output layer: w[e0 + row, ct*32 + i], B[k][j] = W_o[j][k] = woT[k][j].  Each 32-column
  // tile of W_o^T (H x 32 floats) is loaded once per workgroup (coalesced rows, the next tile in
  // registers while the current one computes) and read by the 4 waves from LDS: one L2 read
  // of W_o per 128 edges instead of per 32.
  float ar[RT][KH];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int st = 0; st < KH; ++st) ar[rt][st] = hb[(wave * RT + rt) * 32 * HS + i * HS + hf * KH + st];
  const int nct = (W + 31) >> 5;
  constexpr int BPT = H * 32 / 256;   // tile floats per thread
  float rb[BPT];
  auto load_b = [&](int ct) {
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
      const int e = threadIdx.x + 256 * q, k = e >> 5, col = ct * 32 + (e & 31);
      rb[q] = rad_ld(woT, (size_t)k * W + col, col < W);
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int q = 0; q < BPT; ++q) bt[buf][threadIdx.x + 256 * q] = rb[q];
  };
  load_b(0);
  store_b(0);
  __syncthreads();
  for (int ct = 0; ct < nct; ++ct) {
    if (ct + 1 < nct) load_b(ct + 1);
    const float* __restrict__ bb = bt[ct & 1] + hf * KH * 32 + i;
    rad_f32x16 acc[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[rt][r] = 0.0f;
#pragma unroll
    for (int st = 0; st < KH; ++st) {
      const float bv = bb[st * 32];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) acc[rt] = RAD_MFMA(ar[rt][st], bv, acc[rt]);
    }
    const int col = ct * 32 + i;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint32_t off =
            rad_off(((uint32_t)(e00 + 32 * rt + rad_row(r, hf)) * W + col) * ES, col < W);
        if (BF)
          rad_bst16(ro, off, eelg_f2bf(acc[rt][r]));
        else
          rad_bst(ro, off, acc[rt][r]);
      }
    if (ct + 1 < nct) store_b((ct + 1) & 1);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// backward 1: grad_h[E, H] = grad_w[E, W] W_o[W, H]
// ---------------------------------------------------------------------------------------------
// grad_w rows are read coalesced (4 or 8 rows x 256 B per wave-instruction) and turned into
// the row-per-lane A layout through a wave-private LDS tile; W_o chunks are staged in LDS once
// per workgroup and shared by its 4 waves.
template <int H, bool BF>
__global__ __launch_bounds__(256) void radial_bwd_gh_kernel(const void* __restrict__ gw,
                                                            int n_edges, int W,
                                                            const float* __restrict__ wo,
                                                            float* __restrict__ gh) {
  constexpr int NT = H / 32, KC = 64, ES = BF ? 2 : 4, NB = KC * H / 256;  // B floats per thread
  constexpr int AS = KC + 4;                  // A tile row stride (floats)
  constexpr int NV = BF ? 4 : 8;              // 16-B loads per lane per chunk
  __shared__ float bs[2][KC * H];
  __shared__ float as_[4][32 * AS];
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 31, hf = l >> 5;
  const int e0 = (blockIdx.x * 4 + wave) * 32;   // waves past the last edge still stage / sync
  const uint32_t E = (uint32_t)n_edges;
  const rad_rsrc_t rg = rad_rsrc(gw, E * (uint32_t)W * ES);
  const rad_rsrc_t rw = rad_rsrc(wo, (uint32_t)W * H * 4u);
  const rad_rsrc_t rh = rad_rsrc(gh, E * (uint32_t)H * 4u);
  const int nchunk = (W + KC - 1) / KC;
  const bool vec = (W % (BF ? 8 : 4)) == 0;      // 16-B pieces never straddle a row end
  float* __restrict__ at = as_[wave];

  // raw chunk loads, row-coalesced: fp32 piece q = rows 4q + (l >> 4), columns 4 (l & 15) ..+3;
  // bf16 piece q = rows 8q + (l >> 3), columns 8 (l & 7) ..+7.  Rows past E read zeros.
  uint4 raw[NV];
  auto load_a = [&](int kc) {
    if (vec) {
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const int row = BF ? 8 * q + (l >> 3) : 4 * q + (l >> 4);
        const int col = kc + (BF ? 8 * (l & 7) : 4 * (l & 15));
        const uint32_t off = rad_off(((uint32_t)(e0 + row) * W + col) * ES, col < W);
        raw[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rg, (int)off, 0, 0));
      }
    }
  };
  // raw -> LDS tile at[row][k - kc]; the scalar path loads straight into the tile
  auto stage_a = [&](int kc) {
    if (vec) {
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        if (BF) {
          const int row = 8 * q + (l >> 3), c = 8 * (l & 7);
          const uint32_t w4[4] = {raw[q].x, raw[q].y, raw[q].z, raw[q].w};
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            at[row * AS + c + 2 * u] = __uint_as_float(w4[u] << 16);
            at[row * AS + c + 2 * u + 1] = __uint_as_float(w4[u] & 0xffff0000u);
          }
        } else {
          const int row = 4 * q + (l >> 4), c = 4 * (l & 15);
          *reinterpret_cast<uint4*>(&at[row * AS + c]) = raw[q];
        }
      }
    } else {
#pragma unroll 4
      for (int q = 0; q < 32; ++q) {
        const int idx = l + 64 * q, row = idx >> 6, c = idx & 63;
        const uint32_t off = rad_off(((uint32_t)(e0 + row) * W + kc + c) * ES, kc + c < W);
        at[row * AS + c] = BF ? eelg_bf2f((unsigned short)__builtin_amdgcn_raw_buffer_load_b16(rg, (int)off, 0, 0))
                              : rad_bld(rg, off);
      }
    }
  };
  // B: W_o rows [kc, kc + 64) are one contiguous run of 64 * H floats
  float rb[NB];
  auto load_b = [&](int kc) {
#pragma unroll
    for (int q = 0; q < NB; ++q) rb[q] = rad_bld(rw, ((uint32_t)kc * H + threadIdx.x + 256 * q) * 4u);
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int q = 0; q < NB; ++q) bs[buf][threadIdx.x + 256 * q] = rb[q];
  };

  rad_f32x16 acc[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[ct][r] = 0.0f;
  load_b(0);
  store_b(0);
  load_a(0);
  for (int c = 0; c < nchunk; ++c) {
    __syncthreads();   // chunk c staged; every wave is past chunk c-1's reads of bs[(c+1)&1]
    // A fragments of chunk c: lane (hf, i) takes row i, k = 32 hf + st
    stage_a(c * KC);
    float a[32];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 v = *reinterpret_cast<const float4*>(&at[i * AS + hf * 32 + 4 * q]);
      a[4 * q] = v.x; a[4 * q + 1] = v.y; a[4 * q + 2] = v.z; a[4 * q + 3] = v.w;
    }
    if (c + 1 < nchunk) {   // uniform; in flight during the MFMAs
      load_b((c + 1) * KC);
      load_a((c + 1) * KC);
    }
    const float* __restrict__ b = bs[c & 1];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
      for (int st = 0; st < 32; ++st)
        acc[ct] = RAD_MFMA(a[st], b[(hf * 32 + st) * H + ct * 32 + i], acc[ct]);
    if (c + 1 < nchunk) store_b((c + 1) & 1);
  }
#pragma unroll
  for (int ct = 0; ct < NT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      rad_bst(rh, ((uint32_t)(e0 + rad_row(r, hf)) * H + ct * 32 + i) * 4u, acc[ct][r]);
}

// ---------------------------------------------------------------------------------------------
// backward 2: through SiLU' and the hidden layers
// ---------------------------------------------------------------------------------------------
// A workgroup takes 128-edge tiles.  Per layer (last first) each wave turns its 32 edges'
// grad_h into gz = grad_h * SiLU'(z_n) and stages gz and the layer input h_n in LDS; after a
// barrier the 4 waves split the weight gradient sum_e gz[e]^T h_n[e] (K = 128 edges) into
// 32x32 quadrants that stay in registers across the workgroup's tiles, and threads < H sum
// the bias gradient.  grad_h of the layer below is gz W_n, per wave on its own rows.
// part[block, :] = this workgroup's partial of [grad W_0 (H x F), grad b_0 (H),
//                                              grad W_1 (H x H), grad b_1, ...] (torch layout)
#ifndef RAD_SMALL_WPE
#define RAD_SMALL_WPE 2   // 2 waves/SIMD with a few spilled registers: 0.70 vs 0.90 ms for the whole backward
#endif
template <int H, int NH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RAD_SMALL_WPE))) void radial_bwd_small_kernel(const float* __restrict__ ghin,
                                                               int n_edges, eelg_radial_desc d,
                                                               const float* __restrict__ zsave,
                                                               const float* __restrict__ feats,
                                                               float* __restrict__ part) {
  constexpr int HS = H + 1, NT = H / 32, KH = H / 2, TE = 128, NHM = NH > 1 ? NH - 1 : 1;
  constexpr int NQ = NT * NT;   // 32x32 quadrants of a hidden [H, H] weight (4 or 1)
  __shared__ float G[TE * HS];  // gz_n of the tile
  __shared__ float X[TE * HS];  // h_n (the layer's input) of the tile
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 31, hf = l >> 5;
  const int F = d.n_feat;
  const size_t E = (size_t)n_edges;
  const int ntile = (n_edges + TE - 1) / TE;
  const bool has_q = wave < NQ;          // owns hidden-layer quadrant `wave`
  const bool has_q0 = wave < NT;         // owns layer-0 quadrant (rows wave*32.., cols 0..31)
  const int qj = (wave / NT) * 32, qk = (wave % NT) * 32;

  rad_f32x16 accH[NHM], acc0;
  float bacc[NH];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    acc0[r] = 0.0f;
#pragma unroll
    for (int n = 0; n < NHM; ++n) accH[n][r] = 0.0f;
  }
#pragma unroll
  for (int n = 0; n < NH; ++n) bacc[n] = 0.0f;

  for (int t = blockIdx.x; t < ntile; t += gridDim.x) {
    const int e0 = t * TE + wave * 32;   // this wave's 32 edges
    const int lr0 = wave * 32;           // and their LDS rows
    rad_f32x16 gh[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = e0 + rad_row(r, hf);
        gh[ct][r] = rad_ld(ghin, (size_t)row * H + ct * 32 + i, row < n_edges);
      }
#pragma unroll
    for (int n = NH - 1; n >= 0; --n) {
      // gz at the accumulator positions -> G
#pragma unroll
      for (int ct = 0; ct < NT; ++ct)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = rad_row(r, hf), col = ct * 32 + i;
          const float z = rad_ld(zsave, ((size_t)n * E + e0 + row) * H + col, e0 + row < n_edges);
          G[(lr0 + row) * HS + col] = rad_silu_grad(z, gh[ct][r]);
        }
      // the layer input h_n -> X (coalesced rows; zeros past the last edge / the features)
      if (n == 0) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int idx = l + 64 * q, row = idx >> 5, k = idx & 31;
          X[(lr0 + row) * HS + k] =
              rad_ld(feats, (size_t)(e0 + row) * F + k, k < F && e0 + row < n_edges);
        }
      } else {
#pragma unroll
        for (int q = 0; q < H / 2; ++q) {
          const int idx = l + 64 * q, row = idx / H, k = idx % H;
          X[(lr0 + row) * HS + k] =
              rad_silu(rad_ld(zsave, ((size_t)(n - 1) * E + e0 + row) * H + k, e0 + row < n_edges));
        }
        // grad of h_n for this wave's rows: gh[e][k] = sum_j gz[e][j] W_n[j][k]
        const float* __restrict__ wn = d.w[n];
        float a3[KH];
#pragma unroll
        for (int st = 0; st < KH; ++st) a3[st] = G[(lr0 + i) * HS + hf * KH + st];
#pragma unroll
        for (int c2 = 0; c2 < NT; ++c2) {
#pragma unroll
          for (int r = 0; r < 16; ++r) gh[c2][r] = 0.0f;
#pragma unroll
          for (int st = 0; st < KH; ++st)
            gh[c2] = RAD_MFMA(a3[st], wn[(size_t)(hf * KH + st) * H + c2 * 32 + i], gh[c2]);
        }
      }
      __syncthreads();   // G, X hold the whole tile
      // weight gradient quadrant: A[j][e] = G[e][j], B[e][k] = X[e][k], K = 128 edges
      if (n > 0 ? has_q : has_q0) {
        const int jb = n > 0 ? qj : wave * 32, kb = n > 0 ? qk : 0;
        rad_f32x16 acc = n > 0 ? accH[n > 0 ? n - 1 : 0] : acc0;
#pragma unroll 16
        for (int st = 0; st < 64; ++st) {
          const int e = hf * 64 + st;
          acc = RAD_MFMA(G[e * HS + jb + i], X[e * HS + kb + i], acc);
        }
        if (n > 0) accH[n > 0 ? n - 1 : 0] = acc; else acc0 = acc;
      }
      if (threadIdx.x < H) {
        float sb = 0.0f;
#pragma unroll 8
        for (int e = 0; e < TE; ++e) sb += G[e * HS + threadIdx.x];
        bacc[n] += sb;
      }
      __syncthreads();   // before the next layer / tile rewrites G and X
    }
  }
  float* __restrict__ dst = part + (size_t)blockIdx.x * (size_t)((H * F + H) + (NH - 1) * (H * H + H));
  size_t off = 0;
#pragma unroll
  for (int n = 0; n < NH; ++n) {
    const int din = n == 0 ? F : H;
    if (n == 0) {
      if (has_q0)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (i < F) dst[(size_t)(wave * 32 + rad_row(r, hf)) * F + i] = acc0[r];
    } else if (has_q) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        dst[off + (size_t)(qj + rad_row(r, hf)) * H + qk + i] = accH[n > 0 ? n - 1 : 0][r];
    }
    off += (size_t)H * din;
    if (threadIdx.x < H) dst[off + threadIdx.x] = bacc[n];
    off += H;
  }
}

// ---------------------------------------------------------------------------------------------
// backward 3: grad of the output weight
// ---------------------------------------------------------------------------------------------
// part[s, j, k] = sum over split s's edges of grad_w[e, j] * SiLU(z_last[e, k])
template <int H, int NH, bool BF>
__global__ __launch_bounds__(256) void radial_bwd_wo_kernel(const void* __restrict__ gw,
                                                            int n_edges, int W,
                                                            const float* __restrict__ zsave,
                                                            int tiles_per_split,
                                                            float* __restrict__ part) {
  constexpr int HS = H + 1, NT = H / 32, ES = BF ? 2 : 4, NZ = 32 * H / 256;
  __shared__ float hs[2][32 * HS];
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 31, hf = l >> 5;
  const int j = blockIdx.x * 128 + wave * 32 + i;   // this lane's grad_w column (A row)
  const int s = blockIdx.y;
  const int ntile = (n_edges + 31) >> 5;
  const int t0 = s * tiles_per_split, t1 = min(ntile, t0 + tiles_per_split);
  const uint32_t E = (uint32_t)n_edges;
  const rad_rsrc_t rg = rad_rsrc(gw, E * (uint32_t)W * ES);
  const rad_rsrc_t rz = rad_rsrc(zsave + (size_t)(NH - 1) * E * H, E * (uint32_t)H * 4u);
  rad_f32x16 acc[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[ct][r] = 0.0f;
  float an[16], zn[NZ];
  auto load = [&](int t) {
    // A[j][e] = grad_w[e][j] (32 consecutive columns per lane half); rows past E read zeros
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const uint32_t off = rad_off(((uint32_t)(t * 32 + hf * 16 + st) * W + j) * ES, j < W);
      if (BF)
        an[st] = eelg_bf2f((unsigned short)__builtin_amdgcn_raw_buffer_load_b16(rg, (int)off, 0, 0));
      else
        an[st] = rad_bld(rg, off);
    }
    // z_last of the tile's 32 edges: one contiguous run of 32 * H floats
#pragma unroll
    for (int q = 0; q < NZ; ++q) zn[q] = rad_bld(rz, ((uint32_t)t * 32 * H + threadIdx.x + 256 * q) * 4u);
  };
  if (t0 < t1) load(t0);
  for (int t = t0; t < t1; ++t) {
    // h_last = SiLU(z_last), staged once for the 4 waves.  Double buffered: the barrier of
    // tile t+1 separates tile t's reads of a buffer from its rewrite at tile t+2.
    float* __restrict__ hb = hs[t & 1];
#pragma unroll
    for (int q = 0; q < NZ; ++q) {
      const int idx = threadIdx.x + 256 * q;
      const int r = idx / H, c = idx - r * H;
      hb[r * HS + c] = rad_silu(zn[q]);   // SiLU(0) = 0 past the last edge
    }
    __syncthreads();
    float a[16];
#pragma unroll
    for (int st = 0; st < 16; ++st) a[st] = an[st];
    if (t + 1 < t1) load(t + 1);   // in flight during the MFMAs
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
      for (int st = 0; st < 16; ++st)
        acc[ct] = RAD_MFMA(a[st], hb[(hf * 16 + st) * HS + ct * 32 + i], acc[ct]);
  }
  const int jb = blockIdx.x * 128 + wave * 32;
#pragma unroll
  for (int ct = 0; ct < NT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jj = jb + rad_row(r, hf);
      if (jj < W) part[((size_t)s * W + jj) * H + ct * 32 + i] = acc[ct][r];
    }
}

// ---------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------
static int radial_check(const eelg_radial_desc* d, int n_edges, int out_es) {
  if (!d) return eelg_fail(-2, "radial: null descriptor");
  if (d->hidden != 32 && d->hidden != 64)
    return eelg_fail(-2, "radial: hidden width %d not built (32 or 64)", d->hidden);
  if (d->n_hidden < 1 || d->n_hidden > EELG_RADIAL_MAXH)
    return eelg_fail(-2, "radial: %d hidden layers not built (1..%d)", d->n_hidden, EELG_RADIAL_MAXH);
  if (d->n_feat < 1 || d->n_feat > 32)
    return eelg_fail(-2, "radial: %d input features not built (1..32)", d->n_feat);
  if (d->n_out < 1) return eelg_fail(-2, "radial: n_out must be positive");
  if (n_edges < 0) return eelg_fail(-2, "radial: negative edge count");
  // buffer descriptors address each stream with 32-bit byte offsets (< 2 GiB)
  const long long e = n_edges;
  // (out_es: bytes per output element, 4 fp32 / 2 bf16; the host splits larger edge sets)
  if (e * d->n_out * out_es >= (1LL << 31) || e * d->hidden * d->n_hidden * 4 >= (1LL << 31))
    return eelg_fail(-2, "radial: %d edges x %d outputs exceed the 2 GiB per-stream limit; "
                         "split the edge set", n_edges, d->n_out);
  return 0;
}

#define RAD_LAUNCH3(KERNEL, GRID, ...)                                                          \
  do {                                                                                          \
    const int h_ = d->hidden, nh_ = d->n_hidden;                                                \
    if (h_ == 64 && nh_ == 1) { if (bf) hipLaunchKernelGGL((KERNEL<64, 1, true>), GRID, dim3(256), 0, st, __VA_ARGS__); else hipLaunchKernelGGL((KERNEL<64, 1, false>), GRID, dim3(256), 0, st, __VA_ARGS__); } \
    else if (h_ == 64 && nh_ == 2) { if (bf) hipLaunchKernelGGL((KERNEL<64, 2, true>), GRID, dim3(256), 0, st, __VA_ARGS__); else hipLaunchKernelGGL((KERNEL<64, 2, false>), GRID, dim3(256), 0, st, __VA_ARGS__); } \
    else if (h_ == 64 && nh_ == 3) { if (bf) hipLaunchKernelGGL((KERNEL<64, 3, true>), GRID, dim3(256), 0, st, __VA_ARGS__); else hipLaunchKernelGGL((KERNEL<64, 3, false>), GRID, dim3(256), 0, st, __VA_ARGS__); } \
    else if (h_ == 32 && nh_ == 1) { if (bf) hipLaunchKernelGGL((KERNEL<32, 1, true>), GRID, dim3(256), 0, st, __VA_ARGS__); else hipLaunchKernelGGL((KERNEL<32, 1, false>), GRID, dim3(256), 0, st, __VA_ARGS__); } \
    else if (h_ == 32 && nh_ == 2) { if (bf) hipLaunchKernelGGL((KERNEL<32, 2, true>), GRID, dim3(256), 0, st, __VA_ARGS__); else hipLaunchKernelGGL((KERNEL<32, 2, false>), GRID, dim3(256), 0, st, __VA_ARGS__); } \
    else { if (bf) hipLaunchKernelGGL((KERNEL<32, 3, true>), GRID, dim3(256), 0, st, __VA_ARGS__); else hipLaunchKernelGGL((KERNEL<32, 3, false>), GRID, dim3(256), 0, st, __VA_ARGS__); } \
  } while (0)

#ifndef RAD_WO_WG
#define RAD_WO_WG 1024
#endif
// EELG_RAD_WO_WG overrides the target workgroup count of radial_bwd_wo (each edge split leaves
// one [W, H] partial that the host sums)
static int rad_wo_wg() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("EELG_RAD_WO_WG");
    v = e ? atoi(e) : RAD_WO_WG;
    if (v < 1) v = RAD_WO_WG;
  }
  return v;
}

// launch plan shared by the host (partial-buffer sizes) and the launches below
static void radial_plan(int n_edges, int n_out, int* n_part, int* n_split, int* tiles_per_split) {
  const int ntile = (n_edges + 31) / 32;
  int wg = (n_edges + 127) / 128;   // radial_bwd_small: 128-edge tiles, partials per workgroup
  if (wg > 512) wg = 512;
  if (wg < 1) wg = 1;
  *n_part = wg;
  const int ncb = (n_out + 127) / 128;
  const int wo_wg = rad_wo_wg();
  int s = (wo_wg + ncb - 1) / ncb;  // ~RAD_WO_WG workgroups for the output-weight gradient
  if (s > ntile) s = ntile;
  if (s < 1) s = 1;
  const int tps = (ntile + s - 1) / s;
  *tiles_per_split = tps < 1 ? 1 : tps;
  *n_split = ntile > 0 ? (ntile + *tiles_per_split - 1) / *tiles_per_split : 1;
}

extern "C" {

int eelg_radial_plan(int n_edges, int n_out, int* n_part, int* n_split) {
  int tps;
  if (n_edges < 0 || n_out < 1) return eelg_fail(-2, "radial_plan: bad sizes");
  radial_plan(n_edges, n_out, n_part, n_split, &tps);
  return 0;
}

int eelg_radial_fwd(const float* feats, int n_edges, const eelg_radial_desc* d, const float* wo_t,
                    int out_bf16, float* zsave, void* out, void* stream) {
  if (int rc = radial_check(d, n_edges, out_bf16 ? 2 : 4)) return rc;
  if (n_edges == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const bool bf = out_bf16 != 0;
  const dim3 grid((n_edges + 128 * RAD_FWD_RT - 1) / (128 * RAD_FWD_RT));
  RAD_LAUNCH3(radial_fwd_kernel, grid, feats, n_edges, *d, wo_t, zsave, out);
  return eelg_check_launch("radial_fwd");
}

int eelg_radial_bwd(const void* grad_w, int grad_bf16, int n_edges, const eelg_radial_desc* d,
                    const float* wo, const float* zsave, const float* feats, float* grad_h,
                    float* part_h, float* part_wo, void* stream) {
  if (int rc = radial_check(d, n_edges, grad_bf16 ? 2 : 4)) return rc;
  if (n_edges == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const bool bf = grad_bf16 != 0;
  int nw, ns, tps;
  radial_plan(n_edges, d->n_out, &nw, &ns, &tps);
  const dim3 g1((n_edges + 127) / 128);
  const int W = d->n_out;
  if (d->hidden == 64) {
    if (bf) hipLaunchKernelGGL((radial_bwd_gh_kernel<64, true>), g1, dim3(256), 0, st, grad_w, n_edges, W, wo, grad_h);
    else hipLaunchKernelGGL((radial_bwd_gh_kernel<64, false>), g1, dim3(256), 0, st, grad_w, n_edges, W, wo, grad_h);
  } else {
    if (bf) hipLaunchKernelGGL((radial_bwd_gh_kernel<32, true>), g1, dim3(256), 0, st, grad_w, n_edges, W, wo, grad_h);
    else hipLaunchKernelGGL((radial_bwd_gh_kernel<32, false>), g1, dim3(256), 0, st, grad_w, n_edges, W, wo, grad_h);
  }
  if (int rc = eelg_check_launch("radial_bwd_gh")) return rc;
  const dim3 g2(nw);
  const int h_ = d->hidden, nh_ = d->n_hidden;
#define RAD_SMALL(HH, NN) hipLaunchKernelGGL((radial_bwd_small_kernel<HH, NN>), g2, dim3(256), 0, st, grad_h, n_edges, *d, zsave, feats, part_h)
  if (h_ == 64) { if (nh_ == 1) RAD_SMALL(64, 1); else if (nh_ == 2) RAD_SMALL(64, 2); else RAD_SMALL(64, 3); }
  else { if (nh_ == 1) RAD_SMALL(32, 1); else if (nh_ == 2) RAD_SMALL(32, 2); else RAD_SMALL(32, 3); }
#undef RAD_SMALL
  if (int rc = eelg_check_launch("radial_bwd_small")) return rc;
  const dim3 g3((W + 127) / 128, ns);
  RAD_LAUNCH3(radial_bwd_wo_kernel, g3, grad_w, n_edges, W, zsave, tps, part_wo);
  return eelg_check_launch("radial_bwd_wo");
}

}  // extern "C"
