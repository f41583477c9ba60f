// Radial MLP of the interaction block (gnn/blocks.py:537-549, applied at :590):
//   z_0 = feats W_0^T + b_0,  h_1 = SiLU(z_0), ...,  z_n = h_n W_n^T + b_n,  h_{n+1} = SiLU(z_n),
//   w = h_NH W_o^T              (no bias on the output layer; W_o: [n_out, hidden])
// with w[E, n_out] the per-edge tensor-product weights (n_out = 1344 for the l>=1 layers of
// BASELINE config 2).  The reference runs this as torch.nn.Sequential of Linear + SiLU.
//
// The hidden layers run on v_mfma_f32_32x32x2_f32 (exact f32 products).  Fragment convention
// (32x32x2): lane l = 32*hf + i supplies A[row i][k] and B[k][col i] for the step's k; the two
// lane halves take k = hf*KH + st over a K block of 2*KH, i.e. the K order is permuted (a sum,
// so any bijection shared by A and B is exact up to rounding order).  The three large GEMMs
// (the output layer and its two gradients: 64 x n_out per edge, ~93 % of the MLP's FLOPs) run
// fp32-accurate on bf16 MFMA (v_mfma_f32_32x32x16_bf16, "x6": each fp32 operand split exactly
// into three bf16 parts, six part products, eelg_internal.h), 3/8 of the f32 MFMA time; lane
// (i, hf) holds A[row i][k = 8 hf + t] and B[k = 8 hf + t][col i], t = 0..7, of a K = 16 block.
// W_o comes pre-split (eelg_split_bf16x3).  C/D of both forms: acc[r] is row
// (r&3) + 8*(r>>2) + 4*hf, column i.
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
// RAD_FWD_NT: the forward's w stores nontemporal (cache policy nt: w is read by tp_fwd layers
// later, after the other layers' MLPs have streamed through the caches)
#ifndef RAD_FWD_NT
#define RAD_FWD_NT 1   // r04r: radial forward 0.254 -> 0.202 ms (kbench), step +0.6 %
#endif
#define RAD_W_POLICY (RAD_FWD_NT ? 2 : 0)
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
// RAD_FWD_CT: output column tiles per staged W_o block (one barrier per block, CT independent
// accumulator chains); RAD_FWD_WPE: waves per SIMD asked of the compiler (0 = its choice)
#ifndef RAD_FWD_CT
#define RAD_FWD_CT 1
#endif
#ifndef RAD_FWD_WPE
#define RAD_FWD_WPE 0
#endif
#if RAD_FWD_WPE > 0
#define RAD_FWD_ATTR __attribute__((amdgpu_waves_per_eu(RAD_FWD_WPE)))
#else
#define RAD_FWD_ATTR
#endif
template <int H, int NH, bool BF>
__global__ __launch_bounds__(256) RAD_FWD_ATTR void radial_fwd_kernel(const float* __restrict__ feats,
                                                         int n_edges, eelg_radial_desc d,
                                                         const unsigned short* __restrict__ wop,
                                                         float* __restrict__ zsave,
                                                         void* __restrict__ out) {
  constexpr int HS = H + 1, NT = H / 32, KH = H / 2, ES = BF ? 2 : 4, NKB = H / 16;
  constexpr int CT = RAD_FWD_CT;
  constexpr int NBF = 3 * NKB * 64 * CT;      // B fragments (uint4) of CT 32-column tiles, all parts
  constexpr int BPT = (NBF + 255) / 256;
  // the hidden activations (hb) and, once every wave has its A fragments, the double-buffered
  // W_o blocks (bt: [buf][tile][((part * NKB + kb) * 2 + hf) * 32 + col]) share one LDS region
  constexpr int HB_BYTES = 4 * 32 * HS * 4, BT_BYTES = 2 * NBF * 16;
  __shared__ uint4 smem[(HB_BYTES > BT_BYTES ? HB_BYTES : BT_BYTES) / 16];
  float* __restrict__ hb = reinterpret_cast<float*>(smem);
  uint4 (*bt)[NBF] = reinterpret_cast<uint4 (*)[NBF]>(smem);
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 31, hf = l >> 5;
  const int e0 = (blockIdx.x * 4 + wave) * 32;
  const int F = d.n_feat, W = d.n_out;
  const uint32_t E = (uint32_t)n_edges;
  const rad_rsrc_t rz = rad_rsrc(zsave, (uint32_t)NH * E * H * 4u);
  const rad_rsrc_t ro = rad_rsrc(out, E * (uint32_t)W * ES);
  const int KF = (F + 1) >> 1;  // layer 0: K = F (<= 32) split over the two lane halves
  // waves past the last edge skip the hidden layers but join the output layer's barriers (their
  // stores fall outside the buffer range)
  const bool active = e0 < n_edges;
  float* __restrict__ hw = hb + wave * 32 * HS;
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
  // output layer, fp32-accurate on bf16 MFMA: w[e0 + row, ct*32 + i] = sum_k h[row][k] W_o[col][k].
  // The wave's A fragments (h, split once) stay in registers for every column tile; each
  // 32-column tile of the split W_o (3 x 32 x H bf16) is loaded once per workgroup (coalesced
  // 16-B pieces, the next tile in registers while the current one computes) and read by the
  // 4 waves from LDS in fragment order.
  uint4 ap[NKB][3];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    float v[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) v[t] = hw[i * HS + 16 * kb + 8 * hf + t];
    eelg_split8(v, ap[kb]);
  }
  const int nct = (W + 31) >> 5;
  uint4 rb[BPT];
  auto load_b = [&](int ct) {   // tiles ct .. ct + CT - 1
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
      const int idx = threadIdx.x + 256 * q;
      const int tt = idx / (3 * NKB * 64), r0 = idx - tt * (3 * NKB * 64);
      const int p = r0 / (NKB * 64), rem = r0 - p * (NKB * 64);
      const int kb = rem >> 6, h2 = (rem >> 5) & 1, col = (ct + tt) * 32 + (rem & 31);
      rb[q] = (idx < NBF && col < W)
                  ? *reinterpret_cast<const uint4*>(wop + ((size_t)p * W + col) * H + 16 * kb + 8 * h2)
                  : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
      const int idx = threadIdx.x + 256 * q;
      if (idx < NBF) bt[buf][idx] = rb[q];
    }
  };
  load_b(0);
  __syncthreads();   // every wave has read its hidden activations: the region becomes bt
  store_b(0);
  __syncthreads();
  for (int c0 = 0, buf = 0; c0 < nct; c0 += CT, buf ^= 1) {
    if (c0 + CT < nct) load_b(c0 + CT);
    rad_f32x16 acc[CT];
#pragma unroll
    for (int tt = 0; tt < CT; ++tt)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[tt][r] = 0.0f;
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int tt = 0; tt < CT; ++tt) {
        const uint4* __restrict__ bb = bt[buf] + tt * 3 * NKB * 64 + hf * 32 + i;
        uint4 b[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) b[p] = bb[(p * NKB + kb) * 64];
        EELG_X6(acc[tt], ap[kb], b);
      }
#pragma unroll
    for (int tt = 0; tt < CT; ++tt) {
      const int col = (c0 + tt) * 32 + i;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const uint32_t off = rad_off(((uint32_t)(e0 + rad_row(r, hf)) * W + col) * ES, col < W);
        if (BF)
          __builtin_amdgcn_raw_buffer_store_b16(eelg_f2bf(acc[tt][r]), ro, (int)off, 0, RAD_W_POLICY);
        else
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[tt][r]), ro, (int)off, 0, RAD_W_POLICY);
      }
    }
    if (c0 + CT < nct) store_b(buf ^ 1);
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// backward 1: grad_h[E, H] = grad_w[E, W] W_o[W, H]   (fp32-accurate on bf16 MFMA)
// ---------------------------------------------------------------------------------------------
// A wave owns 32 edges; K = W runs in 32-wide chunks.  grad_w rows are read coalesced (8 or 16
// rows x 128 B per wave-instruction) into a wave-private LDS tile, from which each lane takes its
// A fragment (8 consecutive k of its row) and splits it; bf16 storage (config 5) is exactly one
// bf16 part.  B[k][c] = W_o[k][c] comes from the split W_o^T ([3][H][W], k contiguous): each
// chunk's 3 x H x 32 bf16 are staged in LDS once per workgroup in fragment order, shared by its
// 4 waves, the next chunk's pieces in registers while the current one computes.
template <int H, bool BF>
__global__ __launch_bounds__(256) void radial_bwd_gh_kernel(const void* __restrict__ gw,
                                                            int n_edges, int W,
                                                            const unsigned short* __restrict__ wotp,
                                                            float* __restrict__ gh) {
  constexpr int NT = H / 32, KC = 32, ES = BF ? 2 : 4;
  constexpr int AS = KC + 4;                  // A tile row stride (floats; rows 16-B aligned)
  constexpr int NV = BF ? 2 : 4;              // 16-B loads per lane per chunk
  constexpr int NBF = 3 * NT * 2 * 64;        // B fragments per chunk: parts x col tiles x kb x lanes
  constexpr int BPT = (NBF + 255) / 256;
  __shared__ uint4 bs[2][NBF];                // [buf][((part * NT + ct) * 2 + kb) * 64 + hf * 32 + c]
  __shared__ float as_[4][32 * AS];
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 31, hf = l >> 5;
  const int e0 = (blockIdx.x * 4 + wave) * 32;   // waves past the last edge still stage / sync
  const uint32_t E = (uint32_t)n_edges;
  const rad_rsrc_t rg = rad_rsrc(gw, E * (uint32_t)W * ES);
  const rad_rsrc_t rh = rad_rsrc(gh, E * (uint32_t)H * 4u);
  const int nchunk = (W + KC - 1) / KC;
  float* __restrict__ at = as_[wave];

  // raw chunk loads, row-coalesced: fp32 piece q = rows 8q + (l >> 3), columns 4 (l & 7) ..+3;
  // bf16 piece q = rows 16q + (l >> 2), columns 8 (l & 3) ..+7.  Rows past E and columns past W
  // read zeros (W is a multiple of 8, so a piece is wholly in or out).
  uint4 raw[NV];
  auto load_a = [&](int kc) {
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const int row = BF ? 16 * q + (l >> 2) : 8 * q + (l >> 3);
      const int col = kc + (BF ? 8 * (l & 3) : 4 * (l & 7));
      const uint32_t off = rad_off(((uint32_t)(e0 + row) * W + col) * ES, col < W);
      raw[q] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rg, (int)off, 0, 0));
    }
  };
  auto stage_a = [&]() {
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      if (BF) {
        const int row = 16 * q + (l >> 2), c = 8 * (l & 3);
        const uint32_t w4[4] = {raw[q].x, raw[q].y, raw[q].z, raw[q].w};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          at[row * AS + c + 2 * u] = __uint_as_float(w4[u] << 16);
          at[row * AS + c + 2 * u + 1] = __uint_as_float(w4[u] & 0xffff0000u);
        }
      } else {
        const int row = 8 * q + (l >> 3), c = 4 * (l & 7);
        *reinterpret_cast<uint4*>(&at[row * AS + c]) = raw[q];
      }
    }
  };
  uint4 rb[BPT];
  auto load_b = [&](int kc) {
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
      const int idx = threadIdx.x + 256 * q;
      const int c = idx & 31, h2 = (idx >> 5) & 1, kb = (idx >> 6) & 1, pc = idx >> 7;
      const int p = pc / NT, ct = pc - p * NT;
      const int k = kc + 16 * kb + 8 * h2;
      rb[q] = (idx < NBF && k < W)
                  ? *reinterpret_cast<const uint4*>(wotp + ((size_t)p * H + ct * 32 + c) * W + k)
                  : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int q = 0; q < BPT; ++q) {
      const int idx = threadIdx.x + 256 * q;
      if (idx < NBF) bs[buf][idx] = rb[q];
    }
  };

  rad_f32x16 acc[NT], lo[NT];   // hi (a0 b0) and lo (the small part products), EELG_X6HL
#pragma unroll
  for (int ct = 0; ct < NT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[ct][r] = lo[ct][r] = 0.0f;
  load_b(0);
  store_b(0);
  load_a(0);
  for (int c = 0; c < nchunk; ++c) {
    __syncthreads();   // chunk c staged; every wave is past chunk c-1's reads of bs[(c+1)&1]
    stage_a();
    // this lane's A fragments of chunk c: row i, k = 16 kb + 8 hf + t
    float av[2][8];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const float4 v0 = *reinterpret_cast<const float4*>(&at[i * AS + 16 * kb + 8 * hf]);
      const float4 v1 = *reinterpret_cast<const float4*>(&at[i * AS + 16 * kb + 8 * hf + 4]);
      av[kb][0] = v0.x; av[kb][1] = v0.y; av[kb][2] = v0.z; av[kb][3] = v0.w;
      av[kb][4] = v1.x; av[kb][5] = v1.y; av[kb][6] = v1.z; av[kb][7] = v1.w;
    }
    if (c + 1 < nchunk) {   // uniform; in flight during the MFMAs
      load_b((c + 1) * KC);
      load_a((c + 1) * KC);
    }
    const uint4* __restrict__ bb = bs[c & 1] + hf * 32 + i;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      uint4 ap[3];
      if (BF) {
        // exactly bf16: the high halves are the one part
#define RAD_PK(t) __builtin_amdgcn_perm(__float_as_uint(av[kb][t + 1]), __float_as_uint(av[kb][t]), 0x07060302u)
        ap[0] = make_uint4(RAD_PK(0), RAD_PK(2), RAD_PK(4), RAD_PK(6));
#undef RAD_PK
      } else {
        eelg_split8(av[kb], ap);
      }
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        uint4 b[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) b[p] = bb[((p * NT + ct) * 2 + kb) * 64];
        if (BF)
          EELG_X3HL(acc[ct], lo[ct], ap[0], b);
        else
          EELG_X6HL(acc[ct], lo[ct], ap, b);
      }
    }
    if (c + 1 < nchunk) store_b((c + 1) & 1);
  }
#pragma unroll
  for (int ct = 0; ct < NT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      rad_bst(rh, ((uint32_t)(e0 + rad_row(r, hf)) * H + ct * 32 + i) * 4u, acc[ct][r] + lo[ct][r]);
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
#ifndef RAD_S2_H64N2
#define RAD_S2_H64N2 0   // hidden 64, 2 hidden layers (the reference default): the LDS-quadrant kernel
#endif
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

// backward 2, register form (hidden 64 with up to 2 hidden layers, hidden 32 with up to 3: the
// weight-gradient accumulators fit in registers).  A wave owns whole 32-edge tiles (grid-stride)
// and keeps every tile in the MFMA C layout (rows = edges in registers, column = lane): for
// grad W_n = sum_e gz[e]^T h_n[e] the K axis is the edges, so with the K order permuted to
// the C rows (step st takes edges rad_row(st, 0) and rad_row(st, 1)) both operands ARE the
// C-layout registers of gz and h_n -- no LDS staging, no workgroup barrier per tile.  Only the
// chain to the layer below (gz W_n, K = the hidden units) goes through a wave-private LDS
// transpose.  The 4 waves' accumulators are summed through LDS once, at the end.
// waves per SIMD: 2 (256 registers) where the accumulators fit, else 1 (hidden 64 with 2 hidden
// layers: 96 accumulator registers + the tile's; EELG build flag RAD_S2_H64N2 picks the kernel)
#ifndef RAD_S2_WPE64
#define RAD_S2_WPE64 1   // waves per SIMD asked for hidden 64 with >= 2 hidden layers
#endif
template <int H, int NH>
constexpr int rad_s2_wpe() { return (H == 64 && NH >= 2) ? RAD_S2_WPE64 : 2; }
template <int H, int NH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(rad_s2_wpe<H, NH>()))) void radial_bwd_small2_kernel(
    const float* __restrict__ ghin, int n_edges, eelg_radial_desc d, const float* __restrict__ zsave,
    const float* __restrict__ feats, float* __restrict__ part) {
  constexpr int HS = H + 1, NT = H / 32, KH = H / 2, NHM = NH > 1 ? NH - 1 : 1;
  __shared__ float G[4 * 32 * HS];
  __shared__ float WS[NHM * H * H];   // the hidden layers' weights W_1.. (the chain's B operand)
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 31, hf = l >> 5;
  const int F = d.n_feat;
  const int ntile = (n_edges + 31) >> 5;
  float* __restrict__ gw_ = G + wave * 32 * HS;
  // buffer loads with 32-bit offsets (rows past E read 0): a 64-bit address per load position,
  // hoisted out of the tile loop, would take ~100 registers
  const uint32_t E32 = (uint32_t)n_edges;
  const rad_rsrc_t rgh = rad_rsrc(ghin, E32 * H * 4u);
  const rad_rsrc_t rzs = rad_rsrc(zsave, (uint32_t)NH * E32 * H * 4u);
  const rad_rsrc_t rft = rad_rsrc(feats, E32 * (uint32_t)F * 4u);
#pragma unroll
  for (int n = 1; n < NH; ++n)
    for (int e = threadIdx.x; e < H * H; e += 256) WS[(n - 1) * H * H + e] = d.w[n][e];
  __syncthreads();
  rad_f32x16 accH[NHM][NT][NT], acc0[NT];
  float bacc[NH][NT];
#pragma unroll
  for (int a = 0; a < NT; ++a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc0[a][r] = 0.0f;
#pragma unroll
    for (int n = 0; n < NHM; ++n)
#pragma unroll
      for (int b = 0; b < NT; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) accH[n][a][b][r] = 0.0f;
#pragma unroll
    for (int n = 0; n < NH; ++n) bacc[n][a] = 0.0f;
  }
  for (int t = blockIdx.x * 4 + wave; t < ntile; t += gridDim.x * 4) {
    const int e0 = t * 32;
    rad_f32x16 gh[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = e0 + rad_row(r, hf);
        gh[ct][r] = rad_bld(rgh, rad_off(((uint32_t)row * H + ct * 32 + i) * 4u, row < n_edges));
      }
#pragma unroll
    for (int n = NH - 1; n >= 0; --n) {
      // scheduling fences between the layers: the loads of a layer are not hoisted above the
      // previous layer's MFMAs (their registers would stay live across them and spill)
      __builtin_amdgcn_sched_barrier(0);
      // gz = grad_h * SiLU'(z_n), in place (C layout)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = e0 + rad_row(r, hf);
          const float z = rad_bld(rzs, rad_off((((uint32_t)n * E32 + row) * H + ct * 32 + i) * 4u, row < n_edges));
          gh[ct][r] = rad_silu_grad(z, gh[ct][r]);
        }
#pragma unroll
      for (int ct = 0; ct < NT; ++ct) {
        float sb = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) sb += gh[ct][r];
        bacc[n][ct] += sb;
      }
      if (n == 0) {
        // grad W_0[j][k] += sum_e gz[e][j] feats[e][k], k < F <= 32 (one column tile)
        rad_f32x16 xr;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = e0 + rad_row(r, hf);
          xr[r] = rad_bld(rft, rad_off(((uint32_t)row * F + i) * 4u, row < n_edges && i < F));
        }
#pragma unroll
        for (int jt = 0; jt < NT; ++jt)
#pragma unroll
          for (int st = 0; st < 16; ++st) acc0[jt] = RAD_MFMA(gh[jt][st], xr[st], acc0[jt]);
      } else {
        // the layer input h_n = SiLU(z_{n-1}) in C layout; grad W_n[j][c] += sum_e gz[e][j] h_n[e][c]
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) {   // one column tile of h_n at a time (registers)
          rad_f32x16 xr;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = e0 + rad_row(r, hf);
            xr[r] = rad_silu(rad_bld(rzs, rad_off((((uint32_t)(n - 1) * E32 + row) * H + ct * 32 + i) * 4u, row < n_edges)));
          }
#pragma unroll
          for (int jt = 0; jt < NT; ++jt)
#pragma unroll
            for (int st = 0; st < 16; ++st)
              accH[n - 1][jt][ct] = RAD_MFMA(gh[jt][st], xr[st], accH[n - 1][jt][ct]);
        }
        __builtin_amdgcn_sched_barrier(0);
        // grad of h_n for the layer below: gh[e][c] = sum_j gz[e][j] W_n[j][c] (rows e on the
        // lanes: through the wave's LDS transpose)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct)
#pragma unroll
          for (int r = 0; r < 16; ++r) gw_[rad_row(r, hf) * HS + ct * 32 + i] = gh[ct][r];
        __builtin_amdgcn_wave_barrier();
        float a3[KH];
#pragma unroll
        for (int st = 0; st < KH; ++st) a3[st] = gw_[i * HS + hf * KH + st];
        __builtin_amdgcn_wave_barrier();
        const float* __restrict__ wn = WS + (n - 1) * H * H;
#pragma unroll
        for (int c2 = 0; c2 < NT; ++c2) {
#pragma unroll
          for (int r = 0; r < 16; ++r) gh[c2][r] = 0.0f;
#pragma unroll
          for (int st = 0; st < KH; ++st)
            gh[c2] = RAD_MFMA(a3[st], wn[(hf * KH + st) * H + c2 * 32 + i], gh[c2]);
        }
      }
    }
  }
  // the workgroup's partial: the 4 waves' accumulator tiles summed through LDS, one tile at a time
  float* __restrict__ dst = part + (size_t)blockIdx.x * (size_t)((H * F + H) + (NH - 1) * (H * H + H));
  auto reduce_tile = [&](const rad_f32x16& v, float* out, int ldo, int jb, int cb, int cmax) {
    __syncthreads();
    if (wave > 0)
#pragma unroll
      for (int r = 0; r < 16; ++r) G[((wave - 1) * 16 + r) * 64 + l] = v[r];
    __syncthreads();
    if (wave == 0)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float s = v[r] + G[r * 64 + l] + G[(16 + r) * 64 + l] + G[(32 + r) * 64 + l];
        if (cb + i < cmax) out[(size_t)(jb + rad_row(r, hf)) * ldo + cb + i] = s;
      }
  };
  size_t off = 0;
#pragma unroll
  for (int n = 0; n < NH; ++n) {
    const int din = n == 0 ? F : H;
#pragma unroll
    for (int jt = 0; jt < NT; ++jt) {
      if (n == 0) reduce_tile(acc0[jt], dst + off, F, jt * 32, 0, F);
      else
#pragma unroll
        for (int ct = 0; ct < NT; ++ct) reduce_tile(accH[n > 0 ? n - 1 : 0][jt][ct], dst + off, H, jt * 32, ct * 32, H);
    }
    off += (size_t)H * din;
    // bias: lane (i, hf) holds its half's sum for column jt*32 + i; 8 partial sums per column
    __syncthreads();
#pragma unroll
    for (int jt = 0; jt < NT; ++jt) G[(jt * 4 + wave) * 64 + l] = bacc[n][jt];
    __syncthreads();
    if (threadIdx.x < H) {
      const int jt = threadIdx.x >> 5, c = threadIdx.x & 31;
      float s = 0.0f;
#pragma unroll
      for (int w = 0; w < 4; ++w) s += G[(jt * 4 + w) * 64 + c] + G[(jt * 4 + w) * 64 + 32 + c];
      dst[off + threadIdx.x] = s;
    }
    off += H;
  }
}


// ---------------------------------------------------------------------------------------------
// backward 2, chain form (round 5): only the chain through SiLU' and the hidden layers, no
// weight gradients.  A wave owns one 32-edge tile (grid-stride), in the MFMA C layout; for
// n = NH-1 .. 0 it turns grad_h into gz_n = grad_h * SiLU'(z_n) and stores it, stores the layer
// input h_n = SiLU(z_{n-1}) (n > 0; z_{n-1} is kept for the next layer's SiLU'), and forms the
// grad_h of the layer below, gz_n W_n, through a wave-private LDS transpose.  The weight and bias
// gradients (gz_n^T h_n, gz_0^T feats, column sums of gz_n) are then long-K reductions that the
// linear weight-gradient kernel and eelg_sum_rows run (gnn/ops.py): the fused form kept 96
// accumulator registers per wave across its tiles and ran at one to two waves per SIMD with
// scratch spills (0.24 ms at the bench shape, 11.5 % MFMA busy, profiles/r04l_pmc.md).
template <int H, int NH>
__global__ __launch_bounds__(256) void radial_bwd_chain_kernel(
    const float* __restrict__ ghin, int n_edges, eelg_radial_desc d, const float* __restrict__ zsave,
    float* __restrict__ gz, float* __restrict__ hin) {
  constexpr int HS = H + 1, NT = H / 32, KH = H / 2, NHM = NH > 1 ? NH - 1 : 1;
  __shared__ float G[4 * 32 * HS];
  __shared__ float WS[NHM * H * H];   // W_1 .. W_{NH-1} (the chain's B operand)
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 31, hf = l >> 5;
  const int ntile = (n_edges + 31) >> 5;
  float* __restrict__ gw_ = G + wave * 32 * HS;
  const uint32_t E32 = (uint32_t)n_edges;
  const rad_rsrc_t rgh = rad_rsrc(ghin, E32 * H * 4u);
  const rad_rsrc_t rzs = rad_rsrc(zsave, (uint32_t)NH * E32 * H * 4u);
  const rad_rsrc_t rgz = rad_rsrc(gz, (uint32_t)NH * E32 * H * 4u);
  const rad_rsrc_t rhi = rad_rsrc(hin, (uint32_t)NHM * E32 * H * 4u);
#pragma unroll
  for (int n = 1; n < NH; ++n)
    for (int e = threadIdx.x; e < H * H; e += 256) WS[(n - 1) * H * H + e] = d.w[n][e];
  __syncthreads();
  for (int t = blockIdx.x * 4 + wave; t < ntile; t += gridDim.x * 4) {
    const int e0 = t * 32;
    rad_f32x16 gh[NT], zc[NT];
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = e0 + rad_row(r, hf);
        const uint32_t o = ((uint32_t)row * H + ct * 32 + i) * 4u;
        gh[ct][r] = rad_bld(rgh, rad_off(o, row < n_edges));
        zc[ct][r] = rad_bld(rzs, rad_off((uint32_t)(NH - 1) * E32 * H * 4u + o, row < n_edges));
      }
#pragma unroll
    for (int n = NH - 1; n >= 0; --n) {
      __builtin_amdgcn_sched_barrier(0);
      // gz_n = grad_h * SiLU'(z_n), stored (rows past E dropped by the buffer range check)
#pragma unroll
      for (int ct = 0; ct < NT; ++ct)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = e0 + rad_row(r, hf);
          gh[ct][r] = rad_silu_grad(zc[ct][r], gh[ct][r]);
          rad_bst(rgz, rad_off((((uint32_t)n * E32 + row) * H + ct * 32 + i) * 4u, row < n_edges), gh[ct][r]);
        }
      if (n > 0) {
        // the layer input h_n = SiLU(z_{n-1}); z_{n-1} stays for the next layer's SiLU'
#pragma unroll
        for (int ct = 0; ct < NT; ++ct)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = e0 + rad_row(r, hf);
            const uint32_t o = ((uint32_t)row * H + ct * 32 + i) * 4u;
            zc[ct][r] = rad_bld(rzs, rad_off((uint32_t)(n - 1) * E32 * H * 4u + o, row < n_edges));
            rad_bst(rhi, rad_off((uint32_t)(n - 1) * E32 * H * 4u + o, row < n_edges), rad_silu(zc[ct][r]));
          }
        // grad_h of the layer below: gh[e][c] = sum_j gz[e][j] W_n[j][c] (the wave's rows on the
        // lanes through its LDS transpose)
#pragma unroll
        for (int ct = 0; ct < NT; ++ct)
#pragma unroll
          for (int r = 0; r < 16; ++r) gw_[rad_row(r, hf) * HS + ct * 32 + i] = gh[ct][r];
        __builtin_amdgcn_wave_barrier();
        float a3[KH];
#pragma unroll
        for (int st = 0; st < KH; ++st) a3[st] = gw_[i * HS + hf * KH + st];
        __builtin_amdgcn_wave_barrier();
        const float* __restrict__ wn = WS + (n - 1) * H * H;
#pragma unroll
        for (int c2 = 0; c2 < NT; ++c2) {
#pragma unroll
          for (int r = 0; r < 16; ++r) gh[c2][r] = 0.0f;
#pragma unroll
          for (int st = 0; st < KH; ++st)
            gh[c2] = RAD_MFMA(a3[st], wn[(hf * KH + st) * H + c2 * 32 + i], gh[c2]);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// backward 3: grad of the output weight   (fp32-accurate on bf16 MFMA)
// ---------------------------------------------------------------------------------------------
// part[s, j, k] = sum over split s's edges of grad_w[e, j] * SiLU(z_last[e, k]).  A wave owns 32
// output rows j; K = edges in 32-edge tiles (two K = 16 blocks).  A[j][e] = grad_w[e][j]: a lane
// loads its 16 values (coalesced over j), splits them (bf16 storage: one exact part).  B[e][k] =
// SiLU(z_last[e][k]) is computed, split and stored in LDS in fragment order once per workgroup by
// all its threads (one fragment per thread at H = 64), double buffered.
template <int H, int NH, bool BF>
__global__ __launch_bounds__(256) void radial_bwd_wo_kernel(const void* __restrict__ gw,
                                                            int n_edges, int W,
                                                            const float* __restrict__ zsave,
                                                            int tiles_per_split,
                                                            float* __restrict__ part) {
  constexpr int NT = H / 32, ES = BF ? 2 : 4;
  constexpr int NFR = NT * 2 * 64;             // B fragments of a tile per part (ct, kb, hf, k)
  __shared__ uint4 hs[2][3 * NFR];             // [buf][part * NFR + ((ct * 2 + kb) * 2 + hf) * 32 + k]
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 31, hf = l >> 5;
  const int j = blockIdx.x * 128 + wave * 32 + i;   // this lane's grad_w column (A row)
  const int s = blockIdx.y;
  const int ntile = (n_edges + 31) >> 5;
  const int t0 = s * tiles_per_split, t1 = min(ntile, t0 + tiles_per_split);
  const uint32_t E = (uint32_t)n_edges;
  const rad_rsrc_t rg = rad_rsrc(gw, E * (uint32_t)W * ES);
  const rad_rsrc_t rz = rad_rsrc(zsave + (size_t)(NH - 1) * E * H, E * (uint32_t)H * 4u);
  // the B fragment this thread builds: (ct, kb, hf, k) = decomposition of threadIdx.x
  const bool bmine = threadIdx.x < NFR;
  const int bk = threadIdx.x & 31, bh = (threadIdx.x >> 5) & 1, bkb = (threadIdx.x >> 6) & 1,
            bct = threadIdx.x >> 7;
  rad_f32x16 acc[NT], lo[NT];   // hi / lo accumulators (EELG_X6HL): K = a split's edges
#pragma unroll
  for (int ct = 0; ct < NT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[ct][r] = lo[ct][r] = 0.0f;
  float an[16], zn[8];
  auto load = [&](int t) {
    // A[j][e]: e = t*32 + 16 kb + 8 hf + u; rows past E read zeros
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const uint32_t off = rad_off(((uint32_t)(t * 32 + 16 * kb + 8 * hf + u) * W + j) * ES, j < W);
        if (BF)
          an[8 * kb + u] = eelg_bf2f((unsigned short)__builtin_amdgcn_raw_buffer_load_b16(rg, (int)off, 0, 0));
        else
          an[8 * kb + u] = rad_bld(rg, off);
      }
    // z_last[e][k] of this thread's B fragment: e = t*32 + 16 bkb + 8 bh + u, k = bct*32 + bk
#pragma unroll
    for (int u = 0; u < 8; ++u)
      zn[u] = rad_bld(rz, rad_off(((uint32_t)(t * 32 + 16 * bkb + 8 * bh + u) * H + bct * 32 + bk) * 4u, bmine));
  };
  if (t0 < t1) load(t0);
  for (int t = t0; t < t1; ++t) {
    // h_last = SiLU(z_last) (SiLU(0) = 0 past the last edge), split, in fragment order.  Double
    // buffered: the barrier of tile t+1 separates tile t's reads of a buffer from its rewrite.
    uint4* __restrict__ hb = hs[t & 1];
    if (bmine) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = rad_silu(zn[u]);
      uint4 pp[3];
      eelg_split8(v, pp);
#pragma unroll
      for (int p = 0; p < 3; ++p) hb[p * NFR + threadIdx.x] = pp[p];
    }
    __syncthreads();
    uint4 ap[2][3];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      if (BF) {
#define RAD_PK(t) __builtin_amdgcn_perm(__float_as_uint(an[8 * kb + t + 1]), __float_as_uint(an[8 * kb + t]), 0x07060302u)
        ap[kb][0] = make_uint4(RAD_PK(0), RAD_PK(2), RAD_PK(4), RAD_PK(6));
#undef RAD_PK
      } else {
        eelg_split8(&an[8 * kb], ap[kb]);
      }
    }
    if (t + 1 < t1) load(t + 1);   // in flight during the MFMAs
    const uint4* __restrict__ bb = hb + hf * 32 + i;
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        uint4 b[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) b[p] = bb[p * NFR + (ct * 2 + kb) * 64];
        if (BF)
          EELG_X3HL(acc[ct], lo[ct], ap[kb][0], b);
        else
          EELG_X6HL(acc[ct], lo[ct], ap[kb], b);
      }
  }
  const int jb = blockIdx.x * 128 + wave * 32;
#pragma unroll
  for (int ct = 0; ct < NT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jj = jb + rad_row(r, hf);
      if (jj < W) part[((size_t)s * W + jj) * H + ct * 32 + i] = acc[ct][r] + lo[ct][r];
    }
}

// ---------------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------------
// the exact three-part bf16 split of an fp32 array (eelg_split_bf16x3): parts[p * n + i]
__global__ __launch_bounds__(256) void split_bf16x3_kernel(const float* __restrict__ src, long long n,
                                                           unsigned short* __restrict__ parts) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float x = src[i];
  const unsigned a = __float_as_uint(x) & 0xffff0000u;
  const float r = x - __uint_as_float(a);
  const unsigned b = __float_as_uint(r) & 0xffff0000u;
  parts[i] = (unsigned short)(a >> 16);
  parts[n + i] = (unsigned short)(b >> 16);
  parts[2 * n + i] = (unsigned short)(__float_as_uint(r - __uint_as_float(b)) >> 16);
}

static int radial_check(const eelg_radial_desc* d, int n_edges, int out_es) {
  if (!d) return eelg_fail(-2, "radial: null descriptor");
  if (d->hidden != 32 && d->hidden != 64)
    return eelg_fail(-2, "radial: hidden width %d not built (32 or 64)", d->hidden);
  if (d->n_hidden < 1 || d->n_hidden > EELG_RADIAL_MAXH)
    return eelg_fail(-2, "radial: %d hidden layers not built (1..%d)", d->n_hidden, EELG_RADIAL_MAXH);
  if (d->n_feat < 1 || d->n_feat > 32)
    return eelg_fail(-2, "radial: %d input features not built (1..32)", d->n_feat);
  if (d->n_out < 1 || d->n_out % 8)
    return eelg_fail(-2, "radial: n_out %d must be a positive multiple of 8 (16-B pieces of the "
                         "split W_o rows)", d->n_out);
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

int eelg_split_bf16x3(const float* src, long long n, void* parts, void* stream) {
  if (n < 0) return eelg_fail(-2, "split_bf16x3: negative length");
  if (n == 0) return 0;
  hipLaunchKernelGGL(split_bf16x3_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, src, n, static_cast<unsigned short*>(parts));
  return eelg_check_launch("split_bf16x3");
}

static bool rad_a16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

int eelg_radial_fwd(const float* feats, int n_edges, const eelg_radial_desc* d, const void* wo_parts,
                    int out_bf16, float* zsave, void* out, void* stream) {
  if (int rc = radial_check(d, n_edges, out_bf16 ? 2 : 4)) return rc;
  if (!rad_a16(wo_parts)) return eelg_fail(-2, "radial_fwd: wo_parts must be 16-byte aligned");
  if (n_edges == 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const bool bf = out_bf16 != 0;
  const dim3 grid((n_edges + 127) / 128);
  const unsigned short* wop = static_cast<const unsigned short*>(wo_parts);
  RAD_LAUNCH3(radial_fwd_kernel, grid, feats, n_edges, *d, wop, zsave, out);
  return eelg_check_launch("radial_fwd");
}

int eelg_radial_bwd_chain(const void* grad_w, int grad_bf16, int n_edges, const eelg_radial_desc* d,
                          const void* wot_parts, const float* zsave, float* grad_h, float* gz,
                          float* hin, float* part_wo, void* stream) {
  if (int rc = radial_check(d, n_edges, grad_bf16 ? 2 : 4)) return rc;
  if (!rad_a16(wot_parts) || !rad_a16(grad_w))
    return eelg_fail(-2, "radial_bwd_chain: grad_w and wot_parts must be 16-byte aligned");
  if (d->hidden != 64) return eelg_fail(-2, "radial_bwd_chain: hidden %d not built (64)", d->hidden);
  if (n_edges == 0) return 0;
  const unsigned short* wotp = static_cast<const unsigned short*>(wot_parts);
  hipStream_t st = (hipStream_t)stream;
  const bool bf = grad_bf16 != 0;
  int nw, ns, tps;
  radial_plan(n_edges, d->n_out, &nw, &ns, &tps);
  const dim3 g1((n_edges + 127) / 128);
  const int W = d->n_out;
  if (bf) hipLaunchKernelGGL((radial_bwd_gh_kernel<64, true>), g1, dim3(256), 0, st, grad_w, n_edges, W, wotp, grad_h);
  else hipLaunchKernelGGL((radial_bwd_gh_kernel<64, false>), g1, dim3(256), 0, st, grad_w, n_edges, W, wotp, grad_h);
  if (int rc = eelg_check_launch("radial_bwd_gh")) return rc;
  const int ntile = (n_edges + 31) / 32;
  const dim3 g2((unsigned)((ntile + 3) / 4 < 2048 ? (ntile + 3) / 4 : 2048));
  if (d->n_hidden == 1)
    hipLaunchKernelGGL((radial_bwd_chain_kernel<64, 1>), g2, dim3(256), 0, st, grad_h, n_edges, *d, zsave, gz, hin);
  else if (d->n_hidden == 2)
    hipLaunchKernelGGL((radial_bwd_chain_kernel<64, 2>), g2, dim3(256), 0, st, grad_h, n_edges, *d, zsave, gz, hin);
  else
    hipLaunchKernelGGL((radial_bwd_chain_kernel<64, 3>), g2, dim3(256), 0, st, grad_h, n_edges, *d, zsave, gz, hin);
  if (int rc = eelg_check_launch("radial_bwd_chain")) return rc;
  const dim3 g3((W + 127) / 128, ns);
  RAD_LAUNCH3(radial_bwd_wo_kernel, g3, grad_w, n_edges, W, zsave, tps, part_wo);
  return eelg_check_launch("radial_bwd_wo");
}

int eelg_radial_bwd(const void* grad_w, int grad_bf16, int n_edges, const eelg_radial_desc* d,
                    const void* wot_parts, const float* zsave, const float* feats, float* grad_h,
                    float* part_h, float* part_wo, void* stream) {
  if (int rc = radial_check(d, n_edges, grad_bf16 ? 2 : 4)) return rc;
  if (!rad_a16(wot_parts) || !rad_a16(grad_w))
    return eelg_fail(-2, "radial_bwd: grad_w and wot_parts must be 16-byte aligned");
  if (n_edges == 0) return 0;
  const unsigned short* wotp = static_cast<const unsigned short*>(wot_parts);
  hipStream_t st = (hipStream_t)stream;
  const bool bf = grad_bf16 != 0;
  int nw, ns, tps;
  radial_plan(n_edges, d->n_out, &nw, &ns, &tps);
  const dim3 g1((n_edges + 127) / 128);
  const int W = d->n_out;
  if (d->hidden == 64) {
    if (bf) hipLaunchKernelGGL((radial_bwd_gh_kernel<64, true>), g1, dim3(256), 0, st, grad_w, n_edges, W, wotp, grad_h);
    else hipLaunchKernelGGL((radial_bwd_gh_kernel<64, false>), g1, dim3(256), 0, st, grad_w, n_edges, W, wotp, grad_h);
  } else {
    if (bf) hipLaunchKernelGGL((radial_bwd_gh_kernel<32, true>), g1, dim3(256), 0, st, grad_w, n_edges, W, wotp, grad_h);
    else hipLaunchKernelGGL((radial_bwd_gh_kernel<32, false>), g1, dim3(256), 0, st, grad_w, n_edges, W, wotp, grad_h);
  }
  if (int rc = eelg_check_launch("radial_bwd_gh")) return rc;
  const dim3 g2(nw);
  const int h_ = d->hidden, nh_ = d->n_hidden;
#define RAD_SMALL(HH, NN) hipLaunchKernelGGL((radial_bwd_small_kernel<HH, NN>), g2, dim3(256), 0, st, grad_h, n_edges, *d, zsave, feats, part_h)
#define RAD_SMALL2(HH, NN) hipLaunchKernelGGL((radial_bwd_small2_kernel<HH, NN>), g2, dim3(256), 0, st, grad_h, n_edges, *d, zsave, feats, part_h)
  if (h_ == 64) {
    if (nh_ == 1) RAD_SMALL2(64, 1);
    else if (nh_ == 2) { if (RAD_S2_H64N2) RAD_SMALL2(64, 2); else RAD_SMALL(64, 2); }
    else RAD_SMALL(64, 3);
  }
  else { if (nh_ == 1) RAD_SMALL2(32, 1); else if (nh_ == 2) RAD_SMALL2(32, 2); else RAD_SMALL2(32, 3); }
#undef RAD_SMALL
#undef RAD_SMALL2
  if (int rc = eelg_check_launch("radial_bwd_small")) return rc;
  const dim3 g3((W + 127) / 128, ns);
  RAD_LAUNCH3(radial_bwd_wo_kernel, g3, grad_w, n_edges, W, zsave, tps, part_wo);
  return eelg_check_launch("radial_bwd_wo");
}

}  // extern "C"
