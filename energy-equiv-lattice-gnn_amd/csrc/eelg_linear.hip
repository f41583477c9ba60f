// Channel-mixing linear on e3nn mul-major irreps rows (o3.Linear,
// gnn/blocks.py:516-521,553-559,471-476; gnn/model.py:82-86), fp32 MFMA.
//
// For one output slot (mul_out copies of an irrep of dimension d):
//   y[n, j, m] = sum_src alpha_src * sum_u x[n, x_off + u*d + m] * W[u, j]   (+ bias[j] if d == 1)
// i.e. a GEMM whose rows are (node, component) pairs, K = mul_in, N = mul_out.
//
// HBM access is the cost (the 7360 -> 800 interaction linear moves ~1 GB per call at
// 16 FLOP/B), so every global access is a contiguous per-node run: a node's block of one
// irrep is K*d consecutive floats, and a 32-wide K chunk of it is 32*d consecutive floats.
// A workgroup owns 128 consecutive (node, m) rows of one slot; it stages each K chunk of
// those rows into LDS as A[row][k] with float4 loads, the matching 32x32 weight tile as
// B[k][j], runs v_mfma_f32_32x32x2_f32 (one 32-row tile per wave; exact f32 products),
// and writes the output tile back through LDS as per-node contiguous runs.  grad-x uses
// the same kernel with the transposed weight (ldk/ldj swapped).  grad-W reduces over
// rows into deterministic per-slice partials (summed on the host side).
#include <hip/hip_runtime.h>
#include <cstdlib>

typedef float eelg_f32x16 __attribute__((ext_vector_type(16)));

#define LIN_ROWS 128           // rows per workgroup (4 waves x 32)
#define LIN_KC 32              // K chunk
#define LIN_ST 33              // LDS row stride in floats (conflict-free column reads)

// Walks a flat index f = a * (W*d) + b*d + m in steps of `step` without divisions in the
// loop (a = node in the run list, b = channel in [0, W), m = component in [0, d)).
struct Walk3 {
  int a, b, m;
  int da, db, dm;
  __device__ void init(int f, int step, int W, int d) {
    const int seg = W * d;
    a = f / seg;
    const int r = f - a * seg;
    b = r / d;
    m = r - b * d;
    da = step / seg;
    const int rr = step - da * seg;
    db = rr / d;
    dm = rr - db * d;
  }
  __device__ void next(int W, int d) {
    a += da;
    b += db;
    m += dm;
    if (m >= d) { m -= d; ++b; }
    if (b >= W) { b -= W; ++a; }
  }
};

// Register-staged copy of one A chunk (<= LIN_NV float4 per thread) and one B tile.
#define LIN_NV 5

struct ChunkRef {
  int x_off, k, kc, w_off, ldk, ldj;
  float alpha;
};

__device__ __forceinline__ ChunkRef lin_chunk(const eelg_lin_slot& sl, int c) {
  int s = 0, base = 0;
  for (;;) {
    const int nc = (sl.src[s].k + LIN_KC - 1) / LIN_KC;
    if (c < base + nc || s + 1 >= sl.n_src) break;
    base += nc;
    ++s;
  }
  const eelg_lin_src& src = sl.src[s];
  ChunkRef r;
  r.x_off = src.x_off;
  r.k = src.k;
  r.kc = (c - base) * LIN_KC;
  r.w_off = src.w_off;
  r.ldk = src.ldk;
  r.ldj = src.ldj;
  r.alpha = src.alpha;
  return r;
}

#ifndef LIN_FWD_WPE
#define LIN_FWD_WPE 4
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LIN_FWD_WPE))) void lin_fwd_kernel(const float* __restrict__ x, int x_row,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ bias, int n_nodes,
                                                      float* __restrict__ y, int y_row,
                                                      eelg_lin_desc desc,
                                                      const float* __restrict__ res) {
  __shared__ float As[LIN_ROWS * LIN_ST];
  __shared__ float Bs[LIN_KC * LIN_ST];
  __shared__ float Os[LIN_ROWS * LIN_ST];
  const eelg_lin_slot& sl = desc.slot[blockIdx.y];
  const int d = sl.d;
  const int rows = n_nodes * d;
  const int r0 = blockIdx.x * LIN_ROWS;
  if (r0 >= rows) return;  // uniform per workgroup
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int n_lo = r0 / d;
  const int n_hi = min(n_nodes, (r0 + LIN_ROWS + d - 1) / d);  // exclusive
  const int span = n_hi - n_lo;
  const int seg = LIN_KC * d;
  const int total = span * seg;  // flat (node, k, m) entries of one chunk
  int n_chunks = 0;
  for (int s = 0; s < sl.n_src; ++s) n_chunks += (sl.src[s].k + LIN_KC - 1) / LIN_KC;
  const int n_jt = (sl.n_out + 31) / 32;
  // float4 staging needs 16-B aligned per-node runs and <= LIN_NV float4 per thread
  bool vec = (x_row & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && total <= LIN_NV * 1024;
  for (int s = 0; s < sl.n_src; ++s) vec = vec && (sl.src[s].x_off & 3) == 0 && (sl.src[s].k & 3) == 0;

  float4 va[LIN_NV];
  float vb[4];
  // issue the global loads of chunk c (A rows into va, B tile into vb)
  auto load_chunk = [&](int c, int jt, bool with_a) {
    const ChunkRef ch = lin_chunk(sl, c);
    const int kk = min(LIN_KC, ch.k - ch.kc);
    if (vec && with_a) {
      const float* __restrict__ xb = x + (size_t)n_lo * x_row + ch.x_off + (size_t)ch.kc * d;
      const int len = kk * d;
      Walk3 cw;
      cw.init(4 * tid, 4 * 256, LIN_KC, d);
#pragma unroll
      for (int q = 0; q < LIN_NV; ++q) {
        const int f = 4 * tid + 1024 * q;
        const int within = cw.b * d + cw.m;
        va[q] = (f < total && within < len)
                    ? *reinterpret_cast<const float4*>(xb + (size_t)cw.a * x_row + within)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
        cw.next(LIN_KC, d);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 256 * q;
      const int k = e >> 5, jj = jt * 32 + (e & 31);
      vb[q] = (k < kk && jj < sl.n_out) ? w[ch.w_off + (size_t)(ch.kc + k) * ch.ldk + (size_t)jj * ch.ldj] * ch.alpha
                                        : 0.0f;
    }
  };
  // write the staged registers of chunk c to LDS (scalar path: load + store directly)
  auto store_chunk = [&](int c, bool with_a) {
    if (with_a) {
      if (vec) {
        Walk3 cw;
        cw.init(4 * tid, 4 * 256, LIN_KC, d);
#pragma unroll
        for (int q = 0; q < LIN_NV; ++q) {
          const int f = 4 * tid + 1024 * q;
          if (f < total) {
            int k = cw.b, m = cw.m;
            const int rbase = (n_lo + cw.a) * d - r0;
            const float vv[4] = {va[q].x, va[q].y, va[q].z, va[q].w};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const int row = rbase + m;
              if (row >= 0 && row < LIN_ROWS) As[row * LIN_ST + k] = vv[t];
              if (++m == d) { m = 0; ++k; }
            }
          }
          cw.next(LIN_KC, d);
        }
      } else {
        const ChunkRef ch = lin_chunk(sl, c);
        const int kk = min(LIN_KC, ch.k - ch.kc);
        const float* __restrict__ xb = x + (size_t)n_lo * x_row + ch.x_off + (size_t)ch.kc * d;
        Walk3 cw;
        cw.init(tid, 256, LIN_KC, d);
        for (int f = tid; f < total; f += 256) {
          const int row = (n_lo + cw.a) * d + cw.m - r0;
          if (row >= 0 && row < LIN_ROWS)
            As[row * LIN_ST + cw.b] = (cw.b < kk) ? xb[(size_t)cw.a * x_row + cw.b * d + cw.m] : 0.0f;
          cw.next(LIN_KC, d);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 256 * q;
      Bs[(e >> 5) * LIN_ST + (e & 31)] = vb[q];
    }
  };

  const float* __restrict__ ar = As + (wave * 32 + (lane & 31)) * LIN_ST + (lane >> 5);
  const float* __restrict__ br = Bs + (lane >> 5) * LIN_ST + (lane & 31);
  for (int jt = 0; jt < n_jt; ++jt) {
    eelg_f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
    const bool restage = n_chunks > 1 || jt == 0;
    load_chunk(0, jt, restage);
    for (int c = 0; c < n_chunks; ++c) {
      __syncthreads();  // previous MFMA reads of As / Bs and epilogue reads of Os are done
      store_chunk(c, restage);
      __syncthreads();
      if (c + 1 < n_chunks) load_chunk(c + 1, jt, true);  // in flight during the MFMAs
      // K padded to 32 with zeros (A and B) -> always 16 steps
#pragma unroll
      for (int st = 0; st < 16; ++st)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[2 * st], br[2 * st * LIN_ST], acc, 0, 0, 0);
    }
    // epilogue: stage the 128 x 32 tile, then write per-node contiguous runs
    const int j = jt * 32 + (lane & 31);
    const float bj = (sl.bias_off >= 0 && j < sl.n_out) ? bias[sl.bias_off + j] : 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = wave * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
      Os[row * LIN_ST + (lane & 31)] = acc[i] + bj;
    }
    __syncthreads();
    const int jw = min(32, sl.n_out - jt * 32);
    const int olen = jw * d;  // floats per node in this column tile
    float* __restrict__ yb = y + (size_t)n_lo * y_row + sl.y_off + (size_t)jt * 32 * d;
    // optional residual (same layout as y) added in the epilogue
    const float* __restrict__ rb = res ? res + (size_t)n_lo * y_row + sl.y_off + (size_t)jt * 32 * d : nullptr;
    const bool vst = (y_row & 3) == 0 && (olen & 3) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0 &&
                     ((sl.y_off + jt * 32 * d) & 3) == 0 && (reinterpret_cast<uintptr_t>(res) & 15) == 0;
    if (vst) {
      // float4 per-node runs; nodes cut by the workgroup's row range go element-wise
      Walk3 ow;
      ow.init(4 * tid, 4 * 256, jw, d);
      for (int f = 4 * tid; f < span * olen; f += 4 * 256) {
        const int nrow0 = (n_lo + ow.a) * d - r0;   // row of (node, m = 0)
        float* dst = yb + (size_t)ow.a * y_row + ow.b * d + ow.m;
        int jj = ow.b, m = ow.m;
        if (nrow0 >= 0 && nrow0 + d <= LIN_ROWS) {
          float v[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            v[t] = Os[(nrow0 + m) * LIN_ST + jj];
            if (++m == d) { m = 0; ++jj; }
          }
          if (rb) {
            const float4 r4 = *reinterpret_cast<const float4*>(rb + (dst - yb));
            v[0] += r4.x; v[1] += r4.y; v[2] += r4.z; v[3] += r4.w;
          }
          *reinterpret_cast<float4*>(dst) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int row = nrow0 + m;
            if (row >= 0 && row < LIN_ROWS) dst[t] = Os[row * LIN_ST + jj] + (rb ? rb[(dst - yb) + t] : 0.0f);
            if (++m == d) { m = 0; ++jj; }
          }
        }
        ow.next(jw, d);
      }
    } else {
      Walk3 ow;
      ow.init(tid, 256, jw, d);
      for (int f = tid; f < span * olen; f += 256) {
        const int row = (n_lo + ow.a) * d + ow.m - r0;
        if (row >= 0 && row < LIN_ROWS) {
          const size_t o = (size_t)ow.a * y_row + ow.b * d + ow.m;
          yb[o] = Os[row * LIN_ST + ow.b] + (rb ? rb[o] : 0.0f);
        }
        ow.next(jw, d);
      }
    }
  }
}

// grad W for each instruction: partial[p, w_off + u*n_out + j] =
//   alpha * sum_{nodes of slice p, m} x[n, x_off + u*d + m] * g[n, g_off + j*d + m]
// One workgroup = (node slice, instruction, 32x32 (u, j) tile).  The four waves take
// chunks of floor(32/d) whole nodes round-robin, stage their X[row][u] / G[row][j] tiles
// (node-contiguous 32*d-float runs) in wave-private LDS, reduce over rows with MFMA
// (zero-padded to 32 rows), and the four accumulators are summed through LDS at the end.
// Fast path of grad W (full 32x32 tiles, 16-B aligned rows): each wave stages chunks of
// NB = floor(32/D) whole nodes in their natural global layout -- per node the u-tile's 32*D
// floats of x, then the j-tile's 32*D floats of g, both contiguous runs -- with float4 loads and
// ds_write_b128 (no transposition, conflict-free).  The MFMA K axis runs over the chunk's
// (node, m) rows: row r = (n, m) sits at n*32*D + m, and lane u reads x[r][u] at + u*D, an odd
// stride (D = 2l+1) over the 32 banks, so the operand reads are conflict-free too.  Rows past
// NB*D point at a zeroed node region.  Same partial layout as the general path.
template <int D>
__device__ __forceinline__ void lin_bwdw_fast(const float* __restrict__ x, int x_row,
                                              const float* __restrict__ g, int g_row, int n0,
                                              int n1, const eelg_linw_ins& in, int ut, int jt,
                                              float* __restrict__ xw, float* __restrict__ gw,
                                              eelg_f32x16& acc) {
  constexpr int NB = 32 / D;            // whole nodes per chunk
  constexpr int RUN4 = 8 * D;           // float4 per node run (32 * D floats)
  constexpr int NQ = (NB * RUN4 + 63) / 64;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, u = lane & 31, hf = lane >> 5;
  // zero node region (rows >= NB*D)
  for (int f = lane; f < 32 * D; f += 64) {
    xw[NB * 32 * D + f] = 0.0f;
    gw[NB * 32 * D + f] = 0.0f;
  }
  int off[16];
#pragma unroll
  for (int st = 0; st < 16; ++st) {
    const int r = 2 * st + hf;
    off[st] = (r < NB * D ? (r / D) * 32 * D + (r % D) : NB * 32 * D) + u * D;
  }
  const float* __restrict__ xb = x + in.x_off + (size_t)ut * 32 * D;
  const float* __restrict__ gb = g + in.g_off + (size_t)jt * 32 * D;
  float4 rx[NQ], rg[NQ];
  auto load_chunk = [&](int nc) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int f = lane + 64 * q;
      const int a = f / RUN4, w4 = f - a * RUN4;
      const bool ok = f < NB * RUN4 && nc + a < n1;
      const int nn = ok ? nc + a : 0;
      rx[q] = ok ? *reinterpret_cast<const float4*>(xb + (size_t)nn * x_row + 4 * w4) : make_float4(0.f, 0.f, 0.f, 0.f);
      rg[q] = ok ? *reinterpret_cast<const float4*>(gb + (size_t)nn * g_row + 4 * w4) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  int nc = n0 + wave * NB;
  if (nc < n1) load_chunk(nc);
  for (; nc < n1; nc += 4 * NB) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int f = lane + 64 * q;
      if (f < NB * RUN4) {
        reinterpret_cast<float4*>(xw)[f] = rx[q];
        reinterpret_cast<float4*>(gw)[f] = rg[q];
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (nc + 4 * NB < n1) load_chunk(nc + 4 * NB);
#pragma unroll
    for (int st = 0; st < 16; ++st)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xw[off[st]], gw[off[st]], acc, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
  }
}

#ifndef LIN_BWDW_WPE
#define LIN_BWDW_WPE 2
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(LIN_BWDW_WPE))) void lin_bwdw_kernel(const float* __restrict__ x, int x_row,
                                                       const float* __restrict__ g, int g_row,
                                                       int n_nodes, int nodes_per_slice,
                                                       float* __restrict__ partial, int w_total,
                                                       eelg_linw_desc desc) {
  __shared__ float Xs[4][32 * LIN_ST];
  __shared__ float Gs[4][32 * LIN_ST];
  const eelg_linw_ins& in = desc.ins[blockIdx.y];
  const int d = in.d, K = in.k, NO = in.n_out;
  const int n_ut = (K + 31) / 32, n_jt = (NO + 31) / 32;
  const int t = blockIdx.z;
  if (t >= n_ut * n_jt) return;  // uniform per workgroup
  const int ut = t / n_jt, jt = t - ut * n_jt;
  const int uw = min(32, K - ut * 32), jw = min(32, NO - jt * 32);
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int slice = blockIdx.x;
  const int n0 = slice * nodes_per_slice;
  const int n1 = min(n_nodes, n0 + nodes_per_slice);
  const int nb = 32 / d;  // whole nodes per chunk
  float* __restrict__ xs = Xs[wave];
  float* __restrict__ gs = Gs[wave];
  eelg_f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  // pad rows [nb*d, 32) stay zero for the whole kernel
  for (int f = lane; f < (32 - nb * d) * LIN_ST; f += 64) {
    xs[nb * d * LIN_ST + f] = 0.0f;
    gs[nb * d * LIN_ST + f] = 0.0f;
  }
  const float* __restrict__ xb = x + in.x_off + (size_t)ut * 32 * d;
  const float* __restrict__ gb = g + in.g_off + (size_t)jt * 32 * d;
  // register-staged chunk: lane owns flat entries f = lane + 64 q (q < 16) of the
  // (node, channel, m) runs of <= nb whole nodes; the next chunk's loads are issued
  // before the current chunk's MFMAs
  float rx[16], rg[16];
  auto load_chunk = [&](int nc) {
    const int cn = min(nb, n1 - nc);
    Walk3 w3;
    w3.init(lane, 64, 32, d);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const bool in_node = w3.a < cn;
      rx[q] = (in_node && w3.b < uw) ? xb[(size_t)(nc + w3.a) * x_row + w3.b * d + w3.m] : 0.0f;
      rg[q] = (in_node && w3.b < jw) ? gb[(size_t)(nc + w3.a) * g_row + w3.b * d + w3.m] : 0.0f;
      w3.next(32, d);
    }
  };
  const int flat = nb * 32 * d;  // <= 1024 entries per chunk
  int nc = n0 + wave * nb;
  if (nc < n1) load_chunk(nc);
  for (; nc < n1; nc += 4 * nb) {
    {
      Walk3 w3;
      w3.init(lane, 64, 32, d);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (lane + 64 * q < flat) {
          const int row = w3.a * d + w3.m;
          xs[row * LIN_ST + w3.b] = rx[q];
          gs[row * LIN_ST + w3.b] = rg[q];
        }
        w3.next(32, d);
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (nc + 4 * nb < n1) load_chunk(nc + 4 * nb);
    const float* __restrict__ xr = xs + (lane >> 5) * LIN_ST + (lane & 31);
    const float* __restrict__ gr = gs + (lane >> 5) * LIN_ST + (lane & 31);
#pragma unroll
    for (int st = 0; st < 16; ++st)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(xr[2 * st * LIN_ST], gr[2 * st * LIN_ST], acc, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
  }
  // cross-wave reduction through LDS (reuse Xs: 4 x 32*33 >= 3 x 16*64 floats)
  __syncthreads();
  float* red = &Xs[0][0];
  if (wave > 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) red[((wave - 1) * 16 + i) * 64 + lane] = acc[i];
  }
  __syncthreads();
  if (wave == 0) {
    float* __restrict__ dst = partial + (size_t)slice * w_total + in.w_off;
    const int j = jt * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float v = acc[i] + red[i * 64 + lane] + red[(16 + i) * 64 + lane] + red[(32 + i) * 64 + lane];
      const int uu = ut * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
      if (uu < K && j < NO) dst[(size_t)uu * NO + j] = v * in.alpha;
    }
  }
}

// grad W, every instruction on the fast path (lin_bwdw_fast): same grid and partial layout as
// lin_bwdw_kernel, no register-staged transposition, so the register budget allows 4 waves/SIMD
__global__ __launch_bounds__(256) void lin_bwdw_fast_kernel(const float* __restrict__ x, int x_row,
                                                            const float* __restrict__ g, int g_row,
                                                            int n_nodes, int nodes_per_slice,
                                                            float* __restrict__ partial, int w_total,
                                                            eelg_linw_desc desc) {
  __shared__ float4 lds4[2 * 4 * 1152 / 4];   // per wave (32/D + 1) * 32 * D floats of x and g
  const eelg_linw_ins& in = desc.ins[blockIdx.y];
  const int d = in.d, K = in.k, NO = in.n_out;
  const int n_jt = NO / 32;
  // block id -> (slice, weight tile): the tiles of one node slice (which all read that slice's
  // g rows, and each its own x columns) are dispatched back to back on one XCD (id % 8)
  const int ntile = desc.max_ut * desc.max_jt;
  const int id = blockIdx.x, xcd = id & 7, rest = id >> 3;
  const int t = rest % ntile;
  const int slice = (rest / ntile) * 8 + xcd;
  if (t >= (K / 32) * n_jt) return;  // uniform per workgroup
  const int ut = t / n_jt, jt = t - ut * n_jt;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n0 = slice * nodes_per_slice;
  if (n0 >= n_nodes) return;
  const int n1 = min(n_nodes, n0 + nodes_per_slice);
  eelg_f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.0f;
  float* xw = reinterpret_cast<float*>(lds4) + wave * 2 * 1152;
  float* gwv = xw + 1152;
  switch (d) {
    case 1: lin_bwdw_fast<1>(x, x_row, g, g_row, n0, n1, in, ut, jt, xw, gwv, acc); break;
    case 3: lin_bwdw_fast<3>(x, x_row, g, g_row, n0, n1, in, ut, jt, xw, gwv, acc); break;
    case 5: lin_bwdw_fast<5>(x, x_row, g, g_row, n0, n1, in, ut, jt, xw, gwv, acc); break;
    case 7: lin_bwdw_fast<7>(x, x_row, g, g_row, n0, n1, in, ut, jt, xw, gwv, acc); break;
    default: lin_bwdw_fast<9>(x, x_row, g, g_row, n0, n1, in, ut, jt, xw, gwv, acc); break;
  }
  __syncthreads();
  float* red = reinterpret_cast<float*>(lds4);
  if (wave > 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) red[((wave - 1) * 16 + i) * 64 + lane] = acc[i];
  }
  __syncthreads();
  if (wave == 0) {
    float* __restrict__ dst = partial + (size_t)slice * w_total + in.w_off;
    const int j = jt * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float v = acc[i] + red[i * 64 + lane] + red[(16 + i) * 64 + lane] + red[(32 + i) * 64 + lane];
      const int uu = ut * 32 + (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
      dst[(size_t)uu * NO + j] = v * in.alpha;
    }
  }
}

// whether every instruction of a grad-W descriptor qualifies for lin_bwdw_fast_kernel
static bool lin_bwdw_fast_ok(const float* x, int x_row, const float* g, int g_row,
                             const eelg_linw_desc* desc) {
  if ((x_row & 3) || (g_row & 3) || (reinterpret_cast<uintptr_t>(x) & 15) ||
      (reinterpret_cast<uintptr_t>(g) & 15))
    return false;
  for (int t = 0; t < desc->n_ins; ++t) {
    const eelg_linw_ins& in = desc->ins[t];
    if (in.k % 32 || in.n_out % 32 || (in.x_off & 3) || (in.g_off & 3)) return false;
    if (in.d != 1 && in.d != 3 && in.d != 5 && in.d != 7 && in.d != 9) return false;
  }
  return true;
}

// ---------------------------------------------------------------------------------------------
// Forward / grad-x fast path (every slot: whole 32-wide K chunks and column tiles, d odd <= 9,
// 16-B aligned input rows).  A workgroup (8 waves) owns one output slot, one 32-column tile and
// LINF_GPW node groups per wave; it stages the slot's weight tile (all sources, alpha applied)
// in LDS once.  A wave owns groups of NB = floor(32/D) whole nodes and stages each 32-wide K
// chunk of their rows in the natural global layout (per node the chunk's 32*D floats, one
// contiguous run: float4 loads, ds_write_b128), with node stride SX = 32*D + pad chosen so the
// MFMA operand reads -- lane i = row (n, m) at n*SX + m + k*D -- spread over the banks
// (at most 2-way; 4-way for D = 1).  No workgroup barrier after the weight staging.
// ---------------------------------------------------------------------------------------------
#ifndef LINF_WAVES
#define LINF_WAVES 8
#endif
#ifndef LINF_GPW
#define LINF_GPW 4
#endif
#ifndef LINF_PFD
#define LINF_PFD 1             // K chunks in flight per wave (1 or 2; 2 measured no faster)
#endif
#define LINF_KMAX 320          // sum of the slot's source K held in LDS
// the fast kernel also takes partial column tiles / a partial single-source K chunk (the readout
// tail's 32 -> 16-channel linear and its grad-x: lin_fwd_kernel ~0.072 ms each, partial fast
// path 0.047 ms, kbench r09k; parity r09k / r09l incl. the 16-channel suite).  Off by default:
// no step gain (r09l alternating: off 2209.7 / 2186.0, on 2201.4 / 2120.4 graphs/s)
#ifndef LINF_PARTIAL
#define LINF_PARTIAL 0
#endif
#define LINF_XW 1152           // per-wave X region (floats) >= NB * SX for every D

template <int D>
struct LinfGeom {
  static constexpr int NB = 32 / D;
  static constexpr int SX = 32 * D + (D >= 7 ? 8 : 4);
  static constexpr int RUN4 = 8 * D;                       // float4 per node per K chunk
  static constexpr int NQ = (NB * RUN4 + 63) / 64;          // float4 loads per lane per chunk
};

// ws[k][j] = alpha * W[k][jt*32 + j] for one source: BATCH loads per thread issued before their
// LDS stores (clamped indices, guarded stores).  Rows k in [src.k, 32 ceil(src.k / 32)) and
// columns jt*32 + j >= n_out are zero (a partial K chunk / column tile)
template <int BATCH>
__device__ __forceinline__ void lin_stage_w(const float* __restrict__ w, const eelg_lin_src& src,
                                            int jt, int n_out, float* __restrict__ ws) {
  const int tot = (src.k + 31) / 32 * 32 * 32;
  for (int e0 = threadIdx.x; e0 < tot; e0 += BATCH * 64 * LINF_WAVES) {
    float v[BATCH];
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int e = min(e0 + u * 64 * LINF_WAVES, tot - 1), k = e >> 5, jj = e & 31;
      v[u] = (k < src.k && jt * 32 + jj < n_out)
                 ? w[src.w_off + (size_t)k * src.ldk + (size_t)(jt * 32 + jj) * src.ldj] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < BATCH; ++u) {
      const int e = e0 + u * 64 * LINF_WAVES;
      if (e < tot) ws[e] = v[u] * src.alpha;
    }
  }
}

// LINF_NT: the fast kernel's output stores are nontemporal: the outputs (up to 942 MB for the
// 7360-wide grad-x) are read back by a later kernel, long after any cache could hold them
#ifndef LINF_NT
#define LINF_NT 1   // r04q: 7360 -> 800 grad-x 0.328 -> 0.280 ms, step 2069 -> 2084 graphs/s (two pairs)
#endif
#if LINF_NT
typedef float linf_f4n __attribute__((ext_vector_type(4)));
#define LINF_STORE(v, p) \
  __builtin_nontemporal_store(__builtin_bit_cast(linf_f4n, (v)), reinterpret_cast<linf_f4n*>(p))
#else
#define LINF_STORE(v, p) (*(p) = (v))
#endif
template <int D, bool RES, bool PART>
__device__ __forceinline__ void lin_fwd_fast(const float* __restrict__ x, int x_row,
                                             const float* __restrict__ bias, int n_nodes,
                                             float* __restrict__ y, int y_row,
                                             const eelg_lin_slot& sl, int g_base, int g_lim,
                                             int jt, const float* __restrict__ ws,
                                             float* __restrict__ xw, const float* __restrict__ res) {
  // this wave's node groups: g_base + wave, g_base + wave + LINF_WAVES, ... < g_lim
  using G = LinfGeom<D>;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 31, hf = lane >> 5;
  int nch = 0;
  for (int s = 0; s < sl.n_src; ++s) nch += (sl.src[s].k + 31) / 32;
  // PART: a partial last column tile (n_out % 32 != 0, a multiple of 4) -- float4 per node
  // stored -- and partial K chunks; the full-tile instantiation keeps its register count
  const int jw4 = PART ? min(32, sl.n_out - jt * 32) * D / 4 : G::RUN4;
  const int my_groups = g_base + wave < g_lim ? (g_lim - g_base - wave + LINF_WAVES - 1) / LINF_WAVES : 0;
  const int nq = my_groups * nch;
  if (nq == 0) return;
  // this lane's operand row
  const bool row_ok = i < G::NB * D;
  const int abase = (i / D) * G::SX + (i % D) + hf * D;
  const int bbase = hf * 32 + i;
  const float bj = (sl.bias_off >= 0 && D == 1 && (!PART || jt * 32 + i < sl.n_out)) ? bias[sl.bias_off + jt * 32 + i] : 0.0f;
  // chunk q: node group, x offset, first weight row, and float4 per node run that hold data (a
  // partial last K chunk, k % 32 != 0, reads only its k channels: the rest are zero)
  auto chunk_of = [&](int q, int& group, int& xoff, int& kb, int& kv4) {
    const int k = q / nch;
    int c = q - k * nch;
    group = g_base + k * LINF_WAVES + wave;
    int s = 0;
    kb = 0;
    while (c >= (sl.src[s].k + 31) / 32) { c -= (sl.src[s].k + 31) / 32; kb += (sl.src[s].k + 31) / 32 * 32; ++s; }
    xoff = sl.src[s].x_off + c * 32 * D;
    kb += c * 32;
    kv4 = PART ? min(32, sl.src[s].k - c * 32) * D / 4 : G::RUN4;
  };
  auto load = [&](int q, float4* r) {
    int group, xoff, kb, kv4;
    chunk_of(q, group, xoff, kb, kv4);
    const int n0 = group * G::NB;
#pragma unroll
    for (int qq = 0; qq < G::NQ; ++qq) {
      const int f = lane + 64 * qq;
      const int a = f / G::RUN4, w4 = f - a * G::RUN4;
      const bool ok = f < G::NB * G::RUN4 && n0 + a < n_nodes && w4 < kv4;
      r[qq] = ok ? *reinterpret_cast<const float4*>(x + (size_t)(n0 + a) * x_row + xoff + 4 * w4)
                 : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  eelg_f32x16 acc;
#pragma unroll
  for (int t = 0; t < 16; ++t) acc[t] = bj;
  // one pipeline step: chunk q (registers r) to LDS, chunk q + LINF_PFD's loads into r, MFMAs
  auto step = [&](int q, float4* r) {
    int group, xoff, kb, kv4;
    chunk_of(q, group, xoff, kb, kv4);
#pragma unroll
    for (int qq = 0; qq < G::NQ; ++qq) {
      const int f = lane + 64 * qq;
      if (f < G::NB * G::RUN4) {
        const int a = f / G::RUN4, w4 = f - a * G::RUN4;
        *reinterpret_cast<float4*>(xw + a * G::SX + 4 * w4) = r[qq];
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (q + LINF_PFD < nq) load(q + LINF_PFD, r);
    const float* __restrict__ wk = ws + kb * 32 + bbase;
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const float av = xw[abase + 2 * st * D];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(row_ok ? av : 0.0f, wk[2 * st * 32], acc, 0, 0, 0);
    }
    __builtin_amdgcn_wave_barrier();
    if ((q + 1) % nch == 0) {
      // epilogue of the group: acc[t] = (row (t&3) + 8(t>>2) + 4hf, column i) goes through the
      // wave's LDS region in the output's natural layout (per node the tile's 32*D floats), then
      // out as float4 runs
      const int n0 = group * G::NB;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int row = (t & 3) + 8 * (t >> 2) + 4 * hf;
        const int n = row / D, m = row - (row / D) * D;
        if (row < G::NB * D) xw[n * G::SX + i * D + m] = acc[t];
        acc[t] = bj;
      }
      __builtin_amdgcn_wave_barrier();
      float* __restrict__ yb = y + sl.y_off + (size_t)jt * 32 * D;
      // residual (same layout as y) added in the epilogue: all of a lane's residual loads are
      // issued before its first store (clamped rows, no branch around a load)
      float4 rr[G::NQ];
      if (RES) {
        const float* __restrict__ rb = res + sl.y_off + (size_t)jt * 32 * D;
#pragma unroll
        for (int qq = 0; qq < G::NQ; ++qq) {
          const int f = min(lane + 64 * qq, G::NB * G::RUN4 - 1);
          const int a = f / G::RUN4, w4 = PART ? min(f - a * G::RUN4, jw4 - 1) : f - a * G::RUN4;
          rr[qq] = *reinterpret_cast<const float4*>(rb + (size_t)min(n0 + a, n_nodes - 1) * y_row + 4 * w4);
        }
      }
#pragma unroll
      for (int qq = 0; qq < G::NQ; ++qq) {
        const int f = lane + 64 * qq;
        const int a = f / G::RUN4, w4 = f - a * G::RUN4;
        if (f < G::NB * G::RUN4 && n0 + a < n_nodes && w4 < jw4) {
          const size_t o = (size_t)(n0 + a) * y_row + 4 * w4;
          float4 v = *reinterpret_cast<const float4*>(xw + a * G::SX + 4 * w4);
          if (RES) { v.x += rr[qq].x; v.y += rr[qq].y; v.z += rr[qq].z; v.w += rr[qq].w; }
          LINF_STORE(v, reinterpret_cast<float4*>(yb + o));
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  };
  // LINF_PFD chunks in flight per wave: register sets used round-robin (static indexing)
  float4 ra[G::NQ], rb[G::NQ];
  load(0, ra);
  if (LINF_PFD == 2 && nq > 1) load(1, rb);
  if (LINF_PFD == 2) {
    for (int q = 0; q < nq; q += 2) {
      step(q, ra);
      if (q + 1 < nq) step(q + 1, rb);
    }
  } else {
    for (int q = 0; q < nq; ++q) step(q, ra);
  }
}

template <bool RES, bool PART>
__device__ __forceinline__ void lin_fwd_fast_d(int d, const float* __restrict__ x, int x_row,
                                               const float* __restrict__ bias, int n_nodes,
                                               float* __restrict__ y, int y_row,
                                               const eelg_lin_slot& sl, int g0, int g1, int jt,
                                               const float* __restrict__ ws, float* __restrict__ xw,
                                               const float* __restrict__ res) {
  switch (d) {
    case 1: lin_fwd_fast<1, RES, PART>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, ws, xw, res); break;
    case 3: lin_fwd_fast<3, RES, PART>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, ws, xw, res); break;
    case 5: lin_fwd_fast<5, RES, PART>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, ws, xw, res); break;
    case 7: lin_fwd_fast<7, RES, PART>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, ws, xw, res); break;
    default: lin_fwd_fast<9, RES, PART>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, ws, xw, res); break;
  }
}

// RES: the residual epilogue (y = x W + res), a separate instantiation so the plain linears
// carry no residual registers
template <bool RES, bool PART>
__global__ __launch_bounds__(64 * LINF_WAVES) void lin_fwd_fast_kernel(
    const float* __restrict__ x, int x_row, const float* __restrict__ w,
    const float* __restrict__ bias, int n_nodes, float* __restrict__ y, int y_row,
    eelg_lin_desc desc, const float* __restrict__ res, int ws4) {
  // dynamic LDS: the weight tile (max over slots of the summed source K, x 32 columns) and
  // the waves' X regions; a K = 32 linear (800 -> 800, grad-x of 800 -> 7360) needs 40 KB,
  // three workgroups per CU instead of two
  extern __shared__ float4 linf_smem[];
  float* ws = reinterpret_cast<float*>(linf_smem);
  float4* xw4 = linf_smem + ws4;
  // the last slots (highest l, the most rows) are dispatched first: a shorter tail
  const eelg_lin_slot& sl = desc.slot[desc.n_slots - 1 - blockIdx.y];
  // block id -> (group block gb, column tile jt): the max_jt column-tile blocks of one group
  // block are dispatched back to back on one XCD (id % 8), so the rows they all read come
  // from HBM once and from that XCD's L2 after
  const int id = blockIdx.x, xcd = id & 7, rest = id >> 3;
  const int jt = rest % desc.max_jt, gb = (rest / desc.max_jt) * 8 + xcd;
  const int d = sl.d;
  if (jt * 32 >= sl.n_out) return;
  const int nb = 32 / d;
  const int n_groups = (n_nodes + nb - 1) / nb;
  if (gb * LINF_WAVES * LINF_GPW >= n_groups) return;   // uniform per workgroup
  // weight tile: ws[kb + k][j] = alpha_s * W_s[k][jt*32 + j] over the slot's sources
  // (a source's loads in flight together: batches of 8 per thread, or of 2 when K = 32;
  // clamped indices, guarded stores)
  int kb = 0;
  for (int s = 0; s < sl.n_src; ++s) {
    const eelg_lin_src& src = sl.src[s];
    if (src.k <= 32) lin_stage_w<2>(w, src, jt, sl.n_out, ws + kb * 32);
    else lin_stage_w<8>(w, src, jt, sl.n_out, ws + kb * 32);
    kb += (src.k + 31) / 32 * 32;
  }
  __syncthreads();
  float* xw = reinterpret_cast<float*>(xw4) + (threadIdx.x >> 6) * LINF_XW;
  const int g0 = gb * LINF_WAVES * LINF_GPW, g1 = min(n_groups, g0 + LINF_WAVES * LINF_GPW);
  lin_fwd_fast_d<RES, PART>(d, x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, ws, xw, res);
}

// one column tile per slot (the 800 -> 800 linears): an LDS floor of 64 KB (two workgroups per
// CU) measured faster than three.  Tried and removed: a column-tile loop
// for the K = 32 grad-x, and a cost-balanced resident grid for the single-tile linears.
#define LINF_LDS_1JT (64 * 1024)
// weight region (float4) and total dynamic LDS bytes of lin_fwd_fast_kernel for a descriptor
static void lin_fwd_fast_lds(const eelg_lin_desc* desc, int* ws4, size_t* bytes) {
  int kmax = 0;
  for (int s = 0; s < desc->n_slots; ++s) {
    int kt = 0;
    for (int t = 0; t < desc->slot[s].n_src; ++t) kt += (desc->slot[s].src[t].k + 31) / 32 * 32;
    kmax = kt > kmax ? kt : kmax;
  }
  *ws4 = kmax * 32 / 4;
  *bytes = (size_t)(*ws4) * 16 + (size_t)LINF_WAVES * LINF_XW * 4;
}

// partial: also slots whose n_out is a multiple of 4 but not of 32 (a partial last column tile)
// and single-source slots whose K is a multiple of 4 but not of 32 (a partial last K chunk) --
// the fp32 fast kernel handles both; the packed split-bf16 kernel does not
static bool lin_fwd_fast_ok(const float* x, int x_row, const float* y, int y_row,
                            const eelg_lin_desc* desc, bool partial = false) {
  if ((x_row & 3) || (reinterpret_cast<uintptr_t>(x) & 15) || (y_row & 3) ||
      (reinterpret_cast<uintptr_t>(y) & 15))
    return false;
  for (int s = 0; s < desc->n_slots; ++s) {
    const eelg_lin_slot& sl = desc->slot[s];
    if ((sl.n_out % (partial ? 4 : 32)) || (sl.y_off & 3) || sl.n_src == 0) return false;   // sourceless: general path writes zeros
    if (sl.d != 1 && sl.d != 3 && sl.d != 5 && sl.d != 7 && sl.d != 9) return false;
    int kt = 0;
    for (int t = 0; t < sl.n_src; ++t) {
      const bool kpart = partial && sl.n_src == 1 && sl.src[t].k % 4 == 0;
      if ((sl.src[t].k % 32 && !kpart) || (sl.src[t].x_off & 3)) return false;
      kt += (sl.src[t].k + 31) / 32 * 32;
    }
    if (kt > LINF_KMAX) return false;
  }
  return true;
}

// ---------------------------------------------------------------------------------------------
// Forward / grad-x on bf16 MFMA with fp32-accurate split operands ("x6", eelg_internal.h).
// Same eligibility as the fp32 fast path.  The weights come pre-split, alpha-scaled and in MFMA
// fragment order from eelg_linear_pack: for slot s, column tile jt, K chunk c (32 of the slot's
// summed source K), K block kb and part p, 64 uint4 pieces, piece l = (hf, j) holding
// B[k = 32c + 16kb + 8hf + t][jt*32 + j], t = 0..7.  A workgroup (LINX_WAVES = 16 waves, 4 per
// SIMD) copies its (slot, jt) block -- 6 KB per K chunk, <= 60 KB -- into LDS once; each wave
// stages the K chunks of its node groups through its LDS region in the natural layout exactly as
// the fp32 path does (one chunk in flight), reads 8 consecutive k of its row per K block, splits
// them, and runs 2 x 6 bf16 MFMAs per chunk (3/8 of the f32 MFMA time) against B fragments read
// from LDS (ds_read_b128, conflict-free).
// ---------------------------------------------------------------------------------------------
#ifndef LINX_WAVES
#define LINX_WAVES 16
#endif
#ifndef LINX_GPW
#define LINX_GPW 4   // node groups per wave (r04k kbench, every descriptor packed: 2 -> 4 takes the
                     // 800 -> 800 forward 0.058 -> 0.049 ms, the 7360 -> 800 forward 0.253 -> 0.248)
#endif
#define LINX_KMAX 320   // summed source K of a slot held in LDS (10 chunks x 6 KB)

// ONE: the slot sums a single 32-wide K chunk (K = 32: the grad-x of the 7360 -> 800 linear, the
// 800 -> 800 linears), so every group of the wave multiplies the same B tile: its 2 x 3
// fragments stay in registers instead of being re-read from LDS per group
template <int D, bool RES, bool ONE>
__device__ __forceinline__ void lin_fwd_x6(const float* __restrict__ x, int x_row,
                                           const float* __restrict__ bias, int n_nodes,
                                           float* __restrict__ y, int y_row,
                                           const eelg_lin_slot& sl, int g_base, int g_lim, int jt,
                                           const uint4* __restrict__ bs, float* __restrict__ xw,
                                           const float* __restrict__ res) {
  using G = LinfGeom<D>;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 31, hf = lane >> 5;
  int nch = 0;
  for (int s = 0; s < sl.n_src; ++s) nch += sl.src[s].k / 32;
  const int my_groups = g_base + wave < g_lim ? (g_lim - g_base - wave + LINX_WAVES - 1) / LINX_WAVES : 0;
  const int nq = my_groups * nch;
  if (nq == 0) return;
  const bool row_ok = i < G::NB * D;
  const int abase = (i / D) * G::SX + (i % D) + 8 * hf * D;
  const float bj = (sl.bias_off >= 0 && D == 1) ? bias[sl.bias_off + jt * 32 + i] : 0.0f;
  auto chunk_of = [&](int q, int& group, int& xoff, int& c) {
    const int k = q / nch;
    c = q - k * nch;
    group = g_base + k * LINX_WAVES + wave;
    int s = 0, cc = c;
    while (cc >= sl.src[s].k / 32) { cc -= sl.src[s].k / 32; ++s; }
    xoff = sl.src[s].x_off + cc * 32 * D;
  };
  auto load = [&](int q, float4* r) {
    int group, xoff, c;
    chunk_of(q, group, xoff, c);
    const int n0 = group * G::NB;
#pragma unroll
    for (int qq = 0; qq < G::NQ; ++qq) {
      const int f = lane + 64 * qq;
      const int a = f / G::RUN4, w4 = f - a * G::RUN4;
      const bool ok = f < G::NB * G::RUN4 && n0 + a < n_nodes;
      r[qq] = ok ? *reinterpret_cast<const float4*>(x + (size_t)(n0 + a) * x_row + xoff + 4 * w4)
                 : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  eelg_f32x16v acc;
#pragma unroll
  for (int t = 0; t < 16; ++t) acc[t] = bj;
  uint4 bone[2][3];
  if (ONE) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int p = 0; p < 3; ++p) bone[kb][p] = bs[(kb * 3 + p) * 64 + lane];
  }
  float4 ra[G::NQ];
  load(0, ra);
  for (int q = 0; q < nq; ++q) {
    int group, xoff, c;
    chunk_of(q, group, xoff, c);
#pragma unroll
    for (int qq = 0; qq < G::NQ; ++qq) {
      const int f = lane + 64 * qq;
      if (f < G::NB * G::RUN4) {
        const int a = f / G::RUN4, w4 = f - a * G::RUN4;
        *reinterpret_cast<float4*>(xw + a * G::SX + 4 * w4) = ra[qq];
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (q + 1 < nq) load(q + 1, ra);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      float av[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) av[t] = row_ok ? xw[abase + (16 * kb + t) * D] : 0.0f;
      uint4 ap[3], bp[3];
      eelg_split8(av, ap);
#pragma unroll
      for (int p = 0; p < 3; ++p) bp[p] = ONE ? bone[kb][p] : bs[((c * 2 + kb) * 3 + p) * 64 + lane];
      EELG_X6(acc, ap, bp);
    }
    __builtin_amdgcn_wave_barrier();
    if ((q + 1) % nch == 0) {
      // epilogue of the group: acc[t] = (row (t&3) + 8(t>>2) + 4hf, column i) through the wave's
      // LDS region in the output's natural layout, then out as float4 runs
      const int n0 = group * G::NB;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
        const int row = (t & 3) + 8 * (t >> 2) + 4 * hf;
        const int n = row / D, m = row - (row / D) * D;
        if (row < G::NB * D) xw[n * G::SX + i * D + m] = acc[t];
        acc[t] = bj;
      }
      __builtin_amdgcn_wave_barrier();
      float* __restrict__ yb = y + sl.y_off + (size_t)jt * 32 * D;
      float4 rr[G::NQ];
      if (RES) {
        const float* __restrict__ rb = res + sl.y_off + (size_t)jt * 32 * D;
#pragma unroll
        for (int qq = 0; qq < G::NQ; ++qq) {
          const int f = min(lane + 64 * qq, G::NB * G::RUN4 - 1);
          const int a = f / G::RUN4, w4 = f - a * G::RUN4;
          rr[qq] = *reinterpret_cast<const float4*>(rb + (size_t)min(n0 + a, n_nodes - 1) * y_row + 4 * w4);
        }
      }
#pragma unroll
      for (int qq = 0; qq < G::NQ; ++qq) {
        const int f = lane + 64 * qq;
        const int a = f / G::RUN4, w4 = f - a * G::RUN4;
        if (f < G::NB * G::RUN4 && n0 + a < n_nodes) {
          const size_t o = (size_t)(n0 + a) * y_row + 4 * w4;
          float4 v = *reinterpret_cast<const float4*>(xw + a * G::SX + 4 * w4);
          if (RES) { v.x += rr[qq].x; v.y += rr[qq].y; v.z += rr[qq].z; v.w += rr[qq].w; }
          *reinterpret_cast<float4*>(yb + o) = v;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
}

// packed fragment offset (uint4 pieces) of slot s: sum over earlier slots of n_out * K / 8 ... as
// n_jt * nch * (2 x 3 x 64) pieces per slot
__device__ __host__ inline int lin_pack_slot_off(const eelg_lin_desc& desc, int s) {
  int off = 0;
  for (int t = 0; t < s; ++t) {
    int ks = 0;
    for (int u = 0; u < desc.slot[t].n_src; ++u) ks += desc.slot[t].src[u].k;
    off += ((desc.slot[t].n_out + 31) / 32) * (ks / 32) * 384;
  }
  return off;
}

template <bool RES>
__global__ __launch_bounds__(64 * LINX_WAVES) void lin_fwd_x6_kernel(
    const float* __restrict__ x, int x_row, const uint4* __restrict__ pk,
    const float* __restrict__ bias, int n_nodes, float* __restrict__ y, int y_row,
    eelg_lin_desc desc, const float* __restrict__ res) {
  __shared__ uint4 bs[LINX_KMAX / 32 * 384];            // this (slot, jt)'s B fragments, 60 KB
  __shared__ float4 xw4[LINX_WAVES * LINF_XW / 4];
  const int sidx = desc.n_slots - 1 - blockIdx.y;   // highest l (most rows) first
  const eelg_lin_slot& sl = desc.slot[sidx];
  // block id -> (group block gb, column tile jt): the max_jt column-tile blocks of one group
  // block run back to back on one XCD (id % 8), so the rows they all read come from HBM once
  const int id = blockIdx.x, xcd = id & 7, rest = id >> 3;
  const int jt = rest % desc.max_jt, gb = (rest / desc.max_jt) * 8 + xcd;
  const int d = sl.d;
  if (jt * 32 >= sl.n_out) return;
  const int nb = 32 / d;
  const int n_groups = (n_nodes + nb - 1) / nb;
  if (gb * LINX_WAVES * LINX_GPW >= n_groups) return;   // uniform per workgroup
  int nch = 0;
  for (int s = 0; s < sl.n_src; ++s) nch += sl.src[s].k / 32;
  {
    // the (slot, jt) block of B fragments: one contiguous run of nch x 384 pieces, all of a
    // thread's loads issued before its LDS stores
    const uint4* __restrict__ src = pk + lin_pack_slot_off(desc, sidx) + (size_t)jt * nch * 384;
    const int tot = nch * 384;
    constexpr int BT = (LINX_KMAX / 32 * 384 + 64 * LINX_WAVES - 1) / (64 * LINX_WAVES);
    uint4 v[BT];
#pragma unroll
    for (int u = 0; u < BT; ++u) {
      const int e = threadIdx.x + u * 64 * LINX_WAVES;
      v[u] = src[min(e, tot - 1)];
    }
#pragma unroll
    for (int u = 0; u < BT; ++u) {
      const int e = threadIdx.x + u * 64 * LINX_WAVES;
      if (e < tot) bs[e] = v[u];
    }
  }
  __syncthreads();
  float* xw = reinterpret_cast<float*>(xw4) + (threadIdx.x >> 6) * LINF_XW;
  const int g0 = gb * LINX_WAVES * LINX_GPW, g1 = min(n_groups, g0 + LINX_WAVES * LINX_GPW);
  const bool one = nch == 1;
  switch (d) {
    case 1: if (one) lin_fwd_x6<1, RES, true>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, bs, xw, res);
            else lin_fwd_x6<1, RES, false>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, bs, xw, res);
            break;
    case 3: if (one) lin_fwd_x6<3, RES, true>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, bs, xw, res);
            else lin_fwd_x6<3, RES, false>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, bs, xw, res);
            break;
    case 5: if (one) lin_fwd_x6<5, RES, true>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, bs, xw, res);
            else lin_fwd_x6<5, RES, false>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, bs, xw, res);
            break;
    case 7: if (one) lin_fwd_x6<7, RES, true>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, bs, xw, res);
            else lin_fwd_x6<7, RES, false>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, bs, xw, res);
            break;
    default: if (one) lin_fwd_x6<9, RES, true>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, bs, xw, res);
             else lin_fwd_x6<9, RES, false>(x, x_row, bias, n_nodes, y, y_row, sl, g0, g1, jt, bs, xw, res);
             break;
  }
}

// the weights in fragment order (eelg_linear_pack): one thread per (slot, jt, chunk, kb, lane)
// builds the 8 weights B[k = 32c + 16kb + 8hf + t][jt*32 + j] (alpha applied, zero past n_out)
// and writes their three bf16 parts
__global__ __launch_bounds__(256) void lin_pack_kernel(const float* __restrict__ w, eelg_lin_desc desc,
                                                       int nunits, uint4* __restrict__ pk) {
  const int u = blockIdx.x * 256 + threadIdx.x;   // unit = (slot, jt, c, kb, lane): 3 pieces each
  if (u >= nunits) return;
  int s = 0, base = 0, ks = 0, njt = 0;
  for (;; ++s) {
    ks = 0;
    for (int t = 0; t < desc.slot[s].n_src; ++t) ks += desc.slot[s].src[t].k;
    njt = (desc.slot[s].n_out + 31) / 32;
    const int nu = njt * (ks / 32) * 128;
    if (u < base + nu || s + 1 >= desc.n_slots) break;
    base += nu;
  }
  const eelg_lin_slot& sl = desc.slot[s];
  const int nch = ks / 32;
  int r = u - base;
  const int lane = r & 63; r >>= 6;
  const int kb = r & 1; r >>= 1;
  const int c = r % nch, jt = r / nch;
  const int j = jt * 32 + (lane & 31), k0 = 32 * c + 16 * kb + 8 * (lane >> 5);
  float v[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    int k = k0 + t, q = 0;
    while (k >= sl.src[q].k) { k -= sl.src[q].k; ++q; }
    const eelg_lin_src& src = sl.src[q];
    v[t] = j < sl.n_out ? src.alpha * w[src.w_off + (size_t)k * src.ldk + (size_t)j * src.ldj] : 0.0f;
  }
  uint4 p[3];
  eelg_split8(v, p);
  // a K block holds its 3 parts x 64 pieces: the same order lin_fwd_x6 reads
  const size_t o = (size_t)lin_pack_slot_off(desc, s) + ((size_t)(jt * nch + c) * 2 + kb) * 192 + lane;
#pragma unroll
  for (int q = 0; q < 3; ++q) pk[o + q * 64] = p[q];
}

// ---------------------------------------------------------------------------------------------
// Dense weight gradient on bf16 MFMA with fp32-accurate split operands (round 5):
//   part[s, j, k] = sum over split s's rows r of g[r, j] * x[r, k]
// = the torch-layout grad W = g^T x of a Linear y = x W^T (summed over s by eelg_sum_rows).
// Both operands are data and are split per element on the fly (eelg_split8).  A wave owns 32
// output rows j: A[j][r] = g[r][j], 16 values per lane per 32-row tile, coalesced over j.  The
// tile's x rows [32 x 32 NT] are split once per workgroup into LDS in B-fragment order, shared
// by the 4 waves and double buffered (the barrier of tile t separates tile t-2's reads of a
// buffer from its rewrite).  K = rows, two K = 16 blocks per tile; hi / lo accumulators
// (EELG_X6HL).  For the CGC projections (n_out 256, k 128, 262k rows) the fp32 grad-W kernel
// runs at the fp32 MFMA peak; this form does a K = 16 block in 3/8 of its MFMA cycles.
// ---------------------------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void lin_bwdw_x6_kernel(const float* __restrict__ g, int ldg,
                                                          const float* __restrict__ x, int ldx,
                                                          int n_rows, int n_out,
                                                          int tiles_per_split,
                                                          float* __restrict__ part) {
  constexpr int NFR = NT * 2 * 64;              // B fragments per part: ((ct, kb), hf, column)
  constexpr int FPT = (NFR + 255) / 256;        // fragments each thread builds
  constexpr int K = NT * 32;
  __shared__ uint4 xs[2][3 * NFR];
  const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, i = l & 31, hf = l >> 5;
  const int j = blockIdx.x * 128 + wave * 32 + i;
  const int s = blockIdx.y;
  const int ntile = (n_rows + 31) >> 5;
  const int t0 = s * tiles_per_split, t1 = min(ntile, t0 + tiles_per_split);
  eelg_f32x16v acc[NT], lo[NT];
#pragma unroll
  for (int ct = 0; ct < NT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[ct][r] = lo[ct][r] = 0.0f;
  float an[16], xn[FPT][8];
  auto load = [&](int t) {
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = t * 32 + 16 * kb + 8 * hf + u;
        an[8 * kb + u] = (r < n_rows && j < n_out) ? g[(size_t)r * ldg + j] : 0.0f;
      }
#pragma unroll
    for (int f = 0; f < FPT; ++f) {
      const int fi = threadIdx.x + 256 * f;
      const int bk = fi & 31, bh = (fi >> 5) & 1, bkb = (fi >> 6) & 1, bct = fi >> 7;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = t * 32 + 16 * bkb + 8 * bh + u;
        xn[f][u] = (fi < NFR && r < n_rows) ? x[(size_t)r * ldx + bct * 32 + bk] : 0.0f;
      }
    }
  };
  if (t0 < t1) load(t0);
  for (int t = t0; t < t1; ++t) {
    uint4* __restrict__ hb = xs[t & 1];
#pragma unroll
    for (int f = 0; f < FPT; ++f) {
      const int fi = threadIdx.x + 256 * f;
      if (fi < NFR) {
        uint4 pp[3];
        eelg_split8(xn[f], pp);
#pragma unroll
        for (int p = 0; p < 3; ++p) hb[p * NFR + fi] = pp[p];
      }
    }
    __syncthreads();
    uint4 ap[2][3];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) eelg_split8(&an[8 * kb], ap[kb]);
    if (t + 1 < t1) load(t + 1);   // in flight during the MFMAs
    const uint4* __restrict__ bb = hb + hf * 32 + i;
#pragma unroll
    for (int ct = 0; ct < NT; ++ct)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        uint4 b[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) b[p] = bb[p * NFR + (ct * 2 + kb) * 64];
        EELG_X6HL(acc[ct], lo[ct], ap[kb], b);
      }
  }
  const int jb = blockIdx.x * 128 + wave * 32;
#pragma unroll
  for (int ct = 0; ct < NT; ++ct)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jj = jb + (r & 3) + 8 * (r >> 2) + 4 * hf;
      if (jj < n_out) part[((size_t)s * n_out + jj) * K + ct * 32 + i] = acc[ct][r] + lo[ct][r];
    }
}
