// C ABI of the EnergyEquivGNN hot path (declared in include/eelg.h) plus the
// hand-written kernels: edge embedding and the CSR segmented sum.  The
// irreps-specialised tensor-product and symmetric-contraction kernels are
// generated into generated/eelg_gen.hip (see gen_kernels.py) and compiled in
// this same translation unit.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>
#include <vector>

#include "../../include/eelg.h"
#include "eelg_internal.h"
#include "generated/eelg_gen.hip"
#include "eelg_linear.hip"
#include "eelg_cgc.hip"

#define EELG_VERSION "eelg 0.1.0 gfx950"

static thread_local char g_err[512] = "";

int eelg_fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int eelg_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return eelg_fail(-3, "%s: launch failed: %s", what, hipGetErrorString(e));
  return 0;
}

#define fail eelg_fail
#define check_launch eelg_check_launch

// ---------------------------------------------------------------------------
// edge embedding: one thread per edge
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void edge_embed_kernel(
    const float* __restrict__ pos, const int* __restrict__ sender, const int* __restrict__ receiver,
    const float* __restrict__ shifts, const float* __restrict__ radius, int n_edges, int lmax,
    int nb, float len_end, float rad_end, float* __restrict__ sh, float* __restrict__ feats) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_edges) return;
  const int s = sender[e], r = receiver[e];
  const float vx = pos[3 * r + 0] - pos[3 * s + 0] + shifts[3 * e + 0];
  const float vy = pos[3 * r + 1] - pos[3 * s + 1] + shifts[3 * e + 1];
  const float vz = pos[3 * r + 2] - pos[3 * s + 2] + shifts[3 * e + 2];
  const float len = sqrtf(vx * vx + vy * vy + vz * vz);
  const int nsh = (lmax + 1) * (lmax + 1);
  const int nshp = (nsh + 3) & ~3;   // rows padded to 16 B: the TP kernels read them as float4
  float* __restrict__ she = sh + (size_t)e * nshp;
  switch (lmax) {
    case 1: sh_eval_l1(vx, vy, vz, she); break;
    case 2: sh_eval_l2(vx, vy, vz, she); break;
    case 3: sh_eval_l3(vx, vy, vz, she); break;
    default: sh_eval_l4(vx, vy, vz, she); break;
  }
  for (int j = nsh; j < nshp; ++j) she[j] = 0.0f;
  // soft_one_hot_linspace(x, 0, end, nb, 'gaussian', cutoff=False):
  // values = linspace(0, end, nb); step = values[1]-values[0]; exp(-((x-v)/step)^2)/1.12
  const float rad = radius[e];
  const float lstep = len_end / (float)(nb - 1);
  const float rstep = rad_end / (float)(nb - 1);
  float* __restrict__ f = feats + (size_t)e * 2 * nb;
  for (int k = 0; k < nb; ++k) {
    const float vl = (k == nb - 1) ? len_end : lstep * (float)k;
    const float vr = (k == nb - 1) ? rad_end : rstep * (float)k;
    const float dl = (len - vl) / lstep;
    const float dr = (rad - vr) / rstep;
    f[k] = expf(-dl * dl) / 1.12f;
    f[nb + k] = expf(-dr * dr) / 1.12f;
  }
}

// ---------------------------------------------------------------------------
// CSR segmented sum: one wave per output row, float4 over the row when aligned
// ---------------------------------------------------------------------------
// bf16 source rows (bit patterns, BASELINE config 5's edge-sized gradients) are widened
// exactly to fp32 before the fp32 accumulation.
__device__ __forceinline__ float4 seg_load4(const float* __restrict__ row, int c) {
  return reinterpret_cast<const float4*>(row)[c];
}
__device__ __forceinline__ float4 seg_load4(const unsigned short* __restrict__ row, int c) {
  const uint2 v = reinterpret_cast<const uint2*>(row)[c];
  return make_float4(__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u),
                     __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u));
}
__device__ __forceinline__ float seg_load1(const float* __restrict__ p) { return *p; }
__device__ __forceinline__ float seg_load1(const unsigned short* __restrict__ p) { return eelg_bf2f(*p); }

#ifndef SEG_EB
#define SEG_EB 4     // source rows per batch of loads
#endif
// SEG_KMAX (template): float4 columns per lane, 1..4 (rows up to 1024 floats take the batched
// path); 0 = the column loop
template <bool VEC4, typename T, int SEG_KMAX = 0>
__global__ __launch_bounds__(256) void segment_sum_kernel(
    const T* __restrict__ src, const int* __restrict__ rowptr, const int* __restrict__ idx,
    const float* __restrict__ row_scale, float scale, int n_rows, int width,
    float* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= n_rows) return;
  const int beg = rowptr[row], end = rowptr[row + 1];
  const float sc = scale * (row_scale ? row_scale[row] : 1.0f);
  float* __restrict__ o = out + (size_t)row * width;
  if (VEC4 && SEG_KMAX > 0) {
    // rows up to 64 * SEG_KMAX float4: a lane's SEG_KMAX columns of SEG_EB source rows are
    // loaded at once (row indices first, then every column load), so up to SEG_EB * SEG_KMAX
    // loads per lane are in flight instead of one dependent round trip per (column, row);
    // the sums keep the row order, so results are bitwise those of the loop below
    const int w4 = width >> 2;
    constexpr int KM = SEG_KMAX > 0 ? SEG_KMAX : 1;
    float4 acc[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int j0 = beg; j0 < end; j0 += SEG_EB) {
      int sr[SEG_EB];
#pragma unroll
      for (int q = 0; q < SEG_EB; ++q) {
        const int j = min(j0 + q, end - 1);
        sr[q] = idx ? idx[j] : j;
      }
      float4 v[SEG_EB][KM];
#pragma unroll
      for (int q = 0; q < SEG_EB; ++q)
#pragma unroll
        for (int k = 0; k < KM; ++k) {
          const int c = min(lane + 64 * k, w4 - 1);
          v[q][k] = seg_load4(src + (size_t)sr[q] * width, c);
        }
#pragma unroll
      for (int q = 0; q < SEG_EB; ++q)
        if (j0 + q < end)
#pragma unroll
          for (int k = 0; k < KM; ++k) {
            acc[k].x += v[q][k].x; acc[k].y += v[q][k].y; acc[k].z += v[q][k].z; acc[k].w += v[q][k].w;
          }
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int c = lane + 64 * k;
      if (c < w4) {
        float4 a = acc[k];
        a.x *= sc; a.y *= sc; a.z *= sc; a.w *= sc;
        reinterpret_cast<float4*>(o)[c] = a;
      }
    }
  } else if (VEC4) {
    const int w4 = width >> 2;
    for (int c = lane; c < w4; c += 64) {
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int j = beg; j < end; ++j) {
        const int sr = idx ? idx[j] : j;
        const float4 v = seg_load4(src + (size_t)sr * width, c);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      acc.x *= sc; acc.y *= sc; acc.z *= sc; acc.w *= sc;
      reinterpret_cast<float4*>(o)[c] = acc;
    }
  } else {
    for (int c = lane; c < width; c += 64) {
      float acc = 0.f;
      for (int j = beg; j < end; ++j) {
        const int sr = idx ? idx[j] : j;
        acc += seg_load1(src + (size_t)sr * width + c);
      }
      o[c] = acc * sc;
    }
  }
}

// ---------------------------------------------------------------------------
// Gate nonlinearity (readout): elementwise, one thread per output (fwd) / input (bwd) element
// of a row, rows split over the grid; the gated block of an element is found by a walk over
// the <= EELG_GATE_MAXBLK block offsets
// ---------------------------------------------------------------------------
__device__ __forceinline__ float gate_sig(float v) { return __frcp_rn(1.0f + __expf(-v)); }
__device__ __forceinline__ float gate_silu(float v) { return v * gate_sig(v); }
__device__ __forceinline__ float gate_dsilu(float v) {
  const float s = gate_sig(v);
  return s * (1.0f + v * (1.0f - s));
}
#define EELG_GATE_ROWBUF EELG_GATE_MAXGATED
#define GATE_ROWS 4               // rows per workgroup (the lookup tables are built once per workgroup)

// per-workgroup lookup tables: gated element -> its gate; gate -> first element of its run, d
__device__ __forceinline__ void gate_tables(const eelg_gate_desc& g, unsigned short* tab,
                                            unsigned short* r0s, unsigned char* ds) {
  int off = 0, goff = 0;
  for (int b = 0; b < g.n_blk; ++b) {
    const int mul = g.blk_mul[b], d = g.blk_dim[b];
    for (int e = threadIdx.x; e < mul * d; e += 256) tab[off + e] = (unsigned short)(goff + e / d);
    for (int u = threadIdx.x; u < mul; u += 256) {
      r0s[goff + u] = (unsigned short)(off + u * d);
      ds[goff + u] = (unsigned char)d;
    }
    off += mul * d;
    goff += mul;
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void gate_fwd_kernel(const float* __restrict__ x, int n_nodes,
                                                       eelg_gate_desc g, int din, int dout,
                                                       float cst, float* __restrict__ y) {
  __shared__ unsigned short tab[EELG_GATE_MAXGATED], r0s[EELG_GATE_MAXGATES];
  __shared__ unsigned char ds[EELG_GATE_MAXGATES];
  gate_tables(g, tab, r0s, ds);
  const int n1 = min(n_nodes, (int)(blockIdx.x + 1) * GATE_ROWS);
  for (int n = blockIdx.x * GATE_ROWS; n < n1; ++n) {
    const float* __restrict__ xr = x + (size_t)n * din;
    float* __restrict__ yr = y + (size_t)n * dout;
    for (int j = threadIdx.x; j < dout; j += 256) {
      if (j < g.n_scal) {
        yr[j] = cst * gate_silu(xr[j]);
      } else {
        const int jj = j - g.n_scal;
        yr[j] = xr[g.n_scal + g.n_gates + jj] * (cst * gate_silu(xr[g.n_scal + tab[jj]]));
      }
    }
  }
}

__global__ __launch_bounds__(256) void gate_bwd_kernel(const float* __restrict__ x,
                                                       const float* __restrict__ gy, int n_nodes,
                                                       eelg_gate_desc g, int din, int dout,
                                                       float cst, float* __restrict__ gx) {
  __shared__ unsigned short tab[EELG_GATE_MAXGATED], r0s[EELG_GATE_MAXGATES];
  __shared__ unsigned char ds[EELG_GATE_MAXGATES];
  __shared__ float prod[EELG_GATE_ROWBUF];   // grad_y * x of the gated elements of one row
  gate_tables(g, tab, r0s, ds);
  const int gated0 = g.n_scal + g.n_gates, glen = dout - g.n_scal;
  const int n1 = min(n_nodes, (int)(blockIdx.x + 1) * GATE_ROWS);
  for (int n = blockIdx.x * GATE_ROWS; n < n1; ++n) {
    const float* __restrict__ xr = x + (size_t)n * din;
    const float* __restrict__ gr = gy + (size_t)n * dout;
    float* __restrict__ o = gx + (size_t)n * din;
    // pass 1 (coalesced): scalars, gated elements, and the products the gates sum
    for (int i = threadIdx.x; i < g.n_scal; i += 256) o[i] = gr[i] * cst * gate_dsilu(xr[i]);
    for (int jj = threadIdx.x; jj < glen; jj += 256) {
      const float gyv = gr[g.n_scal + jj], xv = xr[gated0 + jj];
      prod[jj] = gyv * xv;
      o[gated0 + jj] = gyv * (cst * gate_silu(xr[g.n_scal + tab[jj]]));
    }
    __syncthreads();
    // pass 2: each gate sums its run of products from LDS
    for (int gi = threadIdx.x; gi < g.n_gates; gi += 256) {
      const int r0 = r0s[gi], d = ds[gi];
      float s = 0.0f;
      for (int m = 0; m < d; ++m) s += prod[r0 + m];
      o[g.n_scal + gi] = s * cst * gate_dsilu(xr[g.n_scal + gi]);
    }
    __syncthreads();   // prod is rewritten by the next row
  }
}

static int gate_check(const eelg_gate_desc* g, int* din, int* dout) {
  if (!g || g->n_scal < 0 || g->n_blk < 0 || g->n_blk > EELG_GATE_MAXBLK)
    return fail(-2, "gate: bad descriptor");
  int gates = 0, len = 0;
  for (int b = 0; b < g->n_blk; ++b) {
    if (g->blk_mul[b] <= 0 || g->blk_dim[b] <= 0) return fail(-2, "gate: bad gated block %d", b);
    gates += g->blk_mul[b];
    len += g->blk_mul[b] * g->blk_dim[b];
  }
  if (gates != g->n_gates) return fail(-2, "gate: %d gates for %d gated channels", g->n_gates, gates);
  if (len > EELG_GATE_MAXGATED || gates > EELG_GATE_MAXGATES)
    return fail(-2, "gate: %d gated elements / %d gates exceed the built tables (%d / %d)", len,
                gates, EELG_GATE_MAXGATED, EELG_GATE_MAXGATES);
  *din = g->n_scal + g->n_gates + len;
  *dout = g->n_scal + len;
  return 0;
}

static int gate_grid(int n_nodes) { return (n_nodes + GATE_ROWS - 1) / GATE_ROWS; }

// Few long segments (graph pooling: 32 graphs x 1024 nodes): split each segment into
// n_split contiguous pieces, one wave per (segment, piece) -> work[seg][piece][:], then
// a fixed-order combine.  Deterministic, no atomics.
__global__ __launch_bounds__(256) void segment_split_kernel(
    const float* __restrict__ src, const int* __restrict__ rowptr, const int* __restrict__ idx,
    int n_rows, int width, int n_split, float* __restrict__ work) {
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (wid >= n_rows * n_split) return;
  const int row = wid / n_split, sp = wid - row * n_split;
  const int b0 = rowptr[row], len = rowptr[row + 1] - b0;
  const int beg = b0 + (int)(((long long)len * sp) / n_split);
  const int end = b0 + (int)(((long long)len * (sp + 1)) / n_split);
  float* __restrict__ o = work + (size_t)wid * width;
  for (int c = lane; c < width; c += 64) {
    float acc = 0.f;
    for (int j = beg; j < end; ++j) {
      const int sr = idx ? idx[j] : j;
      acc += src[(size_t)sr * width + c];
    }
    o[c] = acc;
  }
}

__global__ __launch_bounds__(256) void segment_combine_kernel(
    const float* __restrict__ work, const float* __restrict__ row_scale, float scale, int n_rows,
    int width, int n_split, float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n_rows * width) return;
  const int row = i / width, c = i - row * width;
  const float* __restrict__ w = work + (size_t)row * n_split * width + c;
  float acc = 0.f;
  for (int s = 0; s < n_split; ++s) acc += w[(size_t)s * width];
  out[i] = acc * scale * (row_scale ? row_scale[row] : 1.0f);
}

// torch_scatter's order reductions over CSR segments (reduce = max / min / mul): one thread
// per (row, column), columns fastest (coalesced rows).  max / min keep the FIRST extreme of
// the segment (strict compare) and its position, so the backward routes the whole gradient
// to that one element as torch_scatter's scatter_max / scatter_min do; rows with no entries
// give 0 (max / min) or 1 (mul) and position -1.
enum { SEG_MAX = 0, SEG_MIN = 1, SEG_MUL = 2 };

__global__ __launch_bounds__(256) void segment_order_kernel(
    const float* __restrict__ src, const int* __restrict__ rowptr, int n_rows, int width, int op,
    float* __restrict__ out, int* __restrict__ arg) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)n_rows * width) return;
  const int row = (int)(i / width), c = (int)(i - (long long)row * width);
  const int beg = rowptr[row], end = rowptr[row + 1];
  if (op == SEG_MUL) {
    float p = 1.0f;
    for (int j = beg; j < end; ++j) p *= src[(size_t)j * width + c];
    out[i] = p;
    return;
  }
  float best = 0.0f;
  int at = -1;
  for (int j = beg; j < end; ++j) {
    const float v = src[(size_t)j * width + c];
    if (at < 0 || (op == SEG_MAX ? v > best : v < best)) { best = v; at = j; }
  }
  out[i] = best;
  if (arg) arg[i] = at;
}

// backward: every source row of a segment gets its gradient (no zero-fill needed when the
// segments cover the rows): max / min -> g at the kept position, 0 elsewhere; mul -> g times
// the product of the segment's other entries (exact with zeros: counted, not divided by)
__global__ __launch_bounds__(256) void segment_order_bwd_kernel(
    const float* __restrict__ src, const int* __restrict__ rowptr, const int* __restrict__ arg,
    const float* __restrict__ g, int n_rows, int width, int op, float* __restrict__ gsrc) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long long)n_rows * width) return;
  const int row = (int)(i / width), c = (int)(i - (long long)row * width);
  const int beg = rowptr[row], end = rowptr[row + 1];
  const float gi = g[i];
  if (op != SEG_MUL) {
    const int at = arg[i];
    for (int j = beg; j < end; ++j) gsrc[(size_t)j * width + c] = j == at ? gi : 0.0f;
    return;
  }
  // product of the others = (product before j) * (product after j): a reverse pass leaves the
  // suffix products in gsrc, a forward pass multiplies in the prefix (no division, so zeros
  // are exact)
  float s = 1.0f;
  for (int j = end - 1; j >= beg; --j) {
    gsrc[(size_t)j * width + c] = s;
    s *= src[(size_t)j * width + c];
  }
  float p = 1.0f;
  for (int j = beg; j < end; ++j) {
    gsrc[(size_t)j * width + c] = gi * (p * gsrc[(size_t)j * width + c]);
    p *= src[(size_t)j * width + c];
  }
}

// Sparse (CSR) x dense with strided operands: out[r, c] = sum_j val[j] * B[col[j], c].
// Four lanes per (r, c) (c fastest across lane quads) split a row's nonzeros and are
// combined with two xor-shuffles in a fixed order, so long rows (U_sym^T: ~120 nnz) do
// not serialise one dependent chain.
__global__ __launch_bounds__(256) void csr_spmm_kernel(
    const int* __restrict__ rowptr, const int* __restrict__ col, const float* __restrict__ val,
    int n_rows, const float* __restrict__ B, int ldb_r, int ldb_c, int n_cols,
    float* __restrict__ out, int ldo_r, int ldo_c) {
  const int gi = blockIdx.x * 256 + threadIdx.x;
  const int sub = gi & 3, i = gi >> 2;
  const bool ok = i < n_rows * n_cols;
  const int r = ok ? i / n_cols : 0, c = ok ? i - r * n_cols : 0;
  float acc = 0.f;
  if (ok)
    for (int j = rowptr[r] + sub; j < rowptr[r + 1]; j += 4)
      acc = fmaf(val[j], B[(size_t)col[j] * ldb_r + (size_t)c * ldb_c], acc);
  acc += __shfl_xor(acc, 1);
  acc += __shfl_xor(acc, 2);
  if (ok && sub == 0) out[(size_t)r * ldo_r + (size_t)c * ldo_c] = acc;
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------
template <typename T>
static int segment_sum_launch(const T* src, const int* rowptr, const int* idx,
                              const float* row_scale, float scale, int n_rows, int width,
                              float* out, void* stream, const char* what) {
  if (n_rows <= 0 || width <= 0) return 0;
  dim3 grid((n_rows + 3) / 4);
  const bool vec = (width % 4 == 0) && ((uintptr_t)src % (4 * sizeof(T)) == 0) &&
                   ((uintptr_t)out % 16 == 0);
  const int km = vec ? (width / 4 + 63) / 64 : 0;
#define SEG_LAUNCH(K) hipLaunchKernelGGL((segment_sum_kernel<true, T, K>), grid, dim3(256), 0, \
                                         (hipStream_t)stream, src, rowptr, idx, row_scale, scale, \
                                         n_rows, width, out)
  if (vec && km == 1) SEG_LAUNCH(1);
  else if (vec && km == 2) SEG_LAUNCH(2);
  else if (vec && km == 3) SEG_LAUNCH(3);
  else if (vec && km == 4) SEG_LAUNCH(4);
#undef SEG_LAUNCH
  else if (vec)
    hipLaunchKernelGGL((segment_sum_kernel<true, T>), grid, dim3(256), 0, (hipStream_t)stream, src,
                       rowptr, idx, row_scale, scale, n_rows, width, out);
  else
    hipLaunchKernelGGL((segment_sum_kernel<false, T>), grid, dim3(256), 0, (hipStream_t)stream, src,
                       rowptr, idx, row_scale, scale, n_rows, width, out);
  return check_launch(what);
}

const eelg_tp_cfg* eelg_tp_table(int* n) {
  // the per-mul tables concatenated once (thread-safe static initialisation)
  static const std::vector<eelg_tp_cfg> all = [] {
    std::vector<eelg_tp_cfg> v;
    for (auto get : {eelg_tp_table_m32, eelg_tp_table_m16, eelg_tp_table_m64}) {
      int k = 0;
      const eelg_tp_cfg* t = get(&k);
      v.insert(v.end(), t, t + k);
    }
    return v;
  }();
  *n = (int)all.size();
  return all.data();
}

const eelg_sc_cfg* eelg_sc_table(int* n) { return eelg_sc_table_m32(n); }

const eelg_sc_cfg* eelg_sc_table_mul(int mul, int* n) {
  switch (mul) {
    case 16: return eelg_sc_table_m16(n);
    case 32: return eelg_sc_table_m32(n);
    case 64: return eelg_sc_table_m64(n);
    default: *n = 0; return nullptr;
  }
}

extern "C" {

const char* eelg_version(void) { return EELG_VERSION; }
const char* eelg_last_error(void) { return g_err; }

int eelg_tp_find(const char* name) {
  int n = 0;
  const eelg_tp_cfg* t = eelg_tp_table(&n);
  for (int i = 0; i < n; ++i)
    if (strcmp(t[i].name, name) == 0) return i;
  return fail(-1, "unknown tensor-product config '%s'", name);
}

int eelg_tp_info(int cfg, int* info, uint64_t* sig) {
  int n = 0;
  const eelg_tp_cfg* t = eelg_tp_table(&n);
  if (cfg < 0 || cfg >= n) return fail(-1, "bad tp config %d", cfg);
  const eelg_tp_cfg& c = t[cfg];
  info[0] = c.din; info[1] = c.dmid; info[2] = c.wn; info[3] = c.nsh;
  info[4] = c.ngroups; info[5] = c.npaths; info[6] = c.lmax;
  *sig = c.sig;
  return 0;
}

int eelg_sc_find(const char* name) {
  int n = 0;
  const eelg_sc_cfg* t = eelg_sc_table(&n);
  for (int i = 0; i < n; ++i)
    if (strcmp(t[i].name, name) == 0) return i;
  return fail(-1, "unknown symmetric-contraction config '%s'", name);
}

int eelg_sc_info(int cfg, int* info, uint64_t* sig) {
  int n = 0;
  const eelg_sc_cfg* t = eelg_sc_table(&n);
  if (cfg < 0 || cfg >= n) return fail(-1, "bad sc config %d", cfg);
  const eelg_sc_cfg& c = t[cfg];
  info[0] = c.D; info[1] = c.drow; info[2] = c.orow; info[3] = c.nterms; info[4] = c.njg;
  info[5] = c.Dout; info[6] = c.nbc; info[7] = c.cld;
  *sig = c.sig;
  return 0;
}

int eelg_edge_embed(const float* pos, const int* sender, const int* receiver, const float* shifts,
                    const float* radius, int n_edges, int lmax, int nb, float len_end,
                    float rad_end, float* sh, float* feats, void* stream) {
  if (lmax < 1 || lmax > 4) return fail(-2, "edge_embed: lmax %d not built (1..4)", lmax);
  if (nb < 2) return fail(-2, "edge_embed: need >= 2 bases, got %d", nb);
  if (n_edges <= 0) return 0;
  hipLaunchKernelGGL(edge_embed_kernel, dim3((n_edges + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, pos, sender, receiver, shifts, radius, n_edges, lmax, nb,
                     len_end, rad_end, sh, feats);
  return check_launch("edge_embed");
}

static const eelg_tp_cfg* tp_cfg(int cfg) {
  int n = 0;
  const eelg_tp_cfg* t = eelg_tp_table(&n);
  if (cfg < 0 || cfg >= n) {
    fail(-1, "bad tp config %d", cfg);
    return nullptr;
  }
  return &t[cfg];
}

// node tiles of 2 * fwpb * nph receivers (fwpb waves x 2 half-waves); the tile count is rounded
// up to a multiple of 8 so every tile's ngroups blocks land on one XCD, which takes a contiguous
// range of tiles (see gen_kernels.py); surplus blocks exit
static dim3 tp_fwd_grid(const eelg_tp_cfg& c, int n_nodes, bool bf = false) {
  const int tn = 2 * c.fwpb * c.nph;
  const int tiles = (n_nodes + tn - 1) / tn;
  return dim3(((tiles + 7) / 8) * 8 * (bf ? c.ngroups_bf : c.ngroups));
}

int eelg_tp_fwd(int cfg, const float* x, const float* sh, const float* w, const int* sender,
                const int* rowptr, int n_nodes, float inv_norm, float* agg, void* stream) {
  const eelg_tp_cfg* c = tp_cfg(cfg);
  if (!c) return -1;
  if (n_nodes <= 0) return 0;
  // the fp32 kernel moves x / SH / weight rows by LDS-DMA in 16-B pieces (every row length is a
  // multiple of 16 B, so aligned bases keep every piece aligned)
  if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(sh) |
        reinterpret_cast<uintptr_t>(w)) & 15) != 0)
    return fail(-2, "tp_fwd: x, sh and w must be 16-byte aligned");
  hipLaunchKernelGGL(c->fwd, tp_fwd_grid(*c, n_nodes), dim3(64 * c->fwpb), 0, (hipStream_t)stream, x,
                     sh, w, sender, rowptr, n_nodes, inv_norm, agg);
  return check_launch("tp_fwd");
}

int eelg_tp_fwd_bf16(int cfg, const float* x, const float* sh, const void* w, const int* sender,
                     const int* rowptr, int n_nodes, float inv_norm, float* agg, void* stream) {
  const eelg_tp_cfg* c = tp_cfg(cfg);
  if (!c) return -1;
  if (!c->fwd_bf) return fail(-2, "tp_fwd_bf16: bf16 storage is generated for mul 32 only (config %s)", c->name);
  if (n_nodes <= 0) return 0;
  // LDS-DMA pieces of 16 B, as the fp32 kernel (bf16 weight rows are wn * 2 B, a multiple of 16)
  if (((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(sh) |
        reinterpret_cast<uintptr_t>(w)) & 15) != 0)
    return fail(-2, "tp_fwd_bf16: x, sh and w must be 16-byte aligned");
  hipLaunchKernelGGL(c->fwd_bf, tp_fwd_grid(*c, n_nodes, true), dim3(64 * c->fwpb), 0, (hipStream_t)stream,
                     x, sh, static_cast<const unsigned short*>(w), sender, rowptr, n_nodes, inv_norm,
                     agg);
  return check_launch("tp_fwd_bf16");
}

// tp_bwd: 8 half-waves x beph edges per block; with bxcd the grid is 1-D, the edge blocks rounded
// up to a multiple of 8 so that XCD k takes one contiguous range of them (gen_kernels.py)
static dim3 tp_bwd_grid(const eelg_tp_cfg& c, int n_edges) {
  const int nb = (n_edges + 8 * c.beph - 1) / (8 * c.beph);
  if (!c.bxcd) return dim3(nb, c.nbgroups);
  return dim3(((nb + 7) / 8) * 8 * c.nbgroups);
}

int eelg_tp_bwd_sorted(int cfg, const float* x, const float* sh, const float* w, const int* sender,
                       const int* receiver, const int* spos, int n_edges, const float* grad_agg,
                       float inv_norm, float* grad_w, float* gxe, void* stream) {
  const eelg_tp_cfg* c = tp_cfg(cfg);
  if (!c) return -1;
  if (n_edges <= 0) return 0;
  hipLaunchKernelGGL(c->bwd, tp_bwd_grid(*c, n_edges), dim3(256), 0,
                     (hipStream_t)stream, x, sh, w, sender, receiver, n_edges, grad_agg, inv_norm,
                     grad_w, gxe, spos);
  return check_launch("tp_bwd");
}

int eelg_tp_bwd(int cfg, const float* x, const float* sh, const float* w, const int* sender,
                const int* receiver, int n_edges, const float* grad_agg, float inv_norm,
                float* grad_w, float* gxe, void* stream) {
  return eelg_tp_bwd_sorted(cfg, x, sh, w, sender, receiver, nullptr, n_edges, grad_agg, inv_norm,
                            grad_w, gxe, stream);
}

int eelg_tp_bwd_sorted_bf16(int cfg, const float* x, const float* sh, const void* w,
                            const int* sender, const int* receiver, const int* spos, int n_edges,
                            const float* grad_agg, float inv_norm, void* grad_w, void* gxe,
                            void* stream) {
  const eelg_tp_cfg* c = tp_cfg(cfg);
  if (!c) return -1;
  if (!c->bwd_bf) return fail(-2, "tp_bwd_bf16: bf16 storage is generated for mul 32 only (config %s)", c->name);
  if (n_edges <= 0) return 0;
  hipLaunchKernelGGL(c->bwd_bf, tp_bwd_grid(*c, n_edges), dim3(256), 0,
                     (hipStream_t)stream, x, sh, static_cast<const unsigned short*>(w), sender,
                     receiver, n_edges, grad_agg, inv_norm, static_cast<unsigned short*>(grad_w),
                     static_cast<unsigned short*>(gxe), spos);
  return check_launch("tp_bwd_bf16");
}

int eelg_tp_bwd_bf16(int cfg, const float* x, const float* sh, const void* w, const int* sender,
                     const int* receiver, int n_edges, const float* grad_agg, float inv_norm,
                     void* grad_w, void* gxe, void* stream) {
  return eelg_tp_bwd_sorted_bf16(cfg, x, sh, w, sender, receiver, nullptr, n_edges, grad_agg,
                                 inv_norm, grad_w, gxe, stream);
}

// fused output-linear grad-x + backward: R-receiver tiles x nbgroups input blocks, 1-D grid with
// the tiles rounded up to a multiple of 8 (the group blocks of a tile share an XCD; gen_kernels.py)
static dim3 tp_bwf_grid(const eelg_tp_cfg& c, int n_nodes) {
  const int nt = (n_nodes + c.bwf_r - 1) / c.bwf_r;
  return dim3(((nt + 7) / 8) * 8 * c.nbgroups);
}

int eelg_tp_bwf_slot(int cfg, int slot, int* w_off, float* alpha, int* gy_off) {
  const eelg_tp_cfg* c = tp_cfg(cfg);
  if (!c) return -1;
  if (!c->bwf) return fail(-2, "tp_bwd_fused: not generated for config %s (mul 32 only)", c->name);
  if (slot < 0 || slot >= c->npaths) return fail(-3, "tp_bwf_slot: slot %d of %d", slot, c->npaths);
  *w_off = c->bwf_slots[slot][0];
  *gy_off = c->bwf_slots[slot][1];
  *alpha = c->bwf_alpha[slot];
  return 0;
}

int eelg_tp_bwd_fused(int cfg, const float* x, const float* sh, const float* w, const int* sender,
                      const int* receiver,
                      const int* rowptr, int n_nodes, const float* gy, const float* lin_w,
                      float inv_norm, float* grad_w, float* gxe, void* stream) {
  const eelg_tp_cfg* c = tp_cfg(cfg);
  if (!c) return -1;
  if (!c->bwf) return fail(-2, "tp_bwd_fused: not generated for config %s (mul 32 only)", c->name);
  if (reinterpret_cast<uintptr_t>(lin_w) & 15) return fail(-3, "tp_bwd_fused: linear weight not 16-B aligned");
  if (n_nodes <= 0) return 0;
  hipLaunchKernelGGL(c->bwf, tp_bwf_grid(*c, n_nodes), dim3(256), 0, (hipStream_t)stream, x, sh, w,
                     sender, receiver, rowptr, n_nodes, gy, lin_w, inv_norm, grad_w, gxe);
  return check_launch("tp_bwd_fused");
}

int eelg_tp_bwd_fused_bf16(int cfg, const float* x, const float* sh, const void* w,
                           const int* sender, const int* receiver, const int* rowptr,
                           int n_nodes, const float* gy,
                           const float* lin_w, float inv_norm, void* grad_w, void* gxe,
                           void* stream) {
  const eelg_tp_cfg* c = tp_cfg(cfg);
  if (!c) return -1;
  if (!c->bwf_bf) return fail(-2, "tp_bwd_fused_bf16: not generated for config %s", c->name);
  if (reinterpret_cast<uintptr_t>(lin_w) & 15) return fail(-3, "tp_bwd_fused: linear weight not 16-B aligned");
  if (n_nodes <= 0) return 0;
  hipLaunchKernelGGL(c->bwf_bf, tp_bwf_grid(*c, n_nodes), dim3(256), 0, (hipStream_t)stream, x, sh,
                     static_cast<const unsigned short*>(w), sender, receiver, rowptr, n_nodes, gy, lin_w,
                     inv_norm, static_cast<unsigned short*>(grad_w), static_cast<unsigned short*>(gxe));
  return check_launch("tp_bwd_fused_bf16");
}

// one half-wave per sender node, nbgroups input blocks on blockIdx.y
int eelg_tp_bwd_sender(int cfg, const float* x, const float* sh, const float* w, const int* sperm,
                       const int* srowptr, const int* receiver, int n_nodes,
                       const float* grad_agg, float inv_norm, float* grad_w, float* grad_x,
                       void* stream) {
  const eelg_tp_cfg* c = tp_cfg(cfg);
  if (!c) return -1;
  if (n_nodes <= 0) return 0;
  hipLaunchKernelGGL(c->bws, dim3((n_nodes + 7) / 8, c->nbgroups), dim3(256), 0,
                     (hipStream_t)stream, x, sh, w, sperm, srowptr, receiver, n_nodes, grad_agg,
                     inv_norm, grad_w, grad_x);
  return check_launch("tp_bwd_sender");
}

int eelg_tp_bwd_sender_bf16(int cfg, const float* x, const float* sh, const void* w,
                            const int* sperm, const int* srowptr, const int* receiver,
                            int n_nodes, const float* grad_agg, float inv_norm, void* grad_w,
                            float* grad_x, void* stream) {
  const eelg_tp_cfg* c = tp_cfg(cfg);
  if (!c) return -1;
  if (!c->bws_bf) return fail(-2, "tp_bwd_sender_bf16: bf16 storage is generated for mul 32 only (config %s)", c->name);
  if (n_nodes <= 0) return 0;
  hipLaunchKernelGGL(c->bws_bf, dim3((n_nodes + 7) / 8, c->nbgroups), dim3(256), 0,
                     (hipStream_t)stream, x, sh, static_cast<const unsigned short*>(w), sperm,
                     srowptr, receiver, n_nodes, grad_agg, inv_norm,
                     static_cast<unsigned short*>(grad_w), grad_x);
  return check_launch("tp_bwd_sender_bf16");
}

int eelg_segment_sum_csr(const float* src, const int* rowptr, const int* idx,
                         const float* row_scale, float scale, int n_rows, int width, float* out,
                         void* stream) {
  return segment_sum_launch(src, rowptr, idx, row_scale, scale, n_rows, width, out, stream,
                            "segment_sum_csr");
}

int eelg_segment_sum_csr_bf16(const void* src, const int* rowptr, const int* idx,
                              const float* row_scale, float scale, int n_rows, int width,
                              float* out, void* stream) {
  return segment_sum_launch(static_cast<const unsigned short*>(src), rowptr, idx, row_scale, scale,
                            n_rows, width, out, stream, "segment_sum_csr_bf16");
}

int eelg_segment_sum_split(const float* src, const int* rowptr, const int* idx,
                           const float* row_scale, float scale, int n_rows, int width, int n_split,
                           float* work, float* out, void* stream) {
  if (n_rows <= 0 || width <= 0) return 0;
  if (n_split <= 0) return fail(-2, "segment_sum_split: n_split must be positive");
  hipLaunchKernelGGL(segment_split_kernel, dim3((n_rows * n_split + 3) / 4), dim3(256), 0,
                     (hipStream_t)stream, src, rowptr, idx, n_rows, width, n_split, work);
  hipLaunchKernelGGL(segment_combine_kernel, dim3((n_rows * width + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, work, row_scale, scale, n_rows, width, n_split, out);
  return check_launch("segment_sum_split");
}

int eelg_segment_order(const float* src, const int* rowptr, int n_rows, int width, int op,
                       float* out, int* arg, void* stream) {
  if (op < SEG_MAX || op > SEG_MUL) return fail(-2, "segment_order: op %d (0 max, 1 min, 2 mul)", op);
  if (op != SEG_MUL && !arg) return fail(-2, "segment_order: max / min need the position output");
  if (n_rows <= 0 || width <= 0) return 0;
  const long long n = (long long)n_rows * width;
  hipLaunchKernelGGL(segment_order_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, src, rowptr, n_rows, width, op, out, arg);
  return check_launch("segment_order");
}

int eelg_segment_order_bwd(const float* src, const int* rowptr, const int* arg, const float* grad_out,
                           int n_rows, int width, int op, float* grad_src, void* stream) {
  if (op < SEG_MAX || op > SEG_MUL) return fail(-2, "segment_order_bwd: op %d (0 max, 1 min, 2 mul)", op);
  if (op != SEG_MUL && !arg) return fail(-2, "segment_order_bwd: max / min need the positions");
  if (n_rows <= 0 || width <= 0) return 0;
  const long long n = (long long)n_rows * width;
  hipLaunchKernelGGL(segment_order_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, src, rowptr, arg, grad_out, n_rows, width, op, grad_src);
  return check_launch("segment_order_bwd");
}

static int cgc_launch_fwd(const float* ps, const float* pr, const float* ep, const float* ef,
                          const float* ea, const int* sender, const int* rowptr,
                          const float* row_scale, int n_nodes, int D, float* agg, void* stream,
                          const float* res = nullptr) {
  if (D <= 0) return fail(-2, "cgc_fwd: D must be positive");
  if (n_nodes <= 0) return 0;
  if (D > EELG_CGC_MAXD) return fail(-2, "cgc_fwd: D = %d > %d not built", D, EELG_CGC_MAXD);
  const dim3 g(cgc_grid((n_nodes + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
#define CGCF(C, E) hipLaunchKernelGGL((cgc_fwd_kernel<C, E>), g, dim3(256), 0, st, ps, pr, ep, ef, ea, \
                                      sender, rowptr, row_scale, n_nodes, D, agg, res)
  const int cpl = D > 128 ? 4 : D > 64 ? 2 : 1;
  if (ef) { if (cpl == 4) CGCF(4, true); else if (cpl == 2) CGCF(2, true); else CGCF(1, true); }
  else { if (cpl == 4) CGCF(4, false); else if (cpl == 2) CGCF(2, false); else CGCF(1, false); }
#undef CGCF
  return check_launch("cgc_fwd");
}

static int cgc_launch_bwd(const float* ps, const float* pr, const float* ep, const float* ef,
                          const float* ea, const int* sender, const int* rowptr,
                          const float* row_scale, int n_nodes, int D, const float* grad_agg,
                          float* dz, float* grad_pr, void* stream) {
  if (D <= 0) return fail(-2, "cgc_bwd: D must be positive");
  if (n_nodes <= 0) return 0;
  if (D > EELG_CGC_MAXD) return fail(-2, "cgc_bwd: D = %d > %d not built", D, EELG_CGC_MAXD);
  const dim3 g(cgc_grid((n_nodes + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
#define CGCB(C, E) hipLaunchKernelGGL((cgc_bwd_kernel<C, E>), g, dim3(256), 0, st, ps, pr, ep, ef, ea, \
                                      sender, rowptr, row_scale, n_nodes, D, grad_agg, dz, grad_pr)
  const int cpl = D > 128 ? 4 : D > 64 ? 2 : 1;
  if (ef) { if (cpl == 4) CGCB(4, true); else if (cpl == 2) CGCB(2, true); else CGCB(1, true); }
  else { if (cpl == 4) CGCB(4, false); else if (cpl == 2) CGCB(2, false); else CGCB(1, false); }
#undef CGCB
  return check_launch("cgc_bwd");
}

int eelg_cgc_fwd(const float* ps, const float* pr, const float* ep, const int* sender,
                 const int* rowptr, const float* row_scale, int n_nodes, int D, float* agg,
                 void* stream) {
  return cgc_launch_fwd(ps, pr, ep, nullptr, nullptr, sender, rowptr, row_scale, n_nodes, D, agg,
                        stream);
}

int eelg_cgc_bwd(const float* ps, const float* pr, const float* ep, const int* sender,
                 const int* rowptr, const float* row_scale, int n_nodes, int D,
                 const float* grad_agg, float* dz, float* grad_pr, void* stream) {
  return cgc_launch_bwd(ps, pr, ep, nullptr, nullptr, sender, rowptr, row_scale, n_nodes, D,
                        grad_agg, dz, grad_pr, stream);
}

// Which factored-edge passes run receiver-streaming (bit 0: forward, bit 1: backward; the others
// one wave per receiver).  r05f (cgc_modified, batch 256, same box): streaming both passes 9.22
// ms/step, neither 9.55; the forward alone measured 0.207 vs 0.197 ms per launch (it is VALU-bound
// on the transcendentals, where the streaming form's selects and lane reads cost more than its
// fewer round trips save), so the default streams the backward only.
static int cgc_stream_mask() {
  static int v = -1;
  if (v < 0) { const char* e = getenv("EELG_CGC_STREAM"); v = e ? atoi(e) : 2; }
  return v;
}
static bool cgc_stream(bool bwd) { return (cgc_stream_mask() >> (bwd ? 1 : 0)) & 1; }

static_assert(CGC_RPW == EELG_CGC_RPW, "eelg.h EELG_CGC_RPW");
static int cgc_launch_stream(bool bwd, const float* ps, const float* pr, const float* ef,
                             const float* ea, const int* sender, const int* receiver, const int* rowptr,
                             const float* row_scale, int n_nodes, int D, float* agg,
                             const float* grad_agg, float* dz, float* grad_pr, float* dea_part,
                             void* stream) {
  if (D <= 0) return fail(-2, "cgc_stream: D must be positive");
  if (n_nodes <= 0) return 0;
  if (D > EELG_CGC_MAXD) return fail(-2, "cgc_stream: D = %d > %d not built", D, EELG_CGC_MAXD);
  const int waves = (n_nodes + CGC_RPW - 1) / CGC_RPW;
  const dim3 g(cgc_grid((waves + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
#define CGCS(C, B) hipLaunchKernelGGL((cgc_stream_kernel<C, B>), g, dim3(256), 0, st, ps, pr, ef, ea, \
                                      sender, receiver, rowptr, row_scale, n_nodes, D, agg, grad_agg, \
                                      dz, grad_pr, dea_part)
  const int cpl = D > 128 ? 4 : D > 64 ? 2 : 1;
  if (bwd) { if (cpl == 4) CGCS(4, true); else if (cpl == 2) CGCS(2, true); else CGCS(1, true); }
  else { if (cpl == 4) CGCS(4, false); else if (cpl == 2) CGCS(2, false); else CGCS(1, false); }
#undef CGCS
  return check_launch(bwd ? "cgc_bwd_stream" : "cgc_fwd_stream");
}

int eelg_cgc_fwd_ef(const float* ps, const float* pr, const float* ef, const float* ea,
                    const int* sender, const int* receiver, const int* rowptr,
                    const float* row_scale, int n_nodes, int D, float* agg, void* stream) {
  if (!ef || !ea) return fail(-2, "cgc_fwd_ef: ef and ea are required");
  if (cgc_stream(false) && receiver)
    return cgc_launch_stream(false, ps, pr, ef, ea, sender, receiver, rowptr, row_scale, n_nodes, D,
                             agg, nullptr, nullptr, nullptr, nullptr, stream);
  return cgc_launch_fwd(ps, pr, nullptr, ef, ea, sender, rowptr, row_scale, n_nodes, D, agg, stream);
}

int eelg_cgc_bwd_ef_parts(int n_nodes) {
  const int waves = (n_nodes + EELG_CGC_RPW - 1) / EELG_CGC_RPW;
  return n_nodes > 0 ? (waves + 3) / 4 : 0;
}

int eelg_cgc_fwd_ef_res(const float* ps, const float* pr, const float* ef, const float* ea,
                        const int* sender, const int* rowptr, const float* row_scale, int n_nodes,
                        int D, const float* res, float* agg, void* stream) {
  if (!ef || !ea) return fail(-2, "cgc_fwd_ef_res: ef and ea are required");
  return cgc_launch_fwd(ps, pr, nullptr, ef, ea, sender, rowptr, row_scale, n_nodes, D, agg, stream, res);
}

int eelg_cgc_bwd_ef(const float* ps, const float* pr, const float* ef, const float* ea,
                    const int* sender, const int* receiver, const int* rowptr,
                    const float* row_scale, int n_nodes, int D, const float* grad_agg, float* dz,
                    float* grad_pr, float* dea_part, void* stream) {
  if (!ef || !ea) return fail(-2, "cgc_bwd_ef: ef and ea are required");
  if (dea_part && !receiver) return fail(-2, "cgc_bwd_ef: dea_part needs the receiver array");
  if ((cgc_stream(true) || dea_part) && receiver)
    return cgc_launch_stream(true, ps, pr, ef, ea, sender, receiver, rowptr, row_scale, n_nodes, D,
                             nullptr, grad_agg, dz, grad_pr, dea_part, stream);
  return cgc_launch_bwd(ps, pr, nullptr, ef, ea, sender, rowptr, row_scale, n_nodes, D, grad_agg,
                        dz, grad_pr, stream);
}

int eelg_csr_spmm(const int* rowptr, const int* col, const float* val, int n_rows, const float* B,
                  int ldb_r, int ldb_c, int n_cols, float* out, int ldo_r, int ldo_c, void* stream) {
  if (n_rows <= 0 || n_cols <= 0) return 0;
  hipLaunchKernelGGL(csr_spmm_kernel, dim3((4 * n_rows * n_cols + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, rowptr, col, val, n_rows, B, ldb_r, ldb_c, n_cols, out,
                     ldo_r, ldo_c);
  return check_launch("csr_spmm");
}

static const eelg_sc_cfg* sc_get(int cfg, int mul) {
  int n = 0;
  const eelg_sc_cfg* t = eelg_sc_table_mul(mul, &n);
  if (!t) { fail(-2, "symmetric contraction built for mul 16 / 32 / 64, got %d", mul); return nullptr; }
  if (cfg < 0 || cfg >= n) { fail(-1, "bad sc config %d", cfg); return nullptr; }
  return &t[cfg];
}

int eelg_gate_fwd(const float* x, int n_nodes, const eelg_gate_desc* desc, float cst, float* y,
                  void* stream) {
  int din, dout;
  if (int rc = gate_check(desc, &din, &dout)) return rc;
  if (n_nodes <= 0) return 0;
  hipLaunchKernelGGL(gate_fwd_kernel, dim3(gate_grid(n_nodes)), dim3(256), 0, (hipStream_t)stream,
                     x, n_nodes, *desc, din, dout, cst, y);
  return check_launch("gate_fwd");
}

int eelg_gate_bwd(const float* x, const float* grad_y, int n_nodes, const eelg_gate_desc* desc,
                  float cst, float* grad_x, void* stream) {
  int din, dout;
  if (int rc = gate_check(desc, &din, &dout)) return rc;
  if (n_nodes <= 0) return 0;
  hipLaunchKernelGGL(gate_bwd_kernel, dim3(gate_grid(n_nodes)), dim3(256), 0, (hipStream_t)stream,
                     x, grad_y, n_nodes, *desc, din, dout, cst, grad_x);
  return check_launch("gate_bwd");
}

// fwd / grad-x / channel-major copy: nb-node tiles x mul/4 channel quads, 1-D; the tile count
// is padded to a multiple of 8 so the quads of tile t all run on XCD t % 8 (gen_kernels.py)
static bool a16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }
static dim3 sc_tile_grid(int n_nodes, int mul, int nb = 64) {
  const int tiles = (n_nodes + nb - 1) / nb;
  return dim3(((tiles + 7) / 8) * 8 * (mul / 4));
}

int eelg_sc_fwd(int cfg, const float* x, const float* coef, int n_nodes, int mul, float* out,
                void* stream) {
  const eelg_sc_cfg* c = sc_get(cfg, mul);
  if (!c) return -1;
  if (n_nodes <= 0) return 0;
  if (!a16(x) || !a16(out) || !a16(coef)) return fail(-2, "sc_fwd: x, coef and out must be 16-byte aligned");
  hipLaunchKernelGGL(c->fwd, sc_tile_grid(n_nodes, mul, c->nb), dim3(c->nth), 0,
                     (hipStream_t)stream, x, coef, n_nodes, out);
  return check_launch("sc_fwd");
}

int eelg_sc_bwd_x(int cfg, const float* x, const float* coef, const float* grad_out, int n_nodes,
                  int mul, float* grad_x, void* stream) {
  return eelg_sc_bwd_x_cm(cfg, x, coef, grad_out, n_nodes, mul, grad_x, nullptr, nullptr, stream);
}

int eelg_sc_bwd_x_cm(int cfg, const float* x, const float* coef, const float* grad_out,
                     int n_nodes, int mul, float* grad_x, float* xt, float* gt, void* stream) {
  const eelg_sc_cfg* c = sc_get(cfg, mul);
  if (!c) return -1;
  if (n_nodes <= 0) return 0;
  if (!a16(x) || !a16(grad_out) || !a16(grad_x) || !a16(coef))
    return fail(-2, "sc_bwd_x: x, coef, grad_out and grad_x must be 16-byte aligned");
  hipLaunchKernelGGL(c->bwd_x, sc_tile_grid(n_nodes, mul, c->nb), dim3(c->nth), 0,
                     (hipStream_t)stream, x, coef, grad_out, n_nodes, grad_x, xt, gt);
  return check_launch("sc_bwd_x");
}

int eelg_sc_cmajor(int cfg, int which, const float* x, int n_nodes, int mul, float* xt,
                   void* stream) {
  const eelg_sc_cfg* c = sc_get(cfg, mul);
  if (!c) return -1;
  if (which != 0 && which != 1) return fail(-2, "sc_cmajor: which must be 0 (input) or 1 (output)");
  if (n_nodes <= 0) return 0;
  if (!a16(x)) return fail(-2, "sc_cmajor: x must be 16-byte aligned");
  hipLaunchKernelGGL(which ? c->cmajor_out : c->cmajor, sc_tile_grid(n_nodes, mul), dim3(256), 0,
                     (hipStream_t)stream, x, n_nodes, xt);
  return check_launch("sc_cmajor");
}

// streaming coefficient gradient: the nodes are split into node ranges (one partial row each)
// of whole chunks, so that mul channels x ranges x the term-group sets make about four rounds
// of one-workgroup-per-CU blocks on the 256 CUs (lmax 4, correlation 3: 4 ranges; lmax 3:
// 16), with ranges of at least 2048 nodes
static int sc_coef_range(const eelg_sc_cfg& c, int n_nodes, int mul) {
  const int per = mul * (c.csets > 0 ? c.csets : 1);
  int nr = (1024 + per - 1) / per;
  const int nmax = (n_nodes + 2047) / 2048;
  nr = nr > nmax ? nmax : nr;
  nr = nr < 1 ? 1 : nr;
  const int rn = (n_nodes + nr - 1) / nr;
  return (rn + c.nbc - 1) / c.nbc * c.nbc;
}

int eelg_sc_bwd_coef_parts(int cfg, int n_nodes, int mul) {
  const eelg_sc_cfg* c = sc_get(cfg, mul);
  if (!c) return -1;
  if (n_nodes <= 0) return 0;
  const int rn = c->bwd_coefs ? sc_coef_range(*c, n_nodes, mul) : c->nbc;
  return (n_nodes + rn - 1) / rn;
}

int eelg_sc_bwd_coef(int cfg, const float* xt, const float* gt, int n_nodes, int mul, int chunk,
                     float* partial, void* stream) {
  const eelg_sc_cfg* c = sc_get(cfg, mul);
  if (!c) return -1;
  if (chunk != c->nbc)
    return fail(-2, "sc_bwd_coef: chunk must be the config's coefficient chunk %d (info[6]), got %d",
                c->nbc, chunk);
  if (n_nodes <= 0) return 0;
  if (c->bwd_coefs) {
    // one workgroup per (channel x node range tile, term-group set); partial[range, channel, t]
    const int rn = sc_coef_range(*c, n_nodes, mul);
    const int tiles = mul * ((n_nodes + rn - 1) / rn);
    hipLaunchKernelGGL(c->bwd_coefs, dim3(((tiles + 7) / 8) * 8 * c->csets), dim3(1024), 0,
                       (hipStream_t)stream, xt, gt, n_nodes, rn, partial);
    return check_launch("sc_bwd_coefs");
  }
  // one workgroup per (chunk of nbc LDS-resident nodes, channel)
  const int nch = (n_nodes + chunk - 1) / chunk;
  hipLaunchKernelGGL(c->bwd_coef, dim3(nch, mul), dim3(64 * c->wpb), 0, (hipStream_t)stream, xt, gt,
                     n_nodes, chunk, partial);
  return check_launch("sc_bwd_coef");
}

int eelg_linear_fwd_res(const float* x, int x_row, const float* w, const float* bias,
                        const float* res, int n_nodes, float* y, int y_row,
                        const eelg_lin_desc* desc, void* stream) {
  if (!desc || desc->n_slots <= 0 || desc->n_slots > EELG_LIN_MAXSLOT)
    return fail(-2, "linear_fwd: bad descriptor");
  for (int s = 0; s < desc->n_slots; ++s) {
    const eelg_lin_slot& sl = desc->slot[s];
    if (sl.n_src < 0 || sl.n_src > EELG_LIN_MAXSRC || sl.d <= 0)
      return fail(-2, "linear_fwd: bad slot %d", s);
    for (int t = 0; t < sl.n_src; ++t)
      if (sl.src[t].k <= 0) return fail(-2, "linear_fwd: empty K in slot %d", s);
    if (sl.bias_off >= 0 && sl.d != 1) return fail(-2, "linear_fwd: bias on a non-scalar slot");
  }
  if (n_nodes <= 0) return 0;
  const bool full = lin_fwd_fast_ok(x, x_row, y, y_row, desc);
  const bool part = !full && !res && LINF_PARTIAL && lin_fwd_fast_ok(x, x_row, y, y_row, desc, true);
  if ((full || part) && !(res && (reinterpret_cast<uintptr_t>(res) & 15))) {
    // groups of 32/d whole nodes; the d = 9 slots have the most (ceil(n / 3))
    int max_groups = 0;
    for (int s = 0; s < desc->n_slots; ++s) {
      const int nb = 32 / desc->slot[s].d;
      const int g = (n_nodes + nb - 1) / nb;
      max_groups = g > max_groups ? g : max_groups;
    }
    const int gblocks = (max_groups + LINF_WAVES * LINF_GPW - 1) / (LINF_WAVES * LINF_GPW);
    dim3 grid(((gblocks + 7) / 8) * 8 * desc->max_jt, desc->n_slots, 1);
    int ws4;
    size_t lds;
    lin_fwd_fast_lds(desc, &ws4, &lds);
    // one column tile per slot (the 800 -> 800 linears): two workgroups per CU measured faster
    if (desc->max_jt == 1 && lds < LINF_LDS_1JT) lds = LINF_LDS_1JT;
    static bool lds_attr = false;   // > 64 KB of dynamic LDS must be allowed explicitly
    if (!lds_attr) {
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(&lin_fwd_fast_kernel<false, false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess ||
          hipFuncSetAttribute(reinterpret_cast<const void*>(&lin_fwd_fast_kernel<true, false>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess ||
          hipFuncSetAttribute(reinterpret_cast<const void*>(&lin_fwd_fast_kernel<false, true>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) != hipSuccess)
        return fail(-3, "linear_fwd: cannot raise the dynamic LDS limit");
      lds_attr = true;
    }
    if (part)
      hipLaunchKernelGGL((lin_fwd_fast_kernel<false, true>), grid, dim3(64 * LINF_WAVES), lds, (hipStream_t)stream,
                         x, x_row, w, bias, n_nodes, y, y_row, *desc, res, ws4);
    else if (res)
      hipLaunchKernelGGL((lin_fwd_fast_kernel<true, false>), grid, dim3(64 * LINF_WAVES), lds, (hipStream_t)stream,
                         x, x_row, w, bias, n_nodes, y, y_row, *desc, res, ws4);
    else
      hipLaunchKernelGGL((lin_fwd_fast_kernel<false, false>), grid, dim3(64 * LINF_WAVES), lds, (hipStream_t)stream,
                         x, x_row, w, bias, n_nodes, y, y_row, *desc, res, ws4);
    return check_launch("linear_fwd");
  }
  dim3 grid((desc->max_rows + 127) / 128, desc->n_slots, 1);  // column tiles loop in-kernel
  hipLaunchKernelGGL(lin_fwd_kernel, grid, dim3(256), 0, (hipStream_t)stream, x, x_row, w, bias,
                     n_nodes, y, y_row, *desc, res);
  return check_launch("linear_fwd");
}

static int lin_desc_check(const eelg_lin_desc* desc, const char* what) {
  if (!desc || desc->n_slots <= 0 || desc->n_slots > EELG_LIN_MAXSLOT)
    return fail(-2, "%s: bad descriptor", what);
  for (int s = 0; s < desc->n_slots; ++s) {
    const eelg_lin_slot& sl = desc->slot[s];
    if (sl.n_src < 0 || sl.n_src > EELG_LIN_MAXSRC || sl.d <= 0 || sl.n_out <= 0)
      return fail(-2, "%s: bad slot %d", what, s);
    for (int t = 0; t < sl.n_src; ++t)
      if (sl.src[t].k <= 0) return fail(-2, "%s: empty K in slot %d", what, s);
  }
  return 0;
}

static int lin_pack_check(const eelg_lin_desc* desc, const char* what) {
  if (int rc = lin_desc_check(desc, what)) return rc;
  for (int s = 0; s < desc->n_slots; ++s) {
    int ks = 0;
    for (int t = 0; t < desc->slot[s].n_src; ++t) {
      if (desc->slot[s].src[t].k % 32) return fail(-2, "%s: source K must be a multiple of 32", what);
      ks += desc->slot[s].src[t].k;
    }
    if (ks > LINX_KMAX) return fail(-2, "%s: slot %d sums K = %d > %d", what, s, ks, LINX_KMAX);
  }
  return 0;
}

// bf16 elements of one part of the packed weights (pack holds 3 parts = 3x this)
long long eelg_linear_pack_size(const eelg_lin_desc* desc) {
  if (int rc = lin_pack_check(desc, "linear_pack_size")) return rc;
  return (long long)lin_pack_slot_off(*desc, desc->n_slots) * 8 / 3;
}

int eelg_linear_pack(const float* w, const eelg_lin_desc* desc, void* pack, void* stream) {
  if (int rc = lin_pack_check(desc, "linear_pack")) return rc;
  if (reinterpret_cast<uintptr_t>(pack) & 15) return fail(-2, "linear_pack: pack must be 16-byte aligned");
  const int nunits = lin_pack_slot_off(*desc, desc->n_slots) / 3;
  if (nunits <= 0) return 0;
  hipLaunchKernelGGL(lin_pack_kernel, dim3((nunits + 255) / 256), dim3(256), 0, (hipStream_t)stream, w,
                     *desc, nunits, static_cast<uint4*>(pack));
  return check_launch("linear_pack");
}

int eelg_linear_fwd_pk(const float* x, int x_row, const void* pack, const float* bias,
                       const float* res, int n_nodes, float* y, int y_row,
                       const eelg_lin_desc* desc, void* stream) {
  if (int rc = lin_pack_check(desc, "linear_fwd_pk")) return rc;
  if (!lin_fwd_fast_ok(x, x_row, y, y_row, desc) || (reinterpret_cast<uintptr_t>(res) & 15) ||
      (reinterpret_cast<uintptr_t>(pack) & 15))
    return fail(-2, "linear_fwd_pk: the descriptor / rows do not qualify for the packed path "
                    "(whole 32-wide K chunks and column tiles, d odd <= 9, 16-B aligned rows)");
  for (int s = 0; s < desc->n_slots; ++s)
    if (desc->slot[s].bias_off >= 0 && desc->slot[s].d != 1)
      return fail(-2, "linear_fwd_pk: bias on a non-scalar slot");
  if (n_nodes <= 0) return 0;
  int max_groups = 0;
  for (int s = 0; s < desc->n_slots; ++s) {
    const int nb = 32 / desc->slot[s].d;
    const int g = (n_nodes + nb - 1) / nb;
    max_groups = g > max_groups ? g : max_groups;
  }
  const int gblocks = (max_groups + LINX_WAVES * LINX_GPW - 1) / (LINX_WAVES * LINX_GPW);
  dim3 grid(((gblocks + 7) / 8) * 8 * desc->max_jt, desc->n_slots, 1);
  const uint4* pk = static_cast<const uint4*>(pack);
  if (res)
    hipLaunchKernelGGL(lin_fwd_x6_kernel<true>, grid, dim3(64 * LINX_WAVES), 0, (hipStream_t)stream,
                       x, x_row, pk, bias, n_nodes, y, y_row, *desc, res);
  else
    hipLaunchKernelGGL(lin_fwd_x6_kernel<false>, grid, dim3(64 * LINX_WAVES), 0, (hipStream_t)stream,
                       x, x_row, pk, bias, n_nodes, y, y_row, *desc, res);
  return check_launch("linear_fwd_pk");
}

int eelg_linear_fwd(const float* x, int x_row, const float* w, const float* bias, int n_nodes,
                    float* y, int y_row, const eelg_lin_desc* desc, void* stream) {
  return eelg_linear_fwd_res(x, x_row, w, bias, nullptr, n_nodes, y, y_row, desc, stream);
}

int eelg_linear_bwd_w(const float* x, int x_row, const float* g, int g_row, int n_nodes,
                      int nodes_per_slice, float* partial, int n_partial, int w_total,
                      const eelg_linw_desc* desc, void* stream) {
  if (!desc || desc->n_ins <= 0 || desc->n_ins > EELG_LINW_MAXINS || nodes_per_slice <= 0)
    return fail(-2, "linear_bwd_w: bad descriptor");
  for (int t = 0; t < desc->n_ins; ++t) {
    const eelg_linw_ins& in = desc->ins[t];
    if (in.k <= 0 || in.n_out <= 0 || in.d <= 0 || in.d > 32)
      return fail(-2, "linear_bwd_w: bad instruction %d", t);
    if ((in.k + 31) / 32 > desc->max_ut || (in.n_out + 31) / 32 > desc->max_jt)
      return fail(-2, "linear_bwd_w: max_ut/max_jt too small for instruction %d", t);
  }
  if (n_nodes <= 0) return 0;
  const int slices = (n_nodes + nodes_per_slice - 1) / nodes_per_slice;
  if (n_partial < slices) return fail(-2, "linear_bwd_w: partial has %d rows, need %d", n_partial, slices);
  dim3 grid(slices, desc->n_ins, desc->max_ut * desc->max_jt);
  if (lin_bwdw_fast_ok(x, x_row, g, g_row, desc)) {
    // 1-D over (slice, tile), XCD-grouped (see lin_bwdw_fast_kernel)
    dim3 gf(((slices + 7) / 8) * 8 * desc->max_ut * desc->max_jt, desc->n_ins, 1);
    hipLaunchKernelGGL(lin_bwdw_fast_kernel, gf, dim3(256), 0, (hipStream_t)stream, x, x_row, g,
                       g_row, n_nodes, nodes_per_slice, partial, w_total, *desc);
  }
  else
    hipLaunchKernelGGL(lin_bwdw_kernel, grid, dim3(256), 0, (hipStream_t)stream, x, x_row, g, g_row,
                       n_nodes, nodes_per_slice, partial, w_total, *desc);
  return check_launch("linear_bwd_w");
}

int eelg_linear_bwd_w_x6(const float* g, int ldg, const float* x, int ldx, int n_rows, int n_out,
                         int k, int tiles_per_split, float* partial, void* stream) {
  if (k != 32 && k != 64 && k != 96 && k != 128)
    return fail(-2, "linear_bwd_w_x6: k must be 32, 64, 96 or 128, got %d", k);
  if (n_out <= 0 || tiles_per_split <= 0 || ldg < n_out || ldx < k)
    return fail(-2, "linear_bwd_w_x6: bad shape (n_out %d, ldg %d, k %d, ldx %d, tiles %d)", n_out,
                ldg, k, ldx, tiles_per_split);
  if (n_rows <= 0) return 0;
  const int ntile = (n_rows + 31) / 32;
  const dim3 grid((n_out + 127) / 128, (ntile + tiles_per_split - 1) / tiles_per_split);
  hipStream_t st = (hipStream_t)stream;
  switch (k / 32) {
    case 1: hipLaunchKernelGGL(lin_bwdw_x6_kernel<1>, grid, dim3(256), 0, st, g, ldg, x, ldx, n_rows, n_out, tiles_per_split, partial); break;
    case 2: hipLaunchKernelGGL(lin_bwdw_x6_kernel<2>, grid, dim3(256), 0, st, g, ldg, x, ldx, n_rows, n_out, tiles_per_split, partial); break;
    case 3: hipLaunchKernelGGL(lin_bwdw_x6_kernel<3>, grid, dim3(256), 0, st, g, ldg, x, ldx, n_rows, n_out, tiles_per_split, partial); break;
    default: hipLaunchKernelGGL(lin_bwdw_x6_kernel<4>, grid, dim3(256), 0, st, g, ldg, x, ldx, n_rows, n_out, tiles_per_split, partial); break;
  }
  return check_launch("linear_bwd_w_x6");
}

}  // extern "C"
