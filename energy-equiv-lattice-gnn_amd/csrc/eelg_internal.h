// Internal declarations shared by the generated and hand-written HIP sources.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef void (*eelg_tp_fwd_fn)(const float*, const float*, const float*, const int*, const int*, int,
                               float, float*);
typedef void (*eelg_tp_bwd_fn)(const float*, const float*, const float*, const int*, const int*, int,
                               const float*, float, float*, float*, const int*);
// bf16 storage (bit patterns in unsigned short) of the edge-sized TP tensors
typedef void (*eelg_tp_fwd_bf_fn)(const float*, const float*, const unsigned short*, const int*,
                                  const int*, int, float, float*);
typedef void (*eelg_tp_bwd_bf_fn)(const float*, const float*, const unsigned short*, const int*,
                                  const int*, int, const float*, float, unsigned short*,
                                  unsigned short*, const int*);
// sender-order backward: (x, sh, w, sperm, srowptr, receiver, n_nodes, grad_agg, inv_norm,
// grad_w, grad_x)
typedef void (*eelg_tp_bws_fn)(const float*, const float*, const float*, const int*, const int*,
                               const int*, int, const float*, float, float*, float*);
typedef void (*eelg_tp_bws_bf_fn)(const float*, const float*, const unsigned short*, const int*,
                                  const int*, const int*, int, const float*, float,
                                  unsigned short*, float*);
// fused output-linear grad-x + backward: (x, sh, w, sender, receiver, rowptr, n_nodes, gy,
// linear weight, inv_norm, grad_w, gxe)
typedef void (*eelg_tp_bwf_fn)(const float*, const float*, const float*, const int*, const int*,
                               const int*, int, const float*, const float*, float, float*, float*);
typedef void (*eelg_tp_bwf_bf_fn)(const float*, const float*, const unsigned short*, const int*,
                                  const int*, const int*, int, const float*, const float*, float,
                                  unsigned short*, unsigned short*);
// one MFMA task of tp_bwf's grad_agg stage: a 32-column tile (ct) of one slot's [32 x R*d3] block
struct eelg_bwf_task {
  int d3, ct, lds, woff, gyoff;
  float alpha;
};
typedef void (*eelg_sc_fwd_fn)(const float*, const float*, int, float*);
typedef void (*eelg_sc_bwdx_fn)(const float*, const float*, const float*, int, float*, float*,
                                float*);
typedef void (*eelg_sc_bwdc_fn)(const float*, const float*, int, int, float*);
typedef void (*eelg_sc_cmajor_fn)(const float*, int, float*);

struct eelg_tp_cfg {
  const char* name;
  int din, dmid, wn, nsh, ngroups, npaths, lmax, nbgroups;
  int nph;   // tp_fwd: receivers per half-wave
  int beph;  // tp_bwd: edges per half-wave
  int fwpb;  // tp_fwd: waves per workgroup
  uint64_t sig;
  eelg_tp_fwd_fn fwd;
  eelg_tp_bwd_fn bwd;
  eelg_tp_fwd_bf_fn fwd_bf;
  eelg_tp_bwd_bf_fn bwd_bf;
  eelg_tp_bws_fn bws;        // sender-order backward (grad_x summed per sender in registers)
  eelg_tp_bws_bf_fn bws_bf;
  int ngroups_bf;            // path groups of the bf16-weight forward (its own accumulator cap)
  int bxcd;                  // tp_bwd block placement (gen_kernels.TP_BWD_XCD): 0 = 2-D grid, else 1-D XCD ranges
  eelg_tp_bwf_fn bwf;        // fused output-linear grad-x + backward (nullptr: not generated)
  eelg_tp_bwf_bf_fn bwf_bf;
  int bwf_r;                 // its receivers per workgroup
  int tdim;                  // the output linear's row (target irreps dim)
  const int (*bwf_slots)[2]; // per slot: linear weight offset, gy offset
  const float* bwf_alpha;    // per slot: the linear's alpha
};

struct eelg_sc_cfg {
  const char* name;
  int D, Dout, drow, orow, nterms, njg, wpb;  // wpb: waves (term groups) per coef-grad workgroup
  uint64_t sig;
  eelg_sc_fwd_fn fwd;
  eelg_sc_bwdx_fn bwd_x;
  eelg_sc_bwdc_fn bwd_coef;
  eelg_sc_cmajor_fn cmajor;      // input (coupling) layout
  eelg_sc_cmajor_fn cmajor_out;  // output layout
  int nbc;                       // nodes per coef-grad staged tile (chunk granularity)
  int nb;                        // nodes per fwd / grad-x workgroup
  int nth;                       // threads per fwd / grad-x workgroup
  int cld;                       // coefficient row stride (nterms rounded up to 16: 64-B aligned rows)
  eelg_sc_bwdc_fn bwd_coefs;     // streaming coefficient gradient (round 6; nullptr: bwd_coef's chunk form)
  int csets;                     // its term-group sets (workgroups per (channel, node range) tile)
};

// every generated tensor-product set, all channel counts (eelg_capi.hip merges the per-mul tables
// of the generated translation units: generated/eelg_gen.hip for mul 32, eelg_gen_m16 / _m64)
const eelg_tp_cfg* eelg_tp_table(int* n);
const eelg_tp_cfg* eelg_tp_table_m16(int* n);
const eelg_tp_cfg* eelg_tp_table_m32(int* n);
const eelg_tp_cfg* eelg_tp_table_m64(int* n);

// error reporting shared by the translation units of libeelg.so (eelg_capi.hip)
int eelg_fail(int code, const char* fmt, ...);
int eelg_check_launch(const char* what);

// bf16 <-> fp32: the widening is exact; the narrowing rounds to nearest even
// (v_cvt_pk_bf16_f32 on gfx950)
__device__ __forceinline__ float eelg_bf2f(unsigned short v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ unsigned short eelg_f2bf(float f) {
  return __builtin_bit_cast(unsigned short, (__bf16)f);
}
// symmetric-contraction sets: one table per channel count, the same configs in the same order
// (eelg_sc_table = the mul-32 table; eelg_sc_table_mul: nullptr for a mul that was not generated)
const eelg_sc_cfg* eelg_sc_table(int* n);
const eelg_sc_cfg* eelg_sc_table_mul(int mul, int* n);
const eelg_sc_cfg* eelg_sc_table_m16(int* n);
const eelg_sc_cfg* eelg_sc_table_m32(int* n);
const eelg_sc_cfg* eelg_sc_table_m64(int* n);

// fp32-accurate GEMM operands on bf16 MFMA ("x6"): an fp32 value splits EXACTLY into three bf16
// parts by truncation, x = p0 + p1 + p2 (p0 = the top 8 significant bits, p1 the next 8 of the
// remainder, p2 the rest, which has at most 8 significant bits).  A product sum_k a_k b_k is
// then sum over (i, j) of a_i b_j; the six part products with i + j <= 2 are computed exactly
// by v_mfma_f32_32x32x16_bf16 and accumulated in fp32, smallest first; the three dropped ones
// are below 2^-23 of |a_k b_k| (the error against fp64 is that of an fp32 fmaf
// chain).  Over one K = 16 block the six 32x32x16 bf16 MFMAs (32 cycles each) take 192 cycles
// against 512 for the eight 32x32x2 f32 MFMAs (64 cycles each): 3/8 of the f32 MFMA time.
typedef __bf16 eelg_bf16x8 __attribute__((ext_vector_type(8)));
typedef float eelg_f32x16v __attribute__((ext_vector_type(16)));

// 8 fp32 -> three packed bf16x8 fragments (element t of the fragment = v[t])
__device__ __forceinline__ void eelg_split8(const float* v, uint4* p) {
  unsigned h0[8], h1[8], h2[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const unsigned a = __float_as_uint(v[t]) & 0xffff0000u;
    const float r = v[t] - __uint_as_float(a);
    const unsigned b = __float_as_uint(r) & 0xffff0000u;
    h0[t] = a;
    h1[t] = b;
    h2[t] = __float_as_uint(r - __uint_as_float(b));
  }
#define EELG_PK(h, t) __builtin_amdgcn_perm(h[t + 1], h[t], 0x07060302u)
  p[0] = make_uint4(EELG_PK(h0, 0), EELG_PK(h0, 2), EELG_PK(h0, 4), EELG_PK(h0, 6));
  p[1] = make_uint4(EELG_PK(h1, 0), EELG_PK(h1, 2), EELG_PK(h1, 4), EELG_PK(h1, 6));
  p[2] = make_uint4(EELG_PK(h2, 0), EELG_PK(h2, 2), EELG_PK(h2, 4), EELG_PK(h2, 6));
#undef EELG_PK
}
#define EELG_MFMA_BF(acc, a, b) \
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(eelg_bf16x8, (a)), \
                                                __builtin_bit_cast(eelg_bf16x8, (b)), acc, 0, 0, 0)
// acc += A B over one K = 16 block, both operands split (a[3], b[3]); smallest products first
#define EELG_X6(acc, a, b)                                                        \
  do {                                                                          \
    EELG_MFMA_BF(acc, (a)[0], (b)[2]); EELG_MFMA_BF(acc, (a)[1], (b)[1]);       \
    EELG_MFMA_BF(acc, (a)[2], (b)[0]); EELG_MFMA_BF(acc, (a)[0], (b)[1]);       \
    EELG_MFMA_BF(acc, (a)[1], (b)[0]); EELG_MFMA_BF(acc, (a)[0], (b)[0]);       \
  } while (0)
// the same with the five small products in their own accumulator (lo) and only a0 b0 in hi:
// over a long K the hi chain rounds once per K block instead of six times, and lo (<= 2^-7 of
// hi) adds nothing visible; the caller returns hi + lo.  For K in the thousands (radial grad_h,
// K = the radial outputs) this is more accurate than an fp32 MFMA chain.
#define EELG_X6HL(hi, lo, a, b)                                                   \
  do {                                                                          \
    EELG_MFMA_BF(lo, (a)[0], (b)[2]); EELG_MFMA_BF(lo, (a)[1], (b)[1]);         \
    EELG_MFMA_BF(lo, (a)[2], (b)[0]); EELG_MFMA_BF(lo, (a)[0], (b)[1]);         \
    EELG_MFMA_BF(lo, (a)[1], (b)[0]); EELG_MFMA_BF(hi, (a)[0], (b)[0]);         \
  } while (0)
#define EELG_X3HL(hi, lo, a, b)                                                   \
  do {                                                                          \
    EELG_MFMA_BF(lo, (a), (b)[2]); EELG_MFMA_BF(lo, (a), (b)[1]);               \
    EELG_MFMA_BF(hi, (a), (b)[0]);                                              \
  } while (0)
// acc += A B with A exactly bf16 (a single part, e.g. bf16 storage) and B split (b[3])
#define EELG_X3(acc, a, b)                                                        \
  do {                                                                          \
    EELG_MFMA_BF(acc, (a), (b)[2]); EELG_MFMA_BF(acc, (a), (b)[1]);             \
    EELG_MFMA_BF(acc, (a), (b)[0]);                                             \
  } while (0)

// Lane reduction of 64 per-lane slots: afterwards lane L holds, in v[0], the sum over all 64
// lanes of slot L.  Recursive halving over the lane bits 32, 16, 8, 4, 2, 1: at the step on
// bit b each lane keeps one half of its remaining slots (the upper half when its bit b is set)
// and adds the partner lane's copy of that half, so every step halves the slot count.  Bits 32
// and 16 use v_permlane32_swap / v_permlane16_swap (one swap moves two slots), bit 8 a DPP
// row rotation, bits 2 and 1 DPP quad permutations, bit 4 a swizzle.  Order is fixed:
// deterministic.
template <int CTRL>
__device__ __forceinline__ float eelg_dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ void eelg_lane_reduce64(float* v) {
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 32]),
                                                    false, false);
    v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v[i]), __float_as_uint(v[i + 16]),
                                                    false, false);
    v[i] = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  const int lane = threadIdx.x & 63;
  {
    const bool up = (lane & 8) != 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float keep = up ? v[i + 8] : v[i], give = up ? v[i] : v[i + 8];
      v[i] = keep + eelg_dpp_f<0x128>(give);   // row_ror:8 = lane ^ 8 within a 16-lane row
    }
  }
  {
    const bool up = (lane & 4) != 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float keep = up ? v[i + 4] : v[i], give = up ? v[i] : v[i + 4];
      v[i] = keep + __shfl_xor(give, 4);
    }
  }
  {
    const bool up = (lane & 2) != 0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float keep = up ? v[i + 2] : v[i], give = up ? v[i] : v[i + 2];
      v[i] = keep + eelg_dpp_f<0x4E>(give);    // quad_perm [2,3,0,1] = lane ^ 2
    }
  }
  {
    const bool up = (lane & 1) != 0;
    const float keep = up ? v[1] : v[0], give = up ? v[0] : v[1];
    v[0] = keep + eelg_dpp_f<0xB1>(give);      // quad_perm [1,0,3,2] = lane ^ 1
  }
}
