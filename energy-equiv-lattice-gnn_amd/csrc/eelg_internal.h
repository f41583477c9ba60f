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
};

const eelg_tp_cfg* eelg_tp_table(int* n);

// error reporting shared by the translation units of libeelg.so (eelg_capi.hip)
int eelg_fail(int code, const char* fmt, ...);
int eelg_check_launch(const char* what);

// bf16 <-> fp32: the widening is exact; the narrowing rounds to nearest even
// (v_cvt_pk_bf16_f32 on gfx950)
__device__ __forceinline__ float eelg_bf2f(unsigned short v) { return __uint_as_float((unsigned)v << 16); }
__device__ __forceinline__ unsigned short eelg_f2bf(float f) {
  return __builtin_bit_cast(unsigned short, (__bf16)f);
}
const eelg_sc_cfg* eelg_sc_table(int* n);

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
