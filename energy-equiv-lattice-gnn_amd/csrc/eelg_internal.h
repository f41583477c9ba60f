// Internal declarations shared by the generated and hand-written HIP sources.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef void (*eelg_tp_fwd_fn)(const float*, const float*, const float*, const int*, const int*, int,
                               float, float*);
typedef void (*eelg_tp_bwd_fn)(const float*, const float*, const float*, const int*, const int*, int,
                               const float*, float, float*, float*);
// bf16 storage (bit patterns in unsigned short) of the edge-sized TP tensors
typedef void (*eelg_tp_fwd_bf_fn)(const float*, const float*, const unsigned short*, const int*,
                                  const int*, int, float, float*);
typedef void (*eelg_tp_bwd_bf_fn)(const float*, const float*, const unsigned short*, const int*,
                                  const int*, int, const float*, float, unsigned short*,
                                  unsigned short*);
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
  uint64_t sig;
  eelg_tp_fwd_fn fwd;
  eelg_tp_bwd_fn bwd;
  eelg_tp_fwd_bf_fn fwd_bf;
  eelg_tp_bwd_bf_fn bwd_bf;
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
  int nb;                        // nodes per fwd / grad-x workgroup
  int nbc;                       // nodes per coef-grad staged tile (chunk granularity)
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
