"""ctypes binding of ``libeelg.so`` (C ABI declared in ``include/eelg.h``).

The library is built in-tree by ``__graft_entry__.build()`` /
``make -C energy-equiv-lattice-gnn_amd/csrc``.  There is no fallback: if the
library is missing or stale every op raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Tuple

import torch  # noqa: F401  (loads torch's libamdhip64 first; the .so binds to it by SONAME)

# EELG_LIB: an alternative build of the same library (kernel-variant experiments, tools/kbench.py)
LIB_PATH = os.environ.get("EELG_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                      "libeelg.so")

_P = ctypes.c_void_p
_I = ctypes.c_int
_F = ctypes.c_float

_SIGS = {
    "eelg_version": ([], ctypes.c_char_p),
    "eelg_last_error": ([], ctypes.c_char_p),
    "eelg_tp_find": ([ctypes.c_char_p], _I),
    "eelg_tp_info": ([_I, _P, _P], _I),
    "eelg_sc_find": ([ctypes.c_char_p], _I),
    "eelg_sc_info": ([_I, _P, _P], _I),
    "eelg_edge_embed": ([_P, _P, _P, _P, _P, _I, _I, _I, _F, _F, _P, _P, _P], _I),
    "eelg_tp_fwd": ([_I, _P, _P, _P, _P, _P, _I, _F, _P, _P], _I),
    "eelg_tp_bwd": ([_I, _P, _P, _P, _P, _P, _I, _P, _F, _P, _P, _P], _I),
    "eelg_tp_fwd_bf16": ([_I, _P, _P, _P, _P, _P, _I, _F, _P, _P], _I),
    "eelg_tp_bwd_bf16": ([_I, _P, _P, _P, _P, _P, _I, _P, _F, _P, _P, _P], _I),
    "eelg_tp_bwd_sorted": ([_I, _P, _P, _P, _P, _P, _P, _I, _P, _F, _P, _P, _P], _I),
    "eelg_tp_bwd_sorted_bf16": ([_I, _P, _P, _P, _P, _P, _P, _I, _P, _F, _P, _P, _P], _I),
    "eelg_tp_bwd_sender": ([_I, _P, _P, _P, _P, _P, _P, _I, _P, _F, _P, _P, _P], _I),
    "eelg_tp_bwd_sender_bf16": ([_I, _P, _P, _P, _P, _P, _P, _I, _P, _F, _P, _P, _P], _I),
    "eelg_tp_bwd_fused": ([_I, _P, _P, _P, _P, _P, _P, _I, _P, _P, _F, _P, _P, _P], _I),
    "eelg_tp_bwd_fused_bf16": ([_I, _P, _P, _P, _P, _P, _P, _I, _P, _P, _F, _P, _P, _P], _I),
    "eelg_tp_bwf_slot": ([_I, _I, _P, _P, _P], _I),
    "eelg_segment_sum_csr": ([_P, _P, _P, _P, _F, _I, _I, _P, _P], _I),
    "eelg_segment_sum_csr_bf16": ([_P, _P, _P, _P, _F, _I, _I, _P, _P], _I),
    "eelg_segment_sum_split": ([_P, _P, _P, _P, _F, _I, _I, _I, _P, _P, _P], _I),
    "eelg_segment_order": ([_P, _P, _I, _I, _I, _P, _P, _P], _I),
    "eelg_segment_order_bwd": ([_P, _P, _P, _P, _I, _I, _I, _P, _P], _I),
    "eelg_gate_fwd": ([_P, _I, _P, _F, _P, _P], _I),
    "eelg_gate_bwd": ([_P, _P, _I, _P, _F, _P, _P], _I),
    "eelg_cgc_fwd": ([_P, _P, _P, _P, _P, _P, _I, _I, _P, _P], _I),
    "eelg_cgc_bwd": ([_P, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P], _I),
    "eelg_cgc_fwd_ef": ([_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P], _I),
    "eelg_cgc_fwd_ef_res": ([_P] * 6 + [_P, _I, _I, _P, _P, _P], _I),
    "eelg_cgc_bwd_ef": ([_P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P, _P, _P], _I),
    "eelg_cgc_bwd_ef_parts": ([_I], _I),
    "eelg_csr_spmm": ([_P, _P, _P, _I, _P, _I, _I, _I, _P, _I, _I, _P], _I),
    "eelg_sc_fwd": ([_I, _P, _P, _I, _I, _P, _P], _I),
    "eelg_sc_bwd_x": ([_I, _P, _P, _P, _I, _I, _P, _P], _I),
    "eelg_sc_bwd_x_cm": ([_I, _P, _P, _P, _I, _I, _P, _P, _P, _P], _I),
    "eelg_sc_bwd_coef": ([_I, _P, _P, _I, _I, _I, _P, _P], _I),
    "eelg_sc_bwd_coef_parts": ([_I, _I, _I], _I),
    "eelg_sc_cmajor": ([_I, _I, _P, _I, _I, _P, _P], _I),
    "eelg_scg_fwd": ([_P, _P, _P, _I, _P, _I, _I, _P, _I, _P], _I),
    "eelg_scg_bwd_x": ([_P, _P, _P, _I, _P, _I, _P, _I, _I, _P, _P], _I),
    "eelg_scg_bwd_coef": ([_P, _P, _P, _I, _P, _I, _P, _I, _I, _P, _P], _I),
    "eelg_linear_fwd": ([_P, _I, _P, _P, _I, _P, _I, _P, _P], _I),
    "eelg_linear_fwd_res": ([_P, _I, _P, _P, _P, _I, _P, _I, _P, _P], _I),
    "eelg_linear_bwd_w": ([_P, _I, _P, _I, _I, _I, _P, _I, _I, _P, _P], _I),
    "eelg_linear_bwd_w_x6": ([_P, _I, _P, _I, _I, _I, _I, _I, _P, _P], _I),
    "eelg_radial_plan": ([_I, _I, _P, _P], _I),
    "eelg_linear_pack_size": ([_P], ctypes.c_longlong),
    "eelg_linear_pack": ([_P, _P, _P, _P], _I),
    "eelg_linear_fwd_pk": ([_P, _I, _P, _P, _P, _I, _P, _I, _P, _P], _I),
    "eelg_split_bf16x3": ([_P, ctypes.c_longlong, _P, _P], _I),
    "eelg_sum_rows_work": ([_I, ctypes.c_longlong], ctypes.c_longlong),
    "eelg_sum_rows": ([_P, ctypes.c_longlong, _I, ctypes.c_longlong, ctypes.c_float, _P, _P,
                       ctypes.c_longlong, _P], _I),
    "eelg_radial_fwd": ([_P, _I, _P, _P, _I, _P, _P, _P], _I),
    "eelg_radial_bwd_chain": ([_P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P], _I),
    "eelg_radial_bwd": ([_P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P], _I),
}

LIN_MAXSRC, LIN_MAXSLOT, LINW_MAXINS = 4, 8, 8


class LinSrc(ctypes.Structure):
    _fields_ = [("x_off", _I), ("k", _I), ("w_off", _I), ("ldk", _I), ("ldj", _I), ("alpha", _F)]


class LinSlot(ctypes.Structure):
    _fields_ = [("y_off", _I), ("n_out", _I), ("d", _I), ("bias_off", _I), ("n_src", _I),
                ("src", LinSrc * LIN_MAXSRC)]


class LinDesc(ctypes.Structure):
    _fields_ = [("n_slots", _I), ("max_jt", _I), ("max_rows", _I), ("pad", _I),
                ("slot", LinSlot * LIN_MAXSLOT)]


class LinWIns(ctypes.Structure):
    _fields_ = [("x_off", _I), ("k", _I), ("g_off", _I), ("n_out", _I), ("d", _I), ("w_off", _I),
                ("alpha", _F)]


class LinWDesc(ctypes.Structure):
    _fields_ = [("n_ins", _I), ("max_jt", _I), ("max_ut", _I), ("max_rows", _I),
                ("ins", LinWIns * LINW_MAXINS)]

RADIAL_MAXH = 3
GATE_MAXBLK = 8
CGC_MAXD = 256           # include/eelg.h EELG_CGC_MAXD
GATE_MAXGATED = 2048     # include/eelg.h EELG_GATE_MAXGATED / EELG_GATE_MAXGATES
GATE_MAXGATES = 512


class GateDesc(ctypes.Structure):
    _fields_ = [("n_scal", _I), ("n_gates", _I), ("n_blk", _I), ("pad", _I),
                ("blk_mul", _I * GATE_MAXBLK), ("blk_dim", _I * GATE_MAXBLK)]


SCG_MAXD = 25            # include/eelg.h EELG_SCG_MAXD / EELG_SCG_CHUNK
SCG_CHUNK = 256


class ScgDesc(ctypes.Structure):
    _fields_ = [("D", _I), ("Dout", _I), ("mul", _I), ("nterms", _I),
                ("xb", _I * SCG_MAXD), ("xs", _I * SCG_MAXD), ("ob", _I * SCG_MAXD),
                ("os", _I * SCG_MAXD), ("orow", _I * (SCG_MAXD + 1))]


class RadialDesc(ctypes.Structure):
    _fields_ = [("n_feat", _I), ("hidden", _I), ("n_hidden", _I), ("n_out", _I),
                ("w", _P * RADIAL_MAXH), ("b", _P * RADIAL_MAXH)]


EXPORTED_SYMBOLS = tuple(_SIGS)

_lib = None


class EELGError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise EELGError(
            f"{LIB_PATH} is missing: build it with `python -c \"import __graft_entry__ as g; g.build()\"` "
            "(there is no CPU fallback for the HIP hot path)")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, (args, res) in _SIGS.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if os.environ.get("EELG_LIB"):   # an older variant build (experiments): entry absent
                continue
            raise EELGError(f"{LIB_PATH} lacks {name}: stale build, rebuild the library")
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().eelg_last_error().decode(errors="replace")
        raise EELGError(f"{what} failed ({rc}): {msg}")


def ptr(t) -> ctypes.c_void_p:
    if t is None:
        return ctypes.c_void_p(0)
    return ctypes.c_void_p(t.data_ptr())


def stream(t: torch.Tensor) -> ctypes.c_void_p:
    """The current stream of ``t``'s device.  Kernels launch on the current HIP device, so
    ``t`` must live there (``torch.cuda.device(...)`` / ``torch.cuda.set_device``)."""
    dev = t.device
    cur = torch.cuda.current_device()
    if dev.index is not None and dev.index != cur:
        raise EELGError(f"operand on {dev} but the current HIP device is cuda:{cur}; run the "
                        f"model under torch.cuda.device({dev.index}) or set_device({dev.index})")
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def tp_config(name: str) -> Tuple[int, Dict[str, int], int]:
    lib = load()
    idx = lib.eelg_tp_find(name.encode())
    if idx < 0:
        check(idx, f"tp config {name}")
    info = (ctypes.c_int * 7)()
    sig = ctypes.c_uint64()
    check(lib.eelg_tp_info(idx, ctypes.cast(info, _P), ctypes.cast(ctypes.byref(sig), _P)), "tp_info")
    keys = ("din", "dmid", "wn", "nsh", "ngroups", "npaths", "lmax")
    return idx, dict(zip(keys, list(info))), sig.value


def sc_config(name: str) -> Tuple[int, Dict[str, int], int]:
    lib = load()
    idx = lib.eelg_sc_find(name.encode())
    if idx < 0:
        check(idx, f"sc config {name}")
    return (idx,) + _sc_info(idx)


def _tp_info(idx: int):
    info = (ctypes.c_int * 7)()
    sig = ctypes.c_uint64()
    rc = load().eelg_tp_info(idx, ctypes.cast(info, _P), ctypes.cast(ctypes.byref(sig), _P))
    if rc != 0:
        return None
    keys = ("din", "dmid", "wn", "nsh", "ngroups", "npaths", "lmax")
    return dict(zip(keys, list(info))), sig.value


def _sc_info(idx: int):
    info = (ctypes.c_int * 8)()
    sig = ctypes.c_uint64()
    rc = load().eelg_sc_info(idx, ctypes.cast(info, _P), ctypes.cast(ctypes.byref(sig), _P))
    if rc != 0:
        return None
    keys = ("D", "x_row", "out_row", "nterms", "njg", "Dout", "coef_chunk", "coef_ld")
    return dict(zip(keys, list(info))), sig.value


def _by_sig(getter, sig: int, what: str):
    idx = 0
    while True:
        got = getter(idx)
        if got is None:
            raise EELGError(f"libeelg.so has no generated {what} kernel with structure signature "
                            f"0x{sig:016x}; add the irreps to csrc/gen_kernels.py and rebuild")
        if got[1] == sig:
            return idx, got[0]
        idx += 1


def tp_config_by_sig(sig: int) -> Tuple[int, Dict[str, int]]:
    """The generated tensor-product kernel set whose structure hash is ``sig``."""
    return _by_sig(_tp_info, sig, "tensor-product")


def sc_config_by_sig(sig: int) -> Tuple[int, Dict[str, int]]:
    """The generated symmetric-contraction kernel set whose structure hash is ``sig``."""
    return _by_sig(_sc_info, sig, "symmetric-contraction")
