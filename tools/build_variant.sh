#!/bin/bash
# Build a kernel variant of libeelg.so into variants/libeelg_<tag>.so with generator env overrides.
# usage: EELG_TP_NPH=8 EELG_TP_MAXACC=24 tools/build_variant.sh <tag>
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=/tmp/eelg_var_$1
rm -rf "$T"; mkdir -p "$T/a/p" "$R/variants"
cp -r "$R/energy-equiv-lattice-gnn_amd/csrc" "$T/a/p/csrc"
cp -r "$R/energy-equiv-lattice-gnn_amd/gnn" "$T/a/p/gnn"
cp -r "$R/include" "$T/a/include"
cd "$T/a/p/csrc"
python3 gen_kernels.py generated > /dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -mcode-object-version=5 -fno-gpu-rdc -fno-slp-vectorize \
  -Wno-unused-variable -Wno-unused-result $EXTRA_FLAGS -Rpass-analysis=kernel-resource-usage \
  -o "$R/variants/libeelg_$1.so" eelg_capi.hip > "$T/ru.log" 2>&1
grep -A7 "Name: _Z13tp_fwd_tpB_l4" "$T/ru.log" | grep -E "VGPRs:|Spill|Occupancy" | sed "s/^/$1 /"
