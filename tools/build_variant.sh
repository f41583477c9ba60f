#!/bin/bash
# Build a kernel variant of libeelg.so into variants/libeelg_<tag>.so with generator env overrides
# (EELG_* knobs of csrc/gen_kernels.py) and optional EXTRA hipcc flags, through the same Makefile.
# usage: EELG_TP_MAXACC=48 tools/build_variant.sh <tag>     (load it with EELG_LIB=...)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
T=/tmp/eelg_var_$1
rm -rf "$T"; mkdir -p "$T/a/p" "$R/variants"
cp -r "$R/energy-equiv-lattice-gnn_amd/csrc" "$T/a/p/csrc"
cp -r "$R/energy-equiv-lattice-gnn_amd/gnn" "$T/a/p/gnn"
cp -r "$R/include" "$T/a/include"
rm -rf "$T/a/p/csrc/build" "$T/a/p/csrc/generated"
make -s -j4 -C "$T/a/p/csrc" OUT="$R/variants/libeelg_$1.so" > "$T/build.log" 2>&1 || { tail -20 "$T/build.log"; exit 1; }
echo "built variants/libeelg_$1.so"
