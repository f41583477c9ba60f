#!/usr/bin/env python3
"""Disassembly of kernels in gnn/libeelg.so (no GPU needed): the instruction histogram of every
kernel whose name matches a regex, or its full listing.

  python tools/kernel_isa.py <regex> [--list] [--top N]
"""
import argparse
import collections
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(so, d):
    fb = os.path.join(d, "fb.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", so], check=True)
    data = open(fb, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    for i, s in enumerate(starts):
        part = os.path.join(d, f"b{i}.bin")
        open(part, "wb").write(data[s: starts[i + 1] if i + 1 < len(starts) else len(data)])
        co = os.path.join(d, f"b{i}.co")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                           capture_output=True)
        if r.returncode == 0:
            yield co


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("regex")
    ap.add_argument("--list", action="store_true")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    so = os.environ.get("EELG_LIB") or os.path.join(ROOT, "energy-equiv-lattice-gnn_amd", "gnn", "libeelg.so")
    pat = re.compile(a.regex)
    with tempfile.TemporaryDirectory() as d:
        for co in code_objects(so, d):
            dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co],
                                 capture_output=True, text=True).stdout
            cur, body = None, []
            for ln in dis.splitlines() + ["<end>:"]:
                m = re.match(r"^[0-9a-f]+ <(.+)>:$", ln) or (ln == "<end>:" and re.match("(.*)", ""))
                if m:
                    if cur and pat.search(cur):
                        ops = [b.split()[0] for b in body if b.strip() and not b.strip().startswith(";")]
                        print(f"== {cur}: {len(ops)} instructions")
                        if a.list:
                            print("\n".join(body))
                        for op, n in collections.Counter(ops).most_common(a.top):
                            print(f"  {n:7d} {op}")
                    cur, body = (m.group(1) if ln != "<end>:" else None), []
                elif cur:
                    body.append(ln.strip())


if __name__ == "__main__":
    main()
