#!/usr/bin/env python3
"""VGPR / SGPR / LDS / spill usage of every kernel in gnn/libeelg.so (from the code-object
metadata notes; no GPU needed).  usage: python tools/kernel_resources.py [regex]"""
import os, re, subprocess, sys, tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
so = os.environ.get("EELG_LIB") or os.path.join(ROOT, "energy-equiv-lattice-gnn_amd", "gnn", "libeelg.so")
pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else ".")
with tempfile.TemporaryDirectory() as d:
    fb = os.path.join(d, "fb.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", so], check=True)
    data = open(fb, "rb").read()
    # the section holds one offload bundle per translation unit, each 4096-aligned
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    rows = []
    for i, s in enumerate(starts):
        part = os.path.join(d, f"b{i}.bin")
        open(part, "wb").write(data[s: starts[i + 1] if i + 1 < len(starts) else len(data)])
        co = os.path.join(d, f"b{i}.co")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"],
                           capture_output=True)
        if r.returncode:
            continue
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True,
                               text=True).stdout
        cur = {}
        for ln in notes.splitlines():
            ln = ln.strip()
            for key in (".name:", ".vgpr_count:", ".sgpr_count:", ".agpr_count:",
                        ".group_segment_fixed_size:", ".vgpr_spill_count:", ".sgpr_spill_count:",
                        ".private_segment_fixed_size:"):
                if ln.startswith("- " + key) or ln.startswith(key):
                    k = key.strip(".:")
                    cur[k] = ln.split(":", 1)[1].strip()
                    if k == "name" and "vgpr_count" in cur:
                        pass
            if ln.startswith(".wavefront_size:") or ln.startswith("- .wavefront_size:"):
                if "name" in cur:
                    rows.append(cur)
                cur = {}
    for r in rows:
        if pat.search(r.get("name", "")):
            print(f"{r.get('vgpr_count','?'):>4} v {r.get('agpr_count','?'):>4} a {r.get('sgpr_count','?'):>4} s "
                  f"lds {r.get('group_segment_fixed_size','?'):>6} scratch {r.get('private_segment_fixed_size','?'):>5} "
                  f"spill v{r.get('vgpr_spill_count','?')} s{r.get('sgpr_spill_count','?')}  {r['name'][:90]}")
