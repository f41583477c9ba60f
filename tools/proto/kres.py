#!/usr/bin/env python3
"""Quick register / LDS check of one generated kernel without the full library build:
generate with the current EELG_* env knobs, cut the preamble + the named kernel into a small
translation unit, compile for gfx950 and print the compiler's resource-usage remarks.
usage: EELG_TP_MAXACC=48 python tools/proto/kres.py tp_fwd_tpB_l4 [more kernels...]"""
import os, re, subprocess, sys, tempfile
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CS = os.path.join(ROOT, "energy-equiv-lattice-gnn_amd", "csrc")
with tempfile.TemporaryDirectory() as d:
    subprocess.run([sys.executable, os.path.join(CS, "gen_kernels.py"), d], check=True, capture_output=True)
    src = open(os.path.join(d, "eelg_gen.hip")).read().split("\n")
    pre = []
    for ln in src:
        if ln.startswith("__global__"):
            break
        pre.append(ln)
    pre = [ln.replace('"../eelg_internal.h"', f'"{CS}/eelg_internal.h"') for ln in pre]
    body = []
    for name in sys.argv[1:]:
        start = next(i for i, ln in enumerate(src) if re.search(rf"void {name}\(", ln))
        i = start
        while not src[i].startswith("__global__"):
            i -= 1
        # the config section's device helpers (e.g. sc_goff_*) precede its first kernel
        k = i
        while k > 0 and not src[k].startswith("// ====="):
            k -= 1
        helpers, inside = [], False
        for ln in src[k:i]:
            if ln.startswith("__device__"):
                inside = True
            if inside:
                helpers.append(ln)
            if inside and ln.startswith("}"):
                inside = False
        body += [ln for ln in helpers if ln not in body]
        j = start + 1
        while j < len(src) and not src[j].startswith("__global__") and not src[j].startswith("// ====="):
            j += 1
        body += src[i:j]
    tu = os.path.join(d, "k.hip")
    open(tu, "w").write("\n".join(pre + body) + "\n")
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-fno-slp-vectorize", "--cuda-device-only", "-c", "-o", os.path.join(d, "k.o"),
                        "-Rpass-analysis=kernel-resource-usage", tu], capture_output=True, text=True)
    for ln in r.stderr.split("\n"):
        if "remark" in ln and any(k in ln for k in ("Function Name", "VGPRs:", "SGPRs:", "Occupancy", "LDS Size", "ScratchSize")):
            print(ln.split("remark: ")[-1])
    if r.returncode:
        print(r.stderr[-3000:])
    if os.environ.get("KRES_ASM"):   # also write the kernel's assembly there
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-fno-slp-vectorize", "--cuda-device-only", "-S", "-o", os.environ["KRES_ASM"], tu],
                       check=True)
