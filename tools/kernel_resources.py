#!/usr/bin/env python3
"""Per-kernel register / LDS / occupancy figures of the product kernels, from the compiler itself.

Compiles csrc/ffd_kernels.hip (and ffd_haar.hip) for gfx950 with the build's flags plus
-Rpass-analysis=kernel-resource-usage and parses the remarks: VGPRs, AGPRs, SGPRs, spills, scratch, static
LDS and the compiler's occupancy bound (waves per SIMD from registers and static LDS; dynamic LDS — the
Gabor kernels' staged face, the traversal's window — lowers it further at launch).  CPU only.

usage: tools/kernel_resources.py OUT.json [FILTER ...]   (FILTER: substrings of demangled names to keep)
"""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = ["face_alignment_cvpr_2012_amd/csrc/ffd_kernels.hip", "face_alignment_cvpr_2012_amd/csrc/ffd_haar.hip"]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wno-unused-function",
         "-Iinclude", "-Rpass-analysis=kernel-resource-usage"]
KEYS = {"TotalSGPRs": "sgprs", "VGPRs": "vgprs", "AGPRs": "agprs", "ScratchSize [bytes/lane]": "scratch_bytes_per_lane",
        "Occupancy [waves/SIMD]": "occupancy_waves_per_simd", "SGPRs Spill": "sgpr_spills", "VGPRs Spill": "vgpr_spills",
        "LDS Size [bytes/block]": "static_lds_bytes"}


def demangle(names):
    filt = "c++filt"
    out = subprocess.run([filt], input="\n".join(names), capture_output=True, text=True, check=True).stdout
    return out.strip().split("\n")


def resources(src):
    r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, "-c", src, "-o", os.devnull], cwd=ROOT, capture_output=True,
                       text=True)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-3000:])
    funcs, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = funcs.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:\s+(.+?): (\S+) \[-Rpass-analysis", line)
        if m and cur is not None and m.group(1) in KEYS:
            v = m.group(2)
            cur[KEYS[m.group(1)]] = v if v in ("True", "False") else int(v)
    return funcs


def main():
    out, filters = sys.argv[1], sys.argv[2:]
    funcs = {}
    for s in SRCS:
        funcs.update(resources(s))
    names = list(funcs)
    table = {}
    for mangled, dem in zip(names, demangle(names)):
        if filters and not any(f in dem for f in filters):
            continue
        table[dem] = funcs[mangled]
    with open(out, "w") as f:
        json.dump({"arch": "gfx950", "flags": " ".join(FLAGS), "kernels": table}, f, indent=1, sort_keys=True)
    print(f"{len(table)} kernels -> {out}")


if __name__ == "__main__":
    main()
