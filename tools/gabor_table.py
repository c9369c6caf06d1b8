#!/usr/bin/env python3
"""Per-scale Gabor table of a HEAD snapshot: time, registers, occupancy, FP32 fraction and PMC traffic side by side.

Inputs (one snapshot directory, profiles/<tag>/):
  bench.json          the bench line (stage_ms_per_step, gabor_fp32)
  traffic.json        PMC FETCH_SIZE x2 + WRITE_SIZE per kernel (tools/pmc_traffic.py)
  kernel_resources.json  compiler figures per kernel (tools/kernel_resources.py)
Writes profiles/<tag>/gabor_scales.json and prints a Markdown table.
Occupancy: the compiler's register bound (waves / SIMD), then the launch's: workgroups per CU from the static plus
dynamic LDS (the staged face of the batch's tallest face, gabor_face_lds) and the
register bound, times waves per workgroup / 4 SIMDs.

usage: tools/gabor_table.py profiles/<tag> [max_face_h]
"""
import json
import os
import sys

LDS_CU = 160 * 1024
PITCH = 128  # ffd_device.hpp
# the batch instance each scale launches at C2 (FFD_GS_CPT2S_MASK 18, FFD_GS_CPT2_MASK 12)
INSTANCE = {
    "7x7": ("void ffd::k_gabor7<false, false>", 512),
    "9x9": ("void ffd::k_gabor_sep<9, false, false, false, 2, 4>", 256),
    "13x13": ("void ffd::k_gabor_sep<13, false, false, false, 2, 8>", 512),
    "19x19": ("void ffd::k_gabor_sep<19, false, false, false, 2, 8>", 512),
    "25x25": ("void ffd::k_gabor_sep<25, false, false, false, 2, 4>", 256),
}


def find(table, prefix):
    for k, v in table.items():
        if k.startswith(prefix + "("):
            return k, v
    raise KeyError(prefix)


def main():
    d = sys.argv[1]
    max_h = int(sys.argv[2]) if len(sys.argv) > 2 else 150
    bench = json.loads(open(os.path.join(d, "bench.json")).read().strip().splitlines()[-1])
    traffic = json.load(open(os.path.join(d, "traffic.json")))["kernels"]
    res = json.load(open(os.path.join(d, "kernel_resources.json")))["kernels"]
    stages = bench["stage_ms_per_step"]
    fp32 = bench.get("gabor_fp32", {}).get("per_scale", {})
    rows = []
    for scale, (prefix, threads) in INSTANCE.items():
        name, r = find(res, prefix)
        w = int(scale.split("x")[0])
        R = (w - 1) // 2
        dyn = 0 if w == 7 else ((max_h + 7) // 8 * 8 + 2 * R) * ((PITCH + 2 * R + 3) // 4 * 4)  # gabor_face_lds
        lds = r["static_lds_bytes"] + dyn
        waves_wg = threads // 64
        wg_lds = LDS_CU // max(lds, 1)
        wg_regs = r["occupancy_waves_per_simd"] * 4 // waves_wg
        wg = max(0, min(wg_lds, wg_regs))
        alts = [prefix, prefix.replace(", 4, 8>", ">")]  # (a demangler may print default template arguments or not)
        tkey = next((k for a in alts for k in traffic if k.startswith(a + "(")), None)
        t = traffic.get(tkey, {})
        per_launch = t.get("traffic_bytes", 0)  # (tools/pmc_traffic.py: already the average per launch)
        rows.append({
            "scale": scale, "kernel": name, "ms": stages.get("gabor_" + scale), "threads": threads,
            "vgprs": r["vgprs"], "sgprs": r["sgprs"], "sgpr_spills": r["sgpr_spills"], "vgpr_spills": r["vgpr_spills"],
            "occupancy_regs_waves_per_simd": r["occupancy_waves_per_simd"], "lds_bytes": lds,
            "workgroups_per_cu": wg, "waves_per_simd": wg * waves_wg / 4,
            "fp32_frac": fp32.get("gabor_" + scale, {}).get("fp32_frac"),
            "pmc_traffic_GB_per_launch": round(per_launch / 1e9, 3) if per_launch else None,
        })
    out = {"source": d, "max_face_h": max_h, "scales": rows,
           "note": "ms = bench HIP-event stage time per step (C2, 4,096 faces); registers from the compiler "
                   "(tools/kernel_resources.py); traffic = PMC FETCH_SIZE x2 + WRITE_SIZE per launch"}
    with open(os.path.join(d, "gabor_scales.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("| scale | instance threads | ms | VGPRs | SGPR spills | LDS B | WG/CU | waves/SIMD | FP32 frac | PMC GB/launch |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for r in rows:
        print(f"| {r['scale']} | {r['threads']} | {r['ms']} | {r['vgprs']} | {r['sgpr_spills']} | {r['lds_bytes']} | "
              f"{r['workgroups_per_cu']} | {r['waves_per_simd']:g} | {r['fp32_frac']} | {r['pmc_traffic_GB_per_launch']} |")


if __name__ == "__main__":
    main()
