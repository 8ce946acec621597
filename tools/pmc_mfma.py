#!/usr/bin/env python3
"""MFMA utilisation per kernel from one rocprofv3 --pmc pass of
SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT (tools/gpu_session.sh pmc_mfma).

Units (MI355X_MICROARCH.md, 'Per-instruction cycle constants' and 'DVFS give-back'): GRBM_GUI_ACTIVE is the
sum over the 8 XCDs of the cycles the GPU was busy, so a dispatch lasted GRBM_GUI_ACTIVE / 8 cycles;
SQ_VALU_MFMA_BUSY_CYCLES counts matrix-core busy cycles summed over every SIMD (32 per v_mfma_f32_32x32x16_bf16),
so the fraction of the chip's matrix-core cycles in use during the dispatch is
    mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
(256 CUs x 4 SIMDs).  That is the issued-MFMA fraction of the dense peak (bf16 kernels: of 2.5 PF; the f32-MFMA
prefill attention: of its own 157 TF rate, every f32 MFMA being busy 64 cycles).

usage: pmc_mfma.py <pmc_counter_collection.csv> <out.json>
"""
import csv
import json
import re
import sys
from collections import defaultdict

SIMDS = 1024
STAGES = {
    "vision": ("gemm_f32a_nt_kernel<false", "attention_split_kernel", "splitk_reduce4", "layernorm_kernel",
               "conv_im2col", "patch_im2col", "sam_relbias2", "clip_embed", "concat_clip_sam", "add_broadcast"),
    "prefill": ("gemm_f32a_nt_kernel<true", "gemm_f32a_grp_kernel", "attention_fwd2_kernel", "attention_merge",
                "rmsnorm_kernel", "rope_kv_kernel", "moe_group_kernel", "moe_combine", "router_topk", "silu_mul",
                "assemble_rows"),
}


def short(n):
    return re.sub(r"^void ", "", n).replace("dsocr::", "").split("(")[0]


def main():
    src, out = sys.argv[1], sys.argv[2]
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(dict)
    for r in csv.DictReader(open(src)):
        k = short(r["Kernel_Name"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
    kernels = {}
    for k, c in per.items():
        n = len(disp[k])
        cyc = c.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        us = sum(disp[k].values())
        kernels[k] = {"launches": n, "us_per_launch": us / n if n else 0.0,
                      "clock_ghz": cyc / us / 1e3 if us else 0.0, "cycles_per_launch": cyc / n if n else 0.0,
                      "mfma_busy_cycles_per_launch": busy / n if n else 0.0,
                      "mfma_busy": busy / (cyc * SIMDS) if cyc else 0.0,
                      "sq_busy_per_xcd_cycle": c.get("SQ_BUSY_CYCLES", 0.0) / cyc if cyc else 0.0}
    stages = {}
    for st, pats in STAGES.items():
        ks = [k for k in kernels if any(k.startswith(p) for p in pats)]
        cyc = sum(kernels[k]["cycles_per_launch"] * kernels[k]["launches"] for k in ks)
        busy = sum(kernels[k]["mfma_busy_cycles_per_launch"] * kernels[k]["launches"] for k in ks)
        us = sum(kernels[k]["us_per_launch"] * kernels[k]["launches"] for k in ks)
        stages[st] = {"kernels": sorted(ks), "gpu_cycles": cyc, "dispatch_us": us,
                      "mfma_busy": busy / (cyc * SIMDS) if cyc else 0.0}
    res = {"source": src, "formula": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)",
           "note": "eager launches (DSOCR_NO_GRAPH=1), one 1024x1024 bench page; stage = the kernels' summed busy "
                   "cycles over their summed dispatch cycles (the stage's time between dispatches not counted)",
           "stages": stages, "kernels": kernels}
    json.dump(res, open(out, "w"), indent=1)
    for st, v in stages.items():
        print(f"{st:8s} mfma_busy {v['mfma_busy']:.3f} over {v['dispatch_us']:.0f} us of dispatches")
    for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["mfma_busy_cycles_per_launch"] * kv[1]["launches"])[:10]:
        print(f"  {k[:48]:48s} n {v['launches']:4d} {v['us_per_launch']:9.1f} us/launch {v['clock_ghz']:.2f} GHz  "
              f"mfma_busy {v['mfma_busy']:.3f}")


if __name__ == "__main__":
    main()
