"""Summarise the LDS / VALU counter passes of tools/gpu_lds.sh into profiles/<tag>_lds.json: per hot
kernel, summed over its dispatches, SQ_LDS_BANK_CONFLICT (extra LDS cycles from bank conflicts),
SQ_LDS_IDX_ACTIVE (all LDS-array cycles), SQ_INSTS_LDS, SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU,
SQ_WAVE_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE, and the derived ratios
  lds_conflict_frac = BANK_CONFLICT / IDX_ACTIVE   (share of LDS cycles lost to conflicts)
  valu_busy         = ACTIVE_INST_VALU / WAVE_CYCLES (share of a wave's life spent issuing VALU)
  valu_per_simd_cycle = INSTS_VALU / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs): wave-instructions per
                      SIMD-cycle over the kernel's life (tools/probes/valu_rate.hip: 0.40 for v_add_f32 /
                      v_mul_f32 / v_add_u32, ~0.23 for most other VALU and DPP forms, profiles/r04j_valu_rate.log).
    python tools/pmc_lds.py profiles/TAG_lds.json gpurun_out/lds_phmm gpurun_out/lds_chain ...
"""
import collections
import csv
import json
import os
import sys

from pmc_summary import name_of

CTR = ["SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU",
       "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"]


def main():
    out_path, dirs = sys.argv[1], sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for d in dirs:
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            n = name_of(r)
            if not n or r["Counter_Name"] not in CTR:
                continue
            acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[n].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    res = {}
    for n, c in acc.items():
        e = dict(c)
        e["dispatches"] = len(disp[n])
        if c["SQ_LDS_IDX_ACTIVE"]:
            e["lds_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
        if c["SQ_WAVE_CYCLES"]:
            e["valu_busy"] = c["SQ_ACTIVE_INST_VALU"] / c["SQ_WAVE_CYCLES"]
        if c["GRBM_GUI_ACTIVE"]:
            e["valu_per_simd_cycle"] = c["SQ_INSTS_VALU"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024)
        res[n] = e
    json.dump(res, open(out_path, "w"), indent=1)
    for n, e in sorted(res.items()):
        print(f"{n:24s} conflict {e.get('lds_conflict_frac', 0):.4f}  valu_busy {e.get('valu_busy', 0):.3f}  "
              f"valu/SIMD-cycle {e.get('valu_per_simd_cycle', 0):.3f}  lds_insts {e['SQ_INSTS_LDS']:.3g}  valu_insts {e['SQ_INSTS_VALU']:.3g}")


if __name__ == "__main__":
    main()
