"""Per-dispatch counter totals of kernels matching a substring in a rocprofv3 --pmc CSV directory.
    python tools/pmc_kernel.py DIR SUBSTRING [SUBSTRING...]"""
import collections
import csv
import os
import sys

d = sys.argv[1]
rows = list(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))))
agg = collections.OrderedDict()
for r in rows:
    if not any(s in r["Kernel_Name"] for s in sys.argv[2:]):
        continue
    key = (r["Kernel_Name"][:60], r["Dispatch_Id"])
    e = agg.setdefault(key, {"ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6,
                             "grid": r["Grid_Size"], "lds": r["LDS_Block_Size"], "vgpr": r["VGPR_Count"]})
    e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for (k, did), e in agg.items():
    ms = e.pop("ms")
    print(f"{k} #{did} ms={ms:.3f} " + " ".join(f"{c}={v:.4g}" if isinstance(v, float) else f"{c}={v}" for c, v in e.items()))
    if "GRBM_GUI_ACTIVE" in e:
        print(f"   clock ~ {e['GRBM_GUI_ACTIVE'] / 8 / ms / 1e6:.2f} GHz (GRBM/8 XCDs)")
    if "SQ_WAVE_CYCLES" in e and "SQ_WAIT_ANY" in e:
        w = e["SQ_WAVE_CYCLES"]
        print(f"   wave time: active {e.get('SQ_ACTIVE_INST_ANY', 0) / w:.2f} wait_inst {e.get('SQ_WAIT_INST_ANY', 0) / w:.2f} wait_any {e['SQ_WAIT_ANY'] / w:.2f}")
