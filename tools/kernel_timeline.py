"""Print the kernel timeline of one step from a rocprofv3 --kernel-trace CSV: every dispatch between
the last two dispatches of MARKER (a kernel that runs once per step), with its start offset from the
step's first dispatch, its duration and its grid, plus the step's span and the busy union.
    python tools/kernel_timeline.py gpurun_out/<dir> [MARKER|all] [STEP_FROM_END]
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else None
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    f = d if d.endswith(".csv") else glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if marker == "all":  # every dispatch but empty warm-up ones
        sel = [r for r in rows if "warm" not in r["Kernel_Name"]]
    elif marker:
        idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
        lo, hi = idx[-1 - back], idx[-back]
        sel = rows[lo:hi]
    else:
        sel = rows[-40:]
    t0 = int(sel[0]["Start_Timestamp"])
    busy, last_end = 0, t0
    for r in sel:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e > last_end:
            busy += e - max(s, last_end)
            last_end = e
        grid = r.get("Grid_Size_X") or r.get("Grid_Size") or ""
        wg = r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or ""
        q = r.get("Stream_Id") or r.get("Queue_Id") or ""
        print(f"{(s - t0) / 1e3:9.1f} us +{(e - s) / 1e3:8.1f} us  q {q:>3} grid {grid:>8} wg {wg:>4}  {r['Kernel_Name'][:90]}")
    span = (int(sel[-1]["End_Timestamp"]) - t0) / 1e3
    print(f"span {span:.1f} us, busy {busy / 1e3:.1f} us, {len(sel)} dispatches")


if __name__ == "__main__":
    main()
