"""MFMA utilisation from rocprofv3 PMC passes (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE): per
dispatch of the named kernel, busy SIMD-cycles / (GPU-active cycles per XCD x CUs x 4 SIMDs).
GRBM_GUI_ACTIVE is summed over the 8 XCDs (its per-XCD value over the dispatch's duration is the
shader clock); SQ_VALU_MFMA_BUSY_CYCLES is summed over every SIMD.

    python scripts/pmc_mfma_summary.py gpurun_out/<pass dir> KERNEL CUS [--json out.json]"""
import collections
import csv
import json
import os
import sys


def main():
    d, kern, cus = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = collections.defaultdict(dict)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Kernel_Name"].split("(")[0].split("<")[0].endswith(kern):
            k = int(r["Dispatch_Id"])
            rows[k][r["Counter_Name"]] = rows[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            if "Start_Timestamp" in r and r.get("End_Timestamp"):
                rows[k]["dur_ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    out = []
    for k in sorted(rows):
        v = rows[k]
        g = v.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
        busy = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        e = {"dispatch": k, "mfma_busy_frac": busy / (g * cus * 4) if g else None}
        if v.get("dur_ms"):
            e["dur_ms"] = v["dur_ms"]
            e["clock_ghz"] = g / (v["dur_ms"] * 1e6)
        out.append(e)
    fr = [e["mfma_busy_frac"] for e in out if e["mfma_busy_frac"] is not None]
    # time-weighted over the dispatches that have durations
    tw = [(e["mfma_busy_frac"], e["dur_ms"]) for e in out if e.get("dur_ms") and e["mfma_busy_frac"]]
    summ = {"kernel": kern, "cus": cus, "dispatches": len(out),
            "mfma_busy_frac_mean": sum(fr) / len(fr) if fr else None,
            "mfma_busy_frac_time_weighted": (sum(f * t for f, t in tw) / sum(t for _, t in tw)
                                             if tw else None)}
    print(json.dumps(summ))
    if "--json" in sys.argv:
        json.dump({"summary": summ, "dispatches": out},
                  open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
