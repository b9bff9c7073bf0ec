"""Per-dispatch FETCH_SIZE / WRITE_SIZE of the step kernel in scripts/pmc_calib.sh's passes
against the known C bytes (T = 127 full triangle of 128-tiles): the counters' scale for the
trailing update's 8-B-per-lane C access, and the panel-read bytes that remain.

    python scripts/pmc_calib_summary.py [--json out.json]"""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
T = 127
C_BYTES = T * (T + 1) // 2 * 128 * 128 * 8


def per_dispatch(cio, counter):
    path = os.path.join(ROOT, "gpurun_out", f"calib_{cio}_{counter}", "run_counter_collection.csv")
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].split("(")[0].endswith("step_kernel"):
            vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"]) * 1024.0
    v = sorted(vals.values())
    return v[len(v) // 2], len(v)  # median over the probe's launches


def main():
    out = {"c_bytes": C_BYTES}
    for cio in (88, 120):
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            out[f"{cio}_{c}"], out[f"{cio}_launches"] = per_dispatch(cio, c)
    fetch_c = out["88_FETCH_SIZE"] - out["120_FETCH_SIZE"]
    out["fetch_scale_c"] = fetch_c / C_BYTES          # raw FETCH_SIZE bytes per C byte read
    out["write_scale_c"] = out["120_WRITE_SIZE"] / C_BYTES  # raw WRITE_SIZE per C byte written
    out["panel_fetch_raw"] = out["120_FETCH_SIZE"]
    for k, v in out.items():
        print(f"{k}: {v:.4g}" if isinstance(v, float) else f"{k}: {v}")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
