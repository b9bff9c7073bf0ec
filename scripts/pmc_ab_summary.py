"""step_kernel HBM bytes per evaluation from scripts/pmc_ab.sh's passes (FETCH_SIZE x2 for the
16-B/lane read streams, WRITE_SIZE as is; MI355X_MICROARCH.md §HBM), per library.

    python scripts/pmc_ab_summary.py liblfm liblfm_x ... [--json out.json]"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EVALS = 3  # bench.py --steps 2 --warmup 1


def main():
    args = [a for a in sys.argv[1:] if not a.endswith(".json") and a != "--json"]
    out = {}
    for lib in args:
        tot = {}
        for c in ("FETCH_SIZE", "WRITE_SIZE"):
            path = os.path.join(ROOT, "gpurun_out", f"pmc_{lib}_{c}", "run_counter_collection.csv")
            s, ids = 0.0, set()
            for r in csv.DictReader(open(path)):
                if r["Kernel_Name"].split("(")[0].endswith("step_kernel"):
                    s += float(r["Counter_Value"]) * 1024.0
                    ids.add(r["Dispatch_Id"])
            tot[c] = (s, len(ids))
        rd = 2.0 * tot["FETCH_SIZE"][0] / EVALS
        wr = tot["WRITE_SIZE"][0] / EVALS
        out[lib] = {"launches": tot["FETCH_SIZE"][1], "read_bytes_per_eval_x2": rd,
                    "write_bytes_per_eval": wr, "hbm_bytes_per_eval": rd + wr}
        print(f"{lib}: read (x2) {rd / 1e9:.1f} GB/eval, write {wr / 1e9:.1f} GB/eval, "
              f"total {(rd + wr) / 1e9:.1f} GB/eval over {tot['FETCH_SIZE'][1]} launches")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
