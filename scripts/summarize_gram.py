"""Gram-fill roofline evidence from one round's rocprofv3 output (scripts/profile_r03.sh):

  gpurun_out/prof_c4/        --kernel-trace --stats of `bench.py --workload c4` (fp32, N = 65536)
  gpurun_out/prof_c4_write/  --pmc WRITE_SIZE of the same fill
  gpurun_out/prof_unfused/   --kernel-trace --stats of the C2 bench with LFM_GRAM_FUSE=0 (fp64
                             lower fill of N = 16384 as its own kernel)
  gpurun_out/prof_unfused_write/  --pmc WRITE_SIZE of that run

writes profiles/<round>_gram.json and profiles/<round>_gram_trace.md: per fill, the rocprof average
duration of gram_grid_aligned_kernel, the algorithmic bytes (elem bytes x N (N + 1) / 2, the
lower triangle with its diagonal), achieved GB/s and the fraction of the 8 TB/s spec, the
WRITE_SIZE bytes per launch (exact for streaming stores, MI355X_MICROARCH.md §HBM), and the
traced bench line's own HIP-event figure beside it.

    python scripts/summarize_gram.py r03
"""

import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")
HBM_PEAK_GBS = 8000.0


def short(name):
    return name.split("(")[0].replace("void ", "").replace("lfm::", "")


def gram_row(stats_csv):
    for r in csv.DictReader(open(stats_csv)):
        if short(r["Name"]).startswith("gram_grid_aligned_kernel"):
            return r
    return None


def write_bytes(pmc_csv):
    per = {}
    for r in csv.DictReader(open(pmc_csv)):
        if r["Counter_Name"] != "WRITE_SIZE" or not short(r["Kernel_Name"]).startswith(
                "gram_grid_aligned_kernel"):
            continue
        per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"]) * 1024
    return (sum(per.values()) / len(per), len(per)) if per else (None, 0)


def one(tag, trace_dir, pmc_dir, bench_json, n, elem):
    stats = os.path.join(OUT, trace_dir, "run_kernel_stats.csv")
    row = gram_row(stats)
    if row is None:
        raise SystemExit(f"{stats}: no gram_grid_aligned_kernel row")
    avg_s = float(row["AverageNs"]) * 1e-9
    alg = elem * n * (n + 1) / 2.0
    gbs = alg / avg_s / 1e9
    wb, nw = write_bytes(os.path.join(OUT, pmc_dir, "run_counter_collection.csv"))
    bench = None
    bj = os.path.join(OUT, bench_json)
    if os.path.exists(bj) and open(bj).read().strip():
        bench = json.loads(open(bj).read().strip().splitlines()[-1])
    rec = {"fill": tag, "kernel": short(row["Name"]), "calls": int(row["Calls"]),
           "rocprof_avg_us": avg_s * 1e6, "algorithmic_bytes_per_launch": alg,
           "achieved_gbs": gbs, "peak_gbs": HBM_PEAK_GBS, "frac": gbs / HBM_PEAK_GBS,
           "pmc_write_bytes_per_launch": wb, "pmc_write_launches": nw,
           "pmc_write_over_algorithmic": wb / alg if wb else None}
    if bench:
        rf = bench.get("gram_roofline") or (
            bench.get("roofline") if bench.get("roofline", {}).get("bound") == "hbm" else None)
        rec["traced_bench_line"] = {"value": bench["value"], "unit": bench["unit"],
                                    "ms_per_step": bench["ms_per_step"]}
        if rf:
            rec["traced_bench_line"].update(hip_event_avg_ms=rf["avg_launch_ms"],
                                            hip_event_frac=rf["frac"])
    return rec


def main():
    rnd = sys.argv[1]
    recs = [one("C4: fp32, N = 65536 (bench.py --workload c4)", "prof_c4", "prof_c4_write",
                "prof_c4_bench.json", 65536, 4),
            one("C2 unfused: fp64, N = 16384 (LFM_GRAM_FUSE=0)", "prof_unfused",
                "prof_unfused_write", "prof_unfused_bench.json", 16384, 8)]
    json.dump(recs, open(os.path.join(PROF, f"{rnd}_gram.json"), "w"), indent=1)
    shutil.copy(os.path.join(OUT, "prof_c4", "run_kernel_stats.csv"),
                os.path.join(PROF, f"{rnd}_gram_c4_kernel_stats.csv"))
    shutil.copy(os.path.join(OUT, "prof_unfused", "run_kernel_stats.csv"),
                os.path.join(PROF, f"{rnd}_gram_unfused_kernel_stats.csv"))
    lines = [f"# {rnd}: gram fill roofline (rocprofv3 kernel trace + WRITE_SIZE pass)", "",
             "| fill | kernel | avg us (rocprof) | algorithmic B / launch | GB/s | frac of 8 TB/s | "
             "PMC WRITE_SIZE B / launch | WRITE / alg | bench HIP-event frac |",
             "|---|---|---|---|---|---|---|---|---|"]
    for r in recs:
        tb = r.get("traced_bench_line", {})
        lines.append(
            f"| {r['fill']} | {r['kernel']} | {r['rocprof_avg_us']:.1f} | "
            f"{r['algorithmic_bytes_per_launch']:.4e} | {r['achieved_gbs']:.0f} | "
            f"**{r['frac']:.3f}** | "
            + (f"{r['pmc_write_bytes_per_launch']:.4e} | {r['pmc_write_over_algorithmic']:.3f}"
               if r["pmc_write_bytes_per_launch"] else "n/a | n/a")
            + f" | {tb.get('hip_event_frac', float('nan')):.3f} |")
    lines += ["", "Algorithmic bytes: the lower triangle with its diagonal, elem x N (N + 1) / 2 "
              "(the fill writes nothing above the diagonal: tests/test_gpu_regimes.py checks a "
              "0xFF sentinel there)."]
    open(os.path.join(PROF, f"{rnd}_gram_trace.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
