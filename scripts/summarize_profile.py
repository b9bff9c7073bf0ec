"""Turn one round's rocprofv3 output (gpurun_out/prof_trace, prof_fetch, prof_write) into the
committed summaries under profiles/:

  profiles/<round>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as produced)
  profiles/<round>_kernels.md         per-kernel table: calls, avg / total us, share
  profiles/<round>_hbm.json           per-kernel FETCH_SIZE / WRITE_SIZE per launch
  profiles/syrk_traffic.json          SYRK HBM bytes per launch (read by bench.py)

HBM accounting follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
FETCH_SIZE reads half of the bytes of a wide (16 B/lane) coalesced stream on gfx950, so
the read side is reported raw and x2-corrected; WRITE_SIZE is exact for 16-B stores and
uncalibrated for 8-B stores (the SYRK's C stores are 8 B/lane, 128-B rows per 16 lanes).

    python scripts/summarize_profile.py r01 [bench_json]
"""

import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def short(name):
    return name.split("(")[0].replace("void ", "").replace("lfm::", "")


def main():
    rnd = sys.argv[1]
    os.makedirs(PROF, exist_ok=True)
    stats = os.path.join(OUT, "prof_trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(PROF, f"{rnd}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    traced = None
    tb = os.path.join(OUT, "prof_trace_bench.json")
    if os.path.exists(tb) and open(tb).read().strip():
        traced = json.loads(open(tb).read().strip().splitlines()[-1])
    evals_traced = (traced["steps"] + traced["warmup"]) if traced else None
    lines = [f"# {rnd}: rocprofv3 --kernel-trace --stats, `bench.py --steps 5 --warmup 2 "
             "--no-cpu-baseline` (7 evaluations at N = 16384)", "",
             "| kernel | calls | avg us | total ms | share % |", "|---|---|---|---|---|"]
    for r in rows:
        lines.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.2f} |")
    hbm = defaultdict(lambda: {"launches": 0, "FETCH_SIZE_KiB": 0.0, "WRITE_SIZE_KiB": 0.0})
    # per dispatch, in dispatch order: (kernel, KiB) per pass (the passes run the same launch
    # sequence, so the i-th dispatch of one is the i-th of the other)
    series = {}
    for counter, sub in (("FETCH_SIZE", "prof_fetch"), ("WRITE_SIZE", "prof_write")):
        path = os.path.join(OUT, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        seen = defaultdict(set)
        per = defaultdict(float)
        names = {}
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] != counter:
                continue
            k = short(r["Kernel_Name"])
            hbm[k][counter + "_KiB"] += float(r["Counter_Value"])
            seen[k].add(r["Dispatch_Id"])
            per[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
            names[int(r["Dispatch_Id"])] = k
        for k, s in seen.items():
            hbm[k]["launches"] = max(hbm[k]["launches"], len(s))
        series[counter] = [(names[d], per[d]) for d in sorted(per)]
    out = {}
    for k, v in hbm.items():
        n = max(1, v["launches"])
        f = v["FETCH_SIZE_KiB"] * 1024 / n
        w = v["WRITE_SIZE_KiB"] * 1024 / n
        out[k] = {"launches": v["launches"], "fetch_bytes_per_launch_raw": f,
                  "fetch_bytes_per_launch_x2": 2 * f, "write_bytes_per_launch": w,
                  "hbm_bytes_per_launch": 2 * f + w}
    json.dump(out, open(os.path.join(PROF, f"{rnd}_hbm.json"), "w"), indent=1)
    # the trailing-update kernels together (schedule 3: step_kernel = SYRK + tall-solve GEMM;
    # schedule 1: every syrk_kernel instantiation): the population bench.py's roofline averages
    syrk = [(k, v) for k, v in out.items() if k.startswith("step_kernel")] or \
        [(k, v) for k, v in out.items() if k.startswith("syrk_kernel")]
    if syrk:
        launches = sum(v["launches"] for _, v in syrk)
        total = sum(v["hbm_bytes_per_launch"] * v["launches"] for _, v in syrk)
        # evaluations in the PMC run = finalize launches (one per MLL evaluation; the gram kernel
        # no longer runs once per evaluation where it is fused); the PMC passes run the timed
        # schedule's own launches serialised by events (LFM_S3_EVENTS=2; round 3: the event-
        # ordered split, LFM_S3_EVENTS=1, whose launches bench.py had to convert to its own)
        evals = max(1, out.get("finalize_kernel", {}).get("launches", 1))
        rec = {"round": rnd, "source": f"profiles/{rnd}_hbm.json (PMC FETCH_SIZE x2 + WRITE_SIZE)",
               "kernels": [k for k, _ in syrk],
               "hbm_bytes_per_eval": total / evals, "evals": evals,
               "hbm_bytes_per_launch": total / max(1, launches), "launches": launches,
               # the PMC passes run bench.py's default C2 line (bench.py uses the record only
               # for a run of the same N)
               "n": int(os.environ.get("PMC_N", "16384"))}
        # the last evaluation's step launches one by one (bytes, dispatch order): with
        # LFM_S3_EVENTS=2 these are the timed schedule's own launches
        fs, ws = series.get("FETCH_SIZE", []), series.get("WRITE_SIZE", [])
        if fs and len(fs) == len(ws) and all(a[0] == b[0] for a, b in zip(fs, ws)):
            fin = [i for i, (k, _) in enumerate(fs) if k == "finalize_kernel"]
            lo = fin[-2] + 1 if len(fin) >= 2 else 0
            hi = fin[-1] if fin else len(fs)
            pre = "step_kernel" if syrk[0][0].startswith("step_kernel") else "syrk_kernel"
            per = [1024 * (2 * f + w) for (k, f), (_, w) in zip(fs[lo:hi], ws[lo:hi])
                   if k.startswith(pre)]
            rec["last_eval_launch_bytes"] = per
            rec["last_eval_bytes"] = sum(per)
            rec["schedule"] = os.environ.get("PMC_SCHEDULE", "LFM_S3_EVENTS=2")
        json.dump(rec, open(os.path.join(PROF, "syrk_traffic.json"), "w"), indent=1)
    # the roofline recomputed from the trace: the step kernel's rocprof average duration and the
    # traced bench line's algorithmic flops per launch (lfm_kstat.flops, the same launches)
    step = next((r for r in rows if short(r["Name"]).startswith("step_kernel")), None)
    if step and traced and traced.get("roofline"):
        rf = traced["roofline"]
        avg_s = float(step["AverageNs"]) * 1e-9
        ach = rf["flops_per_launch"] / avg_s / 1e12
        calls_per_eval = int(step["Calls"]) / evals_traced
        kern_ms = float(step["TotalDurationNs"]) / 1e6 / evals_traced
        lines += ["", "Roofline of step_kernel from this trace (bench.py prices it the same way):", "",
                  f"- algorithmic flops per launch (traced bench line): {rf['flops_per_launch']:.4e} "
                  f"(issued: {rf['issued_flops_per_launch']:.4e})",
                  f"- rocprof average duration: {avg_s * 1e6:.1f} us over {step['Calls']} launches "
                  f"({calls_per_eval:.0f} per evaluation)",
                  f"- achieved {ach:.2f} TFLOP/s = **{ach / 78.6:.3f}** of 78.6 (traced bench line's own "
                  f"HIP-event frac: {rf['frac']:.3f})",
                  f"- step_kernel time per evaluation {kern_ms:.2f} ms; the traced run's wall "
                  f"{traced['ms_per_step']:.2f} ms per evaluation (consecutive step launches overlap "
                  "at their boundaries, so the kernel sum can exceed the wall)"]
        helper = next((r for r in rows if short(r["Name"]).startswith("helper_update_kernel")),
                      None)
        n = traced.get("config", {}).get("N", 16384)
        ev_tf = n ** 3 / 3.0 / (traced["ms_per_step"] * 1e-3) / 1e12
        lines += [f"- whole evaluation: N^3/3 = {n ** 3 / 3.0:.4e} flop over the traced wall = "
                  f"{ev_tf:.2f} TFLOP/s = **{ev_tf / 78.6:.3f}** of 78.6"]
        if helper is not None:
            lines += [f"- side-CU helper (helper_update_kernel, the tail of long steps' updates on "
                      f"the 32 chain CUs): {int(helper['Calls']) / evals_traced:.0f} launches per "
                      f"evaluation, {float(helper['AverageNs']) / 1e3:.1f} us average"]
        json.dump({"round": rnd, "step_kernel_avg_us": avg_s * 1e6, "calls_per_eval": calls_per_eval,
                   "evaluation_tflops": ev_tf, "evaluation_frac": ev_tf / 78.6,
                   "flops_per_launch": rf["flops_per_launch"], "achieved_tflops": ach,
                   "frac": ach / 78.6, "bench_traced_frac": rf["frac"],
                   "step_kernel_ms_per_eval": kern_ms, "traced_wall_ms_per_eval": traced["ms_per_step"]},
                  open(os.path.join(PROF, f"{rnd}_roofline.json"), "w"), indent=1)
        shutil.copy(tb, os.path.join(PROF, f"{rnd}_bench_traced.json"))
    lines += ["", "HBM per launch (PMC, separate passes; read side x2 per MI355X_MICROARCH.md §HBM):",
              "", "| kernel | launches | read B/launch (x2) | write B/launch |", "|---|---|---|---|"]
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"]):
        lines.append(f"| {k} | {v['launches']} | {v['fetch_bytes_per_launch_x2']:.3e} | "
                     f"{v['write_bytes_per_launch']:.3e} |")
    if len(sys.argv) > 2 and os.path.exists(sys.argv[2]):
        b = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
        shutil.copy(sys.argv[2], os.path.join(PROF, f"{rnd}_bench.json"))
        lines += ["", f"bench.py: {b['value']:.3f} {b['unit']}, {b['ms_per_step']:.2f} ms/eval"]
    open(os.path.join(PROF, f"{rnd}_kernels.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
