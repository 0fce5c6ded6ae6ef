"""Summarise a rocprofv3 session of bench.py (scripts/gpu_profile.sh) into profiles/.

Reads gpurun_out/prof_<tag>_trace/*kernel_stats.csv and the separate PMC passes
(gpurun_out/prof_<tag>_pmc_*/*counter_collection.csv) and writes
  profiles/<tag>_kernel_stats.csv      the rocprofv3 --stats summary (copied)
  profiles/<tag>_summary.json          per-launch counters of the SpGEMM kernel + derived numbers
  profiles/traffic_latest.json         HBM bytes per launch, read by bench.py (roofline.traffic)

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) counts 64 B per TCC_EA0_RDREQ while a
request moves a 128-B line on gfx950 (the guide's "double it"), so read bytes = 2 x FETCH_SIZE x 1024;
write bytes = WRITE_SIZE x 1024 (exact for these stores). The raw values are kept alongside.

    python scripts/summarize_profile.py --tag r01 --rows 119705032 --dist uniform
"""
import argparse
import collections
import csv
import glob
import json
import os
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "spgemm_lookback_kernel"


def pmc_means(path):
    out = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                out[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--rows", type=int, default=119_705_032)
    ap.add_argument("--dist", default="uniform")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    args = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = glob.glob(os.path.join(args.src, f"prof_{args.tag}_trace", "*kernel_stats.csv"))
    summary = {"tag": args.tag, "rows": args.rows, "dist": args.dist}
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{args.tag}_kernel_stats.csv"))
        for r in csv.DictReader(open(stats[0])):
            if KERNEL in r["Name"]:
                summary["kernel_avg_ms"] = float(r["AverageNs"]) / 1e6
                summary["kernel_calls"] = int(r["Calls"])
    counters = {}
    for d in glob.glob(os.path.join(args.src, f"prof_{args.tag}_pmc_*")):
        counters.update(pmc_means(d))
    summary["counters_per_launch"] = counters
    if "FETCH_SIZE" in counters and "WRITE_SIZE" in counters:
        rd = 2.0 * counters["FETCH_SIZE"] * 1024
        wr = counters["WRITE_SIZE"] * 1024
        summary["hbm_read_bytes"] = rd
        summary["hbm_write_bytes"] = wr
        summary["hbm_bytes_per_launch"] = rd + wr
        if "kernel_avg_ms" in summary:
            summary["hbm_GBps"] = (rd + wr) / (summary["kernel_avg_ms"] * 1e-3) / 1e9
    if "TCC_HIT_sum" in counters and "TCC_MISS_sum" in counters:
        h, m = counters["TCC_HIT_sum"], counters["TCC_MISS_sum"]
        summary["l2_hit_rate"] = h / (h + m)
    if "TCC_EA0_RDREQ_sum" in counters and "kernel_avg_ms" in summary:
        summary["read_requests_per_launch"] = counters["TCC_EA0_RDREQ_sum"]
        summary["read_requests_G_per_s"] = counters["TCC_EA0_RDREQ_sum"] / (summary["kernel_avg_ms"] * 1e-3) / 1e9
    json.dump(summary, open(os.path.join(prof, f"{args.tag}_summary.json"), "w"), indent=1)
    if "hbm_bytes_per_launch" in summary:
        json.dump({"tag": args.tag, "rows": args.rows, "dist": args.dist,
                   "hbm_bytes_per_launch": summary["hbm_bytes_per_launch"],
                   "source": f"profiles/{args.tag}_summary.json"},
                  open(os.path.join(prof, "traffic_latest.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
