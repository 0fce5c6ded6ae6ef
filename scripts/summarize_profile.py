"""Summarise a rocprofv3 session of bench.py (scripts/gpu_profile.sh) into profiles/.

One projection step = the kernels of rp_project_device: the row-lane pipeline (lpr_* kernels, the
default for short rows over a packed R; staged: reserve/partition/gather + wave) or the tile
pipeline (spgemm_lookback_kernel + scan + tile_heavy_write_kernel + slot_copy_kernel). Reads
gpurun_out/prof_<tag>_trace/*kernel_stats.csv and the separate PMC passes
(gpurun_out/prof_<tag>_pmc_*/*counter_collection.csv) and writes
  profiles/<tag>_kernel_stats.csv      the rocprofv3 --stats summary (copied)
  profiles/<tag>_summary.json          per-step and per-kernel counters + derived numbers
  profiles/traffic_latest.json         HBM bytes per step, read by bench.py (roofline.traffic)

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) counts 64 B per TCC_EA0_RDREQ while a
request moves a 128-B line on gfx950 (the guide's "double it"), so read bytes = 2 x FETCH_SIZE x 1024;
write bytes = WRITE_SIZE x 1024. The raw counter values are kept alongside.

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
STEP_KERNELS = ("spgemm_lookback_kernel", "slot_copy_kernel", "tile_heavy_write_kernel",
                "lpr_reserve_kernel", "lpr_partition_kernel", "lpr_gather_kernel", "lpr_wave_kernel",
                "lpr_main_flat_kernel", "lpr_choose_kernel",
                "lpr_heavy_count_kernel", "lpr_scan_kernel",
                "lpr_copy_kernel", "lpr_heavy_write_kernel")
MAIN_KERNELS = ("lpr_wave_kernel", "lpr_main_flat_kernel", "spgemm_lookback_kernel")


def short(name):
    for k in STEP_KERNELS:
        if k in name:
            return k
    return None


def pmc_means(path):
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k:
                out[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in out.items()}


def derive(c, ms):
    d = {}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        rd, wr = 2.0 * c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
        d.update(hbm_read_bytes=rd, hbm_write_bytes=wr, hbm_bytes=rd + wr)
        if ms:
            d["hbm_GBps"] = (rd + wr) / (ms * 1e-3) / 1e9
    if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
        d["l2_hit_rate"] = c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
    if "TCC_EA0_RDREQ_sum" in c:
        d["read_requests"] = c["TCC_EA0_RDREQ_sum"]
        if ms:
            d["read_requests_G_per_s"] = c["TCC_EA0_RDREQ_sum"] / (ms * 1e-3) / 1e9
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--rows", type=int, default=119_705_032)
    ap.add_argument("--dist", default="uniform")
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--bench-json", default=None, help="the bench.py line of the profiled command (pipeline, "
                                                        "librp source hash)")
    ap.add_argument("--no-latest", action="store_true", help="do not overwrite profiles/traffic_latest.json")
    ap.add_argument("--probe-pmc", default=None,
                    help="TCC_HIT/TCC_MISS pass of the gather probe build (scripts/probes/make_gather_probe.py: the "
                         "gather kernel without its W32 loads): the W32 lookups' own L2 hit rate is the difference")
    args = ap.parse_args()
    bench = {}
    if args.bench_json:
        for line in open(args.bench_json):
            if line.startswith("{"):
                bench = json.loads(line)
    roof = bench.get("roofline", {})
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    summary = {"tag": args.tag, "rows": args.rows, "dist": args.dist, "kernels": {}}
    stats = glob.glob(os.path.join(args.src, f"prof_{args.tag}_trace", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(prof, f"{args.tag}_kernel_stats.csv"))
        for r in csv.DictReader(open(stats[0])):
            k = short(r["Name"])
            if k:
                summary["kernels"][k] = {"avg_ms": float(r["AverageNs"]) / 1e6, "calls": int(r["Calls"])}
    counters = collections.defaultdict(dict)
    for d in glob.glob(os.path.join(args.src, f"prof_{args.tag}_pmc_*")):
        for k, cs in pmc_means(d).items():
            counters[k].update(cs)
    step_ms = sum(v["avg_ms"] for v in summary["kernels"].values()) or None
    step_c = collections.Counter()
    for k, cs in counters.items():
        ent = summary["kernels"].setdefault(k, {})
        ent["counters_per_launch"] = cs
        ent.update(derive(cs, ent.get("avg_ms")))
        step_c.update(cs)
    summary["step_ms"] = step_ms
    summary["step"] = derive(dict(step_c), step_ms)
    json.dump(summary, open(os.path.join(prof, f"{args.tag}_summary.json"), "w"), indent=1)
    plan = roof.get("pipeline", {})
    summary.update(pipeline=plan.get("pipeline"), staged=plan.get("staged"), src_sha16=roof.get("librp_src_sha16"),
                   staged_this_call=bench.get("staged_this_call"))
    mains = [k for k in MAIN_KERNELS if summary["kernels"].get(k, {}).get("avg_ms")]
    main_k = max(mains, key=lambda k: summary["kernels"][k]["avg_ms"]) if mains else None  # the one that ran
    # the kernel that gathers R's descriptors: the staged gather when it ran, else the main kernel
    gk = summary["kernels"].get("lpr_gather_kernel", {})
    gather_k = "lpr_gather_kernel" if gk.get("avg_ms", 0) > 0.05 else main_k
    # the R gathers' own L2 hit rate: the staged gather kernel's requests minus those of its probe
    # build (same S/D streams, no W32 loads); without a probe, the whole kernel's (streams included)
    gc = summary["kernels"].get(gather_k, {}).get("counters_per_launch", {})
    r_hit = summary["kernels"].get(gather_k, {}).get("l2_hit_rate")
    r_scope = ("whole gather kernel (S/D streams included)" if gather_k == "lpr_gather_kernel"
               else "whole main kernel (A and C streams included: R is gathered inside it)")
    if args.probe_pmc and gather_k == "lpr_gather_kernel" and "TCC_HIT_sum" in gc:
        pc = pmc_means(args.probe_pmc).get("lpr_gather_kernel", {})
        if "TCC_HIT_sum" in pc and "TCC_MISS_sum" in pc:
            dh = gc["TCC_HIT_sum"] - pc["TCC_HIT_sum"]
            dr = gc["TCC_HIT_sum"] + gc["TCC_MISS_sum"] - pc["TCC_HIT_sum"] - pc["TCC_MISS_sum"]
            if dr > 0:
                r_hit, r_scope = dh / dr, "W32 lookups only (gather kernel minus its probe build without them)"
                summary["r_gathers"] = {"l2_requests_per_launch": dr, "l2_hits_per_launch": dh, "l2_hit_rate": r_hit,
                                        "probe_counters": pc}
                json.dump(summary, open(os.path.join(prof, f"{args.tag}_summary.json"), "w"), indent=1)
    if "hbm_bytes" in summary["step"]:
        tj = {"tag": args.tag, "rows": args.rows, "dist": args.dist,
              "pipeline": plan.get("pipeline"), "staged": plan.get("staged"), "src_sha16": roof.get("librp_src_sha16"),
              "staged_this_call": bench.get("staged_this_call"),
              "hbm_bytes_per_launch": summary["step"]["hbm_bytes"],
              "main_kernel": main_k,
              "l2_hit_rate_main_kernel": summary["kernels"].get(main_k, {}).get("l2_hit_rate"),
              "gather_kernel": gather_k,
              "l2_hit_rate_r_gathers": r_hit,
              "l2_hit_rate_r_gathers_scope": r_scope,
              "l2_hit_rate_gather_kernel": summary["kernels"].get(gather_k, {}).get("l2_hit_rate"),
              "gather_kernel_read_requests_G_per_s": summary["kernels"].get(gather_k, {}).get("read_requests_G_per_s"),
              "main_kernel_read_requests_per_launch": summary["kernels"].get(main_k, {}).get("read_requests"),
              "l2_hit_rate_step": summary["step"].get("l2_hit_rate"),
              "note": "per projection step (all kernels of rp_project_device)",
              "source": f"profiles/{args.tag}_summary.json"}
        json.dump(tj, open(os.path.join(prof, f"{args.tag}_traffic.json"), "w"), indent=1)
        if not args.no_latest:
            json.dump(tj, open(os.path.join(prof, "traffic_latest.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
