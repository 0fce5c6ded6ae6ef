"""Per-kernel PMC summary of rocprofv3 --pmc passes (gpurun_out/<dir>_*/**/counter_collection.csv):
mean counter value per dispatch for every kernel name, plus derived HBM bytes (MI355X_MICROARCH.md
§HBM: read = 2 x FETCH_SIZE KiB, write = WRITE_SIZE KiB) and L2 hit rate.

    python scripts/pmc_kernels.py gpurun_out/pmc_staged > profiles/<tag>_pmc_kernels.json
"""
import collections
import csv
import glob
import json
import sys


def main(prefix):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(prefix + "*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            vals[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in vals.items():
        d = {c: sum(v) / len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in d:
            d["hbm_read_bytes"] = 2 * d["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in d:
            d["hbm_write_bytes"] = d["WRITE_SIZE"] * 1024
        if "TCC_HIT_sum" in d and "TCC_MISS_sum" in d:
            d["l2_hit_rate"] = d["TCC_HIT_sum"] / max(1.0, d["TCC_HIT_sum"] + d["TCC_MISS_sum"])
        out[k] = d
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
