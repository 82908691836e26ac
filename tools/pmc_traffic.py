"""Reduce the PMC session (tools/pmc_session.sh) to HBM bytes per pyramid launch.

Calibration (same 8-byte-per-lane access width as the kernels, 768 MiB
buffers, tools/pmc_calib.hip): bytes_read = FETCH_SIZE * k_fetch and
bytes_written = WRITE_SIZE * k_write, with k = known bytes / counter.
Writes profiles/blur_traffic.json, which bench.py reports as
roofline.traffic (bytes per launch, like roofline.achieved).

usage: python tools/pmc_traffic.py gpurun_out/pmc [out.json]
"""
import csv
import json
import os
import sys

KNOWN = 96 * 2 ** 20 * 8  # bytes moved each way per calibration launch


def counter_rows(path, name):
    return [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == name]


def main(d, out):
    k = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = [r for r in counter_rows(os.path.join(d, f"calib_{c}", "run_counter_collection.csv"), c)
                if r["Kernel_Name"].startswith("copy_f64_x2")]
        vals = [float(r["Counter_Value"]) for r in rows]
        k[c] = KNOWN / (sum(vals) / len(vals))
    tot = {}
    launches = 0
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = counter_rows(os.path.join(d, f"bench_{c}", "run_counter_collection.csv"), c)
        tot[c] = sum(float(r["Counter_Value"]) for r in rows) * k[c]
        launches = len(rows)
    res = {
        "hbm_bytes_per_launch": (tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) / launches,
        "read_bytes_per_launch": tot["FETCH_SIZE"] / launches,
        "write_bytes_per_launch": tot["WRITE_SIZE"] / launches,
        "launches": launches,
        "kernels": "k_blur + k_octaves_lds (bench.py --steps 5 --warmup 1)",
        "calibration_bytes_per_unit": k,
        "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes; units "
                  "calibrated on an 8-B/lane copy of 768 MiB (tools/pmc_calib.hip)",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "profiles/blur_traffic.json")
