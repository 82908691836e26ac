"""Reduce the PMC session (tools/pmc_session.sh) to HBM bytes per launch of
the pyramid kernels (k_blur, k_blur_tile, k_octaves_lds: what bench.py's
roofline times) and of the extrema kernel.

Calibration (same 8-byte-per-lane access width as the kernels, 768 MiB
buffers, tools/pmc_calib.hip): bytes_read = FETCH_SIZE * k_fetch and
bytes_written = WRITE_SIZE * k_write, with k = known bytes / counter.
Algorithmic bytes per launch come from the bench JSON of the same run
(pyramid) and from the launch geometry (extrema: 8 B x levels
per pixel of the scanned octaves). The result is stamped with the sha256 of
the kernel sources; bench.py reports roofline.traffic only while they match.

usage: python tools/pmc_traffic.py gpurun_out/<dir> [out.json]
"""
import csv
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KNOWN = 96 * 2 ** 20 * 8  # bytes moved each way per calibration launch
KERNEL_SOURCES = ("sift-project_amd/csrc/sift_kernels.hip", "sift-project_amd/csrc/sift_extrema.hip",
                  "sift-project_amd/csrc/sift_kernels.h",
                  "sift-project_amd/csrc/sift_device.h", "sift-project_amd/csrc/sift_types.h")


def kernel_src_sha256(root=ROOT):
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        h.update(open(os.path.join(root, f), "rb").read())
    return h.hexdigest()


def counter_rows(path, name):
    return [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == name]


def family(kernel_name):
    k = kernel_name.split("(")[0]
    if "k_extrema" in k:
        return "extrema"
    return "pyramid"


def main(d, out):
    k = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = [r for r in counter_rows(os.path.join(d, f"calib_{c}", "run_counter_collection.csv"), c)
                if r["Kernel_Name"].startswith("copy_f64_x2")]
        vals = [float(r["Counter_Value"]) for r in rows]
        k[c] = KNOWN / (sum(vals) / len(vals))
    tot = {}
    n = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        for r in counter_rows(os.path.join(d, f"bench_{c}", "run_counter_collection.csv"), c):
            f = family(r["Kernel_Name"])
            tot[(f, c)] = tot.get((f, c), 0.0) + float(r["Counter_Value"]) * k[c]
            if c == "FETCH_SIZE":
                n[f] = n.get(f, 0) + 1
    bench = None
    for line in open(os.path.join(d, "bench_FETCH_SIZE.log")):
        if line.startswith("{"):
            bench = json.loads(line)
    res = {"kernel_src_sha256": kernel_src_sha256(),
           "calibration_bytes_per_unit": k,
           "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes (kernel-trace "
                     "only) over bench.py --steps 20 --warmup 2; units calibrated on an "
                     "8-B/lane copy of 768 MiB (tools/pmc_calib.hip)"}
    for f in ("pyramid", "extrema"):
        if f not in n:
            continue
        rd, wr = tot[(f, "FETCH_SIZE")] / n[f], tot[(f, "WRITE_SIZE")] / n[f]
        res[f] = {"hbm_bytes_per_launch": rd + wr, "read_bytes_per_launch": rd,
                  "write_bytes_per_launch": wr, "launches": n[f]}
    if bench is not None:
        r = bench["roofline"]
        alg = r["algorithmic_bytes_per_image"] / r["launches_per_image"]
        res["pyramid"]["algorithmic_bytes_per_launch"] = alg
        res["pyramid"]["traffic_over_algorithmic"] = res["pyramid"]["hbm_bytes_per_launch"] / alg
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles",
                                                                         "traffic.json"))
