"""Per-kernel totals of a rocprofv3 --pmc counter CSV (tools/pmc_kp.sh).

usage: python tools/sq_summary.py <pass1/run_counter_collection.csv> [...] [--detects N]
Prints, per kernel family (template arguments folded), every counter summed
over the dispatches and divided by the number of detects (default 7 = 5
timed + 2 warm-up steps of the serialised bench run).
"""
import collections
import csv
import re
import sys


def family(name: str) -> str:
    m = re.search(r"sift_amd::(k_[a-z_0-9]+)", name)
    return m.group(1) if m else name[:40]


def main(paths, detects):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in paths:
        for r in csv.DictReader(open(p)):
            tot[family(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    names = sorted({c for k in tot.values() for c in k})
    print(f"{'kernel':22s}" + "".join(f"{n[3:]:>18s}" for n in names))
    for k, v in sorted(tot.items()):
        print(f"{k:22s}" + "".join(f"{v.get(n, 0.0) / detects:18.4g}" for n in names))


if __name__ == "__main__":
    argv = sys.argv[1:]
    n = 7
    if "--detects" in argv:
        i = argv.index("--detects")
        n = int(argv[i + 1])
        del argv[i:i + 2]
    args = [a for a in argv if not a.startswith("--")]
    main(args, n)
