"""Summarise a rocprofv3 kernel trace (CSV) per kernel and for one image.

usage: python tools/prof_summary.py <run_kernel_trace.csv> [--images N]
"""
import collections
import csv
import sys


def main(path, n_images=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        tot[r["Kernel_Name"]] += d
        cnt[r["Kernel_Name"]] += 1
    # k_job_begin (a counter memset, fillBuffer, before round 5) opens every
    # detect; one k_job_done closes every pipelined / serialised job (the
    # image count when present)
    starts = [i for i, r in enumerate(rows) if "k_job_begin" in r["Kernel_Name"]]
    if not starts:
        starts = [i for i, r in enumerate(rows) if "fillBuffer" in r["Kernel_Name"]]
    n_done = sum(1 for r in rows if "k_job_done" in r["Kernel_Name"])
    n_img = n_images or max(1, n_done or len(starts))
    print(f"{n_img} images")
    print(f"{'kernel':40s} {'calls':>6s} {'total us':>10s} {'avg us':>9s} {'us/image':>9s}")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{k[:40]:40s} {cnt[k]:6d} {v:10.1f} {v / cnt[k]:9.2f} {v / n_img:9.1f}")
    # kernel families as bench.py's roofline / keypoint_kernels_alone rows
    fams = {"pyramid": ("k_blur", "k_blur_pair", "k_blur_pair_dma", "k_blur_tile", "k_octaves_lds",
                        "k_octaves_flow", "k_octave_fused"), "extrema": ("k_extrema",),
            "refine": ("k_refine",), "orientation": ("k_orient",), "descriptor": ("k_descriptor",)}
    print(f"\n{'family':12s} {'launches':>9s} {'us/image':>9s} {'avg us/launch':>14s}")
    for f, pre in fams.items():
        ks = [k for k in tot if k.split("(")[0] in pre or
              (f != "pyramid" and any(k.startswith(p) for p in pre))]
        t, c = sum(tot[k] for k in ks), sum(cnt[k] for k in ks)
        if c:
            print(f"{f:12s} {c:9d} {t / n_img:9.1f} {t / c:14.2f}")
    if len(starts) >= 2:
        a, b = starts[-2], starts[-1]
        # (the memset of earlier rounds came after the table upload)
        if "fillBuffer" in rows[a]["Kernel_Name"]:
            a = max(0, a - 2)
            b = max(a + 1, b - 2)
        seg = rows[a:b]
        t0 = int(seg[0]["Start_Timestamp"])
        t1 = int(rows[b]["Start_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg) / 1000.0
        print(f"\none image (second to last): {len(seg)} dispatches, kernel busy {busy:.1f} us, "
              f"span to next image {(t1 - t0) / 1000.0:.1f} us")
        for r in seg:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
            st = (int(r["Start_Timestamp"]) - t0) / 1000.0
            q = r.get("Stream_Id") or r.get("Queue_Id") or "?"
            print(f"  {r['Kernel_Name'][:30]:30s} start {st:8.1f} end {st + d:8.1f} dur {d:8.1f} us"
                  f"  q {q:>3s} grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else None)
