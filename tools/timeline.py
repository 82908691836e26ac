"""Per-queue timeline of one detect from a rocprofv3 kernel trace.

usage: python tools/timeline.py <run_kernel_trace.csv> [image_index_from_end]

Each detect starts with a counter memset (fillBuffer); the image shown is the
one between the n-th and (n-1)-th last memsets (default: second to last).
"""
import csv
import sys


def main(path, back=2):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "fillBuffer" in r["Kernel_Name"]]
    a, b = starts[-back - 1], starts[-back]
    a, b = max(0, a - 1), b - 1
    t0 = int(rows[a]["Start_Timestamp"])
    busy = 0.0
    for r in rows[a:b]:
        s = (int(r["Start_Timestamp"]) - t0) / 1000
        e = (int(r["End_Timestamp"]) - t0) / 1000
        busy += e - s
        print(f"q{r['Queue_Id']:>2} {r['Kernel_Name'][:30]:30s} {s:8.1f} {e:8.1f} {e - s:7.1f}"
              f"  grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}")
    print(f"span {(int(rows[b]['Start_Timestamp']) - t0) / 1000:.1f} us, kernel busy {busy:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2)
