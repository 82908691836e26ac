"""Timeline view of a rocprofv3 kernel trace (CSV): how much of the span the
GPU had at least one kernel running, the idle gaps, and the dispatch list of
the trace's last part (time-ordered, with queue ids).

usage: python tools/prof_timeline.py <run_kernel_trace.csv> [--tail N] [--gap-us G]
"""
import argparse
import csv


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--tail", type=int, default=250, help="dispatches listed at the end")
    ap.add_argument("--gap-us", type=float, default=30.0, help="idle gaps listed above this")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    if not rows:
        print("empty trace")
        return
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r) for r in rows)
    t_first, t_last = ev[0][0], max(e for _, e, _ in ev)
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e, r in ev:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, cur_e, r["Kernel_Name"]))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t_last - t_first
    print(f"{len(ev)} dispatches, span {span / 1e3:.1f} us, >=1 kernel running {busy / 1e3:.1f} us "
          f"({100.0 * busy / span:.1f} %), idle {(span - busy) / 1e3:.1f} us")
    big = [g for g in gaps if g[0] / 1e3 >= a.gap_us]
    print(f"idle gaps >= {a.gap_us} us: {len(big)}, total {sum(g[0] for g in big) / 1e3:.1f} us")
    for d, at, nxt in big[-40:]:
        print(f"  at {(at - t_first) / 1e3:10.1f} us  idle {d / 1e3:8.1f} us  then {nxt[:40]}")
    print(f"\nlast {a.tail} dispatches (us from the trace start):")
    for s, e, r in ev[-a.tail:]:
        q = r.get("Stream_Id") or r.get("Queue_Id") or "?"
        print(f"  {r['Kernel_Name'][:34]:34s} start {(s - t_first) / 1e3:10.1f} dur {(e - s) / 1e3:8.1f}"
              f"  q {q:>3s} grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r.get('Grid_Size_Z', '1')}")


if __name__ == "__main__":
    main()
