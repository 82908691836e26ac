"""Host enqueue vs device execution for one synchronous detect.

Joins a rocprofv3 HIP runtime trace (run_hip_api_trace.csv) with its kernel
trace (run_kernel_trace.csv) by correlation id and prints, for the second
to last image (images are delimited by k_job_begin, the first launch of
every job), each dispatch's launch call time on the host next to its start
and end on the device (µs from the image's first host call), plus the host
calls of that image that took longest. Shows whether a kernel waited for the
host to enqueue it or for the device.

usage: python tools/prof_api.py <dir with run_*_trace.csv>
"""
import csv
import os
import sys


def load(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main(d):
    api = load(os.path.join(d, "run_hip_api_trace.csv"))
    ker = load(os.path.join(d, "run_kernel_trace.csv"))
    cpy = []
    p = os.path.join(d, "run_memory_copy_trace.csv")
    if os.path.exists(p):
        cpy = load(p)
    api.sort(key=lambda r: int(r["Start_Timestamp"]))
    ker.sort(key=lambda r: int(r["Start_Timestamp"]))
    by_corr = {r["Correlation_Id"]: r for r in api}
    begins = [r for r in ker if "k_job_begin" in r["Kernel_Name"]]
    if len(begins) < 3:
        print("fewer than 3 jobs in the trace")
        return
    b0, b1 = begins[-3], begins[-2]
    a0 = by_corr.get(b0["Correlation_Id"])
    a1 = by_corr.get(b1["Correlation_Id"])
    if a0 is None or a1 is None:
        print("k_job_begin launches not found in the API trace")
        return
    # the image's host calls: from the first call after the previous job's
    # last synchronisation up to the next job's k_job_begin launch
    i0 = api.index(a0)
    j = i0
    while j > 0 and "Synchronize" not in api[j - 1]["Function"]:
        j -= 1
    t0 = int(api[j]["Start_Timestamp"])
    calls = api[j:api.index(a1)]
    us = lambda t: (int(t) - t0) / 1000.0
    print(f"image window: {len(calls)} host calls, first at 0.0, next job's begin launch at "
          f"{us(a1['Start_Timestamp']):.1f} us")
    ks = [k for k in ker if k["Correlation_Id"] in {c["Correlation_Id"] for c in calls}]
    print(f"{'kernel':34s} {'launch':>8s} {'start':>8s} {'end':>8s}  q")
    for k in ks:
        c = by_corr[k["Correlation_Id"]]
        q = k.get("Stream_Id") or k.get("Queue_Id") or "?"
        print(f"  {k['Kernel_Name'][:32]:32s} {us(c['Start_Timestamp']):8.1f} "
              f"{us(k['Start_Timestamp']):8.1f} {us(k['End_Timestamp']):8.1f}  {q}")
    cs = [r for r in cpy if r.get("Correlation_Id") in {c["Correlation_Id"] for c in calls}]
    for r in cs:
        c = by_corr[r["Correlation_Id"]]
        print(f"  {'copy ' + r.get('Direction', ''):32s} {us(c['Start_Timestamp']):8.1f} "
              f"{us(r['Start_Timestamp']):8.1f} {us(r['End_Timestamp']):8.1f}")
    print("\nslowest host calls of the window:")
    dur = sorted(calls, key=lambda r: int(r["Start_Timestamp"]) - int(r["End_Timestamp"]))
    for r in dur[:15]:
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        print(f"  {r['Function'][:40]:40s} at {us(r['Start_Timestamp']):8.1f}  {dt:7.1f} us")
    tot = {}
    for r in calls:
        dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        tot.setdefault(r["Function"], [0, 0.0])
        tot[r["Function"]][0] += 1
        tot[r["Function"]][1] += dt
    print("\nhost time per call type in the window:")
    for f, (n, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:15]:
        print(f"  {f[:40]:40s} {n:4d} calls {t:8.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
