#!/usr/bin/env python
"""bench.py — BASELINE metric of ahmedhassayoune/sift-project on MI355X:
keypoints/sec (detect+describe) on 1920x1080, plus the Gaussian-pyramid
kernels' HBM GB/s against the chip's peak.

A "step" is one full pass of detect_keypoints_and_descriptors (reference
src/sift.cpp:712-776: pyramid, extrema, refine, orientation, clean,
descriptors, every stage in f64 as the reference; the keypoints.png side
effect excluded) over --batch synthetic 1920x1080 images
per GPU (BASELINE config 2 at N=1), with the input already resident in HBM
and the final sorted keypoint records returned to the host. With N>1 ranks
(torchrun) every rank processes its own images (weak scaling, BASELINE
config 4) and the per-image descriptor buffers are all-gathered over RCCL.

roofline: the pyramid's algorithmic bytes of every image of the
timed region / its wall time ("chip level"), with the kernel-alone figure
(serialised context, dispatch-timestamped HIP events, comparable with the
rocprofv3 summaries under profiles/) and the FP64-issue fraction beside it.
After the timed region (N=1): kernel-alone legs, latency, API path, 8-image
jobs, BASELINE configs 3 (4096^2) and 5 (8K) with their own rooflines, the
CPU baselines (the oracle port and the reference itself, one core), the
matcher and the stitching consumer.

usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time
import collections

ROOT = os.path.dirname(os.path.abspath(__file__))
# jobs kept in flight by the pipelined legs: four single-image jobs (one
# stream each), two 8-image jobs (a stream pair each)
JOB_DEPTH = max(1, min(8, int(os.environ.get("SIFT_JOB_DEPTH", "4"))))
BATCH_DEPTH = max(1, min(8, int(os.environ.get("SIFT_BATCH_DEPTH", "2"))))
# BASELINE configs 3 / 5: one large image per job, jobs in flight (round 5:
# 3 against 2, config 3 4.15 vs 4.36 ms per image, config 5 10.5 vs 11.6 ms;
# round 6: 4 against 3, config 3 3.65 vs 3.71, config 5 9.40 vs 9.60,
# gpurun_out/r06_depth; the 1080p legs stay at 4 single-image jobs: 3 / 5 / 6
# in flight +6 / +10 / +14 % on the driver's command)
BIG_DEPTH = max(1, min(8, int(os.environ.get("SIFT_BIG_DEPTH", "4"))))
sys.path.insert(0, os.path.join(ROOT, "sift-project_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from sift_hip import (INPUT_F64_DEVICE, INPUT_F64_HOST, PROF_DESC, PROF_EXTREMA,  # noqa: E402
                      PROF_ORIENT, PROF_PYRAMID, PROF_REFINE, Context, SiftParams, synth_image)

METRIC = ("keypoints/sec (detect+describe) on 1920×1080; Gaussian-pyramid HBM GB/s vs peak")
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# FP64 vector issue peak: 256 CUs x 4 SIMDs x 16 lanes per cycle x 2.4 GHz
# (= 78.6 TFLOP/s counting an FMA as two), in lane-operations per second
FP64_PEAK_OPS = 256 * 4 * 16 * 2.4e9


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(img: np.ndarray, seconds: float) -> dict:
    """Oracle (from-scratch restatement, bit-identical to the reference) on one
    host core, repeated on the same image until `seconds` have elapsed."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_bind import OracleRun

    runs, kps, t_total = 0, 0, 0.0
    while runs == 0 or t_total < seconds:
        t0 = time.perf_counter()
        r = OracleRun(img)
        t_total += time.perf_counter() - t0
        kps += len(r.final)
        runs += 1
        r.close()
    return {
        "value": kps / t_total,
        "unit": "keypoints/s",
        "cores": 1,
        "kind": "port",
        "sample": f"{runs} x full 1920x1080 synthetic image (seed 42) through oracle/sift_cpu.cpp "
                  f"(the oracle restatement, bit-identical output; ~3x faster than the "
                  f"reference's own copy-fixed code on the same core, whose column-major blur "
                  f"walk dominates it; single thread, {cpu_model()}), {t_total:.1f} s",
    }


def cpu_baseline_reference(img: np.ndarray, seconds_hint: float) -> dict | None:
    """The reference itself on the bench host: oracle/_ref/ref_harness_cf
    (the reference's src/sift.cpp compiled by oracle/Makefile with its own
    flags, copy-fixed — the four per-item deep copies made const refs,
    outputs byte-identical to the as-is build) runs
    detect_keypoints_and_descriptors' stages (sift.cpp:712-776, minus the
    keypoints.png side effect) once on the same seed-42 image, single
    threaded; its own steady-clock total is the time. None when the harness
    was not built (it needs /root/reference at build time)."""
    import subprocess
    import tempfile

    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness_cf")
    if not os.path.exists(exe):
        return None
    with tempfile.TemporaryDirectory() as d:
        raw = os.path.join(d, "in.raw")
        h, w = img.shape[:2]
        c = 1 if img.ndim == 2 else img.shape[2]
        with open(raw, "wb") as f:
            f.write(b"SIFTRAW1" + np.array([w, h, c], dtype="<i4").tobytes())
            f.write(np.ascontiguousarray(img, dtype="<f8").tobytes())
        r = subprocess.run([exe, raw, os.path.join(d, "out")], capture_output=True, text=True,
                           timeout=max(120.0, 20 * seconds_hint))
        if r.returncode != 0:
            return {"error": f"ref_harness_cf exit {r.returncode}: {r.stderr[-200:]}"}
        meta = dict(line.split(None, 1) for line in open(os.path.join(d, "out.meta.txt")))
    t, n = float(meta["time_total"]), int(meta["final"])
    return {"value": n / t, "unit": "keypoints/s", "cores": 1, "kind": "reference",
            "seconds": t, "keypoints": n,
            "sample": f"1 x full 1920x1080 synthetic image (seed 42) through the reference's own "
                      f"src/sift.cpp (oracle/_ref/ref_harness_cf: compiled from /root/reference "
                      f"with its Makefile flags -std=c++17 -O3, copy-fixed const refs at "
                      f"sift.cpp:311,346,466,616, byte-identical outputs); single thread, "
                      f"{cpu_model()}; time = the harness's steady-clock total of the stages"}


def matcher_bench(ctx, dev, kps_a, W, H, params, cpu_seconds: float) -> dict:
    """the GPU matcher (match_keypoints, sift.cpp:783-815) on
    the bench image's keypoints against those of a second synthetic image
    (seed 43), both record arrays resident in HBM; wall time per call incl.
    the result download and compaction. CPU baseline: the oracle matcher on a
    bounded sample of queries against all references, 1 core."""
    kps_b, _ = ctx.detect(synth_image(W, H, 1, seed=43), params)
    da = torch.from_numpy(kps_a.view(np.uint8).copy()).to(dev)
    db = torch.from_numpy(kps_b.view(np.uint8).copy()).to(dev)
    torch.cuda.synchronize()
    for _ in range(3):
        m = ctx.match_device(da.data_ptr(), len(kps_a), db.data_ptr(), len(kps_b), 0.75)
    reps = 50
    t0 = time.perf_counter()
    for _ in range(reps):
        m = ctx.match_device(da.data_ptr(), len(kps_a), db.data_ptr(), len(kps_b), 0.75)
    dt = (time.perf_counter() - t0) / reps
    pairs = float(len(kps_a)) * len(kps_b)
    out = {"n1": len(kps_a), "n2": len(kps_b), "ratio": 0.75, "matches": len(m),
           "ms_per_match": dt * 1e3, "pairs_per_s": pairs / dt}
    if cpu_seconds > 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from oracle_bind import oracle_match
        nq, t = 0, 0.0
        t0 = time.perf_counter()
        while t < cpu_seconds * 0.2:
            oracle_match(kps_a[nq % len(kps_a):nq % len(kps_a) + 64], kps_b, 0.75)
            nq += 64
            t = time.perf_counter() - t0
        out["cpu_baseline"] = {"pairs_per_s": nq * len(kps_b) / t, "cores": 1, "kind": "port",
                               "sample": f"{nq} queries x {len(kps_b)} references, "
                                         f"oracle/sift_cpu.cpp sift_cpu_match, {t:.1f} s"}
    return out


def load_traffic(path):
    """PMC traffic per launch (tools/pmc_traffic.py), only if it was measured
    on the current kernel sources."""
    if not os.path.exists(path):
        return None, "no PMC traffic file"
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_traffic import kernel_src_sha256
    with open(path) as f:
        t = json.load(f)
    if t.get("kernel_src_sha256") != kernel_src_sha256(ROOT):
        return None, f"stale: {os.path.relpath(path, ROOT)} was measured on other kernel sources"
    return t, f"rocprofv3 FETCH_SIZE+WRITE_SIZE per launch, {os.path.relpath(path, ROOT)}"


def roofline_obj(ms: float, nbytes: float, launches: int, traffic, note) -> dict:
    achieved = nbytes / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
    alg = nbytes / launches if launches else None
    return {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic["hbm_bytes_per_launch"] if traffic else None,
        "traffic_source": note,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": (traffic["hbm_bytes_per_launch"] / alg)
        if (traffic and alg) else None,
        "avg_launch_us": (ms * 1e3 / launches) if launches else None,
        "launches": launches,
    }


def chip_roofline(bytes_img: float, launches_img: float, images: int, elapsed: float, traffic,
                  note) -> dict:
    """Chip-level roofline of a kernel family over the timed region: its
    algorithmic bytes for every image processed / the region's wall time.
    `traffic` (PMC, per launch) is scaled to bytes per image."""
    achieved = bytes_img * images / elapsed / 1e9
    t_img = traffic["hbm_bytes_per_launch"] * launches_img if traffic else None
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": t_img,
            "traffic_source": note, "traffic_unit": "HBM bytes per image",
            "algorithmic_bytes_per_image": bytes_img,
            "traffic_over_algorithmic": (t_img / bytes_img) if t_img else None,
            "launches_per_image": launches_img,
            "scope": "chip level: algorithmic bytes of every image of the timed region / its "
                     "wall time (the kernels share the chip with every other stage)"}


# BASELINE configs 3 and 5 (SURVEY 8d inputs; generator arguments as the
# reference-generated goldens tests/golden/synth_4096x4096_int2_oct5.npz and
# synth_7680x4320_dense.npz, which pin the HIP path's output on them)
BIG_CONFIGS = {
    "config3": {"w": 4096, "h": 4096, "nblobs": 300000, "smax": 6.0, "images": 16,
                "params": {"intervals": 2, "max_octaves": 5},
                "workload": "BASELINE config 3: single 4096x4096 synthetic image (seed 42, 300k "
                            "blobs), 5 octaves x 5 scales (intervals=2, max_octaves=5)",
                "reference_cpu": {"seconds": 109.7, "keypoints": 46242,
                                  "source": "BASELINE.md (survey container, copy-fixed reference, "
                                            "1 thread)"}},
    "config5": {"w": 7680, "h": 4320, "nblobs": 1500000, "smax": 4.0, "images": 12,
                "params": {},
                "workload": "BASELINE config 5: 8K (7680x4320) dense synthetic image (seed 42, "
                            "1.5M blobs), reference default parameters",
                "reference_cpu": {"seconds": 206.5, "keypoints": 166313,
                                  "source": "BASELINE.md (survey container, copy-fixed reference, "
                                            "1 thread)"}},
}


def big_config_leg(name: str, dev) -> dict:
    """One large image per job, BIG_DEPTH jobs in flight (the next image's
    pyramid overlaps the previous one's keypoint tail), input resident in
    HBM, after a warm-up that ran a job in every slot the pipeline cycles
    through: keypoints/s and ms per image, the library's host phases per job; the pyramid's chip-level
    HBM fraction over that time, its kernel-alone fraction and FP64-issue
    fraction (SIFT_SERIAL context, dispatch-timestamped events), and the
    keypoint kernels alone."""
    spec = BIG_CONFIGS[name]
    w, h = spec["w"], spec["h"]
    p = SiftParams(**spec["params"])
    img = synth_image(w, h, 1, nblobs=spec["nblobs"], smax=spec["smax"], seed=42)
    t = torch.from_numpy(img).to(dev)
    torch.cuda.synchronize()
    ptr = [t.data_ptr()]
    c = Context(dev.index)
    sub = lambda k: c.submit(ptr, INPUT_F64_DEVICE, w, h, 1, p)  # noqa: E731
    depth = BIG_DEPTH
    # warm-up: every slot a depth-d pipeline cycles through (d + 1) has run a
    # job, so the timed jobs find their buffers allocated
    pipelined(c, sub, depth + 2, depth)
    n = spec["images"]
    phases = collections.Counter()
    kp, dt = pipelined(c, sub, n, depth,
                       on_fetch=lambda: phases.update(c.host_timing()))
    cnt = c.counts()
    c.close()
    dims = [(cnt["octave0_w"] >> o, cnt["octave0_h"] >> o) for o in range(cnt["octaves"])]
    os.environ["SIFT_SERIAL"] = "1"
    try:
        sc = Context(dev.index)
    finally:
        del os.environ["SIFT_SERIAL"]
    sc.detect_device(ptr[0], w, h, 1, p)
    sc.profile_table(reset=True)
    sc.set_profiling(True)
    n_alone = 3
    for _ in range(n_alone):
        sc.detect_device(ptr[0], w, h, 1, p)
    sc.set_profiling(False)
    pyr, ext, kpk = _rows_roofline(sc.profile_table(reset=True), n_alone)
    sc.close()
    del t
    torch.cuda.empty_cache()
    pyr_b, ext_b = pyr["bytes_per_image"], ext["bytes_per_image"]
    fp64 = pyramid_fp64_ops(dims, p)
    ref = dict(spec["reference_cpu"])
    ref["value"] = ref["keypoints"] / ref["seconds"]
    roof = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "achieved": round(pyr_b * n / dt / 1e9, 1),
            "frac": round(pyr_b * n / dt / 1e9 / HBM_PEAK_GBS, 4),
            "algorithmic_bytes_per_image": pyr_b,
            "scope": "chip level: pyramid bytes per image x images / wall time",
            "alone": pyr,
            "fp64": {"ops_per_image": fp64, "peak_ops_per_s": FP64_PEAK_OPS,
                     "frac": fp64 * n / dt / FP64_PEAK_OPS,
                     "frac_alone": fp64 / (pyr["us_per_image"] * 1e-6) / FP64_PEAK_OPS}}
    host = {k: v / n for k, v in phases.items()}
    return {"workload": spec["workload"], "image": f"{w}x{h}x1", "images": n,
            "jobs_in_flight": depth,
            "host_phases_ms": dict(host, note="per job, library host phases: enqueue "
                                   "(launches), wait_device (chain runs sorted while waiting), "
                                   "download (bulk path only), finalize (merge + unique), "
                                   "output (records into the caller's array), blocked (host "
                                   "waiting on device events)"),
            "value": kp / dt, "unit": "keypoints/s", "ms_per_image": dt / n * 1e3,
            "keypoints_per_image": kp // n, "octaves": cnt["octaves"],
            "levels_per_octave": cnt["levels_per_octave"], "dtype": "f64",
            "roofline": roof,
            "extrema_roofline": {"achieved": round(ext_b * n / dt / 1e9, 1),
                                 "frac": round(ext_b * n / dt / 1e9 / HBM_PEAK_GBS, 4),
                                 "alone": ext},
            "keypoint_kernels_alone": kpk,
            "reference_cpu": ref, "speedup_vs_reference_cpu": (kp / dt) / ref["value"]}


def level_radii(params) -> list:
    """Half-kernel radius R = ceil(3 sigma) (image.cpp:226) of the initial
    blur (sigma = sqrt(s0^2 - 1), sift.cpp:124) and of levels 1..G-1
    (sift.cpp:143-155)."""
    import math
    s0, iv = params.init_sigma, params.intervals
    k = 2.0 ** (1.0 / iv)
    sig = [math.sqrt(s0 * s0 - 1)] + [(k ** (i - 1)) * s0 * math.sqrt(k * k - 1)
                                      for i in range(1, iv + 3)]
    return [int(math.ceil(3 * x)) for x in sig]


def pyramid_fp64_ops(octave_dims, params) -> float:
    """FP64 lane-operations of one image's pyramid (algorithmic, no halo
    redundancy): per output pixel and pass the reference's
    acc = v*k0; acc += k[u]*(v[+u] + v[-u]) (3R+1 ops) and the correctly
    rounded division by sum_w (3: mul, fma, fma), two passes per level
    (image.cpp:168-211)."""
    R = level_radii(params)
    n0 = octave_dims[0][0] * octave_dims[0][1]
    ops = 2 * (3 * R[0] + 4) * n0
    for (w, h) in octave_dims:
        ops += sum(2 * (3 * r + 4) * w * h for r in R[1:])
    return float(ops)


def survey_bpyr(octave_dims, params) -> float:
    """SURVEY 8d's B_pyr of one image: sum over octaves of (G-1) * 16 * N_o,
    plus 8 * N_{o+1} per decimation; the initial blur is not counted (config
    2: 884.7 MB). The headline's bytes also charge the fused initial blur at
    its real I/O; both fractions are reported."""
    G = params.intervals + 3
    b = 0.0
    for o, (w, h) in enumerate(octave_dims):
        b += (G - 1) * 16.0 * w * h
        if o + 1 < len(octave_dims):
            b += 8.0 * octave_dims[o + 1][0] * octave_dims[o + 1][1]
    return b


def _rows_roofline(prof, n_images):
    """Kernel-alone figures from dispatch-timestamped events (SIFT_SERIAL
    context: every kernel alone on the chip)."""
    rows = prof[PROF_PYRAMID:PROF_PYRAMID + 16]
    ms, nb, n = (sum(r[k] for r in rows) for k in range(3))
    pyr = roofline_obj(ms, nb, n, None, None)
    pyr["us_per_image"] = ms * 1e3 / n_images
    pyr["bytes_per_image"] = nb / n_images
    pyr["per_octave"] = [{"octave": o, "us_per_launch": m * 1e3 / k,
                          "us_per_image": m * 1e3 / n_images,
                          "achieved_GBps": b / (m * 1e-3) / 1e9}
                         for o, (m, b, k) in enumerate(rows) if k]
    ems, eb, en = prof[PROF_EXTREMA]
    ext = roofline_obj(ems, eb, en, None, None)
    ext["us_per_image"] = ems * 1e3 / n_images
    ext["bytes_per_image"] = eb / n_images
    for d in (pyr, ext):
        for k in ("traffic", "traffic_source", "traffic_over_algorithmic"):
            d.pop(k)
    kp = {name: {"us_per_image": prof[row][0] * 1e3 / n_images,
                 "launches_per_image": prof[row][2] / n_images}
          for name, row in (("refine", PROF_REFINE), ("orientation", PROF_ORIENT),
                            ("descriptor", PROF_DESC))}
    return pyr, ext, kp


def alone_leg(dev_img, W, H, params, n_images: int = 200, batch_imgs=None) -> dict:
    """Kernel-quality view of the same launches: a second context with
    SIFT_SERIAL=1 runs every kernel of a detect on one stream, so each launch
    has the chip to itself (no other job's kernels share the CUs). The timed
    region's roofline above is the pipelined one, where four jobs' chains
    share the chip and every launch lasts longer while the job rate rises."""
    os.environ["SIFT_SERIAL"] = "1"
    try:
        sctx = Context(torch.cuda.current_device())
    finally:
        del os.environ["SIFT_SERIAL"]
    for _ in range(10):
        sctx.detect_device(dev_img.data_ptr(), W, H, 1, params)
    sctx.set_profiling(True)
    sctx.profile_table(reset=True)
    t0 = time.perf_counter()
    for _ in range(n_images):
        sctx.detect_device(dev_img.data_ptr(), W, H, 1, params)
    dt = time.perf_counter() - t0
    sctx.set_profiling(False)
    pyr, ext, kp = _rows_roofline(sctx.profile_table(reset=True), n_images)
    note = (f"SIFT_SERIAL=1 context, {n_images} synchronous detects of the same image, every "
            f"kernel alone on the chip, per-launch dispatch-timestamped HIP events; "
            f"{dt / n_images * 1e3:.3f} ms per image serialised")
    out = {"pyramid": pyr, "extrema": ext, "keypoint_kernels": kp, "note": note}
    if batch_imgs:
        # BASELINE config 4's per-GPU share: one 8-image job per launch, alone
        ptrs = [t.data_ptr() for t in batch_imgs]
        nb_jobs = max(3, n_images // (4 * len(ptrs)))
        for _ in range(2):
            sctx.fetch(sctx.submit(ptrs, INPUT_F64_DEVICE, W, H, 1, params))
        sctx.set_profiling(True)
        sctx.profile_table(reset=True)
        for _ in range(nb_jobs):
            sctx.fetch(sctx.submit(ptrs, INPUT_F64_DEVICE, W, H, 1, params))
        sctx.set_profiling(False)
        bp, be, bk = _rows_roofline(sctx.profile_table(reset=True), nb_jobs * len(ptrs))
        out["batch"] = {"pyramid": bp, "extrema": be, "keypoint_kernels": bk,
                        "note": f"{nb_jobs} jobs of {len(ptrs)} 1920x1080 images (one launch per "
                                f"kernel covers the job), SIFT_SERIAL=1 context"}
    sctx.close()
    return out


def host_busy_leg(ctx, ptrs, W, H, params, n_steps: int, depth: int) -> dict:
    """Where the host's time goes in the pipelined loop (after the timed
    region): wall time inside submit() (plan + enqueue, pure host) and inside
    fetch() minus the time the library was blocked on device events, per
    step. If their sum approaches ms_per_step the loop is host-bound."""
    q = collections.deque()
    t_sub = t_fetch = t_wait = 0.0
    ph = collections.Counter()
    t0 = time.perf_counter()
    for k in range(n_steps):
        while len(q) < depth and k + len(q) < n_steps:
            a = time.perf_counter()
            q.append(ctx.submit(ptrs, INPUT_F64_DEVICE, W, H, 1, params))
            t_sub += time.perf_counter() - a
        a = time.perf_counter()
        ctx.fetch(q.popleft())
        t_fetch += time.perf_counter() - a
        ht = ctx.host_timing()
        t_wait += ht["blocked"] * 1e-3
        ph.update({"enqueue": ht["enqueue"], "chain_runs": ht["wait_device"] - ht["blocked"],
                   "merge_unique": ht["finalize"], "output_copy": ht["output"]})
    wall = time.perf_counter() - t0
    per = lambda x: x / n_steps * 1e3  # noqa: E731
    return {"ms_per_step": per(wall), "submit_ms": per(t_sub),
            "fetch_minus_device_wait_ms": per(t_fetch - t_wait),
            "host_busy_ms": per(t_sub + t_fetch - t_wait), "steps": n_steps,
            "library_phases_ms": {k: v / n_steps for k, v in ph.items()},
            "note": "pipelined loop as the timed region; host_busy = submit + fetch - the "
                    "time the library was blocked on device events; library_phases_ms: "
                    "enqueue (launches), chain_runs (glibc sizes + sorted run per keypoint "
                    "chain while waiting), merge_unique, output_copy (records into the "
                    "caller's array)"}


def pipelined(ctx, submit, n_steps: int, depth: int = 0, on_fetch=None):
    """Run n_steps jobs with `depth` (default JOB_DEPTH) in flight: job k+d-1
    is submitted before job k is fetched; returns (keypoints, elapsed s).
    on_fetch() runs after every fetch (inside the time)."""
    depth = depth or JOB_DEPTH
    kp = 0
    t0 = time.perf_counter()
    q = collections.deque()
    for k in range(n_steps):
        while len(q) < depth and k + len(q) < n_steps:
            q.append(submit(k + len(q)))
        kps, _ = ctx.fetch(q.popleft())
        kp += sum(len(x) for x in kps)
        if on_fetch is not None:
            on_fetch()
    return kp, time.perf_counter() - t0


def extra_legs(ctx, dev, host_imgs, dev_imgs, W, H, params, seconds: float) -> dict:
    """Secondary measurements at N=1 (after the timed region): single-image
    latency (sync), the reference API path from a host Image buffer (sync and
    pipelined), an 8-image job per step (BASELINE config 4 layout on one GPU),
    and the host-side phase times of a detect."""
    out = {}
    img_dev = dev_imgs[0].data_ptr()
    img_host = host_imgs[0]

    def timed_loop(fn, min_s):
        fn()
        n, t0 = 0, time.perf_counter()
        while True:
            fn()
            n += 1
            dt = time.perf_counter() - t0
            if dt >= min_s and n >= 5:
                return dt / n

    lat = timed_loop(lambda: ctx.detect_device(img_dev, W, H, 1, params), seconds)
    kp1 = ctx.counts()["final_n"]
    phases = ctx.host_timing()
    out["latency"] = {"ms_per_image": lat * 1e3, "keypoints_per_s": kp1 / lat,
                      "note": "one synchronous detect per image (input in HBM), no pipelining"}
    api = timed_loop(lambda: ctx.detect(img_host, params), seconds)
    n_api = max(5, int(seconds / api))
    kp_api, t_api = pipelined(
        ctx, lambda k: ctx.submit([img_host], INPUT_F64_HOST, W, H, 1, params), n_api)
    out["api"] = {
        "value": kp_api / t_api, "unit": "keypoints/s", "ms_per_image": t_api / n_api * 1e3,
        "sync_ms_per_image": api * 1e3, "sync_value": kp1 / api,
        "path": "sift_hip_submit/fetch from a host Image buffer (float64 HWC, reference "
                "image_io.hh:22-26): integer-valued -> packed to u8 on 8 host threads, pinned "
                "staging, async H2D, u8->f64 on device; JOB_DEPTH jobs in flight (value) and "
                "synchronous per call (sync_*), PCIe included"}
    B = 8
    batch_imgs = [synth_image(W, H, 1, seed=42 + i) for i in range(B)]
    bt = [torch.from_numpy(a).to(dev) for a in batch_imgs]
    torch.cuda.synchronize()
    ptrs = [t.data_ptr() for t in bt]
    sub = lambda k: ctx.submit(ptrs, INPUT_F64_DEVICE, W, H, 1, params)  # noqa: E731
    pipelined(ctx, sub, 3, BATCH_DEPTH)
    one = timed_loop(lambda: ctx.fetch(sub(0)), 0.5)
    n_b = max(5, int(seconds / one))
    kp_b, t_b = pipelined(ctx, sub, n_b, BATCH_DEPTH)
    out["batch8"] = {"images_per_s": n_b * B / t_b, "ms_per_image": t_b / (n_b * B) * 1e3,
                     "keypoints_per_s": kp_b / t_b, "jobs": n_b,
                     "note": "8 synthetic 1920x1080 images (seeds 42..49) per job, one batched "
                             "launch per kernel, BATCH_DEPTH jobs in flight, inputs in HBM"}
    out["host_phases_ms"] = phases
    out["stitch"] = stitch_leg(ctx, seconds)
    return out


def stitch_leg(ctx, seconds: float) -> dict:
    """the stitching consumer end to end on the GPU
    (sift_stitch.py: detect every image, GPU match + GPU RANSAC per stitch-graph
    edge, GPU feather compositing) over the committed 5-image slice of the
    reference's CAVE-04_times_square dataset, plus the RANSAC scoring kernel
    alone (hypotheses x point pairs per second)."""
    from sift_stitch import keypoint_xy, load_dataset, stitch

    graph, images = load_dataset(os.path.join(ROOT, "tests", "golden", "stitch"))
    res = stitch(ctx, images, graph)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        res = stitch(ctx, images, graph)
        n += 1
        dt = time.perf_counter() - t0
        if dt >= seconds / 2 and n >= 3:
            break
    p = res.pairs[0]
    m = ctx.match(res.keypoints[p.j], res.keypoints[p.i], 0.75)
    src = keypoint_xy(res.keypoints[p.j])[m["i1"]]
    dst = keypoint_xy(res.keypoints[p.i])[m["i2"]]
    n_hyp = 1 << 16
    ctx.ransac_scores(src, dst, n_hyp=n_hyp)
    k, t1 = 0, time.perf_counter()
    while time.perf_counter() - t1 < 0.2 or k < 3:
        ctx.ransac_scores(src, dst, n_hyp=n_hyp)
        k += 1
    dt_r = (time.perf_counter() - t1) / k
    return {"images": len(images), "edges": len(res.pairs),
            "ms_per_stitch": dt / n * 1e3, "images_per_s": n * len(images) / dt,
            "inliers_per_edge": [int(q.inliers) for q in res.pairs],
            "canvas": list(res.panorama.shape[:2][::-1]),
            "ransac": {"n_hyp": n_hyp, "pairs": int(len(src)), "ms_per_call": dt_r * 1e3,
                       "hyp_pairs_per_s": n_hyp * len(src) / dt_r,
                       "note": "sift_hip_ransac_scores incl. normalisation, upload, score "
                               "download"},
            "data": "tests/golden/stitch: CAVE-04_times_square 00-04 (640x480 RGB) and their "
                    "stitch-graph edges"}


def launch_workers(n_gpus: int, json_out) -> int:
    """bench.py --gpus N (N > 1) run directly: one worker per GPU through
    torch.distributed.run as child processes (127.0.0.1 rendezvous on a free
    port), exactly the driver's multi-GPU command; rank 0's JSON line is
    forwarded to stdout and the launcher's exit status returned. Nothing in
    this process touches the GPU."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n_gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    print("launching: " + " ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, text=True)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    if lines:
        print(lines[-1], file=json_out, flush=True)
    return r.returncode


def main() -> int:
    # stdout carries exactly one JSON line: keep a handle on it and send
    # fd 1 to stderr for everything else (RCCL prints its banner to stdout)
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2500)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=1, help="images per GPU per step")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-matcher", action="store_true",
                    help="skip the matcher measurement (SURVEY §8f row 1)")
    ap.add_argument("--exchange", action="store_true",
                    help="run the RCCL record exchange also at world size 1 (tests the N>1 "
                         "data path on one GPU)")
    ap.add_argument("--exchange-steps", type=int, default=8,
                    help="steps whose records share one all-gather (RCCL's per-call host "
                         "cost amortised over a bucket of steps)")
    ap.add_argument("--sync", action="store_true",
                    help="one job at a time (no pipelining), for profiling / A-B")
    ap.add_argument("--no-big", action="store_true",
                    help="skip the BASELINE config 3 / config 5 legs (4096^2, 8K)")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the latency / API / batch8 legs")
    ap.add_argument("--extra-seconds", type=float, default=2.0)
    ap.add_argument("--no-events", action="store_true",
                    help="no per-launch HIP events anywhere (the kernel-alone legs need them)")
    ap.add_argument("--events-every", type=int, default=0,
                    help="diagnostics: time the pyramid launches of every k-th job of the timed "
                         "region with HIP events (0: none; events slow the pipeline)")
    ap.add_argument("--step-log", action="store_true",
                    help="print the timed region's submit / fetch / done times to stderr")
    ap.add_argument("--no-alone", action="store_true",
                    help="skip the kernel-alone roofline legs (PMC sessions count only the "
                         "timed region's launches)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per launch (tools/pmc_traffic.py); used only "
                         "while its kernel-source hash matches the sources")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # launched without torchrun: start one fresh worker process per GPU
        # (before anything here touched the GPU) and pass the JSON line on
        json_out.flush()
        return launch_workers(args.gpus, json_out)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE={world}: refusing to report a "
              f"different GPU count than asked for", file=sys.stderr)
        return 2
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    use_exchange = world > 1 or args.exchange
    if use_exchange:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("nccl", rank=rank, world_size=world)
        from sift_dist import allgather_records

    W, H, B = args.width, args.height, args.batch
    ids = [rank * B + j for j in range(B)]
    host_imgs = [synth_image(W, H, 1, seed=42 + i) for i in ids]
    dev_imgs = [torch.from_numpy(a).to(dev) for a in host_imgs]
    torch.cuda.synchronize()
    ctx = Context(local_rank)
    params = SiftParams()

    # N > 1: every step's records go to every rank (RCCL all-gather of the
    # descriptor buffers). Warm-up steps use the exact two-phase
    # all-gather and size the slots of the pipelined exchange, which then
    # overlaps each step's all-gather with the next step's detection.
    exchange = None
    max_rows = 0

    # A step = one job over this rank's B images (inputs resident in HBM).
    # Steps are pipelined: step k+1's job is submitted before step k's
    # records are fetched, so the device runs k+1's pyramid while the host
    # sorts k's records. Every step's work is inside the timed region.
    ptrs = [t.data_ptr() for t in dev_imgs]

    def submit():
        return ctx.submit(ptrs, INPUT_F64_DEVICE, W, H, 1, params)

    def finish(ticket) -> int:
        nonlocal max_rows
        if exchange is not None:
            # steady state: the library writes the job's final records
            # straight into the exchange slot in HBM (sift_hip_fetch_device),
            # then one async RCCL all-gather per step
            n_total = sum(ctx.wait(ticket))
            exchange.push_device(ctx, ticket, ids)
            return n_total
        kps, _ = ctx.fetch(ticket)
        n_total = sum(len(k) for k in kps)
        if use_exchange:  # warm-up: the exact two-phase exchange sizes the slots
            bufs = [torch.from_numpy(k.view(np.uint8).reshape(-1, 168)) for k in kps]
            max_rows = max(max_rows, n_total)
            allgather_records([b.to(dev) for b in bufs], ids, B)
        return n_total

    depth = JOB_DEPTH if B == 1 else BATCH_DEPTH

    sample_events = False  # per-launch events on sampled jobs (--events-every)
    in_timed = False  # set for the timed region

    step_log = []  # --step-log: (event, job, t) of the timed region

    def run(n_steps: int) -> int:
        kp = 0
        log = step_log.append if (args.step_log and in_timed) else None
        if args.sync:
            for k in range(n_steps):
                if sample_events:
                    ctx.set_profiling(k % args.events_every == 0)
                kp += finish(submit())
            return kp
        q = collections.deque()
        for k in range(n_steps):
            while len(q) < depth and k + len(q) < n_steps:
                if sample_events:
                    ctx.set_profiling((k + len(q)) % args.events_every == 0)
                if log:
                    log(("submit", k + len(q), time.perf_counter()))
                q.append(submit())
            if log:
                log(("fetch", k, time.perf_counter()))
            kp += finish(q.popleft())
            if log:
                log(("done", k, time.perf_counter()))
        return kp

    run(max(1, args.warmup))
    kp_per_image = ctx.counts()["final_n"] // B
    # the pyramid's / extrema scan's algorithmic bytes and launches per image,
    # from the library's per-launch accounting on one profiled job
    ctx.profile_table(reset=True)
    ctx.set_profiling(True)
    ctx.fetch(submit())
    ctx.set_profiling(False)
    prof0 = ctx.profile_table(reset=True)
    pyr_bytes_img = sum(r[1] for r in prof0[PROF_PYRAMID:PROF_PYRAMID + 16]) / B
    pyr_launches_img = sum(r[2] for r in prof0[PROF_PYRAMID:PROF_PYRAMID + 16]) / B
    ext_bytes_img = prof0[PROF_EXTREMA][1] / B
    ext_launches_img = prof0[PROF_EXTREMA][2] / B
    cnt = ctx.counts()
    dims = [(cnt["octave0_w"] >> o, cnt["octave0_h"] >> o) for o in range(cnt["octaves"])]
    if use_exchange:
        from sift_dist import RecordExchange, agree_capacity
        exchange = RecordExchange(agree_capacity(max_rows * args.exchange_steps, dev), dev,
                                  max_images=max(16, B), verify_ctx=ctx,
                                  steps_per_exchange=args.exchange_steps)
        run(1)  # one untimed pipelined step

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    sample_events = not args.no_events and args.events_every > 0
    sample_events_used = sample_events
    in_timed = True
    ctx.profile_table(reset=True)
    t0 = time.perf_counter()
    kp_total = run(args.steps)
    if exchange is not None:
        exchange.flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if step_log:
        print("step log (ms from the timed region's start):", file=sys.stderr)
        for ev, k, t in step_log:
            print(f"  {ev:6s} job {k:3d} {1e3 * (t - t0):8.3f}", file=sys.stderr)
    sample_events = in_timed = False
    ctx.set_profiling(False)
    prof = ctx.profile_table(reset=True)

    exchange_check = None
    if use_exchange:
        # end-to-end check of the last step's exchange: every rank re-detects
        # the next rank's images (the generator is deterministic) and compares
        # them byte for byte with what the all-gather delivered
        got = exchange.result((exchange.step - 1) & 1)
        peer = (rank + 1) % world
        ok, n_recv = 1, len(got)
        for j in range(B):
            i = peer * B + j
            peer_img = torch.from_numpy(synth_image(W, H, 1, seed=42 + i)).to(dev)
            torch.cuda.synchronize()  # the library's stream does not wait on torch's
            ref, _ = ctx.detect_device(peer_img.data_ptr(), W, H, 1, params)
            del peer_img
            ok &= int(i in got and got[i].cpu().numpy().tobytes() == ref.tobytes())
        bad = exchange.mismatches()
        chk = torch.tensor([ok, n_recv, bad, exchange.checked], dtype=torch.int64, device=dev)
        dist.all_reduce(chk[:2], op=dist.ReduceOp.MIN)
        dist.all_reduce(chk[2:], op=dist.ReduceOp.SUM)
        exchange_check = {"records_match_peer_redetect": bool(chk[0]),
                          "min_images_received_per_rank": int(chk[1]),
                          "images_per_step": world * B,
                          "steps_per_exchange": args.exchange_steps,
                          "slots_checksummed": int(chk[3]),
                          "slot_checksum_mismatches": int(chk[2]),
                          "note": "every step: each received slot's records summed on the device "
                                  "against its sender's checksum (sift_hip_verify_slots); last "
                                  "step: peer images re-detected and compared byte for byte"}
        t = torch.tensor([elapsed, float(kp_total)], dtype=torch.float64, device=dev)
        t_max = t.clone()
        dist.all_reduce(t_max[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        elapsed, kp_all = float(t_max[0]), float(t[1])
    else:
        kp_all = float(kp_total)

    if rank == 0:
        traffic, traffic_note = load_traffic(args.traffic_json)
        images = args.steps * B * world
        # headline roofline, chip level: the algorithmic pyramid
        # bytes of every image of the timed region over its wall time; the
        # kernel-alone figure (serialised context, dispatch-timestamped
        # events; rocprofv3 --kernel-trace of the same shape agrees,
        # profiles/) sits beside it
        roofline = chip_roofline(pyr_bytes_img, pyr_launches_img, images, elapsed,
                                 traffic.get("pyramid") if traffic else None, traffic_note)
        roofline["kernel"] = ("Gaussian pyramid: k_blur_pair (wave-pair walk, octave-0 levels "
                              "1-5) + k_blur (strip walk: the fused gray/x2 initial blur) + "
                              "k_blur_tile (LDS tiles, octaves >= 1) + k_octaves_lds "
                              "(LDS-resident small octaves); 16 B per pixel per level + 8 B per "
                              "decimated pixel (SURVEY 8d)")
        bpyr = survey_bpyr(dims, params)
        roofline["survey_bpyr_bytes_per_image"] = bpyr
        roofline["frac_survey_bpyr"] = round(bpyr * images / elapsed / 1e9 / HBM_PEAK_GBS, 4)
        fp64_img = pyramid_fp64_ops(dims, params)
        roofline["fp64"] = {"ops_per_image": fp64_img, "peak_ops_per_s": FP64_PEAK_OPS,
                            "frac": fp64_img * images / elapsed / FP64_PEAK_OPS,
                            "note": "FP64 lane-operations of the pyramid, 2(3R+4) per pixel per "
                                    "level (two passes; FMA = 1), over the same wall time"}
        extrema_roofline = chip_roofline(ext_bytes_img, ext_launches_img, images, elapsed,
                                         traffic.get("extrema") if traffic else None,
                                         traffic_note)
        extrema_roofline["kernel"] = ("k_extrema_stream (DoG on the fly, 3x3x3 non-strict test): "
                                      "8 B x (intervals+3) levels per scanned pixel")
        out = {
            "metric": METRIC,
            "value": kp_all / elapsed,
            "unit": "keypoints/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "dtype_note": ("every stage in f64 as the reference: pyramid, DoG, extrema, refine, "
                           "orientation and the descriptor's per-sample math (rotation, "
                           "magnitude, atan2, exp, trilinear weights) with f64 "
                           "histograms"),
            "data": "synthetic (deterministic integer-RNG generator: sinusoid + Gaussian blobs, "
                    "~w*h/52 blobs, sigma 1.5-7.5)",
            "config": {
                "workload": "BASELINE config 2 (config 4 layout at N>1): 1920x1080 synthetic gray "
                            "image, full detect_keypoints_and_descriptors incl. sort/unique, "
                            "reference default parameters",
                "image": f"{W}x{H}x1",
                "images_per_gpu_per_step": B,
                "jobs_in_flight": depth,
                "keypoints_per_image": kp_per_image,
                "parallelism": f"image-sharded x{world}" + (
                    ", RCCL all-gather of the descriptor records straight from HBM "
                    f"(sift_hip_fetch_device_async), one collective per {args.exchange_steps} "
                    "steps, overlapping the next steps" if use_exchange else ""),
            },
            "roofline": roofline,
            "extrema_roofline": extrema_roofline,
        }
        out["timed_region_s"] = elapsed
        if sample_events_used:
            prof_rows = prof[PROF_PYRAMID:PROF_PYRAMID + 16]
            out["timed_region_events"] = {
                "every": args.events_every,
                "pyramid_us_per_launch": [ms * 1e3 / n for ms, _, n in prof_rows if n],
                "note": "per-launch events on sampled jobs while four jobs share the chip "
                        "(launches overlap; not a kernel-quality figure)"}
        if world == 1 and not args.no_alone and not args.no_events:
            b8 = [torch.from_numpy(synth_image(W, H, 1, seed=42 + i)).to(dev) for i in range(8)]
            alone = alone_leg(dev_imgs[0], W, H, params, batch_imgs=b8)
            del b8
            roofline["alone"] = alone["pyramid"]
            roofline["alone"]["note"] = alone["note"]
            roofline["fp64"]["frac_alone"] = (fp64_img / (alone["pyramid"]["us_per_image"] * 1e-6)
                                              / FP64_PEAK_OPS)
            extrema_roofline["alone"] = alone["extrema"]
            roofline["alone_batch8"] = alone["batch"]["pyramid"]
            roofline["alone_batch8"]["note"] = alone["batch"]["note"]
            extrema_roofline["alone_batch8"] = alone["batch"]["extrema"]
            out["keypoint_kernels_alone"] = alone["keypoint_kernels"]
            out["keypoint_kernels_alone_batch8"] = alone["batch"]["keypoint_kernels"]
        if world == 1 and not args.no_extra:
            out["host_busy"] = host_busy_leg(ctx, ptrs, W, H, params, max(args.steps, 400), depth)
        if exchange_check is not None:
            out["exchange_check"] = exchange_check
        if world == 1 and not args.no_extra:
            out.update(extra_legs(ctx, dev, host_imgs, dev_imgs, W, H, params,
                                  args.extra_seconds))
        if world == 1 and not args.no_matcher:
            kps_a, _ = ctx.detect_device(dev_imgs[0].data_ptr(), W, H, 1, params)
            out["matcher"] = matcher_bench(ctx, dev, kps_a, W, H, params,
                                           0.0 if args.no_cpu_baseline else args.cpu_seconds)
        if world == 1 and not args.no_big:
            # the 1080p context (its streams and their hardware queues, its
            # slots' arenas) is released first: the big legs' jobs get the
            # process's four hardware queues to themselves
            if not use_exchange:
                ctx.close()
                ctx = None
            for name in ("config3", "config5"):
                out[name] = big_config_leg(name, dev)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(host_imgs[0], args.cpu_seconds)
            ref = cpu_baseline_reference(host_imgs[0], args.cpu_seconds)
            if ref is not None:
                out["cpu_baseline_reference"] = ref
        # the headline figures again, last, so a tail of the line carries them
        summ = {"keypoints_per_s": out["value"], "ms_per_step": out["ms_per_step"],
                "pyramid_frac_chip": roofline["frac"],
                "pyramid_frac_chip_survey_bpyr": roofline["frac_survey_bpyr"]}
        if "alone" in roofline:
            summ["pyramid_frac_alone"] = roofline["alone"]["frac"]
            summ["pyramid_us_alone"] = roofline["alone"]["us_per_image"]
            summ["extrema_frac_alone"] = extrema_roofline["alone"]["frac"]
        if "keypoint_kernels_alone" in out:
            summ["keypoint_kernels_us_alone"] = {
                k: v.get("us_per_image") for k, v in out["keypoint_kernels_alone"].items()
                if isinstance(v, dict)}
        if "latency" in out:
            summ["latency_ms_per_image"] = out["latency"]["ms_per_image"]
        for name in ("config3", "config5"):
            if name in out:
                summ[f"{name}_ms_per_image"] = out[name]["ms_per_image"]
                summ[f"{name}_pyramid_frac_alone"] = out[name]["roofline"]["alone"]["frac"]
        if "cpu_baseline_reference" in out:
            summ["x_reference_cpu_1core"] = out["value"] / out["cpu_baseline_reference"]["value"]
        out["summary"] = summ
        print(json.dumps(out), file=json_out, flush=True)

    if ctx is not None:
        ctx.close()
    if use_exchange:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
