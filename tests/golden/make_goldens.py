"""Generate the golden vectors in tests/golden/ from the REFERENCE itself.

Runs only in the build container (needs /root/reference and the harness
binaries from `make -C oracle ref`). For every case it feeds an input image
to oracle/_ref/ref_harness_cf — the reference src/sift.cpp compiled from
/root/reference with the four deep copies turned into const refs and a hook
that exposes the normalised descriptor floats (oracle/Makefile) — and, for
the small cases, also to the unmodified as-is build, asserting the two agree
byte for byte. Inputs are either regenerated deterministically by
sift_synth_image (their sha256 is stored and checked) or, for image1.jpg,
the stb-decoded pixels written by the harness.

Each case becomes tests/golden/<name>.npz (allow_pickle=False) holding:
  meta_json        parameters, per-stage counts, timings, input sha256
  final            final keypoint records (168 B each, reference layout)
                   (or, for the large cases, a 64-keypoint sample + sha256)
  desc_f32         normalised descriptor floats of the stored keypoints
  extrema          candidate list (x, y, z, octave), sorted
  pyr_sha256       sha256 of every Gaussian level, octave-major (small cases)
  input_u8         the decoded input (image1 only)

usage: python tests/golden/make_goldens.py [--big] [names...] | --match | --cli
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import subprocess
import sys
import tempfile
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "sift-project_amd"))
from sift_hip import KP_DTYPE, synth_image  # noqa: E402

sys.path.insert(0, os.path.dirname(HERE))
from golden_util import coords_sha256  # noqa: E402

HARNESS_CF = os.path.join(ROOT, "oracle", "_ref", "ref_harness_cf")
HARNESS_ASIS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
IMAGE1 = "/root/reference/stitching/image1.jpg"
IMAGE2 = "/root/reference/stitching/image2.jpg"

# name: (w, h, c, nblobs-or-None, smax, seed, intervals, double, max_octaves,
#        kind) where kind: "small" (full dump + as-is cross-check),
#        "medium" (full final list), "big" (sample + hash)
CASES = {
    "synth_64x48": (64, 48, 1, None, 6.0, 42, 3, 1, 0, "small"),
    "synth_320x240": (320, 240, 1, None, 6.0, 42, 3, 1, 0, "small"),
    "synth_161x117x3": (161, 117, 3, 800, 4.0, 7, 3, 1, 0, "small"),
    "synth_200x150_nodbl": (200, 150, 1, None, 6.0, 3, 3, 0, 0, "small"),
    "synth_300x200_int2": (300, 200, 1, None, 6.0, 5, 2, 1, 0, "small"),
    "synth_257x131_int5": (257, 131, 1, None, 6.0, 11, 5, 1, 0, "small"),
    "synth_97x61_maxoct2": (97, 61, 1, None, 4.0, 13, 3, 1, 2, "small"),
    "flat_64x64": (64, 64, 1, 0, 0.0, 1, 3, 1, 0, "small"),
    "tiny_5x4": (5, 4, 1, 2, 1.0, 2, 3, 1, 0, "small"),
    "image1": ("image1", 0, 0, None, 0.0, 0, 3, 1, 0, "medium"),
    "synth_1920x1080": (1920, 1080, 1, None, 6.0, 42, 3, 1, 0, "medium"),
}
# The parameter / shape cases of tests/test_gpu_parity.py (CASES), run
# through the reference with every detect_keypoints_and_descriptors argument
# (sift.hh:65-71) passed explicitly: (w, h, c, seed, params). Inputs: the
# deterministic generator, seed = crc32(name) & 0xFFFF as in that test.
PARAM_CASES = {
    "ragged_67x43": (67, 43, 1, {}),
    "rgb_203x151": (203, 151, 3, {}),
    "nodbl_rgb_250x190": (250, 190, 3, {"double_image_size": 0}),
    "int4_180x140": (180, 140, 1, {"intervals": 4}),
    "int1_150x110": (150, 110, 1, {"intervals": 1}),
    "win5_170x130": (170, 130, 1, {"window_size": 5}),
    "bins72_160x120": (160, 120, 1, {"num_bins": 72, "peak_ratio": 0.5}),
    "lowthr_160x120": (160, 120, 1, {"contrast_threshold": 0.02, "eigen_ratio": 5.0}),
    "oridesc_160x120": (160, 120, 1, {"ori_sigma_factor": 2.0, "desc_scale_factor": 4.0}),
    "sigma2_140x100": (140, 100, 1, {"init_sigma": 2.0}),
    "wide_sigma_90x70": (90, 70, 1, {"init_sigma": 6.5}),
    "maxoct3_300x220": (300, 220, 1, {"max_octaves": 3}),
    "tall_33x400": (33, 400, 1, {}),
    "wide_600x20": (600, 20, 1, {}),
}
DEFAULT_PARAMS = {"double_image_size": 1, "init_sigma": 1.6, "intervals": 3, "window_size": 3,
                  "contrast_threshold": 0.04, "eigen_ratio": 10.0, "num_bins": 36.0,
                  "peak_ratio": 0.8, "ori_sigma_factor": 1.5, "desc_scale_factor": 3.0,
                  "max_octaves": 0}
# Real photographs (stb decode by the reference's image_io.cpp:20-35):
# name: (path under /root/reference, crop (x0, y0, w, h) or None)
PHOTO_CASES = {
    "photo_cave01_00": ("stitching/collection/Dataset/CAVE-01_atrium/00.jpg", None),
    "photo_img6121_crop960x540": ("stitching/collection/own/IMG_6121.jpg", (1536, 1242, 960, 540)),
}
BIG_CASES = {
    # BASELINE config 3: 4096^2, "5 octaves x 5 scales" -> intervals=2 (5 Gaussian
    # levels per octave), max_octaves=5
    "synth_4096x4096_int2_oct5": (4096, 4096, 1, 300000, 6.0, 42, 2, 1, 5, "big"),
    # BASELINE config 5: 8K dense (1.5M blobs, sigma 1.5-5.5)
    "synth_7680x4320_dense": (7680, 4320, 1, 1500000, 4.0, 42, 3, 1, 0, "big"),
}


def write_raw(path, img):
    h, w = img.shape[:2]
    c = 1 if img.ndim == 2 else img.shape[2]
    with open(path, "wb") as f:
        f.write(b"SIFTRAW1" + struct.pack("<3i", w, h, c))
        f.write(np.ascontiguousarray(img, dtype="<f8").tobytes())


def read_raw(path):
    with open(path, "rb") as f:
        assert f.read(8) == b"SIFTRAW1"
        w, h, c = struct.unpack("<3i", f.read(12))
        a = np.frombuffer(f.read(), dtype="<f8")
    return a.reshape((h, w, c)) if c > 1 else a.reshape((h, w))


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def run_harness(exe, inp, prefix, intervals, dbl, max_oct, dump, params=None):
    args = [exe, inp, prefix, str(intervals), str(dbl), str(max_oct), str(int(dump))]
    if params is not None:  # the remaining sift.hh:65-71 arguments, exact reprs
        args += [str(int(params["window_size"]))] + [
            repr(float(params[k])) for k in ("init_sigma", "contrast_threshold", "eigen_ratio",
                                             "num_bins", "peak_ratio", "ori_sigma_factor",
                                             "desc_scale_factor")]
    subprocess.run(args, check=True, stdout=subprocess.DEVNULL)
    meta = {}
    with open(prefix + ".meta.txt") as f:
        for line in f:
            k, *v = line.split()
            meta.setdefault(k, []).append(v)
    return meta


def load_outputs(prefix):
    final = np.fromfile(prefix + ".final.bin", dtype=KP_DTYPE)
    ext = np.fromfile(prefix + ".ext.bin", dtype="<i4").reshape(-1, 4)
    df = np.fromfile(prefix + ".df32.bin", dtype="<f4") if os.path.exists(prefix + ".df32.bin") \
        else np.zeros(0, "<f4")
    return final, ext, df.reshape(-1, 128)


def make_case(name, spec, tmp, params=None, photo=None):
    w, h, c, nb, smax, seed, intervals, dbl, max_oct, kind = spec
    inp = os.path.join(tmp, name + ".raw")
    meta = {"name": name, "intervals": intervals, "double_image_size": dbl,
            "max_octaves": max_oct, "kind": kind}
    if params is not None:
        meta["params"] = params
    if photo is not None:
        # stb decode by the reference harness, then (optionally) a crop
        path, crop = photo
        src = os.path.join("/root/reference", path)
        probe = os.path.join(tmp, name + "_probe")
        run_harness(HARNESS_CF, src, probe, 3, 0, 1, False)
        decoded = read_raw(probe + ".input.raw")
        if crop is not None:
            x0, y0, cw, ch = crop
            decoded = np.ascontiguousarray(decoded[y0:y0 + ch, x0:x0 + cw])
        write_raw(inp, decoded)
        meta["source"] = f"{path} (stb decode via reference image_io.cpp:20-35)" + (
            f", crop x0={crop[0]} y0={crop[1]} {crop[2]}x{crop[3]}" if crop else "")
        w = "photo"
    elif w == "image1":
        inp = IMAGE1
        meta["source"] = "stitching/image1.jpg (stb decode via reference image_io.cpp:20-35)"
    else:
        img = synth_image(w, h, c, nblobs=nb, smax=smax, seed=seed)
        write_raw(inp, img)
        meta.update(source="sift_synth_image", w=w, h=h, c=c,
                    nblobs=nb if nb is not None else max(1, (w * h) // 52), smax=smax,
                    seed=seed, input_sha256=sha(np.ascontiguousarray(img, "<f8").tobytes()))
    prefix = os.path.join(tmp, name + "_cf")
    rm = run_harness(HARNESS_CF, inp, prefix, intervals, dbl, max_oct, kind == "small", params)
    final, ext, df = load_outputs(prefix)
    for k in ("octaves", "levels", "extrema", "refined", "oriented", "final"):
        meta[k] = int(rm[k][0][0])
    meta["octave_dims"] = [[int(v) for v in d[1:]] for d in rm.get("octave_dims", [])]
    meta["ref_time_s"] = {k[5:]: float(v[0][0]) for k, v in rm.items() if k.startswith("time_")}
    meta["final_sha256"] = sha(final.tobytes())
    meta["coords_sha256"] = coords_sha256(final)
    meta["desc_f32_sha256"] = sha(df.tobytes())
    out = {}
    if w == "photo":
        decoded = read_raw(inp)
        meta.update(w=decoded.shape[1], h=decoded.shape[0], c=decoded.shape[2],
                    input_sha256=sha(np.ascontiguousarray(decoded, "<f8").tobytes()))
        out["input_u8"] = decoded.astype(np.uint8)
        assert np.array_equal(out["input_u8"].astype(np.float64), decoded)
    if w == "image1":
        decoded = read_raw(prefix + ".input.raw")
        meta.update(w=decoded.shape[1], h=decoded.shape[0], c=decoded.shape[2],
                    input_sha256=sha(np.ascontiguousarray(decoded, "<f8").tobytes()))
        out["input_u8"] = decoded.astype(np.uint8)
        assert np.array_equal(out["input_u8"].astype(np.float64), decoded)
    order = np.lexsort((ext[:, 2], ext[:, 1], ext[:, 0], ext[:, 3]))
    ext = ext[order]
    if kind == "small":
        # the unmodified reference must agree byte for byte
        p2 = os.path.join(tmp, name + "_asis")
        run_harness(HARNESS_ASIS, inp, p2, intervals, dbl, max_oct, True, params)
        f2, e2, _ = load_outputs(p2)
        assert f2.tobytes() == final.tobytes(), name
        with open(prefix + ".pyr.bin", "rb") as f1, open(p2 + ".pyr.bin", "rb") as g2:
            pyr = f1.read()
            assert pyr == g2.read(), name
        hashes, off = [], 0
        for (ow, oh) in meta["octave_dims"]:
            for _ in range(meta["levels"]):
                n = ow * oh * 8
                hashes.append(sha(pyr[off:off + n]))
                off += n
        assert off == len(pyr)
        out["pyr_sha256"] = np.array(hashes)
        meta["asis_crosscheck"] = True
    if kind in ("small", "medium"):
        out["final"] = np.frombuffer(final.tobytes(), dtype=np.uint8)
        out["desc_f32"] = df
        out["extrema"] = ext
    else:
        rng = np.random.default_rng(0)
        idx = np.sort(rng.choice(len(final), size=min(64, len(final)), replace=False))
        out["sample_idx"] = idx
        out["final"] = np.frombuffer(final[idx].tobytes(), dtype=np.uint8)
        out["desc_f32"] = df[idx]
        meta["extrema_sha256"] = sha(ext.astype("<i4").tobytes())
        # every keypoint's descriptor bytes and orientation (the records'
        # remaining fields are pinned by coords_sha256), plus the normalised
        # descriptor floats of a 4096-keypoint stratified sample: one random
        # keypoint from each of 4096 equal slices of the sorted list
        out["desc_u8_all"] = np.ascontiguousarray(final["desc"])
        out["pori_all"] = np.ascontiguousarray(final["pori"], dtype="<f8")
        n = len(final)
        ns = min(4096, n)
        edges = (np.arange(ns + 1) * n) // ns
        sidx = edges[:-1] + (rng.random(ns) * (edges[1:] - edges[:-1])).astype(np.int64)
        out["strat_idx"] = sidx
        out["strat_desc_f32"] = df[sidx]
    out["meta_json"] = np.array(json.dumps(meta, sort_keys=True))
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(f"{name}: octaves={meta['octaves']} extrema={meta['extrema']} "
          f"final={meta['final']} ref_total={meta['ref_time_s'].get('total', 0):.2f}s")


def ref_match(k1, k2, ratio, tmp):
    """The reference match_keypoints (sift.cpp:783-815) via `ref_harness --match`."""
    a, b, o = (os.path.join(tmp, n) for n in ("m1.bin", "m2.bin", "mo.bin"))
    k1.tofile(a)
    k2.tofile(b)
    subprocess.run([HARNESS_ASIS, "--match", a, b, repr(float(ratio)), o], check=True,
                   stdout=subprocess.DEVNULL)
    return np.fromfile(o, dtype=MATCH_DTYPE)


MATCH_DTYPE = np.dtype([("i1", "<i4"), ("i2", "<i4"), ("distance", "<f8")])


def records_from_desc(desc):
    """Keypoint records carrying only descriptors (x = index keeps them distinct)."""
    k = np.zeros(len(desc), dtype=KP_DTYPE)
    k["x"] = np.arange(len(desc))
    k["desc"] = desc
    return k


def make_match(tmp):
    """tests/golden/match_cases.npz: the reference matcher on
      image1_image2  final keypoints of stitching/image1.jpg vs image2.jpg
                     (main.cpp:15-17, ratio 0.75 = sift.hh default)
      ties_*         tie-heavy descriptors (bytes in {0,1,2}, duplicated rows)
                     at ratios 0.75, 1.0, 1.5
      single_ref     n2 == 1 (second distance = DBL_MAX)
    Each case stores desc1, desc2 (u8 [n,128]), ratio and matches (i1, i2, d)."""
    out = {}
    finals = []
    for img in (IMAGE1, IMAGE2):
        prefix = os.path.join(tmp, os.path.basename(img) + "_m")
        run_harness(HARNESS_CF, img, prefix, 3, 1, 0, False)
        finals.append(np.fromfile(prefix + ".final.bin", dtype=KP_DTYPE))
    cases = {"image1_image2": (finals[0]["desc"], finals[1]["desc"], 0.75)}
    rng = np.random.default_rng(5)
    d1 = rng.integers(0, 3, size=(300, 128), dtype=np.uint8)
    d2 = rng.integers(0, 3, size=(257, 128), dtype=np.uint8)
    d2[100:140] = d2[60:100]        # exact duplicate references
    d1[:40] = d2[60:100]            # queries equal to duplicated references
    d1[40:60] = d2[0:20]            # queries equal to unique references
    for r in (0.75, 1.0, 1.5):
        cases[f"ties_{r}"] = (d1, d2, r)
    cases["single_ref"] = (d1[:37], d2[5:6], 0.75)
    for name, (a, b, r) in cases.items():
        m = ref_match(records_from_desc(a), records_from_desc(b), r, tmp)
        out[name + "__desc1"] = a
        out[name + "__desc2"] = b
        out[name + "__ratio"] = np.array(r)
        out[name + "__matches"] = m
        print(f"match {name}: {len(a)} x {len(b)} ratio {r} -> {len(m)} matches")
    out["names"] = np.array(list(cases))
    np.savez_compressed(os.path.join(HERE, "match_cases.npz"), **out)


def make_cli(tmp):
    """tests/golden/cli_outputs.json + the two input images: the reference
    CLI (main.cpp:6-19, copy-fixed build oracle/_ref/sift_cf) on
    stitching/image1.jpg and image2.jpg; sha256 of the keypoints.png (written
    by every detect, sift.cpp:765-768: the last one, image2's) and
    matches.png (sift.cpp:850-876) it leaves behind."""
    import shutil
    cli = os.path.join(ROOT, "oracle", "_ref", "sift_cf")
    for src, dst in ((IMAGE1, "cli_image1.jpg"), (IMAGE2, "cli_image2.jpg")):
        shutil.copyfile(src, os.path.join(HERE, dst))
        shutil.copyfile(src, os.path.join(tmp, dst))
    subprocess.run([cli, "cli_image1.jpg", "cli_image2.jpg"], cwd=tmp, check=True,
                   stdout=subprocess.DEVNULL)
    res = {"command": "sift cli_image1.jpg cli_image2.jpg (reference main.cpp, copy-fixed "
                      "sift.cpp, oracle/_ref/sift_cf)",
           "inputs": {n: sha(open(os.path.join(HERE, n), "rb").read())
                      for n in ("cli_image1.jpg", "cli_image2.jpg")}}
    for f in ("keypoints.png", "matches.png"):
        res[f] = sha(open(os.path.join(tmp, f), "rb").read())
    with open(os.path.join(HERE, "cli_outputs.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("cli:", res)


def main():
    for exe in (HARNESS_CF, HARNESS_ASIS):
        if not os.path.exists(exe):
            sys.exit(f"{exe} missing: run `make -C oracle ref` (build container only)")
    cases = dict(CASES)
    if "--big" in sys.argv:
        cases.update(BIG_CASES)
    only = [a for a in sys.argv[1:] if not a.startswith("--")]
    if "--cli" in sys.argv:
        with tempfile.TemporaryDirectory() as tmp:
            make_cli(tmp)
        return
    if "--match" in sys.argv:
        with tempfile.TemporaryDirectory() as tmp:
            make_match(tmp)
        return
    with tempfile.TemporaryDirectory() as tmp:
        for name, spec in cases.items():
            if only and name not in only:
                continue
            make_case(name, spec, tmp)
        for name, (w, h, c, over) in PARAM_CASES.items():
            gname = "case_" + name
            if only and gname not in only:
                continue
            prm = dict(DEFAULT_PARAMS, **over)
            spec = (w, h, c, None, 6.0, zlib.crc32(name.encode()) & 0xFFFF, prm["intervals"],
                    prm["double_image_size"], prm["max_octaves"], "small")
            make_case(gname, spec, tmp, params=prm)
        for name, photo in PHOTO_CASES.items():
            if only and name not in only:
                continue
            prm = dict(DEFAULT_PARAMS)
            make_case(name, (0, 0, 0, None, 0.0, 0, 3, 1, 0, "medium"), tmp, params=prm,
                      photo=photo)


if __name__ == "__main__":
    main()
