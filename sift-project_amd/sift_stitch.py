"""Stitching consumer on the MI355X SIFT path.

The reference's consumer of `detect_keypoints_and_descriptors` +
`match_keypoints` is its stitching notebook (stitching/sift_stitch.ipynb,
absent from the checkout: .MISSING_LARGE_BLOBS:3). What survives are its
inputs: image sequences with a stitch graph each,
stitching/collection/Dataset/<name>/<name>-STITCH-GRAPH.txt, lines of the form
`{key | value | description}` with keys center_image_index,
center_image_rotation_angle, images_count and matching_graph_image_edges-<i>
(comma-separated neighbours j of image i). This module stitches such a
dataset with the GPU path end to end:

* every image through the HIP detector (jobs of same-shape images, several in
  flight: sift_hip_submit / sift_hip_fetch);
* every graph edge (i, j) through the GPU 2-NN ratio matcher (queries j,
  references i; reference match_keypoints, src/sift.cpp:783-815) and GPU
  RANSAC (sift_hip_ransac_homography): H_ij maps image j into image i;
* a breadth-first spanning tree from the centre image composes
  H_center<-j (inverting edges walked backwards), then the centre rotation;
* the canvas bounds the warped image corners, and the GPU composites the
  feather-blended panorama (sift_hip_warp_blend).

No CPU fallback: every step that touches pixels or descriptors goes through
libsift_hip.so.
"""
from __future__ import annotations

import argparse
import collections
import dataclasses
import glob
import os
import re
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from sift_hip import INPUT_U8_HOST, MAX_INFLIGHT, Context, SiftParams  # noqa: E402

_LINE = re.compile(r"^\{\s*([^|]+?)\s*\|\s*([^|]*?)\s*\|.*\}\s*$")


@dataclasses.dataclass
class StitchGraph:
    center: int
    rotation: float
    count: int
    edges: dict  # i -> [j, ...]

    def pairs(self):
        """Undirected edges (i, j), i < j, each once, in file order."""
        seen, out = set(), []
        for i, js in self.edges.items():
            for j in js:
                e = (min(i, j), max(i, j))
                if e not in seen and i != j:
                    seen.add(e)
                    out.append(e)
        return out


def read_stitch_graph(path: str) -> StitchGraph:
    """Parse a <name>-STITCH-GRAPH.txt file."""
    kv = {}
    edges = {}
    with open(path) as f:
        for raw in f:
            m = _LINE.match(raw.strip())
            if not m:
                continue
            key, val = m.group(1), m.group(2)
            if key.startswith("matching_graph_image_edges-"):
                i = int(key.rsplit("-", 1)[1])
                edges[i] = [int(t) for t in val.split(",") if t.strip()]
            else:
                kv[key] = val
    return StitchGraph(center=int(kv.get("center_image_index", 0)),
                       rotation=float(kv.get("center_image_rotation_angle", 0.0)),
                       count=int(kv.get("images_count", len(edges) + 1)), edges=edges)


def load_dataset(directory: str):
    """(graph, images): the dataset's stitch graph and its images in name
    order as HWC uint8 (PIL decode; the reference decodes with stb, channels
    capped at 3, image_io.cpp:20-35). Graph indices past the files are
    dropped."""
    from PIL import Image

    graphs = glob.glob(os.path.join(directory, "*-STITCH-GRAPH.txt"))
    if not graphs:
        raise FileNotFoundError(f"no *-STITCH-GRAPH.txt in {directory}")
    g = read_stitch_graph(graphs[0])
    files = sorted(f for f in glob.glob(os.path.join(directory, "*"))
                   if f.lower().endswith((".jpg", ".jpeg", ".png")))
    images = [np.asarray(Image.open(f).convert("RGB")) for f in files]
    return g, images


def keypoint_xy(kps: np.ndarray) -> np.ndarray:
    return np.stack([kps["x"], kps["y"]], axis=1).astype(np.float64)


def detect_all(ctx: Context, images, params: SiftParams | None = None, max_batch: int = 8):
    """Keypoints of every image: jobs of up to max_batch same-shape images,
    up to MAX_INFLIGHT - 1 jobs in flight."""
    groups = collections.defaultdict(list)
    for i, im in enumerate(images):
        groups[im.shape].append(i)
    jobs = []
    for shape, idx in groups.items():
        for k in range(0, len(idx), max_batch):
            jobs.append((shape, idx[k:k + max_batch]))
    out = [None] * len(images)
    q = collections.deque()

    def drain_one():
        t, idx = q.popleft()
        kps, _ = ctx.fetch(t)
        for i, k in zip(idx, kps):
            out[i] = k

    for shape, idx in jobs:
        if len(q) == MAX_INFLIGHT - 1:
            drain_one()
        h, w = shape[:2]
        c = shape[2] if len(shape) == 3 else 1
        arrs = [np.ascontiguousarray(images[i], dtype=np.uint8) for i in idx]
        t = ctx.submit(arrs, INPUT_U8_HOST, w, h, c, params)
        q.append((t, idx))
    while q:
        drain_one()
    return out


@dataclasses.dataclass
class PairResult:
    i: int
    j: int
    H: np.ndarray  # 3x3, image j -> image i
    matches: int
    inliers: int


def pair_homography(ctx: Context, kps_i, kps_j, i: int, j: int, ratio: float = 0.75,
                    min_matches: int = 8, **ransac) -> PairResult | None:
    """H mapping image j into image i from the GPU matcher + GPU RANSAC."""
    if len(kps_i) < 2 or len(kps_j) < 2:
        return None
    m = ctx.match(kps_j, kps_i, ratio)
    if len(m) < min_matches:
        return None
    src = keypoint_xy(kps_j)[m["i1"]]
    dst = keypoint_xy(kps_i)[m["i2"]]
    H, mask, n_in = ctx.ransac_homography(src, dst, **ransac)
    if n_in < min_matches:
        return None
    return PairResult(i, j, H, len(m), n_in)


def compose(graph: StitchGraph, pairs, n_images: int):
    """H_center<-k for every image reachable from the centre (BFS over the
    estimated edges, file order), with the centre rotation applied about the
    origin of the centre image."""
    adj = collections.defaultdict(list)
    for p in pairs:
        adj[p.i].append((p.j, p.H))                 # j -> i
        adj[p.j].append((p.i, np.linalg.inv(p.H)))  # i -> j
    c = graph.center if graph.center < n_images else 0
    a = graph.rotation
    R = np.array([[np.cos(a), -np.sin(a), 0.0], [np.sin(a), np.cos(a), 0.0], [0.0, 0.0, 1.0]])
    Hs = {c: R}
    q = collections.deque([c])
    while q:
        u = q.popleft()
        for v, H_uv in adj[u]:  # H_uv maps v into u
            if v not in Hs:
                Hs[v] = Hs[u] @ H_uv
                q.append(v)
    return Hs


def canvas_for(images, Hs, max_side: int = 8192, center=None):
    """Translation + size of the canvas holding every warped image corner,
    clipped to max_side per axis around the centre image's projected box
    (compose() inserts the centre first). Images with a corner behind the
    camera are left out; if that leaves none, the canvas is the centre
    image's own box."""
    if center is None:
        center = next(iter(Hs))

    def corners(k):
        h, w = images[k].shape[:2]
        c = np.array([[0, 0, 1], [w - 1, 0, 1], [0, h - 1, 1], [w - 1, h - 1, 1]], float).T
        p = Hs[k] @ c
        return None if np.any(p[2] <= 0) else (p[:2] / p[2]).T

    pts = [q for q in (corners(k) for k in Hs) if q is not None]
    cpts = corners(center)
    if cpts is None:  # centre rotated/projected behind the camera: its raw box
        h, w = images[center].shape[:2]
        cpts = np.array([[0.0, 0.0], [w - 1.0, h - 1.0]])
    if not pts:
        pts = [cpts]
    pts = np.concatenate(pts)
    lo = np.floor(pts.min(axis=0))
    hi = np.ceil(pts.max(axis=0))
    mid = 0.5 * (cpts.min(axis=0) + cpts.max(axis=0))
    lo = np.maximum(lo, np.floor(mid - max_side / 2))
    hi = np.minimum(hi, np.floor(mid - max_side / 2) + max_side - 1)
    T = np.array([[1.0, 0.0, -lo[0]], [0.0, 1.0, -lo[1]], [0.0, 0.0, 1.0]])
    return T, int(hi[0] - lo[0]) + 1, int(hi[1] - lo[1]) + 1


@dataclasses.dataclass
class StitchResult:
    panorama: np.ndarray
    H_canvas: dict      # image index -> canvas-from-image homography
    pairs: list         # PairResult per estimated edge
    keypoints: list     # per image
    placed: list        # image indices on the canvas


def stitch(ctx: Context, images, graph: StitchGraph, params: SiftParams | None = None,
           ratio: float = 0.75, max_side: int = 8192, **ransac) -> StitchResult:
    n = len(images)
    kps = detect_all(ctx, images, params)
    pairs = []
    for i, j in graph.pairs():
        if i < n and j < n:
            r = pair_homography(ctx, kps[i], kps[j], i, j, ratio, **ransac)
            if r is not None:
                pairs.append(r)
    Hs = compose(graph, pairs, n)
    T, W, H = canvas_for(images, Hs, max_side)
    placed = sorted(Hs)
    Hc = {k: T @ Hs[k] for k in placed}
    Hinv = np.stack([np.linalg.inv(Hc[k]) for k in placed])
    pano = ctx.warp_blend([images[k] for k in placed], Hinv, W, H)
    return StitchResult(pano, Hc, pairs, kps, placed)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="stitch a dataset directory on the GPU")
    ap.add_argument("dataset", help="directory with images and <name>-STITCH-GRAPH.txt")
    ap.add_argument("--out", default="panorama.png")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--ratio", type=float, default=0.75)
    args = ap.parse_args(argv)
    from PIL import Image

    graph, images = load_dataset(args.dataset)
    ctx = Context(args.device)
    try:
        res = stitch(ctx, images, graph, ratio=args.ratio)
    finally:
        ctx.close()
    Image.fromarray(res.panorama.squeeze()).save(args.out)
    for p in res.pairs:
        print(f"edge {p.i}<-{p.j}: {p.matches} matches, {p.inliers} inliers")
    print(f"{len(res.placed)}/{len(images)} images placed, canvas "
          f"{res.panorama.shape[1]}x{res.panorama.shape[0]} -> {args.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
