"""Stitching fixture (tests/golden/stitch/): images 00-04 of the reference's
stitching/collection/Dataset/CAVE-04_times_square (data files, copied as
bytes) and the part of its CAVE-04_times_square-STITCH-GRAPH.txt among them,
rewritten in the same `{key | value | description}` format with centre 2.
Run in the build container (needs /root/reference):
    python tests/golden/make_stitch_fixture.py
"""
import os
import re
import shutil

SRC = "/root/reference/stitching/collection/Dataset/CAVE-04_times_square"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stitch")
KEEP = 5


def main():
    os.makedirs(OUT, exist_ok=True)
    for i in range(KEEP):
        shutil.copyfile(os.path.join(SRC, f"{i:02d}.jpg"), os.path.join(OUT, f"{i:02d}.jpg"))
    edges = {}
    pat = re.compile(r"^\{matching_graph_image_edges-(\d+) \| ([0-9,]+) \|")
    for line in open(os.path.join(SRC, "CAVE-04_times_square-STITCH-GRAPH.txt")):
        m = pat.match(line.strip())
        if m and int(m.group(1)) < KEEP:
            js = [j for j in map(int, m.group(2).split(",")) if j < KEEP]
            if js:
                edges[int(m.group(1))] = js
    with open(os.path.join(OUT, "cave04_sub-STITCH-GRAPH.txt"), "w") as f:
        f.write("{center_image_index | 2 | center image index}\n")
        f.write("{center_image_rotation_angle | 0 | center image rotation angle}\n")
        f.write(f"{{images_count | {KEEP} | images count}}\n")
        for i, js in sorted(edges.items()):
            f.write(f"{{matching_graph_image_edges-{i} | {','.join(map(str, js))} | "
                    f"matching graph image edge {i}}}\n")


if __name__ == "__main__":
    main()
