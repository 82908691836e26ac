"""Print HIP-vs-golden mismatches for named goldens (GPU diagnostic).

usage: python tests/diag_golden.py synth_1920x1080 [...]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from golden_util import Golden, GOLDEN_DIR  # noqa: E402
from parity import compare_final  # noqa: E402
from sift_hip import Context  # noqa: E402


def show(tag, k):
    print(f"  {tag}: x={k['x']!r} y={k['y']!r} oct={k['octave']} layer={k['layer']} "
          f"size={k['size']!r} pori={k['pori']!r} desc[:8]={list(k['desc'][:8])}")


def main(names):
    ctx = Context(0)
    for name in names:
        g = Golden(os.path.join(GOLDEN_DIR, name + ".npz"))
        kps, df = ctx.detect(g.input(), g.params(), desc_f32=True)
        r = compare_final(kps, df, g.final, g.desc_f32)
        print(name, r)
        if len(kps) != len(g.final):
            continue
        bad = np.nonzero((kps["x"] != g.final["x"]) | (kps["y"] != g.final["y"]) |
                         (kps["size"] != g.final["size"]) | (kps["octave"] != g.final["octave"]) |
                         (kps["layer"] != g.final["layer"]) |
                         (np.abs(kps["pori"] - g.final["pori"]) > 1e-9))[0]
        for i in bad[:10]:
            print(f" index {i}:")
            for j in range(max(0, i - 2), min(len(kps), i + 3)):
                show(f"gpu[{j}]", kps[j])
                show(f"ref[{j}]", g.final[j])


if __name__ == "__main__":
    main(sys.argv[1:])
