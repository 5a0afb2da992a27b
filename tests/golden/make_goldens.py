"""Generate tests/golden/oracle_goldens.npz: small oracle renders of the BASELINE
configs with their exact work counters.

These pin the oracle across rebuilds/compilers (tests/test_goldens.py) and let
GPU tests check librm without running the oracle (tests/test_gpu_goldens.py).
Regenerate only when the oracle intentionally changes:
    python tests/golden/make_goldens.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "opengl-raymarching-in-compute-shader_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import rmarch as rm  # noqa: E402
import oracle as O  # noqa: E402

# name: (W, H, frame, bounces, AA, shadow_mode)
CASES = {
    "cfg1_D": (128, 128, -1, 0, False, 1),
    "cfg1_f0": (128, 128, 0, 0, False, 1),
    "cfg1_f60": (128, 128, 60, 0, False, 1),
    "cfg1_f119": (128, 128, 119, 0, False, 1),
    "cfg2_f0": (96, 54, 0, 1, False, 0),
    "cfg2_f60": (96, 54, 60, 1, False, 0),
    "cfg2_f119": (96, 54, 119, 1, False, 0),
    "cfg3_f0": (96, 54, 0, 3, True, 0),
    "cfg3_f60": (96, 54, 60, 3, True, 0),
    "cfg3_f119": (96, 54, 119, 3, True, 0),
    "cfg4_f60": (64, 36, 60, 5, True, 0),
    "default_D": (64, 64, -1, 0, True, 0),
}


def main():
    arrays, meta = {}, {}
    for name, (W, H, f, b, aa, sm) in CASES.items():
        u = rm.sweep_uniforms(f, 120, b, aa, sm)
        r = O.render(u, W, H)
        arrays[name + "_rgba8"] = r["rgba8"]
        arrays[name + "_rgba32f"] = r["rgba32f"]
        arrays[name + "_counts"] = r["sdf_counts"]
        meta[name] = {"W": W, "H": H, "frame": f, "bounces": b, "aa": aa, "shadow": sm,
                      "counters": r["counters"], "full_counters": r["full_counters"]}
    np.savez_compressed(os.path.join(HERE, "oracle_goldens.npz"), **arrays)
    with open(os.path.join(HERE, "oracle_goldens.json"), "w") as fh:
        json.dump(meta, fh, indent=1, sort_keys=True)
    print("wrote", len(CASES), "cases")


if __name__ == "__main__":
    main()
