"""Throughput of frame batches against frames in flight (diagnostic, not product).

  python tools/probe_batch.py [--cfg 2] [--rounds 7] [--steps 20]

One process, one BASELINE config.  Each round times the bench's K sweep frames
(step k -> frame floor(k * 120 / K)) under every variant, interleaved so box
drift hits them alike; prints the median ms per frame per variant.  Variants:
  fl<N>        N contexts in flight, one rm_dispatch per frame (bench.py --batch 1)
  b<B>x<N>     rm_dispatch_frames of B frames, batches alternating over N contexts
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "opengl-raymarching-in-compute-shader_amd"))

CFGS = {1: (512, 512, 0, False, 1), 2: (1920, 1080, 1, False, 0), 3: (3840, 2160, 3, True, 0),
        4: (3840, 2160, 5, True, 0), 5: (7680, 4320, 3, True, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--variants", default="fl1,fl3,b5x1,b10x1,b20x1,b4x2,b5x2,b10x2,b2x3,b4x3")
    a = ap.parse_args()
    import torch  # noqa: F401  (shares torch's HIP runtime with librm)
    import rmarch as rm

    W, H, b, aa, sm = CFGS[a.cfg]
    frames = [(k * 120) // a.steps for k in range(a.steps)]
    us = [rm.sweep_uniforms(f, 120, b, aa, sm) for f in frames]
    rs = [rm.Renderer(W, H) for _ in range(4)]

    def run(v):
        if v.startswith("fl"):
            n = int(v[2:])
            for k, u in enumerate(us):
                rs[k % n].dispatch(u)
        else:
            B, n = (int(x) for x in v[1:].split("x"))
            for j, i in enumerate(range(0, len(us), B)):
                rs[j % n].dispatch_frames(us[i:i + B])
        for r in rs:
            r.synchronize()

    variants = a.variants.split(",")
    t_end = time.perf_counter() + 0.3  # spin-up to sustained clocks
    while time.perf_counter() < t_end:
        run("fl3")
    res = {v: [] for v in variants}
    for _ in range(a.rounds):
        for v in variants:
            run(v)  # untimed: warm the variant's buffers
            t0 = time.perf_counter()
            run(v)
            res[v].append((time.perf_counter() - t0) * 1e3 / len(us))
    base = statistics.median(res[variants[0]])
    out = {}
    for v in variants:
        m = statistics.median(res[v])
        out[v] = round(m, 5)
        print("cfg%d %-8s median %.4f ms/frame (%+.2f%% vs %s)  %.0f fps  runs %s" % (
            a.cfg, v, m, 100 * (m / base - 1), variants[0], 1e3 / m, " ".join("%.4f" % x for x in res[v])),
            flush=True)
    print(json.dumps({"cfg": a.cfg, "steps": a.steps, "ms_per_frame": out}))
    for r in rs:
        r.close()


if __name__ == "__main__":
    main()
