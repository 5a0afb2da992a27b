"""Interleaved A/B of kernel time per frame: librm.so and tools/variants/librm_*.so.

  python tools/ab_kernel.py [--cfg 3] [--rounds 4] [--frames 30] [--table] [--spec] [variant.so ...]

RM_AB_WIDE=1 with --table / --spec: the reference scene with two more spheres
before its floor (7 bounded entries: the tables' 8-slot instances).

--batch B --ctx N times throughput instead: the frames as rm_dispatch_frames
batches of B over N contexts (wall time per frame, after a 0.3 s spin-up).

A variant given as DIR/ (a directory holding librm.so and the rmarch package of
an older revision, e.g. tools/variants/r2pkg/) is driven through its own
rmarch, so libraries of an older C-ABI can be timed against the current one.

Each (round, variant) runs in its own process (RM_LIBRM selects the library);
the variants alternate within every round, so box drift hits them alike.  Each
run renders `frames` sweep frames one at a time (HIP events on the context's
stream) and reports the mean kernel ms per frame; the summary is the median
over rounds.  Diagnostic tool, not part of the product.
"""
import argparse
import glob
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFGS = {1: (512, 512, 0, False, 1), 2: (1920, 1080, 1, False, 0), 3: (3840, 2160, 3, True, 0),
        4: (3840, 2160, 5, True, 0), 5: (7680, 4320, 3, True, 0)}


def table_scene(rm):
    """The reference scene as a runtime table (RM_AB_WIDE=1: two more spheres
    before its floor, 7 bounded entries: the tables' 8-slot instances)."""
    sc = rm.default_scene()
    if os.environ.get("RM_AB_WIDE") == "1":
        import ctypes as C
        extra = []
        for dx in (40.0, -40.0):
            q = rm.rm_primitive()
            C.memmove(C.byref(q), C.byref(sc[0]), C.sizeof(q))
            q.center[0] += dx
            extra.append(q)
        sc = sc[:-1] + extra + sc[-1:]
    return sc


def child_batch(cfg, frames, B, nctx, table=False, spec=False):
    import time
    sys.path.insert(0, os.environ.get("RM_PKG_DIR") or os.path.join(ROOT, "opengl-raymarching-in-compute-shader_amd"))
    import torch  # noqa: F401
    import rmarch as rm

    W, H, b, aa, sm = CFGS[cfg]
    us = [rm.sweep_uniforms((k * 120) // frames, 120, b, aa, sm) for k in range(frames)]
    rs = [rm.Renderer(W, H) for _ in range(nctx)]
    for r in rs:
        if spec:
            r.specialize_scene(True)
        if table or spec:
            r.set_scene(table_scene(rm))

    def run():
        for j, i in enumerate(range(0, frames, B)):
            if B == 1:  # single frames through rm_dispatch (k_sample / k_pixel), as bench.py
                rs[j % nctx].dispatch(us[i])
            else:
                rs[j % nctx].dispatch_frames(us[i:i + B])
        for r in rs:
            r.synchronize()
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        run()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        run()
        ts.append((time.perf_counter() - t0) * 1e3 / frames)
    ts.sort()
    print(json.dumps({"ms": ts[len(ts) // 2]}))


def child(cfg, frames, table, spec=False):
    sys.path.insert(0, os.environ.get("RM_PKG_DIR") or os.path.join(ROOT, "opengl-raymarching-in-compute-shader_amd"))
    import rmarch as rm

    W, H, b, aa, sm = CFGS[cfg]
    with rm.Renderer(W, H) as r:
        if spec:
            r.specialize_scene(True)
        if table or spec:
            r.set_scene(table_scene(rm))
        r.enable_timing(True)
        for f in range(3):
            r.dispatch(rm.sweep_uniforms(f, 120, b, aa, sm))
        r.kernel_time_ms(reset=True)
        for k in range(frames):
            r.dispatch(rm.sweep_uniforms((k * 120) // frames, 120, b, aa, sm))
        ms, n = r.kernel_time_ms(reset=True)
    print(json.dumps({"ms": ms / n}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--table", action="store_true", help="the reference scene through the table kernel")
    ap.add_argument("--spec", action="store_true", help="the same, specialised for the table (hiprtc)")
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--ctx", type=int, default=1)
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    if a.child:
        if a.batch:
            return child_batch(a.cfg, a.frames, a.batch, a.ctx, a.table, a.spec)
        return child(a.cfg, a.frames, a.table, a.spec)
    libs = a.libs or ([os.path.join(ROOT, "opengl-raymarching-in-compute-shader_amd/librm.so")]
                      + sorted(p for p in glob.glob(os.path.join(ROOT, "tools/variants/librm_*.so"))
                               if "librm_stats" not in p))
    res = {p: [] for p in libs}
    for _ in range(a.rounds):
        for p in libs:
            if p.endswith("/"):  # an older revision: its own rmarch and librm.so
                env = dict(os.environ, RM_PKG_DIR=p, RM_LIBRM=os.path.join(p, "librm.so"))
            else:
                env = dict(os.environ, RM_LIBRM=p)
            out = subprocess.run([sys.executable, __file__, "--child", "--cfg", str(a.cfg), "--frames",
                                  str(a.frames), "--batch", str(a.batch), "--ctx", str(a.ctx)]
                                 + (["--table"] if a.table else []) + (["--spec"] if a.spec else []),
                                 env=env, capture_output=True, text=True, timeout=120)
            if out.returncode != 0:
                sys.stderr.write(out.stderr)
                sys.exit(out.returncode)
            res[p].append(json.loads(out.stdout.strip().splitlines()[-1])["ms"])
    base = statistics.median(res[libs[0]])
    for p in libs:
        m = statistics.median(res[p])
        print("cfg%d %-28s median %.4f ms (%+.2f%%)  runs %s" % (
            a.cfg, os.path.basename(p.rstrip("/")), m, 100.0 * (m / base - 1.0), " ".join("%.4f" % x for x in res[p])),
            flush=True)


if __name__ == "__main__":
    main()
