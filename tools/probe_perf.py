"""Perf probe: kernel time per variant / batch threshold, SIMD utilisation."""
import sys, os, json
sys.path.insert(0, 'opengl-raymarching-in-compute-shader_amd')
import rmarch as rm
cfgs = {3: (3840, 2160, 3, True, 0), 2: (1920, 1080, 1, False, 0)}
variants = [("pixel", rm.RM_KERNEL_PIXEL, None)] + [("wq", rm.RM_KERNEL_WAVEQUEUE, b) for b in sys.argv[1:]]
for ci in (3, 2):
    W, H, b, aa, sm = cfgs[ci]
    for kname, k, batch in variants:
        if batch is not None:
            os.environ["RM_WQ_BATCH"] = str(batch)
        with rm.Renderer(W, H, kernel=k) as r:
            r.enable_timing(True)
            for f in range(3): r.dispatch(rm.sweep_uniforms(f, 120, b, aa, sm))
            r.kernel_time_ms(reset=True)
            for f in range(10): r.dispatch(rm.sweep_uniforms(f, 120, b, aa, sm))
            ms, n = r.kernel_time_ms(reset=True)
        line = {"cfg": ci, "kernel": kname, "batch": batch, "ms": round(ms / n, 3)}
        if k == rm.RM_KERNEL_WAVEQUEUE:
            with rm.Renderer(W, H, kernel=k, counters=True) as r:
                r.dispatch(rm.sweep_uniforms(5, 120, b, aa, sm))
                c = r.counters(); it = r.wave_iterations()
            line.update(util=round(c["sdf_evals"] / (64.0 * it), 3))
        print(json.dumps(line), flush=True)
