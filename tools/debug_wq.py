import sys, os, numpy as np
sys.path.insert(0, 'opengl-raymarching-in-compute-shader_amd'); sys.path.insert(0, 'oracle')
import rmarch as rm, oracle as O
W, H = 96, 64
for case in [(30, 2, True, 0), (30, 2, False, 0), (60, 3, False, 0)]:
    u = rm.sweep_uniforms(case[0], 120, case[1], case[2], case[3])
    ref = O.render(u, W, H)
    out = {}
    for k in (rm.RM_KERNEL_PIXEL, rm.RM_KERNEL_WAVEQUEUE):
        with rm.Renderer(W, H, outputs=3, kernel=k, counters=True) as r:
            r.dispatch(u); out[k] = (r.counters(), r.sdf_counts(), r.read_rgba32f())
    print(case, 'ref', ref['counters'])
    for k in out:
        c, s, f = out[k]
        bad = np.argwhere(s != ref['sdf_counts'])
        print(' kernel', k, c, 'badpx', len(bad), bad[:5].tolist(), 'maxdf', np.abs(f - ref['rgba32f']).max())
        for (y, x) in bad[:3]:
            print('   px', x, y, 'ref', ref['sdf_counts'][y, x], 'got', s[y, x], ref['rgba32f'][y, x], f[y, x])
