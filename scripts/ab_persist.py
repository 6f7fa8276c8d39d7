"""A/B aid (GPU box): stage-2 time of one pass per DDplan stage of the C2 beam, pair kernel
with persistent workgroups (default) vs one workgroup per tile (variant bits 24-25 = 2);
checks the series are identical."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pipeline2.0_amd")]
from hipdedisp import Engine, Opts, PassParams, plan as P  # noqa: E402
from hipdedisp.synth import palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask  # noqa: E402

obs = palfa_obs(N=1 << 22, nbits=8)
synth = palfa_synth()
with Engine(0) as eng:
    eng.set_obs(obs, Opts())
    eng.synth_device(synth)
    pts = rfifind_ptsperint(obs.dt)
    m, pad = synth_mask(obs, synth, pts)
    eng.set_mask(m, pts, pad)
    for st, d in enumerate(P.ddplans_for("pdev")):
        i = d.numpasses // 2
        p = eng.plan(PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                                numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                                numout=P.choose_N(obs.N / d.downsamp)))
        p.run_subband()
        res, ser = {}, {}
        for v in (0, 2 << 24, 0, 2 << 24):
            p.set_variant(v)
            t = []
            for _ in range(5):
                p.run_dedisp(to_host=False)
                eng.sync()
                t.append(p.last_ms()[1])
            res[v] = min(t)
            ser[v] = p.get_series(0, 2)
        same = np.array_equal(ser[0], ser[2 << 24])
        ntiles = (p.nds + 767) // 768
        print("stage %d (ds %d, %d DMs, %d tiles): persistent %.3f ms, per-tile %.3f ms; identical %s"
              % (st, d.sub_downsamp, d.dmsperpass, ntiles, res[0], res[2 << 24], same), flush=True)
        p.destroy()
