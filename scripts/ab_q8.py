"""A/B aid (GPU box): stage-1 time per DDplan stage of the C2 beam with k_stage1_q8's spare
waves summing a share of the passes (default) vs one wave per subband (probe 16); checks the
subbands are identical."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pipeline2.0_amd")]
from hipdedisp import Engine, Opts, PassParams, plan as P  # noqa: E402
from hipdedisp.synth import palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask  # noqa: E402

obs = palfa_obs(N=1 << 22, nbits=int(sys.argv[1]) if len(sys.argv) > 1 else 8)
synth = palfa_synth(nbits=obs.nbits)
tot = {0: 0.0, 16: 0.0}
with Engine(0) as eng:
    eng.set_obs(obs, Opts())
    eng.synth_device(synth)
    pts = rfifind_ptsperint(obs.dt)
    m, pad = synth_mask(obs, synth, pts)
    eng.set_mask(m, pts, pad)
    for st, d in enumerate(P.ddplans_for("pdev")):
        plans = [eng.plan(PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)),
                                     dmstep=float(d.dmstep_arg()), numdms=d.dmsperpass, nsub=d.numsub,
                                     ds=d.sub_downsamp, numout=P.choose_N(obs.N / d.downsamp)))
                 for i in range(d.numpasses)]
        res, subs = {}, {}
        for probe in (16, 0, 16, 0):
            for p in plans:
                p.set_variant(probe << 16)
            t = []
            for _ in range(3):
                eng.run_subband_multi(plans)
                eng.sync()
                t.append(plans[0].last_ms()[0])
            res[probe] = min(t)
            subs[probe] = [plans[0].get_subbands(), plans[-1].get_subbands()]
        same = all(np.array_equal(a, b) for a, b in zip(subs[0], subs[16]))
        tot[0] += res[0]
        tot[16] += res[16]
        print("stage %d (%d passes, ds %d): stage 1 %.3f ms split vs %.3f ms one-wave; identical %s"
              % (st, d.numpasses, d.sub_downsamp, res[0], res[16], same), flush=True)
        for p in plans:
            p.destroy()
print("beam stage 1: %.2f ms split vs %.2f ms one-wave" % (tot[0], tot[16]), flush=True)
