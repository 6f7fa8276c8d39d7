"""Profiling aid (GPU box): stage-1 launch of DDplan stage 0 (28 passes) with the fixup's
probe bits (hd_plan_set_variant bits 16-23): 32 skip block-boundary items, 64 skip
clipped-spectrum items (results invalid under a probe); prints the stage-1 device time and
the number of clipped spectra."""
import os
import sys

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
    _, _, _, ncl = eng.get_clean()
    print("clipped spectra:", ncl, flush=True)
    for st in (0, 3):
        d = P.ddplans_for("pdev")[st]
        plans = [eng.plan(PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)),
                                     dmstep=float(d.dmstep_arg()), numdms=d.dmsperpass, nsub=d.numsub,
                                     ds=d.sub_downsamp, numout=P.choose_N(obs.N / d.downsamp)))
                 for i in range(d.numpasses)]
        for probe in (0, 32, 64, 96):
            for p in plans:
                p.set_variant(probe << 16)
            t = []
            for _ in range(3):
                eng.run_subband_multi(plans)
                eng.sync()
                t.append(plans[0].last_ms()[0])
            print("stage %d stage-1 (%d passes) probe %3d: %.3f ms" % (st, len(plans), probe, min(t)), flush=True)
        for p in plans:
            p.destroy()
