"""Profiling aid (GPU box): time one full-size pass of stage 1 (28-pass stage-0 launch) and
stage 2 with the kernel probes of hd_plan_set_variant bits 16-23 (skip sums / fill / stores)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pipeline2.0_amd")]
from hipdedisp import Engine, Opts, PassParams, plan as P  # noqa: E402
from hipdedisp.synth import palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask  # noqa: E402

obs = palfa_obs(N=1 << 22, nbits=8)
synth = palfa_synth()
masked = "--mask" in sys.argv
with Engine(0) as eng:
    eng.set_obs(obs, Opts())
    eng.synth_device(synth)
    if masked:
        pts = rfifind_ptsperint(obs.dt)
        m, pad = synth_mask(obs, synth, pts)
        eng.set_mask(m, pts, pad)
    for st in (0, 1, 3, 5):
        d = P.ddplans_for("pdev")[st]
        plans = [eng.plan(PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                                     numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                                     numout=P.choose_N(obs.N / d.downsamp))) for i in range(d.numpasses)]
        for probe in (0, 1, 2, 3):
            for p in plans:
                p.set_variant(probe << 16)
            t = []
            for _ in range(3):
                eng.run_subband_multi(plans)
                eng.sync()
                t.append(plans[0].last_ms()[0])
            print("stage %d (%d passes, ds %d) stage-1 probe %d: %.3f ms" % (st, len(plans), d.sub_downsamp, probe, min(t)),
                  flush=True)
        for p in plans:
            p.set_variant(0)
        eng.run_subband_multi(plans)
        for v2, probe in ((5, 0), (5, 1), (5, 2), (5, 3), (3, 0), (4, 0), (2, 0)):
            p = plans[0]
            p.set_variant((probe << 16) | v2)
            t = []
            for _ in range(3):
                p.run_dedisp(to_host=False)
                eng.sync()
                t.append(p.last_ms()[1])
            print("stage %d stage-2 variant %d probe %d: %.3f ms" % (st, v2, probe, min(t)), flush=True)
        for p in plans:
            p.destroy()
