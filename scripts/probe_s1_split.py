"""Profiling aid (GPU box): where k_stage1_q8's time goes per DDplan stage of the C2 beam
(mask, clipping on).  Device time of hd_run_subband_multi with the fixups skipped (probe
bits 5-6), for all the stage's passes and for one pass, with the q8 probe bits: 1 skip the
sums, 2 skip the fill.  Results are invalid under a probe (timing only)."""
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
    for st, d in enumerate(P.ddplans_for("pdev")):
        plans = [eng.plan(PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                                     numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                                     numout=P.choose_N(obs.N / d.downsamp))) for i in range(d.numpasses)]
        for sel, label in ((plans, "all %d" % len(plans)), (plans[:1], "one")):
            for probe in (0, 96, 96 | 1, 96 | 2, 96 | 3):
                sel[0].set_variant(probe << 16)
                t = []
                for _ in range(3):
                    eng.run_subband_multi(sel)
                    eng.sync()
                    t.append(sel[0].last_ms()[0])
                print("ds %2d %-6s probe %3d: %.3f ms" % (d.sub_downsamp, label, probe, min(t)), flush=True)
            sel[0].set_variant(0)
        for p in plans:
            p.destroy()
