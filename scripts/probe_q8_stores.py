"""Profiling aid (GPU box): k_stage1_q8 at DDplan stage 0 of the C2 beam (28 passes, ds 1),
device ms of hd_run_subband_multi with the fixups off (probe 96) and: 8 no int16 stores,
1 no sums (nor stores), 2 no fill.  Timing only (results invalid under a probe)."""
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
    d = P.ddplans_for("pdev")[0]
    plans = [eng.plan(PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                                 numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                                 numout=P.choose_N(obs.N / d.downsamp))) for i in range(d.numpasses)]
    for probe in (96, 96 | 8, 96 | 1, 96 | 2, 96 | 8 | 2):
        plans[0].set_variant(probe << 16)
        t = []
        for _ in range(3):
            eng.run_subband_multi(plans)
            eng.sync()
            t.append(plans[0].last_ms()[0])
        print("stage 0 (28 passes) probe %3d: %.3f ms" % (probe, min(t)), flush=True)
    plans[0].set_variant(0)
    for p in plans:
        p.destroy()
