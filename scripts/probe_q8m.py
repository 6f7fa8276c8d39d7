"""Profiling aid (GPU box): where stage 1's integer launches spend their time on the C2 beam
(mask, clipping on), as the bench calls them: the ds = 1 stage alone (k_stage1_q8) and the five
ds >= 2 stages in one call (k_stage1_q8m).  Device time of hd_run_subband_multi with the fixups
skipped (probe bits 32 | 64) and the q8 / q8m probe bits: 1 skip the sums, 2 skip the fill,
8 skip the stores, 4 (q8m) never take the float fold.  Results are invalid under a probe (timing only)."""
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
    stages = [[eng.plan(PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                                   numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                                   numout=P.choose_N(obs.N / d.downsamp))) for i in range(d.numpasses)]
              for d in P.ddplans_for("pdev")]
    eng.touch_raw()
    groups = [("ds1", stages[0]), ("ds>=2", [p for st in stages[1:] for p in st])]
    for label, sel in groups:
        for probe in ((0, 96, 96 | 1, 96 | 2, 96 | 3, 96 | 8, 96 | 9) if label == "ds1" else (0, 96, 96 | 1, 96 | 2, 96 | 3, 96 | 4, 96 | 8, 96 | 9)):
            sel[0].set_variant(probe << 16)
            t = []
            for _ in range(3):
                eng.run_subband_multi(sel)
                eng.sync()
                t.append(sel[0].last_ms()[0])
            print("%-6s probe %3d: %.3f ms" % (label, probe, min(t)), flush=True)
        sel[0].set_variant(0)
    for st in stages:
        for p in st:
            p.destroy()
