"""Profiling aid (GPU box): the stage-1 launch of one DDplan stage (all its passes from one
raw read) with the rfifind-style mask, repeated; for rocprofv3 --pmc passes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pipeline2.0_amd")]
from hipdedisp import Engine, Opts, PassParams, plan as P  # noqa: E402
from hipdedisp.synth import palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask  # noqa: E402

obs = palfa_obs(N=1 << 22, nbits=8)
st = int(sys.argv[1]) if len(sys.argv) > 1 else 0
synth = palfa_synth()
with Engine(0) as eng:
    eng.set_obs(obs, Opts())
    eng.synth_device(synth)
    pts = rfifind_ptsperint(obs.dt)
    m, pad = synth_mask(obs, synth, pts)
    eng.set_mask(m, pts, pad)
    d = P.ddplans_for("pdev")[st]
    plans = [eng.plan(PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                                 numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                                 numout=P.choose_N(obs.N / d.downsamp))) for i in range(d.numpasses)]
    t = []
    for _ in range(3):
        eng.run_subband_multi(plans)
        eng.sync()
        t.append(plans[0].last_ms()[0])
    print("stage %d stage-1 (%d passes): %.3f ms" % (st, len(plans), min(t)), flush=True)
