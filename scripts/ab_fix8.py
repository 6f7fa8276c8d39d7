"""A/B aid (GPU box): stage-1 time per DDplan stage of the C2 beam (HD_FIX8_LDS_KB sets the
fixup kernel's LDS budget for this process) and a hash of the first and last pass's subbands."""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pipeline2.0_amd")]
from hipdedisp import Engine, Opts, PassParams, plan as P  # noqa: E402
from hipdedisp.synth import palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask  # noqa: E402

obs = palfa_obs(N=1 << 22, nbits=8)
synth = palfa_synth()
tot = 0.0
h = hashlib.sha1()
with Engine(0) as eng:
    eng.set_obs(obs, Opts())
    eng.synth_device(synth)
    pts = rfifind_ptsperint(obs.dt)
    m, pad = synth_mask(obs, synth, pts)
    eng.set_mask(m, pts, pad)
    out = []
    for st, d in enumerate(P.ddplans_for("pdev")):
        plans = [eng.plan(PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)),
                                     dmstep=float(d.dmstep_arg()), numdms=d.dmsperpass, nsub=d.numsub,
                                     ds=d.sub_downsamp, numout=P.choose_N(obs.N / d.downsamp)))
                 for i in range(d.numpasses)]
        t = []
        for _ in range(4):
            eng.run_subband_multi(plans)
            eng.sync()
            t.append(plans[0].last_ms()[0])
        h.update(plans[0].get_subbands().tobytes())
        h.update(plans[-1].get_subbands().tobytes())
        tot += min(t)
        out.append("%.3f" % min(t))
        for p in plans:
            p.destroy()
print("HD_FIX8_LDS_KB=%s: stage 1 per stage %s ms, beam %.2f ms, subbands sha1 %s"
      % (os.environ.get("HD_FIX8_LDS_KB", "40"), " ".join(out), tot, h.hexdigest()[:16]), flush=True)
