"""Probe (GPU box): per DDplan stage of the C2 beam, stage-1 time in full, with the q8 sums
skipped (probe 1: the fill and stores of the tile remain), and with the fill skipped (probe 2)."""
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
        plans = [eng.plan(PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)),
                                     dmstep=float(d.dmstep_arg()), numdms=d.dmsperpass, nsub=d.numsub,
                                     ds=d.sub_downsamp, numout=P.choose_N(obs.N / d.downsamp)))
                 for i in range(d.numpasses)]
        res = {}
        for probe in (0, 1, 2, 1 | 2, 64 | 32):
            for p in plans:
                p.set_variant(probe << 16)
            t = []
            for _ in range(3):
                eng.run_subband_multi(plans)
                eng.sync()
                t.append(plans[0].last_ms()[0])
            res[probe] = min(t)
        print("stage %d (%d passes, ds %d): full %.3f | no sums %.3f | no fill %.3f | neither %.3f | no fixups %.3f ms"
              % (st, d.numpasses, d.sub_downsamp, res[0], res[1], res[2], res[3], res[96]), flush=True)
        for p in plans:
            p.destroy()
