"""Timing aid (GPU box): single-pulse search (hd_single_pulse) over one full-size pass per
DDplan stage of the C2 beam, after its stage 1 + stage 2; prints ms per pass (wall, incl.
the host pruning) and candidates."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pipeline2.0_amd")]
from hipdedisp import Engine, Opts, PassParams, plan as P  # noqa: E402
from hipdedisp import single_pulse as SP  # noqa: E402
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
        p.run_dedisp(to_host=False)
        eng.sync()
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            hits, bad = SP.device_candidates(p, p.sub_dt, 0.1, 5.0)
            ts.append(time.perf_counter() - t)
        print("stage %d pass %d (ds %d, %d DMs x %d): hd_single_pulse %.2f ms (wall), %d candidates"
              % (st, i, d.sub_downsamp, d.dmsperpass, p.numout, 1e3 * min(ts), len(hits)), flush=True)
        p.destroy()
