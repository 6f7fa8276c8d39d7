"""Timing aid (GPU box): realfft + zapbirds + rednoise (hd_fft.hip) on one full-size pass per
DDplan stage of the C2 beam (2^22 spectra), after its stage 1 + stage 2; ms per pass."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pipeline2.0_amd")]
from hipdedisp import Engine, Opts, PassParams, plan as P  # noqa: E402
from hipdedisp import fft_stage as FS  # noqa: E402
from hipdedisp.synth import palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask  # noqa: E402

obs = palfa_obs(N=1 << 22, nbits=8)
synth = palfa_synth()
birds = [(60.0 * k, 0.5, False) for k in range(1, 40)] + [(0.0762 * k, 0.003, False) for k in range(1, 200)]
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
        T = p.numout * p.sub_dt
        lo, hi = FS.birdie_bins(birds, T)
        res = {}
        for name, fn in (("realfft", lambda: FS.realfft(p)), ("zapbirds", lambda: FS.zapbirds(p, lo, hi)),
                         ("rednoise", lambda: FS.rednoise(p, T))):
            ts = []
            for _ in range(3):
                FS.realfft(p) if name != "realfft" else None
                eng.sync()
                t = time.perf_counter()
                fn()
                eng.sync()
                ts.append(time.perf_counter() - t)
            res[name] = 1e3 * min(ts)
        gb = d.dmsperpass * p.numout * 4 / 1e9
        print("stage %d pass %d (%d DMs x %d): realfft %.2f ms, zapbirds %.2f ms (%d ranges), rednoise %.2f ms; "
              "series %.2f GB" % (st, i, d.dmsperpass, p.numout, res["realfft"], res["zapbirds"],
                                   len(FS.zap_ranges(lo, hi, p.numout // 2)), res["rednoise"], gb), flush=True)
        p.destroy()
