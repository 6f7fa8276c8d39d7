"""Debugging aid (GPU box): the fused ds >= 2 stage-1 launch on the C2 beam against the
oracle for one pass; prints where the int16 subbands differ (subband, sample, quarter
position) and the subband's channel-delay parities.  python scripts/debug_q8m.py [stage] [pass]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "pipeline2.0_amd"), ROOT]
import oracle as OR  # noqa: E402
from hipdedisp import Engine, Opts, PassParams, plan as P  # noqa: E402
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask  # noqa: E402

st_sel = int(sys.argv[1]) if len(sys.argv) > 1 else 1
ps_sel = int(sys.argv[2]) if len(sys.argv) > 2 else 0
N = 1 << 22
obs = palfa_obs(N=N, nbits=8)
s = palfa_synth()
with Engine(0) as eng:
    eng.set_obs(obs, Opts())
    eng.synth_device(s)
    raw = host_spectra(obs, s)
    pts = rfifind_ptsperint(obs.dt)
    mask, pad = synth_mask(obs, s, pts)
    eng.set_mask(mask, pts, pad)
    cl = OR.prepare(obs, Opts(), raw, mask=mask, ptsperint=pts, padvals=pad, omp=True)
    dd = P.ddplans_for("pdev")
    stages = [[PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                          numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp, numout=P.choose_N(N / d.downsamp))
               for i in range(d.numpasses)] for d in dd]
    plans = [[eng.plan(pp) for pp in st] for st in stages]
    eng.touch_raw()
    eng.run_subband_multi([p for st in plans[1:] for p in st])
    eng.sync()
    pp = stages[st_sel][ps_sel]
    p = plans[st_sel][ps_sel]
    got = p.get_subbands()
    want, _ = OR.run_pass(obs, Opts(), raw, pp, clean=cl, omp=True)
    bad = np.argwhere(got != want)
    print("stage %d pass %d ds %d: %d of %d subband samples differ" % (st_sel, ps_sel, pp.ds, len(bad), got.size))
    if len(bad):
        S, JQ = 960, 960 // pp.ds
        subs = np.unique(bad[:, 0])
        print("subbands:", subs[:20].tolist(), "...", len(subs))
        for sb, t in bad[:12].tolist():
            tile, r = divmod(t, 4 * JQ)
            q, j = divmod(r, JQ)
            print("  sub %d t %d tile %d quarter %d pos %d (lane %d m %d): got %d want %d"
                  % (sb, t, tile, q, j, j % 64, j // 64, got[sb, t], want[sb, t]))
        idd = p.delays() if hasattr(p, "delays") else None
        if idd is not None:
            print("delays of subband %d:" % subs[0], idd[subs[0] * 10:(subs[0] + 1) * 10])
    for st in plans:
        for q in st:
            q.destroy()
