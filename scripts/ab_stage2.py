"""A/B of stage-2 variants (GPU box): one pass of each requested DDplan stage, the default
kernel under hd_plan_set_variant probe bytes (bits 16-23); every output is compared bit for bit
with the probe-0 run (the probes listed here must not change results).
  python scripts/ab_stage2.py [stages...] --probes=0,32,64
Under rocprofv3 --kernel-trace, scripts/ab_trace.py splits the trace per (stage, probe)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pipeline2.0_amd")]
from hipdedisp import Engine, Opts, PassParams, plan as P  # noqa: E402
from hipdedisp.synth import palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask  # noqa: E402

obs = palfa_obs(N=1 << 22, nbits=8)
args = [x for x in sys.argv[1:] if not x.startswith("--")]
stages = [int(x) for x in (args or ["0", "3", "5"])]
probes = [int(x) for x in next((a[9:] for a in sys.argv[1:] if a.startswith("--probes=")), "0,32,64").split(",")]
reps = int(next((a[7:] for a in sys.argv[1:] if a.startswith("--reps=")), "7"))
with Engine(0) as eng:
    eng.set_obs(obs, Opts())
    synth = palfa_synth()
    eng.synth_device(synth)
    pts = rfifind_ptsperint(obs.dt)                # the bench beam's rfifind-style mask
    mask, pad = synth_mask(obs, synth, pts)
    eng.set_mask(mask, pts, pad)
    for st in stages:
        d = P.ddplans_for("pdev")[st]
        p = eng.plan(PassParams(subdm=float(d.subdmlist[0]), lodm=float(d.lodm_arg(0)), dmstep=float(d.dmstep_arg()),
                                numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                                numout=P.choose_N(obs.N / d.downsamp)))
        p.run_subband()
        ref = None
        for probe in probes:
            p.set_variant(probe << 16)
            t = []
            for _ in range(reps):
                # a queue of launches per timing: host launch gaps hide behind the kernels
                eng.sync()
                t0 = time.perf_counter()
                for _ in range(8):
                    p.run_dedisp(to_host=False)
                eng.sync()
                t.append((time.perf_counter() - t0) * 1e3 / 8)
            out = p.run_dedisp(to_host=True)
            eng.sync()
            same = "ref" if ref is None else ("identical" if np.array_equal(out, ref) else "DIFFERENT")
            if ref is None:
                ref = out.copy()
            print("stage %d probe %3d: min %.3f med %.3f ms/launch (incl. k_pad)  %s" % (st, probe, min(t), float(np.median(t)), same),
                  flush=True)
        p.destroy()
