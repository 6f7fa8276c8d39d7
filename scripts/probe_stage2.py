"""Profiling aid (GPU box): one full-resolution stage-2 pass (DDplan stage 0, pass 0) of the
default kernel with the probe bits of hd_plan_set_variant (bits 16-23): 1 skip sums,
2 skip fill, 4 skip stores, 8 skip expand.  Results are invalid under a probe."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pipeline2.0_amd")]
from hipdedisp import Engine, Opts, PassParams, plan as P  # noqa: E402
from hipdedisp.synth import palfa_obs, palfa_synth  # noqa: E402

obs = palfa_obs(N=1 << 22, nbits=8)
args = [x for x in sys.argv[1:] if not x.startswith("--probes=")]
variant = int(next((a[10:] for a in sys.argv[1:] if a.startswith("--variant=")), "0"))
args = [x for x in args if not x.startswith("--variant=")]
stages = [int(x) for x in (args or ["0"])]
probes = [int(x) for x in next((a[9:] for a in sys.argv[1:] if a.startswith("--probes=")), "0,1,4,5,8,9,13,15").split(",")]
with Engine(0) as eng:
    eng.set_obs(obs, Opts())
    eng.synth_device(palfa_synth())
    for st in stages:
        d = P.ddplans_for("pdev")[st]
        p = eng.plan(PassParams(subdm=float(d.subdmlist[0]), lodm=float(d.lodm_arg(0)), dmstep=float(d.dmstep_arg()),
                                numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                                numout=P.choose_N(obs.N / d.downsamp)))
        p.run_subband()
        for probe in probes:
            p.set_variant((probe << 16) | variant)
            t = []
            for _ in range(5):
                p.run_dedisp(to_host=False)
                eng.sync()
                t.append(p.last_ms()[1])
            print("stage %d stage-2 variant %d probe %2d: %.3f ms" % (st, variant, probe, min(t)), flush=True)
        p.destroy()
