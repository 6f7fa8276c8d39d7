"""GPU debugging aid: one pass through every stage-1 / stage-2 variant against the oracle,
reporting which combination differs (run on the GPU box)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pipeline2.0_amd"), os.path.join(ROOT, "oracle")]
import oracle as OR  # noqa: E402
from hipdedisp import Engine, Opts, PassParams  # noqa: E402
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
obs = palfa_obs(N=N, nbits=8)
synth = palfa_synth()
raw = host_spectra(obs, synth)
for pp in (PassParams(subdm=3.80, lodm=0.0, dmstep=0.1, numdms=76, nsub=96, ds=1),
           PassParams(subdm=230.0, lodm=212.8, dmstep=0.3, numdms=64, nsub=96, ds=2)):
    want_sub, want = OR.run_pass(obs, Opts(), raw, pp, omp=True)
    with Engine(0) as eng:
        eng.set_obs(obs, Opts())
        eng.synth_device(synth)
        for s1 in (1, 2, 3):
            p = eng.plan(pp)
            p.set_variant(s1 << 8)
            p.run_subband()
            got = p.get_subbands()
            print("ds=%d stage1 variant %d: %s (bad %d)" % (pp.ds, s1, np.array_equal(got, want_sub),
                                                             int((got != want_sub).sum())), flush=True)
            p.destroy()
        for s2 in (1, 2, 3, 4, 5):
            p = eng.plan(pp)
            p.set_variant((1 << 8) | s2)
            p.run_subband()
            got = p.run_dedisp()
            bad = np.argwhere(got != want)
            print("ds=%d stage2 variant %d: %s (bad %d, first %s)" % (pp.ds, s2, np.array_equal(got, want), len(bad),
                                                                       bad[:3].tolist()), flush=True)
            p.destroy()
