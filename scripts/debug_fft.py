"""Debugging aid (GPU box): tests/test_gpu_fft.py's ds-3 case step by step, printing where it
departs from the oracle, then the engine's close."""
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "pipeline2.0_amd"), ROOT]
import oracle as OR  # noqa: E402
from hipdedisp import Engine, Opts, PassParams, plan as P  # noqa: E402
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask  # noqa: E402

eng = Engine(0)
try:
    obs = palfa_obs(N=1 << 18, nbits=8)
    s = palfa_synth()
    eng.set_obs(obs, Opts())
    eng.synth_device(s)
    pts = rfifind_ptsperint(obs.dt)
    mask, pad = synth_mask(obs, s, pts)
    eng.set_mask(mask, pts, pad)
    raw = host_spectra(obs, s)
    for ds, numdms in ((1, 12), (3, 76)):
        pp = PassParams(subdm=71.0, lodm=65.0, dmstep=0.5, numdms=numdms, nsub=96, ds=ds, numout=P.choose_N(obs.N / ds))
        p = eng.plan(pp)
        p.run_subband()
        x = p.run_dedisp()
        print("ds %d: stage-2 kernel %s" % (ds, p.kernel()), flush=True)
        want_sub, want = OR.run_pass(obs, Opts(), raw, pp, mask=mask, ptsperint=pts, padvals=pad, omp=True)
        got_sub = p.get_subbands()
        print("  subbands differ: %d" % int((got_sub != want_sub).sum()), flush=True)
        n = obs.N // ds
        d = np.argwhere(x[:, :n] != want[:, :n])
        print("  series differ before N/ds: %d %s" % (len(d), d[:5].tolist()), flush=True)
        p.destroy()
    eng.set_mask()
except Exception:
    traceback.print_exc()
    sys.stdout.flush()
print("closing", flush=True)
eng.close()
print("closed", flush=True)
