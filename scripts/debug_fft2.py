"""Debugging aid (GPU box): tests/test_gpu_fft.py's cases called directly (its fixtures by
hand), printing any failure before the engine closes."""
import os
import sys
import tempfile
import traceback
from pathlib import Path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "pipeline2.0_amd"), ROOT, os.path.join(ROOT, "tests")]
import test_gpu_fft as T  # noqa: E402
from hipdedisp import Engine, Opts  # noqa: E402
from hipdedisp.synth import palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask  # noqa: E402

eng = Engine(0)
obs = palfa_obs(N=1 << 18, nbits=8)
s = palfa_synth()
eng.set_obs(obs, Opts())
eng.synth_device(s)
pts = rfifind_ptsperint(obs.dt)
mask, pad = synth_mask(obs, s, pts)
eng.set_mask(mask, pts, pad)
for ds, numdms in ((1, 12), (3, 76)):
    try:
        T.test_fft_zap_rednoise_match_oracle(eng, obs, ds, numdms, Path(tempfile.mkdtemp()))
        print("ds %d numdms %d: ok" % (ds, numdms), flush=True)
    except Exception:
        print("ds %d numdms %d: FAILED" % (ds, numdms), flush=True)
        traceback.print_exc()
        sys.stdout.flush()
print("closing", flush=True)
eng.close()
print("closed", flush=True)
