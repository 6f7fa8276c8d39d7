"""Timing aid (GPU box): hd_rfifind_stats over the C2-size synthetic beam (2^22 spectra x 960
channels, 8-bit and 4-bit) at the reference's rfifind interval (2^15 * 64 us in whole rows),
plus the host mask decisions; prints ms."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pipeline2.0_amd")]
from hipdedisp import Engine, Opts  # noqa: E402
from hipdedisp import rfifind as RF  # noqa: E402
from hipdedisp.synth import palfa_obs, palfa_synth, rfifind_ptsperint  # noqa: E402

with Engine(0) as eng:
    for nbits in (8, 4):
        obs = palfa_obs(N=1 << 22, nbits=nbits)
        eng.set_obs(obs, Opts())
        eng.synth_device(palfa_synth(nbits=nbits))
        eng.set_mask()
        pts = rfifind_ptsperint(obs.dt)
        RF.device_stats(eng, pts)
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            avg, std, pw = RF.device_stats(eng, pts)
            ts.append(time.perf_counter() - t)
        t = time.perf_counter()
        bm, zi, zc, _ = RF.make_mask(avg, std, pw, pts)
        tm = time.perf_counter() - t
        print("%d-bit: %d intervals of %d: hd_rfifind_stats %.2f ms (wall, incl. clip stats cached), "
              "make_mask %.2f ms; %d bad cells, %d zapped chans, %d zapped ints"
              % (nbits, avg.shape[0], pts, 1e3 * min(ts), 1e3 * tm, int(bm.sum()), len(zc), int(zi.sum())), flush=True)
