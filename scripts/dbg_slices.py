import sys, os
sys.path[:0] = [os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), p) for p in ("pipeline2.0_amd", "oracle", "tests")]
import numpy as np
from hipdedisp import Engine, Opts, plan as P
from hipdedisp import sharding as S
from hipdedisp.synth import palfa_obs, synth_mask
import test_gpu_slices as T
obs = palfa_obs(N=(1 << 18) + 4 * 30720 + 777, nbits=8, nsblk=2048)
synth = T.spiky(); pts = 16384
mask, pad = synth_mask(obs, synth, pts, frac=0.03)
ddplans = T.small_plan()[:1]
eng = Engine(0)
eng.set_obs(obs, Opts()); eng.synth_device(synth); eng.set_mask(mask, pts, pad)
d = ddplans[0]
plans = [eng.plan(T.pass_params(obs, d, i)) for i in range(d.numpasses)]
eng.run_subband_multi(plans)
full = plans[0].run_dedisp()
world = 3
ts = S.TimeSlices(obs, T.small_plan(), world)
table = ts.stats_table(); engs = []
for r in range(world):
    e = Engine(0); engs.append(e)
    t0, own, nloc = ts.slice(r)
    e.set_obs(ts.local_obs(r), Opts()); e.set_slice(t0, obs.N); e.synth_device(synth); e.set_mask(mask, pts, pad)
    mine = ts.stats_table(); ts.contribute_clip_stats(e, r, mine); table += mine
for r, e in enumerate(engs):
    e.clip_set_stats(table)
    ps = [e.plan(T.pass_params(ts.local_obs(r), d, i, ts.numout_local(r, P.choose_N(obs.N / d.downsamp), d.sub_downsamp))) for i in range(d.numpasses)]
    e.run_subband_multi(ps)
    j0, nj = ts.out_range(r, 1)
    for v in (0, 5, 6):
        ps[0].set_variant(v)
        ser = ps[0].run_dedisp()
        s = ps[0].series_sum(0, 0, nj)
        print("rank", r, "variant", v, "j0", j0, "nj", nj, "numout", ps[0].numout, "series_sum", s,
              "host sum", ser[0, :nj].astype(np.float64).sum(), "want", full[0, j0:j0 + nj].astype(np.float64).sum(),
              "equal", np.array_equal(ser[:, :nj], full[:, j0:j0 + nj]), flush=True)
