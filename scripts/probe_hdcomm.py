"""Profiling aid (GPU box): one C2 time slice at world 1 with its exchanges over the library's
RCCL communicator vs plain host tables -- wall ms of each phase (stats, all-reduce, set,
stage 1 of the first DDplan stage) per beam, to find where the hd-comm path spends time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pipeline2.0_amd")]
import numpy as np  # noqa: E402
from hipdedisp import Engine, Opts, PassParams, plan as P  # noqa: E402
from hipdedisp import sharding as S  # noqa: E402
from hipdedisp.synth import palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask  # noqa: E402

obs = palfa_obs(N=1 << 22, nbits=8)
synth = palfa_synth()
ddplans = P.ddplans_for("pdev")
ts = S.TimeSlices(obs, ddplans, 1)
with Engine(0) as eng:
    eng.set_obs(ts.local_obs(0), Opts())
    eng.set_slice(ts.slice(0)[0], obs.N)
    eng.synth_device(synth)
    pts = rfifind_ptsperint(obs.dt)
    m, pad = synth_mask(obs, synth, pts)
    eng.set_mask(m, pts, pad)
    d = ddplans[0]
    plans = [eng.plan(PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                                 numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                                 numout=ts.numout_local(0, P.choose_N(obs.N / d.downsamp), d.sub_downsamp)))
             for i in range(4)]

    def stage1():
        t = time.perf_counter()
        eng.run_subband_multi(plans)
        eng.sync()
        return 1e3 * (time.perf_counter() - t)

    for it in range(2):                                  # host tables
        eng.touch_raw()
        t = time.perf_counter()
        tab = ts.stats_table()
        ts.contribute_clip_stats(eng, 0, tab)
        t1 = time.perf_counter()
        eng.clip_set_stats(tab)
        t2 = time.perf_counter()
        print("host  : stats %.2f ms, set %.2f ms, stage 1 (4 passes) %.2f ms" % (1e3 * (t1 - t), 1e3 * (t2 - t1), stage1()),
              flush=True)
    eng.comm_init(Engine.comm_unique_id(), 0, 1)
    for it in range(3):
        eng.touch_raw()
        t = time.perf_counter()
        eng.slice_exchange_clip(ts.nown_blocks(0), ts.nblk_total)
        t1 = time.perf_counter()
        x = np.arange(57, dtype=np.float64)
        eng.comm_allreduce(x)
        t2 = time.perf_counter()
        print("hdcomm: exchange %.2f ms, allreduce(57) %.2f ms, stage 1 (4 passes) %.2f ms" % (
            1e3 * (t1 - t), 1e3 * (t2 - t1), stage1()), flush=True)
    eng.comm_destroy()
    for it in range(2):
        eng.touch_raw()
        tab = ts.stats_table()
        ts.contribute_clip_stats(eng, 0, tab)
        eng.clip_set_stats(tab)
        print("host after destroy: stage 1 (4 passes) %.2f ms" % stage1(), flush=True)
    for p in plans:
        p.destroy()
