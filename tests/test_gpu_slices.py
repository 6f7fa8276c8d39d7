"""Multi-GPU time slices (hipdedisp.sharding.TimeSlices) on one GPU: the ranks of a world-3
node run one after another on their own contexts, their two exchanges (clip statistics,
padding sums) summed in numpy where the node all-reduces over RCCL.  The union of the
ranks' owned series must equal a whole-beam run bit for bit -- clipping, mask and padding
included -- and so must the per-block cleaning state."""
import copy

import numpy as np
import pytest

from hipdedisp import Engine, Opts, PassParams, plan as P
from hipdedisp import sharding as S
from hipdedisp.synth import palfa_obs, palfa_synth, synth_mask

pytestmark = pytest.mark.gpu


def spiky():
    s = palfa_synth()
    s.spike_frac, s.spike_amp = 0.002, 40.0
    return s


def small_plan():
    out = []
    for st, n in ((0, 2), (3, 1), (5, 1)):
        d = copy.copy(P.ddplans_for("pdev")[st])
        d.numpasses = n
        out.append(d)
    return out


def pass_params(obs, d, i, numout=None):
    return PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                      numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                      numout=P.choose_N(obs.N / d.downsamp) if numout is None else numout)


@pytest.mark.parametrize("world", [2, 3])
def test_time_slices_union_equals_whole_beam(engine, world):
    obs = palfa_obs(N=(1 << 18) + 4 * 30720 + 777, nbits=8, nsblk=2048)
    synth = spiky()
    pts = 16384
    mask, pad = synth_mask(obs, synth, pts, frac=0.03)
    ddplans = small_plan()
    # the whole beam on the test engine
    engine.set_obs(obs, Opts())
    engine.synth_device(synth)
    engine.set_mask(mask, pts, pad)
    want = {}
    gpad, gclip, _, _ = engine.get_clean()
    for d in ddplans:
        plans = [engine.plan(pass_params(obs, d, i)) for i in range(d.numpasses)]
        engine.run_subband_multi(plans)
        for i, p in enumerate(plans):
            want[(d.sub_downsamp, i)] = p.run_dedisp()
            p.destroy()
    engine.set_mask()

    ts = S.TimeSlices(obs, ddplans, world)
    assert ts.cuts[0] == 0 and ts.cuts[-1] == obs.N and all(c % ts.unit == 0 for c in ts.cuts[1:-1])
    engs, plans = [], []
    try:
        table = ts.stats_table()
        for r in range(world):                          # phase A on every rank
            e = Engine(0)
            engs.append(e)
            t0, own, nloc = ts.slice(r)
            e.set_obs(ts.local_obs(r), Opts())
            e.set_slice(t0, obs.N)
            e.synth_device(synth)
            e.set_mask(mask, pts, pad)
            mine = ts.stats_table()
            ts.contribute_clip_stats(e, r, mine)
            table += mine                               # the all-reduce
        for r, e in enumerate(engs):                    # phase B: clip state, then every pass
            e.clip_set_stats(table)
            t0, own, nloc = ts.slice(r)
            lpad, lclip, _, _ = e.get_clean()
            assert np.array_equal(lclip[:own], gclip[t0:t0 + own]), r
            nb = ts.nown_blocks(r)
            assert np.array_equal(lpad[:nb], gpad[t0 // ts.blk:t0 // ts.blk + nb]), r
            mine = []
            for d in ddplans:
                ps = [e.plan(pass_params(ts.local_obs(r), d, i,
                                         ts.numout_local(r, P.choose_N(obs.N / d.downsamp), d.sub_downsamp)))
                      for i in range(d.numpasses)]
                e.run_subband_multi(ps)
                for p in ps:
                    p.run_dedisp(to_host=False)
                mine += ps
            plans.append(mine)
        for r in range(world):                                             # the batched sums (one wait)
            one = [p.series_sum(0, 0, ts.out_range(r, p.pp.ds)[1]) for p in plans[r]]
            assert list(ts.pass_sums(r, plans[r])) == one
            mid = [p.numout // 3 for p in plans[r]]
            assert list(plans[r][0].eng.series_sums(plans[r], 1, mid, mid)) == \
                [p.series_sum(1, m, m) for p, m in zip(plans[r], mid)]
        sums = sum(ts.pass_sums(r, plans[r]) for r in range(world))      # phase C + all-reduce
        for r in range(world):
            ts.pad_passes(r, plans[r], sums)                               # phase D
        for r in range(world):
            k = 0
            for d in ddplans:
                for i in range(d.numpasses):
                    p = plans[r][k]
                    k += 1
                    j0, nj = ts.out_range(r, d.sub_downsamp)
                    full = want[(d.sub_downsamp, i)]
                    n = p.numout if r == world - 1 else nj
                    got = p.get_series(0, None, 0, n)
                    assert np.array_equal(got, full[:, j0:j0 + n]), (r, d.sub_downsamp, i)
    finally:
        for lst in plans:
            for p in lst:
                p.destroy()
        for e in engs:
            e.close()


def _hip():
    """The HIP runtime libhipdedisp.so is linked against (already loaded: same handle)."""
    import ctypes
    h = ctypes.CDLL("libamdhip64.so.7")
    h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    h.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    h.hipFree.argtypes = [ctypes.c_void_p]
    return h


def test_clip_stats_device_pointer_path(engine):
    """hd_clip_stats / hd_clip_set_stats with a DEVICE table (the RCCL path of bench.py
    --mode slices, where the all-reduce runs in HBM): every rank's rows and the finished clip
    state bit-identical to the host-table path of the same ranks."""
    import ctypes
    world = 2
    obs = palfa_obs(N=(1 << 18) + 2 * 30720 + 99, nbits=8, nsblk=2048)
    synth = spiky()
    pts = 16384
    mask, pad = synth_mask(obs, synth, pts, frac=0.03)
    ts = S.TimeSlices(obs, small_plan(), world)
    hip = _hip()
    nbytes = ts.stats_table().nbytes
    dtab = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(dtab), nbytes) == 0
    engs = []
    try:
        host_sum = ts.stats_table()
        dev_sum = ts.stats_table()
        for r in range(world):
            e = Engine(0)
            engs.append(e)
            t0, own, nloc = ts.slice(r)
            e.set_obs(ts.local_obs(r), Opts())
            e.set_slice(t0, obs.N)
            e.synth_device(synth)
            e.set_mask(mask, pts, pad)
            mine = ts.stats_table()
            ts.contribute_clip_stats(e, r, mine)                     # host table
            assert hip.hipMemset(dtab, 0, nbytes) == 0
            ts.contribute_clip_stats(e, r, int(dtab.value))          # device table
            back = ts.stats_table()
            assert hip.hipMemcpy(back.ctypes.data, dtab, nbytes, 2) == 0      # hipMemcpyDeviceToHost
            assert np.array_equal(back.view(np.uint64), mine.view(np.uint64)), r
            host_sum += mine
            dev_sum += back
        assert hip.hipMemcpy(dtab, dev_sum.ctypes.data, nbytes, 1) == 0      # hipMemcpyHostToDevice
        for r, e in enumerate(engs):
            e.clip_set_stats(int(dtab.value))
            dpad, dclip, dzap, dn = e.get_clean()
            e.clip_set_stats(host_sum)
            hpad, hclip, hzap, hn = e.get_clean()
            assert dn == hn and np.array_equal(dclip, hclip) and np.array_equal(dzap, hzap)
            assert np.array_equal(dpad.view(np.uint32), hpad.view(np.uint32)), r
    finally:
        for e in engs:
            e.close()
        hip.hipFree(dtab)


@pytest.mark.parametrize("N", [(1 << 17) + 777, 1 << 22])
def test_in_library_comm_world1(engine, N):
    """hd_comm_* (RCCL loaded by the library, no torch.distributed) at world size 1 -- the
    collective path a C caller of a time-sliced beam takes: the all-reduce of host and device
    doubles returns them unchanged, and hd_slice_exchange_clip on a one-slice context leaves
    the same clip_times state as the whole-beam context; misuse is refused.  At the full C2
    size the device table's copies are large enough that an unordered copy (round 4: a
    null-stream device-to-device hipMemcpy) shows as wrong clip state."""
    from hipdedisp.engine import PrestoError
    obs = palfa_obs(N=N, nbits=8, nsblk=2048)
    synth = spiky()
    engine.set_obs(obs, Opts())
    engine.synth_device(synth)
    gpad, gclip, gzap, _ = engine.get_clean()
    e = Engine(0)
    try:
        with pytest.raises(PrestoError, match="no communicator"):
            e.comm_allreduce(np.zeros(3))
        uid = Engine.comm_unique_id()
        assert len(uid) == 128
        e.comm_init(uid, 0, 1)
        with pytest.raises(PrestoError, match="already has a communicator"):
            e.comm_init(uid, 0, 1)
        x = np.arange(1000, dtype=np.float64) * 0.5
        assert np.array_equal(e.comm_allreduce(x.copy()), x)
        e.set_obs(obs, Opts())
        e.set_slice(0, obs.N)
        e.synth_device(synth)
        ts = S.TimeSlices(obs, small_plan(), 1)
        e.slice_exchange_clip(ts.nown_blocks(0), ts.nblk_total)
        lpad, lclip, lzap, _ = e.get_clean()
        assert np.array_equal(lclip, gclip) and np.array_equal(lpad, gpad) and np.array_equal(lzap, gzap)
        e.comm_destroy()
        e.comm_destroy()                                 # idempotent
    finally:
        e.close()
