"""Multi-GPU partitioning (hipdedisp.sharding): LPT pass assignment, the per-rank .dat sets,
and the raw-block broadcast, on CPU with the gloo backend at world size 2 (the RCCL path is
the same torch.distributed call on GPU tensors).  The GPU leg runs each rank's share on one
device and checks that the union equals a single-rank run."""
import os
import socket

import numpy as np
import pytest

from hipdedisp import plan as P
from hipdedisp import sharding as S
from hipdedisp.synth import palfa_obs


@pytest.mark.parametrize("backend", ["pdev", "wapp"])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 7, 8])
def test_every_pass_exactly_once(backend, world):
    plans = P.ddplans_for(backend)
    asg = S.assign_passes(plans, 1 << 22, 960, world)
    assert len(asg) == world
    got = sorted((p.stage, p.passnum) for lst in asg for p in lst)
    want = sorted((s, i) for s, d in enumerate(plans) for i in range(d.numpasses))
    assert got == want
    dms = S.dm_strings_of(plans, asg)
    flat = [x for lst in dms for x in lst]
    ref = [x for d in plans for lst in d.dmlist for x in lst]
    assert sorted(flat) == sorted(ref) and len(set(flat)) == len(flat)


def test_lpt_balance_on_the_mock_plan():
    plans = P.ddplans_for("pdev")
    for world in (2, 4, 8):
        asg = S.assign_passes(plans, 1 << 22, 960, world)
        assert S.imbalance(asg) < 1.12, world
    # deterministic: every rank derives the same assignment
    a = S.assign_passes(plans, 1 << 22, 960, 8)
    b = S.assign_passes(plans, 1 << 22, 960, 8)
    assert a == b


def test_groups_follow_plan_order():
    plans = P.ddplans_for("pdev")
    asg = S.assign_passes(plans, 1 << 22, 960, 4)
    for lst in asg:
        groups = S.by_stage(lst)
        assert [g[0] for g in groups] == sorted(g[0] for g in groups)
        for stage, passnums in groups:
            assert passnums == sorted(passnums)


def test_sharded_beam_pass_params_match_reference_strings():
    plans = P.ddplans_for("pdev")
    obs = palfa_obs(N=1 << 22)
    sb = S.ShardedBeam(plans, obs, rank=1, world=4)
    for stage, passnums in sb.my_groups():
        for i in passnums:
            pp = sb.pass_params(stage, i)
            d = plans[stage]
            assert "%.2f" % pp.subdm == d.subdmlist[i]
            assert pp.numout == P.choose_N(obs.N / d.downsamp)
    assert sb.out_samples() > 0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 3 * (1 << 20) + 12345
        if rank == 0:
            g = torch.Generator().manual_seed(20261015)
            t = torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g)
        else:
            t = torch.zeros(n, dtype=torch.uint8)
        S.broadcast_raw(t, src=0, chunk_bytes=1 << 20)
        digest = torch.tensor([int(t.to(torch.int64).sum()), int(t[::977].to(torch.int64).sum())], dtype=torch.int64)
        allg = [torch.zeros_like(digest) for _ in range(world)]
        dist.all_gather(allg, digest)
        plans = P.ddplans_for("pdev")
        mine = S.assign_passes(plans, 1 << 22, 960, world)[rank]
        cnt = torch.tensor([len(mine)], dtype=torch.int64)
        dist.all_reduce(cnt)
        q.put((rank, [tuple(x.tolist()) for x in allg], int(cnt.item())))
    finally:
        dist.destroy_process_group()


def test_broadcast_raw_gloo_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, digests, total in res:
        assert digests[0] == digests[1]            # both ranks hold rank 0's bytes
        assert total == 57                         # the two shares cover the whole plan


def _hip():
    """The HIP runtime libhipdedisp.so itself uses (device buffers without torch, whose own
    bundled runtime must not be initialised second in this process)."""
    import ctypes
    from hipdedisp import _lib
    _lib.load()
    return ctypes.CDLL("libamdhip64.so.7")


@pytest.mark.gpu
def test_sharded_union_equals_single_rank(engine):
    """Each of 2 ranks' shares, run on one GPU from a device-resident raw block (the
    post-broadcast state: hd_push_raw_device), reproduces the single-rank series bit for bit."""
    import ctypes
    from hipdedisp import Opts
    from hipdedisp.synth import host_spectra, palfa_synth
    obs = palfa_obs(N=1 << 16, nbits=8)
    synth = palfa_synth()
    raw = np.ascontiguousarray(host_spectra(obs, synth))
    engine.set_obs(obs, Opts())
    hip = _hip()
    dptr = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(dptr), ctypes.c_size_t(raw.nbytes)) == 0
    try:
        assert hip.hipMemcpy(dptr, raw.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(raw.nbytes), 1) == 0
        engine.push_raw_device(dptr.value)
        back = np.zeros_like(raw)
        assert hip.hipMemset(dptr, 0, ctypes.c_size_t(raw.nbytes)) == 0
        engine.get_raw_device(dptr.value)
        assert hip.hipMemcpy(back.ctypes.data_as(ctypes.c_void_p), dptr, ctypes.c_size_t(raw.nbytes), 2) == 0
        assert np.array_equal(back, raw)
    finally:
        hip.hipFree(dptr)
    plans = P.ddplans_for("pdev")[:2]
    plans[0].numpasses, plans[1].numpasses = 3, 2
    ref = S.ShardedBeam(plans, obs, 0, 1)
    want = ref.run(engine, ref.make_plans(engine), to_host=True)
    got = {}
    for r in range(2):
        sb = S.ShardedBeam(plans, obs, r, 2)
        got.update(sb.run(engine, sb.make_plans(engine), to_host=True))
    assert sorted(got) == sorted(want)
    for k in want:
        assert np.array_equal(got[k], want[k]), k


# ---- time slices ----------------------------------------------------------------------

@pytest.mark.parametrize("world", [1, 2, 3, 4, 7, 8])
def test_time_slices_partition(world):
    """Slices cover the beam once, start on lcm(nsblk, every ds) boundaries, carry a halo of
    whole read blocks past the longest delay of any pass, and every downsampled output
    sample of every DDplan stage is owned by exactly one rank."""
    plans = P.ddplans_for("pdev")
    obs = palfa_obs(N=1 << 22)
    ts = S.TimeSlices(obs, plans, world)
    assert ts.unit == 30720 and ts.halo % obs.nsblk == 0 and ts.halo > 0
    owned = 0
    for r in range(world):
        t0, own, nloc = ts.slice(r)
        assert t0 == owned and t0 % ts.unit == 0
        assert nloc == min(obs.N, t0 + own + ts.halo) - t0
        owned += own
        assert abs(own - obs.N / world) <= ts.unit
    assert owned == obs.N
    assert sum(ts.nown_blocks(r) for r in range(world)) == ts.nblk_total
    for d in plans:
        ds = d.sub_downsamp
        cover = np.zeros(obs.N // ds, np.int32)
        for r in range(world):
            j0, nj = ts.out_range(r, ds)
            cover[j0:j0 + nj] += 1
        assert (cover == 1).all(), ds


def test_time_slices_halo_covers_every_pass():
    """The halo reaches the last raw row any owned output sample reads, for every pass."""
    from hipdedisp import Opts, PassParams
    from hipdedisp.engine import plan_tables
    plans = P.ddplans_for("pdev")
    obs = palfa_obs(N=1 << 22)
    ts = S.TimeSlices(obs, plans, 4)
    for d in plans:
        for i in (0, d.numpasses - 1):
            pp = PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                            numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp)
            idd, off, _ = plan_tables(obs, Opts(), pp)
            t0, own, nloc = ts.slice(1)
            last_out = own // d.sub_downsamp - 1
            last_row = (last_out + int(off.max())) * d.sub_downsamp + d.sub_downsamp - 1 + int(idd.max())
            assert last_row < nloc


def _slice_worker(rank, world, port, q):
    """One rank of a sliced beam on CPU: the clip statistics of its own read blocks from its
    own spectra (the oracle's clip_times rows stand in for hd_clip_stats, same layout), the
    gloo all-reduce, then clip_times finished over the summed table for its own spectra;
    the padding sums' all-reduce."""
    import torch
    import torch.distributed as dist
    import oracle as OR
    from hipdedisp import Opts
    from hipdedisp.synth import host_spectra, palfa_synth, synth_mask
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        obs, s, pts, mask, pad = _slice_beam()
        ts = S.TimeSlices(obs, P.ddplans_for("pdev"), world)
        t0, own, nloc = ts.slice(rank)
        raw = host_spectra(obs, s, t0, nloc)                # this rank's spectra only
        t = torch.zeros((ts.nblk_total, obs.nchan + 3), dtype=torch.float64)
        b0, nb = t0 // ts.blk, ts.nown_blocks(rank)
        t.numpy()[b0:b0 + nb] = OR.clip_rows(obs, Opts(), raw, b0, nb, mask=mask, ptsperint=pts)
        dist.all_reduce(t)                                   # phase A exchange
        lpad, lclip, k = OR.clip_finish(obs, Opts(), raw[:own], t.numpy(), t0, own, mask=mask, ptsperint=pts,
                                        padvals=pad)
        sums = torch.tensor([float(rank + 1), 2.0 * (rank + 1)], dtype=torch.float64)
        dist.all_reduce(sums)                                # phase C exchange
        q.put((rank, t0, own, lpad, lclip, k, sums.tolist()))
    finally:
        dist.destroy_process_group()


def _slice_beam():
    from hipdedisp.synth import palfa_synth, rfifind_ptsperint, synth_mask
    obs = palfa_obs(N=(1 << 18) + 3 * 30720 + 777, nbits=8)
    s = palfa_synth()
    s.spike_frac, s.spike_amp = 0.003, 40.0                 # zero-DM spikes for clip_times
    pts = 16384
    mask, pad = synth_mask(obs, s, pts, frac=0.03)
    return obs, s, pts, mask, pad


def test_time_slice_exchanges_gloo_world2():
    """The two all-reduces of a sliced beam on gloo at world size 2, on real clip_times
    statistics: each rank's pad values and clip flags after the exchange equal clip_times
    over the whole beam (oracle.prepare), and the padding sums add."""
    import torch.multiprocessing as mp
    import oracle as OR
    from hipdedisp import Opts
    from hipdedisp.synth import host_spectra
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slice_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    obs, s, pts, mask, pad = _slice_beam()
    whole = OR.prepare(obs, Opts(), host_spectra(obs, s), mask=mask, ptsperint=pts, padvals=pad)
    assert whole.nclipped > 100
    total = 0
    for rank, t0, own, lpad, lclip, k, sums in res:
        assert np.array_equal(lpad, whole.pad), rank          # the recurrence ran over every block
        assert np.array_equal(lclip, whole.clipped[t0:t0 + own]), rank
        total += k
        assert sums == [3.0, 6.0]
    assert total == whole.nclipped


# ---- configs[4]: the pointing schedule (beam x time partitioning) ---------------------------

def test_pointing_schedule_shapes():
    """7 beams on 8 ranks: 7 home ranks with the first f of their beam, one helper with every
    tail; the cut balances the slice cost model; every (beam, slice) has exactly one owner;
    on 7 or fewer ranks the ranks keep whole beams."""
    obs = palfa_obs(N=1 << 22)
    pt = S.Pointing(obs, P.ddplans_for("pdev"), 7, 8)
    assert 0.5 < pt.frac < 1.0 and pt.nslices() == 2
    owned = {}
    for r in range(8):
        for u in pt.units(r):
            assert u not in owned
            owned[u] = r
    assert set(owned) == {(b, s) for b in range(7) for s in range(2)}
    assert [pt.owner(b, 0) for b in range(7)] == list(range(7)) and {pt.pad_owner(b) for b in range(7)} == {7}
    t0, own, nloc = pt.ts.slice(1)
    assert t0 % pt.ts.unit == 0 and t0 + own == obs.N
    assert pt.predicted_ms() < 67.9                           # below one beam per GPU with an idle GPU
    pt7 = S.Pointing(obs, P.ddplans_for("pdev"), 7, 4)
    assert [pt7.units(r) for r in range(4)] == [[(0, 0), (4, 0)], [(1, 0), (5, 0)], [(2, 0), (6, 0)], [(3, 0)]]
    assert S.helper_fraction(7, 0, 6.0, 62.0) == 1.0


@pytest.mark.parametrize("nbeams,world", [(7, 8), (3, 8), (2, 6), (5, 7)])
def test_pointing_balances_home_and_helpers(nbeams, world):
    """with H > 1 helpers each helper still pays the fixed cost once per beam; the
    chosen cut makes the model's home and helper times equal (unless clamped), and
    predicted_ms is the slower of them."""
    obs = palfa_obs(N=1 << 22)
    a, b = S.POINTING_FIXED_MS, S.POINTING_BEAM_MS
    pt = S.Pointing(obs, P.ddplans_for("pdev"), nbeams, world)
    H = world - nbeams
    f = pt.frac
    home, helper = a + b * f, nbeams * a + nbeams * b * (1 - f) / H
    if 0.5 < f < 1.0:
        assert abs(home - helper) < 1e-9 * home
    # predicted_ms uses the slices actually cut (whole multiples of the slice unit)
    fr = [pt.ts.slice(k)[1] / obs.N for k in range(pt.nslices())]
    want = max(a + b * fr[0], max(sum(a + b * fr[sl] for _, sl in pt.units(r)) for r in range(nbeams, world)))
    assert abs(pt.predicted_ms() - want) < 1e-9 * want


class _FakePlan:
    def __init__(self, eng, idx, ds, numout):
        from hipdedisp import PassParams
        self.eng, self.idx = eng, idx
        self.pp = PassParams(subdm=1.0, lodm=0.0, dmstep=0.1, numdms=2, nsub=96, ds=ds)
        self.numout = numout
        self.filled = None

    def series_fill(self, t0, v):
        self.filled = (t0, v)


class _FakeEngine:
    """The pieces of Engine that sharding.pointing_step drives, with the oracle's clip_times
    rows standing in for hd_clip_stats / hd_clip_set_stats (same table layout)."""

    def __init__(self, obs, synth, beam, sl, ts, mask, pts, pad):
        from hipdedisp import Opts
        from hipdedisp.synth import host_spectra
        self.obs, self.beam, self.sl, self.ts = obs, beam, sl, ts
        self.opts = Opts()
        self.t0, self.own, self.nloc = ts.slice(sl)
        self.raw = host_spectra(obs, synth, self.t0, self.nloc)
        self.mask, self.pts, self.pad = mask, pts, pad
        self.result = None

    def touch_raw(self):
        pass

    def clip_stats(self, n, table):
        import oracle as OR
        b0 = self.t0 // self.ts.blk
        table[b0:b0 + n] = OR.clip_rows(self.obs, self.opts, self.raw, b0, n, mask=self.mask, ptsperint=self.pts)

    def clip_set_stats(self, table):
        import oracle as OR
        self.result = OR.clip_finish(self.obs, self.opts, self.raw[:self.own], np.array(table), self.t0, self.own,
                                     mask=self.mask, ptsperint=self.pts, padvals=self.pad)

    def run_subband_multi(self, plans):
        pass

    def run_dedisp_multi(self, plans):
        pass

    def sync(self):
        pass

    def series_sums(self, plans, dm, t0s, counts):
        # a stand-in per (beam, slice, pass) that the pad owner's sum must reassemble
        return np.array([1000.0 * self.beam + 10.0 * self.sl + p.idx for p in plans], np.float64)


def _pointing_worker(rank, world, nbeams, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        obs, _, pts, _, _ = _slice_beam()
        pt = S.Pointing(obs, P.ddplans_for("pdev"), nbeams, world, frac=0.7)
        work = []
        for b, sl in pt.units(rank):
            synth, mask, pad = _pointing_beam(obs, b, pts)
            eng = _FakeEngine(obs, synth, b, sl, pt.ts, mask, pts, pad)
            plans = [_FakePlan(eng, i, ds, obs.N // ds + 100) for i, ds in enumerate((1, 2, 2, 3))]
            work.append((b, sl, eng, plans))
        S.pointing_step(pt, rank, work, dist, torch, on_gpu=False)
        out = []
        for b, sl, eng, plans in work:
            lpad, lclip, k = eng.result
            nhb = -(-(eng.t0 + eng.nloc) // pt.ts.blk)           # blocks up to the held end
            out.append((b, sl, eng.t0, eng.own, lpad[:nhb], lclip, k, [p.filled for p in plans]))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _pointing_beam(obs, beam, pts):
    from hipdedisp.synth import palfa_synth, synth_mask
    s = palfa_synth(beam=beam)
    s.spike_frac, s.spike_amp = 0.003, 40.0
    mask, pad = synth_mask(obs, s, pts, frac=0.03)
    return s, mask, pad


def test_pointing_exchanges_gloo_world3():
    """Two beams on three gloo ranks (two home ranks, one helper taking both tails), with real
    clip_times statistics: the one-way exchanges (own-block rows to later slices, first-DM
    sums to the last slice) give every slice the pad values of every block it holds and the
    clip flags of its own spectra exactly as clip_times over its whole beam, and the helper
    pads each pass with the sum over the beam's slices."""
    import torch.multiprocessing as mp
    import oracle as OR
    from hipdedisp import Opts
    from hipdedisp.synth import host_spectra
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world, nbeams = 3, 2
    procs = [ctx.Process(target=_pointing_worker, args=(r, world, nbeams, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    obs, _, pts, _, _ = _slice_beam()
    units = {}
    for rank, out in res:
        for b, sl, t0, own, lpad, lclip, k, filled in out:
            units[(b, sl)] = (rank, t0, own, lpad, lclip, k, filled)
    assert set(units) == {(0, 0), (0, 1), (1, 0), (1, 1)}
    assert units[(0, 1)][0] == units[(1, 1)][0] == 2
    for b in range(nbeams):
        synth, mask, pad = _pointing_beam(obs, b, pts)
        whole = OR.prepare(obs, Opts(), host_spectra(obs, synth), mask=mask, ptsperint=pts, padvals=pad)
        assert whole.nclipped > 100
        total = 0
        for sl in range(2):
            rank, t0, own, lpad, lclip, k, filled = units[(b, sl)]
            # the pads of every block the slice holds (the home slice never sees the tail's rows)
            assert np.array_equal(lpad, whole.pad[:len(lpad)]), (b, sl)
            assert np.array_equal(lclip, whole.clipped[t0:t0 + own]), (b, sl)
            total += k
        assert total == whole.nclipped
        filled = units[(b, 1)][6]
        for i, ds in enumerate((1, 2, 2, 3)):
            want = (1000.0 * b + i) + (1000.0 * b + 10.0 + i)     # slice 0 + slice 1 sums
            assert filled[i] is not None
            assert filled[i][1] == float(np.float32(want / (obs.N // ds))), (b, i)
        assert all(f is None for f in units[(b, 0)][6])           # only the last slice pads
