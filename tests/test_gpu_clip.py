"""GPU parity of the per-block cleaning model (oracle/oracle.h): rfifind masks applied per
read block (check_mask), PRESTO clip_times on the device (hd_clip.hip), the exact fixup of
clipped spectra and of the integer path's block-boundary outputs, and the subband rounding
and downsampling switches.  Bar: bit-exact against the oracle."""
import os

import numpy as np
import pytest

import oracle as OR
from hipdedisp import Opts, PassParams, plan
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth, synth_mask

pytestmark = pytest.mark.gpu


def beam(engine, obs, opts, synth=None, device=True):
    engine.set_obs(obs, opts)
    s = synth or palfa_synth(nbits=obs.nbits)
    raw = host_spectra(obs, s)
    if device:
        engine.synth_device(s)
    else:
        engine.push_raw(raw)
    return raw, s


def spiky_synth(nbits=8, frac=0.002):
    s = palfa_synth(nbits=nbits)
    s.spike_frac = frac                  # zero-DM broadband spikes: clip_times' targets
    s.spike_amp = {4: 6.0, 8: 40.0, 16: 600.0}[nbits]
    return s


@pytest.mark.parametrize("nbits,calib,masked,nsblk", [(8, False, False, 2048), (8, False, True, 512),
                                                      (4, False, True, 1024), (16, False, False, 4096),
                                                      (16, False, True, 1024),
                                                      (8, True, True, 2048)])
def test_clean_state_matches_oracle(engine, nbits, calib, masked, nsblk):
    """Pad rows (running channel levels), clip flags and per-block zap rows of the device
    clip_times pipeline equal the oracle's sequential restatement, bit for bit."""
    obs = palfa_obs(N=40000, nbits=nbits, nsblk=nsblk)
    raw, s = beam(engine, obs, Opts(), spiky_synth(nbits))
    rng = np.random.default_rng(nbits + nsblk)
    cal = (None, None, None)
    if calib:
        cal = (rng.uniform(0.5, 2.0, obs.nchan).astype(np.float32), rng.uniform(-5, 5, obs.nchan).astype(np.float32),
               (rng.random(obs.nchan) > 0.05).astype(np.float32))
        engine.set_calib(*cal)
    mask = pad = None
    pts = 4096
    if masked:
        mask, pad = synth_mask(obs, s, pts, frac=0.05)
        mask[3] = 1                                    # one zap_int: its blocks are not clipped
        engine.set_mask(mask, pts, pad)
    try:
        gpad, gclip, gzap, ncl = engine.get_clean()
        want = OR.prepare(obs, Opts(), raw, cal, mask, pts, pad)
        assert ncl == want.nclipped > 0
        assert np.array_equal(gclip, want.clipped)
        assert np.array_equal(gzap, want.zap)
        assert np.array_equal(gpad, want.pad)
    finally:
        engine.set_calib()
        engine.set_mask()


@pytest.mark.parametrize("ds", [1, 2, 3, 5, 6, 10])
@pytest.mark.parametrize("s1,masked,N", [(3, True, 65536 + 777), (3, True, 98304 + 388), (3, False, 65536 + 777),
                                         (2, True, 65536 + 777), (1, True, 65536 + 777)])
def test_stage1_clip_bitexact(engine, ds, s1, masked, N):
    """Stage 1 with clipping over 3 passes of one launch, every kernel path: the 8-bit
    integer kernel (3) + its float special tiles + the fixup (clipped spectra and block
    boundaries with changing pad constants; N % 4 == 0 gives the integer kernel its
    channel-major raw copy and the fixup its LDS-window kernel, else the row-major fill and
    the generic fixup), the float tiled kernel (2) + fixup, and the direct kernel (1,
    clipping per cell).  Equal to the oracle."""
    obs = palfa_obs(N=N, nbits=8, nsblk=2048)
    raw, s = beam(engine, obs, Opts(), spiky_synth())
    mask = pad = None
    pts = 8192
    if masked:
        mask, pad = synth_mask(obs, s, pts, frac=0.1)
        engine.set_mask(mask, pts, pad)
    pps = [PassParams(subdm=sd, lodm=sd - 5.0, dmstep=0.5, numdms=4, nsub=96, ds=ds) for sd in (40.0, 350.0, 1020.0)]
    plans = [engine.plan(pp) for pp in pps]
    try:
        for p in plans:
            p.set_variant(s1 << 8)
        engine.run_subband_multi(plans)
        cl = OR.prepare(obs, Opts(), raw, mask=mask, ptsperint=pts, padvals=pad)
        assert cl.nclipped > 10
        for pp, p in zip(pps, plans):
            want = OR.stage1(obs, Opts(), raw, 96, ds, pp.subdm, clean=cl, omp=True)
            assert np.array_equal(p.get_subbands(), want), pp.subdm
    finally:
        for p in plans:
            p.destroy()
        engine.set_mask()


@pytest.mark.parametrize("opts", [Opts(ds_mode=0), Opts(sub_round=1), Opts(ds_mode=0, sub_round=1, clip_sigma=0.0),
                                  Opts(clip_sigma=3.0), Opts(sub_dtype=1)])
def test_switches_bitexact(engine, opts):
    """The PRESTO switches the engine exposes (hd_opts): sum/mean downsampling, PRESTO vs
    nearest rounding, clip threshold, f32 subbands -- a masked ds=3 pass, subbands and
    series against the oracle."""
    obs = palfa_obs(N=30000, nbits=8, nsblk=1024)
    raw, s = beam(engine, obs, opts, spiky_synth())
    pts = 4096
    mask, pad = synth_mask(obs, s, pts, frac=0.05)
    engine.set_mask(mask, pts, pad)
    pp = PassParams(subdm=454.6, lodm=443.2, dmstep=0.3, numdms=76, nsub=96, ds=3,
                    numout=plan.choose_N(obs.N / 3))
    p = engine.plan(pp)
    try:
        p.run_subband()
        got_sub = p.get_subbands()
        got = p.run_dedisp()
        want_sub, want = OR.run_pass(obs, opts, raw, pp, mask=mask, ptsperint=pts, padvals=pad, omp=True)
        assert np.array_equal(got_sub, want_sub)
        nds = obs.N // 3
        assert np.array_equal(got[:, :nds], want[:, :nds])
        np.testing.assert_allclose(got[:, nds:], want[:, nds:], rtol=1e-5, atol=0)
    finally:
        p.destroy()
        engine.set_mask()


def test_rfimask_file_and_stats_pads(engine, tmp_path):
    """An rfifind .mask with zap_ints and intervals not aligned to the read blocks (dtint as
    stored), and pad values from the .stats next to it (determine_padvals), through
    Engine.set_rfimask: subbands equal the oracle given the same mask and pads."""
    from hipdedisp.formats.mask import RfiMask, RfiStats, mask_padvals, read_mask, write_mask, write_stats
    obs = palfa_obs(N=50000, nbits=8, nsblk=2048)
    raw, s = beam(engine, obs, Opts(), spiky_synth())
    pts = 3000                                           # not a multiple of nsblk: unions of two lists
    numint = -(-obs.N // pts)
    rng = np.random.default_rng(3)
    bm = (rng.random((numint, obs.nchan)) < 0.05).astype(np.uint8)
    zi = np.zeros(numint, np.uint8)
    zi[5] = 1
    mfn = str(tmp_path / "beam_rfifind.mask")
    write_mask(mfn, RfiMask(4.0, 10.0, 55000.0, pts * obs.dt * 1.0000003, obs.lofreq, obs.df, obs.nchan, numint,
                            pts, bm, zi))
    avg = rng.normal(96, 3, size=(numint, obs.nchan)).astype(np.float32)
    write_stats(str(tmp_path / "beam_rfifind.stats"),
                RfiStats(obs.nchan, numint, pts, 0, 0, avg, avg, avg))
    m = read_mask(mfn)
    pad = mask_padvals(mfn, obs.nchan)
    assert np.array_equal(pad, OR.stats_padvals(avg))
    engine.set_rfimask(m, pad)
    pp = PassParams(subdm=212.0, lodm=200.0, dmstep=0.3, numdms=64, nsub=96, ds=2)
    p = engine.plan(pp)
    try:
        p.run_subband()
        want = OR.stage1(obs, Opts(), raw, 96, 2, 212.0, mask=m.bitmap, ptsperint=pts, padvals=pad,
                         dtint=m.dtint, zapint=m.zapint, omp=True)
        assert np.array_equal(p.get_subbands(), want)
    finally:
        p.destroy()
        engine.set_mask()


@pytest.mark.parametrize("stage", [0, 1, 3, 5])
def test_fixup_kernels_agree_full_stage(engine, stage):
    """All passes of a Mock DDplan stage in one launch (28 at stage 0: the LDS-window fixup's
    largest delay table), masked, with spikes: the 8-bit LDS-window fixup, the fixup inside
    k_stage1_q8 (HD_QFIX=1) and the generic per-cell fixup (probe bit 128) give identical
    subbands, and pass 0 equals the oracle."""
    obs = palfa_obs(N=1 << 17, nbits=8, nsblk=2048)
    raw, s = beam(engine, obs, Opts(), spiky_synth())
    pts = 16384
    mask, pad = synth_mask(obs, s, pts, frac=0.05)
    engine.set_mask(mask, pts, pad)
    d = plan.ddplans_for("pdev")[stage]
    pps = [PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                      numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp) for i in range(d.numpasses)]
    plans = [engine.plan(pp) for pp in pps]
    try:
        engine.run_subband_multi(plans)
        fast = [p.get_subbands() for p in plans]
        os.environ["HD_QFIX"] = "1"
        try:
            engine.run_subband_multi(plans)
        finally:
            del os.environ["HD_QFIX"]
        for i, p in enumerate(plans):
            assert np.array_equal(p.get_subbands(), fast[i]), ("in-kernel fixup", i)
        for p in plans:
            p.set_variant(128 << 16)
        engine.run_subband_multi(plans)
        for i, p in enumerate(plans):
            assert np.array_equal(p.get_subbands(), fast[i]), i
        cl = OR.prepare(obs, Opts(), raw, mask=mask, ptsperint=pts, padvals=pad)
        assert cl.nclipped > 50
        want = OR.stage1(obs, Opts(), raw, d.numsub, d.sub_downsamp, pps[0].subdm, clean=cl, omp=True)
        assert np.array_equal(fast[0], want)
    finally:
        for p in plans:
            p.destroy()
        engine.set_mask()
