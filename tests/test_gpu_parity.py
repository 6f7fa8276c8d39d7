"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle on the same inputs.

Bar: bit-exact.  Integer delay tables, int16 subbands and every stage-2 sum of int16
subbands are exact integers; the float stage-1 paths (calibration, fractional mask pad
values, clip levels, mean downsampling, f32 subbands) follow the oracle's operation order
with FP contraction off, so they are bit-exact too.  The only float tolerance in this file
is the north-star's 1e-5 relative bound, applied to the padding value of padded series
(prepsubband's running mean of the first DM, computed on the device as the exact mean and
cast to f32; the oracle runs the one-pass update itself), see assert_series.
"""
import numpy as np
import pytest

import oracle as OR
from hipdedisp import Opts, PassParams, PrestoError, plan
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask

pytestmark = pytest.mark.gpu

REL_TOL = 1e-5   # north_star: max relative error per sample for float32 outputs


def assert_series(got, want, nds):
    """Data samples bit-exact; the padding value within the north-star tolerance."""
    assert got.shape == want.shape
    assert np.array_equal(got[:, :nds], want[:, :nds])
    np.testing.assert_allclose(got[:, nds:], want[:, nds:], rtol=REL_TOL, atol=0)


def load_beam(eng, obs, opts=None, synth=None, device_synth=True):
    eng.set_obs(obs, opts or Opts())
    s = synth or palfa_synth(nbits=obs.nbits)
    if device_synth:
        eng.synth_device(s)
        raw = host_spectra(obs, s)
    else:
        raw = host_spectra(obs, s)
        eng.push_raw(raw)
    return raw


def test_device_synth_bytes_equal_host(engine):
    for nbits in (4, 8, 16):
        obs = palfa_obs(N=6144, nbits=nbits)
        raw = load_beam(engine, obs)
        assert np.array_equal(engine.get_raw(), raw), nbits


@pytest.mark.parametrize("nbits,flip,ds", [(8, True, 1), (8, False, 2), (4, True, 3), (16, True, 5),
                                          (8, True, 10), (4, False, 6)])
@pytest.mark.parametrize("s1", [0, 1, 2])
def test_stage1_bitexact(engine, nbits, flip, ds, s1):
    obs = palfa_obs(N=12288 + 37, nbits=nbits, flip=flip)
    raw = load_beam(engine, obs)
    pp = PassParams(subdm=612.0, lodm=600.0, dmstep=0.5, numdms=8, nsub=96, ds=ds)
    p = engine.plan(pp)
    p.set_variant(s1 << 8)
    p.run_subband()
    got = p.get_subbands()
    want = OR.stage1(obs, Opts(), raw, 96, ds, 612.0)
    assert np.array_equal(got, want)
    idd, off = p.delays()
    assert np.array_equal(idd, OR.chan_delays(obs, 96, 612.0))
    assert np.array_equal(off, OR.dm_offsets(obs, Opts(), 96, ds, 600.0, 0.5, 8))


@pytest.mark.parametrize("sub_dtype,ds_mode", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_stage1_calib_mask_bitexact(engine, sub_dtype, ds_mode):
    rng = np.random.default_rng(17 + sub_dtype + 2 * ds_mode)
    obs = palfa_obs(N=16384, nbits=8)
    opts = Opts(sub_dtype=sub_dtype, ds_mode=ds_mode)
    raw = load_beam(engine, obs, opts, device_synth=False)
    scl = rng.uniform(0.5, 2.0, obs.nchan).astype(np.float32)
    offs = rng.uniform(-20, 20, obs.nchan).astype(np.float32)
    wts = (rng.random(obs.nchan) > 0.05).astype(np.float32)
    engine.set_calib(scl, offs, wts)
    pts = 2048
    mask, pad = synth_mask(obs, palfa_synth(), pts, frac=0.05)
    engine.set_mask(mask, pts, pad)
    p = engine.plan(PassParams(subdm=350.0, lodm=340.0, dmstep=0.3, numdms=4, nsub=96, ds=3))
    p.run_subband()
    want = OR.stage1(obs, opts, raw, 96, 3, 350.0, calib=(scl, offs, wts), mask=mask, ptsperint=pts, padvals=pad)
    assert np.array_equal(p.get_subbands(), want)
    engine.set_calib()
    engine.set_mask()


@pytest.mark.parametrize("numdms,ds,numout_mode", [(76, 1, "none"), (64, 2, "none"), (76, 3, "pad"),
                                                   (5, 1, "trunc"), (100, 5, "pad"), (76, 10, "pad")])
@pytest.mark.parametrize("variant", [1, 2, 3, 4, 5, 6, 7, 8, 9])
def test_stage2_bitexact(engine, numdms, ds, numout_mode, variant):
    obs = palfa_obs(N=3 * 8192, nbits=8)
    raw = load_beam(engine, obs)
    nds = obs.N // ds
    numout = {"none": 0, "pad": plan.choose_N(obs.N / ds) if obs.N / ds >= 10000 else nds + 777,
              "trunc": nds - 1000}[numout_mode]
    lodm = 534.4 if ds > 1 else 12.3
    pp = PassParams(subdm=lodm + 19.0, lodm=lodm, dmstep=0.5, numdms=numdms, nsub=96, ds=ds, numout=numout)
    p = engine.plan(pp)
    try:
        p.set_variant(variant)
    except PrestoError:
        if variant in (6, 7, 8, 9):   # wide DM steps: > kPairUMax patterns per pair or LDS (the DDplan passes apply, below)
            pytest.skip("pair variant not applicable to this plan")
        raise
    p.run_subband()
    try:
        got = p.run_dedisp()
    except PrestoError:
        if variant in (6, 7, 8, 9) and ds == 10:
            pytest.skip("pair variant not applicable (subband bound)")
        raise
    sub, want = OR.run_pass(obs, Opts(), raw, pp)
    assert_series(got, want, nds)


@pytest.mark.parametrize("stage,passnum", [(0, 0), (0, 27), (1, 5), (2, 0), (3, 8), (4, 2)])
def test_stage2_pair_ddplan_passes(engine, stage, passnum):
    """The pair-partial kernel (variant 6, the default for 8-bit data) on real Mock DDplan
    passes, rfifind-style mask, bit-exact against the oracle; the default choice must be
    the same kernel (same result) and the ring (variant 5) must agree too."""
    obs = palfa_obs(N=3 * 8192, nbits=8)
    synth = palfa_synth()
    raw = load_beam(engine, obs, synth=synth)
    pts = 2048
    mask, pad = synth_mask(obs, synth, pts)
    engine.set_mask(mask, pts, pad)
    d = plan.ddplans_for("pdev")[stage]
    pp = PassParams(subdm=float(d.subdmlist[passnum]), lodm=float(d.lodm_arg(passnum)), dmstep=float(d.dmstep_arg()),
                    numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp, numout=plan.choose_N(obs.N / d.downsamp))
    p = engine.plan(pp)
    p.run_subband()
    outs = []
    vs = [6, 0, 5, 7, 8, 9]
    for v in list(vs):
        try:
            p.set_variant(v)
        except PrestoError:                                    # variants 7, 8, 9: when their tables fit
            assert v in (7, 8, 9)
            vs.remove(v)
            continue
        outs.append(p.run_dedisp())
        if v == 9:
            assert p.kernel().startswith("k_stage2_qp<")
    assert 8 in vs and 9 in vs                                 # the rw and quarter kernels take every Mock pass
    _, want = OR.run_pass(obs, Opts(), raw, pp, mask=mask, ptsperint=pts, padvals=pad)
    for v, got in zip(vs, outs):
        assert_series(got, want, obs.N // pp.ds)
        assert np.array_equal(got, outs[0]), v
    engine.set_mask()


@pytest.mark.parametrize("stage", [0, 1])
def test_stage2_pair_persistent_bitexact(engine, stage):
    """Pair kernel with persistent workgroups (variant bits 24-25 = 1: one workgroup per CU,
    each over a contiguous range of tiles whose chunks stream through one DMA ring): more
    tiles than CUs and a ragged last tile, masked; bit-exact against the oracle and equal
    to one workgroup per tile (bits = 2)."""
    obs = palfa_obs(N=(1 << 19) + 777, nbits=8)
    synth = palfa_synth()
    raw = load_beam(engine, obs, synth=synth)
    pts = 2048
    mask, pad = synth_mask(obs, synth, pts)
    engine.set_mask(mask, pts, pad)
    d = plan.ddplans_for("pdev")[stage]
    pp = PassParams(subdm=float(d.subdmlist[1]), lodm=float(d.lodm_arg(1)), dmstep=float(d.dmstep_arg()),
                    numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp, numout=plan.choose_N(obs.N / d.downsamp))
    p = engine.plan(pp)
    p.run_subband()
    outs = []
    for v in (6 | (1 << 24), 6 | (2 << 24), 7 | (1 << 24), 7 | (2 << 24), 8 | (1 << 24), 8 | (2 << 24),
              9 | (1 << 24), 9 | (2 << 24)):
        try:
            p.set_variant(v)
        except PrestoError:                                    # variants 7, 8, 9: when their tables fit
            assert v & 0xFF in (7, 8, 9)
            continue
        outs.append(p.run_dedisp())
    p.destroy()
    engine.set_mask()
    _, want = OR.run_pass(obs, Opts(), raw, pp, mask=mask, ptsperint=pts, padvals=pad, omp=True)
    assert_series(outs[0], want, obs.N // pp.ds)
    for o in outs[1:]:
        assert np.array_equal(o, outs[0])


@pytest.mark.parametrize("variant", [8, 9])
@pytest.mark.parametrize("numdms,lodm,dmstep", [(76, 30.0, 0.1), (64, 240.0, 0.3), (17, 500.0, 0.5), (1, 12.0, 0.1)])
def test_stage2_rw_signed_uploaded_subbands(engine, numdms, lodm, dmstep, variant):
    """The register-window kernel (variant 8) and the quarter-layout pair kernel (variant 9)
    on uploaded int16 subbands of both signs (hd_set_subbands; |sub| <= 8000, so pairs stay
    within int16): their one-copy partials are read as sign-extended words -- bit-exact
    against the oracle's stage 2, for y-blocks of Q = 5, 4, 3 and 1 DMs per wave (the
    quarter kernel: 5 or 4), with a ragged last tile."""
    obs = palfa_obs(N=3 * 8192 + 555, nbits=8)
    engine.set_obs(obs, Opts())
    pp = PassParams(subdm=lodm + 3.0, lodm=lodm, dmstep=dmstep, numdms=numdms, nsub=96, ds=1, numout=0)
    p = engine.plan(pp)
    try:
        rng = np.random.default_rng(numdms)
        sub = rng.integers(-8000, 8001, size=(96, p.nds), dtype=np.int16)
        p.set_subbands(sub)
        p.set_variant(variant)
        got = p.run_dedisp()
        _, off = p.delays()
        want = OR.stage2(sub, off, 0, p.nds, omp=True)
        assert np.array_equal(got, want)
        assert p.kernel().startswith("k_stage2_rw<" if variant == 8 else "k_stage2_qp<")
    finally:
        p.destroy()


def test_stage2_pair_rejects_unbounded_subbands(engine):
    """16-bit data: no host bound on |subband| -> the pair variant refuses (HD_E_INVAL) and
    the default falls back to the ring kernel, still bit-exact."""
    obs = palfa_obs(N=2 * 8192, nbits=16)
    raw = load_beam(engine, obs)
    pp = PassParams(subdm=30.0, lodm=26.2, dmstep=0.1, numdms=76, nsub=96, ds=1, numout=0)
    p = engine.plan(pp)
    p.run_subband()
    p.set_variant(6)
    with pytest.raises(PrestoError):
        p.run_dedisp()
    p.set_variant(0)
    got = p.run_dedisp()
    _, want = OR.run_pass(obs, Opts(), raw, pp)
    assert_series(got, want, obs.N)


@pytest.mark.parametrize("mask_pts", [0, 256, 32768])
@pytest.mark.parametrize("s1", [0, 2])
def test_stage1_multipass_bitexact(engine, mask_pts, s1):
    """One launch forms the subbands of many passes (a DDplan stage) from one raw read;
    every pass must equal its own oracle run.  mask_pts=256 takes the per-row interval path,
    32768 the two-interval path; s1=0 picks the 8-bit integer kernel, 2 the float one."""
    obs = palfa_obs(N=40000, nbits=8)
    s = palfa_synth()
    raw = load_beam(engine, obs, synth=s)
    mask = pad = None
    if mask_pts:
        mask, pad = synth_mask(obs, s, mask_pts, frac=0.05)
        engine.set_mask(mask, mask_pts, pad)
    d = plan.ddplans_for("pdev")[1]     # 12 passes, ds 2
    pps = [PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=d.dmstep,
                      numdms=d.dmsperpass, nsub=96, ds=d.sub_downsamp) for i in range(d.numpasses)]
    plans = [engine.plan(pp) for pp in pps]
    for p in plans:
        p.set_variant(s1 << 8)
    engine.run_subband_multi(plans)
    for pp, p in zip(pps, plans):
        want = OR.stage1(obs, Opts(), raw, 96, pp.ds, pp.subdm, mask=mask, ptsperint=mask_pts, padvals=pad)
        assert np.array_equal(p.get_subbands(), want), pp.subdm
    engine.set_mask()


@pytest.mark.parametrize("mask_pts", [2048, 32768])
def test_stage1_16bit_masked_two_block_tiles(engine, mask_pts):
    """16-bit data (the float stage-1 kernel) under a mask, clipping on: tiles over one interval
    boundary run in the main launch (two blocks' pads and zap bits per row), only tiles over
    three or more take the special launch; the clip state (16-bit zero-DM and channel-sum
    kernels, big-endian samples) and every pass's subbands equal the oracle's."""
    obs = palfa_obs(N=40000, nbits=16)
    s = palfa_synth(nbits=16)
    raw = load_beam(engine, obs, synth=s)
    mask, pad = synth_mask(obs, s, mask_pts, frac=0.05)
    engine.set_mask(mask, mask_pts, pad)
    try:
        gpad, gclip, gzap, ncl = engine.get_clean()
        want = OR.prepare(obs, Opts(), raw, (None, None, None), mask, mask_pts, pad)
        assert np.array_equal(gclip, want.clipped) and ncl == want.nclipped
        assert np.array_equal(gzap, want.zap)
        for ds, subdm in ((1, 30.0), (5, 612.0)):
            pp = PassParams(subdm=subdm, lodm=subdm - 10.0, dmstep=0.5, numdms=8, nsub=96, ds=ds)
            p = engine.plan(pp)
            p.run_subband()
            want = OR.stage1(obs, Opts(), raw, 96, ds, subdm, mask=mask, ptsperint=mask_pts, padvals=pad)
            assert np.array_equal(p.get_subbands(), want), ds
            p.destroy()
    finally:
        engine.set_mask()


@pytest.mark.parametrize("ds", [1, 2, 3, 5, 6, 10])
@pytest.mark.parametrize("flip,sub_dtype,ds_mode,masked", [(True, 0, 0, True), (False, 0, 1, False),
                                                          (False, 1, 0, True), (True, 1, 1, True)])
def test_stage1_int8_path_bitexact(engine, ds, flip, sub_dtype, ds_mode, masked):
    """8-bit integer stage-1 kernel (variant 3) over 3 passes of one launch: exact integer sums,
    the integer-prefix + float fold of subbands with zapped channels, and the special tiles
    (mask-interval straddles, last tile) on the float kernel -- all equal to the oracle."""
    obs = palfa_obs(N=65536 + 777, nbits=8, flip=flip)
    opts = Opts(sub_dtype=sub_dtype, ds_mode=ds_mode)
    s = palfa_synth()
    raw = load_beam(engine, obs, opts, synth=s)
    mask = pad = None
    pts = 16384
    if masked:
        mask, pad = synth_mask(obs, s, pts, frac=0.1)
        engine.set_mask(mask, pts, pad)
    pps = [PassParams(subdm=sd, lodm=sd - 5.0, dmstep=0.5, numdms=4, nsub=96, ds=ds) for sd in (40.0, 350.0, 1020.0)]
    plans = [engine.plan(pp) for pp in pps]
    for p in plans:
        p.set_variant(3 << 8)
    engine.run_subband_multi(plans)
    for pp, p in zip(pps, plans):
        want = OR.stage1(obs, opts, raw, 96, ds, pp.subdm, mask=mask, ptsperint=pts if masked else 0, padvals=pad)
        assert np.array_equal(p.get_subbands(), want), pp.subdm
        p.destroy()
    engine.set_mask()


@pytest.mark.parametrize("nbits,N", [(16, 8192), (4, 8190)])
def test_stage1_int8_variant_rejects_other_data(engine, nbits, N):
    """The integer path takes 8-bit data and 4-bit data through its unpacked channel-major
    copy (N % 4 == 0); 16-bit data, and 4-bit beams without that copy, are refused."""
    obs = palfa_obs(N=N, nbits=nbits)
    load_beam(engine, obs)
    p = engine.plan(PassParams(subdm=10.0, lodm=0.0, dmstep=1.0, numdms=4, nsub=96, ds=1))
    p.set_variant(3 << 8)
    with pytest.raises(PrestoError, match="integer path"):
        p.run_subband()


def test_stage2_f32_subbands(engine):
    obs = palfa_obs(N=16384, nbits=8)
    opts = Opts(sub_dtype=1, ds_mode=1)
    raw = load_beam(engine, obs, opts)
    pp = PassParams(subdm=230.0, lodm=222.4, dmstep=0.3, numdms=20, nsub=96, ds=2, numout=8192 + 300)
    p = engine.plan(pp)
    p.run_subband()
    got = p.run_dedisp()
    _, want = OR.run_pass(obs, opts, raw, pp)
    nds = obs.N // 2
    assert np.array_equal(got[:, :nds], want[:, :nds])
    # padding mean: double sums in a different association order -> within REL_TOL
    np.testing.assert_allclose(got[:, nds:], want[:, nds:], rtol=REL_TOL, atol=0)


@pytest.mark.parametrize("ds", [1, 3])
def test_no_subband_pass_nsub_eq_nchan(engine, ds):
    """use_subbands=False (PALFA2_presto_search.py:522-529): every channel is its own float32
    subband (nsub = nchan = 960), -downsamp dd*sub; bit-exact against the oracle on the data
    samples, padding mean within REL_TOL; masked."""
    obs = palfa_obs(N=12288 + 5, nbits=8)
    opts = Opts(sub_dtype=1)
    s = palfa_synth()
    raw = load_beam(engine, obs, opts, synth=s)
    pts = 2048
    mask, pad = synth_mask(obs, s, pts)
    engine.set_mask(mask, pts, pad)
    pp = PassParams(subdm=70.0, lodm=70.0, dmstep=0.3, numdms=12, nsub=obs.nchan, ds=ds,
                    numout=obs.N // ds + 333)
    p = engine.plan(pp)
    idd, _ = p.delays()
    assert not idd.any()
    p.run_subband()
    got = p.run_dedisp()
    p.destroy()
    engine.set_mask()
    _, want = OR.run_pass(obs, opts, raw, pp, mask=mask, ptsperint=pts, padvals=pad)
    nds = obs.N // ds
    assert np.array_equal(got[:, :nds], want[:, :nds])
    np.testing.assert_allclose(got[:, nds:], want[:, nds:], rtol=REL_TOL, atol=0)


def test_sub_input_mode_matches_one_shot(engine):
    """Stage 2 fed from .subNN data (HD_PASS_SUB_INPUT, .sub.inf values) == one-shot pass."""
    obs = palfa_obs(N=20000, nbits=8)
    raw = load_beam(engine, obs)
    pp = PassParams(subdm=454.6, lodm=443.2, dmstep=0.3, numdms=76, nsub=96, ds=3, numout=7000)
    p = engine.plan(pp)
    p.run_subband()
    sub = p.get_subbands()
    ref = p.run_dedisp()
    sobs = palfa_obs(N=sub.shape[1], nchan=96, flip=False)
    sobs.lofreq, sobs.df, sobs.dt = p.sub_lofreq, p.sub_chanwid, p.sub_dt
    engine.set_obs(sobs, Opts())
    q = engine.plan(PassParams(subdm=454.6, lodm=443.2, dmstep=0.3, numdms=76, nsub=96, ds=1, numout=7000,
                               sub_input=True))
    q.set_subbands(sub)
    assert np.array_equal(q.run_dedisp(), ref)
    engine.set_obs(obs, Opts())


def test_state_errors(engine):
    obs = palfa_obs(N=4096, nbits=8)
    engine.set_obs(obs, Opts())
    p = engine.plan(PassParams(subdm=10.0, lodm=0.0, dmstep=1.0, numdms=4, nsub=96, ds=1))
    with pytest.raises(PrestoError, match="no raw data"):
        p.run_subband()
    with pytest.raises(PrestoError, match="hd_run_subband"):
        p.run_dedisp()
    with pytest.raises(PrestoError, match="nsub"):
        engine.plan(PassParams(subdm=10.0, lodm=0.0, dmstep=1.0, numdms=4, nsub=97, ds=1))
    with pytest.raises(PrestoError, match="negative"):
        engine.plan(PassParams(subdm=10.0, lodm=-5.0, dmstep=1.0, numdms=4, nsub=96, ds=1))


def test_c1_config_three_passes_with_mask(engine):
    """Config 1 (BASELINE.json configs[0]): 960 ch x 2^20 samples, one pass each from DDplan
    stages 0, 1 and 3 (216 DMs), rfifind-style mask: full-length bit-exact vs the oracle."""
    N = 1 << 20
    obs = palfa_obs(N=N, nbits=8)
    s = palfa_synth()
    raw = load_beam(engine, obs, synth=s)
    pts = rfifind_ptsperint(obs.dt)
    mask, pad = synth_mask(obs, s, pts)
    engine.set_mask(mask, pts, pad)
    ps = plan.ddplans_for("pdev")
    for st, i in ((0, 0), (1, 0), (3, 0)):
        d = ps[st]
        pp = PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                        numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp, numout=plan.choose_N(N / d.downsamp))
        p = engine.plan(pp)
        p.run_subband()
        got_sub = p.get_subbands()
        got = p.run_dedisp()
        want_sub, want = OR.run_pass(obs, Opts(), raw, pp, mask=mask, ptsperint=pts, padvals=pad, omp=True)
        assert np.array_equal(got_sub, want_sub), st
        assert_series(got, want, N // pp.ds)
        p.destroy()
    engine.set_mask()


def test_injected_single_pulse_recovered(engine):
    """The DM-350 single pulse of the synthetic beam peaks in the trial nearest DM 350 at the
    injected arrival sample (top of band), on the full-resolution pass that covers it."""
    N = 1 << 18
    obs = palfa_obs(N=N, nbits=8)
    s = palfa_synth()
    s.npsr = 0
    s.sp_time[0], s.sp_dm[0], s.sp_amp[0], s.sp_width[0] = 4.0, 350.0, 20.0, 0.002
    s.burst_frac, s.spike_frac = 0.0, 0.0
    load_beam(engine, obs, synth=s)
    pp = PassParams(subdm=350.0, lodm=340.0, dmstep=0.5, numdms=40, nsub=96, ds=1)
    p = engine.plan(pp)
    p.run_subband()
    out = p.run_dedisp().astype(np.float64)
    _, off = p.delays()
    out = out[:, : p.nds - int(off.max()) - 1]          # drop the tail whose reads run past the end
    med = np.median(out, axis=1, keepdims=True)
    mad = 1.4826 * np.median(np.abs(out - med), axis=1, keepdims=True)
    z = (out - med) / mad
    d, t = np.unravel_index(np.argmax(z), z.shape)
    assert abs((pp.lodm + d * pp.dmstep) - 350.0) <= 1.0
    t0 = int(round(4.0 / obs.dt))
    w = int(round(0.002 / obs.dt))
    assert t0 - 2 <= t <= t0 + w + 2
    assert z[d, t] > 8.0


@pytest.mark.parametrize("nbits,flip,block", [(8, True, 0), (4, True, 700000), (16, False, 1 << 20)])
def test_psrfits_stream_ingest(engine, tmp_path, nbits, flip, block):
    """hd_push_raw_file (pinned double-buffered pread -> hipMemcpyAsync): the device raw block
    equals the file's spectra byte for byte, for one block and for many blocks (small block
    sizes force the two pinned buffers to alternate), and a pass run on it matches the oracle."""
    from hipdedisp.formats import psrfits
    obs = palfa_obs(N=8192, nbits=nbits, nsblk=512, flip=flip)
    spectra = host_spectra(obs, palfa_synth(nbits=nbits))
    fn = str(tmp_path / "beam.fits")
    psrfits.write_psrfits(fn, spectra, obs)
    si = psrfits.SpectraInfo([fn])
    engine.set_obs(si.obs_params(), Opts())
    io_s, tot_s, nbytes = si.stream_to(engine, block_bytes=block)
    assert nbytes == spectra.size and 0.0 <= io_s <= tot_s
    assert np.array_equal(engine.get_raw(), spectra)
    pp = PassParams(subdm=30.0, lodm=26.2, dmstep=0.1, numdms=76, nsub=96, ds=1, numout=0)
    p = engine.plan(pp)
    p.run_subband()
    got = p.run_dedisp()
    p.destroy()
    _, want = OR.run_pass(obs, Opts(), spectra, pp)
    assert_series(got, want, obs.N)


def test_psrfits_stream_ingest_errors(engine, tmp_path):
    obs = palfa_obs(N=2048, nbits=8, nsblk=512)
    engine.set_obs(obs, Opts())
    with pytest.raises(PrestoError):
        engine.push_raw_file(str(tmp_path / "missing.fits"), 0, obs.rowbytes * 512, 0, obs.rowbytes * 512, 0, 4)
    with pytest.raises(PrestoError):   # DATA column that is not whole spectra
        engine.push_raw_file(str(tmp_path / "missing.fits"), 0, 1000, 0, 999, 0, 4)


def test_candidate_lists_identical_on_injected_sources(engine):
    """North-star check: the single-pulse and periodicity candidate lists computed from the
    GPU series equal those from the oracle's (prepsubband restatement) series, on a beam
    with the injected 4.6 ms pulsar (DM 71) and DM-350 single pulse plus RFI and mask; and
    the injections are found (pulse near DM 350, pulsar's fundamental at DM ~71)."""
    from candidates import fft_candidates, single_pulse_candidates
    N = 1 << 18
    obs = palfa_obs(N=N, nbits=8)
    s = palfa_synth()
    s.sp_time[0], s.sp_amp[0] = 3.0, 30.0
    raw = load_beam(engine, obs, synth=s)
    pts = rfifind_ptsperint(obs.dt)
    mask, pad = synth_mask(obs, s, pts)
    engine.set_mask(mask, pts, pad)
    d0 = plan.ddplans_for("pdev")[0]
    found = {}
    for name, pp in (("psr", PassParams(subdm=float(d0.subdmlist[9]), lodm=float(d0.lodm_arg(9)),
                                        dmstep=float(d0.dmstep_arg()), numdms=76, nsub=96, ds=1,
                                        numout=plan.choose_N(N))),
                     ("sp", PassParams(subdm=350.0, lodm=340.0, dmstep=0.5, numdms=40, nsub=96, ds=1,
                                       numout=plan.choose_N(N)))):
        p = engine.plan(pp)
        p.run_subband()
        got = p.run_dedisp()
        p.destroy()
        _, want = OR.run_pass(obs, Opts(), raw, pp, mask=mask, ptsperint=pts, padvals=pad, omp=True)
        if name == "sp":
            cg, cw = single_pulse_candidates(got, obs.dt), single_pulse_candidates(want, obs.dt)
        else:
            cg, cw = fft_candidates(got), fft_candidates(want)
        assert cg == cw and len(cg) > 0, name
        found[name] = (cg, pp)
    cands, pp = found["sp"]
    best = max(cands, key=lambda c: c[3])
    assert abs(pp.lodm + best[0] * pp.dmstep - 350.0) <= 2.0
    cands, pp = found["psr"]
    f0 = 1.0 / 0.0046 * N * obs.dt            # fundamental bin of the 4.6 ms pulsar
    hits = [c for c in cands if c[1] == 1 and abs(c[2] - f0) <= 2]
    assert hits, "pulsar fundamental not among the top bins"
    best_dm = pp.lodm + max(hits, key=lambda c: c[3])[0] * pp.dmstep
    assert abs(best_dm - 71.0) <= 1.5
    engine.set_mask()


def test_dual_stream_stage2_matches(engine):
    """hd_set_streams(2): consecutive passes alternate between two streams (and a plan re-run
    on the other stream, and stage 1 rewriting subbands a stream-2 pass still reads, are
    ordered) -- every series equals the single-stream result, over repeated beams."""
    obs = palfa_obs(N=3 * 8192, nbits=8)
    load_beam(engine, obs)
    d = plan.ddplans_for("pdev")[0]
    pps = [PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                      numdms=d.dmsperpass, nsub=d.numsub, ds=1, numout=plan.choose_N(obs.N)) for i in range(5)]
    plans = [engine.plan(pp) for pp in pps]
    engine.run_subband_multi(plans)
    want = [p.run_dedisp() for p in plans]
    engine.set_streams(2)
    try:
        for _ in range(3):
            engine.run_subband_multi(plans)
            for p in plans:
                p.run_dedisp(to_host=False)
            got = [p.run_dedisp() for p in plans]          # host copies, alternating streams again
            for g, w in zip(got, want):
                assert np.array_equal(g, w)
        engine.sync()
    finally:
        engine.set_streams(1)
        for p in plans:
            p.destroy()


def test_stage2_own_stream_overlap_matches(engine):
    """hd_set_streams(3): every stage-2 pass on the second stream behind its stage 1, the next
    DDplan stage's stage 1 overlapping it; beams alternate between two raw contents, so a
    stage 1 that rewrote subbands before their last stage-2 reader finished, or a stage 2
    that read them before they were written, would show -- every series equals the
    single-stream result of its beam."""
    obs = palfa_obs(N=3 * 8192, nbits=8)
    engine.set_obs(obs, Opts())
    stages = []
    for st, n in ((0, 3), (1, 2), (3, 2)):
        d = plan.ddplans_for("pdev")[st]
        stages.append([engine.plan(PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)),
                                              dmstep=float(d.dmstep_arg()), numdms=d.dmsperpass, nsub=d.numsub,
                                              ds=d.sub_downsamp, numout=plan.choose_N(obs.N / d.downsamp)))
                       for i in range(n)])
    synths = [palfa_synth(beam=0), palfa_synth(beam=1)]

    def beam(k):
        engine.synth_device(synths[k])
        for ps in stages:
            engine.run_subband_multi(ps)
            for p in ps:
                p.run_dedisp(to_host=False)

    want = []
    for k in range(2):
        beam(k)
        want.append([p.get_series(0, None, 0, p.numout) for ps in stages for p in ps])
    engine.set_streams(3)
    try:
        for it in range(4):
            beam((it + 1) % 2)              # queued, not read: the next beam's stage 1 must wait
            beam(it % 2)                    # for these stage-2 passes per plan
            got = [p.get_series(0, None, 0, p.numout) for ps in stages for p in ps]
            for g, w in zip(got, want[it % 2]):
                assert np.array_equal(g, w), it
        engine.sync()
    finally:
        engine.set_streams(1)
        for ps in stages:
            for p in ps:
                p.destroy()


def test_stage2_multipass_launch_matches(engine):
    """hd_run_dedisp_multi: the passes of a DDplan stage share one pair-kernel launch (per-pass
    subbands, tables, outputs and padding sums from the launch's pass table).  Passes of three
    stages given in mixed order over a ragged beam with more tiles than CUs, masked: every
    series equals its own one-pass launch (which the oracle pins, checked here for one pass
    per stage), over repeated beams of alternating raw contents and with stage 2 on two
    streams before; the first plan of each shared launch reports its pass count, the others 0."""
    obs = palfa_obs(N=(1 << 19) + 777, nbits=8)
    engine.set_obs(obs, Opts())
    synths = [palfa_synth(beam=0), palfa_synth(beam=1)]
    pts = 2048
    mask, pad = synth_mask(obs, synths[0], pts)
    engine.set_mask(mask, pts, pad)
    plans, pps = [], []
    for st, idx in ((0, (0, 3, 7, 27)), (1, (1, 2, 11)), (3, (0, 8))):
        d = plan.ddplans_for("pdev")[st]
        for i in idx:
            pp = PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                            numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                            numout=plan.choose_N(obs.N / d.downsamp))
            pps.append(pp)
            plans.append(engine.plan(pp))
    order = [0, 4, 7, 1, 5, 2, 8, 3, 6]                      # stages interleaved
    try:
        want = []
        for k in range(2):
            engine.synth_device(synths[k])
            engine.run_subband_multi(plans[0:4])
            engine.run_subband_multi(plans[4:7])
            engine.run_subband_multi(plans[7:9])
            want.append([p.run_dedisp() for p in plans])
            if k == 0:
                raw = host_spectra(obs, synths[0])
                for j in (0, 4, 7):
                    _, w = OR.run_pass(obs, Opts(), raw, pps[j], mask=mask, ptsperint=pts, padvals=pad, omp=True)
                    assert_series(want[0][j], w, obs.N // pps[j].ds)
        for it in range(4):
            k = it % 2
            engine.synth_device(synths[k])
            engine.run_subband_multi(plans[0:4])
            engine.run_subband_multi(plans[4:7])
            engine.run_subband_multi(plans[7:9])
            if it == 2:
                engine.set_streams(2)
                for p in plans[:3]:
                    p.run_dedisp(to_host=False)              # alternating streams, then the shared launch
            engine.run_dedisp_multi([plans[i] for i in order])
            engine.set_streams(1)
            for j, p in enumerate(plans):
                assert np.array_equal(p.get_series(0, None, 0, p.numout), want[k][j]), (it, j)
            n = [p.launch_passes() for p in plans]
            assert sum(n) == len(plans)
            assert n[0] >= 1 and n[4] >= 1 and n[7] >= 1, n
        engine.sync()
        with pytest.raises(PrestoError):
            engine.run_dedisp_multi([])
        with pytest.raises(PrestoError):
            engine.run_dedisp_multi([plans[0], plans[0]])
    finally:
        engine.set_streams(1)
        engine.set_mask()
        for p in plans:
            p.destroy()


def test_stage1_channel_major_fill(engine):
    """The 8-bit stage-1 kernel fills its LDS tile from a channel-major copy of the raw block
    (built once per raw block): results equal the row-major fill (probe bit 2) and the oracle,
    and a new raw block (hd_push_raw) or hd_touch_raw rebuilds the copy."""
    obs = palfa_obs(N=3 * 8192, nbits=8)
    d = plan.ddplans_for("pdev")[3]
    pp = PassParams(subdm=float(d.subdmlist[2]), lodm=float(d.lodm_arg(2)), dmstep=float(d.dmstep_arg()),
                    numdms=d.dmsperpass, nsub=96, ds=d.sub_downsamp, numout=0)
    for beam in (0, 1):
        raw = load_beam(engine, obs, synth=palfa_synth(beam=beam), device_synth=False)
        p = engine.plan(pp)
        p.run_subband()
        a = p.get_subbands()
        p.set_variant(4 << 16)            # probe: row-major fill
        p.run_subband()
        b = p.get_subbands()
        p.set_variant(0)
        engine.touch_raw()
        p.run_subband()
        c = p.get_subbands()
        want, _ = OR.run_pass(obs, Opts(), raw, pp)
        p.destroy()
        assert np.array_equal(a, want) and np.array_equal(b, want) and np.array_equal(c, want), beam


@pytest.mark.parametrize("use_subbands", [True, False])
def test_search_stage_dedisperse_job(engine, tmp_path, use_subbands):
    """search_stage.dedisperse_job (the loop of PALFA2_presto_search.py:494-537) on a PSRFITS
    file, with and without subbands: one pass each from DDplan stages 0 and 3; the
    <base>_DM<dm>.dat files equal the oracle's series for the same command parameters, the
    .inf records N and DM, and the timers go where the reference puts them."""
    import copy
    import os
    from hipdedisp.formats import psrfits
    from hipdedisp.formats.inf import read_inf
    from hipdedisp.search_stage import DedispJob, dedisperse_job, pass_params
    obs = palfa_obs(N=8192, nbits=8, nsblk=512)
    spectra = host_spectra(obs, palfa_synth())
    fn = str(tmp_path / "beam.fits")
    psrfits.write_psrfits(fn, spectra, obs)
    job = DedispJob([fn], resultsdir=str(tmp_path), tmpdir_base=str(tmp_path), device=0,
                    use_subbands=use_subbands, backend="pdev", workdir=str(tmp_path))
    ddplans = []
    for st in (0, 3):
        d = copy.copy(job.ddplans[st])
        d.numpasses = 1
        ddplans.append(d)
    job.ddplans = ddplans
    spdir = tmp_path / "sp"
    spdir.mkdir()
    try:
        dmstrs = dedisperse_job(job, single_pulse=dict(maxwidth=0.1, threshold=5.0, workdir=str(spdir)),
                                fft=dict(zaplist=None, baryv=0.0, write=True))
        assert len(dmstrs) == sum(d.dmsperpass for d in ddplans)
        assert job.singlepulse_time > 0 and job.FFT_time > 0
        from hipdedisp.search_stage import command_lines
        for d in ddplans:                       # the per-pass stdout logs of :511,520
            sub = tmp_path / ("%s_DM%s.subout" % (job.basefilenm, d.subdmlist[0]))
            prep = tmp_path / ("%s_DM%s.prepout" % (job.basefilenm, d.subdmlist[0]))
            if use_subbands:
                cmds = command_lines(job, d, 0, None, job.tempdir)
                assert sub.read_text().startswith("'%s'" % cmds[0]) and "-sub -subdm" in cmds[0]
                assert prep.read_text().startswith("'%s'" % cmds[1]) and "-numout" in cmds[1]
            else:
                assert not sub.exists() and not prep.exists()
        sobs = job.specinfo.obs_params(0.0)
        for d in ddplans:
            pp = pass_params(job, d, 0)
            _, want = OR.run_pass(sobs, job.opts, spectra, pp)
            nds = int(obs.N // pp.ds)
            for k, dmstr in enumerate(d.dmlist[0]):
                base = os.path.join(job.tempdir, "%s_DM%s" % (job.basefilenm, dmstr))
                got = np.fromfile(base + ".dat", np.float32)
                assert got.size == (pp.numout or nds)      # choose_N < 10000 -> 0: no padding
                assert np.array_equal(got[:nds], want[k, :nds]), dmstr
                np.testing.assert_allclose(got[nds:], want[k, nds:], rtol=REL_TOL, atol=0)
                inf = read_inf(base + ".inf")
                assert inf.N == got.size and "%.2f" % inf.dm == dmstr
                # :548-558: the packed, de-reddened spectrum of the same series
                spec = np.fromfile(base + ".fft", np.float32)
                assert spec.size == got.size and spec[0] == 1.0 and spec[1] == 0.0
                # :539-546: <base>_DM<dm>.singlepulse in the work dir, equal to the oracle's
                # single_pulse_search restatement over the .dat just written
                wl = OR.sp_widths(inf.dt, 0.1)
                raw, bad = OR.sp_hits(got[None, :], wl, 5.0)
                ref = OR.sp_candidates(raw, bad, wl, [float(dmstr)], inf.dt, nds, got.size,
                                       ls=got.size // 1000 * 1000 // 8000 * 8000)[0]
                text = open(str(spdir / ("%s_DM%s.singlepulse" % (job.basefilenm, dmstr)))).read()
                assert text == ("# DM      Sigma      Time (s)     Sample    Downfact\n" + "".join(map(str, ref))
                                if ref else "")
        assert job.dedispersing_time > 0
        assert (job.subbanding_time > 0) == use_subbands
    finally:
        job.close()


def test_c4_ddplan2b_passes_to_dm_10000(engine):
    """Config 4 (BASELINE.json configs[3]): the DDplan2b plan from 0 to 10000 pc cm^-3
    (PALFA2_presto_search.py:308-317 -> DDplan2b.py), nsub 96, downsampling 1..64; the
    highest-DM pass of every step, with an rfifind-style mask, bit-exact against the oracle
    (subbands and series, padding included).  N = 2^18 so the DM-10090 sweep (~10.7 s of
    delay) still has data under it."""
    N = 1 << 18
    obs = palfa_obs(N=N, nbits=8)
    s = palfa_synth()
    raw = load_beam(engine, obs, synth=s)
    pts = rfifind_ptsperint(obs.dt)
    mask, pad = synth_mask(obs, s, pts)
    engine.set_mask(mask, pts, pad)
    steps = plan.ddplan2b_plans(obs.dt, 1375.5, 322.6, obs.nchan, 2048, 0.0, 10000.0, 96, 0.1)
    assert max(d.downsamp for d in steps) == 64
    try:
        for d in steps:
            i = d.numpasses - 1
            pp = PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                            numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                            numout=plan.choose_N(N / d.downsamp))
            p = engine.plan(pp)
            p.run_subband()
            got_sub = p.get_subbands()
            got = p.run_dedisp()
            p.destroy()
            want_sub, want = OR.run_pass(obs, Opts(), raw, pp, mask=mask, ptsperint=pts, padvals=pad, omp=True)
            assert np.array_equal(got_sub, want_sub), d.downsamp
            assert_series(got, want, N // pp.ds)
    finally:
        engine.set_mask()


@pytest.mark.parametrize("N,ds,numdms", [(4096, 1, 76), (4096 + 13, 3, 1), (2000, 2, 64), (1, 1, 4), (3, 5, 4)])
def test_beam_shorter_than_the_sweep(engine, N, ds, numdms):
    """Edge sizes: a beam shorter than its own dispersion sweep (DM ~1000: ~1 s = 16k samples
    of delay across the band, every stage-1 and stage-2 read past the end), a single DM, a
    ragged length, a one-sample beam, and fewer samples than the downsampling factor (no
    output: refused).  Bit-exact against the oracle, padding included."""
    obs = palfa_obs(N=N, nbits=8)
    raw = load_beam(engine, obs)
    nds = N // ds
    pp = PassParams(subdm=1000.0, lodm=990.0, dmstep=0.5, numdms=numdms, nsub=96, ds=ds, numout=nds + 100)
    if nds == 0:
        with pytest.raises(PrestoError):
            engine.plan(pp)
        return
    p = engine.plan(pp)
    p.run_subband()
    got_sub = p.get_subbands()
    got = p.run_dedisp()
    p.destroy()
    want_sub, want = OR.run_pass(obs, Opts(), raw, pp)
    assert np.array_equal(got_sub, want_sub)
    assert_series(got, want, nds)


def test_prepsubband_cli_shim_commands(engine, tmp_path):
    """The reference's three command strings (PALFA2_presto_search.py:506-511, :514-520,
    :522-527) through the `prepsubband` shim: exit status 0, and the .dat series equal the
    oracle's for the same parameters (the two-step subband path via .subNN files)."""
    import glob
    import os
    from hipdedisp import prepsubband as cli
    from hipdedisp.formats import psrfits
    obs = palfa_obs(N=8192, nbits=8, nsblk=512)
    spectra = host_spectra(obs, palfa_synth())
    fn = str(tmp_path / "beam.fits")
    psrfits.write_psrfits(fn, spectra, obs)
    sobs = psrfits.SpectraInfo([fn]).obs_params(0.0)
    os.makedirs(str(tmp_path / "subbands"))
    dev = ["-device", "0"]
    assert cli.main(("-psrfits -sub -subdm 30.40 -downsamp 1 -nsub 96 -o %s/subbands/beam %s"
                     % (tmp_path, fn)).split() + dev) == 0
    subs = sorted(glob.glob(str(tmp_path / "subbands" / "beam_DM30.40.sub[0-9]*")))
    assert len(subs) == 96
    assert cli.main(("-lodm 26.60 -dmstep 0.10 -numdms 76 -downsamp 1 -nsub 96 -numout 0 -o %s/beam"
                     % tmp_path).split() + subs + dev) == 0
    pp = PassParams(subdm=30.4, lodm=26.6, dmstep=0.1, numdms=76, nsub=96, ds=1, numout=0)
    _, want = OR.run_pass(sobs, Opts(), spectra, pp)
    for k in (0, 37, 75):
        got = np.fromfile(str(tmp_path / ("beam_DM%.2f.dat" % (26.6 + 0.1 * k))), np.float32)
        assert np.array_equal(got, want[k]), k
    assert cli.main(("-mask none -lodm 100.00 -dmstep 1.00 -numdms 8 -downsamp 2 -numout 0 -o %s/nosub %s"
                     % (tmp_path, fn)).split()[2:] + dev) == 0
    pp = PassParams(subdm=100.0, lodm=100.0, dmstep=1.0, numdms=8, nsub=obs.nchan, ds=2, numout=0)
    _, want = OR.run_pass(sobs, Opts(sub_dtype=1), spectra, pp)
    for k in (0, 7):
        got = np.fromfile(str(tmp_path / ("nosub_DM%.2f.dat" % (100.0 + k))), np.float32)
        assert np.array_equal(got, want[k]), k


def test_write_series_async_files(engine, tmp_path):
    """hd_write_series: the device series of a pass land in .dat files (pinned buffers, copy
    stream, writer threads) equal to the host copy, while the next pass runs; re-running a
    plan with copies still queued is ordered after them; a bad path fails with HD_E_IO."""
    obs = palfa_obs(N=3 * 8192 + 5, nbits=8)
    load_beam(engine, obs)
    d = plan.ddplans_for("pdev")[2]
    plans = [engine.plan(PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)),
                                    dmstep=float(d.dmstep_arg()), numdms=d.dmsperpass, nsub=96, ds=d.sub_downsamp,
                                    numout=obs.N // 3 + 100)) for i in range(3)]
    try:
        engine.run_subband_multi(plans)
        paths = []
        for i, p in enumerate(plans):
            p.run_dedisp(to_host=False)
            paths.append([str(tmp_path / ("p%d_DM%s.dat" % (i, s))) for s in d.dmlist[i]])
            p.write_series(paths[-1], wait=False)
        want0 = plans[0].get_series()
        plans[0].run_dedisp(to_host=False)            # ordered after its queued copies
        sec, nbytes = engine.wait_writes()
        assert nbytes >= 3 * 76 * 4 * plans[0].numout and sec > 0
        for i, p in enumerate(plans):
            want = p.get_series()
            for k in (0, 40, 75):
                got = np.fromfile(paths[i][k], np.float32)
                assert np.array_equal(got, want[k]), (i, k)
        assert np.array_equal(plans[0].get_series(), want0)
        with pytest.raises(PrestoError, match="cannot create"):
            plans[1].write_series([str(tmp_path / "missing_dir" / "x.dat")] * 76)
    finally:
        for p in plans:
            p.destroy()


@pytest.mark.parametrize("fold_rawdata", [True, False])
def test_reference_pass_loop_control_flow(engine, tmp_path, fold_rawdata):
    """The reference's own loop around the drop-in (PALFA2_presto_search.py:494-615 with the
    INTEGRATION.md patch): run_pass, then the per-DM .dat/.inf handling, then :608-614 --
    shutil.rmtree(tempdir/subbands) when folding raw data, else moving the .subNN files to
    workdir/subbands.  Neither branch may raise, and without fold_rawdata the subband files
    the folds need (one per subband plus .sub.inf) must be there to move."""
    import copy
    import glob
    import os
    import shutil
    from hipdedisp.formats import psrfits
    from hipdedisp.search_stage import DedispJob, run_pass
    obs = palfa_obs(N=4096, nbits=8, nsblk=512)
    fn = str(tmp_path / "beam.fits")
    psrfits.write_psrfits(fn, host_spectra(obs, palfa_synth()), obs)
    workdir = tmp_path / "work"
    (workdir / "subbands").mkdir(parents=True)
    job = DedispJob([fn], resultsdir=str(workdir), tmpdir_base=str(tmp_path), device=0, workdir=str(tmp_path),
                    backend="pdev", keep_subbands=not fold_rawdata)
    try:
        d = copy.copy(job.ddplans[0])
        d.numpasses = 2
        for passnum in range(d.numpasses):
            run_pass(job, d, passnum, None, job.tempdir)
            for dmstr in d.dmlist[passnum]:                                    # :531-606
                basenm = os.path.join(job.tempdir, job.basefilenm + "_DM" + dmstr)
                assert os.path.getsize(basenm + ".dat") > 0
                shutil.move(basenm + ".inf", str(workdir))
                os.remove(basenm + ".dat")
            if fold_rawdata:                                                    # :608-611
                shutil.rmtree(os.path.join(job.tempdir, "subbands"))
            else:                                                               # :612-614
                subs = glob.glob(os.path.join(job.tempdir, "subbands", "*"))
                assert len(subs) == d.numsub + 1, len(subs)
                for sub in subs:
                    shutil.move(sub, os.path.join(str(workdir), "subbands"))
        moved = os.listdir(workdir / "subbands")
        assert len(moved) == (0 if fold_rawdata else d.numpasses * (d.numsub + 1))
        assert len(glob.glob(str(workdir / "*.inf"))) == d.numpasses * d.dmsperpass
    finally:
        job.close()
