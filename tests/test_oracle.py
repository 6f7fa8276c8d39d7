"""Pin the CPU oracle: C restatement vs the independent numpy restatement (bit for bit),
plus analytic known-answer tests.  (PRESTO is absent, so against PRESTO itself the oracle
is parity-unpinned; see oracle/oracle.h and DESIGN.md §4-5.)"""
import numpy as np
import pytest

import oracle as OR
import oracle_np as ON
from hipdedisp import Opts, PassParams, stats_padvals
from hipdedisp.synth import palfa_obs

NOCLIP = dict(clip_sigma=0.0)


def small_obs(nchan=64, N=4096, nbits=8, flip=False, nsblk=256):
    return palfa_obs(N=N, nbits=nbits, nchan=nchan, nsblk=nsblk, flip=flip)


@pytest.mark.parametrize("subdm", [0.0, 3.8, 212.7, 1028.4])
@pytest.mark.parametrize("nchan,nsub", [(960, 96), (64, 8), (64, 64)])
def test_chan_delays_c_vs_numpy(nchan, nsub, subdm):
    obs = small_obs(nchan=nchan)
    a = OR.chan_delays(obs, nsub, subdm)
    b = ON.chan_delays(nchan, nsub, subdm, obs.lofreq, obs.df, obs.dt)
    assert np.array_equal(a, b)
    assert a.min() >= 0
    if subdm == 0:
        assert not a.any()
    # the top channel of every subband has zero delay
    assert not a[nsub and (nchan // nsub - 1)::nchan // nsub].any()


@pytest.mark.parametrize("ds", [1, 2, 3, 5, 6, 10])
@pytest.mark.parametrize("roundtrip", [True, False])
def test_dm_offsets_c_vs_numpy(ds, roundtrip):
    obs = small_obs(nchan=960)
    opts = Opts(inf_roundtrip=roundtrip)
    a = OR.dm_offsets(obs, opts, 96, ds, 534.4, 0.5, 76)
    b = ON.dm_offsets(960, 96, ds, obs.lofreq, obs.df, obs.dt, 534.4, 0.5, 76, roundtrip=roundtrip)
    assert np.array_equal(a, b)
    assert (a[:, -1] == 0).all() and (np.diff(a, axis=0) >= 0).all() and (np.diff(a, axis=1) <= 0).all()


def test_sub_params_roundtrip_text():
    obs = small_obs(nchan=960)
    lof, bw, dt = OR.sub_params(obs, Opts(), 96, 3)
    assert lof == float("%.12g" % (obs.lofreq + obs.df * 10 - obs.df))
    assert bw == float("%.12g" % (obs.df * 10)) and dt == float("%.15g" % (obs.dt * 3))


def _rand_case(rng, nbits, nchan=64, N=2048, flip=False, nsblk=256):
    obs = small_obs(nchan=nchan, N=N, nbits=nbits, flip=flip, nsblk=nsblk)
    raw = rng.integers(0, 256, size=(N, obs.rowbytes), dtype=np.uint8)
    if nbits == 16:   # keep 16-bit values moderate so int16 subbands do not saturate everywhere
        v = rng.integers(-300, 300, size=(N, nchan)).astype(">i2")
        raw = v.view(np.uint8).reshape(N, obs.rowbytes)
    return obs, raw


def _np_stage1(obs, opts, raw, nsub, ds, subdm, calib=(None, None, None), mask=None, pts=0, pad=None,
               dtint=0.0, zapint=None):
    """The numpy twin end to end: block masks, clip_times, stage 1."""
    X = ON.decode(raw, obs.nchan, obs.nbits, obs.flip, *calib)
    zap, allzap = ON.block_masks(obs.N, obs.nchan, obs.dt, obs.nsblk, mask, pts, dtint, zapint)
    padrows, clipped = ON.clip_prepare(X, obs.nsblk, allzap, opts.clip_sigma, pad)
    idd = ON.chan_delays(obs.nchan, nsub, subdm, obs.lofreq, obs.df, obs.dt)
    return ON.stage1(raw, obs.nchan, obs.nbits, obs.flip, nsub, ds, idd, *calib, zap=zap, pad=padrows,
                     clipped=clipped, blk=obs.nsblk, sub_dtype=opts.sub_dtype, ds_mode=opts.ds_mode,
                     sub_round=opts.sub_round)


@pytest.mark.parametrize("nbits", [4, 8, 16])
@pytest.mark.parametrize("flip", [False, True])
@pytest.mark.parametrize("ds", [1, 3])
@pytest.mark.parametrize("clip", [0.0, 6.0])
def test_stage1_c_vs_numpy(nbits, flip, ds, clip):
    rng = np.random.default_rng(nbits * 10 + ds + flip)
    obs, raw = _rand_case(rng, nbits, flip=flip)
    opts = Opts(clip_sigma=clip)
    a = OR.stage1(obs, opts, raw, 8, ds, 150.0)
    b = _np_stage1(obs, opts, raw, 8, ds, 150.0)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("sub_dtype,ds_mode,sub_round", [(0, 0, 0), (0, 1, 0), (0, 1, 1), (1, 0, 0), (1, 1, 0)])
@pytest.mark.parametrize("clip", [0.0, 6.0])
def test_stage1_calib_mask_c_vs_numpy(sub_dtype, ds_mode, sub_round, clip):
    rng = np.random.default_rng(5 + sub_dtype + 2 * ds_mode)
    obs, raw = _rand_case(rng, 8, flip=True, N=4096)
    nc = obs.nchan
    scl = rng.uniform(0.5, 2.0, nc).astype(np.float32)
    offs = rng.uniform(-10, 10, nc).astype(np.float32)
    wts = (rng.random(nc) > 0.1).astype(np.float32)
    pts = 512
    mask = (rng.random((obs.N // pts + 1, nc)) < 0.1).astype(np.uint8)
    mask[2] = 1                                                 # a fully zapped interval
    pad = rng.uniform(50, 150, nc).astype(np.float32)
    opts = Opts(sub_dtype=sub_dtype, ds_mode=ds_mode, sub_round=sub_round, clip_sigma=clip)
    a = OR.stage1(obs, opts, raw, 8, 2, 400.0, calib=(scl, offs, wts), mask=mask, ptsperint=pts, padvals=pad)
    b = _np_stage1(obs, opts, raw, 8, 2, 400.0, (scl, offs, wts), mask, pts, pad)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("pts,dtint_scale", [(256, 1.0), (512, 1.0), (128, 1.0), (1000, 1.0), (512, 1.0000001)])
def test_block_masks_c_vs_numpy(pts, dtint_scale):
    """check_mask per read block: union of the block's first and last interval only (so
    with intervals shorter than a block the middle ones are not seen), zap_ints mask all."""
    rng = np.random.default_rng(pts)
    obs = small_obs(N=5000, nsblk=256)
    numint = -(-obs.N // pts)
    mask = (rng.random((numint, obs.nchan)) < 0.2).astype(np.uint8)
    zapint = (rng.random(numint) < 0.15).astype(np.uint8)
    dtint = pts * obs.dt * dtint_scale
    a = OR.block_masks(obs, mask, pts, dtint, zapint)
    b = ON.block_masks(obs.N, obs.nchan, obs.dt, obs.nsblk, mask, pts, dtint, zapint)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    for blk in range(len(a[1])):
        lo = min(int(blk * 256 * obs.dt / dtint), numint - 1)
        assert a[0][blk].astype(bool)[mask[lo].astype(bool)].all() or a[1][blk]


def _spiky(rng, N=8192, nchan=64, nsblk=512, nspike=12, amp=60):
    obs = small_obs(nchan=nchan, N=N, nsblk=nsblk, flip=True)
    raw = np.clip(rng.normal(100, 12, size=(N, nchan)), 0, 255).astype(np.uint8)
    spikes = np.sort(rng.choice(N, nspike, replace=False))
    raw[spikes] = np.clip(raw[spikes].astype(int) + amp, 0, 255).astype(np.uint8)
    return obs, raw, spikes


def test_clip_prepare_c_vs_numpy_and_finds_spikes():
    rng = np.random.default_rng(77)
    obs, raw, spikes = _spiky(rng)
    pad0 = rng.uniform(80, 120, obs.nchan).astype(np.float32)
    mask = np.zeros((obs.N // 1024, obs.nchan), np.uint8)
    mask[3] = 1                                                  # blocks 6, 7 fully masked: no clip there
    cl = OR.prepare(obs, Opts(), raw, mask=mask, ptsperint=1024, padvals=pad0)
    X = ON.decode(raw, obs.nchan, 8, True)
    zap, allzap = ON.block_masks(obs.N, obs.nchan, obs.dt, obs.nsblk, mask, 1024)
    pad, clipped = ON.clip_prepare(X, obs.nsblk, allzap, 6.0, pad0)
    assert np.array_equal(cl.pad, pad) and np.array_equal(cl.clipped, clipped) and np.array_equal(cl.zap, zap)
    assert cl.nclipped == int(clipped.sum())
    # every spike outside the fully masked blocks is clipped, nothing else
    live = [t for t in spikes if not allzap[t // obs.nsblk]]
    assert set(np.nonzero(clipped)[0]) == set(live)
    # pad rows: the initial values until the first clip, then the running channel levels,
    # carried through the masked blocks
    assert np.array_equal(cl.pad[6], cl.pad[5]) and np.array_equal(cl.pad[7], cl.pad[5])
    assert not np.array_equal(cl.pad[0], pad0) and np.abs(cl.pad[0] - 100).max() < 5


def test_clip_first_block_levels_are_good_point_means():
    """Block 0 (no history): running levels = the channel means of the 'good' spectra, i.e.
    those whose zero-DM sum lies within 0.7..1.3 of the block median."""
    rng = np.random.default_rng(5)
    obs, raw, spikes = _spiky(rng, N=512, nsblk=512, nspike=3, amp=120)
    cl = OR.prepare(obs, Opts(), raw)
    X = ON.decode(raw, obs.nchan, 8, True).astype(np.float64)
    z = X.sum(axis=1)
    med = np.sort(z.astype(np.float32))[(len(z) - 1) // 2]
    good = (z > 0.7 * med) & (z < 1.3 * med)
    assert not good[spikes].any()
    assert np.allclose(cl.pad[0], X[good].mean(axis=0), rtol=1e-6)
    assert set(np.nonzero(cl.clipped)[0]) == set(spikes)


def test_stage1_clip_replaces_spectrum_by_levels():
    """A clipped spectrum reads as the block's levels in every channel (ds=1, one channel per
    subband, no delays): the subband sample is the rounded level."""
    rng = np.random.default_rng(9)
    obs, raw, spikes = _spiky(rng, N=2048, nsblk=512, nspike=4, amp=120)
    opts = Opts(ds_mode=0)
    cl = OR.prepare(obs, opts, raw)
    sub = OR.stage1(obs, opts, raw, obs.nchan, 1, 0.0, clean=cl)
    for t in spikes:
        lev = cl.pad[t // obs.nsblk]
        assert np.array_equal(sub[:, t], np.floor(lev.astype(np.float64) + 0.5).astype(np.int16))
    unclipped = OR.stage1(obs, Opts(ds_mode=0, clip_sigma=0.0), raw, obs.nchan, 1, 0.0)
    keep = np.setdiff1d(np.arange(obs.N), spikes)
    assert np.array_equal(sub[:, keep], unclipped[:, keep])


def test_stage1_window_equals_full():
    """or_stage1 over [t0, t0+count) equals the same columns of the full run (bounded sampling)."""
    rng = np.random.default_rng(3)
    obs, raw = _rand_case(rng, 8, N=4096)
    full = OR.stage1(obs, Opts(), raw, 8, 2, 300.0)
    win = OR.stage1(obs, Opts(), raw, 8, 2, 300.0, t0=700, count=900)
    assert np.array_equal(full[:, 700:1600], win)
    omp = OR.stage1(obs, Opts(), raw, 8, 2, 300.0, omp=True)
    assert np.array_equal(full, omp)


def test_presto_short_rounding():
    """(short)(x + 0.5): truncation toward zero of x + 0.5 (so -2.7 -> -2), low 16 bits of
    the int32 conversion (40000 wraps), vs nearest-saturated."""
    vals = np.array([0.49, 0.5, 2.5, -0.4, -0.6, -2.7, 40000.0, -40000.0], np.float32)
    assert np.array_equal(ON._to_sub(vals, 0, 0), np.array([0, 1, 3, 0, 0, -2, -25536, 25537], np.int16))
    assert np.array_equal(ON._to_sub(vals, 0, 1), np.array([0, 1, 3, 0, -1, -3, 32767, -32768], np.int16))
    # the C oracle on a one-channel 16-bit pass: subband = the sample itself
    raw = np.array([0, 1, 3, -2, 30000, -30000, 7, 8], ">i2").view(np.uint8).reshape(8, 2)
    obs = palfa_obs(N=8, nbits=16, nchan=1, nsblk=8, flip=False)
    s = OR.stage1(obs, Opts(clip_sigma=0.0, ds_mode=1), raw, 1, 2, 0.0)
    want = ON._to_sub(np.array([0.5, 0.5, 0.0, 7.5], np.float32), 0, 0)
    assert np.array_equal(s[0], want)


@pytest.mark.parametrize("dtype", [np.int16, np.float32])
def test_stage2_c_vs_numpy(dtype):
    rng = np.random.default_rng(11)
    sub = rng.integers(-2000, 2000, size=(16, 3000)).astype(dtype)
    if dtype == np.float32:
        sub = sub * np.float32(0.37)
    off = np.sort(rng.integers(0, 200, size=(12, 16)), axis=1)[:, ::-1].astype(np.int32)
    off[:, -1] = 0
    a = OR.stage2(sub, off)
    b = ON.stage2(sub, off)
    assert np.array_equal(a, b)
    # windowed + OpenMP equal the full run
    assert np.array_equal(OR.stage2(sub, off, 1000, 500), a[:, 1000:1500])
    assert np.array_equal(OR.stage2(sub, off, omp=True), a)


def test_run_pass_padding_modes():
    rng = np.random.default_rng(2)
    obs, raw = _rand_case(rng, 8, N=3000)
    pp = PassParams(subdm=20.0, lodm=10.0, dmstep=1.0, numdms=5, nsub=8, ds=3, numout=1100)
    nds = 1000
    sub, out = OR.run_pass(obs, Opts(), raw, pp)           # default: first-DM running mean
    assert out.shape == (5, 1100)
    avg = 0.0
    for i, v in enumerate(out[0, :nds].tolist()):
        avg += (v - avg) / (i + 1.0)
    assert (out[:, nds:] == np.float32(avg)).all()
    _, outm = OR.run_pass(obs, Opts(pad_mode=0), raw, pp)
    for d in range(5):
        assert (outm[d, nds:] == np.float32(np.float64(outm[d, :nds]).sum() / nds)).all()
    _, outz = OR.run_pass(obs, Opts(pad_mode=1), raw, pp)
    assert np.array_equal(outz[:, :nds], out[:, :nds]) and not outz[:, nds:].any()
    off = OR.dm_offsets(obs, Opts(), 8, 3, 10.0, 1.0, 5)
    sub_np = _np_stage1(obs, Opts(), raw, 8, 3, 20.0)
    assert np.array_equal(sub_np, sub)
    assert np.array_equal(ON.stage2(sub_np, off, 1100, pad_mode=2), out)


@pytest.mark.parametrize("numint", [1, 7, 40, 333])
def test_stats_padvals_oracle_numpy_and_product(numint):
    """determine_padvals: oracle C, numpy twin and the library's host function agree."""
    rng = np.random.default_rng(numint)
    avg = rng.normal(100, 10, size=(numint, 48)).astype(np.float32)
    avg[rng.random(avg.shape) < 0.02] = 1e4                         # RFI intervals: trimmed away
    a = OR.stats_padvals(avg)
    b = ON.stats_padvals(avg)
    c = stats_padvals(avg)
    assert np.array_equal(a, b) and np.array_equal(a, c)
    if numint >= 40:
        assert np.abs(a - 100).max() < 10


# ---------------------------------------------------------------- known-answer tests
def test_kat_impulse_aligns_in_subband():
    """One impulse per channel at t0 + idispdt[c] -> every subband is cps*A at t0, 0 elsewhere."""
    obs = small_obs(nchan=64, N=2048)
    nsub, subdm, t0, A = 8, 500.0, 300, 7
    idd = OR.chan_delays(obs, nsub, subdm)
    raw = np.zeros((obs.N, obs.rowbytes), np.uint8)
    for c in range(obs.nchan):
        raw[t0 + idd[c], c] = A
    sub = OR.stage1(obs, Opts(**NOCLIP), raw, nsub, 1, subdm)
    assert (sub[:, t0] == (obs.nchan // nsub) * A).all()
    sub[:, t0] = 0
    assert not sub.any()


def test_kat_dispersed_pulse_peaks_at_its_dm():
    """A pulse dispersed by the stage-2 offsets of trial d* sums to nsub*A at t0 for d*."""
    obs = small_obs(nchan=960, N=8192)
    nsub, numdms = 96, 40
    off = OR.dm_offsets(obs, Opts(), nsub, 1, 100.0, 2.0, numdms)
    t0, A, dstar = 1000, 9, 23
    sub = np.zeros((nsub, obs.N), np.int16)
    for s in range(nsub):
        sub[s, t0 + off[dstar, s]] = A
    out = OR.stage2(sub, off)
    assert out[dstar, t0] == nsub * A
    assert out.max() == nsub * A
    assert (out[:, t0] <= nsub * A).all() and (out[np.arange(numdms) != dstar, t0] < nsub * A).all()


@pytest.mark.parametrize("ds_mode", [0, 1])
def test_kat_constant_input(ds_mode):
    """Constant level c0 in every channel -> subband cps*c0 (mean) or cps*ds*c0 (sum) away
    from the tail; stage 2 gives nsub times that wherever no read runs past the end.
    Clipping leaves a constant beam alone (its std is 0 and no point deviates)."""
    obs = small_obs(nchan=64, N=4096)
    c0, nsub, ds = 5, 8, 2
    raw = np.full((obs.N, obs.rowbytes), c0, np.uint8)
    opts = Opts(ds_mode=ds_mode)
    cl = OR.prepare(obs, opts, raw)
    assert cl.nclipped == 0 and (cl.pad == c0).all()
    sub = OR.stage1(obs, opts, raw, nsub, ds, 250.0, clean=cl)
    scale = 1 if ds_mode == 1 else ds
    assert (sub == (obs.nchan // nsub) * scale * c0).all()      # pads at the tail are c0 too
    off = OR.dm_offsets(obs, Opts(), nsub, ds, 0.0, 5.0, 10)
    out = OR.stage2(sub, off)
    lim = obs.N // ds - off.max()
    assert (out[:, :lim] == obs.nchan * scale * c0).all()


def test_kat_sub_input_offsets_equal_direct():
    """Stage 2 run from the .sub.inf values (lofreq/chanwidth/dt as read) gives the same
    offsets as the one-shot pass that wrote them."""
    obs = small_obs(nchan=960)
    opts = Opts()
    for ds in (1, 2, 3, 5, 6, 10):
        lof, bw, sdt = OR.sub_params(obs, opts, 96, ds)
        a = OR.dm_offsets(obs, opts, 96, ds, 443.2, 0.3, 76)
        b = OR.dm_offsets_sub(96, lof, bw, sdt, 443.2, 0.3, 76)
        assert np.array_equal(a, b)
