"""Pin the CPU oracle: C restatement vs the independent numpy restatement (bit for bit),
plus analytic known-answer tests.  (PRESTO is absent, so against PRESTO itself the oracle
is parity-unpinned; see oracle/oracle.h and DESIGN.md §Oracle.)"""
import numpy as np
import pytest

import oracle as OR
import oracle_np as ON
from hipdedisp import Opts, PassParams
from hipdedisp.synth import palfa_obs


def small_obs(nchan=64, N=4096, nbits=8, flip=False):
    return palfa_obs(N=N, nbits=nbits, nchan=nchan, nsblk=256, flip=flip)


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


def _rand_case(rng, nbits, nchan=64, N=2048, flip=False):
    obs = small_obs(nchan=nchan, N=N, nbits=nbits, flip=flip)
    raw = rng.integers(0, 256, size=(N, obs.rowbytes), dtype=np.uint8)
    if nbits == 16:   # keep 16-bit values moderate so int16 subbands do not saturate everywhere
        v = rng.integers(-300, 300, size=(N, nchan)).astype(">i2")
        raw = v.view(np.uint8).reshape(N, obs.rowbytes)
    return obs, raw


@pytest.mark.parametrize("nbits", [4, 8, 16])
@pytest.mark.parametrize("flip", [False, True])
@pytest.mark.parametrize("ds", [1, 3])
def test_stage1_c_vs_numpy(nbits, flip, ds):
    rng = np.random.default_rng(nbits * 10 + ds + flip)
    obs, raw = _rand_case(rng, nbits, flip=flip)
    idd = OR.chan_delays(obs, 8, 150.0)
    a = OR.stage1(obs, Opts(), raw, 8, ds, 150.0)
    b = ON.stage1(raw, obs.nchan, nbits, flip, 8, ds, idd)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("sub_dtype,ds_mode", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_stage1_calib_mask_c_vs_numpy(sub_dtype, ds_mode):
    rng = np.random.default_rng(5 + sub_dtype + 2 * ds_mode)
    obs, raw = _rand_case(rng, 8, flip=True)
    nc = obs.nchan
    scl = rng.uniform(0.5, 2.0, nc).astype(np.float32)
    offs = rng.uniform(-10, 10, nc).astype(np.float32)
    wts = (rng.random(nc) > 0.1).astype(np.float32)
    pts = 256
    mask = (rng.random((obs.N // pts + 1, nc)) < 0.1).astype(np.uint8)
    pad = rng.uniform(50, 150, nc).astype(np.float32)
    idd = OR.chan_delays(obs, 8, 400.0)
    opts = Opts(sub_dtype=sub_dtype, ds_mode=ds_mode)
    a = OR.stage1(obs, opts, raw, 8, 2, 400.0, calib=(scl, offs, wts), mask=mask, ptsperint=pts, padvals=pad)
    b = ON.stage1(raw, nc, 8, True, 8, 2, idd, scl, offs, wts, mask, pts, pad, sub_dtype, ds_mode)
    assert np.array_equal(a, b)


def test_stage1_window_equals_full():
    """or_stage1 over [t0, t0+count) equals the same columns of the full run (bounded sampling)."""
    rng = np.random.default_rng(3)
    obs, raw = _rand_case(rng, 8, N=4096)
    full = OR.stage1(obs, Opts(), raw, 8, 2, 300.0)
    win = OR.stage1(obs, Opts(), raw, 8, 2, 300.0, t0=700, count=900)
    assert np.array_equal(full[:, 700:1600], win)
    omp = OR.stage1(obs, Opts(), raw, 8, 2, 300.0, omp=True)
    assert np.array_equal(full, omp)


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


def test_run_pass_padding_mean_and_zero():
    rng = np.random.default_rng(2)
    obs, raw = _rand_case(rng, 8, N=3000)
    pp = PassParams(subdm=20.0, lodm=10.0, dmstep=1.0, numdms=5, nsub=8, ds=3, numout=1100)
    sub, out = OR.run_pass(obs, Opts(), raw, pp)
    nds = 1000
    assert out.shape == (5, 1100)
    for d in range(5):
        assert (out[d, nds:] == np.float32(np.float64(out[d, :nds]).sum() / nds)).all()
    _, outz = OR.run_pass(obs, Opts(pad_mode=1), raw, pp)
    assert np.array_equal(outz[:, :nds], out[:, :nds]) and not outz[:, nds:].any()
    idd = OR.chan_delays(obs, 8, 20.0)
    off = OR.dm_offsets(obs, Opts(), 8, 3, 10.0, 1.0, 5)
    nsub_np = ON.stage1(raw, obs.nchan, 8, False, 8, 3, idd)
    assert np.array_equal(ON.stage2(nsub_np, off, 1100), out)


# ---------------------------------------------------------------- known-answer tests
def test_kat_impulse_aligns_in_subband():
    """One impulse per channel at t0 + idispdt[c] -> every subband is cps*A at t0, 0 elsewhere."""
    obs = small_obs(nchan=64, N=2048)
    nsub, subdm, t0, A = 8, 500.0, 300, 7
    idd = OR.chan_delays(obs, nsub, subdm)
    raw = np.zeros((obs.N, obs.rowbytes), np.uint8)
    for c in range(obs.nchan):
        raw[t0 + idd[c], c] = A
    sub = OR.stage1(obs, Opts(), raw, nsub, 1, subdm)
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


def test_kat_constant_input():
    """Constant level c0 in every channel -> subband cps*ds*c0 away from the tail; stage 2
    gives nsub times that wherever no read runs past the end."""
    obs = small_obs(nchan=64, N=4096)
    c0, nsub, ds = 5, 8, 2
    raw = np.full((obs.N, obs.rowbytes), c0, np.uint8)
    sub = OR.stage1(obs, Opts(), raw, nsub, ds, 250.0)
    maxd = OR.chan_delays(obs, nsub, 250.0).max()
    good = (obs.N - maxd) // ds - 1
    assert (sub[:, :good] == (obs.nchan // nsub) * ds * c0).all()
    off = OR.dm_offsets(obs, Opts(), nsub, ds, 0.0, 5.0, 10)
    out = OR.stage2(sub, off)
    lim = good - off.max()
    assert (out[:, :lim] == obs.nchan * ds * c0).all()


def test_kat_sub_input_offsets_equal_direct():
    """Stage 2 run from the .sub.inf values (lofreq/chanwid/dt as read) gives the same
    offsets as the one-shot pass that wrote them."""
    obs = small_obs(nchan=960)
    opts = Opts()
    for ds in (1, 2, 3, 5, 6, 10):
        lof, bw, sdt = OR.sub_params(obs, opts, 96, ds)
        a = OR.dm_offsets(obs, opts, 96, ds, 443.2, 0.3, 76)
        b = OR.dm_offsets_sub(96, lof, bw, sdt, 443.2, 0.3, 76)
        assert np.array_equal(a, b)
