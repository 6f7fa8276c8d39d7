"""CPU checks of the rfifind row: the oracle's reading of the raw block
(decode + clip_times replacements) equals the C oracle's stage-1 channel values, its
statistics agree with a plain float64 numpy restatement, and hipdedisp.rfifind's mask
decisions equal the oracle's independent restatement on the same statistics.  Parity with
PRESTO's rfifind is unpinned (it is not in this image)."""
import math

import numpy as np
import pytest

import oracle as OR
import rfifind_oracle as RO
from hipdedisp import Opts
from hipdedisp import rfifind as RF
from hipdedisp.formats.mask import RfiMask, read_mask, write_mask
from hipdedisp.synth import palfa_obs


def spiky_raw(obs, seed=3, nspike=12):
    rng = np.random.default_rng(seed)
    raw = rng.integers(0, 256 if obs.nbits == 8 else 1 << 16, size=(obs.N, obs.rowbytes)).astype(np.uint8)
    if obs.nbits == 8:
        raw = rng.binomial(40, 0.5, size=(obs.N, obs.rowbytes)).astype(np.uint8) + 60
        raw[rng.integers(0, obs.N, nspike)] = 250
    elif obs.nbits == 4:
        lo = rng.binomial(10, 0.5, size=(obs.N, obs.rowbytes))
        hi = rng.binomial(10, 0.5, size=(obs.N, obs.rowbytes))
        raw = (lo | (hi << 4)).astype(np.uint8)
        raw[rng.integers(0, obs.N, nspike)] = 0xff
    return raw


@pytest.mark.parametrize("nbits,flip,hi_first", [(8, True, True), (8, False, True), (4, True, True),
                                                 (4, False, False), (16, True, True)])
def test_samples_equal_c_oracle_channels(nbits, flip, hi_first):
    """nsub = nchan, ds 1, subdm 0, float subbands: the C oracle's stage 1 is the cleaned
    channel values, which the rfifind oracle's samples() must reproduce exactly."""
    obs = palfa_obs(N=4096, nbits=nbits, nchan=64, nsblk=512, flip=flip)
    opts = Opts(nibble_hi_first=hi_first, sub_dtype=1)
    raw = spiky_raw(obs)
    cl = OR.prepare(obs, opts, raw)
    if nbits != 16:
        assert cl.nclipped > 0
    x = RO.samples(obs, opts, raw, cl)
    sub = OR.stage1(obs, opts, raw, obs.nchan, 1, 0.0, clean=cl)
    assert np.array_equal(sub.T, x)


def test_stats_match_numpy():
    rng = np.random.default_rng(5)
    x = rng.normal(100.0, 7.0, size=(3 * 1024, 16)).astype(np.float32)
    x[1024:2048, 3] += 20.0 * np.sin(2 * np.pi * 37 * np.arange(1024) / 1024).astype(np.float32)
    avg, std, pw = RO.stats(x, 1024)
    b = x.astype(np.float64).reshape(3, 1024, 16)
    assert np.allclose(avg, b.mean(axis=1), rtol=1e-6)
    assert np.allclose(std, b.std(axis=1, ddof=1), rtol=1e-6)
    f = np.abs(np.fft.rfft(b, axis=1)[:, 1:512]) ** 2 / (1024 * b.var(axis=1, ddof=1))[:, None, :]
    assert np.allclose(pw, f.max(axis=1), rtol=1e-5)
    assert pw[1, 3] > 300 and np.argmax(pw[:, 3]) == 1


def test_power_for_sigma():
    assert RF.power_for_sigma(4.0, 1) == pytest.approx(-math.log(0.5 * math.erfc(4.0 / math.sqrt(2))))
    # exp(-P) is the single-bin chance: P(4 sigma, 4096 bins) gives 4096 * exp(-P) = tail(4)
    p = RF.power_for_sigma(4.0, 4096)
    assert 4096 * math.exp(-p) == pytest.approx(0.5 * math.erfc(4.0 / math.sqrt(2)), rel=1e-12)


def test_calc_avgmedstd():
    a = np.array([5, 1, 9, 3, 7, 2, 8, 4, 6, 100], np.float32)
    avg, med, sd = RF.calc_avgmedstd(a, 0.8)
    mid = np.sort(a)[1:9].astype(np.float64)
    assert avg == pytest.approx(mid.mean()) and sd == pytest.approx(mid.std(ddof=1), rel=1e-6)
    assert med == np.sort(a)[5]


def _stats_with_rfi(seed, numint=24, nchan=96, pts=4096):
    rng = np.random.default_rng(seed)
    avg = rng.normal(100, 0.5, (numint, nchan)).astype(np.float32)
    std = rng.normal(10, 0.1, (numint, nchan)).astype(np.float32)
    pw = rng.exponential(1.0, (numint, nchan)).astype(np.float32) + 8.0
    avg[:, 7] += 30.0                                  # persistent channel: zapped whole
    std[rng.random((numint, nchan)) < 0.03] *= 3.0     # scattered bad cells
    pw[:, 40][rng.random(numint) < 0.8] = 60.0         # periodic RFI in one channel
    avg[5, :] += rng.normal(0, 20, nchan).astype(np.float32)   # broadband burst: interval zapped
    return avg, std, pw, pts


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_mask_decisions_match_oracle(seed):
    avg, std, pw, pts = _stats_with_rfi(seed)
    bitmap, zapint, zap_chans, bm = RF.make_mask(avg, std, pw, pts)
    want_bitmap, want_zapint = RO.mask(avg, std, pw, pts)
    assert np.array_equal(bitmap, want_bitmap)
    assert np.array_equal(zapint, want_zapint)
    assert 7 in zap_chans and 40 in zap_chans and zapint[5]
    assert np.all(bitmap[bm != 0])


def test_mask_file_round_trip(tmp_path):
    avg, std, pw, pts = _stats_with_rfi(4)
    bitmap, zapint, zap_chans, _ = RF.make_mask(avg, std, pw, pts)
    m = RfiMask(10.0, 4.0, 55000.5, pts * 6.5476e-5, 1214.0, 0.33, 96, 24, pts, bitmap, zapint, zap_chans)
    fn = str(tmp_path / "b_rfifind.mask")
    write_mask(fn, m)
    r = read_mask(fn)
    assert np.array_equal(r.bitmap, bitmap) and np.array_equal(r.zapint, zapint)
    assert np.array_equal(np.sort(r.zap_chans), zap_chans)


def test_ptsperint_for():
    dt = 65.476e-6
    assert RF.ptsperint_for(dt, 2 ** 15 * 64e-6, 64) == 32000
    assert RF.ptsperint_for(dt, 2 ** 15 * 64e-6, 2048) == 32768
    assert RF.ptsperint_for(dt, 1e-3, 2048) == 2048
