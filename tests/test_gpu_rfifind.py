"""GPU rfifind statistics (hd_rfifind_stats) against oracle/rfifind_oracle.py on
the same synthetic beam: per (interval, channel) mean and std bit-exact (double sums in the
kernel's lane order), the largest normalised FFT power within rtol 1e-4 (hipFFT float32 vs
numpy float64: the power is a float quantity, the tolerance is written here), and the mask
made from the device statistics equal to the oracle's mask from its own statistics except
for cells whose power lies within that tolerance of the threshold.  Parity with PRESTO's
rfifind itself is unpinned (not in this image)."""
import numpy as np
import pytest

import oracle as OR
import rfifind_oracle as RO
from hipdedisp import Opts, PrestoError
from hipdedisp import rfifind as RF
from hipdedisp.formats.mask import mask_padvals, read_mask, read_stats
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth, synth_mask

pytestmark = pytest.mark.gpu

POW_RTOL = 1e-4


def beam(engine, obs, opts, seed=0):
    s = palfa_synth(beam=seed, nbits=obs.nbits)
    s.spike_frac = 0.002
    s.spike_amp = 6.0
    engine.set_obs(obs, opts)
    engine.synth_device(s)
    engine.set_mask()
    return s, host_spectra(obs, s)


def oracle_stats(obs, opts, raw, pts):
    cl = OR.prepare(obs, opts, raw, omp=True)
    return RO.stats(RO.samples(obs, opts, raw, cl), pts), cl


def check_masks(dev, want, pts):
    """Masks from device vs oracle statistics: any difference only where a power is within
    POW_RTOL of the rejection threshold."""
    bm, zi, _, _ = RF.make_mask(*dev, pts)
    wb, wz = RO.mask(*want, pts)
    if np.array_equal(bm, wb) and np.array_equal(zi, wz):
        return bm
    reject = RF.power_for_sigma(4.0, pts // 2)
    near = np.abs(want[2] - reject) <= POW_RTOL * reject
    assert near.any(), "masks differ away from the power threshold"
    return bm


@pytest.mark.parametrize("nbits,flip,hi_first,pts,nint", [(8, True, True, 2048, 18), (8, False, True, 2000, 3),
                                                          (4, True, False, 2048, 5), (16, True, True, 1024, 3)])
def test_rfifind_stats_match_oracle(engine, nbits, flip, hi_first, pts, nint):
    """18 intervals cover a full 16-interval batch plus a tail batch; 2000 is not a multiple
    of the wave width; 4-bit reads the unpacked channel-major copy, 16-bit the generic decode."""
    obs = palfa_obs(N=nint * pts + 333, nbits=nbits, nsblk=512, flip=flip)
    opts = Opts(nibble_hi_first=hi_first)
    _, raw = beam(engine, obs, opts)
    avg, std, pw = RF.device_stats(engine, pts)
    (wa, ws, wp), cl = oracle_stats(obs, opts, raw, pts)
    if nbits != 16:
        assert cl.nclipped > 0
    assert avg.shape == (nint, obs.nchan)
    assert np.array_equal(avg, wa)
    assert np.array_equal(std, ws)
    assert np.allclose(pw, wp, rtol=POW_RTOL, atol=1e-3)
    bm = check_masks((avg, std, pw), (wa, ws, wp), pts)
    assert bm.any()


def test_rfifind_writes_mask_and_stats(engine, tmp_path):
    """rfifind() writes <base>_rfifind.mask/.stats from the device statistics; read back they
    are the device arrays and the mask decisions; the mask then loads into the engine with
    the .stats pad values, as stage 1's -mask does (PALFA2_presto_search.py:506)."""
    obs = palfa_obs(N=6 * 4096 + 100, nbits=8, nsblk=2048)
    _, raw = beam(engine, obs, Opts(), seed=1)
    base = str(tmp_path / "beam")
    chunk = 4096 * obs.dt
    maskfn, m, st = RF.rfifind(engine, base, chunk, 2048, mjd=55000.25)
    assert maskfn == base + "_rfifind.mask" and m.ptsperint == 4096 and m.numint == 6
    r = read_mask(maskfn)
    s = read_stats(base + "_rfifind.stats")
    avg, std, pw = RF.device_stats(engine, 4096)
    assert np.array_equal(s.dataavg, avg) and np.array_equal(s.datastd, std) and np.array_equal(s.datapow, pw)
    bm, zi, _, _ = RF.make_mask(avg, std, pw, 4096)
    assert np.array_equal(r.bitmap, bm) and np.array_equal(r.zapint, zi)
    assert r.mjd == 55000.25 and r.numchan == obs.nchan
    engine.set_rfimask(r, mask_padvals(maskfn, obs.nchan))
    try:
        with pytest.raises(PrestoError):         # rfifind reads the data before any mask
            RF.device_stats(engine, 4096)
    finally:
        engine.set_mask()


def test_rfifind_rejects_bad_interval(engine):
    obs = palfa_obs(N=8192, nbits=8, nsblk=2048)
    beam(engine, obs, Opts())
    for pts in (3, 2047, 16384):
        with pytest.raises(PrestoError):
            RF.device_stats(engine, pts)
