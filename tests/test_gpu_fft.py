"""GPU realfft / zapbirds / rednoise (hd_fft.hip) on the series a pass leaves in
HBM, against oracle/fft_oracle.py: the packed float32 hipFFT spectrum within a written
tolerance of numpy's float64 FFT of the same series (|dX| <= 1e-5 * sqrt(n) * std(x) +
3e-7 * |sum(x)|: float32 rounding over the butterfly stages, plus the twiddle rounding that
leaks ~eps * |DC| into every bin -- the series carry a large mean; the DC term within rtol
1e-5), then zapbirds and rednoise bit-exact against the oracle applied to the device's own
spectra (double powers and scales, no fused multiply-adds).  Reference: PALFA2_presto_search.py:548-558.  Parity with PRESTO unpinned."""
import numpy as np
import pytest

import fft_oracle as FO
from hipdedisp import Opts, PassParams, PrestoError
from hipdedisp import fft_stage as FS
from hipdedisp import plan as P
from hipdedisp.synth import palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask

pytestmark = pytest.mark.gpu

FFT_ATOL = 1e-5
DC_LEAK = 3e-7


@pytest.fixture(scope="module")
def beam(engine):
    obs = palfa_obs(N=1 << 18, nbits=8)
    s = palfa_synth()
    engine.set_obs(obs, Opts())
    engine.synth_device(s)
    pts = rfifind_ptsperint(obs.dt)
    mask, pad = synth_mask(obs, s, pts)
    engine.set_mask(mask, pts, pad)
    yield obs
    engine.set_mask()


def birds(T, nb):
    """Zaplist-style birdies: the 60 Hz mains comb, a wide one, two overlapping, one past
    the spectrum, one barycentric."""
    b = [(60.0 * k, 0.5, False) for k in range(1, 6)]
    b += [(3.3, 2.0, False), (17.0, 0.05, False), (17.02, 0.05, False), (nb / T + 5.0, 1.0, False),
          (29.946923, 0.02, True)]
    return b


@pytest.mark.parametrize("ds,numdms", [(1, 12), (3, 76)])
def test_fft_zap_rednoise_match_oracle(engine, beam, ds, numdms, tmp_path):
    obs = beam
    numout = P.choose_N(obs.N / ds)
    pp = PassParams(subdm=71.0, lodm=65.0, dmstep=0.5, numdms=numdms, nsub=96, ds=ds, numout=numout)
    p = engine.plan(pp)
    try:
        p.run_subband()
        x = p.run_dedisp()
        dt = p.sub_dt
        T = p.numout * dt
        FS.realfft(p)
        F0 = FS.spectra_complex(FS.get_fft(p))
        want = FO.realfft(x)
        xd = x.astype(np.float64)
        tol = (FFT_ATOL * np.sqrt(p.numout) * xd.std(axis=1) + DC_LEAK * np.abs(xd.sum(axis=1)))[:, None]
        err = np.abs(F0.astype(np.complex128) - want)
        assert np.all(err[:, 1:] <= tol), (err[:, 1:] / tol).max()
        np.testing.assert_allclose(F0[:, 0].real, want[:, 0].real, rtol=FFT_ATOL)   # DC: n * mean
        assert np.all(np.abs(F0[:, 0].imag - want[:, 0].imag) <= tol[:, 0])        # Nyquist
        # the 4.6 ms pulsar at DM 71 stands out at its fundamental
        k = int(round(T / 0.0046))
        pw = np.abs(want[:, k - 3:k + 4]) ** 2
        assert pw.max() > 20 * np.median(np.abs(want[:, 1000:20000]) ** 2)

        nb = p.numout // 2
        lo, hi = FS.birdie_bins(birds(T, nb), T, baryv=3e-5)
        FS.zapbirds(p, lo, hi)
        F1 = FS.spectra_complex(FS.get_fft(p))
        r = FS.zap_ranges(lo, hi, nb)
        assert len(r) >= 6
        assert np.array_equal(F1, FO.zap(F0, r))

        FS.rednoise(p, T)
        F2 = FS.spectra_complex(FS.get_fft(p))
        assert np.array_equal(F2, FO.rednoise(F1, FO.rednoise_blocks(nb, T)))
        pm = np.abs(F2[:, 1:].astype(np.complex128)) ** 2
        assert 0.8 < np.median(pm.mean(axis=1)) < 1.6   # roughly unit mean power after rednoise
    finally:
        p.destroy()


def test_zapbirds_palfa_zaplist_matches_oracle(engine, beam):
    """zapbirds with the reference's own zaplist (lib/zaplists/PALFA.zaplist, committed as
    tests/golden/palfa_zaplist.json): every one of its 221 birdies zapped on the device
    exactly as the oracle zaps the device's own spectrum."""
    import json
    import os
    g = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "palfa_zaplist.json")))
    birdies = [tuple(b) for b in g["birdies"]]
    pp = PassParams(subdm=71.0, lodm=65.0, dmstep=0.5, numdms=8, nsub=96, ds=1, numout=beam.N)
    p = engine.plan(pp)
    try:
        p.run_subband()
        p.run_dedisp(to_host=False)
        T = p.numout * p.sub_dt
        FS.realfft(p)
        F0 = FS.spectra_complex(FS.get_fft(p))
        nb = p.numout // 2
        lo, hi = FS.birdie_bins(birdies, T, baryv=0.0)
        r = FS.zap_ranges(lo, hi, nb)
        assert len(r) >= 20                          # the low-frequency families merge
        FS.zapbirds(p, lo, hi)
        F1 = FS.spectra_complex(FS.get_fft(p))
        assert np.array_equal(F1, FO.zap(F0, r))
        assert not np.array_equal(F1, F0)
    finally:
        p.destroy()


def test_run_fft_writes_packed_files(engine, beam, tmp_path):
    obs = beam
    d = P.ddplans_for("pdev")[1]
    pp = PassParams(subdm=float(d.subdmlist[0]), lodm=float(d.lodm_arg(0)), dmstep=float(d.dmstep_arg()),
                    numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                    numout=P.choose_N(obs.N / d.downsamp))
    p = engine.plan(pp)
    try:
        p.run_subband()
        p.run_dedisp(to_host=False)
        zl = tmp_path / "t.zaplist"
        zl.write_text("# Freq Width\n60.0 0.5\n120.0 0.5\nB 29.946923 0.02\n")
        dms = ["%.2f" % (pp.lodm + i * pp.dmstep) for i in range(pp.numdms)]
        base = str(tmp_path / "beam")
        t = FS.run_fft(p, p.sub_dt, FS.read_zaplist(str(zl)), 1e-4, base, dms, write=True)
        assert t > 0
        spec = FS.get_fft(p)
        for i in (0, pp.numdms - 1):
            got = np.fromfile("%s_DM%s.fft" % (base, dms[i]), np.float32)
            assert got.size == p.numout and np.array_equal(got, spec[i])
        assert spec[0, 0] == 1.0 and spec[0, 1] == 0.0
    finally:
        p.destroy()


def test_fft_state_errors(engine, beam):
    pp = PassParams(subdm=71.0, lodm=65.0, dmstep=0.5, numdms=4, nsub=96, ds=2, numout=P.choose_N(beam.N / 2))
    p = engine.plan(pp)
    try:
        with pytest.raises(PrestoError):
            FS.realfft(p)                        # before hd_run_dedisp
        with pytest.raises(PrestoError):
            FS.rednoise(p, 10.0)                 # before hd_realfft
        p.run_subband()
        p.run_dedisp(to_host=False)
        FS.realfft(p)
        with pytest.raises(PrestoError):
            FS.rednoise(p, 10.0, endwidth=300)   # blocks wider than a wave's 128
        with pytest.raises(PrestoError):
            FS.get_fft(p, 3, 2)
    finally:
        p.destroy()


def test_fft_state_shared_per_geometry(engine, beam):
    """Two passes of one geometry share the context's hipFFT plan and spectra buffer: the
    second hd_realfft takes it over, the first plan's spectra calls then fail loudly."""
    mk = lambda sd: PassParams(subdm=sd, lodm=sd - 5.0, dmstep=0.5, numdms=8, nsub=96, ds=3,
                               numout=P.choose_N(beam.N / 3))
    p1, p2 = engine.plan(mk(71.0)), engine.plan(mk(90.0))
    try:
        for p in (p1, p2):
            p.run_subband()
            p.run_dedisp(to_host=False)
        FS.realfft(p1)
        a = FS.get_fft(p1)
        FS.realfft(p2)
        with pytest.raises(PrestoError):
            FS.get_fft(p1)
        with pytest.raises(PrestoError):
            FS.rednoise(p1, 10.0)
        b = FS.get_fft(p2)
        assert not np.array_equal(a, b)
        FS.realfft(p1)                                    # and back
        assert np.array_equal(FS.get_fft(p1), a)
    finally:
        p1.destroy()
        p2.destroy()
