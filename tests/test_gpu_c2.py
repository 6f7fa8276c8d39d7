"""Config 2 at full size (BASELINE.json configs[1]): the bench workload -- a PALFA Mock beam of
960 channels x 2^22 spectra x 8 bits (a 4.03 GB raw block), the full 57-pass Mock DDplan
(4188 DM trials), an rfifind-style mask, clipping on -- through the HIP path, checked
against the oracle:

* the device clip_times state of the whole beam (pad rows, clip flags, block zap rows);
* for every pass, sampled windows of the subbands and of the series, bit-exact: t = 0, the
  outputs whose raw reads cross byte offset 2^31 of the raw block (spectrum 2,236,963;
  signed 32-bit offsets would wrap there), and the last samples before N/ds;
* the padded tail of every padded pass (the first DM's mean, within the 1e-5 bound);
* two passes compared over their full length (stage 0 pass 0, stage 5);
* the injected DM-350 single pulse and the 4.6 ms pulsar at DM 71 recovered.
"""
import numpy as np
import pytest

import oracle as OR
from hipdedisp import Opts, PassParams, plan
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

N = 1 << 22
W = 4096                       # window length (output samples)
OFF31 = (1 << 31) // 960 + 1   # first spectrum starting past byte 2^31 of the raw block


def pass_params(d, i):
    return PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                      numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp, numout=plan.choose_N(N / d.downsamp))


def windows(nds, ds, maxd):
    """Window starts: t = 0; outputs whose reads cross spectrum OFF31; the end of the data."""
    hi = max(0, (OFF31 - maxd) // ds - W // 2)
    return [0, min(hi, nds - W), nds - W]


@pytest.fixture(scope="module")
def c2(engine):
    obs = palfa_obs(N=N, nbits=8)
    s = palfa_synth()
    engine.set_obs(obs, Opts())
    engine.synth_device(s)
    raw = host_spectra(obs, s)
    pts = rfifind_ptsperint(obs.dt)
    mask, pad = synth_mask(obs, s, pts)
    engine.set_mask(mask, pts, pad)
    cl = OR.prepare(obs, Opts(), raw, mask=mask, ptsperint=pts, padvals=pad, omp=True)
    yield obs, s, raw, cl
    engine.set_mask()


def test_c2_clean_state(engine, c2):
    obs, s, raw, cl = c2
    gpad, gclip, gzap, ncl = engine.get_clean()
    assert ncl == cl.nclipped > 1000          # the beam's zero-DM spikes
    assert np.array_equal(gclip, cl.clipped)
    assert np.array_equal(gzap, cl.zap)
    assert np.array_equal(gpad, cl.pad)


@pytest.mark.parametrize("stage", [0, 1, 2, 3, 4, 5])
def test_c2_stage_windows_bitexact(engine, c2, stage):
    obs, s, raw, cl = c2
    d = plan.ddplans_for("pdev")[stage]
    pps = [pass_params(d, i) for i in range(d.numpasses)]
    plans = [engine.plan(pp) for pp in pps]
    try:
        engine.run_subband_multi(plans)
        engine.run_dedisp_multi(plans)                       # the bench's path: one launch per stage
        for pp, p in zip(pps, plans):
            idd, off = p.delays()
            nds = N // pp.ds
            maxoff = int(off.max())
            for t0 in windows(nds, pp.ds, int(idd.max())):
                cnt = min(W + maxoff, nds - t0)
                want_sub = OR.stage1(obs, Opts(), raw, pp.nsub, pp.ds, pp.subdm, t0=t0, count=cnt, clean=cl, omp=True)
                got_sub = p.get_subbands_window(t0, cnt)
                assert np.array_equal(got_sub, want_sub), (pp.subdm, t0)
                want = OR.stage2(want_sub, off, 0, W, omp=True)      # reads past nds are 0, as in the engine
                got = p.get_series(0, pp.numdms, t0, W)
                assert np.array_equal(got, want), (pp.subdm, t0)
            if pp.numout > nds:                                    # padded: the first DM's running mean
                dm0 = p.get_series(0, 1, 0, pp.numout)
                ref = OR.pad_series(dm0.copy(), nds, 2)[0, nds]
                tail = p.get_series(0, pp.numdms, nds, pp.numout - nds)
                assert (tail == tail[0, 0]).all()
                np.testing.assert_allclose(tail[0, 0], ref, rtol=1e-5, atol=0)
    finally:
        for p in plans:
            p.destroy()


@pytest.mark.parametrize("stage,passnum", [(0, 0), (5, 0)])
def test_c2_full_pass_bitexact(engine, c2, stage, passnum):
    obs, s, raw, cl = c2
    pp = pass_params(plan.ddplans_for("pdev")[stage], passnum)
    p = engine.plan(pp)
    try:
        p.run_subband()
        got_sub = p.get_subbands()
        got = p.run_dedisp()
        want_sub, want = OR.run_pass(obs, Opts(), raw, pp, clean=cl, omp=True)
        assert np.array_equal(got_sub, want_sub)
        nds = N // pp.ds
        assert np.array_equal(got[:, :nds], want[:, :nds])
        np.testing.assert_allclose(got[:, nds:], want[:, nds:], rtol=1e-5, atol=0)
    finally:
        p.destroy()


def test_c2_injected_sources_recovered(engine, c2):
    obs, s, raw, cl = c2
    ps = plan.ddplans_for("pdev")
    # the DM-350 single pulse: stage 1 (ds 2), the pass whose DMs cover 350
    d = ps[1]
    k = next(i for i in range(d.numpasses) if float(d.dmlist[i][0]) <= 350.0 <= float(d.dmlist[i][-1]))
    pp = pass_params(d, k)
    p = engine.plan(pp)
    try:
        p.run_subband()
        p.run_dedisp(to_host=False)
        tp = int(round(s.sp_time[0] / (obs.dt * pp.ds)))
        win = p.get_series(0, pp.numdms, tp - 4000, 8000).astype(np.float64)
    finally:
        p.destroy()
    med = np.median(win, axis=1, keepdims=True)
    mad = 1.4826 * np.median(np.abs(win - med), axis=1, keepdims=True)
    z = (win - med) / mad
    dd, tt = np.unravel_index(np.argmax(z), z.shape)
    assert abs(float(d.dmlist[k][dd]) - 350.0) <= 1.0
    assert abs(tt - 4000) <= 2 + int(s.sp_width[0] / (obs.dt * pp.ds))
    assert z[dd, tt] > 8.0
    # the 4.6 ms pulsar: periodicity at its fundamental, strong at DM 71, washed out at DM 0
    d = ps[0]
    k = next(i for i in range(d.numpasses) if float(d.dmlist[i][0]) <= 71.0 <= float(d.dmlist[i][-1]))
    j = d.dmlist[k].index("71.00")
    pows = []
    for kk, jj in ((k, j), (0, 0)):
        p = engine.plan(pass_params(d, kk))
        try:
            p.run_subband()
            p.run_dedisp(to_host=False)
            x = p.get_series(jj, 1, 0, N)[0].astype(np.float64)
        finally:
            p.destroy()
        f = np.abs(np.fft.rfft(x - x.mean())) ** 2
        b = int(round(N * obs.dt / s.psr_period[0]))
        pows.append(f[b - 2:b + 3].max() / np.median(f[b - 2000:b + 2000]))
    assert pows[0] > 50.0 and pows[0] > 10.0 * pows[1]
