"""Config 4 at full size (BASELINE.json configs[3]): the DDplan2b plan from 0 to 10000 pc cm^-3
(PALFA2_presto_search.py:305-317 -> DDplan2b.py:197-267; 7 steps, 93 passes, downsampling 1..64,
76 / 64 DMs per pass) on a PALFA Mock beam of 960 channels x 2^22 spectra x 8 bits with an
rfifind-style mask and clipping on, every step through the bench's path (run_subband_multi:
one stage-1 launch per step; run_dedisp_multi: one stage-2 launch per step), checked against
the oracle:

* every pass of every step, sampled windows of the subbands and of the series bit-exact: t = 0,
  the outputs whose raw reads cross byte 2^31 of the raw block, and the last samples before
  N/ds (at ds 64 the DM-10000 sweep spans ~2500 output samples, so the windows there read far
  past the window start);
* the padded tail of every padded pass (the first DM's mean, within the 1e-5 bound);
* the highest-DM pass of the last step (DM ~10090, ds 64) over its full length.
"""
import numpy as np
import pytest

import oracle as OR
from hipdedisp import Opts, PassParams, plan
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(1200)]

N = 1 << 22
W = 4096                       # window length (output samples)
OFF31 = (1 << 31) // 960 + 1   # first spectrum starting past byte 2^31 of the raw block


def steps(obs):
    return plan.ddplan2b_plans(obs.dt, 1375.5, 322.6, obs.nchan, 2048, 0.0, 10000.0, 96, 0.1)


def pass_params(d, i):
    return PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                      numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp, numout=plan.choose_N(N / d.downsamp))


def windows(nds, ds, maxd):
    """Window starts: t = 0; outputs whose reads cross spectrum OFF31; the end of the data."""
    hi = max(0, (OFF31 - maxd) // ds - W // 2)
    return sorted({0, min(hi, nds - W), nds - W})


@pytest.fixture(scope="module")
def c4(engine):
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


def test_c4_plan_shape():
    obs = palfa_obs(N=N, nbits=8)
    st = steps(obs)
    assert [d.downsamp for d in st] == [1, 2, 4, 8, 16, 32, 64]
    assert sum(d.numpasses for d in st) == 93
    assert float(st[-1].dmlist[-1][-1]) >= 10000.0


@pytest.mark.parametrize("step", range(7))
def test_c4_step_windows_bitexact(engine, c4, step):
    obs, s, raw, cl = c4
    d = steps(obs)[step]
    pps = [pass_params(d, i) for i in range(d.numpasses)]
    plans = [engine.plan(pp) for pp in pps]
    try:
        engine.run_subband_multi(plans)
        engine.run_dedisp_multi(plans)
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


def test_c4_dm10000_pass_full(engine, c4):
    """The highest-DM pass of the plan (ds 64, DMs up to ~10090) over its full length."""
    obs, s, raw, cl = c4
    d = steps(obs)[-1]
    pp = pass_params(d, d.numpasses - 1)
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
