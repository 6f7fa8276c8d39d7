"""GPU single-pulse search (hd_single_pulse, csrc/hd_sp.hip) on the series a pass leaves in
HBM, against the oracle (oracle/sp_oracle.c + the script's candidate logic in oracle.py):
every bad block equal and the per-DM candidate lists (DM, bin, width and the sigma as a
bit-equal double) and .singlepulse files of hipdedisp.single_pulse identical to the
oracle's; the injected DM-350 pulse is found at its DM.  Reference: PALFA2_presto_search.py:539-546."""
import numpy as np
import pytest

import oracle as OR
from hipdedisp import Opts, PassParams, plan
from hipdedisp import single_pulse as SP
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def beam(engine):
    obs = palfa_obs(N=1 << 18, nbits=8)
    s = palfa_synth()
    s.sp_time[0] = 8.0                        # the DM-350 pulse inside this 17 s beam, at an
    s.sp_amp[0] = 1.0                         # amplitude the block-std rule does not flag bad
    engine.set_obs(obs, Opts())
    engine.synth_device(s)
    pts = rfifind_ptsperint(obs.dt)
    mask, pad = synth_mask(obs, s, pts)
    engine.set_mask(mask, pts, pad)
    yield obs, s
    engine.set_mask()


def run(engine, obs, subdm, lodm, dmstep, ds, numout=0):
    pp = PassParams(subdm=subdm, lodm=lodm, dmstep=dmstep, numdms=76, nsub=96, ds=ds, numout=numout)
    p = engine.plan(pp)
    p.run_subband()
    series = p.run_dedisp()
    return p, series


def check_pass(p, series, dm_strs, tmp_path, threshold=5.0):
    dt = p.sub_dt
    wl = SP.widths(dt, 0.1)
    assert wl == OR.sp_widths(dt, 0.1)
    got, bad = SP.device_candidates(p, dt, 0.1, threshold)
    raw, wbad = OR.sp_hits(series, wl, threshold)
    assert np.array_equal(bad, wbad)
    dms = [float(s) for s in dm_strs]
    ref = OR.sp_candidates(raw, wbad, wl, dms, dt, p.nds, p.numout, ls=series.shape[1] // 1000 * 1000 // 8000 * 8000)
    want = [(d, c.bin, c.downfact, c.sigma) for d, cl in enumerate(ref) for c in cl]
    have = [(r[0], r[1], wl[r[2]], r[4]) for r in got.tolist()]
    assert have == want                                          # sigma: bit-equal doubles
    # the files of PALFA2_presto_search.py:540-545
    base = str(tmp_path / "beam")
    secs, lists = SP.run_single_pulse(p, base, dm_strs, threshold=threshold)
    for s, r in zip(dm_strs, ref):
        text = open("%s_DM%s.singlepulse" % (base, s)).read()
        assert text == (SP.HEADER + "".join(str(c) for c in r) if r else "")
    return lists


def test_single_pulse_dm350_pass(engine, beam, tmp_path):
    """A full-resolution pass around the injected DM-350 pulse: device candidates = oracle
    candidates; the brightest candidate of the pass sits at DM 350."""
    obs, s = beam
    p, series = run(engine, obs, subdm=350.0, lodm=346.2, dmstep=0.1, ds=1)
    try:
        dm_strs = ["%.2f" % (346.2 + 0.1 * k) for k in range(76)]
        got = check_pass(p, series, dm_strs, tmp_path)
        best = max(((c.sigma, d) for d, cl in enumerate(got) for c in cl), default=(0, -1))
        assert best[0] > 8.0                                    # oracle on CPU: 10.8 at DM 350.0
        assert abs(float(dm_strs[best[1]]) - 350.0) <= 0.5
    finally:
        p.destroy()


@pytest.mark.parametrize("ds,numout_extra", [(2, 3000), (5, 0), (10, 1234)])
def test_single_pulse_downsampled_and_padded(engine, beam, tmp_path, ds, numout_extra):
    """Downsampled passes (fewer widths fit 0.1 s), padded series (border pruning and the
    constant padding: zero-std / bad blocks), bit-equal hits and identical lists."""
    obs, s = beam
    nds = obs.N // ds
    p, series = run(engine, obs, subdm=220.0, lodm=210.0, dmstep=0.3 * ds, ds=ds, numout=nds + numout_extra)
    try:
        dm_strs = ["%.2f" % (210.0 + 0.3 * ds * k) for k in range(76)]
        check_pass(p, series, dm_strs, tmp_path)
    finally:
        p.destroy()


@pytest.mark.parametrize("lodm,threshold", [(380.0, 5.0), (380.0, 3.0), (250.0, 3.0)])
def test_single_pulse_dense_runs(engine, beam, tmp_path, lodm, threshold):
    """ds-2 passes at DM 250-420, where the C2 beam's wide boxcars give dense, slowly varying
    runs of hits: the walk's true chain and the lanes' speculative chains run in step there
    without meeting for long stretches (csrc/hd_sp.hip), so most kept pivots come from the
    serial part -- lists identical to the oracle's, thresholds 5 and 3."""
    obs, s = beam
    ds = 2
    p, series = run(engine, obs, subdm=lodm + 10.0, lodm=lodm, dmstep=0.3, ds=ds)
    try:
        dm_strs = ["%.2f" % (lodm + 0.3 * k) for k in range(76)]
        check_pass(p, series, dm_strs, tmp_path, threshold=threshold)
    finally:
        p.destroy()


def test_single_pulse_many_hits_and_short_series(engine, beam, tmp_path):
    """A low threshold (many candidates, the 4.6-ms pulsar's train at DM 71) and a series
    shorter than one 8000-sample chunk (no candidates)."""
    obs, s = beam
    p, series = run(engine, obs, subdm=71.0, lodm=67.2, dmstep=0.1, ds=1)
    try:
        dm_strs = ["%.2f" % (67.2 + 0.1 * k) for k in range(76)]
        lists = check_pass(p, series, dm_strs, tmp_path, threshold=2.5)
        assert sum(len(c) for c in lists) > 1000
    finally:
        p.destroy()
    p, series = run(engine, obs, subdm=900.0, lodm=880.0, dmstep=1.0, ds=10, numout=6000)
    try:
        got, bad = SP.device_candidates(p, p.sub_dt, 0.1, 5.0)
        assert len(got) == 0 and bad.shape == (76, 6)
    finally:
        p.destroy()


def test_single_pulse_ties_constant_blocks_and_negatives(engine, beam, tmp_path):
    """Crafted subbands (hd_set_subbands) instead of the synthetic beam: small-integer noise
    (1000-sample blocks full of equal detrended values: the block-std sort's ties), a
    constant stretch (zero-std blocks), a stretch of negative values and a bright pulse --
    device bad blocks, hits and candidate lists equal to the oracle's, sigma bit-equal."""
    obs, s = beam
    pp = PassParams(subdm=4.0, lodm=0.2, dmstep=0.1, numdms=76, nsub=96, ds=1, numout=0)
    p = engine.plan(pp)
    try:
        rng = np.random.default_rng(11)
        nds = p.nds
        sub = rng.integers(0, 4, size=(96, nds)).astype(np.int16)
        sub[:, 20000:26000] = 3                                  # constant: zero-std blocks
        sub[:, 40000:48000] = rng.integers(-3, 1, size=(96, 8000)).astype(np.int16)
        sub[:, 100000:100040] += 6                               # a pulse at DM ~0
        sub[:, 150000:150600] += rng.integers(0, 3, size=(96, 600)).astype(np.int16)   # a wide hump
        p.set_subbands(sub)
        series = p.run_dedisp()
        dm_strs = ["%.2f" % (0.2 + 0.1 * k) for k in range(76)]
        lists = check_pass(p, series, dm_strs, tmp_path)
        assert sum(len(c) for c in lists) > 0
    finally:
        p.destroy()


def test_candidate_lists_end_to_end_clip_vs_noclip(engine):
    """North-star 'identical candidate lists' on two independent paths, end to end: the
    product (stage 1 + stage 2 on the GPU, then hd_single_pulse on the series still in HBM)
    against the oracle (the C prepsubband restatement's own series, then sp_oracle's search),
    for a low-DM pass of a beam with zero-DM spikes, once with clipping on (-clip 6, what the
    reference's commands leave on) and once with -noclip.  The two settings give different
    series, so the test also asserts the candidate lists follow them: without clipping the
    spikes make thousands of DM ~ 0 candidates that clip_times removes."""
    N = 1 << 18
    obs = palfa_obs(N=N, nbits=8)
    s = palfa_synth()
    raw = host_spectra(obs, s)
    pp = PassParams(subdm=3.8, lodm=0.0, dmstep=0.1, numdms=76, nsub=96, ds=1, numout=plan.choose_N(N))
    dms = [0.1 * i for i in range(76)]
    lists = {}
    for clip in (6.0, 0.0):
        opts = Opts(clip_sigma=clip)
        engine.set_obs(obs, opts)
        engine.synth_device(s)
        p = engine.plan(pp)
        try:
            p.run_subband()
            p.run_dedisp(to_host=False)
            dt = p.sub_dt
            wl = SP.widths(dt, 0.1)
            got, gbad = SP.device_candidates(p, dt, 0.1, 5.0)
            have = [(r[0], r[1], wl[r[2]], r[4]) for r in got.tolist()]
            nds, numout = p.nds, p.numout
        finally:
            p.destroy()
        _, series = OR.run_pass(obs, opts, raw, pp, omp=True)      # the oracle's own series
        hits, bad = OR.sp_hits(series, wl, 5.0)
        ref = OR.sp_candidates(hits, bad, wl, dms, dt, nds, numout, ls=series.shape[1] // 1000 * 1000 // 8000 * 8000)
        want = [(d, c.bin, c.downfact, c.sigma) for d, cl in enumerate(ref) for c in cl]
        assert np.array_equal(gbad, bad)
        assert have == want, "clip %g: device and oracle candidate lists differ" % clip
        lists[clip] = have
    low = {k: sum(1 for c in v if c[0] < 20) for k, v in lists.items()}     # DM < 2
    assert lists[6.0] != lists[0.0]
    assert low[0.0] > 10 * max(low[6.0], 1) and len(lists[0.0]) > 5 * len(lists[6.0])
    engine.set_obs(obs, Opts())


def test_single_pulse_launch_collect_pipelined(engine, beam):
    """hd_single_pulse_launch / _collect: the device searches of several passes queued before
    any host pruning (device_candidates_many) give each pass's one-shot candidates and bad
    blocks; a launch again before the collect replaces the pending search; a collect with
    too little room returns HD_E_NOMEM and stays collectable; a collect with nothing
    launched is refused."""
    import ctypes
    from hipdedisp import _lib
    from hipdedisp.engine import PrestoError
    obs, s = beam
    engine.set_obs(obs, Opts())                   # (an earlier test may have replaced the beam)
    engine.synth_device(s)
    specs = [(350.0, 346.2, 0.1, 1, 0), (220.0, 210.0, 0.6, 2, 0), (390.0, 380.0, 0.6, 2, 0),
             (71.0, 67.2, 0.1, 1, 0), (220.0, 210.0, 3.0, 10, (1 << 18) // 10 + 1234)]
    plans = []
    try:
        for subdm, lodm, dmstep, ds, numout in specs:
            p, _ = run(engine, obs, subdm, lodm, dmstep, ds, numout)
            plans.append(p)
        want = [SP.device_candidates(p, p.sub_dt, 0.1, 5.0) for p in plans]
        assert sum(len(w[0]) for w in want) > 100
        for depth in (1, 4, 8):
            got = list(SP.device_candidates_many(plans, 0.1, 5.0, depth=depth))
            assert [g[0] for g in got] == plans
            for (_, h, b), (wh, wb) in zip(got, want):
                assert np.array_equal(h, wh) and np.array_equal(b, wb)
        p = plans[0]
        SP._launch(p, p.sub_dt, 0.1, 3.0)                     # replaced before its collect
        SP._launch(p, p.sub_dt, 0.1, 5.0)
        h, b = SP._collect(p)
        assert np.array_equal(h, want[0][0]) and np.array_equal(b, want[0][1])
        SP._launch(p, p.sub_dt, 0.1, 5.0)
        small = np.empty(1, SP.HIT)
        n, nbk = ctypes.c_int64(), ctypes.c_int64()
        rc = engine._L.hd_single_pulse_collect(p._p, small.ctypes.data_as(ctypes.c_void_p), 1, ctypes.byref(n),
                                               None, ctypes.byref(nbk))
        assert rc == _lib.HD_E_NOMEM and n.value > 1
        h, b = SP._collect(p)                                   # still pending
        assert np.array_equal(h, want[0][0])
        with pytest.raises(PrestoError, match="no search launched"):
            SP._collect(p)
    finally:
        for p in plans:
            p.destroy()
