"""Barycentric output (prepsubband without -nobary; reference PALFA2_presto_search.py:514-520):
the add/remove-bin list from a TEMPO table and the barycentred series.

Parity unpinned: PRESTO (prepsubband's barycentring) and TEMPO are not in the reference or the
image, so the library's hd_bary_diffbins is checked against the oracle's literal restatement
(oracle.bary_diffbins) on synthetic TEMPO tables, and the device's barycentred series against
the oracle's sample-by-sample output loop (oracle.bary_series) applied to the same plan's
topocentric series.  Bar: bit-exact (the diffbins are integers; the series are copies and the
padding value, exact mean of integer-valued samples cast to f32)."""
import numpy as np
import pytest

import oracle as OR
from hipdedisp import Opts, PassParams, PrestoError
from hipdedisp.engine import bary_diffbins

MJD0 = 55000.25


def tempo_table(T, tdt, v, acc=0.0, amp=0.0, per=1e9, r0=0.0):
    """Synthetic TEMPO table: topocentric MJDs every tdt s over T (+ margin) and barycentric
    ones offset by r0 + v*t + acc*t^2/2 + amp*sin(2 pi t / per) seconds."""
    n = int(T * 1.1 / tdt + 5.5) + 1
    t = np.arange(n, dtype=np.float64) * tdt
    topo = MJD0 + t / 86400.0
    dly = r0 + v * t + 0.5 * acc * t * t + amp * np.sin(2 * np.pi * t / per)
    return topo, topo + dly / 86400.0


TABLES = [
    dict(v=1.0e-4),                         # Earth-like: ~bins added steadily
    dict(v=-0.8e-4, acc=3e-8),              # bins removed
    dict(v=2e-4, amp=3e-3, per=80.0),       # non-monotone: adds and removes
    dict(v=0.0),                            # nothing to do
    dict(v=3e-6, r0=480.0),                 # a large constant Roemer delay cancels
]


@pytest.mark.parametrize("k", range(len(TABLES)))
@pytest.mark.parametrize("dsdt", [65.476e-6, 2 * 65.476e-6, 10 * 65.476e-6])
def test_diffbins_match_oracle(k, dsdt):
    topo, bary = tempo_table(268.0, 10.0, **TABLES[k])
    got = bary_diffbins(topo, bary, 10.0, dsdt)
    want = OR.bary_diffbins(topo, bary, 10.0, dsdt)
    assert np.array_equal(got, want)
    # each entry is one bin of the net drift between consecutive table points
    drift = ((bary - topo) - (bary[0] - topo[0])) * 86400.0 / dsdt
    if k == 0:
        assert len(got) == int(np.floor(drift[-1] + 0.5)) and np.all(got > 0)
        assert np.all(np.diff(got) > 0)
    if k == 1:
        assert np.all(got < 0)
    if k == 3:
        assert len(got) == 0


def test_diffbins_errors():
    topo, bary = tempo_table(100.0, 10.0, v=1e-4)
    with pytest.raises(PrestoError):
        bary_diffbins(topo[:1], bary[:1], 10.0, 1e-4)
    with pytest.raises(PrestoError):
        bary_diffbins(topo, bary, 10.0, 0.0)
    with pytest.raises(PrestoError):
        bary_diffbins(topo, bary[:-1], 10.0, 1e-4)


def test_bary_series_oracle_properties():
    """The oracle's output loop on a ramp: adds repeat the padding value, removes drop
    samples; the result is numout long."""
    topo = np.arange(20, dtype=np.float32)[None, :]
    pv = np.array([-1.0], np.float32)
    got = OR.bary_series(topo, 20, 22, np.array([3, 3, -7, 12], np.int32), pv)[0]
    want = [0, 1, 2, -1, -1, 3, 4, 5, 6, 8, 9, 10, 11, -1, 12, 13, 14, 15, 16, 17, 18, 19]
    assert got.tolist() == want
    got = OR.bary_series(topo, 20, 25, np.array([-0, 19, 25], np.int32), pv)[0]
    assert got.tolist() == list(range(1, 19)) + [-1, 19] + [-1] * 5
    # the data end: one past the last topocentric sample written
    assert OR.bary_data_end(20, 22, np.array([3, 3, -7, 12], np.int32)) == 22
    assert OR.bary_data_end(20, 25, np.array([-0, 19, 25], np.int32)) == 20
    assert OR.bary_data_end(20, 30, np.array([-2, -5, -9], np.int32)) == 17
    assert OR.bary_data_end(20, 20, np.array([-2, 19], np.int32)) == 20
    assert OR.bary_data_end(20, 19, np.array([-2, 19], np.int32)) == 18


@pytest.mark.gpu
@pytest.mark.parametrize("numout_kind", ["pad", "cut", "exact"])
@pytest.mark.parametrize("k", [0, 1, 2])
def test_gpu_bary_series(engine, numout_kind, k):
    """hd_plan_set_bary: the device's barycentred series == oracle.bary_series of the same
    plan's topocentric series (bit-exact), for added, removed and mixed bins; padded,
    truncated and exact output lengths; the first-DM padding value of the reference's pad mode."""
    from hipdedisp.synth import palfa_obs, palfa_synth
    obs = palfa_obs(N=1 << 18, nbits=8)
    engine.set_obs(obs, Opts())
    engine.synth_device(palfa_synth())
    nds = obs.N
    numout = {"pad": nds + 3000, "cut": nds - 5000, "exact": nds}[numout_kind]
    pp = PassParams(subdm=30.0, lodm=25.0, dmstep=0.5, numdms=76, nsub=96, ds=1, numout=numout)
    p = engine.plan(pp)
    try:
        p.run_subband()
        topo = p.run_dedisp(to_host=True)
        T = obs.N * obs.dt
        # drifts large enough for hundreds of bins in a 17-s beam
        tab = [dict(v=3e-3), dict(v=-2e-3), dict(v=1e-3, amp=2e-3, per=5.0)][k]
        top, bar = tempo_table(T, 1.0, **tab)
        db = bary_diffbins(top, bar, 1.0, obs.dt)
        assert len(db) > 50
        p.set_bary(db)
        got = p.run_dedisp(to_host=True)
        nvalid = min(nds, numout)
        padv = OR.pad_values(topo, nds, Opts().pad_mode)
        want = OR.bary_series(topo, nvalid, numout, db, padv)
        assert np.array_equal(got, want)
        assert p.data_end() == OR.bary_data_end(nvalid, numout, db)
        p.set_bary(db)                                     # the same list again: a no-op
        assert p.data_end() == OR.bary_data_end(nvalid, numout, db)
        p.set_bary(None)                                   # back to topocentric
        assert p.data_end() == nvalid
        assert np.array_equal(p.run_dedisp(to_host=True), topo)
    finally:
        p.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("k", [1, 2])
def test_gpu_bary_inf_and_single_pulse_border(engine, tmp_path, k):
    """A barycentred, padded pass: the .inf on/off pair ends the data at hd_plan_data_end - 1
    (the barycentred count, not N/ds - 1), and hd_single_pulse's border-case prune uses the same
    boundary -- candidates identical to the oracle's with nds = that data end."""
    from hipdedisp import single_pulse as SP
    from hipdedisp.formats import inf as INF
    from hipdedisp.formats.series import write_dats_device
    from hipdedisp.synth import palfa_obs, palfa_synth
    obs = palfa_obs(N=1 << 18, nbits=8)
    engine.set_obs(obs, Opts())
    engine.synth_device(palfa_synth())
    nds = obs.N
    numout = nds + 2000
    pp = PassParams(subdm=30.0, lodm=25.0, dmstep=0.5, numdms=76, nsub=96, ds=1, numout=numout)
    p = engine.plan(pp)
    try:
        p.run_subband()
        topo = p.run_dedisp(to_host=True)
        top, bar = tempo_table(obs.N * obs.dt, 1.0, **[dict(v=3e-3), dict(v=-2e-3), dict(v=1e-3, amp=2e-3, per=5.0)][k])
        db = bary_diffbins(top, bar, 1.0, obs.dt)
        p.set_bary(db)
        series = p.run_dedisp(to_host=True)
        dend = OR.bary_data_end(nds, numout, db)
        assert p.data_end() == dend and dend != nds
        dms = ["%.2f" % (25.0 + 0.5 * i) for i in range(76)]
        info = INF.InfoData(name="beam", dt=obs.dt, num_chan=96)
        write_dats_device(p, str(tmp_path / "beam"), dms[:76], info, p.data_end())
        d = INF.read_inf(str(tmp_path / ("beam_DM%s.inf" % dms[0])))
        assert d.onoff == [0.0, float(dend - 1), float(numout - 1), float(numout - 1)]
        wl = SP.widths(obs.dt, 0.1)
        got, bad = SP.device_candidates(p, obs.dt, 0.1, 3.0)
        raw, wbad = OR.sp_hits(series, wl, 3.0)
        assert np.array_equal(bad, wbad)
        ref = OR.sp_candidates(raw, wbad, wl, [float(x) for x in dms], obs.dt, dend, numout,
                               ls=numout // 1000 * 1000 // 8000 * 8000)
        want = [(d_, c.bin, c.downfact, c.sigma) for d_, cl in enumerate(ref) for c in cl]
        have = [(r[0], r[1], wl[r[2]], r[4]) for r in got.tolist()]
        assert have == want
    finally:
        p.destroy()
