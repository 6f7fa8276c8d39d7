"""Overlapped ingest of the next beam (BASELINE configs[4], the 7-beam pointing: one beam per
job, reference queue_managers/pbs.py:67): hd_prefetch_raw_file reads beam b+1's PSRFITS into
the second raw slot on a reader thread and its own copy stream while beam b's passes run;
hd_swap_raw makes it current.  Bar: every series of every beam bit-identical to a serial run
(hd_push_raw_file, then the passes), through three swaps, so the slot a prefetch refills is
the one the previous beam's queued work still read (the ev_free ordering)."""
import numpy as np
import pytest

from hipdedisp import Opts, PassParams, PrestoError
from hipdedisp.formats import psrfits
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth

pytestmark = pytest.mark.gpu

PASSES = [PassParams(subdm=30.0, lodm=26.2, dmstep=0.1, numdms=76, nsub=96, ds=1, numout=0),
          PassParams(subdm=250.0, lodm=241.0, dmstep=0.3, numdms=64, nsub=96, ds=2, numout=0)]


def _run(engine):
    out = []
    plans = [engine.plan(pp) for pp in PASSES]
    try:
        for p in plans:
            p.run_subband()
            out.append(p.run_dedisp())
    finally:
        for p in plans:
            p.destroy()
    return out


def _beams(tmp_path, obs, n):
    si = []
    for b in range(n):
        fn = str(tmp_path / ("beam%d.fits" % b))
        psrfits.write_psrfits(fn, host_spectra(obs, palfa_synth(beam=b)), obs, beam=b)
        si.append(psrfits.SpectraInfo([fn]))
    return si


def test_prefetch_beams_identical_to_serial(engine, tmp_path):
    obs = palfa_obs(N=1 << 18, nbits=8, nsblk=2048)
    si = _beams(tmp_path, obs, 2)
    engine.set_obs(si[0].obs_params(), Opts())
    want = []
    for b in range(2):                                  # serial: push, then the passes
        si[b].stream_to(engine, block_bytes=1 << 22)
        want.append(_run(engine))
    # overlapped: beam 0 current, beam 1 prefetched while beam 0 computes; then 0 again and 1
    engine.set_obs(si[0].obs_params(), Opts())
    si[0].stream_to(engine, block_bytes=1 << 22)
    order = [0, 1, 0, 1]
    for k, b in enumerate(order):
        if k + 1 < len(order):
            si[order[k + 1]].stream_to(engine, block_bytes=1 << 22, prefetch=True)
        got = _run(engine)
        for g, w in zip(got, want[b]):
            assert np.array_equal(g, w)
        if k + 1 < len(order):
            io, tot = engine.swap_raw()
            assert 0.0 <= io <= tot + 1e-3
    with pytest.raises(PrestoError):                    # nothing queued since the last swap
        engine.swap_raw()


def test_prefetch_errors(engine, tmp_path):
    obs = palfa_obs(N=1 << 14, nbits=8, nsblk=2048)
    engine.set_obs(obs, Opts())
    row = obs.rowbytes * 2048
    engine.prefetch_raw_file(str(tmp_path / "missing.fits"), 0, row, 0, row, 0, 8)
    with pytest.raises(PrestoError):                    # the reader's open failure, at the swap
        engine.swap_raw()
    with pytest.raises(PrestoError):                    # rows past N
        engine.prefetch_raw_file(str(tmp_path / "missing.fits"), 0, row, 0, row, 0, 9)


@pytest.mark.timeout(900)
def test_prefetch_full_beam_windows_bitexact(engine, tmp_path):
    """configs[4] at full size: a 960 ch x 2^22 x 8-bit beam read from PSRFITS into the second
    raw slot by hd_prefetch_raw_file while a stage-0 pass of the current beam runs, made current
    by hd_swap_raw; then passes of three DDplan stages of the prefetched beam (one shared
    stage-1 and stage-2 launch per stage, the bench's path) checked against the oracle on that
    beam's own spectra with its own clip_times state (clipping on): subband and series windows
    at t = 0, across raw byte 2^31 and at the end of the data, bit-exact."""
    import os
    import shutil
    import tempfile

    import oracle as OR
    from hipdedisp import plan

    N, W = 1 << 22, 4096
    off31 = (1 << 31) // 960 + 1
    obs = palfa_obs(N=N, nbits=8)
    d = tempfile.mkdtemp(dir="/dev/shm") if os.path.isdir("/dev/shm") else str(tmp_path)
    try:
        fns = []
        for b in range(2):
            fn = os.path.join(d, "beam%d.fits" % b)
            psrfits.write_psrfits(fn, host_spectra(obs, palfa_synth(beam=b)), obs, beam=b)
            fns.append(fn)
        si = [psrfits.SpectraInfo([fn]) for fn in fns]
        engine.set_obs(si[0].obs_params(), Opts())
        si[0].stream_to(engine)
        si[1].stream_to(engine, prefetch=True)                  # beam 1 streams in meanwhile
        ps = plan.ddplans_for("pdev")
        pp0 = PassParams(subdm=float(ps[0].subdmlist[5]), lodm=float(ps[0].lodm_arg(5)), dmstep=0.1, numdms=76,
                         nsub=96, ds=1, numout=N)
        p = engine.plan(pp0)
        p.run_subband()
        p.run_dedisp(to_host=False)
        p.destroy()
        io, tot = engine.swap_raw()
        assert 0.0 <= io <= tot + 1e-3
        raw = host_spectra(obs, palfa_synth(beam=1))
        cl = OR.prepare(obs, Opts(), raw, omp=True)
        for st, picks in ((0, (0, 27)), (1, (6,)), (5, (0,))):
            dd = ps[st]
            pps = [PassParams(subdm=float(dd.subdmlist[i]), lodm=float(dd.lodm_arg(i)), dmstep=float(dd.dmstep_arg()),
                              numdms=dd.dmsperpass, nsub=dd.numsub, ds=dd.sub_downsamp,
                              numout=plan.choose_N(N / dd.downsamp)) for i in range(dd.numpasses)]
            plans = [engine.plan(q) for q in pps]
            try:
                engine.run_subband_multi(plans)
                engine.run_dedisp_multi(plans)
                for i in picks:
                    q, pl = pps[i], plans[i]
                    idd, off = pl.delays()
                    nds = N // q.ds
                    hi = max(0, (off31 - int(idd.max())) // q.ds - W // 2)
                    for t0 in sorted({0, min(hi, nds - W), nds - W}):
                        cnt = min(W + int(off.max()), nds - t0)
                        want_sub = OR.stage1(obs, Opts(), raw, q.nsub, q.ds, q.subdm, t0=t0, count=cnt, clean=cl,
                                             omp=True)
                        assert np.array_equal(pl.get_subbands_window(t0, cnt), want_sub), (q.subdm, t0)
                        want = OR.stage2(want_sub, off, 0, W, omp=True)
                        assert np.array_equal(pl.get_series(0, q.numdms, t0, W), want), (q.subdm, t0)
            finally:
                for pl in plans:
                    pl.destroy()
    finally:
        shutil.rmtree(d, ignore_errors=True)
