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
