"""GPU Mock ingest: the two half-band files streamed straight into their channel
ranges of the device raw block (hd_push_raw_file_band, rows 7.. as `fitsdelrow 1 7` leaves
them) equal the merged view checked on the CPU (tests/test_mock.py); PSRFITS gaps are
zero-filled on the device (hd_fill_raw); a DedispJob on the two halves dedisperses the merged
beam bit-exactly against the oracle.  Reference: lib/python/datafile.py:474-508,
formats/psrfits.py:272-280."""
import copy
import os

import numpy as np
import pytest

import oracle as OR
from hipdedisp import Opts
from hipdedisp.formats import mock, psrfits
from hipdedisp.search_stage import DedispJob, dedisperse_job, pass_params
from hipdedisp.synth import palfa_obs
from test_mock import halves

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nbits,flip", [(8, True), (4, True), (4, False)])
def test_mock_stream_equals_merged_view(engine, tmp_path, nbits, flip):
    paths, _ = halves(tmp_path, nbits, flip, nrows=20, nsblk=512)
    mb = mock.MockBeam(paths)
    engine.set_obs(mb.obs_params(), Opts())
    engine.fill_raw(0, mb.N, 0xA5)                         # stale bytes must all be overwritten
    io, tot, nbytes = mb.stream_to(engine, block_bytes=1 << 18)
    assert nbytes == 2 * 13 * 512 * (512 * nbits // 8)
    assert np.array_equal(engine.get_raw(), mb.read_spectra())


def test_gap_zero_filled_on_device(engine, tmp_path):
    obs = palfa_obs(N=4 * 512, nbits=8, nchan=64, nsblk=512)
    rng = np.random.default_rng(2)
    a = rng.integers(0, 256, size=(obs.N, obs.rowbytes)).astype(np.uint8)
    b = rng.integers(0, 256, size=(obs.N, obs.rowbytes)).astype(np.uint8)
    fa, fb = str(tmp_path / "a.fits"), str(tmp_path / "b.fits")
    psrfits.write_psrfits(fa, a, obs, mjd=56000.5)
    psrfits.write_psrfits(fb, b, obs, mjd=56000.5 + (obs.N + 1536) * obs.dt / 86400.0)
    si = psrfits.SpectraInfo([fa, fb])
    engine.set_obs(si.obs_params(), Opts())
    engine.fill_raw(0, int(si.N), 0x5A)
    si.stream_to(engine)
    assert np.array_equal(engine.get_raw(), si.read_spectra())


def test_dedisp_job_on_mock_halves(engine, tmp_path):
    paths, _ = halves(tmp_path, 4, True, nrows=23, nsblk=512, seed=5)
    job = DedispJob(paths, resultsdir=str(tmp_path), tmpdir_base=str(tmp_path), device=0, backend="pdev",
                    workdir=str(tmp_path))
    d = copy.copy(job.ddplans[0])
    d.numpasses = 1
    job.ddplans = [d]
    try:
        dedisperse_job(job)
        mb = job.specinfo
        raw = mb.read_spectra()
        pp = pass_params(job, d, 0)
        _, want = OR.run_pass(mb.obs_params(0.0), job.opts, raw, pp)
        nds = mb.N // pp.ds
        for k in (0, d.dmsperpass - 1):
            base = os.path.join(job.tempdir, "%s_DM%s" % (job.basefilenm, d.dmlist[0][k]))
            got = np.fromfile(base + ".dat", np.float32)
            assert np.array_equal(got[:nds], want[k, :nds])
        assert job.basefilenm == mock.merged_basename(paths)
    finally:
        job.close()
