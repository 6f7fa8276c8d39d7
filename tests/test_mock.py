"""CPU checks of Mock ingest: the file-name logic of
lib/python/datafile.py:395-508 (grouping, completeness, the merged name), the merged view of
two half-band files (channel selection by frequency, the 7 deleted rows, both band orders,
8- and 4-bit) against an independent channel-level construction, and PSRFITS gaps between
files (psrfits.py:272-280).  combine_mocks' own arithmetic is unpinned (not in this image)."""
import numpy as np
import pytest

from hipdedisp.formats import mock, psrfits
from hipdedisp.search_stage import DedispJob
from hipdedisp.synth import palfa_obs

S0 = "4bit-p2030.20120314.G34.5+0.1.b3s0g0.00123.fits"
S1 = "4bit-p2030.20120314.G34.5+0.1.b3s1g0.00123.fits"
DF = 0.336059375


def test_names():
    assert mock.are_grouped(S0, S1) and mock.are_grouped("/x/" + S1, "/y/" + S0)
    assert not mock.are_grouped(S0, S0)
    assert not mock.are_grouped(S0, S1.replace(".b3", ".b4"))
    assert not mock.are_grouped(S0, S1.replace("00123", "00124"))
    assert not mock.are_grouped(S0, "p2030.20120314.G34.5+0.1.b3.00123.fits")
    assert mock.is_complete([S0, S1]) and not mock.is_complete([S0]) and not mock.is_complete([S0, S1, S0])
    assert mock.merged_basename([S0, S1]) == "p2030.20120314.G34.5+0.1.b3.00123"
    m = mock.fnmatch(S1).groupdict()
    assert m == dict(projid="p2030", date="20120314", source="G34.5+0.1", beam="3", subband="1", scan="00123")


def unpack(raw, nbits, nchan):
    if nbits == 8:
        return raw[:, :nchan].astype(np.int32)
    x = np.empty((raw.shape[0], 2 * raw.shape[1]), np.int32)
    x[:, 0::2], x[:, 1::2] = raw >> 4, raw & 15            # high nibble first (PALFA)
    return x[:, :nchan]


def halves(tmp_path, nbits, flip, nrows=12, nsblk=256, nchan=512, lofreq=1214.14, sep=448, seed=0):
    """Two half-band files: channel k of the low band at lofreq + k*df, the high band's
    channels sep channels up; returns (paths, per-band channel values ascending in freq)."""
    rng = np.random.default_rng(seed)
    paths, vals = [], []
    for sb, lof in ((0, lofreq), (1, lofreq + sep * DF)):
        obs = palfa_obs(N=nrows * nsblk, nbits=nbits, nchan=nchan, nsblk=nsblk, flip=flip)
        obs.lofreq, obs.df = lof, DF
        raw = rng.integers(0, 256, size=(obs.N, obs.rowbytes)).astype(np.uint8)
        fn = str(tmp_path / (S0 if sb == 0 else S1))
        psrfits.write_psrfits(fn, raw, obs, beam=3)
        ch = unpack(raw, nbits, nchan)                     # file channel order
        vals.append(ch[:, ::-1] if flip else ch)           # ascending frequency
        paths.append(fn)
    return paths, vals


@pytest.mark.parametrize("nbits,flip", [(8, True), (8, False), (4, True), (4, False)])
def test_merged_view(tmp_path, nbits, flip):
    paths, (lo, hi) = halves(tmp_path, nbits, flip)
    mb = mock.MockBeam(paths[::-1])                        # order of the arguments is free
    assert mb.nchan == 960 and mb.N == (12 - 7) * 256 and mb.nsblk == 256
    assert mb.lofreq == pytest.approx(1214.14) and mb.df == pytest.approx(DF) and mb.flip == flip
    # 1024 - 960 = 64 overlapping channels dropped: 32 from the top of the low band, 32 from
    # the bottom of the high band; rows 0..6 deleted
    want = np.concatenate([lo[7 * 256:, :480], hi[7 * 256:, 32:]], axis=1)
    if flip:
        want = want[:, ::-1]
    got = unpack(mb.read_spectra(), nbits, 960)
    assert np.array_equal(got, want)
    o = mb.obs_params()
    assert (o.nchan, o.N, o.nbits, o.flip) == (960, mb.N, nbits, flip)
    assert mb.start_MJD[0] == pytest.approx(56000.5 + 7 * 256 * o.dt / 86400.0, abs=1e-12)


def test_merged_calibration(tmp_path):
    paths, _ = halves(tmp_path, 8, True)
    scl, offs, wts = mock.MockBeam(paths).read_calib()
    assert scl is None and offs is None and wts is None


def test_rejects(tmp_path):
    paths, _ = halves(tmp_path, 8, True)
    with pytest.raises(ValueError):
        mock.MockBeam(paths, nchan_out=1100)
    with pytest.raises(ValueError):
        mock.MockBeam(paths, rows_deleted=12)
    with pytest.raises(ValueError):
        mock.MockBeam([paths[0]])


def test_dedisp_job_uses_merged_beam(tmp_path):
    paths, _ = halves(tmp_path, 4, True)
    job = DedispJob(paths, resultsdir=str(tmp_path), tmpdir_base=str(tmp_path), backend="pdev", workdir=str(tmp_path))
    try:
        assert isinstance(job.specinfo, mock.MockBeam)
        assert job.basefilenm == "p2030.20120314.G34.5+0.1.b3.00123"
        assert job.nchan == 960 and job.orig_N == 5 * 256 and job.samp_per_row == 256
        assert job.BW == pytest.approx(960 * DF)
    finally:
        job.close()


def test_psrfits_gap_between_files(tmp_path):
    obs = palfa_obs(N=4 * 512, nbits=8, nchan=64, nsblk=512)
    rng = np.random.default_rng(1)
    a = rng.integers(0, 256, size=(obs.N, obs.rowbytes)).astype(np.uint8)
    b = rng.integers(0, 256, size=(obs.N, obs.rowbytes)).astype(np.uint8)
    fa, fb = str(tmp_path / "a.fits"), str(tmp_path / "b.fits")
    psrfits.write_psrfits(fa, a, obs, mjd=56000.5)
    gap = 3 * 512                                          # file b starts 3 rows after a ends
    psrfits.write_psrfits(fb, b, obs, mjd=56000.5 + (obs.N + gap) * obs.dt / 86400.0)
    si = psrfits.SpectraInfo([fa, fb])
    assert si.gaps() == [(obs.N, gap)] and int(si.N) == 2 * obs.N + gap
    x = si.read_spectra()
    assert np.array_equal(x[:obs.N], a) and not x[obs.N:obs.N + gap].any() and np.array_equal(x[obs.N + gap:], b)
    assert si.obs_params().N == 2 * obs.N + gap
