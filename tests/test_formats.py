"""File formats either side of the path (PSRFITS in, rfifind .mask in, .subNN between the two
prepsubband calls, .dat/.inf out) and the search-stage host logic.  CPU only."""
import json
import os

import numpy as np
import pytest

from hipdedisp import plan as P
from hipdedisp.formats import psrfits
from hipdedisp.formats.inf import InfoData, format_inf, read_inf, write_inf
from hipdedisp.formats.mask import RfiMask, read_mask, write_mask
from hipdedisp.formats.series import read_subbands, write_dats, write_subbands
from hipdedisp.prepsubband import parse as parse_cli
from hipdedisp.search_stage import pass_params, report_lines
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth

GOLD = os.path.join(os.path.dirname(__file__), "golden", "ddplan_ref.json")


@pytest.mark.parametrize("nbits,flip", [(8, True), (4, True), (16, False)])
def test_psrfits_roundtrip(tmp_path, nbits, flip):
    obs = palfa_obs(N=4096, nbits=nbits, nsblk=512, flip=flip)
    spectra = host_spectra(obs, palfa_synth(nbits=nbits))
    fn = str(tmp_path / "p2030.20120314.G00.00+00.b3.00100.fits")
    scl = np.linspace(0.5, 1.5, obs.nchan).astype(np.float32)
    psrfits.write_psrfits(fn, spectra, obs, scl=scl)
    assert psrfits.is_PSRFITS(fn)
    si = psrfits.SpectraInfo([fn])
    assert isinstance(si.N, float) and si.N == 4096.0        # float, as psrfits.py:29/280
    assert si.num_channels == obs.nchan and si.bits_per_sample == nbits
    assert si.dt == obs.dt and si.spectra_per_subint == 512
    assert si.need_flipband == flip and si.df > 0
    assert si.lo_freq == pytest.approx(obs.lofreq) and si.df == pytest.approx(obs.df)
    assert si.BW == pytest.approx(obs.nchan * obs.df)
    assert si.need_scale and not si.need_offset and not si.need_weight
    assert np.array_equal(si.read_spectra(), spectra)
    o2 = si.obs_params()
    assert (o2.nchan, o2.nbits, o2.N, o2.flip) == (obs.nchan, nbits, obs.N, flip)
    s2, of2, w2 = si.read_calib()
    assert np.array_equal(s2, scl) and of2 is None and w2 is None
    assert si.backend == "pdev"


def test_inf_format_and_roundtrip(tmp_path):
    d = InfoData(name="base_DM71.00", dm=71.0, N=1408000, dt=0.000196428, freq=1215.2, freqband=322.6,
                 num_chan=96, chan_wid=3.36, onoff=[0, 1398100, 1407999, 1407999])
    txt = format_inf(d)
    lines = txt.splitlines()
    assert lines[0] == " Data file name without suffix          =  base_DM71.00"
    assert " Number of bins in the time series      =  1408000    " in lines
    assert " Any breaks in the data? (1=yes, 0=no)  =  1" in lines
    assert any(l.startswith(" On/Off bin pair #  2") for l in lines)
    assert " Dispersion measure (cm-3 pc)           =  71" in lines
    write_inf(str(tmp_path / "a.inf"), d)
    r = read_inf(str(tmp_path / "a.inf"))
    assert (r.name, r.dm, r.N, r.dt, r.num_chan) == (d.name, d.dm, d.N, d.dt, d.num_chan)
    assert r.onoff == [0.0, 1398100.0, 1407999.0, 1407999.0]


def test_mask_roundtrip(tmp_path):
    rng = np.random.default_rng(4)
    bm = (rng.random((37, 960)) < 0.05).astype(np.uint8)
    bm[:, [101, 460, 777]] = 1        # zapped channels
    bm[[3, 20]] = 1                   # zapped intervals
    m = RfiMask(10.0, 4.0, 56000.5, 2.097, 1214.0, 0.336, 960, 37, 32768, bm)
    fn = str(tmp_path / "x_rfifind.mask")
    write_mask(fn, m)
    r = read_mask(fn)
    assert (r.numchan, r.numint, r.ptsperint) == (960, 37, 32768)
    assert np.array_equal(r.bitmap, bm)


def test_series_files(tmp_path):
    rng = np.random.default_rng(5)
    sub = rng.integers(-100, 100, (96, 1000)).astype(np.int16)
    info = InfoData(name="b_DM3.80", dm=3.8, N=1000, dt=6.5e-5, freq=1215.0, num_chan=96, chan_wid=3.36)
    os.makedirs(tmp_path / "subbands")
    write_subbands(str(tmp_path / "subbands" / "b_DM3.80"), sub, info)
    names = sorted(os.listdir(tmp_path / "subbands"))
    assert names[0] == "b_DM3.80.sub.inf" and names[1] == "b_DM3.80.sub00" and names[-1] == "b_DM3.80.sub95"
    import glob
    got, ginfo = read_subbands(glob.glob(str(tmp_path / "subbands" / "b_DM3.80.sub[0-9]*")))
    assert np.array_equal(got, sub) and ginfo.dm == 3.8
    series = rng.standard_normal((3, 1100)).astype(np.float32)
    write_dats(str(tmp_path / "b"), ["0.00", "0.10", "0.20"], series, info, 1000)
    assert np.array_equal(np.fromfile(str(tmp_path / "b_DM0.10.dat"), np.float32), series[1])
    r = read_inf(str(tmp_path / "b_DM0.20.inf"))
    assert r.dm == 0.2 and r.N == 1100 and r.onoff == [0.0, 999.0, 1099.0, 1099.0]


class _Job:
    use_subbands = True
    orig_N = float(1 << 22)


def test_pass_params_mirror_command_lines():
    """The parameters run_pass hands the engine equal what the reference's two command
    strings carry (PALFA2_presto_search.py:506-520), for every pass of the Mock plan."""
    gold = json.load(open(GOLD))["backends"]["pdev"]
    for d, g in zip(P.ddplans_for("pdev"), gold):
        for i in range(d.numpasses):
            pp = pass_params(_Job(), d, i)
            stage1 = "prepsubband -psrfits -sub -subdm %s -downsamp %d -nsub %d" % (
                d.subdmlist[i], d.sub_downsamp, d.numsub)
            stage2 = "prepsubband -lodm %.2f -dmstep %.2f -numdms %d -downsamp %d -nsub %d -numout %d" % (
                d.lodm + i * d.sub_dmstep, d.dmstep, d.dmsperpass, d.dd_downsamp, d.numsub,
                P.choose_N(_Job.orig_N / d.downsamp))
            a1 = parse_cli(stage1.split()[1:] + ["-mask", "m.mask", "-o", "x", "in.fits"])
            a2 = parse_cli(stage2.split()[1:] + ["-o", "y", "y_DM1.00.sub[0-9]*"])
            assert pp.subdm == a1.subdm and pp.ds == a1.downsamp and pp.nsub == a1.nsub
            assert pp.lodm == a2.lodm and pp.dmstep == a2.dmstep and pp.numdms == a2.numdms
            assert pp.numout == a2.numout and a2.downsamp == 1
            assert "%.2f" % pp.lodm == g["passes"][i]["lodm_arg"]


class _JobNoSub:
    use_subbands = False
    orig_N = float(1 << 22)
    nchan = 960


def test_pass_params_no_subbands_mirror_command_line():
    """use_subbands=False: one command per pass (PALFA2_presto_search.py:522-527), no -nsub
    (channels are the subbands, nsub = nchan [PRESTO-ext]) and -downsamp dd*sub."""
    for d in P.ddplans_for("pdev"):
        for i in range(d.numpasses):
            pp = pass_params(_JobNoSub(), d, i)
            cmd = "prepsubband -mask %s -lodm %.2f -dmstep %.2f -numdms %d -downsamp %d -numout %d -o %s %s" % (
                "m.mask", d.lodm + i * d.sub_dmstep, d.dmstep, d.dmsperpass, d.dd_downsamp * d.sub_downsamp,
                P.choose_N(_JobNoSub.orig_N / d.downsamp), "t/b", "in.fits")
            a = parse_cli(cmd.split()[1:])
            assert pp.lodm == a.lodm and pp.dmstep == a.dmstep and pp.numdms == a.numdms
            assert pp.ds == a.downsamp and pp.numout == a.numout and pp.nsub == 960 and a.nsub == 0
            assert not a.sub and a.subdm is None


def test_report_lines():
    class J:
        subbanding_time, dedispersing_time = 12.5, 30.25
    lines = report_lines(J(), 100.0)
    assert lines[0] == "       subbanding time =    12.5 sec (12.50%)"
    assert lines[1] == "     dedispersing time =    30.2 sec (30.25%)"


def test_psrfits_stream_geometry(tmp_path):
    """SpectraInfo.stream_to hands hd_push_raw_file the DATA column geometry of each SUBINT
    table; reading the file with exactly that geometry (as the C reader does) gives the
    spectra read_spectra() gives.  CPU: the engine is a recorder."""
    obs = palfa_obs(N=4096, nbits=8, nsblk=512)
    spectra = host_spectra(obs, palfa_synth())
    fn = str(tmp_path / "beam.fits")
    psrfits.write_psrfits(fn, spectra, obs)
    si = psrfits.SpectraInfo([fn])

    class Rec:
        def push_raw_file(self, path, table_offset, row_bytes, col_offset, col_bytes, row0, nrows, start=0,
                          block_bytes=0):
            raw = np.fromfile(path, np.uint8)
            rows = [raw[table_offset + (row0 + i) * row_bytes + col_offset:][:col_bytes] for i in range(nrows)]
            self.got = (start, np.concatenate(rows).reshape(-1, obs.rowbytes))
            return 0.0, 0.0

    rec = Rec()
    _, _, nbytes = si.stream_to(rec)
    assert nbytes == spectra.size
    assert rec.got[0] == 0 and np.array_equal(rec.got[1], spectra)
