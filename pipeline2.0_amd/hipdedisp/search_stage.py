"""Drop-in replacement for the dedispersion stage of PALFA2_presto_search.search_job().

Reference (pipeline2.0, lib/python/PALFA2_presto_search.py):
  :444-465  set_up_job: obs_info(filenms) + tempdir in config.processing.base_tmp_dir
  :494-529  for ddplan in job.ddplans: for passnum: two `prepsubband` calls via
            timed_execute(), accumulating job.subbanding_time / job.dedispersing_time
  :531-537  per-DM names  <tempdir>/<base>_DM<dm %.2f>.dat/.inf
  :352-358  the two timers go to the .report

`run_pass(job, ddplan, passnum, maskfilenm, tempdir)` replaces the body of :500-529 one for
one: it creates <tempdir>/subbands as :500-503 does (the reference's own :608-611 removes or
empties it after every pass), leaves the same .dat/.inf files (and, with keep_subbands, the
same .subNN/.sub.inf files, which the reference moves to the workdir when it folds from
subbands, fold_rawdata=False) and returns (t_sub, t_dd) wall seconds, which it also adds to
the job's timers.
Failures raise PrestoError, the reference's exception for a failed prepsubband.
`dedisperse_job(job, per_dm=None)` is the whole loop of :494-537, calling `per_dm(job,
dmstr, basenm)` where the reference runs single_pulse_search/realfft/accelsearch.
"""
import os
import socket
import tempfile
import time

import numpy as np

from . import plan as P
from .engine import Engine, Opts, PassParams, PrestoError
from .formats import psrfits
from .formats import mock
from .formats.inf import InfoData
from .formats.mask import mask_padvals, read_mask
from .formats.series import write_dats_device, write_subbands


class DedispJob:
    """The part of obs_info (PALFA2_presto_search.py:231-294) the dedispersion stage uses."""

    def __init__(self, filenms, resultsdir=".", tmpdir_base=None, device=0, opts=None,
                 use_subbands=True, keep_subbands=False, backend=None, voverc=0.0, bary_table=None, workdir=None):
        self.filenms = list(filenms)
        self.filenmstr = " ".join(self.filenms)
        self.outputdir = resultsdir
        base = os.path.split(self.filenms[0])[1]
        self.basefilenm = base[:-5] if base.endswith(".fits") else base
        if mock.is_complete(self.filenms):
            # the two Mock halves: merged in-stream (datafile.py:474-508), named as the
            # merged file the reference would have searched
            self.specinfo = mock.MockBeam(self.filenms)
            self.basefilenm = self.specinfo.basename
        else:
            self.specinfo = psrfits.SpectraInfo(self.filenms)
        si = self.specinfo
        self.backend = backend or si.backend
        self.MJD = si.start_MJD[0]
        self.ra_string, self.dec_string = si.ra_str, si.dec_str
        self.orig_N = si.N                      # float64, as in the reference
        self.dt = si.dt
        self.BW = si.BW
        self.N = self.orig_N
        self.T = self.N * self.dt
        self.nchan = si.num_channels
        self.samp_per_row = si.spectra_per_subint
        self.fctr = si.fctr
        # average barycentric v/c (the reference's obs_info.baryv, :269-270, from TEMPO): it
        # enters PRESTO's delay tables -- 0 is prepsubband -nobary.  bary_table = (topo, bary,
        # tdt): the TEMPO table (MJDs every tdt s from the start of the data, as
        # presto.barycenter returns them, :43-57) that makes the series barycentred, as the
        # reference's stage-2 command (no -nobary, :514-520) leaves them; without one (TEMPO is
        # not in this image) the series stay topocentric and the .inf says so
        self.baryv = voverc
        self.bary_table = bary_table
        self._diffbins = {}
        self.hostname = socket.gethostname()
        self.use_subbands = use_subbands
        self.keep_subbands = keep_subbands
        self.subbanding_time = 0.0
        self.dedispersing_time = 0.0
        self.singlepulse_time = 0.0     # :539-546 on device (run_pass(single_pulse=...))
        self.FFT_time = 0.0             # :548-558 on device (run_pass(fft=...))
        self.ddplans = P.ddplans_for(self.backend)
        self.tempdir = tempfile.mkdtemp(suffix="_tmp", prefix=self.basefilenm,
                                        dir=tmpdir_base or ("/dev/shm" if os.path.isdir("/dev/shm") else None))
        # where the reference runs (search_job chdirs there, :416): the per-pass .subout /
        # .prepout logs go here
        self.workdir = workdir or os.getcwd()
        # without subbands prepsubband dedisperses the channels themselves (nsub = nchan
        # [PRESTO-ext]) and no .sub int16 file is written, so they stay float32 (:522-529)
        self.opts = opts or (Opts() if use_subbands else Opts(sub_dtype=1))
        self.engine = None
        self.device = device
        self._mask_loaded = None

    # -- engine state ------------------------------------------------------------------
    def open_engine(self):
        if self.engine is None:
            self.engine = Engine(self.device)
            self.obs = self.specinfo.obs_params(self.baryv)
            self.engine.set_obs(self.obs, self.opts)
            scl, offs, wts = self.specinfo.read_calib()
            if scl is not None or offs is not None or wts is not None:
                self.engine.set_calib(scl, offs, wts)
            self.ingest = self.specinfo.stream_to(self.engine)   # (pread s, total s, bytes)
        return self.engine

    def load_mask(self, maskfilenm):
        """`-mask M` of the reference's commands: the rfifind mask (prepsubband fails when it
        is missing, so this raises PrestoError) and the pad values determine_padvals derives
        from the `.stats` next to it (zeros without one)."""
        if maskfilenm == self._mask_loaded:
            return
        eng = self.open_engine()
        if maskfilenm:
            if not os.path.exists(maskfilenm):
                raise PrestoError("rfifind mask %s does not exist" % maskfilenm)
            m = read_mask(maskfilenm)
            if m.numchan != self.nchan:
                raise PrestoError("mask %s has %d channels, data %d" % (maskfilenm, m.numchan, self.nchan))
            try:
                padvals = mask_padvals(maskfilenm, self.nchan)
            except ValueError as e:
                raise PrestoError(str(e))
            eng.set_rfimask(m, padvals)
        else:
            eng.set_mask(None, 0, None)
        self._mask_loaded = maskfilenm

    def close(self):
        if self.engine is not None:
            self.engine.close()
            self.engine = None

    def set_bary(self, plan):
        """Barycentred output for a plan (its output sample time) when a TEMPO table is set."""
        if self.bary_table is None:
            return
        from .engine import bary_diffbins
        topo, bary, tdt = self.bary_table
        dsdt = plan.sub_dt
        if dsdt not in self._diffbins:
            self._diffbins[dsdt] = bary_diffbins(topo, bary, tdt, dsdt)
        plan.set_bary(self._diffbins[dsdt])

    def info_template(self, nsub, lofreq, chanwid, dt, series=False):
        """.inf fields; series=True for the stage-2 .dat files, which are barycentred (bary = 1,
        epoch = the barycentric MJD of the first sample) when a TEMPO table is set."""
        bary = series and self.bary_table is not None
        mjd = float(self.bary_table[1][0]) if bary else float(self.MJD)
        return InfoData(name="", telescope=self.specinfo.telescope or "Arecibo",
                        instrument=self.backend, object=self.specinfo.source or "Unknown",
                        ra=self.ra_string, dec=self.dec_string, observer=self.specinfo.observer or "Unknown",
                        mjd=mjd, bary=int(bary), dt=dt, freq=lofreq, freqband=nsub * chanwid,
                        num_chan=nsub, chan_wid=chanwid)


def pass_params(job, ddplan, passnum):
    """The parameters of the two prepsubband command lines (PALFA2_presto_search.py:506-520),
    parsed the way prepsubband parses them (DM strings are "%.2f" text)."""
    lodm = float(ddplan.lodm_arg(passnum))
    numout = P.choose_N(job.orig_N / ddplan.downsamp)
    if not job.use_subbands:
        # :522-527: no -sub / -subdm / -nsub; -downsamp dd_downsamp*sub_downsamp.  With one
        # channel per subband every stage-1 channel delay is 0, so subdm is immaterial.
        return PassParams(subdm=lodm, lodm=lodm, dmstep=float(ddplan.dmstep_arg()), numdms=ddplan.dmsperpass,
                          nsub=job.nchan, ds=ddplan.sub_downsamp * ddplan.dd_downsamp, numout=numout)
    return PassParams(subdm=float(ddplan.subdmlist[passnum]), lodm=lodm,
                      dmstep=float(ddplan.dmstep_arg()), numdms=ddplan.dmsperpass, nsub=ddplan.numsub,
                      ds=ddplan.sub_downsamp, numout=numout)


def command_lines(job, ddplan, passnum, maskfilenm, tempdir):
    """The two prepsubband command strings of the pass (PALFA2_presto_search.py:506-509,
    514-518) -- or the one of :522-527 without subbands -- as the reference formats them."""
    numout = P.choose_N(job.orig_N / ddplan.downsamp)
    lodm = ddplan.lodm + passnum * ddplan.sub_dmstep
    flag = "-psrfits"
    if not job.use_subbands:
        return ["prepsubband -mask %s -lodm %.2f -dmstep %.2f -numdms %d -downsamp %d -numout %d -o %s/%s %s"
                % (maskfilenm, lodm, ddplan.dmstep, ddplan.dmsperpass, ddplan.dd_downsamp * ddplan.sub_downsamp,
                   numout, tempdir, job.basefilenm, job.filenmstr)]
    subbasenm = "%s_DM%s" % (job.basefilenm, ddplan.subdmlist[passnum])
    return ["prepsubband %s -sub -subdm %s -downsamp %d -nsub %d -mask %s -o %s/subbands/%s %s"
            % (flag, ddplan.subdmlist[passnum], ddplan.sub_downsamp, ddplan.numsub, maskfilenm, tempdir,
               job.basefilenm, job.filenmstr),
            "prepsubband -lodm %.2f -dmstep %.2f -numdms %d -downsamp %d -nsub %d -numout %d -o %s/%s "
            "%s/subbands/%s.sub[0-9]*" % (lodm, ddplan.dmstep, ddplan.dmsperpass, ddplan.dd_downsamp, ddplan.numsub,
                                          numout, tempdir, job.basefilenm, tempdir, subbasenm)]


def _write_log(path, cmd, lines):
    """The per-pass stdout capture the reference keeps (<subbasenm>.subout / .prepout,
    :511,520, in the working directory): the command it stands for, then what ran."""
    from . import _lib
    with open(path, "w") as f:
        f.write("'%s'\n\n" % cmd)
        f.write("hipdedisp %s (libhipdedisp, MI355X gfx950)\n" % _lib.load().hd_version().decode())
        for ln in lines:
            f.write(ln + "\n")


def _single_pulse(job, plan, ddplan, passnum, tempdir, sp):
    """:539-546 for the pass's DMs on the device-resident series (hipdedisp.single_pulse):
    <base>_DM<dm>.singlepulse in sp['workdir'] (or tempdir); adds to job.singlepulse_time."""
    from .single_pulse import run_single_pulse
    t, _ = run_single_pulse(plan, os.path.join(tempdir, job.basefilenm), ddplan.dmlist[passnum],
                            workdir=sp.get("workdir"), maxwidth=sp.get("maxwidth", 0.1),
                            threshold=sp.get("threshold", 5.0))
    job.singlepulse_time = getattr(job, "singlepulse_time", 0.0) + t


def _fft(job, plan, ddplan, passnum, tempdir, fft):
    """:548-558 (realfft, zapbirds, rednoise) for the pass's DMs on the device (hipdedisp.fft_stage);
    adds to job.FFT_time."""
    from .fft_stage import fft_pass
    fft_pass(job, plan, ddplan, passnum, tempdir, fft)


def run_pass(job, ddplan, passnum, maskfilenm, tempdir, single_pulse=None, fft=None):
    """PALFA2_presto_search.py:498-529 for one pass: subbands (stage 1) then the DM sweep
    (stage 2); writes <tempdir>/<base>_DM<dm>.dat/.inf; returns (t_sub, t_dd).  Without
    subbands (:522-529) the reference makes one prepsubband call, timed as dedispersing
    time only: t_sub is 0 and the whole pass goes to t_dd.  single_pulse (a dict of
    maxwidth / threshold / workdir, config.searching's singlepulse_*) also runs :539-546 on
    the series while they are in HBM; fft (a dict of zaplist / baryv / write) then runs
    :548-558 on them."""
    if not job.use_subbands:
        return _run_pass_nosub(job, ddplan, passnum, maskfilenm, tempdir, single_pulse, fft)
    subbasenm = "%s_DM%s" % (job.basefilenm, ddplan.subdmlist[passnum])
    eng = job.open_engine()
    job.load_mask(maskfilenm)
    pp = pass_params(job, ddplan, passnum)
    plan = eng.plan(pp)
    os.makedirs(os.path.join(tempdir, "subbands"), exist_ok=True)     # :500-503
    try:
        t0 = time.time()
        plan.run_subband()
        eng.sync()
        if job.keep_subbands:
            info = job.info_template(pp.nsub, plan.sub_lofreq, plan.sub_chanwid, plan.sub_dt)
            info.name, info.dm, info.N = subbasenm, pp.subdm, plan.nds
            write_subbands(os.path.join(tempdir, "subbands", subbasenm), plan.get_subbands(), info)
        t_sub = time.time() - t0
        t0 = time.time()
        job.set_bary(plan)
        plan.run_dedisp(to_host=False)
        info = job.info_template(pp.nsub, plan.sub_lofreq, plan.sub_chanwid, plan.sub_dt, series=True)
        write_dats_device(plan, os.path.join(tempdir, job.basefilenm), ddplan.dmlist[passnum], info, plan.data_end())
        t_dd = time.time() - t0
        ms_sub, ms_dd = plan.last_ms()
        cmds = command_lines(job, ddplan, passnum, maskfilenm, tempdir)
        _write_log(os.path.join(job.workdir, subbasenm + ".subout"), cmds[0],
                   ["stage 1: %d subbands x %d samples (downsamp %d, subDM %s), %.3f ms on the device, %.3f s wall"
                    % (pp.nsub, plan.nds, pp.ds, ddplan.subdmlist[passnum], ms_sub, t_sub)])
        _write_log(os.path.join(job.workdir, subbasenm + ".prepout"), cmds[1],
                   ["stage 2: %d DMs x %d samples (%s), %.3f ms on the device, %.3f s wall with the .dat writes"
                    % (pp.numdms, plan.numout, plan.kernel(), ms_dd, t_dd)])
        if single_pulse is not None:
            _single_pulse(job, plan, ddplan, passnum, tempdir, single_pulse)
        if fft is not None:
            _fft(job, plan, ddplan, passnum, tempdir, fft)
    finally:
        plan.destroy()
    job.subbanding_time += t_sub
    job.dedispersing_time += t_dd
    return t_sub, t_dd


def _run_pass_nosub(job, ddplan, passnum, maskfilenm, tempdir, single_pulse=None, fft=None):
    """PALFA2_presto_search.py:522-529: `prepsubband -mask M -lodm -dmstep -numdms -downsamp
    (dd*sub) -numout N` straight on the raw data: channels (downsampled, float32) are the
    subbands of a nsub = nchan pass."""
    eng = job.open_engine()
    job.load_mask(maskfilenm)
    pp = pass_params(job, ddplan, passnum)
    plan = eng.plan(pp)
    try:
        t0 = time.time()
        plan.run_subband()
        job.set_bary(plan)
        plan.run_dedisp(to_host=False)
        info = job.info_template(pp.nsub, plan.sub_lofreq, plan.sub_chanwid, plan.sub_dt, series=True)
        write_dats_device(plan, os.path.join(tempdir, job.basefilenm), ddplan.dmlist[passnum], info, plan.data_end())
        t_dd = time.time() - t0
        if single_pulse is not None:
            _single_pulse(job, plan, ddplan, passnum, tempdir, single_pulse)
        if fft is not None:
            _fft(job, plan, ddplan, passnum, tempdir, fft)
    finally:
        plan.destroy()
    job.dedispersing_time += t_dd
    return 0.0, t_dd


def prepare_fft(job):
    """The FFT stage's hipFFT plans, one per DDplan stage's series geometry, built before the
    passes (hd_fft_prepare): rocFFT's kernel builds stay out of job.FFT_time."""
    from .fft_stage import prepare
    eng = job.open_engine()
    for ddplan in job.ddplans:
        if ddplan.numpasses < 1:
            continue
        p = eng.plan(pass_params(job, ddplan, 0))
        try:
            if p.numout >= 4 and p.numout % 2 == 0:
                prepare(p)
        finally:
            p.destroy()


def dedisperse_job(job, maskfilenm=None, per_dm=None, remove_dat=False, single_pulse=None, fft=None):
    """The loop of PALFA2_presto_search.py:494-537: every pass of every DDplan stage (with
    the device single-pulse search of :539-546 when single_pulse is given), then
    `per_dm(job, dmstr, basenm)` for each new DM (the reference's downstream tools)."""
    if fft is not None:
        prepare_fft(job)
    dmstrs = []
    for ddplan in job.ddplans:
        for passnum in range(ddplan.numpasses):
            run_pass(job, ddplan, passnum, maskfilenm, job.tempdir, single_pulse, fft)
            for dmstr in ddplan.dmlist[passnum]:
                dmstrs.append(dmstr)
                basenm = os.path.join(job.tempdir, job.basefilenm + "_DM" + dmstr)
                if per_dm is not None:
                    per_dm(job, dmstr, basenm)
                if remove_dat:
                    try:
                        os.remove(basenm + ".dat")
                    except OSError:
                        pass
    return dmstrs


def report_lines(job, total_time):
    """The two .report lines of the stage (PALFA2_presto_search.py:352-358)."""
    tt = total_time if total_time > 0 else 1.0
    return ["       subbanding time = %7.1f sec (%5.2f%%)" % (job.subbanding_time, job.subbanding_time / tt * 100.0),
            "     dedispersing time = %7.1f sec (%5.2f%%)" % (job.dedispersing_time, job.dedispersing_time / tt * 100.0)]
