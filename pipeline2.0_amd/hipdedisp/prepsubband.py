"""`prepsubband` command-line shim: the reference's command strings run unchanged.

    python -m hipdedisp.prepsubband -psrfits -sub -subdm 3.80 -downsamp 1 -nsub 96 \
        -mask base_rfifind.mask -o tmp/subbands/base base.fits          (stage 1, :506-511)
    python -m hipdedisp.prepsubband -lodm 0.00 -dmstep 0.10 -numdms 76 -downsamp 1 \
        -nsub 96 -numout 4194304 -o tmp/base tmp/subbands/base_DM3.80.sub[0-9]*   (stage 2, :514-520)
    python -m hipdedisp.prepsubband -mask M -lodm L -dmstep D -numdms n -downsamp ds \
        -numout N -o tmp/base base.fits                                   (no subbands, :522-529)

Exit status is 0 on success and 1 on failure, so timed_execute() (PALFA2_presto_search.py:
95-139) raises PrestoError exactly as it does for a failing PRESTO binary.  Flags the
reference never passes are rejected rather than ignored, except prepsubband's own
-clip/-noclip (default -clip 6, as the reference's commands leave it) and -nobary.

Barycentring: without -nobary PRESTO resamples the series to the barycentre with TEMPO,
which is not available here.  The shim computes the delay tables at v/c = -baryv (a
hipdedisp option; 0 by default, or $HIPDEDISP_BARYV) and writes topocentric series, and
says so on stderr unless -nobary is given.
"""
import argparse
import glob
import os
import sys

import numpy as np

from .engine import Engine, ObsParams, Opts, PassParams, PrestoError
from .formats import psrfits
from .formats.inf import InfoData, read_inf
from .formats.mask import mask_padvals, read_mask
from .formats.series import read_subbands, write_dats, write_subbands


def parse(argv):
    ap = argparse.ArgumentParser(prog="prepsubband", allow_abbrev=False)
    ap.add_argument("-psrfits", action="store_true")
    ap.add_argument("-sub", action="store_true")
    ap.add_argument("-subdm", type=float)
    ap.add_argument("-lodm", type=float, default=0.0)
    ap.add_argument("-dmstep", type=float, default=1.0)
    ap.add_argument("-numdms", type=int, default=10)
    ap.add_argument("-downsamp", type=int, default=1)
    ap.add_argument("-nsub", type=int, default=0)
    ap.add_argument("-numout", type=int, default=0)
    ap.add_argument("-mask", type=str, default=None)
    ap.add_argument("-nobary", action="store_true")
    ap.add_argument("-clip", type=float, default=6.0)
    ap.add_argument("-noclip", action="store_true")
    ap.add_argument("-baryv", type=float, default=float(os.environ.get("HIPDEDISP_BARYV", "0")))
    ap.add_argument("-o", dest="outfile", required=True)
    ap.add_argument("-device", type=int, default=int(os.environ.get("HIPDEDISP_DEVICE", "0")))
    ap.add_argument("infiles", nargs="+")
    return ap.parse_args(argv)


def _expand(files):
    out = []
    for f in files:
        g = sorted(glob.glob(f))
        out += g if g else [f]
    return out


def _dm_strings(lodm, dmstep, numdms):
    return ["%.2f" % (lodm + i * dmstep) for i in range(numdms)]


def _mask_state(eng, maskfn, nchan):
    """-mask M: the rfifind mask plus determine_padvals' pad values from <root>.stats."""
    if not maskfn:
        return
    if not os.path.exists(maskfn):
        raise PrestoError("rfifind mask %s does not exist" % maskfn)
    m = read_mask(maskfn)
    if m.numchan != nchan:
        raise PrestoError("mask has %d channels, data has %d" % (m.numchan, nchan))
    eng.set_rfimask(m, mask_padvals(maskfn, nchan))


def _opts(a, **kw):
    return Opts(clip_sigma=0.0 if a.noclip else a.clip, **kw)


def run(argv):
    a = parse(argv)
    files = _expand(a.infiles)
    opts = _opts(a)
    voverc = 0.0 if a.nobary else a.baryv
    if not a.nobary:
        sys.stderr.write("prepsubband (hipdedisp): no barycentric resampling (TEMPO unavailable); "
                         "topocentric series, delays at v/c = %g\n" % voverc)
    if files[0].endswith(".fits") or a.psrfits:
        si = psrfits.SpectraInfo(files)
        obs = si.obs_params(voverc)
        nsub = a.nsub or obs.nchan
        base_info = InfoData(name="", telescope=si.telescope or "Arecibo", instrument=si.backend,
                             object=si.source or "Unknown", ra=si.ra_str, dec=si.dec_str,
                             observer=si.observer or "Unknown", mjd=float(si.start_MJD[0]))
        with Engine(a.device) as eng:
            if not a.sub and nsub == obs.nchan:
                opts = _opts(a, sub_dtype=1)    # no .sub int16 round trip without -sub (:522-529)
            eng.set_obs(obs, opts)
            scl, offs, wts = si.read_calib()
            if scl is not None or offs is not None or wts is not None:
                eng.set_calib(scl, offs, wts)
            si.stream_to(eng)
            _mask_state(eng, a.mask, obs.nchan)
            if a.sub:
                if a.subdm is None:
                    raise PrestoError("-sub needs -subdm")
                p = eng.plan(PassParams(subdm=a.subdm, lodm=a.subdm, dmstep=1.0, numdms=1, nsub=nsub,
                                        ds=a.downsamp))
                p.run_subband()
                info = InfoData(**{**base_info.__dict__})
                info.name = os.path.basename(a.outfile) + "_DM%.2f" % a.subdm
                info.dm, info.N, info.dt = a.subdm, p.nds, p.sub_dt
                info.freq, info.chan_wid, info.num_chan = p.sub_lofreq, p.sub_chanwid, nsub
                info.freqband = nsub * p.sub_chanwid
                write_subbands(a.outfile + "_DM%.2f" % a.subdm, p.get_subbands(), info)
                p.destroy()
            else:
                p = eng.plan(PassParams(subdm=a.lodm, lodm=a.lodm, dmstep=a.dmstep, numdms=a.numdms,
                                        nsub=nsub, ds=a.downsamp, numout=a.numout))
                p.run_subband()
                series = p.run_dedisp()
                info = InfoData(**{**base_info.__dict__})
                info.dt, info.freq, info.chan_wid, info.num_chan = p.sub_dt, p.sub_lofreq, p.sub_chanwid, nsub
                info.freqband = nsub * p.sub_chanwid
                write_dats(a.outfile, _dm_strings(a.lodm, a.dmstep, a.numdms), series, info, p.nds)
                p.destroy()
    else:
        # stage 2 on .subNN files (+ .sub.inf)
        sub, sinfo = read_subbands(files, dtype=np.int16)
        if sinfo is None:
            raise PrestoError("missing .sub.inf next to %s" % files[0])
        nsub = sub.shape[0]
        if a.nsub and a.nsub != nsub:
            raise PrestoError("-nsub %d but %d subband files" % (a.nsub, nsub))
        if a.downsamp != 1:
            raise PrestoError("stage-2 -downsamp > 1 is not used by the reference (dd_downsamp = 1)")
        sobs = ObsParams(nchan=nsub, nbits=16, dt=sinfo.dt, lofreq=sinfo.freq, df=sinfo.chan_wid,
                         N=sub.shape[1], nsblk=sub.shape[1], flip=False, voverc=voverc)
        with Engine(a.device) as eng:
            eng.set_obs(sobs, opts)
            p = eng.plan(PassParams(subdm=sinfo.dm, lodm=a.lodm, dmstep=a.dmstep, numdms=a.numdms, nsub=nsub,
                                    ds=1, numout=a.numout, sub_input=True))
            p.set_subbands(sub)
            series = p.run_dedisp()
            info = InfoData(**{**sinfo.__dict__})
            info.freqband = nsub * sinfo.chan_wid
            write_dats(a.outfile, _dm_strings(a.lodm, a.dmstep, a.numdms), series, info, p.nds)
            p.destroy()
    return 0


def main(argv=None):
    try:
        return run(sys.argv[1:] if argv is None else argv)
    except (PrestoError, OSError, ValueError) as e:
        sys.stderr.write("prepsubband (hipdedisp): %s\n" % e)
        return 1


if __name__ == "__main__":
    sys.exit(main())
