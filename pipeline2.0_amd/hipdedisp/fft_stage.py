"""realfft, zapbirds and rednoise on a pass's device-resident DM series.

The reference runs, for every .dat of a pass (lib/python/PALFA2_presto_search.py:548-558):

    realfft <dat>
    zapbirds -zap -zapfile <zaplist> -baryv <job.baryv> <fft>
    rednoise <fft>;  mv <base>_red.fft <base>.fft

Here the spectra are made and cleaned in HBM (hd_realfft / hd_zapbirds / hd_rednoise, see
csrc/hd_fft.hip and include/hipdedisp.h for the restated algorithms [PRESTO-ext; parity with
PRESTO unpinned]) and written as <base>_DM<dm>.fft (PRESTO's packed float32 layout) only when
asked.  The zaplist (:472-474, lib/zaplists/PALFA.zaplist) is parsed on the host: lines of
`freq width` (Hz), '#' comments, a leading 'B' marking a barycentric frequency, taken to the
topocentric frame as freq / (1 + baryv).
"""
import ctypes
import os
import time

import numpy as np

from . import _lib
from .engine import PrestoError

RED_STARTWIDTH, RED_ENDWIDTH, RED_ENDFREQ = 6, 100, 6.0     # rednoise's defaults

_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int32)


def read_zaplist(path):
    """[(freq, width, barycentric)] of a PRESTO .zaplist."""
    out = []
    with open(path) as f:
        for line in f:
            s = line.strip()
            if not s or s.startswith("#"):
                continue
            bary = s[0] in "Bb"
            if bary:
                s = s[1:]
            parts = s.split()
            if len(parts) < 2:
                continue
            out.append((float(parts[0]), float(parts[1]), bary))
    return out


def birdie_bins(birds, T, baryv=0.0):
    """(lobins, hibins) float64 of zaplist birdies for a series of T seconds."""
    lo = np.empty(len(birds))
    hi = np.empty(len(birds))
    for i, (f, w, bary) in enumerate(birds):
        if bary:
            f = f / (1.0 + baryv)
        lo[i] = (f - 0.5 * w) * T
        hi[i] = (f + 0.5 * w) * T
    return lo, hi


def zap_ranges(lobins, hibins, numbins):
    """hd_zap_ranges: int32 [k][4] = (lo, hi, wlo, whi) merged bin ranges and median windows."""
    L = _lib.load()
    lo = np.ascontiguousarray(lobins, np.float64)
    hi = np.ascontiguousarray(hibins, np.float64)
    nr = ctypes.c_int32()
    cap = max(1, len(lo))
    out = np.zeros((cap, 4), np.int32)
    rc = L.hd_zap_ranges(lo.ctypes.data_as(_dp), hi.ctypes.data_as(_dp), len(lo), int(numbins),
                         out.ctypes.data_as(_ip), cap, ctypes.byref(nr))
    if rc:
        raise PrestoError("hd_zap_ranges: %s" % _lib.last_error())
    return out[:nr.value]


def rednoise_blocks(numbins, T, startwidth=RED_STARTWIDTH, endwidth=RED_ENDWIDTH, endfreq=RED_ENDFREQ):
    """hd_rednoise_blocks: int32 block offsets [nblk + 1] over bins 1 .. numbins - 1."""
    L = _lib.load()
    n = ctypes.c_int32()
    rc = L.hd_rednoise_blocks(int(numbins), float(T), int(startwidth), int(endwidth), float(endfreq), None, 0,
                              ctypes.byref(n))
    if rc and rc != _lib.HD_E_NOMEM:
        raise PrestoError("hd_rednoise_blocks: %s" % _lib.last_error())
    out = np.zeros(n.value + 1, np.int32)
    rc = L.hd_rednoise_blocks(int(numbins), float(T), int(startwidth), int(endwidth), float(endfreq),
                              out.ctypes.data_as(_ip), len(out), ctypes.byref(n))
    if rc:
        raise PrestoError("hd_rednoise_blocks: %s" % _lib.last_error())
    return out


def prepare(plan):
    """hd_fft_prepare: the hipFFT plan + spectra buffer of the plan's series geometry built
    now (rocFFT's kernel builds, seconds per new size), so a later realfft only transforms."""
    plan.eng._chk(plan.eng._L.hd_fft_prepare(plan._p), "fft prepare")


def realfft(plan):
    plan.eng._chk(plan.eng._L.hd_realfft(plan._p), "realfft")


def zapbirds(plan, lobins, hibins):
    lo = np.ascontiguousarray(lobins, np.float64)
    hi = np.ascontiguousarray(hibins, np.float64)
    plan.eng._chk(plan.eng._L.hd_zapbirds(plan._p, lo.ctypes.data_as(_dp), hi.ctypes.data_as(_dp), len(lo)),
                  "zapbirds")


def rednoise(plan, T, startwidth=RED_STARTWIDTH, endwidth=RED_ENDWIDTH, endfreq=RED_ENDFREQ):
    plan.eng._chk(plan.eng._L.hd_rednoise(plan._p, int(startwidth), int(endwidth), float(endfreq), float(T)),
                  "rednoise")


def get_fft(plan, dm0=0, ndm=None):
    """Packed spectra float32 [ndm][numout] (numout/2 complex; bin 0 = (DC, Nyquist))."""
    if ndm is None:
        ndm = plan.pp.numdms - dm0
    out = np.empty((ndm, plan.numout), np.float32)
    plan.eng._chk(plan.eng._L.hd_get_fft(plan._p, int(dm0), int(ndm), out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))),
                  "hd_get_fft")
    return out


def spectra_complex(packed):
    """complex64 [ndm][numout/2] view of packed spectra."""
    return np.ascontiguousarray(packed).view(np.complex64)


def run_fft(plan, dt, birds=None, baryv=0.0, basenm=None, dm_strs=None, write=False):
    """:548-558 for one pass: realfft, zapbirds (when birds are given), rednoise on the
    device; <basenm>_DM<dm>.fft written when `write`; returns seconds (job.FFT_time's share)."""
    t0 = time.time()
    T = plan.numout * dt
    realfft(plan)
    if birds:
        lo, hi = birdie_bins(birds, T, baryv)
        zapbirds(plan, lo, hi)
    rednoise(plan, T)
    if write:
        spec = get_fft(plan)
        for s, row in zip(dm_strs, spec):
            with open("%s_DM%s.fft" % (basenm, s), "wb") as f:
                f.write(row.tobytes())
    plan.eng.sync()
    return time.time() - t0


def fft_pass(job, plan, ddplan, passnum, tempdir, opts):
    """search_stage hook: opts = dict(zaplist=path or None, baryv=..., write=bool)."""
    birds = read_zaplist(opts["zaplist"]) if opts.get("zaplist") else None
    t = run_fft(plan, plan.sub_dt, birds, opts.get("baryv", getattr(job, "baryv", 0.0)),
                os.path.join(tempdir, job.basefilenm), ddplan.dmlist[passnum], opts.get("write", False))
    job.FFT_time = getattr(job, "FFT_time", 0.0) + t
    return t
