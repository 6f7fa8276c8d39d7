"""rfifind on the device-resident raw block.

The reference runs, before the dedispersion loop (lib/python/PALFA2_presto_search.py:482-490):

    rfifind <datatype_flag> -time <rfifind_chunk_time> -o <base> <files>

(rfifind_chunk_time = 2**15 * 64 us: lib/python/config/searching_example.py:12) and passes
<base>_rfifind.mask to stage 1 (`-mask`, :506), prepsubband taking its pad values from the
.stats beside it.  Here the per-interval statistics come from the GPU (hd_rfifind_stats:
clip_times, mean, std, the largest normalised FFT power of every (interval, channel)) and
this module makes rfifind's decisions from them [PRESTO-ext, rfifind.c restated]:

* calc_avgmedstd over all (interval, channel) cells: the middle `fraction` of the sorted
  values (0.8 for the means and stds, 0.5 for the powers) gives the average and std, the
  median is the element numarr/2 of the sorted values;
* a cell is bad when |avg - median(avg)| > timesigma * std(avg) (or the same for the stds),
  or when its power exceeds power_for_sigma(freqsigma, 1, ptsperint/2) -- the single-bin
  exponential tail exp(-P) with the Gaussian tail of freqsigma spread over ptsperint/2 bins;
* channels bad in more than chanfrac of the intervals, and intervals bad in more than
  intfrac of the channels, are zapped whole (defaults: timesigma 10, freqsigma 4, chanfrac
  0.7, intfrac 0.3);
* <base>_rfifind.mask (per-interval channel lists, zap_ints) and <base>_rfifind.stats
  (datapow, dataavg, datastd) in PRESTO's layout (formats/mask.py).

Parity with PRESTO is unpinned (rfifind is not in this image); the oracle
(oracle/rfifind_oracle.py) restates the same steps independently.
"""
import ctypes
import math
import os
import time

import numpy as np

from .formats.mask import RfiMask, RfiStats, write_mask, write_stats

BAD_AVG, BAD_STD, BAD_POW = 1, 2, 4


def ptsperint_for(dt, chunk_time, nsblk):
    """Samples per interval for `-time chunk_time`: a whole number of PSRFITS rows, the
    nearest to chunk_time (at least one row) [PRESTO-ext]."""
    return max(1, int(chunk_time / (nsblk * dt) + 0.5)) * nsblk


def device_stats(engine, ptsperint):
    """(dataavg, datastd, datapow) float32 [N // ptsperint][nchan] of the engine's raw block."""
    numint = engine.obs.N // ptsperint
    shape = (numint, engine.obs.nchan)
    avg, std, pw = (np.zeros(shape, np.float32) for _ in range(3))
    f = ctypes.POINTER(ctypes.c_float)
    engine._chk(engine._L.hd_rfifind_stats(engine._ctx, int(ptsperint), avg.ctypes.data_as(f), std.ctypes.data_as(f),
                                           pw.ctypes.data_as(f)), "rfifind")
    return avg, std, pw


def calc_avgmedstd(arr, fraction):
    """(avg, median, std) of the middle `fraction` of the sorted values (float32 results)."""
    a = np.sort(np.asarray(arr, np.float32).ravel())
    n = a.size
    ln = int(n * fraction + 0.5)
    start = (n - ln) // 2
    mid = a[start:start + ln].astype(np.float64)
    avg = mid.mean() if ln else 0.0
    var = ((mid - avg) ** 2).sum() / (ln - 1) if ln > 1 else 0.0
    return np.float32(avg), a[n // 2], np.float32(math.sqrt(var))


def power_for_sigma(sigma, numtrials):
    """Normalised single-bin power whose chance of being exceeded in any of numtrials bins
    is the Gaussian tail probability of `sigma`."""
    p = 0.5 * math.erfc(sigma / math.sqrt(2.0)) / numtrials
    return -math.log(p)


def make_mask(avg, std, pw, ptsperint, timesigma=10.0, freqsigma=4.0, chanfrac=0.7, intfrac=0.3):
    """rfifind's bytemask and zap decisions -> (bitmap [numint][nchan] u8, zapint [numint] u8,
    zap_chans int32 [k], bytemask [numint][nchan] u8 of BAD_AVG | BAD_STD | BAD_POW)."""
    avg_avg, avg_med, avg_std = calc_avgmedstd(avg, 0.8)
    std_avg, std_med, std_std = calc_avgmedstd(std, 0.8)
    reject = power_for_sigma(freqsigma, ptsperint // 2)
    bm = np.zeros(avg.shape, np.uint8)
    if avg_std > 0:
        bm |= (np.abs(avg - avg_med) > timesigma * avg_std).astype(np.uint8) * BAD_AVG
    if std_std > 0:
        bm |= (np.abs(std - std_med) > timesigma * std_std).astype(np.uint8) * BAD_STD
    bm |= (pw > reject).astype(np.uint8) * BAD_POW
    bad = bm != 0
    numint, nchan = bm.shape
    zapchan = bad.sum(axis=0) > chanfrac * numint
    zapint = bad.sum(axis=1) > intfrac * nchan
    bitmap = bad | zapchan[None, :]
    bitmap[zapint, :] = True
    return bitmap.astype(np.uint8), zapint.astype(np.uint8), np.nonzero(zapchan)[0].astype(np.int32), bm


def rfifind(engine, outbase, chunk_time, nsblk, mjd=0.0, timesigma=10.0, freqsigma=4.0, chanfrac=0.7, intfrac=0.3):
    """`rfifind -time chunk_time -o outbase` on the engine's raw block (before any mask):
    writes outbase_rfifind.mask / .stats; returns (maskfilenm, RfiMask, RfiStats)."""
    obs = engine.obs
    pts = ptsperint_for(obs.dt, chunk_time, nsblk)
    avg, std, pw = device_stats(engine, pts)
    bitmap, zapint, zap_chans, _ = make_mask(avg, std, pw, pts, timesigma, freqsigma, chanfrac, intfrac)
    numint = bitmap.shape[0]
    m = RfiMask(timesigma, freqsigma, mjd, pts * obs.dt, obs.lofreq, obs.df, obs.nchan, numint, pts, bitmap, zapint,
                zap_chans)
    st = RfiStats(obs.nchan, numint, pts, 0, 0, pw, avg, std)
    maskfn = outbase + "_rfifind.mask"
    write_mask(maskfn, m)
    write_stats(outbase + "_rfifind.stats", st)
    return maskfn, m, st


def run_rfifind(job, chunk_time, outdir=None):
    """PALFA2_presto_search.py:482-490 with the raw block already on the device (the
    reference writes <base>_rfifind.* into its working directory; outdir here): returns
    (seconds, maskfilenm) -- what the reference adds to job.rfifind_time and feeds to -mask."""
    t0 = time.time()
    eng = job.open_engine()
    eng.set_mask(None, 0, None)
    base = os.path.join(outdir, job.basefilenm) if outdir else job.basefilenm
    maskfn, _, _ = rfifind(eng, base, chunk_time, int(job.samp_per_row), mjd=float(job.MJD))
    return time.time() - t0, maskfn
