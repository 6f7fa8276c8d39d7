"""TEST INFRASTRUCTURE ONLY (never imported by the product): numpy restatement of rfifind
[PRESTO-ext; parity with PRESTO unpinned: rfifind is not in this image] as the reference runs
it before the dedispersion loop (lib/python/PALFA2_presto_search.py:482-490).

stats(): per whole interval of ptsperint spectra and channel, the samples rfifind reads
(clip_times replacements from oracle.prepare with no mask, channels ascending), mean and
std (variance over n - 1) summed in hd_rfi.hip's order (64 lane partials over samples
l, l + 64, ..., then a xor butterfly) so they compare exactly, and the largest power of the
interval's real FFT (float64 here) over bins 1 .. n/2 - 1 divided by n * variance.

mask(): rfifind's decisions restated on their own (not hipdedisp.rfifind): trimmed
average/median/std of all cells (middle 80 % for means and stds), a cell bad beyond
timesigma of them or above the freqsigma power threshold, channels (intervals) bad in more
than chanfrac (intfrac) of their cells zapped whole.
"""
import math

import numpy as np


def _butterfly(p):
    p = np.array(p, np.float64)
    for m in (32, 16, 8, 4, 2, 1):
        p = p + p[np.arange(64) ^ m]
    return p[0]


def decode(obs, opts, raw):
    """File rows uint8 [N][rowbytes] -> float32 [N][nchan], channels ascending (no
    calibration): 8-bit bytes, 4-bit nibbles in opts.nibble_hi_first order, 16-bit ints."""
    raw = np.asarray(raw, np.uint8)
    if obs.nbits == 8:
        x = raw[:, :obs.nchan].astype(np.float32)
    elif obs.nbits == 4:
        hi, lo = raw >> 4, raw & 15
        a, b = (hi, lo) if opts.nibble_hi_first else (lo, hi)
        x = np.empty((raw.shape[0], 2 * raw.shape[1]), np.float32)
        x[:, 0::2], x[:, 1::2] = a, b
        x = x[:, :obs.nchan]
    else:
        dt = ">i2" if opts.be16 else "<i2"
        x = np.ascontiguousarray(raw).view(dt)[:, :obs.nchan].astype(np.float32)
    return x[:, ::-1].copy() if obs.flip else x


def samples(obs, opts, raw, clean):
    """[N][nchan] float32 channel values (ascending frequency) with clip_times applied
    (clean = oracle.prepare(obs, opts, raw) with no mask)."""
    x = decode(obs, opts, raw)
    if clean is not None and clean.nclipped:
        t = np.nonzero(clean.clipped)[0]
        x[t] = clean.pad[np.minimum(t // clean.blk, clean.nblk - 1)]
    return x


def stats(x, ptsperint):
    n = ptsperint
    numint = x.shape[0] // n
    nch = x.shape[1]
    avg = np.zeros((numint, nch), np.float32)
    std = np.zeros((numint, nch), np.float32)
    pw = np.zeros((numint, nch), np.float32)
    rows = (n + 63) // 64
    valid = (np.arange(rows * 64) < n).reshape(rows, 64, 1)
    for i in range(numint):
        blk = x[i * n:(i + 1) * n].astype(np.float64)          # [n][nch]
        lanes = np.zeros((rows * 64, nch))
        lanes[:n] = blk
        lanes = lanes.reshape(rows, 64, nch)                    # lane l: samples l, l + 64, ...
        part = np.zeros((64, nch))
        for r in range(rows):
            part += lanes[r]
        mean = np.array([_butterfly(part[:, c]) for c in range(nch)]) / n
        part = np.zeros((64, nch))
        for r in range(rows):
            d = np.where(valid[r], lanes[r] - mean, 0.0)
            part += d * d
        q = np.array([_butterfly(part[:, c]) for c in range(nch)])
        var = q / (n - 1)
        avg[i] = mean.astype(np.float32)
        std[i] = np.sqrt(var).astype(np.float32)
        spec = np.fft.rfft(blk.astype(np.float32).astype(np.float64), axis=0)
        norm = np.where(var * n > 0, var * n, 1.0)
        p = (spec.real ** 2 + spec.imag ** 2)[1:n // 2] / norm
        pw[i] = p.max(axis=0).astype(np.float32)
    return avg, std, pw


def _trimmed(a, fraction):
    s = np.sort(a.ravel().astype(np.float32))
    ln = int(s.size * fraction + 0.5)
    st = (s.size - ln) // 2
    m = s[st:st + ln].astype(np.float64)
    mu = m.sum() / ln
    sd = math.sqrt(((m - mu) ** 2).sum() / (ln - 1)) if ln > 1 else 0.0
    return np.float32(mu), s[s.size // 2], np.float32(sd)


def mask(avg, std, pw, ptsperint, timesigma=10.0, freqsigma=4.0, chanfrac=0.7, intfrac=0.3):
    """-> (bitmap [numint][nchan] u8, zapint [numint] u8)."""
    _, amed, asd = _trimmed(avg, 0.8)
    _, smed, ssd = _trimmed(std, 0.8)
    ptail = 0.5 * math.erfc(freqsigma / math.sqrt(2.0))
    reject = math.log((ptsperint // 2) / ptail)
    bad = np.zeros(avg.shape, bool)
    if asd > 0:
        bad |= np.abs(avg - amed) > timesigma * asd
    if ssd > 0:
        bad |= np.abs(std - smed) > timesigma * ssd
    bad |= pw > reject
    numint, nch = bad.shape
    zint = bad.sum(axis=1) > intfrac * nch
    zch = bad.sum(axis=0) > chanfrac * numint
    out = bad.copy()
    out[:, zch] = True
    out[zint] = True
    return out.astype(np.uint8), zint.astype(np.uint8)
