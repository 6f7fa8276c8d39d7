"""TEST INFRASTRUCTURE ONLY (never imported by the product): numpy restatement of the per-.dat
`realfft; zapbirds -zap -zapfile Z -baryv v; rednoise` chain the reference runs after the
single-pulse search (lib/python/PALFA2_presto_search.py:548-558), as hd_fft.hip and
include/hipdedisp.h restate it [PRESTO-ext; parity with PRESTO unpinned: none of the three
tools is in this image, and PALFA.zaplist (lib/zaplists/PALFA.zaplist) is the only fixture
the reference holds for them].

realfft(): float64 FFT, PRESTO's packed layout (bin 0 = (DC, Nyquist)) -- the device's float32
hipFFT is compared within a tolerance.  zap_ranges() / rednoise_blocks(): the host layouts,
restated on their own.  zap() / rednoise(): from a given packed float32 spectrum (the device's
own realfft output in the GPU tests), the same double arithmetic in the same order, so the
device result must match bit for bit.
"""
import math

import numpy as np

LN2 = 0.69314718055994530942


def realfft(x):
    """Packed complex128 [ndm][n/2] of real series [ndm][n] (n even)."""
    X = np.fft.rfft(np.asarray(x, np.float64), axis=-1)
    n2 = X.shape[-1] - 1
    out = X[..., :n2].copy()
    out[..., 0] = X[..., 0].real + 1j * X[..., n2].real
    return out


def birdie_bins(birds, T, baryv=0.0):
    """zapbirds' bin ranges of zaplist entries (freq, width, barycentric) for T seconds:
    (f -/+ w/2) * T, a barycentric frequency divided by (1 + baryv) first."""
    lo = np.array([((f / (1.0 + baryv)) if b else f) * T - 0.5 * w * T for f, w, b in birds], np.float64)
    hi = np.array([((f / (1.0 + baryv)) if b else f) * T + 0.5 * w * T for f, w, b in birds], np.float64)
    return lo, hi


def zap_ranges(lobins, hibins, numbins):
    r = []
    for a, b in zip(lobins, hibins):
        if not a <= b:
            continue
        lo, hi = max(int(math.floor(a)), 1), min(int(math.ceil(b)), numbins)
        if lo < hi:
            r.append([lo, hi])
    r.sort()
    m = []
    for lo, hi in r:
        if m and lo <= m[-1][1]:
            m[-1][1] = max(m[-1][1], hi)
        else:
            m.append([lo, hi])
    out = []
    for lo, hi in m:
        side = min(max(50, hi - lo), 2048)
        out.append((lo, hi, max(1, lo - side), min(numbins, hi + side)))
    return np.array(out, np.int32).reshape(-1, 4)


def rednoise_blocks(numbins, T, startwidth=6, endwidth=100, endfreq=6.0):
    lg = math.log(1.0 + endfreq)
    offs = []
    o = 1
    while o < numbins:
        f = o / T
        w = endwidth if f >= endfreq else startwidth + int(math.floor((endwidth - startwidth) * math.log(1.0 + f) / lg))
        offs.append(o)
        o = min(numbins, o + w)
    offs.append(numbins)
    return np.array(offs, np.int32)


def _powers(z):
    re = z.real.astype(np.float64)
    im = z.imag.astype(np.float64)
    return re * re + im * im


def zap(F, ranges):
    """F complex64 [ndm][nb] packed; ranges int [k][4] -> zapped copy (medians from F)."""
    F = np.array(F, np.complex64, copy=True)
    G = F.copy()
    for d in range(F.shape[0]):
        p = _powers(F[d])
        for lo, hi, wlo, whi in ranges:
            w = np.concatenate([p[wlo:lo], p[hi:whi]])
            med = np.sort(w)[(len(w) - 1) // 2] if len(w) else 0.0
            G[d, lo:hi] = np.float32(math.sqrt(med / LN2))
    return G


def rednoise(F, boff):
    """F complex64 [ndm][nb] packed; boff block offsets -> de-reddened copy."""
    F = np.asarray(F, np.complex64)
    G = F.copy()
    nblk = len(boff) - 1
    o = boff[:-1].astype(np.int64)
    w = (boff[1:] - boff[:-1]).astype(np.int64)
    cen = o.astype(np.float64) + (w - 1).astype(np.float64) / 2.0
    nb = F.shape[1]
    i = np.arange(1, nb)
    j = np.searchsorted(boff, i, side="right") - 1                    # block of bin i
    left = i.astype(np.float64) < cen[j]
    ja = np.where(left, j - 1, j)
    jb = np.where(left, j, j + 1)
    lo_clamp = ja < 0
    hi_clamp = jb >= nblk
    jac = np.clip(ja, 0, nblk - 1)
    jbc = np.clip(jb, 0, nblk - 1)
    for d in range(F.shape[0]):
        p = _powers(F[d])
        m = np.array([np.sort(p[boff[k]:boff[k + 1]])[(boff[k + 1] - boff[k] - 1) // 2] for k in range(nblk)])
        with np.errstate(invalid="ignore", divide="ignore"):
            mi = m[jac] + (m[jbc] - m[jac]) * ((i.astype(np.float64) - cen[jac]) / (cen[jbc] - cen[jac]))
        mi = np.where(lo_clamp, m[0], np.where(hi_clamp, m[nblk - 1], mi))
        z = F[d, 1:]
        pos = mi > 0.0
        s = np.where(pos, 1.0 / np.sqrt(np.where(pos, mi, 1.0) / LN2), 0.0)
        re = (z.real.astype(np.float64) * s).astype(np.float32)
        im = (z.imag.astype(np.float64) * s).astype(np.float32)
        G[d, 1:] = np.where(pos, re + 1j * im, 0).astype(np.complex64)
        G[d, 0] = 1.0 + 0.0j
    return G
