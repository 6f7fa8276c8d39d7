"""Downstream candidate lists from dedispersed series (test helper; CPU, numpy).

The north star asks for identical single-pulse and accelsearch candidate lists from the
GPU series and from prepsubband's.  PRESTO's single_pulse_search.py and accelsearch are not
in this image, so this restates their first steps, simplified and named as such:

* single_pulse_candidates: single_pulse_search.py's core -- per series, detrend in blocks
  of `detrendlen` samples (block median), normalise by the series' robust sigma, convolve
  with boxcars of the reference's downfactors (1 and 2..150) and keep, per boxcar, local
  maxima above `threshold` (the reference's default threshold 5.0, maxwidth 0.1 s from
  lib/python/config/searching_example.py), one per `2*downfact` window; returns a sorted
  list of (dm_index, sample, downfact, round(sigma, 6)).
* fft_candidates: the zero-acceleration part of accelsearch's candidate list -- power
  spectrum of the mean-subtracted series, normalised by the median power / ln 2, top `n`
  bins with their incoherent harmonic sums (numharm 1, 2, 4, 8).

Both are deterministic functions of the series, so bit-identical series give identical
lists; the tests check the lists (not only the arrays) and that the injected sources are
found, so the comparison is the one the north star names.
"""
import numpy as np

DOWNFACTS = [1, 2, 3, 4, 6, 9, 14, 20, 30, 45, 70, 100, 150]


def single_pulse_candidates(series, dt, threshold=5.0, maxwidth=0.1, detrendlen=1000):
    out = []
    for d, x in enumerate(np.asarray(series, np.float64)):
        n = (len(x) // detrendlen) * detrendlen
        if n == 0:
            continue
        y = x[:n].reshape(-1, detrendlen)
        y = (y - np.median(y, axis=1, keepdims=True)).ravel()
        mad = np.median(np.abs(y - np.median(y)))
        sig = 1.4826 * mad if mad > 0 else (np.std(y) or 1.0)
        y = y / sig
        cs = np.concatenate([[0.0], np.cumsum(y)])
        for w in DOWNFACTS:
            if w * dt > maxwidth:
                break
            conv = (cs[w:] - cs[:-w]) / np.sqrt(w)
            hits = np.nonzero(conv > threshold)[0]
            last = -10 ** 9
            for h in hits:
                lo, hi = max(0, h - w), min(len(conv), h + w + 1)
                if h - last < 2 * w or conv[h] < conv[lo:hi].max():
                    continue
                last = h
                out.append((d, int(h), w, round(float(conv[h]), 6)))
    return sorted(out)


def fft_candidates(series, n=10, numharm=(1, 2, 4, 8)):
    out = []
    for d, x in enumerate(np.asarray(series, np.float64)):
        p = np.abs(np.fft.rfft(x - x.mean())) ** 2
        p[0] = 0.0
        p = p / (np.median(p[1:]) / np.log(2.0))
        for h in numharm:
            m = len(p) // h
            s = np.zeros(m)
            for k in range(1, h + 1):
                s += p[: m * k: k][:m]
            top = np.argsort(s)[::-1][:n]
            out.extend((d, h, int(b), round(float(s[b]), 4)) for b in sorted(top))
    return out


HARM_THRESH = {1: 20.0, 2: 24.0, 4: 32.0, 8: 48.0}


def spectrum_candidates(F, thresh=HARM_THRESH):
    """accelsearch's zero-acceleration candidates from de-reddened packed spectra
    [ndm][nb] (complex, the rednoise output: unit mean noise power): per DM and harmonic
    count h, every fundamental bin b >= 1 whose incoherently summed power
    sum_{k=1..h} |F[k*b]|^2 exceeds thresh[h]; {(dm, h, b): summed power}."""
    out = {}
    F = np.asarray(F)
    for d in range(F.shape[0]):
        p = F[d].real.astype(np.float64) ** 2 + F[d].imag.astype(np.float64) ** 2
        p[0] = 0.0
        for h, thr in thresh.items():
            m = len(p) // h
            s = np.zeros(m)
            for k in range(1, h + 1):
                s += p[: m * k: k][:m]
            for b in np.nonzero(s > thr)[0]:
                if b >= 1:
                    out[(d, h, int(b))] = float(s[b])
    return out


def candidate_mismatch(a, b, thresh=HARM_THRESH, rel=1e-3):
    """Entries of one list missing from the other that are NOT explained by a power within
    `rel` of the threshold (float32 vs float64 FFT rounding can move such a bin across it),
    plus entries in both whose powers differ by more than `rel`."""
    bad = []
    for key in set(a) ^ set(b):
        v = a.get(key, b.get(key))
        if v > thresh[key[1]] * (1.0 + rel):
            bad.append((key, a.get(key), b.get(key)))
    for key in set(a) & set(b):
        if abs(a[key] - b[key]) > rel * max(a[key], b[key]):
            bad.append((key, a[key], b[key]))
    return sorted(bad)
