"""TEST INFRASTRUCTURE ONLY — an independent numpy restatement of the same prepsubband
arithmetic as oracle/prepsubband_oracle.c, written from the rules in oracle.h rather
than from the C code, so the two can pin each other (tests/test_oracle.py).
Small cases only (vectorised over time, Python loops over channels/subbands/DMs).
"""
import math

import numpy as np


def delay_from_dm(dm, f):
    return dm / (0.000241 * f * f)


def nearest_long(x):
    x = np.asarray(x, dtype=np.float64)
    return np.where(x < 0, np.ceil(x - 0.5), np.floor(x + 0.5)).astype(np.int64)


def chan_delays(nchan, nsub, subdm, lofreq, df, dt, voverc=0.0):
    cps = nchan // nsub
    f = (lofreq + np.arange(nchan) * df) * (1.0 + voverc)
    d = delay_from_dm(subdm, f)
    sbw = df * cps
    subtop = (lofreq + sbw - df + np.arange(nsub) * sbw) * (1.0 + voverc)
    ds = delay_from_dm(subdm, subtop)
    return nearest_long((d - np.repeat(ds, cps)) / dt).astype(np.int32)


def _rt(v, fmt):
    return float(fmt % v)


def sub_params(nchan, nsub, ds, lofreq, df, dt, roundtrip=True):
    cps = nchan // nsub
    sbw = df * cps
    lof = lofreq + sbw - df
    sdt = dt * ds
    if roundtrip:
        return _rt(lof, "%.12g"), _rt(sbw, "%.12g"), _rt(sdt, "%.15g")
    return lof, sbw, sdt


def dm_offsets(nchan, nsub, ds, lofreq, df, dt, lodm, dmstep, numdms, voverc=0.0, roundtrip=True):
    lof, sbw, sdt = sub_params(nchan, nsub, ds, lofreq, df, dt, roundtrip)
    losubhi = lof + sbw - sbw            # subband_delays with one channel per subband
    f = (losubhi + np.arange(nsub) * sbw) * (1.0 + voverc)
    out = np.zeros((numdms, nsub), np.int32)
    for i in range(numdms):
        dm = lodm + i * dmstep
        d = delay_from_dm(dm, f)
        out[i] = nearest_long((d - d[-1]) / sdt)
    return out


def unpack(raw, nchan, nbits, flip, nibble_hi_first=True, be16=True):
    """raw uint8 [N][rowbytes] -> float32 [N][nchan], ascending-frequency channels."""
    raw = np.asarray(raw, np.uint8)
    if nbits == 8:
        v = raw.astype(np.float32)
    elif nbits == 4:
        hi = (raw >> 4).astype(np.float32)
        lo = (raw & 15).astype(np.float32)
        first, second = (hi, lo) if nibble_hi_first else (lo, hi)
        v = np.empty((raw.shape[0], nchan), np.float32)
        v[:, 0::2], v[:, 1::2] = first, second
    else:
        v = raw.view(">i2" if be16 else "<i2").astype(np.float32)
    return v[:, ::-1] if flip else v


def stage1(raw, nchan, nbits, flip, nsub, ds, idispdt, scl=None, offs=None, wts=None,
           mask=None, ptsperint=0, padvals=None, sub_dtype=0, ds_mode=0):
    """Whole-length stage 1: [nsub][N//ds]."""
    N = raw.shape[0]
    x = unpack(raw, nchan, nbits, flip)
    order = np.arange(nchan)[::-1] if flip else np.arange(nchan)   # raw channel of ascending c
    if scl is not None:
        x = (x * np.asarray(scl, np.float32)[order]).astype(np.float32)
    if offs is not None:
        x = (x + np.asarray(offs, np.float32)[order]).astype(np.float32)
    if wts is not None:
        x = (x * np.asarray(wts, np.float32)[order]).astype(np.float32)
    pv = np.zeros(nchan, np.float32) if padvals is None else np.asarray(padvals, np.float32)
    if mask is not None:
        iv = np.arange(N) // ptsperint
        ok = iv < mask.shape[0]
        m = np.zeros((N, nchan), bool)
        m[ok] = mask[iv[ok]].astype(bool)
        x = np.where(m, pv[None, :], x).astype(np.float32)
    maxd = int(idispdt.max()) if len(idispdt) else 0
    xp = np.concatenate([x, np.tile(pv, (maxd + ds + 1, 1))], axis=0)
    nds = N // ds
    cps = nchan // nsub
    out = np.zeros((nsub, nds), np.int16 if sub_dtype == 0 else np.float32)
    for s in range(nsub):
        acc = np.zeros(nds, np.float32)
        for k in range(ds):
            sk = np.zeros(nds, np.float32)
            for cc in range(cps):
                c = s * cps + cc
                t = np.arange(nds) * ds + k + idispdt[c]
                sk = (sk + xp[t, c]).astype(np.float32)
            acc = (acc + sk).astype(np.float32)
        if ds_mode == 1:
            acc = (acc / np.float32(ds)).astype(np.float32)
        if sub_dtype == 0:
            out[s] = np.clip(nearest_long(acc), -32768, 32767).astype(np.int16)
        else:
            out[s] = acc
    return out


def stage2(sub, off, numout=None, pad_mode=0):
    nsub, nds = sub.shape
    numdms = off.shape[0]
    numout = nds if numout is None else numout
    n = min(nds, numout)
    res = np.zeros((numdms, numout), np.float32)
    subz = np.concatenate([sub.astype(np.float32), np.zeros((nsub, int(off.max()) + n + 1), np.float32)], axis=1)
    for d in range(numdms):
        acc = np.zeros(n, np.float32)
        for s in range(nsub):
            acc = (acc + subz[s, off[d, s]:off[d, s] + n]).astype(np.float32)
        res[d, :n] = acc
        if numout > nds:
            v = np.float32(float(np.sum(acc.astype(np.float64))) / nds) if pad_mode == 0 else np.float32(0)
            res[d, nds:] = v
    return res
