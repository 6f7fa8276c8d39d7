"""rfifind `.mask` and `.stats` files [PRESTO-ext: read_mask / write_mask of src/mask.c and
write_statsfile / determine_padvals of rfifind, restated].

.mask layout (native-endian): doubles timesigma, freqsigma, mjd, dtint, lofreq, dfreq;
ints numchan, numint, ptsperint; int num_zap_chans + list; int num_zap_ints + list;
int num_chans_per_int[numint]; then, for each interval with 0 < n < numchan, its channel
list (n == numchan: every channel).  prepsubband's check_mask uses the zap_ints and the
per-interval lists only; rfifind writes the globally zapped channels into every interval's
list too, and write_mask below does the same.

.stats layout: ints numchan, numint, ptsperint, lobin, numbetween; then float32
datapow[numint][numchan], dataavg[numint][numchan], datastd[numint][numchan].

The reference produces both at PALFA2_presto_search.py:482-490 and feeds the mask to
stage 1 with `-mask` (:506); prepsubband derives its pad values from the .stats next to
the mask (`<root>.stats` for `<root>.mask`).
"""
import os
from dataclasses import dataclass, field
from typing import Optional

import numpy as np


@dataclass
class RfiMask:
    timesigma: float
    freqsigma: float
    mjd: float
    dtint: float
    lofreq: float
    dfreq: float
    numchan: int
    numint: int
    ptsperint: int
    bitmap: np.ndarray          # uint8 [numint][numchan], 1 = in the interval's channel list
    zapint: Optional[np.ndarray] = None    # uint8 [numint], 1 = interval in zap_ints
    zap_chans: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int32))


def read_mask(path) -> RfiMask:
    raw = open(path, "rb").read()
    pos = 0

    def take(dtype, n):
        nonlocal pos
        a = np.frombuffer(raw, dtype=dtype, count=n, offset=pos)
        pos += a.nbytes
        return a

    d = take(np.float64, 6)
    numchan, numint, ptsperint = (int(x) for x in take(np.int32, 3))
    bitmap = np.zeros((numint, numchan), dtype=np.uint8)
    zapint = np.zeros(numint, dtype=np.uint8)
    nzc = int(take(np.int32, 1)[0])
    zap_chans = take(np.int32, nzc).copy() if nzc else np.zeros(0, np.int32)
    nzi = int(take(np.int32, 1)[0])
    if nzi:
        zapint[take(np.int32, nzi)] = 1
    per = take(np.int32, numint)
    for i, n in enumerate(per):
        if n >= numchan:
            bitmap[i, :] = 1
        elif n > 0:
            bitmap[i, take(np.int32, int(n))] = 1
    return RfiMask(*[float(x) for x in d], numchan, numint, ptsperint, bitmap, zapint, zap_chans)


def write_mask(path, m: RfiMask):
    """Write a mask as rfifind does: channels listed in every interval also go to the
    zap-channel list (and stay in each interval's list); zap_ints are m.zapint (or the rows
    listing every channel) and are written with n = numchan."""
    bm = np.asarray(m.bitmap, dtype=np.uint8)
    zap_chans = np.nonzero(bm.all(axis=0))[0].astype(np.int32)
    zi = bm.all(axis=1) if m.zapint is None else np.asarray(m.zapint).astype(bool)
    zap_ints = np.nonzero(zi)[0].astype(np.int32)
    with open(path, "wb") as f:
        f.write(np.array([m.timesigma, m.freqsigma, m.mjd, m.dtint, m.lofreq, m.dfreq], np.float64).tobytes())
        f.write(np.array([m.numchan, m.numint, m.ptsperint], np.int32).tobytes())
        f.write(np.array([len(zap_chans)], np.int32).tobytes() + zap_chans.tobytes())
        f.write(np.array([len(zap_ints)], np.int32).tobytes() + zap_ints.tobytes())
        counts, lists = [], []
        for i in range(m.numint):
            if zi[i]:
                counts.append(m.numchan)
                lists.append(None)
                continue
            ch = np.nonzero(bm[i])[0].astype(np.int32)
            counts.append(len(ch))
            lists.append(ch)
        f.write(np.array(counts, np.int32).tobytes())
        for n, ch in zip(counts, lists):
            if ch is not None and 0 < n < m.numchan:
                f.write(ch.tobytes())


@dataclass
class RfiStats:
    numchan: int
    numint: int
    ptsperint: int
    lobin: int
    numbetween: int
    datapow: np.ndarray          # float32 [numint][numchan]
    dataavg: np.ndarray
    datastd: np.ndarray


def read_stats(path) -> RfiStats:
    raw = open(path, "rb").read()
    numchan, numint, ptsperint, lobin, numbetween = (int(x) for x in np.frombuffer(raw, np.int32, 5))
    n = numchan * numint
    arrs = np.frombuffer(raw, np.float32, 3 * n, offset=20).reshape(3, numint, numchan)
    return RfiStats(numchan, numint, ptsperint, lobin, numbetween, arrs[0].copy(), arrs[1].copy(), arrs[2].copy())


def write_stats(path, st: RfiStats):
    with open(path, "wb") as f:
        f.write(np.array([st.numchan, st.numint, st.ptsperint, st.lobin, st.numbetween], np.int32).tobytes())
        for a in (st.datapow, st.dataavg, st.datastd):
            f.write(np.ascontiguousarray(a, np.float32).tobytes())


def stats_path(maskfilenm):
    """determine_padvals' file name: the mask's root (up to the last '.') + '.stats'."""
    root, dot, suffix = maskfilenm.rpartition(".")
    if not dot or not suffix:
        raise ValueError("the mask filename (%s) must have a suffix" % maskfilenm)
    return root + ".stats"


def mask_padvals(maskfilenm, numchan):
    """prepsubband's pad values for -mask M: from `<root>.stats` when it exists (the middle-80%
    channel averages, hd_stats_padvals), else zeros (determine_padvals [PRESTO-ext])."""
    from ..engine import stats_padvals
    sp = stats_path(maskfilenm)
    if not os.path.exists(sp):
        return np.zeros(numchan, np.float32)
    st = read_stats(sp)
    if st.numchan != numchan:
        raise ValueError("%s has %d channels, the data %d" % (sp, st.numchan, numchan))
    return stats_padvals(st.dataavg)
