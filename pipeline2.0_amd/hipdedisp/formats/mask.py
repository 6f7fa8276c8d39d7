"""rfifind `.mask` files [PRESTO-ext: read_mask/write_mask of src/mask.c, restated].

Layout (native-endian): doubles timesigma, freqsigma, mjd, dtint, lofreq, dfreq;
ints numchan, numint, ptsperint; int num_zap_chans + list; int num_zap_ints + list;
int num_chans_per_int[numint]; then for each interval with 0 < n < numchan its channel
list.  n == numchan means the whole interval is zapped.  The reference produces it at
PALFA2_presto_search.py:482-490 and feeds it to stage 1 with `-mask` (:506).
"""
from dataclasses import dataclass

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
    bitmap: np.ndarray          # uint8 [numint][numchan], 1 = zapped


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
    nzc = int(take(np.int32, 1)[0])
    if nzc:
        bitmap[:, take(np.int32, nzc)] = 1
    nzi = int(take(np.int32, 1)[0])
    if nzi:
        bitmap[take(np.int32, nzi), :] = 1
    per = take(np.int32, numint)
    for i, n in enumerate(per):
        if n >= numchan:
            bitmap[i, :] = 1
        elif n > 0:
            bitmap[i, take(np.int32, int(n))] = 1
    return RfiMask(*[float(x) for x in d], numchan, numint, ptsperint, bitmap)


def write_mask(path, m: RfiMask):
    """Write a mask; channels zapped in every interval go to the zap-channel list,
    fully zapped intervals to the zap-interval list, the rest per interval."""
    bm = np.asarray(m.bitmap, dtype=np.uint8)
    zap_chans = np.nonzero(bm.all(axis=0))[0].astype(np.int32)
    zap_ints = np.nonzero(bm.all(axis=1))[0].astype(np.int32)
    rest = bm.copy()
    rest[:, zap_chans] = 0
    with open(path, "wb") as f:
        f.write(np.array([m.timesigma, m.freqsigma, m.mjd, m.dtint, m.lofreq, m.dfreq], np.float64).tobytes())
        f.write(np.array([m.numchan, m.numint, m.ptsperint], np.int32).tobytes())
        f.write(np.array([len(zap_chans)], np.int32).tobytes() + zap_chans.tobytes())
        f.write(np.array([len(zap_ints)], np.int32).tobytes() + zap_ints.tobytes())
        lists, counts = [], []
        for i in range(m.numint):
            if i in set(zap_ints.tolist()):
                counts.append(m.numchan)
                lists.append(None)
                continue
            ch = np.nonzero(rest[i])[0].astype(np.int32)
            counts.append(len(ch))
            lists.append(ch)
        f.write(np.array(counts, np.int32).tobytes())
        for n, ch in zip(counts, lists):
            if ch is not None and 0 < n < m.numchan:
                f.write(ch.tobytes())
