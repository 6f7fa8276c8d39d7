"""TEST INFRASTRUCTURE ONLY — an independent numpy restatement of the same prepsubband
arithmetic as oracle/prepsubband_oracle.c, written from the rules in oracle.h rather
than from the C code, so the two can pin each other (tests/test_oracle.py).
Small cases only (vectorised over time, Python loops over channels/subbands/DMs/blocks).
"""
import numpy as np

F32 = np.float32


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
        v = raw.astype(F32)
    elif nbits == 4:
        hi = (raw >> 4).astype(F32)
        lo = (raw & 15).astype(F32)
        first, second = (hi, lo) if nibble_hi_first else (lo, hi)
        v = np.empty((raw.shape[0], nchan), F32)
        v[:, 0::2], v[:, 1::2] = first, second
    else:
        v = raw.view(">i2" if be16 else "<i2").astype(F32)
    return v[:, ::-1] if flip else v


def decode(raw, nchan, nbits, flip, scl=None, offs=None, wts=None):
    x = unpack(raw, nchan, nbits, flip)
    order = np.arange(nchan)[::-1] if flip else np.arange(nchan)   # raw channel of ascending c
    if scl is not None:
        x = (x * np.asarray(scl, F32)[order]).astype(F32)
    if offs is not None:
        x = (x + np.asarray(offs, F32)[order]).astype(F32)
    if wts is not None:
        x = (x * np.asarray(wts, F32)[order]).astype(F32)
    return x


# ---------------------------------------------------------------- per-block cleaning
def block_masks(N, nchan, dt, blk, mask, ptsperint, dtint=0.0, zapint=None):
    """check_mask over read blocks: the union of the first and last interval a block
    touches, or every channel when either interval is a zap_int."""
    nblk = -(-N // blk)
    zap = np.zeros((nblk, nchan), np.uint8)
    allzap = np.zeros(nblk, np.uint8)
    if mask is None:
        return zap, allzap
    mask = np.asarray(mask, np.uint8)
    numint = mask.shape[0]
    dti = dtint if dtint > 0 else ptsperint * dt
    zi = (mask.sum(axis=1) == nchan) if zapint is None else np.asarray(zapint).astype(bool)
    for b in range(nblk):
        st = float(b * blk) * dt
        en = st + blk * dt
        lo, hi = min(int(st / dti), numint - 1), min(int(en / dti), numint - 1)
        if zi[lo] or zi[hi]:
            allzap[b] = 1
            zap[b] = 1
        else:
            zap[b] = mask[lo] | mask[hi]
    return zap, allzap


def _as52(x):
    """mean and (n-1)-variance by the one-pass AS 52 update, in double."""
    mean = float(x[0])
    var = 0.0
    an1 = 0.0
    for i in range(1, len(x)):
        an = float(i + 1)
        an1 = float(i)
        dx = (float(x[i]) - mean) / an
        var += an * an1 * dx * dx
        mean += dx
    if len(x) > 1:
        var /= an1
    return mean, var


def clip_prepare(X, blk, allzap, clip_sigma, padvals0=None):
    """clip_times over the decoded blocks of X [N][nchan] (float32), in order.
    -> (pad [nblk][nchan], clipped [N])."""
    N, nchan = X.shape
    nblk = -(-N // blk)
    pad = np.zeros((nblk, nchan), F32)
    clipped = np.zeros(N, np.uint8)
    levels = np.zeros(nchan, F32) if padvals0 is None else np.asarray(padvals0, F32).copy()
    ravg, rstd, nread = F32(0), F32(0), 0
    chan_ravg = np.zeros(nchan, F32)
    for b in range(nblk):
        t0 = b * blk
        x = X[t0:t0 + blk]
        n = x.shape[0]
        if clip_sigma > 0 and not allzap[b]:
            zdm = np.zeros(n, F32)
            for c in range(nchan):                      # channel-order float fold
                zdm = (zdm + x[:, c]).astype(F32)
            med = np.sort(zdm)[(n - 1) // 2]
            lo, hi = F32(0.7 * float(med)), F32(1.3 * float(med))
            good = (zdm > lo) & (zdm < hi)
            if good.any():
                cur_avg, cur_var = _as52(zdm[good])
                cur_std = float(np.sqrt(cur_var))
                acc = np.zeros(nchan, np.float64)
                for t in np.nonzero(good)[0]:
                    acc += x[t].astype(np.float64)
                cat = acc / int(good.sum())
            else:
                cur_avg, cur_std = float(ravg), float(rstd)
                cat = chan_ravg.astype(np.float64)
            if nread:
                ravg = F32((float(F32(ravg * F32(29))) + cur_avg) / 30)
                rstd = F32((float(F32(rstd * F32(29))) + cur_std) / 30)
                chan_ravg = ((chan_ravg * F32(29)).astype(F32).astype(np.float64) + cat) / 30
                chan_ravg = chan_ravg.astype(F32)
            else:
                ravg, rstd = F32(cur_avg), F32(cur_std)
                chan_ravg = cat.astype(F32)
            levels = chan_ravg.copy()
            trig = F32(F32(clip_sigma) * rstd)
            bad = np.abs((zdm - ravg).astype(F32)) > trig
            clipped[t0:t0 + n][bad] = 1
            nread += 1
        pad[b] = levels
    return pad, clipped


def _to_sub(acc, sub_dtype, sub_round):
    if sub_dtype != 0:
        return acc
    if sub_round == 1:
        return np.clip(nearest_long(acc), -32768, 32767).astype(np.int16)
    y = acc.astype(np.float64) + 0.5
    ok = (y > -2147483649.0) & (y < 2147483648.0)
    i = np.where(ok, np.trunc(np.where(ok, y, 0.0)), -2147483648.0).astype(np.int64)
    return (i & 0xFFFF).astype(np.uint16).view(np.int16)


def stage1(raw, nchan, nbits, flip, nsub, ds, idispdt, scl=None, offs=None, wts=None,
           zap=None, pad=None, clipped=None, blk=0, sub_dtype=0, ds_mode=1, sub_round=0):
    """Whole-length stage 1: [nsub][N//ds] from the cleaned data (oracle.h model)."""
    N = raw.shape[0]
    x = decode(raw, nchan, nbits, flip, scl, offs, wts)
    nblk = -(-N // blk) if blk else 1
    padrows = np.zeros((nblk, nchan), F32) if pad is None else np.asarray(pad, F32)
    bidx = np.minimum(np.arange(N) // blk, nblk - 1) if blk else np.zeros(N, np.int64)
    repl = np.zeros((N, nchan), bool)
    if zap is not None:
        repl |= np.asarray(zap, bool)[bidx]
    if clipped is not None:
        repl |= np.asarray(clipped, bool)[:, None]
    x = np.where(repl, padrows[bidx], x).astype(F32)
    maxd = int(idispdt.max()) if len(idispdt) else 0
    xp = np.concatenate([x, np.tile(padrows[-1], (maxd + ds + 1, 1))], axis=0)
    nds = N // ds
    cps = nchan // nsub
    out = np.zeros((nsub, nds), np.int16 if sub_dtype == 0 else F32)
    for s in range(nsub):
        acc = np.zeros(nds, F32)
        for k in range(ds):
            sk = np.zeros(nds, F32)
            for cc in range(cps):
                c = s * cps + cc
                t = np.arange(nds) * ds + k + idispdt[c]
                sk = (sk + xp[t, c]).astype(F32)
            acc = (acc + sk).astype(F32)
        if ds_mode == 1:
            acc = (acc / F32(ds)).astype(F32)
        out[s] = _to_sub(acc, sub_dtype, sub_round)
    return out


def stage2(sub, off, numout=None, pad_mode=2):
    nsub, nds = sub.shape
    numdms = off.shape[0]
    numout = nds if numout is None else numout
    n = min(nds, numout)
    res = np.zeros((numdms, numout), F32)
    subz = np.concatenate([sub.astype(F32), np.zeros((nsub, int(off.max()) + n + 1), F32)], axis=1)
    for d in range(numdms):
        acc = np.zeros(n, F32)
        for s in range(nsub):
            acc = (acc + subz[s, off[d, s]:off[d, s] + n]).astype(F32)
        res[d, :n] = acc
    if numout > nds:
        if pad_mode == 2:       # update_stats' running mean of the first DM
            avg = 0.0
            for i, v in enumerate(res[0, :nds].tolist()):
                avg += (v - avg) / (i + 1.0)
            res[:, nds:] = F32(avg)
        for d in range(numdms):
            if pad_mode == 0:
                res[d, nds:] = F32(float(np.sum(res[d, :nds].astype(np.float64))) / nds)
            elif pad_mode == 1:
                res[d, nds:] = 0
    return res


def stats_padvals(dataavg, fraction=0.8):
    """determine_padvals: per channel, AS 52 mean of the middle 80 % of sorted averages."""
    numint, numchan = dataavg.shape
    ln = int(float(F32(numint * F32(fraction))) + 0.5)
    st = (numint - ln) // 2
    out = np.zeros(numchan, F32)
    for c in range(numchan):
        v = np.sort(np.asarray(dataavg[:, c], F32))
        out[c] = F32(_as52(v[st:st + ln])[0]) if ln > 0 else F32(0)
    return out
