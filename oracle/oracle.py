"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the C oracle (oracle/liboracle*.so).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the
checker.  Parity status: see oracle/oracle.h (PRESTO absent -> pinned by the reference's
plan code, analytic KATs and an independent numpy restatement, oracle/oracle_np.py).
"""
import ctypes
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


class or_obs(ctypes.Structure):
    _fields_ = [("nchan", ctypes.c_int32), ("nbits", ctypes.c_int32), ("npol", ctypes.c_int32),
                ("flip", ctypes.c_int32), ("dt", ctypes.c_double), ("lofreq", ctypes.c_double),
                ("df", ctypes.c_double), ("N", ctypes.c_int64), ("nsblk", ctypes.c_int32),
                ("_pad0", ctypes.c_int32), ("voverc", ctypes.c_double)]


class or_opts(ctypes.Structure):
    _fields_ = [("sub_dtype", ctypes.c_int32), ("ds_mode", ctypes.c_int32), ("pad_mode", ctypes.c_int32),
                ("nibble_hi_first", ctypes.c_int32), ("be16", ctypes.c_int32),
                ("inf_roundtrip", ctypes.c_int32), ("clip_sigma", ctypes.c_float), ("sub_round", ctypes.c_int32)]


class or_mask(ctypes.Structure):
    _fields_ = [("chans", ctypes.c_void_p), ("zapint", ctypes.c_void_p), ("numint", ctypes.c_int32),
                ("ptsperint", ctypes.c_int32), ("dtint", ctypes.c_double)]


_libs = {}


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib(omp=False):
    key = bool(omp)
    if key not in _libs:
        path = os.path.join(HERE, "liboracle_omp.so" if omp else "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        vp, i64, d = ctypes.c_void_p, ctypes.c_int64, ctypes.c_double
        P = ctypes.POINTER
        ci = ctypes.c_int
        L.or_chan_delays.argtypes = [P(or_obs), ci, d, P(ctypes.c_int32)]
        L.or_sub_params.argtypes = [P(or_obs), P(or_opts), ci, ci, P(d), P(d), P(d)]
        L.or_dm_offsets.argtypes = [P(or_obs), P(or_opts), ci, ci, d, d, ci, P(ctypes.c_int32)]
        L.or_dm_offsets_sub.argtypes = [ci, d, d, d, d, d, d, ci, P(ctypes.c_int32)]
        L.or_check_mask_blocks.argtypes = [P(or_obs), P(or_mask), ci, ci, vp, vp]
        L.or_check_mask_blocks.restype = None
        L.or_clip_prepare.argtypes = [P(or_obs), P(or_opts), vp, vp, vp, vp, vp, vp, ci, ci, vp, vp]
        L.or_clip_prepare.restype = i64
        L.or_clip_rows.argtypes = [P(or_obs), P(or_opts), vp, vp, vp, vp, vp, ci, i64, i64, vp]
        L.or_clip_rows.restype = ci
        L.or_clip_finish.argtypes = [P(or_obs), P(or_opts), vp, vp, vp, vp, vp, vp, ci, ci, vp, i64, i64, vp, vp]
        L.or_clip_finish.restype = i64
        L.or_stage1.argtypes = [P(or_obs), P(or_opts), vp, vp, vp, vp, vp, vp, vp, ci, ci, ci, ci, vp,
                                i64, i64, vp, i64]
        L.or_stage2.argtypes = [vp, ci, i64, i64, ci, vp, ci, i64, i64, vp, i64]
        L.or_pad.argtypes = [vp, ci, i64, i64, ci]
        L.or_pad.restype = None
        L.or_stats_padvals.argtypes = [vp, ci, ci, vp]
        L.or_stats_padvals.restype = None
        L.or_num_threads.restype = ci
        L.or_nearest_long.restype = i64
        L.or_nearest_long.argtypes = [d]
        L.or_delay_from_dm.restype = d
        L.or_delay_from_dm.argtypes = [d, d]
        L.sp_oracle_hits.argtypes = [vp, i64, ci, i64, vp, ci, d, vp, i64, vp]
        L.sp_oracle_hits.restype = i64
        L.sp_prune_related1.argtypes = [vp, vp, i64, ci, vp]
        L.sp_prune_related1.restype = None
        _libs[key] = L
    return _libs[key]


def _obs(o):
    return or_obs(nchan=o.nchan, nbits=o.nbits, npol=o.npol, flip=int(bool(o.flip)), dt=o.dt,
                  lofreq=o.lofreq, df=o.df, N=int(o.N), nsblk=o.nsblk, voverc=o.voverc)


def _opts(p):
    return or_opts(sub_dtype=p.sub_dtype, ds_mode=p.ds_mode, pad_mode=p.pad_mode,
                   nibble_hi_first=int(p.nibble_hi_first), be16=int(p.be16),
                   inf_roundtrip=int(p.inf_roundtrip), clip_sigma=p.clip_sigma, sub_round=p.sub_round)


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def chan_delays(obs, nsub, subdm):
    out = np.zeros(obs.nchan, np.int32)
    o = _obs(obs)
    lib().or_chan_delays(ctypes.byref(o), nsub, subdm, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return out


def sub_params(obs, opts, nsub, ds):
    a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    o, p = _obs(obs), _opts(opts)
    lib().or_sub_params(ctypes.byref(o), ctypes.byref(p), nsub, ds, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
    return a.value, b.value, c.value


def dm_offsets(obs, opts, nsub, ds, lodm, dmstep, numdms):
    out = np.zeros((numdms, nsub), np.int32)
    o, p = _obs(obs), _opts(opts)
    lib().or_dm_offsets(ctypes.byref(o), ctypes.byref(p), nsub, ds, lodm, dmstep, numdms,
                        out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return out


def dm_offsets_sub(nsub, lof, bw, dsdt, lodm, dmstep, numdms, voverc=0.0):
    out = np.zeros((numdms, nsub), np.int32)
    lib().or_dm_offsets_sub(nsub, lof, bw, dsdt, voverc, lodm, dmstep, numdms,
                            out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return out


@dataclass
class Clean:
    """Per-block cleaning state of a raw block (oracle.h model): blocks of `blk` spectra."""
    blk: int
    nblk: int
    zap: np.ndarray          # uint8 [nblk][nchan]
    allzap: np.ndarray       # uint8 [nblk]
    pad: np.ndarray          # float32 [nblk][nchan]
    clipped: np.ndarray      # uint8 [N]
    nclipped: int


def block_masks(obs, mask, ptsperint, dtint=0.0, zapint=None, blk=None):
    """mask.c check_mask per read block: (zap [nblk][nchan], allzap [nblk])."""
    blk = int(blk or obs.nsblk)
    nblk = (obs.N + blk - 1) // blk
    zap = np.zeros((nblk, obs.nchan), np.uint8)
    allzap = np.zeros(nblk, np.uint8)
    if mask is None:
        return zap, allzap
    m = np.ascontiguousarray(mask, np.uint8)
    zi = None if zapint is None else np.ascontiguousarray(zapint, np.uint8)
    om = or_mask(chans=_ptr(m), zapint=_ptr(zi), numint=m.shape[0], ptsperint=int(ptsperint), dtint=float(dtint))
    o = _obs(obs)
    lib().or_check_mask_blocks(ctypes.byref(o), ctypes.byref(om), blk, nblk, _ptr(zap), _ptr(allzap))
    return zap, allzap


def prepare(obs, opts, raw, calib=(None, None, None), mask=None, ptsperint=0, padvals=None, dtint=0.0,
            zapint=None, blk=None, omp=False):
    """Block masks + clip_times over the whole raw block -> Clean."""
    blk = int(blk or obs.nsblk)
    nblk = (obs.N + blk - 1) // blk
    zap, allzap = block_masks(obs, mask, ptsperint, dtint, zapint, blk)
    pad = np.zeros((nblk, obs.nchan), np.float32)
    clipped = np.zeros(obs.N, np.uint8)
    raw = np.ascontiguousarray(raw, np.uint8)
    cal = [None if c is None else np.ascontiguousarray(c, np.float32) for c in calib]
    pv = None if padvals is None else np.ascontiguousarray(padvals, np.float32)
    o, p = _obs(obs), _opts(opts)
    n = lib(omp).or_clip_prepare(ctypes.byref(o), ctypes.byref(p), _ptr(raw), _ptr(cal[0]), _ptr(cal[1]), _ptr(cal[2]),
                              _ptr(allzap), _ptr(pv), blk, nblk, _ptr(pad), _ptr(clipped))
    if n < 0:
        raise ValueError("or_clip_prepare rejected its arguments")
    return Clean(blk, nblk, zap, allzap, pad, clipped, int(n))


def clip_rows(obs, opts, raw, b0, nrows, mask=None, ptsperint=0, blk=None, omp=False):
    """clip_times' exchange rows [nrows][nchan + 3] of global read blocks [b0, b0 + nrows)
    (hd_clip_stats' layout) from raw = the observation's spectra b0 * blk onward; obs.N is
    the whole observation's length."""
    blk = int(blk or obs.nsblk)
    _, allzap = block_masks(obs, mask, ptsperint, blk=blk)
    rows = np.zeros((nrows, obs.nchan + 3), np.float64)
    raw = np.ascontiguousarray(raw, np.uint8)
    o, p = _obs(obs), _opts(opts)
    if lib(omp).or_clip_rows(ctypes.byref(o), ctypes.byref(p), _ptr(raw), None, None, None, _ptr(allzap), blk,
                             int(b0), int(nrows), _ptr(rows)):
        raise ValueError("or_clip_rows rejected its arguments")
    return rows


def clip_finish(obs, opts, raw, table, t0, n, mask=None, ptsperint=0, padvals=None, blk=None):
    """clip_times' recurrence over the summed exchange table -> (pad [nblk][nchan], clipped
    flags of spectra [t0, t0 + n), count clipped among them); raw holds those spectra."""
    blk = int(blk or obs.nsblk)
    nblk = (obs.N + blk - 1) // blk
    _, allzap = block_masks(obs, mask, ptsperint, blk=blk)
    pad = np.zeros((nblk, obs.nchan), np.float32)
    clipped = np.zeros(n, np.uint8)
    pv = None if padvals is None else np.ascontiguousarray(padvals, np.float32)
    table = np.ascontiguousarray(table, np.float64)
    raw = np.ascontiguousarray(raw, np.uint8)
    o, p = _obs(obs), _opts(opts)
    k = lib().or_clip_finish(ctypes.byref(o), ctypes.byref(p), _ptr(raw), None, None, None, _ptr(allzap), _ptr(pv),
                             blk, nblk, _ptr(table), int(t0), int(n), _ptr(pad), _ptr(clipped))
    if k < 0:
        raise ValueError("or_clip_finish rejected its arguments")
    return pad, clipped, int(k)


def stage1(obs, opts, raw, nsub, ds, subdm, t0=0, count=None, calib=(None, None, None),
           mask=None, ptsperint=0, padvals=None, omp=False, clean=None, dtint=0.0, zapint=None):
    """Subbands [nsub][count] for output samples [t0, t0+count)."""
    nds = obs.N // ds
    if count is None:
        count = nds - t0
    if clean is None:
        clean = prepare(obs, opts, raw, calib, mask, ptsperint, padvals, dtint, zapint, omp=omp)
    idd = chan_delays(obs, nsub, subdm)
    dt = np.int16 if opts.sub_dtype == 0 else np.float32
    out = np.zeros((nsub, count), dt)
    raw = np.ascontiguousarray(raw, np.uint8)
    cal = [None if c is None else np.ascontiguousarray(c, np.float32) for c in calib]
    o, p = _obs(obs), _opts(opts)
    rc = lib(omp).or_stage1(ctypes.byref(o), ctypes.byref(p), _ptr(raw), _ptr(cal[0]), _ptr(cal[1]), _ptr(cal[2]),
                            _ptr(clean.zap), _ptr(clean.pad), _ptr(clean.clipped), clean.blk, clean.nblk,
                            nsub, ds, _ptr(idd), int(t0), int(count), _ptr(out), int(count))
    if rc:
        raise ValueError("or_stage1 rejected its arguments")
    return out


def stage2(sub, off, t0=0, count=None, omp=False):
    """DM series [numdms][count] for samples [t0, t0+count) (no padding)."""
    sub = np.ascontiguousarray(sub)
    nsub, nds = sub.shape
    numdms = off.shape[0]
    if count is None:
        count = nds - t0
    out = np.zeros((numdms, count), np.float32)
    sd = 0 if sub.dtype == np.int16 else 1
    off = np.ascontiguousarray(off, np.int32)
    lib(omp).or_stage2(_ptr(sub), sd, nds, nds, nsub, _ptr(off), numdms, int(t0), int(count), _ptr(out), int(count))
    return out


def pad_series(out, nds, pad_mode):
    """Pad [numdms][numout] series in place past nds (or_pad)."""
    out = np.ascontiguousarray(out, np.float32)
    lib().or_pad(_ptr(out), out.shape[0], int(nds), out.shape[1], int(pad_mode))
    return out


def run_pass(obs, opts, raw, pp, calib=(None, None, None), mask=None, ptsperint=0, padvals=None, omp=False,
             clean=None, dtint=0.0, zapint=None):
    """Full pass -> (subbands [nsub][nds], series [numdms][numout]) exactly as the engine defines it."""
    nds = obs.N // pp.ds
    numout = pp.numout if pp.numout > 0 else nds
    sub = stage1(obs, opts, raw, pp.nsub, pp.ds, pp.subdm, calib=calib, mask=mask, ptsperint=ptsperint,
                 padvals=padvals, omp=omp, clean=clean, dtint=dtint, zapint=zapint)
    off = dm_offsets(obs, opts, pp.nsub, pp.ds, pp.lodm, pp.dmstep, pp.numdms)
    out = np.zeros((pp.numdms, numout), np.float32)
    n = min(numout, nds)
    out[:, :n] = stage2(sub, off, 0, n, omp=omp)
    lib(omp).or_pad(_ptr(out), pp.numdms, nds, numout, opts.pad_mode)
    return sub, out


def _nearest_long(x):
    return int(x - 0.5) if x < 0 else int(x + 0.5)       # PRESTO's NEAREST_LONG (truncating casts)


def bary_diffbins(topo, bary, tdt, dsdt):
    """prepsubband's add/remove-bin list [PRESTO-ext restatement, parity unpinned: PRESTO is not
    in the reference]: the barycentric - topocentric time of each TEMPO table point relative to
    the first, in output bins; between points ii-1 and ii every half-bin crossing of its nearest
    integer gives one entry, NEAREST_LONG of the crossing linearly interpolated onto the points'
    output-bin positions ((ii-1)*tdt/dsdt, ii*tdt/dsdt), negated when the difference falls.
    Reference call site: PALFA2_presto_search.py:514-520 (stage-2 prepsubband, no -nobary)."""
    SECPERDAY = 86400.0
    dtmp = bary[0] - topo[0]
    b = [((bary[i] - topo[i]) - dtmp) * SECPERDAY / dsdt for i in range(len(topo))]
    out = []
    oldbin = 0
    for ii in range(1, len(b)):
        currentbin = _nearest_long(b[ii])
        if currentbin != oldbin:
            if currentbin > 0:
                calcpt = oldbin + 0.5
                lobin = (ii - 1) * tdt / dsdt
                hibin = ii * tdt / dsdt
            else:
                calcpt = oldbin - 0.5
                lobin = -((ii - 1) * tdt / dsdt)
                hibin = -(ii * tdt / dsdt)
            while abs(calcpt) < abs(b[ii]):
                out.append(_nearest_long((calcpt - b[ii - 1]) * (hibin - lobin) / (b[ii] - b[ii - 1]) + lobin))
                calcpt = calcpt + 1.0 if currentbin > 0 else calcpt - 1.0
            oldbin = currentbin
    return np.array(out, np.int32)


def pad_values(topo, nds, pad_mode):
    """The padding value per DM of a [numdms][>= min(nds, numout)] topocentric series, as k_pad /
    or_pad define it: 1 zero; 2 (prepsubband's one avg) the first DM's sum / nds for every DM;
    0 each DM's own."""
    nd = topo.shape[0]
    if pad_mode == 1 or nds <= 0:
        return np.zeros(nd, np.float32)
    n = min(nds, topo.shape[1])
    sums = np.sum(topo[:, :n].astype(np.float64), axis=1)
    if pad_mode == 2:
        sums[:] = sums[0]
    return (sums / float(nds)).astype(np.float32)


def bary_series(topo, nvalid, numout, diffbins, padv):
    """Barycentred series [numdms][numout] from topocentric ones [numdms][>= nvalid], written
    sample by sample as prepsubband's output loop does: before topocentric sample |v| a
    padding sample (v > 0) or sample |v| dropped (v < 0); entries at or past nvalid unused;
    truncated to numout, then padded."""
    nd = topo.shape[0]
    out = np.empty((nd, numout), np.float32)
    for d in range(nd):
        col = []
        k = 0
        for t in range(nvalid):
            skip = False
            while k < len(diffbins) and abs(int(diffbins[k])) == t:
                if diffbins[k] > 0:
                    col.append(padv[d])
                else:
                    skip = True
                k += 1
            if not skip:
                col.append(topo[d, t])
            if len(col) >= numout:
                break
        col = col[:numout]
        out[d, :len(col)] = col
        out[d, len(col):] = padv[d]
    return out


def bary_data_end(nvalid, numout, diffbins):
    """Samples of real data at the head of a barycentred series (prepsubband's datawrote, the
    .inf on/off boundary): one past the output index of the last topocentric sample
    bary_series writes, counting the bins added before it."""
    n, k, end = 0, 0, 0
    for t in range(nvalid):
        skip = False
        while k < len(diffbins) and abs(int(diffbins[k])) == t:
            if diffbins[k] > 0:
                n += 1
            else:
                skip = True
            k += 1
        if n >= numout:
            break
        if not skip:
            n += 1
            end = n
        if n >= numout:
            break
    return end


def stats_padvals(dataavg):
    """determine_padvals from rfifind .stats interval averages [numint][numchan]."""
    a = np.ascontiguousarray(dataavg, np.float32)
    out = np.zeros(a.shape[1], np.float32)
    lib().or_stats_padvals(_ptr(a), a.shape[0], a.shape[1], _ptr(out))
    return out


def num_threads(omp=True):
    return lib(omp).or_num_threads()


# ---- single_pulse_search.py [PRESTO-ext] (sp_oracle.c + the script's candidate logic) ----
SP_HIT = np.dtype([("dm", "<i4"), ("bin", "<i4"), ("widx", "<i4"), ("pad", "<i4"), ("sigma", "<f8")])
SP_DOWNFACTS = [2, 3, 4, 6, 9, 14, 20, 30, 45, 70, 100, 150, 220, 300]


def sp_widths(dt, maxwidth):
    return [1] + [w for w in SP_DOWNFACTS if w * dt <= maxwidth]


def sp_hits(series, widths, threshold=5.0):
    """Boxcar hits of the [ndm][n] float32 series, sorted by (dm, widx, bin), and the bad
    blocks [ndm][n // 1000]."""
    x = np.ascontiguousarray(series, dtype=np.float32)
    ndm, n = x.shape
    w = np.asarray(widths, dtype=np.int32)
    nb = n // 1000
    bad = np.zeros((ndm, max(nb, 1)), np.uint8)
    L = lib(False)
    cap = 1 << 16
    while True:
        hits = np.zeros(cap, SP_HIT)
        cnt = L.sp_oracle_hits(_ptr(x), n, ndm, n, _ptr(w), len(w), float(threshold), _ptr(hits), cap, _ptr(bad))
        if cnt <= cap:
            break
        cap = int(cnt)
    hits = hits[:cnt]
    hits = hits[np.lexsort((hits["bin"], hits["widx"], hits["dm"]))]
    return hits, bad[:, :nb]


class SpCand:
    """candidate of single_pulse_search.py: DM, sigma, time, bin, downfact; ordered by bin."""

    def __init__(self, DM, sigma, time, bin, downfact):
        self.DM, self.sigma, self.time, self.bin, self.downfact = DM, sigma, time, bin, downfact

    def __str__(self):
        return "%7.2f %7.2f %13.6f %10d     %3d\n" % (self.DM, self.sigma, self.time, self.bin, self.downfact)


def prune_related1(bins, sig, downfact):
    """The script's prune_related1 greedy walk (sp_oracle.c, literal): bool mask of the kept
    entries of one (chunk, width) hit list in bin order."""
    bins = np.ascontiguousarray(bins, dtype=np.int32)
    sig = np.ascontiguousarray(sig, dtype=np.float64)
    rem = np.zeros(len(bins), np.uint8)
    if len(bins) > 1:
        lib(False).sp_prune_related1(_ptr(bins), _ptr(sig), len(bins), int(downfact), _ptr(rem))
    return rem == 0


def _prune_related2(cands, downfacts):
    toremove = set()
    maxd = max(downfacts) // 2 if downfacts else 0
    for ii in range(0, len(cands) - 1):
        if ii in toremove:
            continue
        xx = cands[ii]
        for jj in range(ii + 1, len(cands)):
            yy = cands[jj]
            if abs(yy.bin - xx.bin) > maxd:
                break
            if jj in toremove:
                continue
            prox = max([xx.downfact // 2, yy.downfact // 2, 1])
            if abs(yy.bin - xx.bin) <= prox:
                if xx.sigma > yy.sigma:
                    toremove.add(jj)
                else:
                    toremove.add(ii)
    for b in sorted(toremove, reverse=True):
        del cands[b]
    return cands


def _prune_border_cases(cands, offregions):
    toremove = set()
    for ii in range(len(cands) - 1, -1, -1):
        c = cands[ii]
        loside, hiside = c.bin - c.downfact // 2, c.bin + c.downfact // 2
        if hiside < offregions[0][0]:
            break
        for off, on in offregions:
            if hiside > off and loside < on:
                toremove.add(ii)
    for b in sorted(toremove, reverse=True):
        del cands[b]
    return cands


def sp_candidates(hits, bad, widths, dms, dt, nds=None, numout=None, ls=None):
    """single_pulse_search.py's per-DM candidate list from the raw hits (every boxcar value
    above threshold in [0, ls)), chunk by chunk (8000 samples) as the script builds it:
    width-1 hits outside bad blocks; per width > 1 the chunk's hits through prune_related1
    (the greedy walk) and then the script's `zip(hibins, hivals, hiblocks)` -- survivor m
    kept when the block of the m-th UNPRUNED hit is good; the list in bin order (widths
    ascending among equal bins: the script's append + bisect.insort), prune_related2 across
    widths and, for padded series, prune_border_cases.  -> [list of SpCand per DM]"""
    downfacts = list(widths[1:])
    out = []
    for d in range(len(dms)):
        hd = hits[hits["dm"] == d]
        kept = []
        for wi, w in enumerate(widths):
            hw = hd[hd["widx"] == wi]
            hw = hw[np.argsort(hw["bin"], kind="stable")]
            b_all = hw["bin"].astype(np.int64)
            if wi == 0:
                ok = bad[d][b_all // 1000] == 0 if bad.size else np.ones(len(hw), bool)
                kept += [(int(b), wi, float(v)) for b, v in zip(b_all[ok], hw["sigma"][ok])]
                continue
            chunk = b_all // 8000
            for c in np.unique(chunk):
                sel = chunk == c
                bins, sig = b_all[sel], hw["sigma"][sel]
                k = prune_related1(bins, sig, w)
                blocks = bins // 1000                               # hiblocks of the unpruned list
                for m, (b, v) in enumerate(zip(bins[k], sig[k])):
                    if not (bad.size and bad[d][blocks[m]]):
                        kept.append((int(b), wi, float(v)))
        kept.sort(key=lambda r: (r[0], r[1]))
        cl = [SpCand(dms[d], v, b * dt, b, widths[wi]) for b, wi, v in kept]
        cl = _prune_related2(cl, downfacts)
        if nds is not None and numout is not None and numout > nds and cl:
            cl = _prune_border_cases(cl, [(nds - 1, numout - 1)])
        out.append(cl)
    return out
