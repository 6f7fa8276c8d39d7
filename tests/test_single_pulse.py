"""CPU checks of the single_pulse_search.py restatement (oracle/sp_oracle.c + oracle.py):
an independent float64 numpy restatement of the script's numeric steps agrees with the
oracle's hits away from the threshold, injected pulses come out as single candidates at
their bin and width, and the candidate bookkeeping follows the script (pruning, bad blocks,
padding).  Parity with PRESTO itself is unpinned (the script is not in this image)."""
import numpy as np
import pytest

import oracle as OR


def numpy_hits(x, widths, threshold):
    """Float64 restatement: np.polyfit line per block, sorted middle-95% std * 1.148, the
    bad-block rule, boxcars by cumulative sums over [0, numchunks*8000)."""
    n = x.shape[0]
    nb = n // 1000
    ls = nb * 1000 // 8000 * 8000
    t = np.arange(1000, dtype=np.float64)
    y = np.zeros(ls)
    stds = np.zeros(nb)
    det = np.zeros((nb, 1000))
    for b in range(nb):
        blk = x[b * 1000:(b + 1) * 1000].astype(np.float64)
        p = np.polyfit(t, blk, 1)
        det[b] = blk - np.polyval(p, t)
        s = np.sort(det[b])[25:975]
        stds[b] = np.sqrt((s ** 2).sum() / 950.0) * 1.148
    srt = np.sort(stds)
    h = nb // 2
    locut = int(np.argmax(srt[1:h + 1] - srt[:h])) + 1
    hicut = int(np.argmax(srt[h + 1:] - srt[h:-1])) + h - 2
    bad = np.zeros(nb, bool)
    if hicut > locut:
        sd = srt[locut:hicut].std()
        med = srt[(locut + hicut) // 2]
        bad = (stds < med - 4 * sd) | (stds > med + 4 * sd)
    for b in range(min(nb, ls // 1000)):
        if not bad[b] and stds[b] > 0:
            y[b * 1000:(b + 1) * 1000] = det[b] / stds[b]
    cs = np.concatenate([[0.0], np.cumsum(y)])
    out = {}
    for wi, w in enumerate(widths):
        if w == 1:
            s = y
        else:
            lo = np.arange(ls) - w // 2
            hi = np.arange(ls) + (w // 2 if w % 2 else w // 2 - 1) + 1
            s = (cs[np.clip(hi, 0, ls)] - cs[np.clip(lo, 0, ls)]) / np.sqrt(w)
        out[wi] = s
    return out, bad


def test_widths():
    assert OR.sp_widths(65.476e-6, 0.1) == [1, 2, 3, 4, 6, 9, 14, 20, 30, 45, 70, 100, 150, 220, 300]
    assert OR.sp_widths(65.476e-6 * 10, 0.1) == [1, 2, 3, 4, 6, 9, 14, 20, 30, 45, 70, 100, 150]
    assert OR.sp_widths(1e-3, 0.005) == [1, 2, 3, 4]


def test_oracle_hits_match_numpy_restatement():
    rng = np.random.default_rng(7)
    n = 64000 + 517
    x = rng.normal(100.0, 7.0, size=(2, n)).astype(np.float32)
    x[0, 20000:20030] += 40.0                       # a 30-sample pulse
    x[1, 5000:6000] += rng.normal(0, 60.0, 1000)    # a noisy (bad) block
    x[1, 40001] += 90.0                             # a one-sample spike
    widths = OR.sp_widths(65.476e-6, 0.1)
    hits, bad = OR.sp_hits(x, widths, 3.0)
    for d in range(2):
        ref, rbad = numpy_hits(x[d], widths, 3.0)
        assert np.array_equal(bad[d].astype(bool), rbad)
        hd = hits[hits["dm"] == d]
        for wi in range(len(widths)):
            got = hd[hd["widx"] == wi]
            s = ref[wi]
            # the oracle rounds detrended and normalised samples to float32 (as the script's
            # float32 arrays do): agreement to float32 precision
            np.testing.assert_allclose(got["sigma"], s[got["bin"]], rtol=2e-6, atol=2e-6)
            clear = np.flatnonzero(s > 3.0 + 1e-4)      # away from the threshold: the same set
            assert set(clear.tolist()) <= set(got["bin"].tolist())
            assert len(got) - len(clear) <= np.count_nonzero(np.abs(s - 3.0) <= 1e-4)
    assert bad[1, 5] == 1                            # the noisy block is flagged


def test_candidates_find_injected_pulses():
    rng = np.random.default_rng(11)
    n = 80000
    x = rng.normal(50.0, 5.0, size=(3, n)).astype(np.float32)
    x[1, 30000:30020] += 12.0                         # 20-sample pulse, ~10.7 sigma boxcar
    x[2, 60000] += 45.0                                # 1-sample spike, 9 sigma
    widths = OR.sp_widths(65.476e-6, 0.1)
    hits, bad = OR.sp_hits(x, widths, 5.0)
    cl = OR.sp_candidates(hits, bad, widths, [10.0, 20.0, 30.0], 65.476e-6)
    strong = [[c for c in l if c.sigma > 7.0] for l in cl]
    assert strong[0] == []
    assert len(strong[1]) == 1 and abs(strong[1][0].bin - 30010) <= 3 and strong[1][0].downfact in (14, 20, 30)
    assert len(strong[2]) == 1 and strong[2][0].bin == 60000 and strong[2][0].downfact == 1
    line = str(strong[2][0])
    assert line == "%7.2f %7.2f %13.6f %10d     %3d\n" % (30.0, strong[2][0].sigma, 60000 * 65.476e-6, 60000, 1)


def test_candidate_bookkeeping_follows_script():
    """prune_related1 within a width (the greedy walk), the script's bad-block zip (survivor m
    takes the block of the m-th unpruned hit), prune_related2 across widths and border
    pruning on a padded series, on a hand-made hit list."""
    rows = [(0, 100, 0, 6.0), (0, 5000, 0, 5.5),                 # width 1
            (0, 101, 1, 7.0), (0, 102, 1, 6.5),                 # width 2: 102 within 1 of 101 -> pruned
            (0, 2990, 2, 8.0), (0, 2991, 2, 8.5), (0, 4000, 2, 6.0),   # width 3, blocks 2, 2, 4
            (0, 7990, 1, 9.0), (0, 7999, 2, 9.5)]               # near the padding
    hits = np.zeros(len(rows), OR.SP_HIT)
    for i, r in enumerate(rows):
        hits[i]["dm"], hits[i]["bin"], hits[i]["widx"], hits[i]["sigma"] = r
    bad = np.zeros((1, 8), np.uint8)
    bad[0, 2] = 1
    cl = OR.sp_candidates(hits, bad, [1, 2, 3], [5.0], 1e-3, nds=7995, numout=8000)[0]
    got = [(c.bin, c.downfact) for c in cl]
    # width 3: 2990 loses to 2991; the survivors 2991, 4000, 7999 are zipped with the blocks
    # of the unpruned hits 2990, 2991, 4000 -> blocks 2, 2, 4: 2991 and 4000 both read the bad
    # block 2 (the script's quirk), 7999 reads block 4 and reaches the padding after
    # nds - 1 = 7994; 100 (w1, 6.0) loses to 101 (w2, 7.0) within max(1, 1, 1)
    assert got == [(101, 2), (5000, 1), (7990, 2)]


def greedy_walk(bins, vals, downfact):
    """prune_related1 of single_pulse_search.py, transcribed (kept bins)."""
    gone = set()
    for ii in range(len(bins) - 1):
        if ii in gone:
            continue
        for jj in range(ii + 1, len(bins)):
            if abs(bins[jj] - bins[ii]) > downfact // 2:
                break
            if jj in gone:
                continue
            if vals[ii] > vals[jj]:
                gone.add(jj)
            else:
                gone.add(ii)
    return [b for k, b in enumerate(bins) if k not in gone]


def pivot_walk(bins, vals, downfact):
    """The O(n) form hd_sp.hip's k_sp_hits walks: a hit is a pivot unless the last pivot
    lies within h = downfact // 2 bins and is strictly stronger; a pivot is kept when the
    next pivot lies more than h bins after it (or there is none)."""
    h = downfact // 2
    out, lp = [], None
    for b, x in zip(bins, vals):
        if lp is not None and b - lp[0] <= h and lp[1] > x:
            continue
        if lp is not None and b - lp[0] > h:
            out.append(lp[0])
        lp = (b, x)
    if lp is not None:
        out.append(lp[0])
    return out


def _hit_lists(rng):
    """Hit lists of one (chunk, width): random sparse/dense bins, monotone chains, wide humps,
    plateaus with ties, trains of pulses closer than the width."""
    kind = rng.integers(0, 5)
    n = int(rng.integers(1, 400))
    if kind == 0:                                              # random bins, random values
        bins = np.sort(rng.choice(2000, size=min(n, 2000), replace=False))
        vals = rng.normal(7.0, 1.0, len(bins)).round(int(rng.integers(0, 3)))
    elif kind == 1:                                            # one falling / rising chain
        bins = np.arange(n) + 5
        vals = 10.0 - 0.01 * np.arange(n) if rng.integers(0, 2) else 5.0 + 0.01 * np.arange(n)
    elif kind == 2:                                            # humps longer than the width
        c = np.arange(n)
        vals = 8.0 + 3.0 * np.sin(c / rng.uniform(2.0, 40.0)) ** 2
        bins = c[vals > 8.5]
        vals = vals[vals > 8.5]
    elif kind == 3:                                            # plateaus: many equal values
        bins = np.sort(rng.choice(600, size=min(n, 600), replace=False))
        vals = rng.integers(5, 8, len(bins)).astype(np.float64)
    else:                                                      # a pulse train, gaps in it
        per = int(rng.integers(2, 80))
        c = np.arange(2000)
        vals = 6.0 + 4.0 * np.exp(-((c % per) - per / 2) ** 2 / rng.uniform(0.5, 30.0)) + rng.normal(0, 0.3, c.size)
        bins, vals = c[vals > 7.0], vals[vals > 7.0]
    return [int(b) for b in bins], [float(v) for v in vals]


def test_prune_related1_walks_agree():
    """The script's walk (transcribed here), the oracle's C transcription and the device's
    O(n) pivot form keep the same hits on monotone chains, wide humps, ties, dense trains."""
    rng = np.random.default_rng(5)
    for trial in range(600):
        w = int(rng.choice([2, 3, 4, 6, 9, 14, 20, 30, 45, 70, 100, 150, 220, 300]))
        bins, vals = _hit_lists(rng)
        want = greedy_walk(bins, vals, w)
        keep = OR.prune_related1(np.array(bins, np.int32), np.array(vals), w)
        assert [b for b, k in zip(bins, keep) if k] == want, (trial, w)
        assert pivot_walk(bins, vals, w) == want, (trial, w)
    # the advisor's example: 10, 9, 8 at consecutive bins with downfact 2 keeps bins 0 and 2
    assert greedy_walk([0, 1, 2], [10.0, 9.0, 8.0], 2) == [0, 2] == pivot_walk([0, 1, 2], [10.0, 9.0, 8.0], 2)


def segment_walk(bins, vals, downfact, seg=128):
    """The parallel form of k_sp_hits's walk (csrc/hd_sp.hip): next(p) = the first hit q > p
    with q - p > h or x_q >= x_p; p is kept when that step is a gap or p is last.  Each
    segment of `seg` bins walks its own chain from its first hit (spec pivots, keep flags,
    exit = first pivot past the segment); the true chain from the first hit jumps to a
    segment's exit as soon as it reaches one of that segment's spec pivots (merge) and walks
    only the pivots before.  Kept = spec pivots at or after the merge with the keep flag,
    plus the kept pivots the true chain walked itself."""
    h = downfact // 2
    n = len(bins)
    pos = {b: k for k, b in enumerate(bins)}

    def nxt(k):
        for j in range(k + 1, n):
            if bins[j] - bins[k] > h or vals[j] >= vals[k]:
                return j
        return -1

    nseg = (bins[-1] // seg + 1) if n else 0
    spec, keepf, exitp = set(), set(), {}
    for sg in range(nseg):
        members = [k for k in range(n) if bins[k] // seg == sg]
        if not members:
            continue
        k = members[0]
        exitp[sg] = -1
        while True:
            spec.add(k)
            q = nxt(k)
            if q < 0 or bins[q] - bins[k] > h:
                keepf.add(k)
            if q < 0:
                break
            k = q
            if bins[k] // seg != sg:
                exitp[sg] = k
                break
    merge, extra = {}, set()
    k = 0 if n else -1
    while k >= 0:
        sg = bins[k] // seg
        if k in spec:
            merge[sg] = bins[k]
            k = exitp[sg]
            continue
        q = nxt(k)
        if q < 0 or bins[q] - bins[k] > h:
            extra.add(k)
        k = q
    kept = {k for k in spec & keepf if bins[k] >= merge.get(bins[k] // seg, 1 << 30)} | extra
    assert all(bins[k] in pos for k in kept)
    return [bins[k] for k in sorted(kept)]


def test_prune_related1_segment_form_agrees():
    """The segmented, merge-based walk of the device kernel keeps the same hits as the
    script's greedy walk: random lists, monotone chains (where the true and speculative chains
    run in step without meeting), humps, ties and pulse trains, at 128-bin segments and at
    tiny segments (many merges), over every downfactor."""
    rng = np.random.default_rng(11)
    for trial in range(400):
        w = int(rng.choice([2, 3, 4, 6, 9, 14, 20, 30, 45, 70, 100, 150, 220, 300]))
        bins, vals = _hit_lists(rng)
        want = greedy_walk(bins, vals, w)
        for seg in (128, 8):
            assert segment_walk(bins, vals, w, seg) == want, (trial, w, seg)


@pytest.mark.parametrize("padded", [False, True])
def test_host_prune_matches_script(padded):
    """hd_sp_prune (the host half of hd_single_pulse: grouping by DM, bin order, prune_related2
    visiting only the pairs that can act, border cases) keeps exactly the script's candidates
    (oracle._prune_related2 / _prune_border_cases) on dense and sparse multi-width hit sets
    with ties and equal bins.  Host only: no device is touched."""
    import ctypes
    from hipdedisp import _lib
    from hipdedisp.single_pulse import HIT
    L = _lib.load()
    widths = [1, 2, 3, 4, 6, 9, 14, 20, 30, 45, 70, 100, 150, 220, 300]
    rng = np.random.default_rng(3 + padded)
    for trial in range(42):
        ndm = int(rng.integers(1, 5))
        nds = 20000 if trial < 40 else 4_000_000             # the last two: > 64 Ki hits (threaded grouping)
        numout = nds + 3000 if padded else nds
        n = int(rng.integers(0, 4000)) if trial < 40 else 150_000
        h = np.zeros(n, HIT)
        h["dm"] = rng.integers(0, ndm, n)
        dense = rng.integers(0, 2)
        h["bin"] = rng.integers(0, 600 if dense else nds, n) + (nds - 600 if padded and dense else 0)
        h["widx"] = rng.integers(0, len(widths), n)
        h["sigma"] = rng.normal(7.0, 1.0, n).round(int(rng.integers(0, 3)))   # ties
        # the device emits each (dm, bin, width) once
        _, first = np.unique(h[["dm", "bin", "widx"]], return_index=True)
        h = h[np.sort(first)]
        want = []
        for d in range(ndm):
            hd = h[h["dm"] == d]
            hd = hd[np.lexsort((hd["widx"], hd["bin"]))]
            cl = [OR.SpCand(float(d), float(r["sigma"]), float(r["bin"]), int(r["bin"]), widths[r["widx"]]) for r in hd]
            cl = OR._prune_related2(cl, widths[1:])
            if padded and cl:
                cl = OR._prune_border_cases(cl, [(nds - 1, numout - 1)])
            want += [(d, c.bin, c.downfact, c.sigma) for c in cl]
        a = np.ascontiguousarray(h)
        w = (ctypes.c_int32 * len(widths))(*widths)
        nk = ctypes.c_int64()
        rc = L.hd_sp_prune(a.ctypes.data_as(ctypes.c_void_p), len(a), ndm, w, len(widths), nds, numout,
                           ctypes.byref(nk))
        assert rc == 0
        got = [(int(r["dm"]), int(r["bin"]), widths[r["widx"]], float(r["sigma"])) for r in a[:nk.value]]
        assert got == want, trial


def test_block_sort_int_keys_preserve_float_order():
    """csrc/hd_sp.hip k_sp_blocks sorts the detrended f32 values as int32 keys
    b ^ ((b >> 31) & 0x7FFFFFFF) (complemented keys for descending lanes): the key order is
    the float order (-0 just below +0, infinities at the ends), the map is its own inverse
    and complementing a key reverses the order -- so the sorted values, and the trimmed sum
    of squares taken over them, equal a float sort's."""
    rng = np.random.default_rng(5)
    v = np.concatenate([rng.normal(0, 3, 5000), rng.normal(0, 1e-30, 50), [0.0, -0.0, np.inf, -np.inf, 7.0, 7.0]])
    v = v.astype(np.float32)
    b = v.view(np.int32)
    key = b ^ ((b >> 31) & np.int32(0x7FFFFFFF))
    assert np.array_equal((key ^ ((key >> 31) & np.int32(0x7FFFFFFF))).view(np.float32).view(np.int32), b)
    by_key = v[np.argsort(key, kind="stable")]
    assert np.array_equal(by_key, np.sort(v))                 # same values in the same order
    assert np.all(np.diff(by_key.astype(np.float64)) >= 0)
    assert np.all(np.diff(np.sort(~key)) >= 0) and np.array_equal(np.sort(v)[::-1], v[np.argsort(~key, kind="stable")])
    i = np.flatnonzero(v == 0.0)
    neg0, pos0 = i[np.signbit(v[i])], i[~np.signbit(v[i])]
    assert key[neg0][0] < key[pos0][0]
