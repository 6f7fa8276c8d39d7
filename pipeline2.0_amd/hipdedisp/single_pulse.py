"""single_pulse_search.py on the device-resident series of a pass.

The reference runs, for every .dat a pass writes (lib/python/PALFA2_presto_search.py:539-546):

    single_pulse_search.py -p -m <singlepulse_maxwidth> -t <singlepulse_threshold> <base>_DM<dm>.dat

(maxwidth 0.1 s, threshold 5.0: lib/python/config/searching_example.py:13-15), adds the
wall time to job.singlepulse_time and moves <base>_DM<dm>.singlepulse to the work dir.  Here
the whole search runs in libhipdedisp over the series still in HBM (hd_single_pulse):
per-block detrend and trimmed std, bad blocks, normalisation, the boxcar hits of every
downfactor, prune_related1 (the script's greedy walk per 8000-sample chunk and width) and its
bad-block test on the GPU (csrc/hd_sp.hip), prune_related2 and the border cases on the host
(csrc/hd_api.hip, one thread per DM).  This module turns the candidates into the script's
`.singlepulse` text: "# DM      Sigma      Time (s)     Sample    Downfact" and one
"%7.2f %7.2f %13.6f %10d     %3d" line per candidate (the file exists, empty, when a DM has
none).  [PRESTO-ext] restated; there is no CPU fallback.
"""
import ctypes
import os
import time

import numpy as np

from . import _lib
from .engine import PrestoError

HIT = np.dtype([("dm", "<i4"), ("bin", "<i4"), ("widx", "<i4"), ("pad", "<i4"), ("sigma", "<f8")])
HEADER = "# DM      Sigma      Time (s)     Sample    Downfact\n"


class Candidate:
    """One single-pulse candidate (the script's `candidate`: compared by bin)."""
    __slots__ = ("DM", "sigma", "time", "bin", "downfact")

    def __init__(self, DM, sigma, time, bin, downfact):
        self.DM, self.sigma, self.time, self.bin, self.downfact = DM, sigma, time, bin, downfact

    def line(self):
        return "%7.2f %7.2f %13.6f %10d     %3d\n" % (self.DM, self.sigma, self.time, self.bin, self.downfact)

    def key(self):
        return (self.bin, self.downfact, round(self.sigma, 9))


def widths(dt, maxwidth):
    """[1] + the script's downfactors with width * dt <= maxwidth (hd_sp_widths)."""
    L = _lib.load()
    w = (ctypes.c_int32 * 16)()
    n = ctypes.c_int32()
    if L.hd_sp_widths(float(dt), float(maxwidth), w, ctypes.byref(n)) != 0:
        raise ValueError("hd_sp_widths: dt must be > 0")
    return [int(w[i]) for i in range(n.value)]


def _collect(plan):
    """hd_single_pulse_collect of the plan's launched search: (HIT records sorted by (dm, bin,
    widx), bad[numdms][nblocks])."""
    eng = plan.eng
    nb = plan.numout // 1000
    bad = np.zeros((plan.pp.numdms, max(nb, 1)), np.uint8)
    cap = getattr(eng, "_sp_cap", 1 << 20)                   # room for the device hits (pre prune_related2)
    while True:
        hits = np.empty(cap, HIT)
        n, nbk = ctypes.c_int64(), ctypes.c_int64()
        rc = eng._L.hd_single_pulse_collect(plan._p, hits.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(n),
                                            bad.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ctypes.byref(nbk))
        if rc == _lib.HD_E_NOMEM and n.value > cap:           # room for every device hit
            cap = int(n.value) + int(n.value) // 4
            eng._sp_cap = cap
            continue
        eng._chk(rc, "single_pulse_search.py")
        return hits[:n.value], bad[:, :nb]


def _launch(plan, dt, maxwidth, threshold):
    plan.eng._chk(plan.eng._L.hd_single_pulse_launch(plan._p, float(dt), float(maxwidth), float(threshold)),
                  "single_pulse_search.py")


def device_candidates(plan, dt, maxwidth=0.1, threshold=5.0):
    """(candidates sorted by (dm, bin, widx) as HIT records, bad[numdms][nblocks]) of the
    plan's series (hd_single_pulse)."""
    _launch(plan, dt, maxwidth, threshold)
    return _collect(plan)


def device_candidates_many(plans, maxwidth=0.1, threshold=5.0, depth=4):
    """device_candidates of several plans (each at its own sub_dt), yielded in order as
    (plan, hits, bad): the device searches of the next `depth` plans are queued before a
    plan's hits are pruned on the host, so both halves run at once."""
    plans = list(plans)
    for k in range(min(depth, len(plans))):
        _launch(plans[k], plans[k].sub_dt, maxwidth, threshold)
    for i, p in enumerate(plans):
        if i + depth < len(plans):
            q = plans[i + depth]
            _launch(q, q.sub_dt, maxwidth, threshold)
        hits, bad = _collect(p)
        yield p, hits, bad


def candidates(hits, wlist, dm_values, dt):
    """Per-DM lists of Candidate from the library's records."""
    out = [[] for _ in dm_values]
    for r in hits.tolist():
        d, b, wi, _, sig = r
        out[d].append(Candidate(dm_values[d], sig, b * dt, b, wlist[wi]))
    return out


def write_singlepulse(path, cands):
    with open(path, "w") as f:
        if cands:
            f.write(HEADER)
            f.writelines(c.line() for c in cands)


def search_plan(plan, dm_strs, maxwidth=0.1, threshold=5.0):
    """Candidate lists of every DM of the plan's last hd_run_dedisp (series on device)."""
    dt = plan.sub_dt
    hits, _ = device_candidates(plan, dt, maxwidth, threshold)
    return candidates(hits, widths(dt, maxwidth), [float(s) for s in dm_strs], dt)


def run_single_pulse(plan, basenm, dm_strs, workdir=None, maxwidth=0.1, threshold=5.0):
    """PALFA2_presto_search.py:539-546 for one pass: `<basenm>_DM<dm>.singlepulse` per DM
    (moved to workdir when given, as :545 does); returns (seconds, candidate lists), the
    seconds being what the reference adds to job.singlepulse_time."""
    t0 = time.time()
    try:
        lists = search_plan(plan, dm_strs, maxwidth, threshold)
    except PrestoError:
        raise
    except Exception as e:                                    # library errors surface as PrestoError
        raise PrestoError("single_pulse_search.py failed: %s" % e)
    for s, cl in zip(dm_strs, lists):
        path = "%s_DM%s.singlepulse" % (basenm, s)
        if workdir:
            path = os.path.join(workdir, os.path.basename(path))
        write_singlepulse(path, cl)
    return time.time() - t0, lists
