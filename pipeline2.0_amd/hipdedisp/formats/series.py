"""Subband (.subNN + .sub.inf) and dedispersed (.dat + .inf) file I/O.

Names follow the reference exactly:
  stage-1 output  tmp/subbands/<base>_DM<subdm>.subNN   (PALFA2_presto_search.py:498,506-507,515)
  stage-2 output  tmp/<base>_DM<dm %.2f>.dat / .inf       (:532-537)
.subNN hold native int16 (or float32 with sub_dtype=f32) samples [PRESTO-ext]; .dat hold
native float32 samples with no header.
"""
import glob
import os
import re

import numpy as np

from .inf import InfoData, read_inf, write_inf


def sub_suffix(nsub, i):
    return ".sub%02d" % i if nsub <= 100 else ".sub%04d" % i


def write_subbands(subbase, sub, info: InfoData):
    """sub: [nsub][nds]; writes <subbase>.subNN and <subbase>.sub.inf."""
    nsub = sub.shape[0]
    for i in range(nsub):
        sub[i].tofile(subbase + sub_suffix(nsub, i))
    write_inf(subbase + ".sub.inf", info)


def read_subbands(paths, dtype=np.int16):
    """Read the files matched by the stage-2 glob (`.sub[0-9]*`), ordered by index."""
    def idx(p):
        m = re.search(r"\.sub(\d+)$", p)
        return int(m.group(1)) if m else -1
    paths = sorted((p for p in paths if idx(p) >= 0), key=idx)
    if not paths:
        raise FileNotFoundError("no subband files")
    arrs = [np.fromfile(p, dtype=dtype) for p in paths]
    n = min(len(a) for a in arrs)
    base = re.sub(r"\.sub\d+$", "", paths[0])
    info = read_inf(base + ".sub.inf") if os.path.exists(base + ".sub.inf") else None
    return np.stack([a[:n] for a in arrs]), info


def dat_basename(outbase, dmstr):
    return "%s_DM%s" % (outbase, dmstr)


def write_infs(outbase, dmstrs, info_template: InfoData, nds, numout):
    """<outbase>_DM<dm>.inf per DM (the padded tail recorded as an on/off break)."""
    for dmstr in dmstrs:
        base = dat_basename(outbase, dmstr)
        d = InfoData(**{**info_template.__dict__})
        d.name = os.path.basename(base)
        d.dm = float(dmstr)
        d.N = numout
        d.onoff = [0.0, float(nds - 1), float(numout - 1), float(numout - 1)] if numout > nds else []
        write_inf(base + ".inf", d)


def write_dats(outbase, dmstrs, series, info_template: InfoData, nds):
    """series: [numdms][numout] float32 on the host.  Writes <outbase>_DM<dm>.dat/.inf per DM."""
    for dmstr, row in zip(dmstrs, series):
        row.astype(np.float32, copy=False).tofile(dat_basename(outbase, dmstr) + ".dat")
    write_infs(outbase, dmstrs, info_template, nds, series.shape[1])


def write_dats_device(plan, outbase, dmstrs, info_template: InfoData, nds, wait=True):
    """The device-resident series of plan (after run_dedisp(to_host=False)) straight to
    <outbase>_DM<dm>.dat through the library's pinned-buffer writer threads
    (hd_write_series), the .inf files meanwhile from here."""
    plan.write_series([dat_basename(outbase, d) + ".dat" for d in dmstrs], wait=False)
    write_infs(outbase, dmstrs, info_template, nds, plan.numout)
    if wait:
        plan.eng.wait_writes()
