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


def write_dats(outbase, dmstrs, series, info_template: InfoData, nds):
    """series: [numdms][numout] float32.  Writes <outbase>_DM<dm>.dat/.inf per DM."""
    numout = series.shape[1]
    for dmstr, row in zip(dmstrs, series):
        base = dat_basename(outbase, dmstr)
        row.astype(np.float32, copy=False).tofile(base + ".dat")
        d = InfoData(**{**info_template.__dict__})
        d.name = os.path.basename(base)
        d.dm = float(dmstr)
        d.N = numout
        d.onoff = [0.0, float(nds - 1), float(numout - 1), float(numout - 1)] if numout > nds else []
        write_inf(base + ".inf", d)
