"""Python view of the engine: contexts (one GPU each) and per-pass plans.

Errors are raised as PrestoError, the exception the reference's search driver
raises when a PRESTO program fails (lib/python/PALFA2_presto_search.py:740-744,
raised at :123-128), so callers' retry/cleanup semantics are unchanged.
"""
import ctypes
import os
import weakref
from dataclasses import dataclass, field
from typing import Optional

import numpy as np

from . import _lib
from ._lib import hd_obs, hd_opts, hd_pass, hd_synth


class PrestoError(Exception):
    """Error raised when a dedispersion step fails (reference: PALFA2_presto_search.py:740)."""


def _check(rc, what, ctx=None):
    if rc != _lib.HD_OK:
        raise PrestoError("Execution of command (%s) failed with status (%s)! %s"
                          % (what, _lib.ERROR_NAMES.get(rc, rc), _lib.last_error(ctx)))


@dataclass
class ObsParams:
    """Observation parameters (reference: lib/python/formats/psrfits.py:116-134, 210-314)."""
    nchan: int
    nbits: int
    dt: float
    lofreq: float          # MHz, lowest-frequency channel centre (after flip)
    df: float              # MHz, > 0
    N: int
    nsblk: int = 2048
    flip: bool = False     # raw channel order descending in frequency
    npol: int = 1
    voverc: float = 0.0

    @property
    def rowbytes(self):
        return self.nchan * self.nbits // 8

    def to_c(self):
        return hd_obs(nchan=self.nchan, nbits=self.nbits, npol=self.npol, flip=int(bool(self.flip)),
                      dt=self.dt, lofreq=self.lofreq, df=self.df, N=int(self.N),
                      nsblk=self.nsblk, voverc=self.voverc)


@dataclass
class Opts:
    """PRESTO-semantics switches; defaults mirror the reference's use:
    the stage-1 command (PALFA2_presto_search.py:506-511) passes no -noclip, so
    prepsubband's default -clip 6 applies; downsampling averages, int16 subbands are
    (short)(x + 0.5), padding is the first DM's running mean."""
    sub_dtype: int = _lib.HD_SUB_I16
    ds_mode: int = _lib.HD_DS_MEAN
    pad_mode: int = _lib.HD_PAD_DM0
    nibble_hi_first: bool = True
    be16: bool = True
    inf_roundtrip: bool = True
    clip_sigma: float = 6.0
    sub_round: int = _lib.HD_ROUND_PRESTO

    def to_c(self):
        return hd_opts(sub_dtype=self.sub_dtype, ds_mode=self.ds_mode, pad_mode=self.pad_mode,
                       nibble_hi_first=int(self.nibble_hi_first), be16=int(self.be16),
                       inf_roundtrip=int(self.inf_roundtrip), clip_sigma=self.clip_sigma,
                       sub_round=self.sub_round)


@dataclass
class PassParams:
    """One prepsubband pass (the two calls at PALFA2_presto_search.py:506-520)."""
    subdm: float
    lodm: float
    dmstep: float
    numdms: int
    nsub: int
    ds: int
    numout: int = 0
    sub_input: bool = False   # stage-2-only run on .subNN files (obs describes the .sub.inf)

    def to_c(self):
        return hd_pass(subdm=self.subdm, lodm=self.lodm, dmstep=self.dmstep, numdms=self.numdms,
                       nsub=self.nsub, ds=self.ds, numout=int(self.numout),
                       flags=_lib.HD_PASS_SUB_INPUT if self.sub_input else 0)


def device_count():
    n = ctypes.c_int(0)
    _check(_lib.load().hd_device_count(ctypes.byref(n)), "hd_device_count")
    return n.value


def plan_tables(obs: "ObsParams", opts: "Opts", pp: "PassParams"):
    """Host-only integer tables of a pass (no device needed):
    (idispdt [nchan], offsets [numdms][nsub], (sub_lofreq, sub_chanwid, sub_dt))."""
    L = _lib.load()
    idd = np.zeros(obs.nchan, np.int32)
    off = np.zeros((pp.numdms, pp.nsub), np.int32)
    a, b, c = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    o, p, q = obs.to_c(), (opts or Opts()).to_c(), pp.to_c()
    I32 = ctypes.POINTER(ctypes.c_int32)
    _check(L.hd_plan_tables(ctypes.byref(o), ctypes.byref(p), ctypes.byref(q), idd.ctypes.data_as(I32),
                            off.ctypes.data_as(I32), ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
           "hd_plan_tables")
    return idd, off, (a.value, b.value, c.value)


def plan_extents(obs: "ObsParams", opts: "Opts", pp: "PassParams"):
    """Host-only DMA extent check of the stage-2 kernels a plan would build (hd_plan_extents):
    a list of dicts {kernel, region ('subbands' | 'offsets'), ppc, reach, size} in bytes."""
    L = _lib.load()
    o, p, q = obs.to_c(), (opts or Opts()).to_c(), pp.to_c()
    n = ctypes.c_int32(0)
    _check(L.hd_plan_extents(ctypes.byref(o), ctypes.byref(p), ctypes.byref(q), None, 0, ctypes.byref(n)),
           "hd_plan_extents")
    buf = (_lib.hd_extent * max(n.value, 1))()
    _check(L.hd_plan_extents(ctypes.byref(o), ctypes.byref(p), ctypes.byref(q), buf, len(buf), ctypes.byref(n)),
           "hd_plan_extents")
    names = {_lib.HD_EXT_SUBBANDS: "subbands", _lib.HD_EXT_OFFSETS: "offsets"}
    return [dict(kernel=x.kernel, region=names[x.region], ppc=x.ppc, reach=x.reach, size=x.size)
            for x in buf[:n.value]]


def bary_diffbins(topo, bary, tdt, dsdt):
    """prepsubband's add/remove-bin list [PRESTO-ext] from a TEMPO table (hd_bary_diffbins;
    host only): topo/bary MJDs spaced tdt s, output sample time dsdt s.  int32 array, > 0 =
    a padding bin before topocentric sample v, < 0 = sample -v removed."""
    t = np.ascontiguousarray(topo, dtype=np.float64)
    b = np.ascontiguousarray(bary, dtype=np.float64)
    if t.shape != b.shape or t.ndim != 1:
        raise PrestoError("topo and bary must be 1-D arrays of the same length")
    L = _lib.load()
    D = ctypes.POINTER(ctypes.c_double)
    I32 = ctypes.POINTER(ctypes.c_int32)
    n = ctypes.c_int32(0)
    rc = L.hd_bary_diffbins(t.ctypes.data_as(D), b.ctypes.data_as(D), len(t), float(tdt), float(dsdt), None, 0,
                            ctypes.byref(n))
    if rc and n.value == 0:                       # bad arguments (the count query itself fails)
        _check(rc, "hd_bary_diffbins")
    cap = max(n.value, 1)
    out = np.zeros(cap, np.int32)
    _check(L.hd_bary_diffbins(t.ctypes.data_as(D), b.ctypes.data_as(D), len(t), float(tdt), float(dsdt),
                              out.ctypes.data_as(I32), cap, ctypes.byref(n)), "hd_bary_diffbins")
    return out[:n.value]


def stats_padvals(dataavg):
    """determine_padvals [PRESTO-ext] from rfifind .stats interval averages [numint][numchan]
    (hd_stats_padvals; host only)."""
    a = np.ascontiguousarray(dataavg, dtype=np.float32)
    out = np.zeros(a.shape[1], np.float32)
    _check(_lib.load().hd_stats_padvals(_f32p(a), a.shape[0], a.shape[1], _f32p(out)), "hd_stats_padvals")
    return out


def _f32p(a):
    if a is None:
        return None
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class Engine:
    """One device context (hd_ctx).  device = _lib.HD_HOST_ONLY opens a context bound to no
    device (host tables only; for life-cycle tests without a GPU)."""

    def __init__(self, device=0):
        self._L = _lib.load()
        self._ctx = ctypes.c_void_p()
        _check(self._L.hd_open(device, ctypes.byref(self._ctx)), "hd_open(%d)" % device)
        self.device = device
        self.obs: Optional[ObsParams] = None
        self.opts: Optional[Opts] = None
        self._keep = []
        self._plans = weakref.WeakSet()     # live plans: destroyed before the context

    # -- lifecycle --
    def close(self, check=True):
        """Destroy the live plans, then the context.  After a device fault (a sticky HIP error
        an earlier call already reported) both make no device call and return HD_E_HIP, which
        is raised here as PrestoError when check is true -- the process stays alive, so the
        caller's failure path runs (the job pool retries the beam, job.py:140-165)."""
        if not self._ctx:
            return
        first = None
        for pl in list(self._plans):
            rc = pl._destroy_rc()
            if rc != _lib.HD_OK and first is None:
                first = (rc, "hd_plan_destroy", _lib.last_error(self._ctx))
        self._plans = weakref.WeakSet()
        rc = self._L.hd_close(self._ctx)
        self._ctx = ctypes.c_void_p()
        if rc != _lib.HD_OK:
            first = (rc, "hd_close", _lib.last_error(None))
        if check and first is not None:
            raise PrestoError("Execution of command (%s) failed with status (%s)! %s"
                              % (first[1], _lib.ERROR_NAMES.get(first[0], first[0]), first[2]))

    def debug_fault(self):
        """Mark the context faulted as a sticky HIP error would (hd_debug_fault; tests only)."""
        self._chk(self._L.hd_debug_fault(self._ctx), "hd_debug_fault")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        # an exception already in flight is the one to report
        self.close(check=exc[0] is None)

    def _chk(self, rc, what):
        _check(rc, what, self._ctx)

    def sync(self):
        self._chk(self._L.hd_sync(self._ctx), "hd_sync")

    def touch_raw(self):
        """The raw block changed outside the library: rebuild derived layouts (hd_touch_raw)."""
        self._chk(self._L.hd_touch_raw(self._ctx), "hd_touch_raw")

    def set_streams(self, n):
        """1 (default), 2 or 3 HIP streams for stage 2 (hd_set_streams)."""
        self._chk(self._L.hd_set_streams(self._ctx, int(n)), "hd_set_streams")

    # -- observation state --
    def set_obs(self, obs: ObsParams, opts: Optional[Opts] = None):
        opts = opts or Opts()
        o, p = obs.to_c(), opts.to_c()
        self._chk(self._L.hd_set_obs(self._ctx, ctypes.byref(o), ctypes.byref(p)), "hd_set_obs")
        self.obs, self.opts = obs, opts

    def set_calib(self, scl=None, offs=None, wts=None):
        arrs = [None if a is None else np.ascontiguousarray(a, dtype=np.float32) for a in (scl, offs, wts)]
        self._chk(self._L.hd_set_chan_calib(self._ctx, *[_f32p(a) for a in arrs]), "hd_set_chan_calib")

    def set_mask(self, mask=None, ptsperint=0, padvals=None, dtint=0.0, zapint=None):
        """rfifind mask [numint][nchan] (the per-interval channel lists), applied per read
        block with check_mask's rule; zapint [numint] marks zap_ints (None: full rows);
        dtint = seconds per interval as stored (0: ptsperint * dt); padvals = initial pad
        values (e.g. stats_padvals of the rfifind .stats)."""
        m = zi = None
        numint = 0
        u8p = ctypes.POINTER(ctypes.c_uint8)
        if mask is not None:
            mask = np.ascontiguousarray(mask, dtype=np.uint8)
            numint = mask.shape[0]
            m = mask.ctypes.data_as(u8p)
            if zapint is not None:
                zapint = np.ascontiguousarray(zapint, dtype=np.uint8)
                zi = zapint.ctypes.data_as(u8p)
        pv = None if padvals is None else np.ascontiguousarray(padvals, dtype=np.float32)
        self._chk(self._L.hd_set_mask(self._ctx, m, numint, int(ptsperint), float(dtint), zi, _f32p(pv)),
                  "hd_set_mask")

    def set_rfimask(self, rfimask, padvals=None):
        """An RfiMask (formats.mask.read_mask) as prepsubband -mask applies it."""
        self.set_mask(rfimask.bitmap, rfimask.ptsperint, padvals, rfimask.dtint, rfimask.zapint)

    def get_clean(self):
        """Per-block cleaning state of the current raw block: (pad [nblk][nchan] f32,
        clipped [N] u8, zap [nblk][nchan] u8, nclipped) -- computes it if needed."""
        o = self.obs
        blk = min(o.nsblk if o.nsblk > 0 else o.N, o.N)
        nblk = (o.N + blk - 1) // blk
        pad = np.zeros((nblk, o.nchan), np.float32)
        clipped = np.zeros(o.N, np.uint8)
        zap = np.zeros((nblk, o.nchan), np.uint8)
        n = ctypes.c_int64()
        u8p = ctypes.POINTER(ctypes.c_uint8)
        self._chk(self._L.hd_get_clean(self._ctx, _f32p(pad), clipped.ctypes.data_as(u8p), zap.ctypes.data_as(u8p),
                                       ctypes.byref(n)), "hd_get_clean")
        return pad, clipped, zap, n.value

    def push_raw(self, spectra, start=0):
        a = np.ascontiguousarray(spectra, dtype=np.uint8)
        n = a.size // self.obs.rowbytes
        self._chk(self._L.hd_push_raw(self._ctx, a.ctypes.data_as(ctypes.c_void_p), int(start), int(n)),
                  "hd_push_raw")

    def push_raw_file(self, path, table_offset, row_bytes, col_offset, col_bytes, row0, nrows, start=0,
                      block_bytes=0):
        """Stream the DATA column of rows [row0, row0+nrows) of a PSRFITS SUBINT table from
        `path` into device spectra [start, ...) through two pinned host blocks
        (hd_push_raw_file).  Returns (seconds in pread, seconds for the call)."""
        src = _lib.hd_rows_src(table_offset=int(table_offset), row_bytes=int(row_bytes), col_offset=int(col_offset),
                               col_bytes=int(col_bytes), row0=int(row0), nrows=int(nrows),
                               block_bytes=int(block_bytes))
        io, tot = ctypes.c_double(), ctypes.c_double()
        self._chk(self._L.hd_push_raw_file(self._ctx, os.fsencode(path), ctypes.byref(src), int(start),
                                           ctypes.byref(io), ctypes.byref(tot)), "hd_push_raw_file(%s)" % path)
        return io.value, tot.value

    def push_raw_file_band(self, path, table_offset, row_bytes, col_offset, col_bytes, row0, nrows, start,
                           spec_bytes, src_offset, dst_offset, nbytes, block_bytes=0):
        """hd_push_raw_file_band: bytes [src_offset, +nbytes) of each spectrum (spec_bytes long) of
        rows [row0, row0+nrows) into bytes [dst_offset, +nbytes) of device spectra [start, ...)."""
        src = _lib.hd_rows_src(table_offset=int(table_offset), row_bytes=int(row_bytes), col_offset=int(col_offset),
                               col_bytes=int(col_bytes), row0=int(row0), nrows=int(nrows),
                               block_bytes=int(block_bytes))
        io, tot = ctypes.c_double(), ctypes.c_double()
        self._chk(self._L.hd_push_raw_file_band(self._ctx, os.fsencode(path), ctypes.byref(src), int(start),
                                                int(spec_bytes), int(src_offset), int(dst_offset), int(nbytes),
                                                ctypes.byref(io), ctypes.byref(tot)),
                  "hd_push_raw_file_band(%s)" % path)
        return io.value, tot.value

    def prefetch_raw_file(self, path, table_offset, row_bytes, col_offset, col_bytes, row0, nrows, start=0,
                          block_bytes=0, band=None):
        """hd_prefetch_raw_file(_band): queue rows of a PSRFITS table for the NEXT beam (the
        context's second raw slot, read on a background thread while this beam computes);
        band = (spec_bytes, src_offset, dst_offset, nbytes) for a Mock half.  Returns at once."""
        src = _lib.hd_rows_src(table_offset=int(table_offset), row_bytes=int(row_bytes), col_offset=int(col_offset),
                               col_bytes=int(col_bytes), row0=int(row0), nrows=int(nrows),
                               block_bytes=int(block_bytes))
        if band is None:
            self._chk(self._L.hd_prefetch_raw_file(self._ctx, os.fsencode(path), ctypes.byref(src), int(start)),
                      "hd_prefetch_raw_file(%s)" % path)
        else:
            sb, so, do, nb = (int(x) for x in band)
            self._chk(self._L.hd_prefetch_raw_file_band(self._ctx, os.fsencode(path), ctypes.byref(src), int(start),
                                                        sb, so, do, nb), "hd_prefetch_raw_file_band(%s)" % path)

    def prefetch_fill(self, start, count, byte_value=0):
        """hd_prefetch_fill: a file gap of the NEXT beam."""
        self._chk(self._L.hd_prefetch_fill(self._ctx, int(start), int(count), int(byte_value)), "hd_prefetch_fill")

    def swap_raw(self):
        """hd_swap_raw: the prefetched beam becomes the current raw block once its reads are
        done (compute already queued keeps running).  Returns (pread s, s since the first
        prefetch call)."""
        io, tot = ctypes.c_double(), ctypes.c_double()
        self._chk(self._L.hd_swap_raw(self._ctx, ctypes.byref(io), ctypes.byref(tot)), "hd_swap_raw")
        return io.value, tot.value

    def fill_raw(self, start, count, byte_value=0):
        """hd_fill_raw: spectra [start, start+count) set to byte_value (file-gap padding)."""
        self._chk(self._L.hd_fill_raw(self._ctx, int(start), int(count), int(byte_value)), "hd_fill_raw")

    def push_raw_device(self, dev_ptr, start=0, count=None):
        """Raw spectra from device memory of this context's GPU (an int address, e.g. a
        torch tensor's data_ptr() after an RCCL broadcast)."""
        count = self.obs.N - start if count is None else count
        self._chk(self._L.hd_push_raw_device(self._ctx, ctypes.c_void_p(int(dev_ptr)), int(start), int(count)),
                  "hd_push_raw_device")

    def get_raw_device(self, dev_ptr, start=0, count=None):
        count = self.obs.N - start if count is None else count
        self._chk(self._L.hd_get_raw_device(self._ctx, ctypes.c_void_p(int(dev_ptr)), int(start), int(count)),
                  "hd_get_raw_device")

    def get_raw(self, start=0, count=None):
        count = self.obs.N - start if count is None else count
        out = np.empty((count, self.obs.rowbytes), np.uint8)
        self._chk(self._L.hd_get_raw(self._ctx, out.ctypes.data_as(ctypes.c_void_p), int(start), int(count)),
                  "hd_get_raw")
        return out

    # -- time slices (multi-GPU, hipdedisp.sharding.TimeSlices) --
    def set_slice(self, t0, n_total):
        """This context holds spectra [t0, t0 + obs.N) of an observation of n_total spectra
        (hd_set_slice; (0, 0) = the whole observation)."""
        self._chk(self._L.hd_set_slice(self._ctx, int(t0), int(n_total)), "hd_set_slice")

    def clip_stats(self, nown, stats):
        """Rows of this slice's first `nown` read blocks into `stats` (hd_clip_stats): a
        float64 numpy array [nblk_total][nchan + 3] or an int device address of one."""
        ptr = stats if isinstance(stats, int) else stats.ctypes.data
        self._chk(self._L.hd_clip_stats(self._ctx, int(nown), ctypes.c_void_p(ptr)), "hd_clip_stats")

    def clip_set_stats(self, stats):
        """Finish clip_times for this slice from the observation's per-block statistics."""
        ptr = stats if isinstance(stats, int) else stats.ctypes.data
        self._chk(self._L.hd_clip_set_stats(self._ctx, ctypes.c_void_p(ptr)), "hd_clip_set_stats")

    # -- in-library collectives (hd_comm_*: RCCL, no torch.distributed) --
    @staticmethod
    def comm_unique_id():
        """A new 128-byte communicator id (rank 0; hand it to every rank)."""
        L = _lib.load()
        buf = (ctypes.c_uint8 * 128)()
        _check(L.hd_comm_unique_id(buf), "hd_comm_unique_id")
        return bytes(buf)

    def comm_init(self, uid, rank, world):
        """Join the communicator `uid` as rank `rank` of `world` (collective)."""
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(bytes(uid))
        self._chk(self._L.hd_comm_init(self._ctx, buf, int(rank), int(world)), "hd_comm_init")

    def comm_allreduce(self, x):
        """Sum a float64 numpy array (in place) or (address, n) of device doubles over the ranks."""
        if isinstance(x, tuple):
            ptr, n = x
        else:
            assert x.dtype == np.float64 and x.flags.c_contiguous
            ptr, n = x.ctypes.data, x.size
        self._chk(self._L.hd_comm_allreduce_sum_f64(self._ctx, ctypes.c_void_p(ptr), int(n)), "hd_comm_allreduce_sum_f64")
        return x

    def slice_exchange_clip(self, nown, nblk_total):
        """hd_clip_stats -> all-reduce -> hd_clip_set_stats over the communicator."""
        self._chk(self._L.hd_slice_exchange_clip(self._ctx, int(nown), int(nblk_total)), "hd_slice_exchange_clip")

    def comm_destroy(self):
        self._chk(self._L.hd_comm_destroy(self._ctx), "hd_comm_destroy")

    def synth_device(self, synth: hd_synth):
        self._chk(self._L.hd_synth_device(self._ctx, ctypes.byref(synth)), "hd_synth_device")

    def wait_writes(self):
        """hd_wait_writes: every queued .dat write done; (writer busy seconds, bytes) so far."""
        sec, nb = ctypes.c_double(), ctypes.c_int64()
        self._chk(self._L.hd_wait_writes(self._ctx, ctypes.byref(sec), ctypes.byref(nb)), "hd_wait_writes")
        return sec.value, nb.value

    def plan(self, pp: PassParams):
        return Plan(self, pp)

    def series_sums(self, plans, dm, t0, count):
        """hd_series_sum of several plans in one call (hd_series_sum_multi): float64 array."""
        n = len(plans)
        arr = (ctypes.c_void_p * max(n, 1))(*[p._p for p in plans])
        a0 = (ctypes.c_int64 * max(n, 1))(*[int(x) for x in t0])
        a1 = (ctypes.c_int64 * max(n, 1))(*[int(x) for x in count])
        out = (ctypes.c_double * max(n, 1))()
        self._chk(self._L.hd_series_sum_multi(arr, n, int(dm), a0, a1, out), "hd_series_sum_multi")
        return np.array(out[:n], np.float64)

    def run_subband_multi(self, plans):
        """Stage 1 of several passes of one DDplan stage from one read of the raw block."""
        arr = (ctypes.c_void_p * len(plans))(*[p._p.value for p in plans])
        self._chk(self._L.hd_run_subband_multi(arr, len(plans)),
                  "prepsubband -sub (x%d passes)" % len(plans))

    def run_dedisp_multi(self, plans):
        """Stage 2 of several passes, series left on the device (hd_run_dedisp_multi): the
        passes of one DDplan stage share one pair-kernel launch."""
        arr = (ctypes.c_void_p * len(plans))(*[p._p.value for p in plans])
        self._chk(self._L.hd_run_dedisp_multi(arr, len(plans)), "prepsubband (x%d passes)" % len(plans))


class Plan:
    """One DDplan pass on a context (hd_plan)."""

    def __init__(self, eng: Engine, pp: PassParams):
        self.eng, self.pp = eng, pp
        self._p = ctypes.c_void_p()
        c = pp.to_c()
        eng._chk(eng._L.hd_plan_create(eng._ctx, ctypes.byref(c), ctypes.byref(self._p)),
                 "hd_plan_create(subdm=%.2f)" % pp.subdm)
        lof, cw, dt, nds = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
        eng._chk(eng._L.hd_plan_sub_params(self._p, ctypes.byref(lof), ctypes.byref(cw), ctypes.byref(dt),
                                           ctypes.byref(nds)), "hd_plan_sub_params")
        self.sub_lofreq, self.sub_chanwid, self.sub_dt, self.nds = lof.value, cw.value, dt.value, nds.value
        self.numout = pp.numout if pp.numout > 0 else self.nds
        eng._plans.add(self)

    def _destroy_rc(self):
        rc = _lib.HD_OK
        if self._p:
            rc = self.eng._L.hd_plan_destroy(self._p)
            self._p = ctypes.c_void_p()
        return rc

    def destroy(self):
        self._destroy_rc()

    def __del__(self):
        try:
            if self._p and self.eng._ctx:
                self.destroy()
        except Exception:
            pass

    def delays(self):
        nchan = self.eng.obs.nchan
        idd = np.zeros(nchan, dtype=np.int32)
        off = np.zeros((self.pp.numdms, self.pp.nsub), dtype=np.int32)
        self.eng._chk(self.eng._L.hd_plan_get_delays(
            self._p, idd.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
            off.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))), "hd_plan_get_delays")
        return idd, off

    def set_variant(self, v):
        self.eng._chk(self.eng._L.hd_plan_set_variant(self._p, int(v)), "hd_plan_set_variant")

    def set_bary(self, diffbins=None):
        """Barycentred output (hd_plan_set_bary): the add/remove-bin list of bary_diffbins for
        this plan's output sample time; None or empty = topocentric."""
        if diffbins is None or len(diffbins) == 0:
            self.eng._chk(self.eng._L.hd_plan_set_bary(self._p, None, 0), "hd_plan_set_bary")
            return
        d = np.ascontiguousarray(diffbins, dtype=np.int32)
        self.eng._chk(self.eng._L.hd_plan_set_bary(self._p, d.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(d)),
                      "hd_plan_set_bary")

    def data_end(self):
        """Samples of real data at the head of the output (hd_plan_data_end): min(nds,
        numout), or where the barycentred data ends; the .inf on/off boundary."""
        n = ctypes.c_int64()
        self.eng._chk(self.eng._L.hd_plan_data_end(self._p, ctypes.byref(n)), "hd_plan_data_end")
        return n.value

    def run_subband(self):
        self.eng._chk(self.eng._L.hd_run_subband(self._p), "prepsubband -sub -subdm %.2f" % self.pp.subdm)

    def _sub_dtype(self):
        return np.int16 if self.eng.opts.sub_dtype == _lib.HD_SUB_I16 else np.float32

    def get_subbands(self):
        out = np.empty((self.pp.nsub, self.nds), dtype=self._sub_dtype())
        self.eng._chk(self.eng._L.hd_get_subbands(self._p, out.ctypes.data_as(ctypes.c_void_p)),
                      "hd_get_subbands")
        return out

    def get_subbands_window(self, t0, count):
        out = np.empty((self.pp.nsub, int(count)), dtype=self._sub_dtype())
        self.eng._chk(self.eng._L.hd_get_subbands_window(self._p, int(t0), int(count),
                                                         out.ctypes.data_as(ctypes.c_void_p)), "hd_get_subbands_window")
        return out

    def get_series(self, dm0=0, ndm=None, t0=0, count=None):
        """Window of the device-resident series of the last run_dedisp: [ndm][count] f32."""
        ndm = self.pp.numdms - dm0 if ndm is None else ndm
        count = self.numout - t0 if count is None else count
        out = np.empty((int(ndm), int(count)), dtype=np.float32)
        self.eng._chk(self.eng._L.hd_get_series(self._p, int(dm0), int(ndm), int(t0), int(count), _f32p(out)),
                      "hd_get_series")
        return out

    def series_sum(self, dm, t0, count):
        """Exact double sum of series samples [t0, t0+count) of DM dm (hd_series_sum)."""
        v = ctypes.c_double()
        self.eng._chk(self.eng._L.hd_series_sum(self._p, int(dm), int(t0), int(count), ctypes.byref(v)),
                      "hd_series_sum")
        return v.value

    def series_fill(self, t0, value):
        """Samples [t0, numout) of every DM := value (hd_series_fill)."""
        self.eng._chk(self.eng._L.hd_series_fill(self._p, int(t0), float(value)), "hd_series_fill")

    def set_subbands(self, sub):
        a = np.ascontiguousarray(sub, dtype=self._sub_dtype())
        if a.shape != (self.pp.nsub, self.nds):
            raise PrestoError("subbands must have shape %s, got %s" % ((self.pp.nsub, self.nds), a.shape))
        self.eng._chk(self.eng._L.hd_set_subbands(self._p, a.ctypes.data_as(ctypes.c_void_p)),
                      "hd_set_subbands")

    def run_dedisp(self, to_host=True):
        out = None
        ptr = None
        if to_host:
            out = np.empty((self.pp.numdms, self.numout), dtype=np.float32)
            ptr = _f32p(out)
        self.eng._chk(self.eng._L.hd_run_dedisp(self._p, ptr),
                      "prepsubband -lodm %.2f -dmstep %.2f -numdms %d"
                      % (self.pp.lodm, self.pp.dmstep, self.pp.numdms))
        return out

    def write_series(self, paths, wait=True):
        """hd_write_series: the device series of the last run_dedisp to paths[numdms] (.dat)."""
        if len(paths) != self.pp.numdms:
            raise PrestoError("write_series needs %d paths, got %d" % (self.pp.numdms, len(paths)))
        arr = (ctypes.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
        self.eng._chk(self.eng._L.hd_write_series(self._p, arr, int(bool(wait))), "hd_write_series")

    def kernel(self):
        """Name of the stage-2 kernel of the last run_dedisp (hd_plan_kernel), as rocprofv3
        prints it without namespace and arguments."""
        buf = ctypes.create_string_buffer(64)
        self.eng._chk(self.eng._L.hd_plan_kernel(self._p, buf, 64), "hd_plan_kernel")
        return buf.value.decode()

    def launch_passes(self):
        """Passes the last stage-2 launch this plan led carried (hd_plan_launch_passes): 1
        for run_dedisp, n for the first plan of a shared launch, 0 for the others."""
        n = ctypes.c_int32()
        self.eng._chk(self.eng._L.hd_plan_launch_passes(self._p, ctypes.byref(n)), "hd_plan_launch_passes")
        return n.value

    def last_ms(self):
        a, b = ctypes.c_float(), ctypes.c_float()
        self.eng._chk(self.eng._L.hd_plan_last_ms(self._p, ctypes.byref(a), ctypes.byref(b)), "hd_plan_last_ms")
        return a.value, b.value
