"""Minimal PSRFITS (SEARCH mode) reader/writer with no pyfits/astropy dependency.

Header semantics follow the reference's SpectraInfo (lib/python/formats/psrfits.py:25-320):
dt = TBIN, nchan = NCHAN, NSBLK, NBITS, N = sum(NSBLK * NAXIS2) (float in the reference,
:272-280), lo/hi freq and df from row 0's DAT_FREQ (:210-220), band flip when
hi < lo (:306-312), BW = nchan * df (:314), need_scale/offset/weight when row 0's
DAT_SCL/DAT_OFFS/DAT_WTS differ from 1/0/1 (:236-270), start MJD from STT_* plus the
OFFS_SUB row correction (:102-177).  The DATA column is returned as raw file bytes
(4-bit packed, 16-bit big-endian) — the engine unpacks on the GPU.
"""
import math
import os

import numpy as np

BLOCK = 2880
SECPERDAY = 86400.0


# ---------------------------------------------------------------------------------
# generic FITS header / binary-table plumbing
# ---------------------------------------------------------------------------------
def _fmt_value(v):
    if isinstance(v, bool):
        return "%20s" % ("T" if v else "F")
    if isinstance(v, (int, np.integer)):
        return "%20d" % v
    if isinstance(v, (float, np.floating)):
        s = "%.17G" % v
        if "." not in s and "E" not in s:
            s += "."
        return "%20s" % s
    s = str(v).replace("'", "''")
    return "'%-8s'" % s


def _card(key, value=None, comment=""):
    if key in ("END",):
        return "%-80s" % key
    body = "%-8s= %s" % (key, _fmt_value(value))
    if comment:
        body += " / " + comment
    return "%-80s" % body[:80]


def _header_bytes(cards):
    s = "".join(cards) + _card("END")
    pad = (-len(s)) % BLOCK
    return (s + " " * pad).encode("ascii")


def _parse_value(raw):
    raw = raw.strip()
    if raw.startswith("'"):
        # string: up to the closing quote ('' is an escaped quote)
        out, i = [], 1
        while i < len(raw):
            if raw[i] == "'":
                if i + 1 < len(raw) and raw[i + 1] == "'":
                    out.append("'")
                    i += 2
                    continue
                break
            out.append(raw[i])
            i += 1
        return "".join(out).rstrip()
    val = raw.split("/")[0].strip()
    if val in ("T", "F"):
        return val == "T"
    if val == "":
        return None
    try:
        return int(val)
    except ValueError:
        try:
            return float(val.replace("D", "E"))
        except ValueError:
            return val


def read_header(f):
    """Read one header unit from file object f; return (dict, ordered keys) or (None, None) at EOF."""
    hdr, keys = {}, []
    while True:
        blk = f.read(BLOCK)
        if len(blk) < BLOCK:
            return None, None
        text = blk.decode("ascii", errors="replace")
        for i in range(0, BLOCK, 80):
            card = text[i:i + 80]
            key = card[:8].strip()
            if key == "END":
                return hdr, keys
            if card[8:10] == "= ":
                hdr[key] = _parse_value(card[10:])
                keys.append(key)


_TFORM_DTYPES = {"B": ">u1", "I": ">i2", "J": ">i4", "K": ">i8", "E": ">f4", "D": ">f8", "A": "S1", "L": "S1"}
_TFORM_SIZES = {"B": 1, "I": 2, "J": 4, "K": 8, "E": 4, "D": 8, "A": 1, "L": 1}


def _parse_tform(tf):
    tf = tf.strip()
    i = 0
    while i < len(tf) and tf[i].isdigit():
        i += 1
    rep = int(tf[:i]) if i else 1
    return rep, tf[i]


class BinTable:
    """A binary-table HDU: header dict + column layout + data offset in the file."""

    def __init__(self, hdr, data_offset):
        self.hdr = hdr
        self.data_offset = data_offset
        self.nrows = hdr["NAXIS2"]
        self.rowlen = hdr["NAXIS1"]
        self.cols = {}
        off = 0
        for i in range(1, hdr["TFIELDS"] + 1):
            rep, code = _parse_tform(hdr["TFORM%d" % i])
            name = hdr["TTYPE%d" % i].strip()
            self.cols[name] = (off, rep, code)
            off += rep * _TFORM_SIZES[code]

    def column_bytes(self, mm, name, rows=None):
        """Raw bytes of a column for the given rows (default: all): uint8 [nrows][colbytes]."""
        off, rep, code = self.cols[name]
        nb = rep * _TFORM_SIZES[code]
        table = np.ndarray((self.nrows, self.rowlen), dtype=np.uint8, buffer=mm, offset=self.data_offset)
        sel = table if rows is None else table[rows]
        return sel[:, off:off + nb]

    def column(self, mm, name, row=0):
        off, rep, code = self.cols[name]
        raw = self.column_bytes(mm, name, slice(row, row + 1))[0]
        return np.frombuffer(raw.tobytes(), dtype=_TFORM_DTYPES[code]).astype(_TFORM_DTYPES[code][1:] if code != "A" else "S1")


def read_hdus(fn):
    """[(header, data_offset, data_bytes)] for every HDU in the file."""
    out = []
    with open(fn, "rb") as f:
        while True:
            pos = f.tell()
            hdr, _ = read_header(f)
            if hdr is None:
                break
            data_off = f.tell()
            naxis = hdr.get("NAXIS", 0)
            nbytes = 0
            if naxis:
                nbytes = abs(hdr.get("BITPIX", 8)) // 8
                for i in range(1, naxis + 1):
                    nbytes *= hdr["NAXIS%d" % i]
                nbytes += hdr.get("PCOUNT", 0)
                nbytes *= hdr.get("GCOUNT", 1)
            out.append((hdr, data_off, nbytes))
            f.seek(data_off + nbytes + ((-nbytes) % BLOCK))
            if pos == f.tell():
                break
    return out


# ---------------------------------------------------------------------------------
# PSRFITS
# ---------------------------------------------------------------------------------
def is_PSRFITS(fn):
    """lib/python/formats/psrfits.py:409-423"""
    try:
        hdus = read_hdus(fn)
    except Exception:
        return False
    if not hdus:
        return False
    p = hdus[0][0]
    return p.get("FITSTYPE") == "PSRFITS" and p.get("OBS_MODE") == "SEARCH"


class SpectraInfo:
    """Header information of a list of PSRFITS files (psrfits.py:25-320, subset used by
    the dedispersion stage)."""

    def __init__(self, filenames):
        self.filenames = list(filenames)
        self.num_files = len(self.filenames)
        self.N = 0
        self.start_MJD = np.empty(self.num_files)
        self.num_subint = np.empty(self.num_files)
        self.start_subint = np.empty(self.num_files)
        self.start_spec = np.empty(self.num_files)
        self.num_pad = np.zeros(self.num_files)
        self.num_spec = np.empty(self.num_files)
        self.need_scale = self.need_offset = self.need_weight = self.need_flipband = False
        self._tables = []
        for ii, fn in enumerate(self.filenames):
            if not is_PSRFITS(fn):
                raise ValueError("File '%s' does not appear to be PSRFITS!" % fn)
            hdus = read_hdus(fn)
            primary = hdus[0][0]
            sub = [h for h in hdus if h[0].get("EXTNAME", "").strip() == "SUBINT"]
            if not sub:
                raise ValueError("File '%s' has no SUBINT HDU" % fn)
            shdr, doff, _ = sub[0]
            tab = BinTable(shdr, doff)
            self._tables.append(tab)
            self.beam_id = primary.get("IBEAM", shdr.get("BEAM"))
            tel = primary.get("TELESCOP", "")
            self.telescope = "Arecibo" if tel == "ARECIBO 305m" else tel
            self.observer = primary.get("OBSERVER", "")
            self.source = primary.get("SRC_NAME", "")
            self.frontend = primary.get("FRONTEND", "")
            self.backend = primary.get("BACKEND", "")
            self.project_id = primary.get("PROJID", "")
            self.date_obs = primary.get("DATE-OBS", "")
            self.poln_type = primary.get("FD_POLN", "")
            self.ra_str = primary.get("RA", "00:00:00.0")
            self.dec_str = primary.get("DEC", "00:00:00.0")
            self.fctr = primary.get("OBSFREQ", 0.0)
            self.orig_num_chan = primary.get("OBSNCHAN", 0)
            self.orig_df = primary.get("OBSBW", 0.0)
            self.beam_FWHM = primary.get("BMIN", 0.0)
            self.chan_dm = primary.get("CHAN_DM", 0.0)
            self.start_MJD[ii] = primary.get("STT_IMJD", 0) + (primary.get("STT_SMJD", 0) +
                                                              primary.get("STT_OFFS", 0.0)) / SECPERDAY
            self.tracking = primary.get("TRK_MODE", "TRACK") == "TRACK"
            self.dt = shdr["TBIN"]
            self.num_channels = shdr["NCHAN"]
            self.num_polns = shdr["NPOL"]
            self.poln_order = shdr.get("POL_TYPE", "AA+BB")
            self.spectra_per_subint = shdr["NSBLK"]
            self.bits_per_sample = shdr["NBITS"]
            self.num_subint[ii] = shdr["NAXIS2"]
            self.start_subint[ii] = shdr.get("NSUBOFFS", 0)
            self.time_per_subint = self.dt * self.spectra_per_subint
            with open(fn, "rb") as f:
                mm = np.frombuffer(f.read(), dtype=np.uint8) if os.path.getsize(fn) < (1 << 26) else \
                    np.memmap(fn, dtype=np.uint8, mode="r")
            if "OFFS_SUB" in tab.cols:
                offs_sub = float(tab.column(mm, "OFFS_SUB")[0])
                numrows = int((offs_sub - 0.5 * self.time_per_subint) / self.time_per_subint + 1e-7)
                self.start_subint[ii] = numrows
            self.start_MJD[ii] += (self.time_per_subint * self.start_subint[ii]) / SECPERDAY
            MJDf = self.start_MJD[ii] - self.start_MJD[0]
            if MJDf < 0.0:
                raise ValueError("File %d seems to be from before file 0!" % ii)
            self.start_spec[ii] = MJDf * SECPERDAY / self.dt + 0.5
            freqs = tab.column(mm, "DAT_FREQ").astype(np.float64)
            if ii == 0:
                self.df = freqs[1] - freqs[0] if len(freqs) > 1 else 1.0
                self.lo_freq = freqs[0]
                self.hi_freq = freqs[-1]
            if "DAT_WTS" in tab.cols and np.any(tab.column(mm, "DAT_WTS") != 1.0):
                self.need_weight = True
            if "DAT_OFFS" in tab.cols and np.any(tab.column(mm, "DAT_OFFS") != 0.0):
                self.need_offset = True
            if "DAT_SCL" in tab.cols and np.any(tab.column(mm, "DAT_SCL") != 1.0):
                self.need_scale = True
            self.num_spec[ii] = self.spectra_per_subint * self.num_subint[ii]
            if ii > 0 and self.start_spec[ii] > self.N:
                self.num_pad[ii - 1] = self.start_spec[ii] - self.N
                self.N += self.num_pad[ii - 1]
            self.N += self.num_spec[ii]
            del mm
        self.N = float(self.N)   # the reference carries N as float64 (psrfits.py:29, 275, 280)
        self.summed_polns = self.poln_order in ("AA+BB", "INTEN")
        self.T = self.N * self.dt
        if self.orig_num_chan:
            self.orig_df /= float(self.orig_num_chan)
        if self.hi_freq < self.lo_freq:
            self.hi_freq, self.lo_freq = self.lo_freq, self.hi_freq
            self.df *= -1.0
            self.need_flipband = True
        self.BW = self.num_channels * self.df
        self.start_lst = 0.0

    def obs_params(self, voverc=0.0):
        """Engine ObsParams for this observation."""
        from ..engine import ObsParams
        return ObsParams(nchan=int(self.num_channels), nbits=int(self.bits_per_sample), dt=float(self.dt),
                         lofreq=float(self.lo_freq), df=float(self.df), N=int(self.N),
                         nsblk=int(self.spectra_per_subint), flip=bool(self.need_flipband),
                         npol=int(self.num_polns) if not self.summed_polns else 1, voverc=voverc)

    def gaps(self):
        """[(start, count)] spectra of padding between files (psrfits.py:272-280): a file that
        starts after the previous one ends leaves the gap, filled with zero bytes here (PRESTO
        pads with the mask's pad values, 0 without a mask) [PRESTO-ext]."""
        out = []
        for ii in range(1, self.num_files):
            end = int(self.start_spec[ii - 1]) + int(self.num_spec[ii - 1])
            if int(self.start_spec[ii]) > end:
                out.append((end, int(self.start_spec[ii]) - end))
        return out

    def read_spectra(self):
        """All raw spectra of all files: uint8 [N][nchan*nbits/8] in file order, gaps zero."""
        rb = self.num_channels * self.bits_per_sample // 8
        out = np.zeros((int(self.N), rb), np.uint8)
        for ii, (fn, tab) in enumerate(zip(self.filenames, self._tables)):
            mm = np.memmap(fn, dtype=np.uint8, mode="r")
            data = np.ascontiguousarray(tab.column_bytes(mm, "DATA")).reshape(-1, rb)
            s0 = int(self.start_spec[ii])
            out[s0:s0 + data.shape[0]] = data
        return out

    def stream_to(self, engine, block_bytes=0, prefetch=False):
        """Stream every file's DATA column into the engine's device raw block through the
        library's pinned double-buffered reader (hd_push_raw_file), file after file at its
        start spectrum.  Returns (seconds in pread, seconds total, bytes).  prefetch=True
        queues the same reads for the NEXT beam (hd_prefetch_raw_file, background; times 0)
        -- engine.swap_raw() then makes it current."""
        if self.num_polns > 1 and not self.summed_polns:
            raise ValueError("multi-polarisation PSRFITS DATA is not supported by the stream reader")
        io = tot = 0.0
        nbytes = 0
        for ii, (fn, tab) in enumerate(zip(self.filenames, self._tables)):
            off, rep, code = tab.cols["DATA"]
            col_bytes = rep * _TFORM_SIZES[code]
            if prefetch:
                engine.prefetch_raw_file(fn, tab.data_offset, tab.rowlen, off, col_bytes, 0, tab.nrows,
                                         start=int(self.start_spec[ii]), block_bytes=block_bytes)
            else:
                a, b = engine.push_raw_file(fn, tab.data_offset, tab.rowlen, off, col_bytes, 0, tab.nrows,
                                            start=int(self.start_spec[ii]), block_bytes=block_bytes)
                io += a
                tot += b
            nbytes += col_bytes * tab.nrows
        for start, count in self.gaps():
            if prefetch:
                engine.prefetch_fill(start, count, 0)
            else:
                engine.fill_raw(start, count, 0)
        return io, tot, nbytes

    def read_calib(self):
        """Row-0 DAT_SCL / DAT_OFFS / DAT_WTS (None where not needed), file channel order."""
        tab = self._tables[0]
        mm = np.memmap(self.filenames[0], dtype=np.uint8, mode="r")
        nc = self.num_channels
        scl = tab.column(mm, "DAT_SCL")[:nc].astype(np.float32) if self.need_scale else None
        offs = tab.column(mm, "DAT_OFFS")[:nc].astype(np.float32) if self.need_offset else None
        wts = tab.column(mm, "DAT_WTS")[:nc].astype(np.float32) if self.need_weight else None
        return scl, offs, wts


def write_psrfits(fn, spectra, obs, src_name="SYNTH", backend="pdev", telescope="Arecibo",
                  ra="19:00:00.0000", dec="+05:00:00.000", mjd=56000.5, scl=None, offs=None, wts=None,
                  beam=0, projid="P2030"):
    """Write a SEARCH-mode PSRFITS file from raw file-layout spectra (uint8 [N][rowbytes])
    and engine ObsParams.  Frequencies are stored descending when obs.flip is set."""
    spectra = np.ascontiguousarray(spectra, dtype=np.uint8)
    N, rowbytes = spectra.shape
    nsblk = obs.nsblk
    if N % nsblk:
        raise ValueError("N (%d) must be a multiple of NSBLK (%d)" % (N, nsblk))
    nrows = N // nsblk
    nchan = obs.nchan
    freqs = obs.lofreq + obs.df * np.arange(nchan)
    if obs.flip:
        freqs = freqs[::-1]
    imjd = int(mjd)
    smjd = int((mjd - imjd) * SECPERDAY)
    soffs = (mjd - imjd) * SECPERDAY - smjd
    prim = [_card("SIMPLE", True), _card("BITPIX", 8), _card("NAXIS", 0), _card("EXTEND", True),
            _card("FITSTYPE", "PSRFITS"), _card("HDRVER", "3.4"), _card("OBS_MODE", "SEARCH"),
            _card("TELESCOP", telescope), _card("OBSERVER", "hipdedisp"), _card("PROJID", projid),
            _card("FRONTEND", "alfa"), _card("BACKEND", backend), _card("IBEAM", beam),
            _card("FD_POLN", "LIN"), _card("DATE-OBS", "2012-03-14T12:00:00"),
            _card("OBSFREQ", float(obs.lofreq + 0.5 * (nchan - 1) * obs.df)),
            _card("OBSBW", float(nchan * obs.df) * (-1.0 if obs.flip else 1.0)),
            _card("OBSNCHAN", nchan), _card("CHAN_DM", 0.0), _card("SRC_NAME", src_name),
            _card("TRK_MODE", "TRACK"), _card("RA", ra), _card("DEC", dec), _card("BMIN", 0.0583),
            _card("STT_IMJD", imjd), _card("STT_SMJD", smjd), _card("STT_OFFS", float(soffs)),
            _card("STT_LST", 0.0)]
    if obs.nbits == 16:
        dcode, drep = "I", nsblk * nchan
    else:
        dcode, drep = "B", nsblk * rowbytes
    cols = [("TSUBINT", 1, "D"), ("OFFS_SUB", 1, "D"), ("DAT_FREQ", nchan, "D"), ("DAT_WTS", nchan, "E"),
            ("DAT_OFFS", nchan, "E"), ("DAT_SCL", nchan, "E"), ("DATA", drep, dcode)]
    rowlen = sum(r * _TFORM_SIZES[c] for _, r, c in cols)
    ext = [_card("XTENSION", "BINTABLE"), _card("BITPIX", 8), _card("NAXIS", 2), _card("NAXIS1", rowlen),
           _card("NAXIS2", nrows), _card("PCOUNT", 0), _card("GCOUNT", 1), _card("TFIELDS", len(cols))]
    for i, (name, rep, code) in enumerate(cols, 1):
        ext.append(_card("TTYPE%d" % i, name))
        ext.append(_card("TFORM%d" % i, "%d%s" % (rep, code)))
    ext += [_card("EXTNAME", "SUBINT"), _card("TBIN", float(obs.dt)), _card("NCHAN", nchan),
            _card("NPOL", 1), _card("POL_TYPE", "AA+BB"), _card("NCHNOFFS", 0), _card("NSBLK", nsblk),
            _card("NBITS", obs.nbits), _card("NSUBOFFS", 0), _card("NUMIFS", 2)]
    rec = np.zeros((nrows, rowlen), dtype=np.uint8)
    tsub = nsblk * obs.dt
    o = 0
    for name, rep, code in cols:
        nb = rep * _TFORM_SIZES[code]
        if name == "TSUBINT":
            val = np.full((nrows, 1), tsub, dtype=">f8")
        elif name == "OFFS_SUB":
            val = ((np.arange(nrows) + 0.5) * tsub).astype(">f8").reshape(nrows, 1)
        elif name == "DAT_FREQ":
            val = np.tile(freqs.astype(">f8"), (nrows, 1))
        elif name == "DAT_WTS":
            val = np.tile((np.ones(nchan) if wts is None else wts).astype(">f4"), (nrows, 1))
        elif name == "DAT_OFFS":
            val = np.tile((np.zeros(nchan) if offs is None else offs).astype(">f4"), (nrows, 1))
        elif name == "DAT_SCL":
            val = np.tile((np.ones(nchan) if scl is None else scl).astype(">f4"), (nrows, 1))
        else:
            rec[:, o:o + nb] = spectra.reshape(nrows, nb)   # raw bytes already in file layout
            o += nb
            continue
        rec[:, o:o + nb] = np.ascontiguousarray(val).view(np.uint8).reshape(nrows, nb)
        o += nb
    with open(fn, "wb") as f:
        f.write(_header_bytes(prim))
        f.write(_header_bytes(ext))
        data = rec.tobytes()
        f.write(data)
        f.write(b"\0" * ((-len(data)) % BLOCK))
