"""Mock spectrometer ingest in-stream.

The reference preprocesses a PALFA Mock beam before searching it
(lib/python/datafile.py:474-508, MockPsrfitsData.preprocess):

    combine_mocks <...s0g0...fits> <...s1g0...fits> -o <projid>.<date>.<source>.b<beam>.<scan>
    fitsdelrow <base>_0001.fits[SUBINT] 1 7
    mv <base>_0001.fits <base>.fits

i.e. the two half-band files of a beam are merged into one file of nchan_out channels, the
first 7 rows are deleted, and the merged file is what the search reads.  Here nothing is
rewritten: MockBeam computes the merged geometry and streams each half's rows (from row 7)
straight into its channel range of the device raw block (hd_push_raw_file_band).

The file-name logic (filename_re, are_grouped, is_complete, the output base name) follows
datafile.py:395-508.  combine_mocks itself is psrfits_utils code that is not in this image
[parity unpinned]: the merge is restated as a channel concatenation in frequency order that
drops the overlap between the bands (nchan_lo + nchan_hi - nchan_out channels: the lower
half of them from the top of the low band, the rest from the bottom of the high band), with
no rescaling between the two boards; the merged lofreq is the low band's, the spacing its.
"""
import os
import re

import numpy as np

from .psrfits import _TFORM_SIZES, SECPERDAY, SpectraInfo

FILENAME_RE = re.compile(r'^4bit-(?P<projid>[Pp]\d{4})\.(?P<date>\d{8})\.'
                         r'(?P<source>.*)\.b(?P<beam>[0-7])'
                         r's(?P<subband>[01])g0.(?P<scan>\d{5})\.fits')   # datafile.py:395-397
ROWS_DELETED = 7                                                       # `fitsdelrow ... 1 7`
PALFA_NCHAN = 960


def fnmatch(fn):
    return FILENAME_RE.match(os.path.split(fn)[-1])


def are_grouped(fn1, fn2):
    """datafile.py:424-456: the s0/s1 halves of the same beam and scan."""
    m1, m2 = fnmatch(fn1), fnmatch(fn2)
    if m1 is None or m2 is None:
        return False
    d1, d2 = m1.groupdict(), m2.groupdict()
    s1, s2 = d1.pop("subband"), d2.pop("subband")
    if {s1, s2} != {"0", "1"}:
        return False
    return d1 == d2


def is_complete(fns):
    """datafile.py:458-475: exactly two grouped files."""
    return len(fns) == 2 and are_grouped(*fns)


def merged_basename(fns):
    """datafile.py:494-496: <projid>.<date>.<source>.b<beam>.<scan> (the merged file is this
    + '.fits')."""
    return "%(projid)s.%(date)s.%(source)s.b%(beam)s.%(scan)s" % fnmatch(fns[0]).groupdict()


class MockBeam:
    """The merged view of a Mock beam's two half-band files."""

    def __init__(self, fns, nchan_out=PALFA_NCHAN, rows_deleted=ROWS_DELETED):
        if not is_complete(fns):
            raise ValueError("not the two halves of one Mock beam: %s" % (fns,))
        fns = sorted(fns, key=lambda f: fnmatch(f).group("subband"))
        self.filenames = fns
        self.basename = merged_basename(fns)
        self.parts = [SpectraInfo([fn]) for fn in fns]
        a, b = self.parts
        for attr in ("dt", "spectra_per_subint", "bits_per_sample", "need_flipband"):
            if getattr(a, attr) != getattr(b, attr):
                raise ValueError("Mock halves differ in %s" % attr)
        if abs(abs(a.df) - abs(b.df)) > 1e-7:
            raise ValueError("Mock halves differ in channel spacing")
        if a.num_polns > 1 and not a.summed_polns:
            raise ValueError("multi-polarisation Mock data is not supported")
        if int(a.num_subint[0]) != int(b.num_subint[0]) or abs(a.start_MJD[0] - b.start_MJD[0]) * SECPERDAY > 0.5 * a.dt:
            raise ValueError("Mock halves do not cover the same rows")
        lo, hi = (a, b) if a.lo_freq <= b.lo_freq else (b, a)
        nlo, nhi = int(lo.num_channels), int(hi.num_channels)
        drop = nlo + nhi - int(nchan_out)
        if drop < 0 or drop > min(nlo, nhi):
            raise ValueError("cannot make %d channels from %d + %d" % (nchan_out, nlo, nhi))
        dlo, dhi = drop // 2, drop - drop // 2
        self.nchan = int(nchan_out)
        self.nbits = int(a.bits_per_sample)
        self.flip = bool(a.need_flipband)
        self.df = abs(lo.df)
        self.lofreq = lo.lo_freq
        self.dt = a.dt
        self.nsblk = int(a.spectra_per_subint)
        self.rows_deleted = int(rows_deleted)
        self.nrows = int(a.num_subint[0]) - self.rows_deleted
        if self.nrows <= 0:
            raise ValueError("no rows left after deleting %d" % self.rows_deleted)
        self.N = self.nrows * self.nsblk
        self.start_MJD = np.array([a.start_MJD[0] + self.rows_deleted * self.nsblk * self.dt / SECPERDAY])
        # (part, first source channel, channels, first merged channel), file channel order
        if not self.flip:
            bands = [(lo, 0, nlo - dlo, 0), (hi, dhi, nhi - dhi, nlo - dlo)]
        else:
            bands = [(hi, 0, nhi - dhi, 0), (lo, dlo, nlo - dlo, nhi - dhi)]
        bpc = self.nbits / 8.0
        self.bands = []
        for part, c0, nc, m0 in bands:
            if self.nbits == 4 and (c0 % 2 or nc % 2 or m0 % 2):
                raise ValueError("4-bit band edges must fall on whole bytes")
            self.bands.append((part, int(c0 * bpc), int(nc * bpc), int(m0 * bpc)))
        self.rowbytes = int(self.nchan * bpc)
        # the SpectraInfo surface DedispJob / the shim read (header fields: the s0 file's)
        self.num_channels = self.nchan
        self.bits_per_sample = self.nbits
        self.spectra_per_subint = self.nsblk
        self.need_flipband = self.flip
        self.lo_freq = self.lofreq
        self.hi_freq = self.lofreq + (self.nchan - 1) * self.df
        self.BW = self.nchan * self.df
        self.fctr = self.lofreq + 0.5 * (self.nchan - 1) * self.df
        self.T = self.N * self.dt
        self.num_files = 1
        self.num_polns = 1
        self.summed_polns = True
        self._lo_hi = (lo, hi, dlo, dhi)

    def __getattr__(self, name):
        if name.startswith("_") or name == "parts":
            raise AttributeError(name)
        return getattr(self.parts[0], name)


    def obs_params(self, voverc=0.0):
        from ..engine import ObsParams
        return ObsParams(nchan=self.nchan, nbits=self.nbits, dt=float(self.dt), lofreq=float(self.lofreq),
                         df=float(self.df), N=int(self.N), nsblk=self.nsblk, flip=self.flip, npol=1, voverc=voverc)

    def stream_to(self, engine, block_bytes=0, prefetch=False):
        """Both halves into the engine's raw block (hd_set_obs(obs_params()) first), rows from
        rows_deleted on; returns (seconds in pread, seconds total, bytes read).  prefetch=True
        queues them for the NEXT beam (hd_prefetch_raw_file_band; engine.swap_raw() after)."""
        io = tot = 0.0
        nbytes = 0
        for part, s_off, nb, d_off in self.bands:
            tab = part._tables[0]
            off, rep, code = tab.cols["DATA"]
            col_bytes = rep * _TFORM_SIZES[code]
            spec_bytes = col_bytes // self.nsblk
            if prefetch:
                engine.prefetch_raw_file(part.filenames[0], tab.data_offset, tab.rowlen, off, col_bytes,
                                         self.rows_deleted, self.nrows, 0, block_bytes=block_bytes,
                                         band=(spec_bytes, s_off, d_off, nb))
            else:
                x, y = engine.push_raw_file_band(part.filenames[0], tab.data_offset, tab.rowlen, off, col_bytes,
                                                 self.rows_deleted, self.nrows, 0, spec_bytes, s_off, d_off, nb,
                                                 block_bytes=block_bytes)
                io += x
                tot += y
            nbytes += col_bytes * self.nrows
        return io, tot, nbytes

    def read_calib(self):
        """DAT_SCL / DAT_OFFS / DAT_WTS of the merged channels (file channel order; None where
        neither half needs it)."""
        cal = [p.read_calib() for p in self.bands_parts()]
        out = []
        for k in range(3):
            if all(c[k] is None for c in cal):
                out.append(None)
                continue
            merged = np.empty(self.nchan, np.float32)
            for (part, s_off, nb, d_off), c in zip(self.bands, cal):
                bpc = self.nbits / 8.0
                c0, m0, nc = int(s_off / bpc), int(d_off / bpc), int(nb / bpc)
                src = c[k] if c[k] is not None else np.full(part.num_channels, 0.0 if k == 1 else 1.0, np.float32)
                merged[m0:m0 + nc] = src[c0:c0 + nc]
            out.append(merged)
        return tuple(out)

    def bands_parts(self):
        return [b[0] for b in self.bands]

    def read_spectra(self):
        """The merged raw block on the host (what combine_mocks + fitsdelrow leave in the
        merged file's DATA): uint8 [N][rowbytes]."""
        out = np.zeros((self.N, self.rowbytes), np.uint8)
        for part, s_off, nb, d_off in self.bands:
            x = part.read_spectra()[self.rows_deleted * self.nsblk:]
            out[:, d_off:d_off + nb] = x[:self.N, s_off:s_off + nb]
        return out

