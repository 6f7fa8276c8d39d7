"""Synthetic PALFA-shaped beams: geometry, sources, RFI and mask.

The sample generator itself is native (hd_synth_host / hd_synth_device share one
integer-only implementation), so a beam generated on the GPU is byte-identical to
the same spectra generated on the host for the CPU oracle.
"""
import ctypes

import numpy as np

from . import _lib
from .engine import ObsParams

# PALFA Mock geometry (not in the reference; SURVEY.md §8d states these values and
# asks that they stay configurable).
PALFA_NCHAN = 960
PALFA_DT = 65.476e-6
PALFA_FCTR = 1375.5
PALFA_BW = 322.617        # MHz -> df = 0.33606 MHz
PALFA_NSBLK = 2048
SEED0 = 20261015


def palfa_obs(N=1 << 22, nbits=8, nchan=PALFA_NCHAN, dt=PALFA_DT, fctr=PALFA_FCTR, bw=PALFA_BW,
              nsblk=PALFA_NSBLK, flip=True):
    """Observation geometry of a PALFA Mock beam.  Stored with descending channels
    (flip=True) so the band-flip path of psrfits.py:306-312 is exercised."""
    df = bw / nchan
    lofreq = fctr - 0.5 * bw + 0.5 * df
    return ObsParams(nchan=nchan, nbits=nbits, dt=dt, lofreq=lofreq, df=df, N=int(N),
                     nsblk=nsblk, flip=flip)


def palfa_synth(beam=0, nbits=8, nchan=PALFA_NCHAN):
    """Source/RFI model: 3 pulsars (4.6 ms @ DM 71.0, 0.253 s @ 217.3, 1.2 s @ 612.0),
    a single pulse @ DM 350.0, 3 persistent RFI channels, 1% bursty cells, spikes."""
    L = _lib.load()
    s = _lib.hd_synth()
    L.hd_synth_default(ctypes.byref(s))
    s.seed = SEED0 + beam
    if nbits == 4:
        s.base_level, s.noise_sigma = 7.0, 1.5
        for i in range(s.npsr):
            s.psr_amp[i] = 0.6
        s.sp_amp[0], s.rfi_amp, s.burst_amp, s.spike_amp = 3.0, 4.0, 3.0, 2.0
    elif nbits == 16:
        s.base_level, s.noise_sigma = 2000.0, 200.0
        for i in range(s.npsr):
            s.psr_amp[i] *= 16.0
        s.sp_amp[0] *= 16.0
        s.rfi_amp, s.burst_amp, s.spike_amp = 480.0, 400.0, 240.0
    chans = [c for c in (int(nchan * 0.105), int(nchan * 0.479), int(nchan * 0.809))]
    s.rfi_nchan = len(chans)
    for i, c in enumerate(chans):
        s.rfi_chan[i] = c
    return s


def host_spectra(obs: ObsParams, synth, start=0, count=None):
    """Spectra [start, start+count) of the synthetic beam, file layout, uint8 [count][rowbytes]."""
    if count is None:
        count = obs.N - start
    out = np.empty((count, obs.rowbytes), dtype=np.uint8)
    o = obs.to_c()
    rc = _lib.load().hd_synth_host(ctypes.byref(o), ctypes.byref(synth), int(start), int(count),
                                   out.ctypes.data_as(ctypes.c_void_p))
    if rc != 0:
        raise RuntimeError("hd_synth_host failed: %s" % _lib.last_error())
    return out


def rfifind_ptsperint(dt, chunk_time=2 ** 15 * 0.000064, nsblk=PALFA_NSBLK):
    """Samples per rfifind interval for `rfifind -time chunk_time`
    (searching_example.py:12): rfifind.ptsperint_for, whole PSRFITS rows."""
    from .rfifind import ptsperint_for
    return ptsperint_for(dt, chunk_time, nsblk)


def synth_mask(obs: ObsParams, synth, ptsperint, frac=0.02, seed=7):
    """An rfifind-style mask for the synthetic beam: the persistent RFI channels are
    zapped in every interval, plus a random `frac` of (interval, channel) cells.
    Returns (mask [numint][nchan] uint8, padvals [nchan] float32)."""
    numint = (obs.N + ptsperint - 1) // ptsperint
    rng = np.random.default_rng(seed)
    mask = (rng.random((numint, obs.nchan)) < frac).astype(np.uint8)
    for i in range(synth.rfi_nchan):
        mask[:, synth.rfi_chan[i]] = 1
    # pad values: per-channel bandpass level (what rfifind's .stats median would give),
    # deliberately non-integer so the float path is exercised.
    x = (np.arange(obs.nchan) / max(obs.nchan - 1, 1)) - 0.5
    padvals = (synth.base_level * (1.0 + synth.bandpass_slope * x)).astype(np.float32)
    return mask, padvals
