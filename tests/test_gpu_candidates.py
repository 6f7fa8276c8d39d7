"""North star: identical accelsearch candidate lists on an injected-pulsar beam, the periodicity
half checked on INDEPENDENT paths (PALFA2_presto_search.py:548-558):

* device: stage 1 + stage 2 on the GPU, then hd_realfft -> hd_zapbirds (the reference's own
  PALFA.zaplist) -> hd_rednoise on the device series (float32 hipFFT);
* oracle: the oracle's OWN series (prepsubband restatement, oracle.run_pass), then
  fft_oracle's realfft (float64) -> zap -> rednoise, with the zap ranges from fft_oracle's
  own birdie_bins.

Candidates (tests/candidates.spectrum_candidates): per DM and harmonic count (1, 2, 4, 8) every
fundamental bin whose summed normalised power exceeds the stated threshold.  Bar: the two
lists identical as (DM, harmonics, bin) sets, except entries whose power lies within a
relative 1e-3 of the threshold (the FFT tolerance: float32 vs float64 transforms,
test_gpu_fft.py), and powers of common entries within 1e-3.  The injected 4.6 ms pulsar's
fundamental is among them at DM ~71.  Negative case: the oracle with clip_times off
(-noclip) must give a list that differs beyond that tolerance.  Parity with PRESTO unpinned."""
import json
import os

import numpy as np
import pytest

import fft_oracle as FO
import oracle as OR
from candidates import candidate_mismatch, spectrum_candidates
from hipdedisp import Opts, PassParams
from hipdedisp import fft_stage as FS
from hipdedisp import plan
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask

HERE = os.path.dirname(os.path.abspath(__file__))
N = 1 << 18


def zaplist():
    g = json.load(open(os.path.join(HERE, "golden", "palfa_zaplist.json")))
    return [tuple(b) for b in g["birdies"]]


def setup_beam():
    obs = palfa_obs(N=N, nbits=8)
    s = palfa_synth()
    pts = rfifind_ptsperint(obs.dt)
    mask, pad = synth_mask(obs, s, pts)
    d0 = plan.ddplans_for("pdev")[0]
    k = next(i for i in range(d0.numpasses) if float(d0.dmlist[i][0]) <= 71.0 <= float(d0.dmlist[i][-1]))
    pp = PassParams(subdm=float(d0.subdmlist[k]), lodm=float(d0.lodm_arg(k)), dmstep=float(d0.dmstep_arg()),
                    numdms=d0.dmsperpass, nsub=d0.numsub, ds=1, numout=plan.choose_N(N))
    return obs, s, pts, mask, pad, pp


def oracle_candidates(obs, raw, pp, mask, pts, pad, opts):
    _, x = OR.run_pass(obs, opts, raw, pp, mask=mask, ptsperint=pts, padvals=pad, omp=True)
    T = pp.numout * obs.dt
    nb = pp.numout // 2
    F = FO.realfft(x).astype(np.complex64)
    F = FO.zap(F, FO.zap_ranges(*FO.birdie_bins(zaplist(), T), nb))
    F = FO.rednoise(F, FO.rednoise_blocks(nb, T))
    return spectrum_candidates(F)


def test_oracle_candidates_clip_sensitive():
    """CPU: the negative case's premise -- clip_times on and off give different lists -- and
    the pulsar's fundamental in the clipped list (no GPU)."""
    obs, s, pts, mask, pad, pp = setup_beam()
    raw = host_spectra(obs, s)
    a = oracle_candidates(obs, raw, pp, mask, pts, pad, Opts())
    b = oracle_candidates(obs, raw, pp, mask, pts, pad, Opts(clip_sigma=0.0))
    assert candidate_mismatch(a, b)
    f0 = int(round(N * obs.dt / 0.0046))
    hits = [k for k in a if k[1] == 1 and abs(k[2] - f0) <= 1]
    assert hits
    best = max(hits, key=lambda k: a[k])
    assert abs(pp.lodm + best[0] * pp.dmstep - 71.0) <= 1.5


@pytest.mark.gpu
def test_periodicity_candidates_independent_paths(engine):
    obs, s, pts, mask, pad, pp = setup_beam()
    engine.set_obs(obs, Opts())
    engine.synth_device(s)
    engine.set_mask(mask, pts, pad)
    p = engine.plan(pp)
    try:
        p.run_subband()
        p.run_dedisp(to_host=False)
        T = p.numout * p.sub_dt
        FS.realfft(p)
        FS.zapbirds(p, *FS.birdie_bins(zaplist(), T))
        FS.rednoise(p, T)
        dev = spectrum_candidates(FS.spectra_complex(FS.get_fft(p)))
    finally:
        p.destroy()
        engine.set_mask()
    raw = host_spectra(obs, s)
    ora = oracle_candidates(obs, raw, pp, mask, pts, pad, Opts())
    assert len(dev) > 10
    assert candidate_mismatch(dev, ora) == []
    f0 = int(round(N * obs.dt / 0.0046))
    assert any(k[1] == 1 and abs(k[2] - f0) <= 1 for k in dev)
    noclip = oracle_candidates(obs, raw, pp, mask, pts, pad, Opts(clip_sigma=0.0))
    assert candidate_mismatch(dev, noclip)                  # the comparison discriminates
