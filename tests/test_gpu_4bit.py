"""4-bit data on the integer stage-1 path (PALFA's production format: the reference's
download config says "4 or 16", lib/python/config/download_example.py:34, and Mock data is
4-bit, lib/python/datafile.py:398).  The raw block is unpacked into the one-byte-per-sample
channel-major copy (k_raw_transpose<4>), so k_stage1_q8 and the LDS-window fixup
(k_stage1_fix8) run it; variant 3 forces the integer kernel, which fails with HD_E_INVAL if it
does not apply, so these tests prove the path taken.  Bar: bit-exact against the oracle."""
import numpy as np
import pytest

import oracle as OR
from hipdedisp import Opts, PassParams, plan
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth, synth_mask

pytestmark = pytest.mark.gpu


def spiky4(frac=0.002):
    s = palfa_synth(nbits=4)
    s.spike_frac = frac                  # zero-DM spikes: clip_times' targets
    s.spike_amp = 6.0
    return s


def setup(engine, obs, opts, synth, pts=8192, frac=0.1):
    engine.set_obs(obs, opts)
    engine.synth_device(synth)
    raw = host_spectra(obs, synth)
    mask, pad = synth_mask(obs, synth, pts, frac=frac)
    engine.set_mask(mask, pts, pad)
    return raw, mask, pad


@pytest.mark.parametrize("ds", [1, 2, 3, 5, 6, 10])
@pytest.mark.parametrize("hi_first,flip", [(True, True), (False, True), (True, False)])
def test_stage1_4bit_integer_path(engine, ds, hi_first, flip):
    """Three passes of one launch at every integer-path ds, masked, clipping on, both nibble
    orders and band orders: the forced integer kernel's subbands equal the oracle's."""
    obs = palfa_obs(N=65536 + 776, nbits=4, nsblk=2048, flip=flip)
    opts = Opts(nibble_hi_first=hi_first)
    s = spiky4()
    raw, mask, pad = setup(engine, obs, opts, s)
    pps = [PassParams(subdm=sd, lodm=sd - 5.0, dmstep=0.5, numdms=4, nsub=96, ds=ds) for sd in (40.0, 350.0, 1020.0)]
    plans = [engine.plan(pp) for pp in pps]
    try:
        for p in plans:
            p.set_variant(3 << 8)
        engine.run_subband_multi(plans)
        cl = OR.prepare(obs, opts, raw, mask=mask, ptsperint=8192, padvals=pad)
        assert cl.nclipped > 10
        for pp, p in zip(pps, plans):
            want = OR.stage1(obs, opts, raw, 96, ds, pp.subdm, clean=cl, omp=True)
            assert np.array_equal(p.get_subbands(), want), pp.subdm
    finally:
        for p in plans:
            p.destroy()
        engine.set_mask()


@pytest.mark.parametrize("stage", [0, 4])
def test_4bit_full_stage_fixups_agree(engine, stage):
    """All passes of a Mock DDplan stage in one launch at 4 bits: the LDS-window fixup over
    the unpacked copy and the generic per-cell fixup (probe bit 128, packed rows) give
    identical subbands; pass 0 equals the oracle."""
    obs = palfa_obs(N=1 << 17, nbits=4, nsblk=2048)
    s = spiky4()
    raw, mask, pad = setup(engine, obs, Opts(), s, pts=16384, frac=0.05)
    d = plan.ddplans_for("pdev")[stage]
    pps = [PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                      numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp) for i in range(d.numpasses)]
    plans = [engine.plan(pp) for pp in pps]
    try:
        engine.run_subband_multi(plans)
        fast = [p.get_subbands() for p in plans]
        for p in plans:
            p.set_variant(128 << 16)
        engine.run_subband_multi(plans)
        for i, p in enumerate(plans):
            assert np.array_equal(p.get_subbands(), fast[i]), i
        cl = OR.prepare(obs, Opts(), raw, mask=mask, ptsperint=16384, padvals=pad)
        assert cl.nclipped > 50
        want = OR.stage1(obs, Opts(), raw, d.numsub, d.sub_downsamp, pps[0].subdm, clean=cl, omp=True)
        assert np.array_equal(fast[0], want)
    finally:
        for p in plans:
            p.destroy()
        engine.set_mask()


@pytest.mark.parametrize("ds", [1, 5])
def test_4bit_pass_series_bitexact(engine, ds):
    """A whole 76-DM pass at 4 bits (stage 1 on the integer path, stage 2 auto: the pair
    kernel at ds 1), masked and clipped: subbands and series equal the oracle; the padded
    tail within the 1e-5 relative bound."""
    obs = palfa_obs(N=1 << 17, nbits=4, nsblk=2048)
    s = spiky4()
    raw, mask, pad = setup(engine, obs, Opts(), s, pts=16384, frac=0.05)
    pp = PassParams(subdm=71.10, lodm=68.20, dmstep=0.1 if ds == 1 else 0.5, numdms=76, nsub=96, ds=ds,
                    numout=plan.choose_N(obs.N / ds))
    p = engine.plan(pp)
    try:
        p.set_variant(3 << 8)
        p.run_subband()
        got_sub = p.get_subbands()
        p.set_variant(0)
        got = p.run_dedisp()
        want_sub, want = OR.run_pass(obs, Opts(), raw, pp, mask=mask, ptsperint=16384, padvals=pad, omp=True)
        assert np.array_equal(got_sub, want_sub)
        nds = obs.N // ds
        assert np.array_equal(got[:, :nds], want[:, :nds])
        np.testing.assert_allclose(got[:, nds:], want[:, nds:], rtol=1e-5, atol=0)
    finally:
        p.destroy()
        engine.set_mask()
