"""Whole-beam parity, C4 (DDplan2b 0..10000): every pass of every step, every sample
(VERDICT r4 "what's missing" #2; the C2 half is tests/test_gpu_wholebeam.py).

C2 (BASELINE.json configs[1]): the PALFA Mock beam of 960 channels x 2^22 spectra x 8 bits,
rfifind-style mask, clipping on, run exactly as `bench.py` runs a step (`run_step`): the
beam's channel-major copy rebuilt (`touch_raw`), stage 1 for the ds = 1 DDplan stage alone and
for the five ds >= 2 stages in ONE `run_subband_multi` call (the fused `k_stage1_q8m` launch
and its one `k_stage1_fix8` launch), stage 2 as one `run_dedisp_multi` launch per DDplan
stage.  Then, for every one of the 57 passes (PALFA2_presto_search.py:494-529): the 96 int16
subbands over their full length and every sample of every DM (4188 trials) against the
OpenMP oracle's `run_pass` -- bit-exact before N/ds, the padded tail within 1e-5 relative.

C4 (BASELINE.json configs[3]): the DDplan2b plan 0..10000 pc cm^-3 (93 passes, ds 1..64), each
step through `run_subband_multi` + `run_dedisp_multi`, every pass compared in full the same
way.

The oracle is test infrastructure (oracle/); the device path is libhipdedisp.so.
"""
import numpy as np
import pytest

import oracle as OR
from hipdedisp import Opts, PassParams, plan
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(1200)]

N = 1 << 22
CHUNK = 8                     # passes per test (each test ends well inside the box's silence limit)


def pass_params(d, i):
    return PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                      numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp, numout=plan.choose_N(N / d.downsamp))


def beam_setup(engine):
    obs = palfa_obs(N=N, nbits=8)
    s = palfa_synth()
    engine.set_obs(obs, Opts())
    engine.synth_device(s)
    raw = host_spectra(obs, s)
    pts = rfifind_ptsperint(obs.dt)
    mask, pad = synth_mask(obs, s, pts)
    engine.set_mask(mask, pts, pad)
    cl = OR.prepare(obs, Opts(), raw, mask=mask, ptsperint=pts, padvals=pad, omp=True)
    return obs, raw, cl


def compare_pass(obs, raw, cl, pp, p):
    want_sub, want = OR.run_pass(obs, Opts(), raw, pp, clean=cl, omp=True)
    got_sub = p.get_subbands()
    assert np.array_equal(got_sub, want_sub), ("subbands", pp.subdm)
    del got_sub, want_sub
    got = p.get_series(0, pp.numdms, 0, pp.numout)
    nds = N // pp.ds
    n = min(nds, pp.numout)
    if not np.array_equal(got[:, :n], want[:, :n]):
        bad = np.argwhere(got[:, :n] != want[:, :n])
        raise AssertionError("pass subdm %.2f: %d samples differ, first (dm, t) %s"
                             % (pp.subdm, len(bad), bad[:4].tolist()))
    if pp.numout > nds:
        np.testing.assert_allclose(got[:, nds:], want[:, nds:], rtol=1e-5, atol=0)


# ---- C4: DDplan2b 0..10000 ------------------------------------------------------------------

def c4_steps(obs):
    return plan.ddplan2b_plans(obs.dt, 1375.5, 322.6, obs.nchan, 2048, 0.0, 10000.0, 96, 0.1)


@pytest.fixture(scope="module")
def c4_beam(engine):
    obs, raw, cl = beam_setup(engine)
    yield obs, raw, cl
    engine.set_mask()


@pytest.mark.parametrize("step", range(7))
def test_c4_step_every_sample(engine, c4_beam, step):
    obs, raw, cl = c4_beam
    d = c4_steps(obs)[step]
    pps = [pass_params(d, i) for i in range(d.numpasses)]
    plans = [engine.plan(pp) for pp in pps]
    try:
        engine.run_subband_multi(plans)
        engine.run_dedisp_multi(plans)
        for pp, p in zip(pps, plans):
            compare_pass(obs, raw, cl, pp, p)
    finally:
        for p in plans:
            p.destroy()
