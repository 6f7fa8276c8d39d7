"""Whole-beam parity of the bench's own path, every sample (VERDICT r4 "what's missing" #2).

C2 (BASELINE.json configs[1]): the PALFA Mock beam of 960 channels x 2^22 spectra at 8 bits and
at 4 bits (PALFA's production format: lib/python/datafile.py:398, config/download_example.py:34
-- the nibbles unpacked by k_raw_transpose<4> into the channel-major copy, then the same integer
kernels as 8 bits: q8, the fused q8m, fix8),
rfifind-style mask, clipping on, run exactly as `bench.py` runs a step (`run_step`): the
beam's channel-major copy rebuilt (`touch_raw`), stage 1 for the ds = 1 DDplan stage alone and
for the five ds >= 2 stages in ONE `run_subband_multi` call (the fused `k_stage1_q8m` launch
and its one `k_stage1_fix8` launch), stage 2 as one `run_dedisp_multi` launch per DDplan
stage.  Then, for every one of the 57 passes (PALFA2_presto_search.py:494-529): the 96 int16
subbands over their full length and every sample of every DM (4188 trials) against the
OpenMP oracle's `run_pass` -- bit-exact before N/ds, the padded tail within 1e-5 relative.

C4 (DDplan2b 0..10000) is compared the same way in tests/test_gpu_wholebeam_c4.py.

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


def beam_setup(engine, nbits=8):
    obs = palfa_obs(N=N, nbits=nbits)
    s = palfa_synth(nbits=nbits)
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


# ---- C2: the bench beam --------------------------------------------------------------------

def c2_cases():
    out = []
    for st, d in enumerate(plan.ddplans_for("pdev")):
        for i0 in range(0, d.numpasses, CHUNK):
            out.append((st, i0))
    return out


@pytest.fixture(scope="module", params=[8, 4], ids=["8bit", "4bit"])
def c2_beam(engine, request):
    obs, raw, cl = beam_setup(engine, request.param)
    ddplans = plan.ddplans_for("pdev")
    stages = [[(pass_params(d, i)) for i in range(d.numpasses)] for d in ddplans]
    plans = [[engine.plan(pp) for pp in st] for st in stages]
    try:
        # bench.run_step: touch_raw, the ds = 1 stage alone, the ds >= 2 stages fused, then
        # one stage-2 launch per DDplan stage
        engine.touch_raw()
        lone = [st for st in plans if st[0].pp.ds < 2]
        multi = [st for st in plans if st[0].pp.ds >= 2]
        for grp in [[st] for st in lone] + [multi]:
            engine.run_subband_multi([p for st in grp for p in st])
            for st in grp:
                engine.run_dedisp_multi(st)
        engine.sync()
        yield obs, raw, cl, stages, plans
    finally:
        for st in plans:
            for p in st:
                p.destroy()
        engine.set_mask()


def test_c2_bench_path_kernels(c2_beam):
    """The beam ran through the kernels the bench reports (not a fallback variant)."""
    obs, raw, cl, stages, plans = c2_beam
    kern = {p.kernel() for st in plans for p in st}

    def unprobed_pair_kernel(k):      # k_stage2_pair / k_stage2_qp with the probe flag (5th argument) off
        if not k.startswith(("k_stage2_pair<", "k_stage2_qp<")):
            return False
        args = [x.strip() for x in k[k.index("<") + 1:-1].split(",")]
        return len(args) >= 5 and args[4] == "false"
    assert any(unprobed_pair_kernel(k) for k in kern), kern


@pytest.mark.parametrize("stage,i0", c2_cases())
def test_c2_whole_beam_every_sample(c2_beam, stage, i0):
    obs, raw, cl, stages, plans = c2_beam
    for pp, p in list(zip(stages[stage], plans[stage]))[i0:i0 + CHUNK]:
        compare_pass(obs, raw, cl, pp, p)
