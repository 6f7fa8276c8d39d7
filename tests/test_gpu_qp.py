"""The quarter-layout pair kernel (k_stage2_qp, hd_plan_set_variant s2 = 9) through the bench's
multi-pass launch (hd_run_dedisp_multi): for every Mock DDplan stage (PALFA2_presto_search.py:
319-326), three passes of a ragged masked beam with more tiles than CUs share one launch; each
series equals the auto kernel's one-pass result (the pair kernel, or the ring where the pair
kernel's LDS does not fit) bit for bit, and one pass per stage equals the oracle.  Stage 2 reference: PALFA2_presto_search.py:514-520.
"""
import numpy as np
import pytest

import oracle as OR
from hipdedisp import Opts, PassParams, plan
from hipdedisp.synth import palfa_obs, palfa_synth, synth_mask
from test_gpu_parity import assert_series, load_beam

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("stage", range(6))
def test_qp_multipass_stage_matches_pair_and_oracle(engine, stage):
    obs = palfa_obs(N=(1 << 19) + 777, nbits=8)
    synth = palfa_synth()
    raw = load_beam(engine, obs, synth=synth)
    pts = 2048
    mask, pad = synth_mask(obs, synth, pts)
    engine.set_mask(mask, pts, pad)
    d = plan.ddplans_for("pdev")[stage]
    idx = sorted({0, d.numpasses // 2, d.numpasses - 1})
    pps = [PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                      numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp, numout=plan.choose_N(obs.N / d.downsamp))
           for i in idx]
    plans = [engine.plan(pp) for pp in pps]
    try:
        engine.run_subband_multi(plans)
        ref = []
        for p in plans:
            p.set_variant(0)                 # the auto one-pass kernel (pair, or the ring where its LDS does not fit)
            ref.append(p.run_dedisp())
        for p in plans:
            p.set_variant(9)
        engine.run_dedisp_multi(plans)
        n = [p.launch_passes() for p in plans]      # one shared launch at the passes' smallest pairs-per-chunk
        assert sum(n) == len(plans) and n[0] >= 1, n
        for p, r in zip(plans, ref):
            assert p.kernel().startswith("k_stage2_qp<"), p.kernel()
            assert np.array_equal(p.get_series(0, None, 0, p.numout), r)
        _, want = OR.run_pass(obs, Opts(), raw, pps[-1], mask=mask, ptsperint=pts, padvals=pad, omp=True)
        assert_series(ref[-1], want, obs.N // pps[-1].ds)
    finally:
        for p in plans:
            p.destroy()
        engine.set_mask()


@pytest.mark.parametrize("N", [700, 767, 768, 769, 5000])
def test_qp_stage2_short_beams(engine, N):
    """Beams of less than one to a few 768-sample tiles (every quarter's ragged tail)."""
    obs = palfa_obs(N=N, nbits=8)
    raw = load_beam(engine, obs)
    pp = PassParams(subdm=3.8, lodm=0.0, dmstep=0.1, numdms=76, nsub=96, ds=1, numout=0)
    p = engine.plan(pp)
    try:
        p.run_subband()
        p.set_variant(9)
        got = p.run_dedisp()
        _, want = OR.run_pass(obs, Opts(), raw, pp)
        assert_series(got, want, obs.N)
    finally:
        p.destroy()


@pytest.mark.parametrize("nsub", [120, 60])
def test_qp_odd_chunk_count_persistent(engine, nsub):
    """tiles with an odd chunk count (nsub 120 at 4 pairs per chunk: 15
    chunks; nsub 60 at 2: 15) on persistent workgroups that each take several tiles (683 tiles
    over the CUs) -- the kernel's running buffer parity and the offsets table's in-tile parity
    differ on every other tile.  Single-pass and shared launches bit-exact vs the oracle."""
    obs = palfa_obs(N=1 << 19, nbits=8)
    raw = load_beam(engine, obs)
    steps = {120: (0.1, 0.3), 60: (0.3, 0.3)}[nsub]
    pps = [PassParams(subdm=lodm + 38 * st, lodm=lodm, dmstep=st, numdms=76, nsub=nsub, ds=2, numout=0)
           for lodm, st in ((212.8, steps[0]), (443.2, steps[1]))]
    plans = [engine.plan(pp) for pp in pps]
    try:
        engine.run_subband_multi(plans)
        want = [OR.run_pass(obs, Opts(), raw, pp, omp=True)[1] for pp in pps]
        for p, w in zip(plans, want):
            p.set_variant(9)
            assert_series(p.run_dedisp(), w, obs.N // 2)
        engine.run_dedisp_multi(plans)
        assert plans[0].launch_passes() == 2, [p.launch_passes() for p in plans]
        k = plans[0].kernel()
        ppc = int(k.split(",")[2])
        assert (nsub // 2 // ppc) % 2 == 1, k            # the case the test is for
        for p, w in zip(plans, want):
            assert_series(p.get_series(0, None, 0, p.numout), w, obs.N // 2)
    finally:
        for p in plans:
            p.destroy()


def test_qp_merged_pairs_per_chunk(engine):
    """passes whose own pairs-per-chunk differ (4, 3, 2 at ds 2) share ONE
    launch at the smallest, the others through their smaller-ppc offset tables (boffp);
    bit-exact against their single-pass runs and the oracle."""
    obs = palfa_obs(N=(1 << 19) + 777, nbits=8)
    raw = load_beam(engine, obs)
    pps = [PassParams(subdm=lodm + 38 * st, lodm=lodm, dmstep=st, numdms=76, nsub=96, ds=2, numout=plan.choose_N(obs.N / 2))
           for lodm, st in ((600.0, 0.3), (50.0, 0.3), (100.0, 0.5))]
    plans = [engine.plan(pp) for pp in pps]
    try:
        engine.run_subband_multi(plans)
        ref = []
        for p in plans:
            p.set_variant(9)
            ref.append(p.run_dedisp())
        own = [int(p.kernel().split(",")[2]) for p in plans]
        assert own == [4, 3, 2], own
        engine.run_dedisp_multi(plans)
        assert [p.launch_passes() for p in plans] == [3, 0, 0]
        assert plans[0].kernel().split(",")[2].strip() == "2", plans[0].kernel()
        for p, r in zip(plans, ref):
            assert np.array_equal(p.get_series(0, None, 0, p.numout), r)
        _, want = OR.run_pass(obs, Opts(), raw, pps[0], omp=True)
        assert_series(ref[0], want, obs.N // 2)
    finally:
        for p in plans:
            p.destroy()
