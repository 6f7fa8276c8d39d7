"""Stage 1 of several DDplan stages in one call (hd_run_subband_multi with mixed ds): the
passes of every stage with ds in {2, 3, 5, 6, 10} share one k_stage1_q8m launch (tiles of
4 x 960 raw rows, one channel-major fill for all of them), then per stage the float kernel's
special tiles, and one k_stage1_fix8 launch (per-pass ds) for the clipped-spectrum /
block-boundary outputs of all of them.  Every pass must equal its own oracle run, the
per-stage fixups (HD_FIX8M=0) and the per-stage launches (HD_Q8M=0) -- over 8/4-bit data, flipped bands,
int16 and float32 subbands, mean and sum downsampling, masks whose blocks a tile crosses
(two- and three-block tiles, and wider ones on the special list), cps 8 / 10 / 16."""
import numpy as np
import pytest

import oracle as OR
from hipdedisp import Opts, PassParams, plan
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth, synth_mask

pytestmark = pytest.mark.gpu

# (stage, pass) of the Mock DDplan: ds 1 (run alone), 2, 3, 5, 6, 10; two passes of stage 1
PASSES = ((0, 5), (1, 0), (1, 11), (2, 3), (3, 7), (4, 2), (5, 0))


def mixed_plans(engine, nsub, N):
    pps = []
    for st, i in PASSES:
        d = plan.ddplans_for("pdev")[st]
        pps.append(PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                              numdms=8, nsub=nsub, ds=d.sub_downsamp, numout=plan.choose_N(N / d.downsamp)))
    order = [3, 0, 6, 1, 5, 2, 4]                 # stages interleaved in the call
    pps = [pps[k] for k in order]
    return pps, [engine.plan(pp) for pp in pps]


def subband_launches(plans):
    """Plans whose stage-1 events hold a launch's time (the first plan of each launch)."""
    return sum(1 for p in plans if p.last_ms()[0] > 0.0)


@pytest.mark.parametrize("nbits,nsub,flip,sub_dtype,ds_mode,pts,extra", [
    (8, 96, False, 0, 1, 8192, 776),   # the bench's case: mean, int16, mask blocks of 8192 rows
    (8, 96, True, 0, 0, 2048, 776),    # tiles across 3+ blocks: special list and 3-block tiles
    (8, 120, False, 1, 1, 0, 776),     # cps 8, float32 subbands, no mask
    (8, 60, True, 1, 0, 4096, 776),    # cps 16 (ds 10 exceeds its packed sums: per-stage launch)
    (4, 96, False, 0, 1, 8192, 776),   # 4-bit data through its unpacked channel-major copy
    (8, 96, False, 0, 1, 8192, 777),   # N % 4 != 0: no channel-major copy, per-stage launches
])
def test_fused_stage1_bitexact(engine, monkeypatch, nbits, nsub, flip, sub_dtype, ds_mode, pts, extra):
    N = (1 << 19) + extra
    obs = palfa_obs(N=N, nbits=nbits, flip=flip)
    opts = Opts(sub_dtype=sub_dtype, ds_mode=ds_mode)
    s = palfa_synth(nbits=nbits)
    engine.set_obs(obs, opts)
    engine.synth_device(s)
    raw = host_spectra(obs, s)
    mask = pad = None
    if pts:
        mask, pad = synth_mask(obs, s, pts, frac=0.1)
        engine.set_mask(mask, pts, pad)
    pps, plans = mixed_plans(engine, nsub, N)
    try:
        monkeypatch.setenv("HD_Q8M", "1")
        engine.run_subband_multi(plans)
        engine.sync()
        fused = [p.get_subbands() for p in plans]
        # ds 1 alone, then one launch for the ds >= 2 stages the fused kernel takes
        assert subband_launches(plans) == (6 if N % 4 else 3 if nsub == 60 else 2)
        cl = OR.prepare(obs, opts, raw, mask=mask, ptsperint=pts, padvals=pad, omp=True)
        for pp, g in zip(pps, fused):
            want = OR.stage1(obs, opts, raw, nsub, pp.ds, pp.subdm, clean=cl, omp=True)
            assert np.array_equal(g, want), (pp.ds, pp.subdm)
        monkeypatch.setenv("HD_FIX8M", "0")                  # fixups per DDplan stage
        engine.run_subband_multi(plans)
        engine.sync()
        for p, g in zip(plans, fused):
            assert np.array_equal(p.get_subbands(), g)
        monkeypatch.setenv("HD_Q8M", "0")
        engine.run_subband_multi(plans)
        engine.sync()
        assert subband_launches(plans) == 6             # one per ds
        for p, g in zip(plans, fused):
            assert np.array_equal(p.get_subbands(), g)
    finally:
        for p in plans:
            p.destroy()
        if pts:
            engine.set_mask()


def test_fused_stage1_then_stage2_repeated_beams(engine):
    """The bench's order (one fused stage-1 call, then every stage's stage-2 launch) over
    alternating beams: the series equal the per-stage schedule's."""
    N = (1 << 19) + 776
    obs = palfa_obs(N=N, nbits=8)
    engine.set_obs(obs, Opts())
    synths = [palfa_synth(beam=0), palfa_synth(beam=1)]
    pts = 8192
    mask, pad = synth_mask(obs, synths[0], pts)
    engine.set_mask(mask, pts, pad)
    pps, plans = mixed_plans(engine, 96, N)
    try:
        want = []
        for k in range(2):
            engine.synth_device(synths[k])
            for ds in sorted({pp.ds for pp in pps}):
                engine.run_subband_multi([p for pp, p in zip(pps, plans) if pp.ds == ds])
            want.append([p.run_dedisp() for p in plans])
        for it in range(3):
            k = it % 2
            engine.synth_device(synths[k])
            engine.run_subband_multi(plans)
            for ds in sorted({pp.ds for pp in pps}):
                engine.run_dedisp_multi([p for pp, p in zip(pps, plans) if pp.ds == ds])
            for j, p in enumerate(plans):
                assert np.array_equal(p.get_series(0, None, 0, p.numout), want[k][j]), (it, j)
    finally:
        for p in plans:
            p.destroy()
        engine.set_mask()
