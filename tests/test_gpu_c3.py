"""Config 3 at full size (BASELINE.json configs[2]): the C2 beam -- 960 channels x 2^22
spectra x 8 bits, the full 57-pass Mock DDplan (4188 DM trials), an rfifind-style mask,
clipping on -- cut into the time slices of hipdedisp.sharding.TimeSlices at world 4 and 8,
every rank's slice run in turn on its own context of this one GPU.  The ranks' two
exchanges are the real ones: hd_clip_stats of each slice's own read blocks, summed on the
host where the node all-reduces over RCCL, then hd_clip_set_stats; and the per-pass series
sums that fix the last rank's padding.  Checked against the whole beam on one context
(itself checked against the oracle by test_gpu_c2.py), bit for bit:

* every rank's exchange rows of its first and last owned read blocks equal the oracle's
  clip_times statistics (oracle.clip_rows) of those blocks;
* every rank's clip flags and per-block pad values equal the whole beam's;
* for every pass and every rank: windows of all DMs at the start and the end of the rank's
  owned output range (so both sides of every slice boundary), the window around the output
  whose raw reads cross byte 2^31 of the whole beam, and the exact sum of every DM over the
  rank's owned range (a checksum of the whole series);
* the padded tail of every padded pass on the last rank.

Reference: lib/python/PALFA2_presto_search.py:494-529 (the pass loop being split).
"""
import numpy as np
import pytest

import oracle as OR
from hipdedisp import Engine, Opts, PassParams, plan as P
from hipdedisp import sharding as S
from hipdedisp.synth import host_spectra, palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

N = 1 << 22
W = 2048                        # window length (output samples)
OFF31 = (1 << 31) // 960 + 1    # first spectrum starting past byte 2^31 of the whole raw block


def pass_params(obs, d, i, numout):
    return PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                      numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp, numout=numout)


@pytest.mark.parametrize("world", [4, 8])
def test_c3_time_slices_full_beam(engine, world):
    obs = palfa_obs(N=N, nbits=8)
    s = palfa_synth()
    pts = rfifind_ptsperint(obs.dt)
    mask, pad = synth_mask(obs, s, pts)
    ddplans = P.ddplans_for("pdev")
    ts = S.TimeSlices(obs, ddplans, world)
    engine.set_obs(obs, Opts())
    engine.synth_device(s)
    engine.set_mask(mask, pts, pad)
    gpad, gclip, _, ncl = engine.get_clean()
    assert ncl > 1000                                    # the beam's zero-DM spikes are clipped
    engs = []
    try:
        # phase A: every rank's statistics of its own read blocks -> the "all-reduce"
        table = ts.stats_table()
        for r in range(world):
            e = Engine(0)
            engs.append(e)
            t0, own, nloc = ts.slice(r)
            e.set_obs(ts.local_obs(r), Opts())
            e.set_slice(t0, obs.N)
            e.synth_device(s)
            e.set_mask(mask, pts, pad)
            mine = ts.stats_table()
            ts.contribute_clip_stats(e, r, mine)
            b0, nb = t0 // ts.blk, ts.nown_blocks(r)
            assert not mine[:b0].any() and not mine[b0 + nb:].any()
            for bb in (b0, b0 + 1, b0 + nb - 2, b0 + nb - 1):  # the oracle's rows of the same blocks
                raw = host_spectra(obs, s, bb * ts.blk, min(ts.blk, obs.N - bb * ts.blk))
                want = OR.clip_rows(obs, Opts(), raw, bb, 1, mask=mask, ptsperint=pts)
                assert np.array_equal(mine[bb:bb + 1], want), (r, bb)
            table += mine
        # phase B: clip_times finished on every slice == the whole beam's
        for r, e in enumerate(engs):
            e.clip_set_stats(table)
            t0, own, nloc = ts.slice(r)
            lpad, lclip, _, _ = e.get_clean()
            assert np.array_equal(lclip[:own], gclip[t0:t0 + own]), r
            nb = ts.nown_blocks(r)
            assert np.array_equal(lpad[:nb], gpad[t0 // ts.blk:t0 // ts.blk + nb]), r
        # every DDplan stage: the whole beam, then each rank's slice of it
        for d in ddplans:
            ds = d.sub_downsamp
            numout = P.choose_N(obs.N / d.downsamp)
            whole = [engine.plan(pass_params(obs, d, i, numout)) for i in range(d.numpasses)]
            last = []
            try:
                engine.run_subband_multi(whole)
                for p in whole:
                    p.run_dedisp(to_host=False)
                sums = np.zeros(d.numpasses)
                for r, e in enumerate(engs):
                    t0, own, nloc = ts.slice(r)
                    j0, nj = ts.out_range(r, ds)
                    ps = [e.plan(pass_params(ts.local_obs(r), d, i, ts.numout_local(r, numout, ds)))
                          for i in range(d.numpasses)]
                    try:
                        e.run_subband_multi(ps)
                        for p in ps:
                            p.run_dedisp(to_host=False)
                        wins = {0, max(0, nj - W)}
                        j31 = OFF31 // ds - W // 2
                        if j0 <= j31 < j0 + nj - W:
                            wins.add(j31 - j0)
                        for i, (pw, p) in enumerate(zip(whole, ps)):
                            for jl in sorted(wins):
                                n = min(W, nj - jl)
                                assert np.array_equal(p.get_series(0, None, jl, n),
                                                      pw.get_series(0, None, j0 + jl, n)), (ds, i, r, jl)
                            for dm in range(d.dmsperpass):
                                a = p.series_sum(dm, 0, nj)
                                assert a == pw.series_sum(dm, j0, nj), (ds, i, r, dm)
                                if dm == 0:
                                    sums[i] += a
                    finally:
                        if r == world - 1:
                            last = ps
                        else:
                            for p in ps:
                                p.destroy()
                # phase D: the last rank pads with the observation's first-DM mean
                ts.pad_passes(world - 1, last, sums)
                j0, nj = ts.out_range(world - 1, ds)
                for pw, p in zip(whole, last):
                    if p.numout > nj:
                        assert p.numout == numout - j0
                        tail = p.get_series(0, None, nj, p.numout - nj)
                        assert np.array_equal(tail, pw.get_series(0, None, j0 + nj, numout - j0 - nj)), ds
            finally:
                for p in whole + last:
                    p.destroy()
    finally:
        for e in engs:
            e.close()
        engine.set_mask()
