"""Benchmark: full PALFA-beam dedispersion (BASELINE.json metric) on MI355X.

A step = one whole beam through the reference's Mock DDplan: 57 passes x (stage 1
subbanding + stage 2 DM sweep), 4188 DM trials of N/ds samples each, inputs (raw beam,
mask) resident in HBM, outputs left resident (no .dat writes: the end-to-end file path is
measured separately).  At N GPUs every rank dedisperses its own beam (the
7-beam ALFA pointing of configs[4]; per-GPU work fixed -> "weak" scaling); value = total
output samples of all ranks / max-over-ranks wall time.

  python bench.py --gpus N --steps K --warmup W
  torchrun --nproc-per-node N ... bench.py --gpus N ...     (one rank per GPU)
"""
import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "pipeline2.0_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

METRIC = "dedispersed samples/sec (DM-trials x samples/s, node) + % HBM peak, PALFA beam"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_ADD_PEAK = 78.6e12        # fp32 vector adds/s (157.3 TFLOPS / 2), SURVEY §8d


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--nspec", type=int, default=1 << 22, help="spectra per beam (2^22 = config 2)")
    ap.add_argument("--nbits", type=int, default=8)
    ap.add_argument("--variant", type=int, default=0,
                    help="hd_plan_set_variant value for every plan (0 auto; probe bits are for profiling only)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU-baseline leg")
    ap.add_argument("--streams", type=int, default=1, choices=(1, 2, 3),
                    help="stage-2 HIP streams (hd_set_streams): 2 overlaps consecutive passes (no launch tails), 3 runs "
                         "stage 2 on its own stream so the next DDplan stage's stage 1 overlaps it; per-kernel event "
                         "times then include the shared time, so the roofline is taken at 1")
    ap.add_argument("--dd-single", action="store_true",
                    help="stage 2 as one launch per pass (hd_run_dedisp) instead of one launch per DDplan stage "
                         "(hd_run_dedisp_multi)")
    ap.add_argument("--s1-per-stage", action="store_true",
                    help="stage 1 as one hd_run_subband_multi call per DDplan stage instead of one for every "
                         "stage with ds >= 2 (the fused k_stage1_q8m launch)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU work for the baseline sample")
    # the legs after the timed steps characterise one GPU: by default (-1) they run at world
    # size 1 only (8 ranks each writing a beam's 47 GB of .dat files, or two 4 GB PSRFITS
    # beams, would share one host's tmpfs)
    ap.add_argument("--e2e-beams", type=int, default=-1,
                    help="beams run end to end (.dat/.inf files written) after the timed steps; 0 = skip")
    ap.add_argument("--sp-beams", type=int, default=-1,
                    help="beams of single-pulse search (hd_single_pulse) timed after the steps; 0 = skip")
    ap.add_argument("--fft-beams", type=int, default=-1,
                    help="beams of realfft + zapbirds + rednoise (hd_fft.hip) timed after the steps; 0 = skip")
    ap.add_argument("--rfi-beams", type=int, default=-1,
                    help="beams of rfifind statistics + mask decisions (hd_rfi.hip) timed last; 0 = skip")
    ap.add_argument("--stream-beams", type=int, default=-1,
                    help="beams of the overlapped PSRFITS-streaming leg (configs[4]; prefetch thread; 3 at world "
                         "size 1), run last; 0 = skip")
    ap.add_argument("--beams", type=int, default=7,
                    help="--mode pointing: beams of the ALFA pointing (configs[4]: 7)")
    ap.add_argument("--helper-frac", type=float, default=None,
                    help="--mode pointing: each home rank's share of its beam (default: balanced by the slice "
                         "cost model, sharding.helper_fraction)")
    ap.add_argument("--mode", choices=["beam", "slices", "shard", "pointing"], default="beam",
                    help="beam: one beam per rank (weak scaling, configs[4]); slices: ONE beam cut into per-rank "
                         "time slices, every rank runs all 57 passes on its slice (strong, configs[2]; RCCL carries "
                         "only the clip statistics and padding sums); shard: ONE beam's passes LPT-sharded after "
                         "an RCCL broadcast of the raw block (strong, the round-1 design, kept for comparison); "
                         "pointing: --beams beams on the node's ranks (configs[4]): ranks 0..beams-1 take the head of "
                         "their beam, the remaining ranks the tails of every beam (time slices, one-way exchanges)")
    ap.add_argument("--check-union", action="store_true",
                    help="--mode slices: after the timed steps, gather every rank's exact per-DM sums of its owned "
                         "series (and the last rank's padding values) and check, on rank 0, that their union equals a "
                         "whole-beam one-context run of the same beam")
    ap.add_argument("--comm", choices=["torch", "hd"], default="torch",
                    help="--mode slices: the two exchanges over torch.distributed (default) or over the library's own "
                         "RCCL communicator (hd_comm_*: hd_slice_exchange_clip, hd_comm_allreduce_sum_f64), the path a "
                         "C caller takes; inside this torch process it measured far slower (a second RCCL "
                         "instance beside torch's, INTEGRATION.md), so it checks the path, not its speed")
    ap.add_argument("--sim-slice", default=None, metavar="R/G",
                    help="--mode slices on ONE process: run only rank R's slice of a G-way cut (no collectives; the "
                         "other ranks' clip statistics are absent, so only the timing is meaningful) -- the per-rank "
                         "compute time behind the multi-GPU prediction, not a scaling measurement")
    return ap.parse_args()


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist
        # one rank per GPU; HD_DIST_BACKEND=gloo (and ranks sharing a GPU) only to rehearse the
        # multi-rank logic on a one-GPU box -- the node run is RCCL ("nccl" on ROCm) over xGMI
        local = local % max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local)
        dist.init_process_group(os.environ.get("HD_DIST_BACKEND", "nccl"), init_method="env://")
        return world, rank, local, dist, torch
    return 1, 0, 0, None, None


def barrier(dist, torch):
    if dist is not None:
        dist.barrier()


def max_over_ranks(x, dist, torch):
    if dist is None:
        return x
    t = torch.tensor([x], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def build_plans(eng, obs, ddplans, variant):
    """Plans grouped by DDplan stage: [[plan, ...] per stage]."""
    from hipdedisp import PassParams, plan as P
    stages = []
    for d in ddplans:
        plans = []
        stages.append(plans)
        for i in range(d.numpasses):
            pp = PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)),
                            dmstep=float(d.dmstep_arg()), numdms=d.dmsperpass, nsub=d.numsub,
                            ds=d.sub_downsamp, numout=P.choose_N(obs.N / d.downsamp))
            p = eng.plan(pp)
            p.dmstrs = list(d.dmlist[i])
            if variant:
                p.set_variant(variant)
            plans.append(p)
    return stages


def run_step(eng, stages):
    """One beam: per DDplan stage, stage 1 for all its passes from one raw read, then the
    stage-2 sweep of each pass.  Every step is a new beam for the engine (hd_touch_raw), so
    the per-beam channel-major copy of the raw block is rebuilt and timed in each step."""
    eng.touch_raw()
    for grp in subband_groups(stages):
        eng.run_subband_multi([p for st in grp for p in st])
        for plans in grp:
            run_dedisp_stage(eng, plans)
    eng.sync()


DD_MULTI = True
S1_FUSE = True


def subband_groups(stages):
    """The beam's stage-1 calls: the ds = 1 stage alone, then every stage with ds >= 2 in one
    hd_run_subband_multi call (one k_stage1_q8m launch reads the channel-major copy once for
    all of them); with --s1-per-stage one call per DDplan stage."""
    live = [st for st in stages if st]
    if not S1_FUSE:
        return [[st] for st in live]
    lone = [[st] for st in live if st[0].pp.ds < 2]
    multi = [st for st in live if st[0].pp.ds >= 2]
    return lone + ([multi] if multi else [])


def run_dedisp_stage(eng, plans):
    """Stage 2 of one DDplan stage's passes: one pair-kernel launch for all of them
    (hd_run_dedisp_multi), or one per pass with --dd-single."""
    if DD_MULTI:
        eng.run_dedisp_multi(plans)
    else:
        for p in plans:
            p.run_dedisp(to_host=False)


def single_pulse_leg(eng, stages, beams):
    """single_pulse_search.py over every DM of the beam (PALFA2_presto_search.py:539-546):
    hd_single_pulse on each pass's device-resident series (as left by the timed steps),
    candidates back on the host; wall seconds per beam and the candidate count."""
    from hipdedisp import single_pulse as SP
    plans = [p for st in stages for p in st]

    def beam():
        n = 0
        for _, hits, _ in SP.device_candidates_many(plans, 0.1, 5.0):
            n += len(hits)
        return n

    eng.sync()
    t = time.perf_counter()
    ncand0 = beam()                               # the first beam also sizes the context's search pool
    first = time.perf_counter() - t
    t = time.perf_counter()
    ncand = 0
    for _ in range(beams):
        ncand += beam()
    s = (time.perf_counter() - t) / beams
    assert ncand == ncand0 * beams, "single-pulse candidates differ between beams"
    return {"s_per_beam": s, "first_beam_s": first, "candidates_per_beam": ncand // beams,
            "note": "hd_single_pulse over the 57 passes' series in HBM (-m 0.1 -t 5.0): detrend, block stds, "
                    "boxcars, prune_related1 on the GPU; prune_related2 + border cases on the host, the device "
                    "searches of the next 4 passes queued meanwhile (hd_single_pulse_launch/_collect); wall time "
                    "per beam after one untimed beam (first_beam_s: that beam, which also allocates the "
                    "context's pooled search buffers)"}


def fft_leg(eng, stages, beams):
    """realfft; zapbirds -zap; rednoise over every DM of the beam (PALFA2_presto_search.py:548-558)
    on each pass's device-resident series: wall seconds per beam, with the reference's own
    zaplist (lib/zaplists/PALFA.zaplist, committed as tests/golden/palfa_zaplist.json)."""
    from hipdedisp import fft_stage as FS
    birds = [tuple(b) for b in json.load(open(os.path.join(ROOT, "tests", "golden", "palfa_zaplist.json")))["birdies"]]
    bins = {}

    def beam():
        for plans in stages:
            for p in plans:
                T = p.numout * p.sub_dt
                FS.realfft(p)
                if p.numout not in bins:
                    bins[p.numout] = FS.birdie_bins(birds, T)
                FS.zapbirds(p, *bins[p.numout])
                FS.rednoise(p, T)
        eng.sync()

    t = time.perf_counter()
    for plans in stages:                          # hipFFT plans (rocFFT kernel builds), one per geometry
        if plans:
            FS.prepare(plans[0])
    prep = time.perf_counter() - t
    t = time.perf_counter()
    beam()
    first = time.perf_counter() - t
    t = time.perf_counter()
    for _ in range(beams):
        beam()
    s = (time.perf_counter() - t) / beams
    return {"s_per_beam": s, "first_beam_s": first, "plan_build_s": prep,
            "note": "hd_realfft + hd_zapbirds (the 221 PALFA.zaplist birdies) + hd_rednoise over the 57 passes' series in HBM "
                    "(spectra stay on the device); wall time with the plans' FFT state built (plan_build_s: the six "
                    "hipFFT plans built ahead by hd_fft_prepare; first_beam_s: the first beam after that)"}


def rfifind_leg(eng, obs, beams):
    """rfifind -time 2^15*64us (PALFA2_presto_search.py:482-490) on the beam in HBM: the device
    statistics (clip_times, per-interval channel mean/std, max normalised FFT power) and the
    host mask decisions; wall seconds per beam.  Clears the engine's mask (run last)."""
    from hipdedisp import rfifind as RF
    from hipdedisp.synth import rfifind_ptsperint
    eng.set_mask()
    pts = rfifind_ptsperint(obs.dt)
    RF.device_stats(eng, pts)                     # the clip state for the unmasked block
    eng.sync()
    t = time.perf_counter()
    for _ in range(beams):
        avg, std, pw = RF.device_stats(eng, pts)
        RF.make_mask(avg, std, pw, pts)
    s = (time.perf_counter() - t) / beams
    return {"s_per_beam": s, "intervals": int(avg.shape[0]), "ptsperint": pts,
            "note": "hd_rfifind_stats + rfifind's mask decisions (host) for the beam; wall time"}


def stream_leg(eng, stages, obs, synth_beams, beams):
    """configs[4]'s overlapped PSRFITS streaming (one beam per job, queue_managers/pbs.py:67):
    two beams written as PSRFITS files (tmpfs); per timed beam the NEXT beam's file is read on
    the library's prefetch thread + copy stream (hd_prefetch_raw_file) while this beam's 57
    passes run, then hd_swap_raw.  Wall seconds per beam, and the reads' own rate."""
    import shutil
    from hipdedisp.formats import psrfits
    nbytes = obs.N * obs.rowbytes
    d = e2e_dir(2.2 * nbytes)
    if d is None:
        return None
    files = []
    try:
        for k, sy in enumerate(synth_beams):
            eng.synth_device(sy)
            fn = os.path.join(d, "beam%d.fits" % k)
            psrfits.write_psrfits(fn, eng.get_raw(), obs, beam=k)
            files.append(psrfits.SpectraInfo([fn]))
        files[0].stream_to(eng, prefetch=True)
        eng.swap_raw()
        eng.sync()
        io = 0.0
        t = time.perf_counter()
        for k in range(beams):
            files[(k + 1) % len(files)].stream_to(eng, prefetch=True)
            run_step(eng, stages)
            a, _ = eng.swap_raw()
            io += a
        eng.sync()
        s = (time.perf_counter() - t) / beams
    finally:
        shutil.rmtree(d, ignore_errors=True)
    return {"s_per_beam": s, "samples_per_s": sum(p.pp.numdms * p.nds for st in stages for p in st) / s,
            "read_GBps": nbytes / (io / beams) / 1e9 if io > 0 else None, "pread_s_per_beam": io / beams,
            "dir": os.path.dirname(d),
            "note": "configs[4] per GPU: each beam's PSRFITS read (pread -> pinned -> HBM on the prefetch thread and "
                    "copy stream) overlapped with the previous beam's 57 passes; wall time per beam"}


def e2e_dir(need_bytes):
    """tmpfs when it has room (the reference's base_tmp_dir is /dev/shm), else the temp dir."""
    import shutil
    import tempfile
    for base in ("/dev/shm", tempfile.gettempdir()):
        try:
            if os.path.isdir(base) and shutil.disk_usage(base).free > need_bytes:
                return tempfile.mkdtemp(prefix="hd_e2e_", dir=base)
        except OSError:
            pass
    return None


def end_to_end(eng, stages, obs, outdir):
    """One beam as the reference's search loop produces it (PALFA2_presto_search.py:494-537):
    per DDplan stage, stage 1 of its passes, then per pass stage 2 and the pass's
    <base>_DM<dm>.dat/.inf files in outdir (device series -> pinned buffers -> writer
    threads, hd_write_series; .inf text from Python), the clock running until every file
    of the stage is complete.  The files of each stage are then deleted with the clock
    stopped (the reference removes each .dat after its per-DM tools, :598-606)."""
    from hipdedisp.formats.inf import InfoData
    from hipdedisp.formats.series import write_dats_device
    info = InfoData(name="", telescope="Arecibo", instrument="Mock", object="synthetic", ra="00:00:00.0000",
                    dec="00:00:00.0000", observer="hipdedisp bench", mjd=56000.0, bary=0, dt=obs.dt,
                    freq=obs.lofreq, freqband=obs.nchan * obs.df, num_chan=obs.nchan, chan_wid=obs.df)
    base = os.path.join(outdir, "beam")
    w0, b0 = eng.wait_writes()
    elapsed = 0.0
    eng.sync()
    t = time.perf_counter()
    eng.touch_raw()
    for grp in subband_groups(stages):
        eng.run_subband_multi([p for st in grp for p in st])
        for plans in grp:
            run_dedisp_stage(eng, plans)
            for p in plans:
                info.dt, info.freq, info.chan_wid, info.num_chan = p.sub_dt, p.sub_lofreq, p.sub_chanwid, p.pp.nsub
                info.freqband = p.pp.nsub * p.sub_chanwid
                write_dats_device(p, base, p.dmstrs, info, p.nds, wait=False)
            eng.wait_writes()
            elapsed += time.perf_counter() - t
            for f in os.listdir(outdir):
                os.remove(os.path.join(outdir, f))
            t = time.perf_counter()
    w1, b1 = eng.wait_writes()
    return elapsed, b1 - b0, w1 - w0


def shard_stages(eng, obs, ddplans, rank, world, variant):
    """This rank's LPT share of the beam's passes (hipdedisp.sharding), grouped by stage."""
    from hipdedisp import sharding as S
    sb = S.ShardedBeam(ddplans, obs, rank, world)
    stages = [[] for _ in ddplans]
    for stage, passnums in sb.my_groups():
        for i in passnums:
            p = eng.plan(sb.pass_params(stage, i))
            if variant:
                p.set_variant(variant)
            stages[stage].append(p)
    return stages


def slice_stages(eng, ts, rank, variant):
    """This rank's time slice of the beam: every pass, -numout local (the last rank pads)."""
    from hipdedisp import PassParams, plan as P
    stages = []
    for d in ts.ddplans:
        plans = []
        stages.append(plans)
        for i in range(d.numpasses):
            pp = PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                            numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp,
                            numout=ts.numout_local(rank, P.choose_N(ts.obs.N / d.downsamp), d.sub_downsamp))
            p = eng.plan(pp)
            if variant:
                p.set_variant(variant)
            plans.append(p)
    return stages


SLICE_COMM = ["torch"]
# --sim-slice R/G with R > 0: the other slices' clip statistics rows (what the all-reduce would
# bring), computed once from a whole-beam context before the timed steps
SLICE_SIM_TABLE = [None]


def run_slice_step(eng, ts, rank, stages, dist, torch):
    """One beam as time slices: clip statistics of the owned read blocks -> all-reduce ->
    clip_times finished on each slice; every pass; padding sums -> all-reduce -> last rank pads."""
    import numpy as np
    eng.touch_raw()
    on_gpu = dist is not None and dist.get_backend() == "nccl"
    hdc = SLICE_COMM[0] == "hd"
    if eng.opts.clip_sigma > 0:
        if hdc:
            eng.slice_exchange_clip(ts.nown_blocks(rank), ts.nblk_total)
        elif on_gpu:
            table = torch.zeros((ts.nblk_total, ts.obs.nchan + 3), dtype=torch.float64, device="cuda")
            ts.contribute_clip_stats(eng, rank, table.data_ptr())
            dist.all_reduce(table)
            torch.cuda.current_stream().synchronize()
            eng.clip_set_stats(table.data_ptr())
        else:
            table = ts.stats_table() if SLICE_SIM_TABLE[0] is None else SLICE_SIM_TABLE[0].copy()
            ts.contribute_clip_stats(eng, rank, table)
            if dist is not None:
                t = torch.from_numpy(table)
                dist.all_reduce(t)
            eng.clip_set_stats(table)
    plans = []
    for grp in subband_groups(stages):
        eng.run_subband_multi([p for st in grp for p in st])
        for st in grp:
            run_dedisp_stage(eng, st)
            plans += st
    sums = ts.pass_sums(rank, plans)
    if hdc:
        eng.comm_allreduce(sums)
    elif dist is not None:
        t = torch.from_numpy(sums)
        if on_gpu:
            t = t.cuda()
        dist.all_reduce(t)
        sums = t.cpu().numpy().astype(np.float64)
    ts.pad_passes(rank, plans, sums)
    eng.sync()


def slice_checksums(ts, rank, stages):
    """Per pass of this rank's slice: the exact double sum of every DM's owned output samples
    (hd_series_sum; the series are integer-valued, so the sums over ranks add exactly) and,
    on the last rank, the padding value of the padded tail (NaN elsewhere)."""
    import numpy as np
    out = []
    for st in stages:
        for p in st:
            nj = ts.out_range(rank, p.pp.ds)[1]
            sums = np.array([p.series_sum(d, 0, nj) for d in range(p.pp.numdms)], np.float64)
            padv = float(p.get_series(0, 1, nj, 1)[0, 0]) if p.numout > nj else float("nan")
            out.append((sums, padv))
    return out


def union_check(eng_factory, obs, synth, ddplans, mask, pts, pad, gathered):
    """Rank 0: the union of the ranks' slice checksums against one whole-beam context."""
    import numpy as np
    from hipdedisp import Opts
    eng = eng_factory()
    try:
        eng.set_obs(obs, Opts())
        eng.synth_device(synth)
        eng.set_mask(mask, pts, pad)
        stages = build_plans(eng, obs, ddplans, 0)
        run_step(eng, stages)
        k, bad, ndm = 0, [], 0
        for st in stages:
            for p in st:
                want = np.array([p.series_sum(d, 0, p.nds) for d in range(p.pp.numdms)], np.float64)
                got = sum(g[k][0] for g in gathered)
                ndm += p.pp.numdms
                if not np.array_equal(got, want):
                    bad.append((k, "sums", int(np.sum(got != want))))
                if p.numout > p.nds:
                    wpad = float(p.get_series(0, 1, p.nds, 1)[0, 0])
                    gpad = gathered[-1][k][1]
                    if wpad != gpad:
                        bad.append((k, "pad", wpad, gpad))
                k += 1
                p.destroy()
    finally:
        eng.close()
    return {"passes": k, "dm_trials": ndm, "ranks": len(gathered), "equal": not bad, "mismatches": bad[:8],
            "note": "per DM: sum over ranks of hd_series_sum of the owned samples == the whole-beam run's sum over "
                    "[0, N/ds), exact; last rank's padding value == the whole-beam padding value, exact"}


def broadcast_beam(eng, obs, rank, dist, torch):
    """Rank 0's raw block to every rank over RCCL (xGMI), then into each engine."""
    from hipdedisp import sharding as S
    t = torch.empty(obs.N * obs.rowbytes, dtype=torch.uint8, device="cuda")
    if rank == 0:
        eng.get_raw_device(t.data_ptr())
    torch.cuda.synchronize()
    S.broadcast_raw(t, src=0)
    torch.cuda.synchronize()
    if rank != 0:
        eng.push_raw_device(t.data_ptr())
    del t


def cpu_baseline(obs, synth, ddplans, target_s, mask, pts, pad, omp):
    """Oracle (restatement of prepsubband's two stages, clip_times and mask included) on the
    host cores, on a bounded sample: per DDplan stage, pass 0 over the first W output
    samples -- read-block cleaning (check_mask + clip_times) of the raw window, stage 1,
    stage 2 -- extrapolated to the whole plan by passes x (N/ds)/W.  As in the reference,
    every pass pays its own raw read and clip (each -sub prepsubband call redoes them).
    omp=False is the reference's one core per beam (ppn=1, pbs.py:67); omp=True spreads the
    sums over the host threads (the clip recurrence stays serial).  W is sized so the
    sample costs ~target_s seconds."""
    import copy

    import oracle as OR
    from hipdedisp import Opts
    from hipdedisp.synth import host_spectra
    opts = Opts()
    threads = OR.num_threads(True) if omp else 1

    def one(d, W):
        subdm = float(d.subdmlist[0])
        off = OR.dm_offsets(obs, opts, d.numsub, d.sub_downsamp, float(d.lodm_arg(0)), d.dmstep, d.dmsperpass)
        idd = OR.chan_delays(obs, d.numsub, subdm)
        ws = W + int(off.max())
        nraw = min(obs.N, ws * d.sub_downsamp + int(idd.max()) + d.sub_downsamp)
        wobs = copy.copy(obs)
        wobs.N = nraw
        raw = host_spectra(obs, synth, 0, nraw)
        numint = -(-nraw // pts)
        t0 = time.perf_counter()
        cl = OR.prepare(wobs, opts, raw, mask=mask[:numint], ptsperint=pts, padvals=pad, omp=omp)
        sub = OR.stage1(wobs, opts, raw, d.numsub, d.sub_downsamp, subdm, t0=0, count=ws, omp=omp, clean=cl)
        OR.stage2(sub, off, 0, W, omp=omp)
        return time.perf_counter() - t0

    # per stage: probe a small window, then size the measured window to ~target_s/6 seconds
    budget = target_s / len(ddplans)
    est_full, done_out, done_t = 0.0, 0, 0.0
    for d in ddplans:
        nds = obs.N // d.sub_downsamp
        probe_w = 32768 if omp else 2048      # OpenMP: enough 8192-sample blocks to spread
        one(d, probe_w)                       # warm-up (thread pool, first touch)
        tp = one(d, probe_w)
        W = int(min(nds - 8192, max(probe_w, probe_w * budget / max(tp, 1e-3))))
        t = one(d, W)
        est_full += d.numpasses * t * nds / W
        done_out += d.dmsperpass * W
        done_t += t
    total_out = sum(d.numpasses * d.dmsperpass * (obs.N // d.sub_downsamp) for d in ddplans)
    return {"value": total_out / est_full, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": "oracle/prepsubband_oracle.c (%s): per DDplan stage, pass 0 over its first W output samples "
                      "(clip_times + mask + stage 1 + stage 2; %d DM-samples, %.1f s), extrapolated by passes x "
                      "(N/ds)/W to the full 57-pass beam (est. %.0f s per beam)"
                      % ("OpenMP, %d threads" % threads if omp else "1 thread, the reference's ppn=1",
                         done_out, done_t, est_full),
            "est_full_beam_s": est_full}


def pointing_main(args, world, rank, local, dist, torch):
    """configs[4]: the beams of one ALFA pointing over the node's ranks (sharding.Pointing):
    each rank runs its (beam, time slice) units -- one context each -- through all 57 passes;
    the exchanges are one-way point-to-point messages.  value = output samples of every
    beam / max-over-ranks wall time per pointing."""
    import numpy as np
    from hipdedisp import Engine, Opts, plan as P
    from hipdedisp import sharding as S
    from hipdedisp.synth import palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask
    obs = palfa_obs(N=args.nspec, nbits=args.nbits)
    ddplans = P.ddplans_for("pdev")
    pt = S.Pointing(obs, ddplans, args.beams, world, frac=args.helper_frac)
    ts = pt.ts
    pts = rfifind_ptsperint(obs.dt)
    work, out_per_step = [], 0
    for b, sl in pt.units(rank):
        synth = palfa_synth(beam=b, nbits=args.nbits)
        eng = Engine(local)
        eng.set_obs(ts.local_obs(sl), Opts())
        eng.set_slice(ts.slice(sl)[0], obs.N)
        eng.set_streams(args.streams)
        eng.synth_device(synth)
        mask, pad = synth_mask(obs, synth, pts)
        eng.set_mask(mask, pts, pad)
        plans = [p for st in slice_stages(eng, ts, sl, args.variant) for p in st]
        out_per_step += sum(p.pp.numdms * ts.out_range(sl, p.pp.ds)[1] for p in plans)
        work.append((b, sl, eng, plans))
    on_gpu = dist is not None and dist.get_backend() == "nccl"
    for _ in range(args.warmup):
        S.pointing_step(pt, rank, work, dist, torch, on_gpu)
    barrier(dist, torch)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        S.pointing_step(pt, rank, work, dist, torch, on_gpu)
    barrier(dist, torch)
    dt = time.perf_counter() - t0
    dt_max = max_over_ranks(dt, dist, torch)
    total_out = out_per_step
    if dist is not None:
        tt = torch.tensor([float(out_per_step)], dtype=torch.float64, device="cuda" if on_gpu else "cpu")
        dist.all_reduce(tt)
        total_out = tt.item()
    ms1 = sum(p.last_ms()[0] for _, _, _, pl in work for p in pl)
    ms2 = sum(p.last_ms()[1] for _, _, _, pl in work for p in pl)
    line = {
        "metric": METRIC, "value": total_out * args.steps / dt_max, "unit": "samples/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt_max / args.steps * 1e3,
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "u8->f32 subbanding, i16 subbands, i16x2/i32 exact sums, f32 out", "data": "synthetic",
        "config": {"workload": "C5: an ALFA pointing of %d PALFA Mock beams (960 ch x 2^%d x %d-bit), 57-pass "
                               "DDplan each, rfifind-style masks" % (args.beams, int(np.log2(obs.N)), args.nbits),
                   "parallelism": "beam x time: %d home ranks take the first %.4f of their beam, %d helper rank(s) "
                                  "the tails of every beam; one-way clip-row and first-DM-sum messages"
                                  % (min(args.beams, world), pt.frac, pt.nhelpers),
                   "cuts": ts.cuts, "halo": ts.halo},
        "this_rank": {"rank": rank, "units": pt.units(rank), "kernel_ms_per_step": {"stage1": ms1, "stage2": ms2}},
        "predicted_ms_per_pointing": pt.predicted_ms(),
        "prediction_note": "sharding.Pointing.predicted_ms: slice cost t(x) = %.1f + %.1f x ms fitted to one-rank "
                           "slice timings (a prediction, not a measurement)"
                           % (S.POINTING_FIXED_MS, S.POINTING_BEAM_MS),
    }
    if args.check_union:
        mine_ck = {(b, sl): slice_checksums(ts, sl, [pl]) for b, sl, _, pl in work}
        gathered = [None] * world
        if dist is not None:
            dist.all_gather_object(gathered, mine_ck)
        else:
            gathered = [mine_ck]
        if rank == 0:
            allck = {}
            for g in gathered:
                allck.update(g)
            res = []
            for b in range(args.beams):
                synth = palfa_synth(beam=b, nbits=args.nbits)
                mask, pad = synth_mask(obs, synth, pts)
                per_slice = [allck[(b, k)] for k in range(pt.nslices())]
                res.append(union_check(lambda: Engine(local), obs, synth, ddplans, mask, pts, pad, per_slice))
            line["union_check"] = {"beams": len(res), "equal": all(r["equal"] for r in res),
                                   "dm_trials": sum(r["dm_trials"] for r in res),
                                   "mismatches": [m for r in res for m in r["mismatches"]][:8],
                                   "note": res[0]["note"] if res else ""}
        barrier(dist, torch)
    if rank == 0:
        print(json.dumps(line), flush=True)
    for _, _, eng, pl in work:
        for p in pl:
            p.destroy()
        eng.close()
    if "union_check" in line and not line["union_check"]["equal"]:
        sys.exit("union check failed: %s" % line["union_check"]["mismatches"])
    if dist is not None:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.mode == "pointing":
        world, rank, local, dist, torch = dist_setup(args)
        return pointing_main(args, world, rank, local, dist, torch)
    global DD_MULTI, S1_FUSE
    DD_MULTI = not args.dd_single
    S1_FUSE = not args.s1_per_stage
    world, rank, local, dist, torch = dist_setup(args)
    for leg, n1 in (("e2e_beams", 1), ("sp_beams", 1), ("fft_beams", 1), ("rfi_beams", 1), ("stream_beams", 3)):
        if getattr(args, leg) < 0:
            setattr(args, leg, n1 if world == 1 else 0)
    from hipdedisp import Engine, Opts, plan as P
    from hipdedisp.synth import palfa_obs, palfa_synth, rfifind_ptsperint, synth_mask

    obs = palfa_obs(N=args.nspec, nbits=args.nbits)
    synth = palfa_synth(beam=rank, nbits=args.nbits)
    ddplans = P.ddplans_for("pdev")
    shard = args.mode == "shard"
    slices = args.mode == "slices"
    if shard or slices:
        synth = palfa_synth(beam=0, nbits=args.nbits)       # one beam for the whole node
    eng = Engine(local)
    ts = None
    srank = rank                                     # slices: this process's slice
    if slices:
        from hipdedisp.sharding import TimeSlices
        sworld = world
        if args.sim_slice:
            if world != 1:
                sys.exit("--sim-slice runs one process")
            srank, sworld = (int(x) for x in args.sim_slice.split("/"))
        ts = TimeSlices(obs, ddplans, sworld)
        if args.sim_slice and srank > 0 and Opts().clip_sigma > 0:
            # the earlier slices' clip statistics, as the all-reduce would bring them (untimed):
            # without them a later slice's clip_times runs from empty blocks
            full = Engine(local)
            full.set_obs(obs, Opts())
            full.set_slice(0, obs.N)
            full.synth_device(synth)
            fm, fpad = synth_mask(obs, synth, rfifind_ptsperint(obs.dt))
            full.set_mask(fm, rfifind_ptsperint(obs.dt), fpad)
            t1 = TimeSlices(obs, ddplans, 1)
            SLICE_SIM_TABLE[0] = t1.stats_table()
            t1.contribute_clip_stats(full, 0, SLICE_SIM_TABLE[0])
            full.close()
            del full
        eng.set_obs(ts.local_obs(srank), Opts())
        eng.set_slice(ts.slice(srank)[0], obs.N)
    else:
        eng.set_obs(obs, Opts())
    eng.set_streams(args.streams)
    if not shard or rank == 0:
        eng.synth_device(synth)
    pts = rfifind_ptsperint(obs.dt)
    mask, pad = synth_mask(obs, synth, pts)
    eng.set_mask(mask, pts, pad)
    if shard:
        stages = shard_stages(eng, obs, ddplans, rank, world, args.variant)
    elif slices:
        stages = slice_stages(eng, ts, srank, args.variant)
    else:
        stages = build_plans(eng, obs, ddplans, args.variant)
    plans = [p for st in stages for p in st]
    if slices:                                                      # this rank's owned samples
        out_per_step = sum(p.pp.numdms * ts.out_range(srank, p.pp.ds)[1] for p in plans)
    else:
        out_per_step = sum(p.pp.numdms * p.nds for p in plans)
    if shard and world > 1:
        broadcast_beam(eng, obs, rank, dist, torch)                 # untimed: makes warmup valid
    if slices and args.comm == "hd" and not args.sim_slice:
        # the library's communicator: rank 0's id reaches the others over the process group
        uid = Engine.comm_unique_id() if rank == 0 else bytes(128)
        if dist is not None:
            t = torch.tensor(list(uid), dtype=torch.uint8, device="cuda" if dist.get_backend() == "nccl" else "cpu")
            dist.broadcast(t, 0)
            uid = bytes(t.cpu().tolist())
        eng.comm_init(uid, rank, world)
        SLICE_COMM[0] = "hd"

    bcast_s = 0.0

    def step():
        if slices:
            run_slice_step(eng, ts, srank, stages, dist, torch)
        else:
            run_step(eng, stages)

    for _ in range(args.warmup):
        step()
    barrier(dist, torch)
    eng.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if shard and world > 1:      # the exchange is part of every sharded beam
            tb = time.perf_counter()
            broadcast_beam(eng, obs, rank, dist, torch)
            bcast_s += time.perf_counter() - tb
        step()
    eng.sync()
    barrier(dist, torch)
    dt = time.perf_counter() - t0
    dt_max = max_over_ranks(dt, dist, torch)
    total_out = out_per_step
    if dist is not None:
        tt = torch.tensor([float(out_per_step)], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt)
        total_out = tt.item()

    # per-kernel device time of the last step (hipEvents on the engine's stream); stage 2 is
    # grouped by the kernel each plan launched (hd_plan_kernel, the names rocprofv3 prints)
    ms1 = ms2 = 0.0
    per_kernel = {}
    for p in plans:
        a, b = p.last_ms()
        ms1 += a
        ms2 += b
        k = per_kernel.setdefault(p.kernel(), {"ms": 0.0, "launches": 0, "units": 0})
        k["ms"] += b
        k["launches"] += 1 if p.launch_passes() > 0 else 0      # passes sharing a launch count once
        k["units"] += p.pp.numdms * (ts.out_range(srank, p.pp.ds)[1] if slices else p.nds)
    raw_bytes = (ts.slice(srank)[1] if slices else obs.N) * obs.rowbytes
    adds2 = sum(p.pp.numdms * p.nds * p.pp.nsub for p in plans)
    # algorithmic bytes per output sample (SURVEY §8d compulsory model): raw once + 4 B out
    b_unit = (raw_bytes + 4.0 * out_per_step) / out_per_step
    dom = max(per_kernel, key=lambda k: per_kernel[k]["ms"])
    kd = per_kernel[dom]
    achieved = kd["units"] * b_unit / (kd["ms"] * 1e-3) / 1e9
    launch_ms = kd["ms"] / kd["launches"]
    alg_per_launch = kd["units"] * b_unit / kd["launches"]
    # HBM traffic of exactly this kernel from the committed PMC summary (scripts/pmc_summary.py;
    # keyed by kernel name -- a figure for any other kernel is refused)
    traffic, traffic_src = None, None
    for pmc in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_r*.json")), reverse=True):
        try:
            j = json.load(open(pmc))
        except Exception:
            continue
        e = j.get("kernels", {}).get(dom)
        if e and e.get("hbm_bytes"):
            traffic = e["hbm_bytes"]
            traffic_src = "%s (commit %s)" % (os.path.relpath(pmc, ROOT), j.get("commit", "?"))
            break
    step_s = dt_max / args.steps
    line = {
        "metric": METRIC,
        "value": total_out * args.steps / dt_max,
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": step_s * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if (shard or slices) else "weak",
        "vs_baseline": None,
        "dtype": "u8->f32 subbanding, i16 subbands, i16x2/i32 exact sums, f32 out",
        "data": "synthetic",
        "config": {"workload": "C2: full PALFA Mock beam per GPU (960 ch x 2^22 x %d-bit, 65.476 us), "
                               "57-pass DDplan = 4188 DM trials, rfifind-style mask" % args.nbits,
                   "nchan": obs.nchan, "nspec": obs.N, "nbits": obs.nbits, "dm_trials": 4188, "passes": len(plans),
                   "out_samples_per_beam": sum(d.numpasses * d.dmsperpass * (obs.N // d.sub_downsamp) for d in ddplans),
                   "parallelism": ("1 beam, passes LPT-sharded x%d, RCCL raw broadcast" % world) if shard
                   else ("1 beam, time slices x%d (halo %d spectra), RCCL clip-stats + padding all-reduce"
                         % (world, ts.halo)) if slices and not args.sim_slice
                   else ("ONE rank's time slice (%s, halo %d spectra) alone, no collectives: per-rank compute time, "
                         "a prediction input, not a scaling measurement" % (args.sim_slice, ts.halo)) if slices
                   else "beam-per-GPU x%d" % world},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src, "algorithmic_bytes_per_launch": alg_per_launch,
                     "launches_per_step": kd["launches"], "avg_launch_ms": launch_ms, "bytes_per_unit": b_unit},
        "kernel_ms_per_step": {"stage1": ms1, "stage2": ms2},
        "stage2_kernels": {k: {"ms": v["ms"], "launches": v["launches"],
                               "GBps_alg": v["units"] * b_unit / (v["ms"] * 1e-3) / 1e9 if v["ms"] > 0 else None}
                           for k, v in sorted(per_kernel.items(), key=lambda kv: -kv[1]["ms"])},
        "stage2_streams": args.streams,
        "stage2_launch": "one per pass" if args.dd_single else "one per DDplan stage (hd_run_dedisp_multi)",
        "slice_exchanges": (("library RCCL communicator (hd_comm_*)" if SLICE_COMM[0] == "hd" else "torch.distributed")
                            if slices else None),
        "stage1_launch": "one per DDplan stage" if args.s1_per_stage else
                         "ds=1 stage alone, the ds>=2 stages in one hd_run_subband_multi call (k_stage1_q8m)",
        "step_compulsory_hbm_frac": (raw_bytes + 4.0 * out_per_step) / step_s / (HBM_PEAK_GBS * 1e9),
        "stage2_valu_frac": adds2 / (ms2 * 1e-3) / VALU_ADD_PEAK if ms2 > 0 else None,
    }
    if shard:
        line["broadcast_ms_per_step"] = 1e3 * bcast_s / args.steps
    if not (shard or slices) and args.e2e_beams > 0:
        out_bytes = 4 * sum(p.pp.numdms * p.numout for p in plans)
        outdir = e2e_dir(1.1 * max(4 * p.pp.numdms * p.numout for p in plans) * 30)
        if outdir:
            tot = nb = wsec = 0.0
            for _ in range(args.e2e_beams):
                el, b, w = end_to_end(eng, stages, obs, outdir)
                tot, nb, wsec = tot + el, nb + b, wsec + w
            os.rmdir(outdir)
            beams = args.e2e_beams
            line["end_to_end"] = {
                "samples_per_s": out_per_step * beams / tot, "s_per_beam": tot / beams,
                "dat_bytes_per_beam": out_bytes, "write_GBps": nb / tot / 1e9,
                "writer_busy_s_per_beam": wsec / beams, "dir": os.path.dirname(outdir),
                "note": "stage 1 + stage 2 + every .dat/.inf file of the 57 passes complete in the directory; "
                        "per-rank (this rank's beam)"}
            line["end_to_end_samples_per_s"] = line["end_to_end"]["samples_per_s"]
    if not (shard or slices) and args.sp_beams > 0:
        line["single_pulse"] = single_pulse_leg(eng, stages, args.sp_beams)
    if not (shard or slices) and args.fft_beams > 0:
        line["fft_stage"] = fft_leg(eng, stages, args.fft_beams)
    if not (shard or slices) and args.rfi_beams > 0:
        line["rfifind"] = rfifind_leg(eng, obs, args.rfi_beams)
    if not (shard or slices) and args.stream_beams > 0:
        st = stream_leg(eng, stages, obs, [synth, palfa_synth(beam=rank + 8, nbits=args.nbits)], args.stream_beams)
        if st:
            line["stream_beams"] = st
    if slices and args.check_union:
        mine = slice_checksums(ts, srank, stages)
        gathered = [None] * world
        if dist is not None:
            dist.all_gather_object(gathered, mine)
        else:
            gathered = [mine]
        if rank == 0:
            for p in plans:
                p.destroy()
            plans = []
            eng.close()
            line["union_check"] = union_check(lambda: Engine(local), obs, synth, ddplans, mask, pts, pad, gathered)
        barrier(dist, torch)
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(obs, synth, ddplans, args.cpu_seconds, mask, pts, pad, omp=False)
        line["cpu_baseline_openmp"] = cpu_baseline(obs, synth, ddplans, args.cpu_seconds, mask, pts, pad, omp=True)
    if rank == 0:
        print(json.dumps(line), flush=True)
    for p in plans:
        p.destroy()
    eng.close()
    if "union_check" in line and not line["union_check"]["equal"]:
        sys.exit("union check failed: %s" % line["union_check"]["mismatches"])
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
