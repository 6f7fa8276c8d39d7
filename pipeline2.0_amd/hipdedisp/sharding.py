"""Multi-GPU partitioning of a beam's DDplan (north_star (d)).

Two ways to spread ONE beam over the G GPUs of a node, plus the trivial beam-per-GPU mode:

* **time slices** (`TimeSlices`, the default for one beam): rank r dedisperses spectra
  [t0_r, t0_r + own_r) through ALL 57 passes; it holds those spectra plus a halo of the next
  rank's first spectra (the longest delay of any pass), so its output samples are exact and
  each output sample is computed once.  No raw-block exchange: each rank ingests only its
  own rows.  The one true exchange is PRESTO's clip_times, whose running statistics carry
  across read blocks: every rank contributes the per-block statistics of its own blocks
  (an all-reduce of a [nblk][nchan + 3] double table, ~16 MB for a PALFA beam) and runs the
  serial recurrence up to its end.  The padding value of each pass (the first DM's mean) is
  the observation's: one all-reduce of a [passes] vector of series sums at the end.

The reference runs one beam per batch job on one core (`nodes=X:ppn=1`,
lib/python/queue_managers/pbs.py:67) and its passes strictly in sequence
(lib/python/PALFA2_presto_search.py:494-529).  The passes are independent: each has its own
subband DM, subbands and DM trials, and no reduction joins them.  On one node of G GPUs:

* **beam x pass sharding** (config 3): the passes of one beam are spread over the G ranks by
  LPT on their work; the raw block (4 GB for a 2^22 x 960 x 8-bit beam) is the only thing the
  ranks share, and it travels once, as an RCCL broadcast over xGMI
  (`torch.distributed` backend "nccl" is RCCL on ROCm), in chunks so it can stream.  Each
  rank forms the subbands of its own passes (one raw read per DDplan stage it holds) and
  writes its own `.dat`/`.inf` files.
* **beam per rank** (config 5, the 7-beam ALFA pointing): no exchange at all.

Process model: one process per GPU, launched by `torch.distributed.run`; ranks read RANK /
LOCAL_RANK / WORLD_SIZE.  No data-path collective other than the raw broadcast.
"""
from dataclasses import dataclass
from typing import List, Sequence, Tuple

import numpy as np

from . import plan as P


@dataclass(frozen=True)
class PassRef:
    """One prepsubband pass of the plan: DDplan stage index and pass index within it."""
    stage: int
    passnum: int
    work: float          # relative cost (see pass_work)


def pass_work(ddplan, N, nchan):
    """Relative device work of one pass: the stage-2 sweep (numdms x N/ds x nsub adds) plus the
    stage-1 subband formation (N x nchan channel samples; integer adds are ~4x cheaper per
    sample than the packed stage-2 adds, and the raw read is shared within a DDplan stage)."""
    nds = N / ddplan.sub_downsamp
    return ddplan.dmsperpass * nds * ddplan.numsub + 0.25 * N * nchan


def pass_list(ddplans, N, nchan) -> List[PassRef]:
    return [PassRef(si, i, pass_work(d, N, nchan)) for si, d in enumerate(ddplans) for i in range(d.numpasses)]


def lpt_assign(items: Sequence[PassRef], nranks: int) -> List[List[PassRef]]:
    """Longest-processing-time-first: each pass, heaviest first, to the least-loaded rank
    (ties to the lower rank, so the assignment is deterministic on every rank)."""
    if nranks < 1:
        raise ValueError("nranks must be >= 1")
    load = [0.0] * nranks
    out: List[List[PassRef]] = [[] for _ in range(nranks)]
    for it in sorted(items, key=lambda x: (-x.work, x.stage, x.passnum)):
        r = min(range(nranks), key=lambda k: (load[k], k))
        out[r].append(it)
        load[r] += it.work
    for lst in out:
        lst.sort(key=lambda x: (x.stage, x.passnum))
    return out


def assign_passes(ddplans, N, nchan, nranks) -> List[List[PassRef]]:
    return lpt_assign(pass_list(ddplans, N, nchan), nranks)


def imbalance(assignment: List[List[PassRef]]) -> float:
    """max rank load / mean rank load (1.0 = perfect)."""
    loads = [sum(p.work for p in lst) for lst in assignment]
    mean = sum(loads) / max(len(loads), 1)
    return max(loads) / mean if mean > 0 else 1.0


def by_stage(passes: Sequence[PassRef]) -> List[Tuple[int, List[int]]]:
    """[(stage, [passnum, ...])] in plan order: the groups a rank forms with one stage-1 launch."""
    groups = {}
    for p in passes:
        groups.setdefault(p.stage, []).append(p.passnum)
    return [(s, groups[s]) for s in sorted(groups)]


def broadcast_raw(tensor, src=0, group=None, chunk_bytes=256 << 20):
    """Broadcast a flat uint8 tensor (the raw block) from `src` in chunks of `chunk_bytes`
    (RCCL on GPU tensors, gloo on CPU tensors).  Chunking bounds the staging each collective
    needs.  Returns when the data is in `tensor` on this rank (GPU: stream synchronised)."""
    import torch.distributed as dist
    flat = tensor.view(-1)
    n = flat.numel()
    for off in range(0, n, chunk_bytes):
        dist.broadcast(flat[off:off + chunk_bytes], src=src, group=group)
    # RCCL queues the broadcast on torch's current stream; hd_push_raw_device copies on the
    # engine's own stream, which has no ordering with it: return only once the data landed
    if flat.is_cuda:
        import torch
        torch.cuda.current_stream(flat.device).synchronize()


class ShardedBeam:
    """Run one beam's DDplan sharded over the ranks of the default process group.

        sb = ShardedBeam(ddplans, obs, rank, world)
        for stage, passnums in sb.my_groups():      # this rank's passes, by DDplan stage
            ...
    `run(engine, per_pass)` executes them on a hipdedisp Engine: one multi-pass stage-1 launch
    per group, then the stage-2 sweep of each pass, calling per_pass(stage, passnum, plan).
    """

    def __init__(self, ddplans, obs, rank, world):
        self.ddplans = list(ddplans)
        self.obs = obs
        self.rank = rank
        self.world = world
        self.assignment = assign_passes(self.ddplans, obs.N, obs.nchan, world)

    def my_passes(self) -> List[PassRef]:
        return self.assignment[self.rank]

    def my_groups(self):
        return by_stage(self.my_passes())

    def pass_params(self, stage, passnum):
        from .engine import PassParams
        d = self.ddplans[stage]
        return PassParams(subdm=float(d.subdmlist[passnum]), lodm=float(d.lodm_arg(passnum)),
                          dmstep=float(d.dmstep_arg()), numdms=d.dmsperpass, nsub=d.numsub,
                          ds=d.sub_downsamp, numout=P.choose_N(self.obs.N / d.downsamp))

    def make_plans(self, engine):
        """{stage: [(passnum, Plan), ...]} for this rank."""
        return {stage: [(i, engine.plan(self.pass_params(stage, i))) for i in passnums]
                for stage, passnums in self.my_groups()}

    def run(self, engine, plans, per_pass=None, to_host=False):
        out = {}
        for stage, lst in plans.items():
            engine.run_subband_multi([p for _, p in lst])
            for i, p in lst:
                series = p.run_dedisp(to_host=to_host)
                if per_pass is not None:
                    per_pass(stage, i, p, series)
                out[(stage, i)] = series
        return out

    def out_samples(self):
        return sum(self.ddplans[p.stage].dmsperpass * (self.obs.N // self.ddplans[p.stage].sub_downsamp)
                   for p in self.my_passes())


def dm_strings_of(ddplans, assignment: List[List[PassRef]]):
    """Per rank, the `%.2f` DM strings whose .dat files it writes (the union over ranks is the
    reference's full list, lib/python/PALFA2_presto_search.py:531-537, each exactly once)."""
    return [[dm for p in lst for dm in ddplans[p.stage].dmlist[p.passnum]] for lst in assignment]


def sample_counts(ddplans, N):
    return np.array([d.dmsperpass * (N // d.sub_downsamp) for d in ddplans for _ in range(d.numpasses)])


# ---------------------------------------------------------------------------------------
# time slices
# ---------------------------------------------------------------------------------------

def _lcm(a, b):
    from math import gcd
    return a * b // gcd(a, b)


class TimeSlices:
    """One beam's spectra cut into `world` contiguous slices (one per rank) for the DDplan
    `ddplans`.  Slice boundaries are multiples of lcm(nsblk, every downsampling factor), so
    every read block and every downsampled output sample belongs to exactly one rank.

        ts = TimeSlices(obs, ddplans, world)
        t0, own, n_local = ts.slice(rank)      # spectra [t0, t0 + n_local) held, own computed
        j0, nj = ts.out_range(rank, ds)        # output samples [j0, j0 + nj) this rank owns
    """

    def __init__(self, obs, ddplans, world, opts=None, fractions=None):
        """fractions: optional relative slice lengths (one per rank; default equal slices)."""
        from .engine import Opts, PassParams, plan_tables
        if world < 1:
            raise ValueError("world must be >= 1")
        if fractions is not None and (len(fractions) != world or min(fractions) < 0 or sum(fractions) <= 0):
            raise ValueError("fractions: one non-negative length per slice")
        self.obs, self.ddplans, self.world = obs, list(ddplans), world
        self.opts = opts or Opts()
        if world > 1 and self.opts.pad_mode == 0:        # HD_PAD_MEAN: one value per DM
            raise ValueError("time slices support pad_mode HD_PAD_DM0 / HD_PAD_ZERO")
        blk = obs.nsblk if 0 < obs.nsblk < obs.N else obs.N
        unit = blk
        reach = 0
        for d in self.ddplans:
            unit = _lcm(unit, d.sub_downsamp)
            for i in range(d.numpasses):
                pp = PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)),
                                dmstep=float(d.dmstep_arg()), numdms=d.dmsperpass, nsub=d.numsub,
                                ds=d.sub_downsamp)
                idd, off, _ = plan_tables(obs, self.opts, pp)
                # last raw row output j uses: (j + max offset) * ds + ds - 1 + max channel delay
                reach = max(reach, int(off.max()) * d.sub_downsamp + int(idd.max()) + d.sub_downsamp)
        self.blk, self.unit = blk, unit
        self.halo = -(-reach // blk) * blk
        N = obs.N
        if fractions is None:
            cuts = [0] + [min(N, round(k * N / world / unit) * unit) for k in range(1, world)] + [N]
        else:
            cum = np.cumsum(np.asarray(fractions, np.float64)) / float(np.sum(fractions))
            cuts = [0] + [min(N, int(round(c * N / unit)) * unit) for c in cum[:-1]] + [N]
        for k in range(1, len(cuts)):
            cuts[k] = max(cuts[k], cuts[k - 1])
        self.cuts = cuts
        self.nblk_total = -(-N // blk)

    def slice(self, rank):
        """(t0, own, n_local): first spectrum, spectra owned, spectra held (own + halo)."""
        t0, t1 = self.cuts[rank], self.cuts[rank + 1]
        n_local = min(self.obs.N, t1 + self.halo) - t0
        return t0, t1 - t0, n_local

    def local_obs(self, rank):
        import copy
        o = copy.copy(self.obs)
        o.N = self.slice(rank)[2]
        return o

    def nown_blocks(self, rank):
        t0, own, _ = self.slice(rank)
        return -(-own // self.blk) if rank == self.world - 1 else own // self.blk

    def out_range(self, rank, ds):
        """(first global output sample, count) this rank owns at downsampling ds."""
        t0, own, _ = self.slice(rank)
        nds = self.obs.N // ds
        j0 = t0 // ds
        nj = nds - j0 if rank == self.world - 1 else own // ds
        return j0, max(nj, 0)

    def numout_local(self, rank, numout_global, ds):
        """-numout of a rank's local pass: the last rank pads to the global length."""
        if rank == self.world - 1:
            return max(numout_global - self.slice(rank)[0] // ds, 0)
        return 0

    def stats_table(self):
        """A zeroed [nblk_total][nchan + 3] float64 table for the clip statistics."""
        return np.zeros((self.nblk_total, self.obs.nchan + 3), np.float64)

    # -- the two exchanges of a sliced beam (callers all-reduce between the phases) --
    def contribute_clip_stats(self, engine, rank, table):
        """Phase A: this rank's own read blocks' clip statistics into `table` (a zeroed
        stats_table(), or the device address of one); sum the tables over the ranks, then
        engine.clip_set_stats(table) (phase B) before stage 1."""
        engine.clip_stats(self.nown_blocks(rank), table)

    def pass_sums(self, rank, plans):
        """Phase C: per plan, the exact sum of the first DM's owned output samples (the
        padding value of prepsubband is the observation's first-DM mean)."""
        if not plans:
            return np.zeros(0, np.float64)
        return plans[0].eng.series_sums(plans, 0, [0] * len(plans),
                                        [self.out_range(rank, p.pp.ds)[1] for p in plans])

    def pad_passes(self, rank, plans, sums):
        """Phase D (after summing pass_sums over the ranks): the last rank pads its series
        from N/ds to -numout with the observation's value (HD_PAD_DM0) or 0 (HD_PAD_ZERO)."""
        if rank != self.world - 1:
            return
        for p, s in zip(plans, sums):
            nj = self.out_range(rank, p.pp.ds)[1]
            if p.numout > nj:
                nds = self.obs.N // p.pp.ds
                v = np.float32(s / nds) if self.opts.pad_mode == 2 and nds > 0 else np.float32(0.0)
                p.series_fill(nj, float(v))


# ---------------------------------------------------------------------------------------
# configs[4]: the 7 beams of an ALFA pointing on one node (beam x time partitioning)
# ---------------------------------------------------------------------------------------

# slice cost model t(x) = a + b x (ms per slice of x of a beam), fitted to round 6's one-rank
# measurements (profiles/r06_simslice.jsonl, profiles/r06_ab_stage2_sload.txt): the whole beam
# 56.8 ms, slice 0 of 8 (x = 1/8 + the 18,432-spectrum halo) 11.2 ms, the last slice of 8 12.1 ms
# -> b = 51.7, a = 5.1 (the mean of the two slices' fixed costs); round 5: 5.7 / 51.4
POINTING_FIXED_MS, POINTING_BEAM_MS = 5.1, 51.7


def helper_fraction(nbeams, nhelpers, fixed_ms, beam_ms):
    """Home share f of each beam that balances a home rank (one slice of f N spectra) against
    a helper, for a slice cost t(x) = a + b x (a = fixed_ms, b = beam_ms).  Pointing.units gives
    EACH of the H helpers one slice of EVERY beam, (1 - f) / H of it, so a helper pays the fixed
    cost once per beam: home a + b f = helper n a + (n / H) b (1 - f) with n = nbeams, solved for
    f and clamped to [0.5, 1].  With no helpers every rank keeps whole beams."""
    if nhelpers <= 0:
        return 1.0
    n, H = float(nbeams), float(nhelpers)
    a, b = float(fixed_ms), float(beam_ms)
    f = ((n - 1.0) * a + (n / H) * b) / (b * (1.0 + n / H))
    return min(1.0, max(0.5, f))


class Pointing:
    """configs[4] (BASELINE.json): the `nbeams` beams of an ALFA pointing on a node of `world`
    ranks.  The reference runs one beam per batch job (queue_managers/pbs.py:67), which on 8
    GPUs leaves one idle for a 7-beam pointing.  Here ranks 0 .. nbeams-1 are HOME ranks:
    rank b dedisperses the first `f` of beam b's spectra through all passes (a time slice,
    TimeSlices semantics: its own rows plus the halo); the H = world - nbeams HELPER ranks
    split the tail of EVERY beam between them (slice 1 + h of beam b is helper h's).  The
    exchanges are one-way, so no home rank ever waits for a helper mid-beam:

    * clip_times (its running statistics carry across read blocks, forwards only): the home
      rank computes the statistics rows of every block it holds (own + halo) itself, so it
      needs nothing; each slice owner sends its OWN blocks' rows to the later slice owners of
      the beam, which sum them into their table before finishing clip_times;
    * padding (the observation's first-DM mean): every slice owner but the last sends its
      first-DM sums per pass to the last owner, which pads -- after all its beams.

    With world <= nbeams there are no helpers: rank r keeps beams r, r + world, ... whole.
    `units(rank)` lists (beam, slice) pairs in processing order; `slices(beam)` the beam's
    TimeSlices; `owner(beam, slice)` the rank."""

    def __init__(self, obs, ddplans, nbeams, world, frac=None, opts=None, fixed_ms=POINTING_FIXED_MS,
                 beam_ms=POINTING_BEAM_MS):
        if nbeams < 1 or world < 1:
            raise ValueError("need nbeams >= 1 and world >= 1")
        self.obs, self.ddplans, self.nbeams, self.world = obs, list(ddplans), nbeams, world
        self.nhelpers = max(0, world - nbeams)
        self.frac = float(frac) if frac is not None else helper_fraction(nbeams, self.nhelpers, fixed_ms, beam_ms)
        if self.nhelpers:
            tail = (1.0 - self.frac) / self.nhelpers
            fr = [self.frac] + [tail] * self.nhelpers
            self.ts = TimeSlices(obs, ddplans, 1 + self.nhelpers, opts=opts, fractions=fr)
        else:
            self.ts = TimeSlices(obs, ddplans, 1, opts=opts)

    def nslices(self):
        return self.ts.world

    def owner(self, beam, sl):
        if self.nhelpers == 0:
            return beam % self.world
        return beam if sl == 0 else self.nbeams + sl - 1

    def units(self, rank):
        if self.nhelpers == 0:
            return [(b, 0) for b in range(rank, self.nbeams, self.world)]
        if rank < self.nbeams:
            return [(rank, 0)]
        return [(b, rank - self.nbeams + 1) for b in range(self.nbeams)]

    def slices(self, beam):
        return self.ts                           # every beam is cut the same way

    def clip_sources(self, beam, sl):
        """Ranks whose own-block clip rows slice `sl` of `beam` must receive (earlier slices)."""
        return [self.owner(beam, k) for k in range(sl)]

    def clip_targets(self, beam, sl):
        return [self.owner(beam, k) for k in range(sl + 1, self.nslices())]

    def pad_owner(self, beam):
        return self.owner(beam, self.nslices() - 1)

    def clip_rows(self, sl):
        """(first block, blocks) of slice sl's own read blocks in the beam's stats table."""
        t0 = self.ts.slice(sl)[0]
        return t0 // self.ts.blk, self.ts.nown_blocks(sl)

    def predicted_ms(self, fixed_ms=POINTING_FIXED_MS, beam_ms=POINTING_BEAM_MS):
        """Predicted node time per pointing from the slice cost model (a prediction, not a
        measurement): the slowest rank's units."""
        fr = [(self.ts.slice(k)[1]) / float(self.obs.N) for k in range(self.nslices())]
        best = 0.0
        for r in range(self.world):
            t = sum(fixed_ms + beam_ms * fr[sl] for _, sl in self.units(r))
            best = max(best, t)
        return best


def pointing_step(pt, rank, work, dist, torch, on_gpu):
    """One pointing on this rank: `work` = [(beam, slice, engine, plans)] in pt.units(rank)
    order.  Per unit: clip statistics (earlier slices' own-block rows received, every held
    block's rows computed here), clip_times finished, every pass, first-DM sums kept.  Sends
    are non-blocking and ordered so each (source, destination) pair sees clip rows of every
    beam first, then the sums (NCCL matches point-to-point messages in order); the last slice
    of a beam pads after this rank's beams are done.  Returns the per-unit first-DM sums."""
    import numpy as np
    ts = pt.ts
    width = ts.obs.nchan + 3
    reqs, keep, sums_of = [], [], []

    def tensor(a):
        t = torch.from_numpy(np.ascontiguousarray(a))
        return t.cuda() if on_gpu else t

    for b, sl, eng, plans in work:
        eng.touch_raw()
        if eng.opts.clip_sigma > 0:
            if on_gpu:
                table = torch.zeros((ts.nblk_total, width), dtype=torch.float64, device="cuda")
                tp = table.data_ptr()
            else:
                table = torch.zeros((ts.nblk_total, width), dtype=torch.float64)
                tp = table.numpy()
            for k in range(sl):                               # earlier slices' own rows
                r0, n = pt.clip_rows(k)
                if n:
                    v = table[r0:r0 + n]
                    dist.recv(v, src=pt.owner(b, k))
            if on_gpu:
                torch.cuda.current_stream().synchronize()
            # every block this unit holds (own + halo): the recurrence is causal, so rows of the
            # halo blocks computed here equal the next slice's own
            t0, own, nloc = ts.slice(sl)
            nheld = -(-nloc // ts.blk)
            eng.clip_stats(nheld, tp)
            r0, n = pt.clip_rows(sl)
            for dst in pt.clip_targets(b, sl):
                if n:
                    v = table[r0:r0 + n].clone()
                    keep.append(v)
                    reqs.append(dist.isend(v, dst=dst))
            eng.clip_set_stats(tp)
        # bench.run_step's launches: the ds = 1 stage alone, the ds >= 2 stages' stage 1 in one
        # call, stage 2 per DDplan stage
        grp = {}
        for p in plans:
            grp.setdefault(p.pp.ds, []).append(p)
        lone = [g for d, g in grp.items() if d < 2]
        multi = [p for d, g in sorted(grp.items()) if d >= 2 for p in g]
        for g in lone:
            eng.run_subband_multi(g)
            eng.run_dedisp_multi(g)
        if multi:
            eng.run_subband_multi(multi)
            for d, g in sorted(grp.items()):
                if d >= 2:
                    eng.run_dedisp_multi(g)
        sums_of.append(ts.pass_sums(sl, plans))
    # the sums, after every beam's clip rows (message order per pair)
    for (b, sl, eng, plans), sums in zip(work, sums_of):
        dst = pt.pad_owner(b)
        if dst != rank:
            v = tensor(sums)
            keep.append(v)
            reqs.append(dist.isend(v, dst=dst))
    for (b, sl, eng, plans), sums in zip(work, sums_of):
        if sl != pt.nslices() - 1:
            continue
        total = np.array(sums, np.float64)
        for k in range(sl):
            src = pt.owner(b, k)
            if src == rank:
                continue
            v = tensor(np.zeros(len(sums), np.float64))
            dist.recv(v, src=src)
            total = total + v.cpu().numpy()
        ts.pad_passes(sl, plans, total)
    for r in reqs:
        r.wait()
    for _, _, eng, _ in work:
        eng.sync()
    return sums_of
