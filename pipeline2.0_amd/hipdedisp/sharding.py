"""Multi-GPU partitioning of a beam's DDplan (north_star (d)).

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
