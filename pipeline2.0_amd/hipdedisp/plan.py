"""Dedispersion plans: the reference's hard-coded DDplan tables, its dedisp_plan class,
PRESTO's choose_N, and a restatement of the on-demand planner DDplan2b.

* dedisp_plan      reference lib/python/PALFA2_presto_search.py:374-410 (pinned by
                   tests/golden/ddplan_ref.json, produced by running the reference class)
* ddplans_for      obs_info.set_DDplan, PALFA2_presto_search.py:296-333
* choose_N         psr_utils.choose_N (PRESTO, external; called at :518, :527) [PRESTO-ext]
* DDplan2b         lib/python/DDplan2b.py:49-434 (needed for config 4, DM to ~10000)
"""
import math

import numpy as np


class dedisp_plan:
    """dedisp_plan(lodm, dmstep, dmsperpass, numpasses, numsub, downsamp)
    (PALFA2_presto_search.py:374-410).  DM lists are strings because the search
    compares them with file names; they reach prepsubband only as "%.2f" text."""

    def __init__(self, lodm, dmstep, dmsperpass, numpasses, numsub, downsamp):
        self.lodm = float(lodm)
        self.dmstep = float(dmstep)
        self.dmsperpass = int(dmsperpass)
        self.numpasses = int(numpasses)
        self.numsub = int(numsub)
        self.downsamp = int(downsamp)
        # :393-394 — subbands carry the whole downsampling, stage 2 runs at ds 1
        self.sub_downsamp = self.downsamp
        self.dd_downsamp = 1
        self.sub_dmstep = self.dmsperpass * self.dmstep
        self.dmlist = []
        self.subdmlist = []
        for ii in range(self.numpasses):
            self.subdmlist.append("%.2f" % (self.lodm + (ii + 0.5) * self.sub_dmstep))
            lodm = self.lodm + ii * self.sub_dmstep
            self.dmlist.append(["%.2f" % dm for dm in np.arange(self.dmsperpass) * self.dmstep + lodm])

    def lodm_arg(self, passnum):
        """The stage-2 "-lodm %.2f" argument (:514-516)."""
        return "%.2f" % (self.lodm + passnum * self.sub_dmstep)

    def dmstep_arg(self):
        return "%.2f" % self.dmstep


# obs_info.set_DDplan (PALFA2_presto_search.py:319-331):
#                 lodm  dmstep dms/call #calls #subbands downsamp
PLANS = {
    "pdev": [(0.0, 0.1, 76, 28, 96, 1),
             (212.8, 0.3, 64, 12, 96, 2),
             (443.2, 0.3, 76, 4, 96, 3),
             (534.4, 0.5, 76, 9, 96, 5),
             (876.4, 0.5, 76, 3, 96, 6),
             (990.4, 1.0, 76, 1, 96, 10)],
    "wapp": [(0.0, 0.3, 76, 9, 96, 1),
             (205.2, 2.0, 76, 5, 96, 5),
             (965.2, 10.0, 76, 1, 96, 25)],
}


def ddplans_for(backend):
    """obs_info.set_DDplan: the hard-coded plan for a backend (Mock = 'pdev')."""
    key = backend.lower()
    if key not in PLANS:
        raise ValueError("No dediserpsion plan for unknown backend (%s)!" % backend)
    return [dedisp_plan(*t) for t in PLANS[key]]


# psr_utils.choose_N's table of 4-digit numbers with only small prime factors [PRESTO-ext]
_GOODFACTORS = [1008, 1024, 1056, 1120, 1152, 1200, 1232, 1280, 1296, 1344, 1408, 1440, 1536,
                1568, 1584, 1600, 1680, 1728, 1760, 1792, 1920, 1936, 2000, 2016, 2048, 2112,
                2160, 2240, 2304, 2352, 2400, 2464, 2560, 2592, 2640, 2688, 2800, 2816, 2880,
                3024, 3072, 3136, 3168, 3200, 3360, 3456, 3520, 3584, 3600, 3696, 3840, 3872,
                3888, 3920, 4000, 4032, 4096, 4224, 4320, 4400, 4480, 4608, 4704, 4752, 4800,
                4928, 5040, 5120, 5184, 5280, 5376, 5488, 5600, 5632, 5760, 5808, 6000, 6048,
                6144, 6160, 6272, 6336, 6400, 6480, 6720, 6912, 7040, 7056, 7168, 7200, 7392,
                7680, 7744, 7776, 7840, 7920, 8000, 8064, 8192, 8400, 8448, 8624, 8640, 8800,
                8960, 9072, 9216, 9408, 9504, 9600, 9680, 9856, 10000]


def choose_N(orig_N):
    """psr_utils.choose_N [PRESTO-ext, restated; table and tie rules unverified]:
    the smaller of (a) the first good-factor number > the first four digits of orig_N,
    scaled by 10 until >= orig_N, and (b) the next power of two >= orig_N.
    `orig_N` may be a float: the reference passes orig_N/ds with orig_N a float64
    (psrfits.py:29,275,280), e.g. 2**22/3 = 1398101.33 -> 1408000."""
    if orig_N < 10000:
        return 0
    first4 = int(str(orig_N)[:4])
    factor = _GOODFACTORS[-1]
    for f in _GOODFACTORS:
        if f > first4:
            factor = f
            break
    new_N = factor
    while new_N < orig_N:
        new_N *= 10
    two_N = 2
    while two_N < orig_N:
        two_N *= 2
    return int(two_N) if two_N < new_N else int(new_N)


def plan_summary(ddplans, N):
    """Counts used throughout DESIGN.md/bench.py: passes, DM trials, output samples."""
    passes = sum(p.numpasses for p in ddplans)
    dms = sum(p.numpasses * p.dmsperpass for p in ddplans)
    out = sum(p.numpasses * p.dmsperpass * (N // p.downsamp) for p in ddplans)
    return {"passes": passes, "dms": dms, "out_samples": out}


# ----------------------------------------------------------------------------------
# DDplan2b (lib/python/DDplan2b.py) restated for Python 3
# ----------------------------------------------------------------------------------
ALLOW_DMSTEPS = [0.01, 0.02, 0.03, 0.05, 0.1, 0.2, 0.3, 0.5, 1.0,
                 2.0, 3.0, 5.0, 10.0, 20.0, 30.0, 50.0, 100.0, 200.0, 300.0]   # :29-30
MAX_DOWNFACTOR = 64   # :32
FF = 1.2              # :35
SMEARFACT = 2.0       # :44


def dm_smear(DM, BW, fctr):
    """psr_utils.dm_smear [PRESTO-ext]: smearing (s) of DM across BW MHz at fctr MHz.
    Its form is fixed by DDplan2b.guess_DMstep (:425-434) being its inverse."""
    return np.fabs(DM) * BW / (0.0001205 * fctr ** 3.0)


def guess_DMstep(dt, BW, fctr):
    """DDplan2b.py:425-434"""
    return dt * 0.0001205 * fctr ** 3.0 / BW


class Observation:
    """DDplan2b.py:49-96"""

    def __init__(self, dt, fctr, BW, numchan, numsamp=0):
        self.dt, self.fctr, self.BW, self.numchan = dt, fctr, BW, numchan
        self.chanwidth = BW / numchan
        self.numsamp = numsamp
        self.allow_factors = self.get_allow_downfactors()

    def gen_ddplan(self, loDM, hiDM, numsub=0, resolution=0.0):
        return DDplan(loDM, hiDM, self, numsub, resolution)

    def get_allow_downfactors(self):
        if self.numsamp:
            factors = np.arange(1, MAX_DOWNFACTOR + 1)
            return [int(f) for f in factors[(self.numsamp % factors) == 0]]
        return [int(f) for f in 2 ** np.arange(0, int(np.log2(MAX_DOWNFACTOR)) + 1)]


class DDstep:
    """DDplan2b.py:99-194"""

    def __init__(self, ddplan, downsamp, loDM, dDM, numDMs=0, numsub=0, smearfact=2.0):
        self.ddplan, self.downsamp, self.loDM, self.dDM, self.numsub = ddplan, downsamp, loDM, dDM, numsub
        obs = ddplan.obs
        self.BW_smearing = dm_smear(dDM * 0.5, obs.BW, obs.fctr)
        self.numprepsub = 0
        DMs_per_prepsub = 0
        if numsub:
            DMs_per_prepsub = 2
            while True:
                next_dsubDM = (DMs_per_prepsub + 2) * dDM
                next_ss = dm_smear(next_dsubDM * 0.5, obs.BW / numsub, obs.fctr)
                if next_ss > 0.8 * min(self.BW_smearing, obs.dt * self.downsamp):
                    self.dsubDM = DMs_per_prepsub * dDM
                    self.DMs_per_prepsub = DMs_per_prepsub
                    self.sub_smearing = dm_smear(self.dsubDM * 0.5, obs.BW / self.numsub, obs.fctr)
                    break
                DMs_per_prepsub += 2
        else:
            self.dsubDM = dDM
            self.sub_smearing = 0.0
            self.DMs_per_prepsub = 0
        cross_DM = self.DM_for_smearfact(smearfact)
        if cross_DM > ddplan.hiDM:
            cross_DM = ddplan.hiDM
        if numDMs == 0:
            self.numDMs = int(np.ceil((cross_DM - self.loDM) / self.dDM))
            if numsub:
                self.numprepsub = int(np.ceil(self.numDMs * self.dDM / self.dsubDM))
                self.numDMs = self.numprepsub * DMs_per_prepsub
        else:
            self.numDMs = numDMs
        self.hiDM = loDM + self.numDMs * dDM
        self.DMs = np.arange(self.numDMs, dtype="d") * self.dDM + self.loDM

    def DM_for_smearfact(self, smearfact):
        obs = self.ddplan.obs
        other_smear = np.sqrt(obs.dt ** 2.0 + (obs.dt * self.downsamp) ** 2.0 +
                              self.BW_smearing ** 2.0 + self.sub_smearing ** 2.0)
        return guess_DMstep(smearfact * other_smear, obs.chanwidth, obs.fctr)

    def as_dedisp_plan(self):
        """The mapping of the commented code at PALFA2_presto_search.py:315-317."""
        return dedisp_plan(self.loDM, self.dDM, self.DMs_per_prepsub, self.numprepsub,
                           self.numsub, self.downsamp)


class DDplan:
    """DDplan2b.py:197-324"""

    def __init__(self, loDM, hiDM, obs, numsub=0, resolution=0.0):
        self.loDM, self.hiDM, self.obs, self.numsub = loDM, hiDM, obs, numsub
        self.req_resolution = resolution * 0.001
        self.current_downfact = obs.allow_factors[0]
        self.current_dDM = ALLOW_DMSTEPS[0]
        self.DDsteps = []
        self.calc_min_smearing()
        while obs.dt * self.get_next_downfact() < self.resolution:
            self.current_downfact = self.get_next_downfact()
        dDM = guess_DMstep(obs.dt * self.current_downfact, 0.5 * obs.BW, obs.fctr)
        while self.get_next_dDM() < dDM:
            self.current_dDM = self.get_next_dDM()
        self.DDsteps.append(DDstep(self, self.current_downfact, self.loDM, self.current_dDM,
                                   numsub=self.numsub, smearfact=SMEARFACT))
        while self.DDsteps[-1].hiDM < self.hiDM:
            self.current_downfact = self.get_next_downfact()
            eff_dt = obs.dt * self.current_downfact
            while dm_smear(0.5 * self.get_next_dDM(), obs.BW, obs.fctr) < FF * eff_dt:
                self.current_dDM = self.get_next_dDM()
            self.DDsteps.append(DDstep(self, self.current_downfact, self.DDsteps[-1].hiDM,
                                       self.current_dDM, numsub=self.numsub, smearfact=SMEARFACT))
        wfs = [step.numDMs / float(step.downsamp) for step in self.DDsteps]
        self.work_fracts = np.asarray(wfs) / np.sum(wfs)

    def get_next_dDM(self):
        for dDM in ALLOW_DMSTEPS:
            if dDM > self.current_dDM:
                return dDM
        raise ValueError("No allowable DM steps left!")

    def get_next_downfact(self):
        index = self.obs.allow_factors.index(self.current_downfact)
        if index + 1 < len(self.obs.allow_factors):
            return self.obs.allow_factors[index + 1]
        raise ValueError("No allowable downsample factors left!")

    def calc_min_smearing(self):
        obs = self.obs
        half_dDMmin = 0.5 * ALLOW_DMSTEPS[0]
        self.min_chan_smear = dm_smear(self.loDM + half_dDMmin, obs.chanwidth, obs.fctr)
        self.min_bw_smear = dm_smear(half_dDMmin, obs.BW, obs.fctr)
        self.best_resolution = max([self.req_resolution, self.min_chan_smear, self.min_bw_smear, obs.dt])
        self.resolution = self.best_resolution
        if (FF * self.min_chan_smear > obs.dt) or (self.resolution > obs.dt):
            if self.resolution <= FF * self.min_chan_smear:
                self.resolution = FF * self.min_chan_smear

    def dedisp_plans(self):
        return [s.as_dedisp_plan() for s in self.DDsteps]


def ddplan2b_plans(dt, fctr, BW, numchan, numsamp, loDM, hiDM, numsub, resolution_ms):
    """On-demand plan (the commented path at PALFA2_presto_search.py:308-317)."""
    obs = Observation(dt, fctr, BW, numchan, numsamp)
    return obs.gen_ddplan(loDM, hiDM, numsub, resolution_ms).dedisp_plans()
