"""Distinct offset patterns per subband pair and per quad over each pass's 76-DM y-block
(quad partials would pay only with <= ~8 patterns per quad).  Host only:
python3 scripts/count_patterns.py  (C2's pdev DDplan at 2^22)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "pipeline2.0_amd")]
from hipdedisp import Opts, PassParams, plan  # noqa: E402
from hipdedisp.engine import plan_tables  # noqa: E402
from hipdedisp.synth import palfa_obs  # noqa: E402

obs = palfa_obs(N=1 << 22)
for st, d in enumerate(plan.ddplans_for("pdev")):
    for i in sorted({0, d.numpasses // 2, d.numpasses - 1}):
        pp = PassParams(subdm=float(d.subdmlist[i]), lodm=float(d.lodm_arg(i)), dmstep=float(d.dmstep_arg()),
                        numdms=d.dmsperpass, nsub=d.numsub, ds=d.sub_downsamp, numout=0)
        _, off, _ = plan_tables(obs, Opts(), pp)
        u2 = [len({tuple(off[k, 2 * c + 1:2 * c + 2] - off[k, 2 * c]) for k in range(pp.numdms)}) for c in range(pp.nsub // 2)]
        u4 = [len({tuple(off[k, 4 * c + 1:4 * c + 4] - off[k, 4 * c]) for k in range(pp.numdms)}) for c in range(pp.nsub // 4)]
        print("stage %d pass %2d: pairs mean %.2f max %d sum %d | quads mean %.2f max %d sum %d"
              % (st, i, np.mean(u2), max(u2), sum(u2), np.mean(u4), max(u4), sum(u4)))
