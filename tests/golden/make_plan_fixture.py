"""Generate tests/golden/ddplan_ref.json by RUNNING the reference's own plan code.

Run once, in the build container (where /root/reference exists):

    python tests/golden/make_plan_fixture.py

The reference module `lib/python/PALFA2_presto_search.py` is Python 2 and imports
PRESTO (`psr_utils`, `presto`, `sifting`), so it cannot be imported whole under
python3.  Its `dedisp_plan` class (lines 374-410) is, however, valid Python 3 and
depends only on numpy.  This script lifts exactly that class body out of the
reference source text, executes it with numpy, and feeds it the hard-coded
(lodm, dmstep, dms/call, #calls, #subbands, downsamp) tuples it finds in
`obs_info.set_DDplan` (lines 319-331).  What is recorded is therefore the
reference's own output: subDM strings, per-pass DM strings, the stage-2
`-lodm` strings (format of line 514) and the subband base names (line 498).

The committed JSON is data (inputs + the reference's outputs), not source; the
product and the tests never read /root/reference at run time.
"""
import ast
import json
import os
import re
import sys

import numpy as np

REF = "/root/reference/lib/python/PALFA2_presto_search.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ddplan_ref.json")


def lift_class(src_lines, name):
    start = None
    for i, line in enumerate(src_lines):
        if line.startswith("class %s" % name):
            start = i
            continue
        if start is not None and i > start and line and not line[0].isspace():
            return "".join(src_lines[start:i]), start + 1, i
    raise RuntimeError("class %s not found" % name)


def lift_plans(src_lines):
    """Return {backend: [tuple, ...]} from obs_info.set_DDplan's hard-coded calls."""
    plans, backend = {}, None
    in_fn = False
    for line in src_lines:
        if "def set_DDplan" in line:
            in_fn = True
            continue
        if in_fn and line.strip().startswith("def "):
            break
        if not in_fn:
            continue
        m = re.search(r"self\.backend\.lower\(\) == '(\w+)'", line)
        if m:
            backend = m.group(1)
            plans[backend] = []
            continue
        m = re.match(r"\s*self\.ddplans\.append\(dedisp_plan\((.*)\)\)\s*$", line)
        if m and backend:
            plans[backend].append(tuple(ast.literal_eval("(%s)" % m.group(1))))
    return plans


def main():
    if not os.path.exists(REF):
        sys.exit("reference not present; the committed fixture is authoritative")
    lines = open(REF).read().splitlines(True)
    cls_src, l0, l1 = lift_class(lines, "dedisp_plan")
    ns = {"np": np}
    exec(compile(cls_src, REF, "exec"), ns)
    dedisp_plan = ns["dedisp_plan"]
    plans = lift_plans(lines)
    out = {"source": "lib/python/PALFA2_presto_search.py:%d-%d (dedisp_plan), "
                     ":319-331 (set_DDplan tables)" % (l0, l1),
           "generator": "tests/golden/make_plan_fixture.py",
           "backends": {}}
    for backend, tuples in plans.items():
        stages = []
        for tup in tuples:
            p = dedisp_plan(*tup)
            passes = []
            for passnum in range(p.numpasses):
                passes.append({
                    "subdm": p.subdmlist[passnum],
                    # stage-2 "-lodm %.2f" argument, PALFA2_presto_search.py:514-516
                    "lodm_arg": "%.2f" % (p.lodm + passnum * p.sub_dmstep),
                    "dmstep_arg": "%.2f" % p.dmstep,
                    "dms": p.dmlist[passnum],
                })
            stages.append({
                "args": list(tup),
                "lodm": p.lodm, "dmstep": p.dmstep, "dmsperpass": p.dmsperpass,
                "numpasses": p.numpasses, "numsub": p.numsub, "downsamp": p.downsamp,
                "sub_downsamp": p.sub_downsamp, "dd_downsamp": p.dd_downsamp,
                "sub_dmstep": p.sub_dmstep,
                "passes": passes,
            })
        out["backends"][backend] = stages
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    n = {b: sum(len(ps["dms"]) for s in st for ps in s["passes"]) for b, st in out["backends"].items()}
    print("wrote", OUT, "DM counts:", n)


if __name__ == "__main__":
    main()
