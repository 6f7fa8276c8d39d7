"""Generate tests/golden/ddplan2b_ref.json by RUNNING the reference's own DDplan2b planner.

Run once, in the build container (where /root/reference exists):

    python tests/golden/make_ddplan2b_fixture.py

`lib/python/DDplan2b.py` is Python 2 (print statements, classic integer division) and
imports matplotlib and PRESTO's psr_utils at module level, so it cannot be imported under
python3 here.  This script takes the module text from the constants (ALLOW_DMSTEPS, :29)
through guess_DMstep (:425-434), i.e. the Observation / DDstep / DDplan classes, and:

  * converts it with lib2to3's print fixer (the only Python-2 syntax in that span);
  * rewrites every `/` into `_py2div(a, b)`, which is Python 2's `/`: floor division when
    both operands are ints, true division otherwise (an AST pass, so the semantics stay
    those of the reference);
  * drops the `plt.rc(...)` styling call (plotting is never invoked) and supplies
    `psr_utils.dm_smear` in the form hipdedisp.plan restates [PRESTO-ext: PRESTO is absent;
    the form is the one DDplan2b.guess_DMstep, :425-434, inverts], labelled in the JSON.

It then runs gen_ddplan for the config-4 plan (PALFA Mock, DM 0-10000, 96 subbands,
0.1 ms) and a few others, and records every DDstep.  The JSON is data (inputs + the
reference's outputs), not source; nothing reads /root/reference at test time.
"""
import ast
import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "pipeline2.0_amd"))
REF = "/root/reference/lib/python/DDplan2b.py"
OUT = os.path.join(HERE, "ddplan2b_ref.json")

CASES = [
    # (dt, fctr, BW, numchan, numsamp, loDM, hiDM, numsub, resolution_ms)
    (65.476e-6, 1375.5, 322.6, 960, 2048, 0.0, 10000.0, 96, 0.1),    # config 4 (tests/test_gpu_parity.py)
    (65.476e-6, 1375.5, 322.6, 960, 2048, 0.0, 1100.0, 96, 0.1),
    (65.476e-6, 1375.5, 322.6, 960, 0, 0.0, 3000.0, 96, 0.5),       # numsamp 0: powers of 2
    (64e-6, 1400.0, 300.0, 1024, 0, 0.0, 1000.0, 0, 0.0),           # DDplan2.py's defaults, no subbands
    (6.5476e-5, 1375.5, 322.6, 960, 7680, 100.0, 2000.0, 32, 1.0),
]


def _py2div(a, b):
    """Python 2 `/`."""
    if isinstance(a, (int, np.integer)) and isinstance(b, (int, np.integer)) \
            and not isinstance(a, bool) and not isinstance(b, bool):
        return a // b
    return a / b


class _Py2Div(ast.NodeTransformer):
    def visit_BinOp(self, node):
        self.generic_visit(node)
        if isinstance(node.op, ast.Div):
            return ast.copy_location(ast.Call(func=ast.Name("_py2div", ast.Load()), args=[node.left, node.right],
                                              keywords=[]), node)
        return node

    def visit_AugAssign(self, node):
        self.generic_visit(node)
        if isinstance(node.op, ast.Div):
            tgt = node.target
            load = ast.Name(tgt.id, ast.Load()) if isinstance(tgt, ast.Name) else \
                ast.Attribute(tgt.value, tgt.attr, ast.Load())
            return ast.copy_location(ast.Assign(targets=[tgt], value=ast.Call(
                func=ast.Name("_py2div", ast.Load()), args=[load, node.value], keywords=[])), node)
        return node


def load_reference():
    from lib2to3 import refactor
    lines = open(REF).read().splitlines(True)
    start = next(i for i, l in enumerate(lines) if l.startswith("ALLOW_DMSTEPS"))
    stop = next(i for i, l in enumerate(lines) if l.startswith("def main"))
    body = [l for l in lines[start:stop] if not l.startswith("plt.rc(")]
    text = "".join(body)
    tool = refactor.RefactoringTool(["lib2to3.fixes.fix_print"])
    text = str(tool.refactor_string(text, "DDplan2b.py"))
    tree = _Py2Div().visit(ast.parse(text))
    ast.fix_missing_locations(tree)
    from hipdedisp import plan as P
    ns = {"np": np, "_py2div": _py2div, "plt": None,
          "psr_utils": types.SimpleNamespace(dm_smear=P.dm_smear)}
    exec(compile(tree, REF, "exec"), ns)
    return ns, start + 1, stop


def main():
    if not os.path.exists(REF):
        sys.exit("reference not present; the committed fixture is authoritative")
    ns, l0, l1 = load_reference()
    out = {"source": "lib/python/DDplan2b.py:%d-%d (Observation, DDstep, DDplan, guess_DMstep), "
                     "lib2to3 print fixer + Python-2 division" % (l0, l1),
           "dm_smear": "psr_utils.dm_smear [PRESTO-ext, absent]: |DM| * BW / (0.0001205 * fctr**3), "
                       "the inverse of DDplan2b.guess_DMstep (hipdedisp.plan.dm_smear)",
           "generator": "tests/golden/make_ddplan2b_fixture.py",
           "cases": []}
    for case in CASES:
        dt, fctr, BW, numchan, numsamp, loDM, hiDM, numsub, res = case
        obs = ns["Observation"](dt, fctr, BW, numchan, numsamp)
        plan = obs.gen_ddplan(loDM, hiDM, numsub, res)
        steps = []
        for s in plan.DDsteps:
            steps.append({"loDM": float(s.loDM), "hiDM": float(s.hiDM), "dDM": float(s.dDM),
                          "downsamp": int(s.downsamp), "dsubDM": float(s.dsubDM), "numDMs": int(s.numDMs),
                          "DMs_per_prepsub": int(getattr(s, "DMs_per_prepsub", 0)), "numprepsub": int(s.numprepsub),
                          "str": str(s)})
        out["cases"].append({"args": list(case), "allow_factors": [int(f) for f in obs.allow_factors],
                             "resolution": float(plan.resolution),
                             "work_fracts": [float(w) for w in plan.work_fracts], "steps": steps})
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", OUT, [len(c["steps"]) for c in out["cases"]])


if __name__ == "__main__":
    main()
