"""Generate tests/golden/palfa_zaplist.json from the reference's one numeric input file,
lib/zaplists/PALFA.zaplist (the default zaplist search_job feeds to zapbirds,
lib/python/PALFA2_presto_search.py:472-474, 548-553; bin/search.py:180-182).

The parse here is independent of hipdedisp.fft_stage.read_zaplist (which the tests check
against this fixture): numpy.loadtxt over the lines that are not '#' comments, after noting
which lines carry the 'B' (barycentric) prefix.  Run in the build container, where
/root/reference exists:   python tests/golden/make_zaplist_fixture.py
"""
import json
import os

import numpy as np

SRC = "/root/reference/lib/zaplists/PALFA.zaplist"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "palfa_zaplist.json")


def main():
    lines = open(SRC).read().splitlines()
    data = [ln for ln in lines if ln.strip() and not ln.lstrip().startswith("#")]
    bary = [ln.lstrip()[:1] in ("B", "b") for ln in data]
    vals = np.loadtxt([ln.lstrip().lstrip("Bb") for ln in data], dtype=np.float64, ndmin=2)
    out = {
        "source": "lib/zaplists/PALFA.zaplist (reference)",
        "lines": len(lines),
        "comment_lines": sum(1 for ln in lines if ln.lstrip().startswith("#")),
        "birdies": [[float(f), float(w), bool(b)] for (f, w), b in zip(vals, bary)],
    }
    with open(OUT, "w") as f:
        f.write(json.dumps({k: v for k, v in out.items() if k != "birdies"})[:-1] + ", \"birdies\": [\n")
        f.write(",\n".join(json.dumps(b) for b in out["birdies"]) + "]}\n")
    print("%s: %d lines, %d birdies" % (OUT, out["lines"], len(out["birdies"])))


if __name__ == "__main__":
    main()
