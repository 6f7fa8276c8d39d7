"""Summary of the bench JSON line in a log (its last line); exits 1 -- loudly -- when the log
holds no parsable bench line, so an A/B harness cannot lose a number silently.
    python3 scripts/benchline.py LOG [step|ms]"""
import json
import sys

log, mode = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "step")
lines = [ln for ln in open(log, errors="replace").read().splitlines() if ln.strip().startswith("{")]
try:
    d = json.loads(lines[-1])
    if mode == "ms":
        print("%.2f ms/step" % d["ms_per_step"])
    else:
        print("%.2f ms/step, stage1 %.2f, stage2 %.2f" % (d["ms_per_step"], d["kernel_ms_per_step"]["stage1"],
                                                          d["kernel_ms_per_step"]["stage2"]))
except (IndexError, ValueError, KeyError) as e:
    sys.stderr.write("no bench line in %s (%s: %s)\n" % (log, type(e).__name__, e))
    sys.exit(1)
