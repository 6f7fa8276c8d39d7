"""Print name / calls / average us of the kernels of a kstats.py CSV whose names contain any of
the given substrings.  Usage: kstats_grep.py <csv> <substr>..."""
import csv
import sys

for r in csv.reader(open(sys.argv[1])):
    if r[0] != "Name" and any(k in r[0] for k in sys.argv[2:]):
        print("%-60s %5s %9.1f us" % (r[0].replace("void hd::", "")[:60], r[1], float(r[3]) / 1e3))
