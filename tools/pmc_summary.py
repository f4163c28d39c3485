"""Summarise rocprofv3 --pmc counter_collection.csv files: mean counter value per dispatch, per
(kernel, grid size).  Usage: python tools/pmc_summary.py <csv> [<csv> ...]"""
import csv
import sys
from collections import defaultdict


def main(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        per = defaultdict(float)
        for r in csv.DictReader(open(p)):
            key = (r["Kernel_Name"], int(r["Grid_Size"]), r["Dispatch_Id"], r["Counter_Name"])
            per[key] += float(r["Counter_Value"])
        for (k, g, _, c), v in per.items():
            acc[(k, g)][c].append(v)
    for (k, g), cs in sorted(acc.items()):
        print("%s  grid %d" % (k, g))
        for c, vs in sorted(cs.items()):
            print("  %-28s %14.1f   (%d dispatches)" % (c, sum(vs) / len(vs), len(vs)))
        if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
            f = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"])
            w = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"])
            print("  traffic/launch: FETCH x2 (gfx950 correction) %.2f MB + WRITE %.2f MB = %.2f MB"
                  % (2 * f * 1024 / 1e6, w * 1024 / 1e6, (2 * f + w) * 1024 / 1e6))
        if "SQ_WAVE_CYCLES" in cs:
            wc = sum(cs["SQ_WAVE_CYCLES"]) / len(cs["SQ_WAVE_CYCLES"])
            m = lambda c: sum(cs[c]) / len(cs[c]) / wc * 100   # noqa: E731
            print("  wave cycles: wait %.0f%%, issue-stalled %.0f%%, issuing %.0f%%"
                  % (m("SQ_WAIT_ANY"), m("SQ_WAIT_INST_ANY"), m("SQ_ACTIVE_INST_ANY")))


if __name__ == "__main__":
    main(sys.argv[1:])
