"""Per-dispatch timeline of one FRI commit from a rocprofv3 kernel trace.

Usage: python tools/timeline.py <kernel_trace.csv> [commit_index_from_end=1] [min_layer0_us=0]

A commit starts at its first k_ntt_pass dispatch; prints, for the chosen
commit, every kernel's start offset, duration and the idle gap before it, plus
per-kernel-name totals and the sum of gaps.
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*$", "", name)
    name = name.replace("void ", "").replace("fri::", "")
    return name


def main():
    path = sys.argv[1]
    which = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    first = [i for i, r in enumerate(rows) if r[2].startswith("k_ntt_pass") and r[2].split(",")[2].strip() == "true"]
    min_us = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0      # layer-0 leaf duration filter
    l0 = [i for i, r in enumerate(rows)
          if r[2].startswith("k_layer_leaf<false, true") and (r[1] - r[0]) / 1e3 >= min_us]
    anchor = l0[-which]
    lo = max(i for i in first if i < anchor)
    later = [i for i in first if i > anchor]
    hi = later[0] if later else len(rows)
    seg = rows[lo:hi]
    t0 = seg[0][0]
    prev_end = t0
    tot = defaultdict(float)
    cnt = defaultdict(int)
    gaps = 0.0
    for s, e, n in seg:
        gap = (s - prev_end) / 1e3
        gaps += max(gap, 0.0)
        dur = (e - s) / 1e3
        tot[n] += dur
        cnt[n] += 1
        print(f"{(s - t0) / 1e3:9.1f} us  gap {gap:6.1f}  dur {dur:8.1f}  {n}")
        prev_end = max(prev_end, e)
    span = (prev_end - t0) / 1e3
    print(f"\ncommit span {span:.1f} us, dispatches {len(seg)}, sum of gaps {gaps:.1f} us")
    for n in sorted(tot, key=lambda k: -tot[k]):
        print(f"  {tot[n]:8.1f} us  x{cnt[n]:3d}  {n}")


if __name__ == "__main__":
    main()
