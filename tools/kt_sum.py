"""Per-kernel averages and per-commit totals from kt_ab.sh output dirs:
python tools/kt_sum.py gpurun_out/kt_<lib>_<round> ...
(commits = launches of the first LDE pass kernel in the run)."""
import csv, glob, sys
for d in sys.argv[1:]:
    f = glob.glob(d + '/**/*kernel_stats.csv', recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    commits = max(int(r['Calls']) for r in rows if 'k_ntt_pass<4, 4, true' in r['Name'] or 'k_ntt_first' in r['Name'])
    print(f"{d} ({commits} commits)")
    for r in rows:
        tot = float(r['TotalDurationNs']) / 1e3 / commits
        if tot > 5:
            print(f"  {r['Name'].split('(')[0][:48]:48s} calls {r['Calls']:>5} avg {float(r['AverageNs'])/1e3:8.1f} us  per commit {tot:8.1f} us")
