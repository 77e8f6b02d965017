"""Per-kernel totals per commit from kt_ab.sh output dirs:
python tools/kt_sum.py gpurun_out/kt_<lib>_<round> ...  (13 commits per run)."""
import csv, glob, sys
for d in sys.argv[1:]:
    f = glob.glob(d + '/**/*kernel_stats.csv', recursive=True)[0]
    print(d)
    for r in csv.DictReader(open(f)):
        tot = float(r['TotalDurationNs']) / 1e3 / 24
        if tot > 5:
            print(f"  {r['Name'].split('(')[0][:48]:48s} calls {r['Calls']:>5} avg {float(r['AverageNs'])/1e3:8.1f} us  per commit {tot:8.1f} us")
