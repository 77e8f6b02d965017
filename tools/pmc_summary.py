"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv:
python3 tools/pmc_summary.py DIR [name-substring ...]"""
import collections, csv, glob, sys

path = glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0]
keys = sys.argv[2:] or [""]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"]
    if not any(k in n for k in keys):
        continue
    acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[n].add(r["Dispatch_Id"])
for n, c in acc.items():
    k = len(cnt[n])
    print(n[:60], "launches", k)
    for name, v in sorted(c.items()):
        print(f"   {name:24s} {v / k:16.4g}")
