"""Per-kernel average durations from tools/kt_ab.sh output, one column per
library:  python3 tools/kt_summary.py gpurun_out lib_a lib_b ..."""
import collections, csv, glob, sys

root, libs = sys.argv[1], sys.argv[2:]
rows = collections.defaultdict(dict)
for lib in libs:
    per = collections.defaultdict(list)
    for d in sorted(glob.glob(f"{root}/kt_{lib}_[0-9]*/")):
        for p in glob.glob(d + "**/run_kernel_stats.csv", recursive=True):
            for r in csv.DictReader(open(p)):
                per[r["Name"]].append((float(r["TotalDurationNs"]), int(r["Calls"])))
    for name, v in per.items():
        rows[name][lib] = sum(t for t, _ in v) / sum(c for _, c in v) / 1e3
        rows[name]["_calls"] = v[0][1]
print(f"{'kernel':50s}" + "".join(f"{l[-14:]:>16s}" for l in libs))
for name, r in sorted(rows.items(), key=lambda kv: -max(v for k, v in kv[1].items() if k != "_calls") * kv[1]["_calls"]):
    if r["_calls"] * max(v for k, v in r.items() if k != "_calls") < 1000:
        continue
    print(f"{name[:50]:50s}" + "".join(f"{r.get(l, float('nan')):16.1f}" for l in libs))
