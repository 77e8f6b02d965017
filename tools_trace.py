"""Summarise a rocprofv3 kernel trace: per-kernel stats and the timeline of the
last FRI commit (dev tool, reads gpurun_out/<dir>/run_kernel_trace.csv)."""
import csv
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
tr = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(tr) if "k_ntt_pass" in r["Kernel_Name"] and "true" in r["Kernel_Name"]]
s = idx[-1]
t0 = int(tr[s]["Start_Timestamp"])
prev = t0
agg = {}
for r in tr[s:]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fri::", "")
    g = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
    if len(sys.argv) > 2:
        print(f"{(st - t0) / 1e3:9.1f} {(en - st) / 1e3:8.1f} gap={(st - prev) / 1e3:5.1f} {name[:48]:48s} grid={g}")
    a = agg.setdefault(name, [0, 0.0])
    a[0] += 1
    a[1] += (en - st) / 1e3
    prev = en
for k, (n, us) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k[:60]:60s} n={n:3d} total_us={us:9.1f}")
print("commit span us", (prev - t0) / 1e3)
