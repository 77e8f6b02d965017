"""Per-launch timeline of one FRI commit from a rocprofv3 kernel trace (csv).

    python tools/trace_commit.py DIR [which=-2]

Dev tool: the commit is delimited by the first NTT pass of consecutive commits."""
import csv
import sys

d = sys.argv[1]
which = int(sys.argv[2]) if len(sys.argv) > 2 else -2
tr = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
gx = "Grid_Size" if "Grid_Size" in tr[0] else "Grid_Size_X"
wx = "Workgroup_Size" if "Workgroup_Size" in tr[0] else "Workgroup_Size_X"
idx = [i for i, r in enumerate(tr) if "k_ntt_pass" in r["Kernel_Name"] and ", true" in r["Kernel_Name"]]
s = idx[which]
e = idx[which + 1] if which + 1 < 0 or which + 1 < len(idx) else len(tr)
t0 = int(tr[s]["Start_Timestamp"])
agg = {}
end = t0
for r in tr[s:e]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("fri::", "")
    g = int(r[gx]) // int(r[wx])
    print(f"{(st - t0) / 1e3:8.1f} {(en - st) / 1e3:7.1f} {name[:44]:44s} grid={g}")
    a = agg.setdefault(name, [0, 0.0])
    a[0] += 1
    a[1] += (en - st) / 1e3
    end = max(end, en)
for k, (n, us) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k[:60]:60s} n={n:3d} total_us={us:9.1f}")
print("commit span us", (end - t0) / 1e3)
