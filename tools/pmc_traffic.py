"""HBM traffic per launch from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE
collected in separate runs, as MI355X_MICROARCH.md "HBM" prescribes).

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR LOG_N [OUT_JSON]

Corrections (MI355X_MICROARCH.md §HBM): the counters are in KiB; on gfx950
FETCH_SIZE reports half the bytes of 16-B/lane streaming reads, so it is
doubled (the leaf kernel reads values as uint4 per lane); WRITE_SIZE is exact
for 16-B/lane stores (digests are stored as two uint4 per lane).
"""
import csv
import json
import os
import sys

DOMINANT_KERNEL = "fri::k_layer_leaf<false, true"       # layer 0 (prefix: + ", 256u>"): leaves + levels 1-4


def per_launch(path, counter):
    vals = {}
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].replace("void ", "").split("(")[0]
        vals.setdefault(name, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    fdir, wdir, log_n = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = sys.argv[4] if len(sys.argv) > 4 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                             "pmc_traffic.json")
    fetch, nf = per_launch(fdir, "FETCH_SIZE")
    write, nw = per_launch(wdir, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        fb = 2.0 * 1024.0 * fetch.get(k, 0.0)
        wb = 1024.0 * write.get(k, 0.0)
        kernels[k] = {"fetch_bytes_corrected": fb, "write_bytes": wb, "hbm_bytes_per_launch": fb + wb,
                      "launches_fetch": nf.get(k, 0), "launches_write": nw.get(k, 0)}
    dom_name = next(k for k in kernels if k.startswith(DOMINANT_KERNEL))
    dom = kernels[dom_name]
    res = {}
    if os.path.exists(out):
        res = json.load(open(out))
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from bench import source_hash          # the sources this library was built from (bench.py checks it)
    res[str(log_n)] = {
        "source_hash": source_hash(),
        "merkle_layer0_leaf": dict(dom, kernel=dom_name),
        "all_kernels_avg_per_launch": kernels,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes (csv), KiB -> bytes, "
                  "FETCH_SIZE x2 (gfx950 16-B/lane read correction), averaged over every launch in the run",
    }
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(res[str(log_n)]["merkle_layer0_leaf"]))


if __name__ == "__main__":
    main()
