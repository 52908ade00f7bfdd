"""Per-launch HBM traffic of the engine kernels from rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

usage: python tools/pmc_traffic.py <pmc_FETCH_SIZE dir> <pmc_WRITE_SIZE dir> <key>
Updates profiles/pmc_traffic.json[key].  FETCH_SIZE / WRITE_SIZE are in KiB; FETCH_SIZE
is doubled (MI355X_MICROARCH.md, HBM section: gfx950 tallies 128-B requests at 64 B for
16-B-per-lane streaming reads; the other access widths in these kernels are
uncalibrated).  k_update is averaged over its instantiations (non-last iterations and
the last one), weighted by how often a forward launches each (num_it - 1 : 1).
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(d, counter):
    acc = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            per[r["Dispatch_Id"]] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"]
        for disp, v in per.items():
            acc[names[disp]].append(v)
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(fdir, wdir, key, source=None, num_it=2):
    fe, wr = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    out = {}
    for k in fe:
        short = k.split("(")[0].replace("void ", "")
        out[short] = {"fetch_bytes_corrected": 2 * fe[k] * 1024, "write_bytes": wr.get(k, 0.0) * 1024}
        out[short]["bytes"] = out[short]["fetch_bytes_corrected"] + out[short]["write_bytes"]
    upd_mid = [v["bytes"] for k, v in out.items() if k.startswith("nrx::k_update") and k.endswith(", 0>")]
    # last iteration: readout tail (", 1>") or its paired heads-in-WB form (", 2>")
    upd_last = [v["bytes"] for k, v in out.items() if k.startswith("nrx::k_update") and k.endswith((", 1>", ", 2>"))]
    rec = {"kernels": out, "unit": "bytes per launch",
           "note": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), rocprofv3 separate --pmc passes"}
    if source:
        rec["source"] = source
    if upd_mid and upd_last:
        rec["k_update_bytes_per_launch"] = round(((num_it - 1) * upd_mid[0] + upd_last[0]) / num_it)
    # the one-launch forward (k_forward<A2P, CHP>): one instantiation per model shape
    fwd = [v["bytes"] for k, v in out.items() if k.startswith("nrx::k_forward")]
    if fwd:
        rec["k_forward_bytes_per_launch"] = round(fwd[0])
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    # keep the fields of an earlier capture of the other path (three-launch / one-launch)
    old = data.get(key, {})
    for f in ("k_update_bytes_per_launch", "k_forward_bytes_per_launch"):
        if f not in rec and f in old:
            rec[f] = old[f]
            rec.setdefault("earlier_source", {})[f] = old.get("source")
    data[key] = rec
    json.dump(data, open(path, "w"), indent=1, sort_keys=True)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else None)
