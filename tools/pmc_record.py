"""Record the PMC passes of one bench configuration into the JSON files bench.py reads.

usage: python tools/pmc_record.py <key> <source-note> <pmc dir>...

Each <pmc dir> is one rocprofv3 ``--pmc`` pass (``-d <dir> --output-format csv``) over
``bench.py --profile-only``; the passes may hold any of the counters below.  Per dispatch of
the dominant kernel (k_forward, else k_update averaged over its instantiations):

* profiles/pmc_traffic.json[key]: ``k_forward_bytes_per_launch`` = 2 x FETCH_SIZE + WRITE_SIZE
  (KiB -> bytes; FETCH x 2 is the gfx950 correction of MI355X_MICROARCH.md's HBM section).
* profiles/pmc_sq.json[key][kernel] (k_forward, or k_update pooled over its instantiations for
  the three-launch forward): per-SIMD fractions of the wave lifetime --
  ``mfma_busy_frac`` = SQ_VALU_MFMA_BUSY_CYCLES / SIMDs / lifetime, ``valu_issue_frac`` =
  SQ_INSTS_VALU x 4.5 cycles (the measured issue cost) / SIMDs /
  lifetime, ``wait_frac`` = SQ_WAIT_ANY / SQ_WAVE_CYCLES, where lifetime = 4 x SQ_WAVE_CYCLES /
  SQ_WAVES (SQ_WAVE_CYCLES counts quad-cycles) and SIMDs = 4 x CUs.
Every record carries ``build_id`` = nrx_build_id() of the profiled library; bench.py quotes the
counters only when it matches the library it runs (``roofline.counters_match_build``).
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VALU_ISSUE_CYCLES = 4.5


def per_dispatch(dirs):
    """{kernel short name: {counter: mean over dispatches of the per-dispatch sum}}"""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = collections.defaultdict(float)
            names = {}
            for r in csv.DictReader(open(f)):
                key = (r["Dispatch_Id"], r["Counter_Name"])
                per[key] += float(r["Counter_Value"])
                names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0].replace("void ", "")
            for (disp, c), v in per.items():
                acc[names[disp]][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def dispatch_counts(dirs):
    """{kernel short name: dispatches} of the first pass directory that has counters"""
    for d in dirs:
        seen = collections.defaultdict(set)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                seen[r["Kernel_Name"].split("(")[0].replace("void ", "")].add(r["Dispatch_Id"])
        if seen:
            return {k: len(v) for k, v in seen.items()}
    return {}


def forwards_run(dirs):
    """forwards the profiled bench run executed: bench.py --profile-only prints them in the
    pass's log (<dir>.log); a forward split into slot chunks runs one k_init per chunk, so
    counting k_init dispatches would report per-chunk bytes"""
    for d in dirs:
        log = d.rstrip("/") + ".log"
        if os.path.exists(log):
            for line in open(log):
                if line.startswith("{") and '"forwards"' in line:
                    return json.loads(line)["forwards"]
    return 0


def running_build_id():
    """nrx_build_id() of the in-tree libnrx.so -- the library the passes just profiled"""
    sys.path.insert(0, ROOT)
    from neural_rx_amd import _lib
    return _lib.load().nrx_build_id().decode()


def main(key, source, dirs, cus=256):
    build_id = running_build_id()
    pk = per_dispatch(dirs)
    fwd = {k: v for k, v in pk.items() if k.startswith("nrx::k_forward") or k.startswith("nrx::k_fwd_col")}
    name, c = next(iter(fwd.items())) if fwd else (None, {})
    sq_key = "k_fwd_col" if name and name.startswith("nrx::k_fwd_col") else "k_forward"
    if not fwd:
        # three-launch forward: the dominant kernel is k_update (its instantiations pooled,
        # per-dispatch means weighted by their dispatch counts)
        cnt = dispatch_counts(dirs)
        ups = {k: v for k, v in pk.items() if k.startswith("nrx::k_update")}
        n = sum(cnt.get(k, 0) for k in ups)
        if ups and n:
            keys = set().union(*[set(v) for v in ups.values()])
            c = {ck: sum(v.get(ck, 0.0) * cnt.get(k, 0) for k, v in ups.items()) / n for ck in keys}
            name, sq_key = "nrx::k_update (all instantiations)", "k_update"
    traffic, sq = {}, {}

    def sq_fracs(cs):
        life = 4 * cs["SQ_WAVE_CYCLES"] / cs["SQ_WAVES"]
        simds = 4 * cus
        r = {"wave_lifetime_cycles": round(life)}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in cs:
            r["mfma_busy_frac"] = round(cs["SQ_VALU_MFMA_BUSY_CYCLES"] / simds / life, 4)
        if "SQ_INSTS_VALU" in cs:
            r["valu_issue_frac"] = round(cs["SQ_INSTS_VALU"] * VALU_ISSUE_CYCLES / simds / life, 4)
        if "SQ_WAIT_ANY" in cs:
            r["wait_frac"] = round(cs["SQ_WAIT_ANY"] / cs["SQ_WAVE_CYCLES"], 4)
        r["counters"] = {k: round(v, 1) for k, v in sorted(cs.items())}
        return r
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        fb, wb = 2 * c["FETCH_SIZE"] * 1024, c["WRITE_SIZE"] * 1024
        traffic = {"k_forward_bytes_per_launch": round(fb + wb), "source": source, "build_id": build_id,
                   "kernels": {name: {"fetch_bytes_corrected": fb, "write_bytes": wb, "bytes": fb + wb}},
                   "unit": "bytes per launch",
                   "note": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), rocprofv3 separate --pmc passes"}
    if "SQ_WAVE_CYCLES" in c and "SQ_WAVES" in c:
        simds = 4 * cus
        life = 4 * c["SQ_WAVE_CYCLES"] / c["SQ_WAVES"]
        rec = {"kernel": name, "source": source, "wave_lifetime_cycles": round(life), "build_id": build_id}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            rec["mfma_busy_frac"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / simds / life, 4)
        if "SQ_INSTS_VALU" in c:
            rec["valu_issue_frac"] = round(c["SQ_INSTS_VALU"] * VALU_ISSUE_CYCLES / simds / life, 4)
        if "SQ_WAIT_ANY" in c:
            rec["wait_frac"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
        rec["counters"] = {k: round(v, 1) for k, v in sorted(c.items())}
        sq = {sq_key: rec}
        # every kernel of the forward on its own (StateInit included: VERDICT r05 item 1)
        sq["per_kernel"] = {"source": source, "build_id": build_id,
                            **{k: sq_fracs(cs) for k, cs in pk.items()
                               if k.startswith("nrx::") and "SQ_WAVE_CYCLES" in cs and cs.get("SQ_WAVES")}}
    if not fwd:
        # three-launch forward (e.g. cfg5's per-GPU shard, U = 8): every kernel's bytes per
        # dispatch, and the forward's total = sum over kernels of mean x dispatches per forward
        # (forwards = the count bench.py --profile-only logged, else k_init dispatches)
        cnt = dispatch_counts(dirs)
        n_fwd = forwards_run(dirs) or max((v for k, v in cnt.items() if k.startswith("nrx::k_init")), default=0)
        kern, tot = {}, 0.0
        for k, cs in pk.items():
            if "FETCH_SIZE" in cs and "WRITE_SIZE" in cs and k.startswith("nrx::"):
                b = 2 * cs["FETCH_SIZE"] * 1024 + cs["WRITE_SIZE"] * 1024
                per_fwd = cnt.get(k, 0) / n_fwd if n_fwd else 0
                kern[k] = {"bytes_per_dispatch": round(b), "dispatches_per_forward": per_fwd}
                tot += b * per_fwd
        if kern:
            ub = [(v["bytes_per_dispatch"], cnt.get(k, 0)) for k, v in kern.items() if k.startswith("nrx::k_update")]
            nu = sum(n for _, n in ub)
            traffic = {"forward_bytes": round(tot), "kernels": kern, "source": source, "build_id": build_id,
                       "k_update_bytes_per_launch": round(sum(bb * n for bb, n in ub) / nu) if nu else None,
                       "unit": "bytes per forward (sum over its launches)",
                       "note": "2 x FETCH_SIZE + WRITE_SIZE per dispatch, rocprofv3 separate --pmc passes"}
    for fname, rec in (("pmc_traffic.json", traffic), ("pmc_sq.json", sq)):
        if not rec:
            continue
        path = os.path.join(ROOT, "profiles", fname)
        data = json.load(open(path)) if os.path.exists(path) else {}
        if fname == "pmc_sq.json":
            data.setdefault(key, {}).update(rec)
        else:
            old = data.get(key, {})
            if "k_update_bytes_per_launch" in old and rec.get("k_update_bytes_per_launch") is None:
                rec["k_update_bytes_per_launch"] = old["k_update_bytes_per_launch"]
                rec.setdefault("earlier_source", {})["k_update_bytes_per_launch"] = old.get("source")
            data[key] = rec
        json.dump(data, open(path, "w"), indent=1, sort_keys=True)
        print(fname, json.dumps(rec, indent=1)[:2000])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
