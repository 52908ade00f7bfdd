"""Diagnostic: per-kernel durations and the idle gaps between consecutive kernels of a rocprofv3
kernel trace (``--kernel-trace --output-format csv``), for the kernels of one forward in steady
state.  usage: python tools/kt_gaps.py <kernel_trace.csv> [first kernel name substring]"""
import csv
import statistics as st
import sys


def main(path, head="k_init"):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if "nrx::" in r["Kernel_Name"]]
    dur, gap = {}, {}
    for a, b in zip(rows, rows[1:]):
        na, nb = a["Kernel_Name"].split("(")[0], b["Kernel_Name"].split("(")[0]
        g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) * 1e-3
        if g < 50:   # same forward stream (the bench's host runs ahead), not a host pause
            gap.setdefault((na, nb), []).append(g)
    for r in rows:
        n = r["Kernel_Name"].split("(")[0]
        dur.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    for n, v in dur.items():
        print(f"{n:60s} n={len(v):5d} median {st.median(v):8.2f} us")
    for (a, b), v in gap.items():
        print(f"gap {a} -> {b}: n={len(v)} median {st.median(v):.2f} us, p10 {sorted(v)[len(v) // 10]:.2f}")


if __name__ == "__main__":
    main(*sys.argv[1:])
