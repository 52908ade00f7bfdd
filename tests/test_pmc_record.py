"""tools/pmc_record.py on synthetic rocprofv3 counter CSVs (CPU only).

The PMC records bench.py quotes must be per forward and per launch of the library that is
running: a forward split into slot chunks runs one k_init per chunk, so
the record takes the forward count bench.py --profile-only logs, not the k_init dispatches;
the update launches of both kernels (k_update, k_update_rr) are pooled; every record carries
the running library's nrx_build_id."""
import csv
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture
def pmc_record(monkeypatch, tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import pmc_record as m
    monkeypatch.setattr(m, "ROOT", str(tmp_path))
    monkeypatch.setattr(m, "running_build_id", lambda: "feedfacecafe0001")
    (tmp_path / "profiles").mkdir()
    return m


def _pass(dirpath, counter, per_kernel, forwards=None):
    """one --pmc pass: per_kernel = {kernel name: [value per dispatch]}"""
    os.makedirs(dirpath)
    rows, disp = [], 0
    for k, vals in per_kernel.items():
        for v in vals:
            disp += 1
            # two counter instances per dispatch (summed by the record)
            for part in (0.25, 0.75):
                rows.append({"Dispatch_Id": disp, "Counter_Name": counter, "Counter_Value": v * part,
                             "Kernel_Name": f"void {k}(args)"})
    with open(os.path.join(dirpath, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Counter_Name", "Counter_Value", "Kernel_Name"])
        w.writeheader()
        w.writerows(rows)
    if forwards is not None:
        with open(str(dirpath) + ".log", "w") as f:
            f.write("noise line\n" + json.dumps({"profile_only": True, "ms_per_step": 1.0, "forwards": forwards}) + "\n")


def test_chunked_forward_traffic_per_forward(pmc_record, tmp_path):
    # 2 forwards, each in 3 slot chunks: per chunk 1 k_init, 2 k_combine, 1 RR update, 1 readout
    fw, ch = 2, 3
    kern = {"nrx::k_init<P>": 3, "nrx::k_combine<P>": 2, "nrx::k_update_rr<16, 0>": 1, "nrx::k_update<P, 16, 1>": 1}
    fetch = {k: [1000.0 * (i + 1)] * (n * fw * ch) for i, (k, n) in enumerate(kern.items())}
    write = {k: [100.0 * (i + 1)] * (n * fw * ch) for i, (k, n) in enumerate(kern.items())}
    # (k_init dispatches counted 3 per chunk here only to make a wrong divisor visible)
    d1, d2 = str(tmp_path / "p1"), str(tmp_path / "p2")
    _pass(d1, "FETCH_SIZE", fetch, forwards=fw)
    _pass(d2, "WRITE_SIZE", write, forwards=fw)
    pmc_record.main("cfgX", "src", [d1, d2])
    rec = json.load(open(tmp_path / "profiles" / "pmc_traffic.json"))["cfgX"]
    assert rec["build_id"] == "feedfacecafe0001"
    want = 0.0
    for i, (k, n) in enumerate(kern.items()):
        per_disp = (2 * 1000.0 * (i + 1) + 100.0 * (i + 1)) * 1024
        assert rec["kernels"][k]["bytes_per_dispatch"] == round(per_disp)
        assert rec["kernels"][k]["dispatches_per_forward"] == n * ch
        want += per_disp * n * ch
    assert rec["forward_bytes"] == round(want)
    # the update launch figure pools k_update_rr and k_update by their dispatch counts
    u_rr, u_st = (2 * 3000 + 300) * 1024, (2 * 4000 + 400) * 1024
    assert rec["k_update_bytes_per_launch"] == round((u_rr + u_st) / 2)


def test_forward_count_falls_back_to_k_init(pmc_record, tmp_path):
    d1, d2 = str(tmp_path / "q1"), str(tmp_path / "q2")
    kern = {"nrx::k_init<P>": [10.0] * 4, "nrx::k_update<P, 16, 0>": [20.0] * 8}
    _pass(d1, "FETCH_SIZE", kern)
    _pass(d2, "WRITE_SIZE", kern)
    assert pmc_record.forwards_run([d1, d2]) == 0
    pmc_record.main("cfgY", "src", [d1, d2])
    rec = json.load(open(tmp_path / "profiles" / "pmc_traffic.json"))["cfgY"]
    assert rec["kernels"]["nrx::k_update<P, 16, 0>"]["dispatches_per_forward"] == 2.0
