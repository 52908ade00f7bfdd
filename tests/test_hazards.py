"""No inline-asm depthwise result (DPP FMAC) may feed an MFMA, and no VALU result a DPP read, with
fewer than the 2 wait states gfx940+ requires (tools/hazard_scan.py; DESIGN.md sections 4.5, A.14: an
s_waitcnt alone between the two gave the RR kernel wrong B operands; ADVICE r05: one wait state is
not enough either).  Compiles every kernel translation unit to gfx950 assembly in parallel (~2 min
on 8 cores) and scans it; skipped where hipcc is absent."""
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TUS = ["nrx_k_rr.hip", "nrx_k_col.hip", "nrx_k_p16.hip", "nrx_k_p16m.hip", "nrx_k_p16s.hip", "nrx_k_fwd0.hip", "nrx_k_fwd1.hip",
       "nrx_k_fwd2.hip"]


def test_no_dpp_mfma_hazard(tmp_path):
    hipcc = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc")
    if not hipcc:
        pytest.skip("hipcc not available")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import hazard_scan

    def one(tu):
        out = tmp_path / (tu + ".s")
        src = os.path.join(ROOT, "neural_rx_amd", "csrc", tu)
        subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--offload-device-only", "-S",
                        "-o", str(out), src], check=True, capture_output=True)
        hits = hazard_scan.scan(out.read_text().splitlines())
        return tu, hits

    with ThreadPoolExecutor(min(len(TUS), os.cpu_count() or 4)) as ex:
        for tu, bad in ex.map(one, TUS):
            assert not bad, (tu, len(bad), bad[:5])
