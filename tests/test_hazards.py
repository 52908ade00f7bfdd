"""The register-resident update kernel's depthwise (inline-asm DPP FMACs) must never feed an MFMA
without a wait state in between (tools/hazard_scan.py; DESIGN.md section 14: an s_waitcnt alone
between the two gave wrong B operands).  Compiles nrx_k_rr.hip to gfx950 assembly (~20 s) and
scans it; skipped where hipcc is absent."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rr_kernel_has_no_dpp_mfma_hazard(tmp_path):
    hipcc = "/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else shutil.which("hipcc")
    if not hipcc:
        pytest.skip("hipcc not available")
    out = tmp_path / "rr.s"
    src = os.path.join(ROOT, "neural_rx_amd", "csrc", "nrx_k_rr.hip")
    subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--offload-device-only", "-S",
                    "-o", str(out), src], check=True, capture_output=True)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import hazard_scan
    hits = hazard_scan.scan(out.read_text().splitlines(), "k_update_rr")
    adjacent = [h for h in hits if h[1].endswith("d=1")]
    assert not adjacent, adjacent[:5]
