"""Diagnostic / A-B variant libraries at neural_rx_amd/lib/diag/NAME/libnrx.so (git-ignored, not
gpurun-ignored: they travel to the GPU box; objects stay in /tmp).  Never the product path.

    python tools/build_diag.py stamps="-DNRX_STAMPS" nol2="-DNRX_COL_L2TOUCH=0" ...
"""
import os
import shlex
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from neural_rx_amd import build as B  # noqa: E402

if __name__ == "__main__":
    for spec in sys.argv[1:]:
        name, flags = spec.split("=", 1)
        out = os.path.join(ROOT, "neural_rx_amd", "lib", "diag", name)
        os.makedirs(out, exist_ok=True)
        B.build(force=False, verbose=False, lib=os.path.join(out, "libnrx.so"), obj_dir=f"/tmp/nrx_diag_{name}",
                extra_flags=shlex.split(flags))
        print(name, "ok", flush=True)
