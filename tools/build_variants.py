"""Build kernel-variant libraries for A/B timing and diagnostics (never the product path).

    python tools/build_variants.py NAME="-DFOO=1 -DBAR=2" NAME2="..."

Each variant lands in neural_rx_amd/lib/var/NAME/libnrx.so (git-ignored; travels to the GPU
box; objects in lib/var/NAME/obj, rebuilt when stale); select it with NRX_LIB_PATH.  Its
nrx_build_id carries the flags, so committed counters never match a variant.
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
        out = os.path.join(ROOT, "neural_rx_amd", "lib", "var", name)
        B.build(force=False, verbose=False, lib=os.path.join(out, "libnrx.so"), obj_dir=os.path.join(out, "obj"),
                extra_flags=shlex.split(flags))
        print(name, "ok")
