"""Build kernel-variant libraries for A/B timing (diagnostic only).

    python tools/build_variants.py NAME="-DFOO=1 -DBAR=2" NAME2="..."

Each variant lands in neural_rx_amd/lib/var/NAME/libnrx.so (git-ignored; travels to the
GPU box); tools/bench_variants.sh times them with NRX_LIB_PATH.
"""
import os
import shlex
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from neural_rx_amd import build as B  # noqa: E402


def one(spec):
    name, flags = spec.split("=", 1)
    out = os.path.join(ROOT, "neural_rx_amd", "lib", "var", name)
    os.makedirs(out, exist_ok=True)
    cmd = [B.hipcc(), f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-function", *shlex.split(flags), *B.SOURCES, "-o", os.path.join(out, "libnrx.so")]
    r = subprocess.run(cmd, capture_output=True, text=True)
    return name, r.returncode, r.stderr[-2000:]


if __name__ == "__main__":
    with ThreadPoolExecutor(4) as ex:
        for name, rc, err in ex.map(one, sys.argv[1:]):
            print(name, "ok" if rc == 0 else "FAILED\n" + err)
