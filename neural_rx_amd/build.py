"""Build ``libnrx.so`` in-tree with hipcc for gfx950.

    python -m neural_rx_amd.build [--force]

The library is written to ``neural_rx_amd/lib/libnrx.so`` (git-ignored, but it
travels to the GPU box with the repository snapshot).
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "lib", "libnrx.so")
# one translation unit per strip tier / k_forward mode, so that an edit of one schedule recompiles
# only its own code object; nrx_device.inc / nrx_launch.inc hold the shared device and launch code
KERNEL_TUS = ["nrx_k_p16.hip", "nrx_k_p16m.hip", "nrx_k_p16s.hip", "nrx_k_p64.hip", "nrx_k_fwd0.hip",
              "nrx_k_fwd1.hip", "nrx_k_fwd2.hip", "nrx_k_rr.hip", "nrx_k_col.hip", "nrx_dispatch.hip"]
SOURCES = [os.path.join(CSRC, f) for f in KERNEL_TUS] + [
    os.path.join(CSRC, "nrx_aerial.hip"), os.path.join(CSRC, "nrx_synth.hip"), os.path.join(CSRC, "nrx_api.cpp")]
HEADERS = [os.path.join(CSRC, "nrx_internal.h"), os.path.join(HERE, "..", "include", "nrx.h")]
KERNEL_INCS = [os.path.join(CSRC, "nrx_device.inc"), os.path.join(CSRC, "nrx_launch.inc"),
               os.path.join(CSRC, "nrx_rr.inc"), os.path.join(CSRC, "nrx_col.inc")]
DEPS = SOURCES + HEADERS + KERNEL_INCS
ARCH = os.environ.get("NRX_OFFLOAD_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    raise RuntimeError("hipcc not found")


def needs_build() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    if any(os.path.getmtime(d) > t for d in DEPS if os.path.exists(d)):
        return True
    return any(_stale(os.path.join(OBJ_DIR, os.path.basename(s) + ".o"), s) for s in SOURCES)


OBJ_DIR = os.path.join(HERE, "lib", "obj")


def _includes(src: str) -> list:
    if os.path.basename(src) in KERNEL_TUS:
        return HEADERS + KERNEL_INCS
    return HEADERS


def _sig(src: str) -> str:
    """mtimes of a source and the headers it includes, taken when its compile starts (an edit
    made while that compile runs leaves the object stale)"""
    return " ".join(repr(os.path.getmtime(d)) for d in [src] + _includes(src) if os.path.exists(d))


def _stale(obj: str, src: str) -> bool:
    sig = obj + ".sig"
    if not os.path.exists(obj) or not os.path.exists(sig):
        return True
    return open(sig).read() != _sig(src)


def source_hash() -> str:
    """Content hash of every source the library is built from (the kernels, their includes, the
    host side).  Compiled into the library (nrx_build_id) at every link, so a counter capture
    (tools/pmc_record.py) and a later bench line can tell whether they describe the same kernels."""
    h = hashlib.sha256()
    for p in sorted(set(SOURCES + HEADERS + KERNEL_INCS)):
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def _build_id_object(verbose: bool, obj_dir: str = OBJ_DIR, tag: str = "") -> str:
    src = os.path.join(obj_dir, "nrx_build_id.cpp")
    obj = src + ".o"
    with open(src, "w") as f:
        f.write('extern "C" const char* nrx_build_id(void) { return "%s%s"; }\n' % (source_hash(), tag))
    cmd = [hipcc(), "-O2", "-fPIC", "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return obj


def build(force: bool = False, verbose: bool = True, lib: str = LIB, obj_dir: str = OBJ_DIR,
          extra_flags=()) -> str:
    """Compile the sources whose object is stale (force: all of them), in parallel, then link.
    Objects are kept in lib/obj/ (git-ignored) so that an edit of one source recompiles only
    that source.  lib / obj_dir / extra_flags: a diagnostic variant library (tools/build_variants.py)."""
    if lib == LIB and not force and not needs_build():
        return LIB
    os.makedirs(obj_dir, exist_ok=True)
    tmp = lib + f".tmp{os.getpid()}"
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
             *extra_flags]
    objs, procs = [], []
    for src in SOURCES:
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        objs.append(obj)
        if not force and not _stale(obj, src):
            continue
        part = obj + f".{os.getpid()}.part"
        cmd = [hipcc(), *flags, "-c", src, "-o", part]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((subprocess.Popen(cmd), part, obj, _sig(src)))
    bad = 0
    for p, part, obj, sig in procs:
        rc = p.wait()
        if rc:
            bad = rc
            if os.path.exists(part):
                os.remove(part)
        else:
            os.replace(part, obj)
            with open(obj + ".sig", "w") as f:
                f.write(sig)
    if bad:
        raise subprocess.CalledProcessError(bad, "hipcc -c")
    # a variant library carries its flags in the id, so its counters never pass for the default's
    objs.append(_build_id_object(verbose, obj_dir, "+" + "".join(extra_flags) if extra_flags else ""))
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", *objs, "-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv)
