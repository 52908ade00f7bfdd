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
# build.py itself: a change of the id rule (source_hash) relinks with a new nrx_build_id
DEPS = SOURCES + HEADERS + KERNEL_INCS + [os.path.abspath(__file__)]
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


def strip_comments(text: str) -> str:
    """C / C++ / HIP source without its comments, whitespace runs collapsed to one space (string
    and character literals kept verbatim): the code the compiler sees, for source_hash."""
    out, i, n = [], 0, len(text)
    while i < n:
        c = text[i]
        if c == "/" and i + 1 < n and text[i + 1] == "/":
            j = text.find("\n", i)
            i = n if j < 0 else j
            out.append(" ")
        elif c == "/" and i + 1 < n and text[i + 1] == "*":
            j = text.find("*/", i + 2)
            i = n if j < 0 else j + 2
            out.append(" ")
        elif c in "\"'":
            j = i + 1
            while j < n and text[j] != c:
                j += 2 if text[j] == "\\" else 1
            out.append(text[i:j + 1])
            i = j + 1
        else:
            out.append(c)
            i += 1
    return " ".join("".join(out).split())


def hash_sources(texts: dict) -> str:
    """16-hex-digit hash of {file name: source text}, comments and whitespace ignored."""
    h = hashlib.sha256()
    for name in sorted(texts):
        h.update(name.encode() + b"\0" + strip_comments(texts[name]).encode() + b"\0")
    return h.hexdigest()[:16]


def source_hash() -> str:
    """Hash of the code of every source the library is built from (the kernels, their includes,
    the host side) -- comments and whitespace excluded, so a comment-only edit keeps the id
    (VERDICT r05 item 5).  Compiled into the library (nrx_build_id) at every link, so a counter
    capture (tools/pmc_record.py) and a later bench line can tell whether they describe the same
    kernels."""
    texts = {}
    for p in sorted(set(SOURCES + HEADERS + KERNEL_INCS)):
        with open(p, encoding="utf-8") as f:
            texts[os.path.basename(p)] = f.read()
    return hash_sources(texts)


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
