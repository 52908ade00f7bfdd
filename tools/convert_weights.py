"""Convert the reference's pickled Keras ``get_weights()`` lists into ``.npz`` files.

The reference stores trained weights as a pickled ``list[np.ndarray]``
(``utils/utils.py:34-51`` writes them, ``:53-70`` reads them with ``pickle.load``).
Loading such a file with ``pickle`` would execute whatever the file asks for, so
this tool never unpickles anything.  It walks the opcode stream with
``pickletools.genops`` (a pure parser) and interprets only the handful of opcodes a
``list`` of ``numpy.ndarray`` produces.  Globals are recorded as *names* and compared
against an allow-list; nothing is imported or called.  Array payloads are rebuilt
with ``numpy.frombuffer`` from the raw bytes in the ``BUILD`` state tuple
``(version, shape, dtype, is_fortran, rawdata)``.

Run once in the build container (where ``/root/reference`` exists):

    python tools/convert_weights.py

Output: ``weights/<label>.npz`` with arrays ``w000 .. wNNN`` in Keras order plus a
``count`` entry.  The layer order is documented in SURVEY.md section 8(a) row a15.
"""
from __future__ import annotations

import os
import pickletools
import sys

import numpy as np

REF_WEIGHTS = "/root/reference/weights"
OUT_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "weights")

# The five configurations in scope (BASELINE.json configs).
LABELS = [
    "nrx_rt",
    "nrx_rt_var_mcs",
    "nrx_large",
    "nrx_large_64qam",
    "nrx_large_var_mcs_64qam_masking",
]

_ALLOWED_GLOBALS = {
    ("numpy.core.multiarray", "_reconstruct"),
    ("numpy._core.multiarray", "_reconstruct"),   # numpy >= 2 spelling
    ("numpy", "ndarray"),
    ("numpy", "dtype"),
}
_RECONSTRUCT = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct")}


class _Global:
    def __init__(self, module, name):
        if (module, name) not in _ALLOWED_GLOBALS:
            raise ValueError(f"refusing pickle global {module}.{name}")
        self.key = (module, name)


class _ArrayStub:
    """Placeholder produced by ``_reconstruct(ndarray, (0,), b'b')``."""

    array = None


class _DtypeStub:
    def __init__(self, code):
        self.code = code
        self.byteorder = "="


_MARK = object()


def read_weight_list(path: str) -> list[np.ndarray]:
    data = open(path, "rb").read()
    stack: list = []
    memo: dict = {}
    result = None
    for op, arg, _pos in pickletools.genops(data):
        name = op.name
        if name in ("PROTO", "FRAME"):
            continue
        if name == "EMPTY_LIST":
            stack.append([])
        elif name == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif name in ("BINGET", "LONG_BINGET"):
            stack.append(memo[arg])
        elif name == "MARK":
            stack.append(_MARK)
        elif name in ("SHORT_BINUNICODE", "BINUNICODE", "BININT1", "BININT", "BININT2",
                      "SHORT_BINBYTES", "BINBYTES", "BINBYTES8"):
            stack.append(arg)
        elif name == "NEWFALSE":
            stack.append(False)
        elif name == "NEWTRUE":
            stack.append(True)
        elif name == "NONE":
            stack.append(None)
        elif name == "STACK_GLOBAL":
            gname = stack.pop()
            gmod = stack.pop()
            stack.append(_Global(gmod, gname))
        elif name in ("TUPLE1", "TUPLE2", "TUPLE3"):
            n = int(name[-1])
            items = tuple(stack[-n:])
            del stack[-n:]
            stack.append(items)
        elif name == "TUPLE":
            i = len(stack) - 1 - stack[::-1].index(_MARK)
            items = tuple(stack[i + 1:])
            del stack[i:]
            stack.append(items)
        elif name == "REDUCE":
            args = stack.pop()
            fn = stack.pop()
            if not isinstance(fn, _Global):
                raise ValueError("REDUCE on a non-global")
            if fn.key in _RECONSTRUCT:
                stack.append(_ArrayStub())
            elif fn.key == ("numpy", "dtype"):
                stack.append(_DtypeStub(args[0]))
            else:
                raise ValueError(f"REDUCE on {fn.key}")
        elif name == "BUILD":
            state = stack.pop()
            obj = stack[-1]
            if isinstance(obj, _DtypeStub):
                obj.byteorder = state[1]
            elif isinstance(obj, _ArrayStub):
                _ver, shape, dt, fortran, raw = state
                if dt.code not in ("f4", "f8", "i4", "i8"):
                    raise ValueError(f"unexpected dtype {dt.code}")
                order = "<" if dt.byteorder in ("<", "=", "|") else ">"
                arr = np.frombuffer(raw, dtype=np.dtype(order + dt.code))
                arr = arr.reshape(shape, order="F" if fortran else "C")
                obj.array = np.ascontiguousarray(arr.astype(arr.dtype.newbyteorder("=")))
            else:
                raise ValueError("BUILD on unexpected object")
        elif name == "APPENDS":
            i = len(stack) - 1 - stack[::-1].index(_MARK)
            items = stack[i + 1:]
            del stack[i:]
            stack[-1].extend(items)
        elif name == "APPEND":
            item = stack.pop()
            stack[-1].append(item)
        elif name == "STOP":
            result = stack.pop()
            break
        else:
            raise ValueError(f"unsupported pickle opcode {name}")
    if not isinstance(result, list):
        raise ValueError("top-level object is not a list")
    out = []
    for item in result:
        if not isinstance(item, _ArrayStub) or item.array is None:
            raise ValueError("list element is not an ndarray")
        out.append(item.array)
    return out


def main(labels=LABELS):
    os.makedirs(OUT_DIR, exist_ok=True)
    for label in labels:
        arrays = read_weight_list(os.path.join(REF_WEIGHTS, f"{label}_weights"))
        payload = {f"w{i:03d}": a.astype(np.float32) for i, a in enumerate(arrays)}
        payload["count"] = np.array(len(arrays), dtype=np.int64)
        out = os.path.join(OUT_DIR, f"{label}.npz")
        np.savez_compressed(out, **payload)
        nparams = sum(a.size for a in arrays)
        print(f"{label}: {len(arrays)} arrays, {nparams} params -> {os.path.relpath(out)}")


if __name__ == "__main__":
    main(sys.argv[1:] or LABELS)
