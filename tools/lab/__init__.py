"""ctypes loader of the probe library `tools/lab/libfem355_lab.so` (declared in `tools/lab/fem355_lab.h`).

Probe and layout-experiment kernels only; the product library `libfem355.so` does not contain them. Built on
demand by `make -C tools/lab` (after the product library)."""
import ctypes
import os
import subprocess

import fem355  # noqa: F401  (loads libfem355.so first: the probe library resolves its error plumbing there)
from fem355 import _capi as C

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libfem355_lab.so")

_P, _I, _L = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
SIGNATURES = {
    "fem_lab_copy": (_I, [_I, _I, _P, _P, _L, _I, _P]),
    "fem_lab_sell_pair": (_I, [_L, _P, _P, _P, _P, _P, _P]),
    "fem_lab_spmv16_pair": (_I, [_I, _I, _L, _P, _P, _P, _P, _P, _P]),
    "fem_lab_sell3_layout": (_I, [_I, _L, _P, _P, _P, _P, _P, _P]),
    "fem_lab_spmv_persist": (_I, [_I, _I, _I, _L, _L, _P, _P, _P, _P, _P, _P]),
    "fem_lab_spmv3": (_I, [_I, _I, _I, _I, _L, _P, _P, _P, _P, _P, _P]),
    "fem_lab_sell_uniform": (_I, [_L, _P, _P, _P, _P, _P, _P, _P, _P]),
    "fem_lab_spmv_persist_uni": (_I, [_I, _L, _L, _P, _P, _P, _P, _P, _P, _P, _P]),
    "fem_lab_spmv_gather": (_I, [_I, _I, _L, _L, _P, _P, _P, _P, _P, _P, _P]),
    "fem_lab_spmv_sym": (_I, [_I, _L, _L, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
}
_lab = None


def load():
    global _lab
    if _lab is None:
        C.load_library()
        if not os.path.exists(LIB_PATH):
            subprocess.run(["make", "-C", HERE], check=True)
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _lab = lib
    return _lab
