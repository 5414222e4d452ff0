"""ctypes binding of the fem355 C-ABI (`include/fem355.h`, built into `lib/libfem355.so`).

There is no CPU fallback: every compute entry point of the package goes through this library on a HIP device,
and `lib()` raises if the library or the device is missing. `torch` is imported first on purpose: it loads the
HIP runtime (libamdhip64.so.7) that the library then binds to by SONAME, so torch tensors' device pointers and
streams are valid in both.
"""
from __future__ import annotations

import atexit
import ctypes
import functools
import inspect
import os
import threading

import torch

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FEM355_LIB", os.path.join(PKG_DIR, "lib", "libfem355.so"))

FEM_OK, FEM_EBADTYPE, FEM_ESINGULAR, FEM_EHIP, FEM_ERCCL, FEM_EARG, FEM_ESTATE = range(7)
(PCG_RUNNING, PCG_CONVERGED, PCG_MAXITER, PCG_BREAKDOWN, PCG_ALPHA_NAN, PCG_BETA_NAN, PCG_SYNC_TIMEOUT,
 PCG_BAD_WINDOW) = range(8)
MODE_CG_STABLE, MODE_PCG, MODE_CG_CONSTRAINED = 0, 1, 2
# include/fem355.h FEM_TUNE_*: the library's default set for a new context, and the merged-update flag
TUNE_UPD1 = 1024
TUNE_U2_HOLD, TUNE_U2_SMALL = 2048, 4096   # test-only knobs of the merged update (include/fem355.h)
TUNE_MF_GATHER = 8192   # element-chunk operator: q summed by a gather launch instead of inside the merged update
TUNE_PK_GV = 16384      # persistent schedule, small bs = 1 systems: the pipelined (Ghysels-Vanroose) iteration
TUNE_DEFAULT = 1 | 2 | 4 | 8 | 128 | TUNE_UPD1
KIND_ELASTIC, KIND_POISSON, KIND_MASS = 0, 1, 2
ISO_SUM, ISO_STACK, ISO_VOLUME, ISO_MASS = 0, 1, 2, 3

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_D = ctypes.c_double

# name -> (restype, argtypes)
SIGNATURES = {
    "fem_last_error": (ctypes.c_char_p, []),
    "fem_version": (_I, []),
    "fem_tet4_ke": (_I, [_P, _P, _L, _D, _D, _I, _P, _P, _P]),
    "fem_tet4_geom": (_I, [_P, _P, _L, _P, _P, _P, _P, _P]),
    "fem_iso_ke": (_I, [_P, _P, _L, _I, _D, _D, _P, _P, _I, _I, _P, _P]),
    "fem_iso_geom": (_I, [_P, _P, _L, _I, _P, _P, _P, _P, _P]),
    "fem_ke_sym_stride": (_I, [_I]),
    "fem_iso_ke_sym": (_I, [_P, _P, _L, _I, _D, _D, _P, _P, _I, _I, _P, _P]),
    "fem_assemble_from_ke_sym": (_I, [_P, _P, _I, _P, _P, _L, _P, _P, _P, _I, _I, _I, _P, _P]),
    "fem_assemble_from_ke_mass_sl": (_I, [_P, _P, _P, _I, _P, _P, _L, _P, _P, _P, _I, _I, _P, _P, _P]),
    "fem_iso_mass": (_I, [_P, _P, _L, _I, _D, _P, _P, _P, _I, _P, _P]),
    "fem_iso_mass_scalar": (_I, [_P, _P, _L, _I, _D, _P, _P, _P, _I, _P, _P]),
    "fem_pcg_scalars": (_I, [_P, ctypes.POINTER(_D)]),
    "fem_scan_work_len": (_L, [_L]),
    "fem_incidence_work_bytes": (_L, [_L, _L]),
    "fem_incidence": (_I, [_P, _L, _I, _L, _P, _P, _P, _P]),
    "fem_incidence_checked": (_I, [_P, _L, _I, _L, _P, _P, _P, _P, _P]),
    "fem_rcm_work_len": (_L, [_L]),
    "fem_rcm": (_I, [_P, _P, _L, _P, _P, _P, _P, _P]),
    "fem_graph_count": (_I, [_P, _I, _P, _P, _L, _P, _P, _P]),
    "fem_graph_fill": (_I, [_P, _I, _P, _P, _L, _P, _P, _P, _P]),
    "fem_graph_tmp_len": (_L, [_L]),
    "fem_graph_count2": (_I, [_P, _I, _P, _P, _L, _P, _P, _P, _P]),
    "fem_graph_fill2": (_I, [_P, _I, _P, _P, _L, _P, _P, _P, _P, _P]),
    "fem_graph_sell_fill": (_I, [_P, _I, _P, _P, _L, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "fem_graph_sell_fill_sl": (_I, [_P, _I, _P, _P, _L, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P, _P, _P]),
    "fem_scan_i32": (_I, [_P, _L, _P, _P, _P]),
    "fem_scan_i64": (_I, [_P, _L, _P, _P, _P]),
    "fem_sell_widths": (_I, [_P, _L, _P, _P]),
    "fem_graph_sizes": (_I, [_P, _P, _P, _L, _P, _P, _P, _P]),
    "fem_sell_fill": (_I, [_P, _P, _L, _P, _P, _P, _P]),
    "fem_sell_csr2sell": (_I, [_P, _L, _P, _P, _P]),
    "fem_assemble_from_ke": (_I, [_P, _P, _I, _I, _P, _P, _L, _P, _P, _P, _P, _P, _P]),
    "fem_assemble_from_ke_ex": (_I, [_P, _P, _I, _I, _P, _P, _L, _P, _P, _P, _P, _L, _L, _I, _P, _P]),
    "fem_assemble_from_ke_ex2": (_I, [_P, _P, _I, _I, _P, _P, _L, _P, _P, _P, _P, _L, _L, _I, _I, _P, _P]),
    "fem_assemble_tet4": (_I, [_P, _P, _D, _D, _I, _P, _P, _L, _P, _P, _P, _P, _P, _P, _P]),
    "fem_assemble_tet4_ex": (_I, [_P, _P, _D, _D, _I, _P, _P, _L, _P, _P, _P, _P, _I, _P, _P, _P]),
    "fem_assemble_tet4_ex2": (_I, [_P, _P, _D, _D, _I, _P, _P, _L, _P, _P, _P, _P, _I, _I, _P, _P, _P]),
    "fem_sell_to_csr_vals": (_I, [_P, _I, _P, _L, _P, _P, _P, _P]),
    "fem_jacobi": (_I, [_P, _I, _P, _P, _P, _P, _L, _P, _P, _P]),
    "fem_ebe_apply": (_I, [_P, _P, _I, _I, _P, _P, _L, _P, _P, _P]),
    "fem_ebe_diag": (_I, [_P, _P, _I, _I, _P, _P, _L, _I, _P, _P]),
    "fem_invert_diag": (_I, [_P, _L, _P, _P]),
    "fem_tet4_stress": (_I, [_P, _P, _L, _P, _D, _D, _P, _P, _P, _P]),
    "fem_iso_stress": (_I, [_P, _P, _L, _I, _P, _D, _D, _P, _P, _I, _I, _P, _P, _P]),
    "fem_voigt_to_tensor": (_I, [_P, _L, _P, _P]),
    "fem_von_mises": (_I, [_P, _L, _P, _P]),
    "fem_node_average": (_I, [_P, _I, _P, _P, _L, _P, _P]),
    "fem_face_forces": (_I, [_P, _P, _L, _I, _P, _P]),
    "fem_shared_face_sum": (_I, [_P, _P, _I, _L, _P, _P]),
    "fem_topo_create": (_I, [_P, _L, _I, _P, _I, _I, _L, _P, ctypes.POINTER(_P)]),
    "fem_topo_counts": (_I, [_P, ctypes.POINTER(_L), ctypes.POINTER(_L), ctypes.POINTER(_L)]),
    "fem_topo_pairs": (_I, [_P, _P]),
    "fem_topo_unique": (_I, [_P, _P]),
    "fem_topo_boundary": (_I, [_P, _P, _I, _P, _P, _P, _P, _P, ctypes.POINTER(_L)]),
    "fem_topo_destroy": (None, [_P]),
    "fem_sub_elements": (_I, [_P, _L, _I, _P, _I, _I, _P, _P]),
    "fem_element_face_normals": (_I, [_P, _P, _L, _I, _P, _P, _P, _P, _I, _D, _I, _I, _P, _P]),
    "fem_surface_normals": (_I, [_P, _P, _P, _L, _I, _I, _P, _P]),
    "fem_solid_ke": (_I, [_I, _P, _P, _L, _D, _D, _P, _P, _I, _I, _P, _P]),
    "fem_csr_pattern": (_I, [_P, _L, _I, _I, _L, _P, _P, _P, ctypes.POINTER(_L), _P]),
    "fem_csr_fill": (_I, [_P, _P, _L, _I, _I, _L, _P, _P, _P, _P]),
    "fem_spmv_csr": (_I, [_P, _P, _P, _P, _P, _L, _P]),
    "fem_pcg_csr": (_I, [_P, _P, _P, _L, _P, _P, _P, _P, _D, _I, _D, _I, ctypes.POINTER(_I), ctypes.POINTER(_I), _P,
                         _P]),
    "fem_vtk_read": (_I, [ctypes.c_char_p, ctypes.POINTER(_P)]),
    "fem_vtk_sizes": (_I, [_P, ctypes.POINTER(_L), ctypes.POINTER(_L), ctypes.POINTER(_L), ctypes.POINTER(_L)]),
    "fem_vtk_copy": (_I, [_P, _P, _P, _P]),
    "fem_vtk_free": (None, [_P]),
    "fem_spmv": (_I, [_L, _I, _P, _P, _P, _P, _P, _P]),
    "fem_sell_delta16": (_I, [_P, _L, _P, _P, _P, _P]),
    "fem_spmv16": (_I, [_L, _I, _P, _P, _P, _P, _P, _P]),
    "fem_pcg_set_cols16": (_I, [_P, _P]),
    "fem_pcg_set_tuning": (_I, [_P, _I]),
    "fem_stream_copy": (_I, [_P, _P, _L, _I, _P]),
    "fem_stream_read": (_I, [_P, _P, _L, _I, _P]),
    "fem_pcg_create": (_I, [_L, _I, _P, _P, _P, _P, _P, _P, _I, _D, _D, _P, _L, _P, ctypes.POINTER(_P)]),
    "fem_pcg_start": (_I, [_P]),
    "fem_pcg_iterate": (_I, [_P, _I]),
    "fem_pcg_poll": (_I, [_P, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_D)]),
    "fem_pcg_sync_site": (_I, [_P, ctypes.POINTER(_I)]),
    "fem_pcg_debug_window": (_I, [_P, _I, _I, _I]),
    "fem_pcg_solve": (_I, [_P, _I, _I, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_D)]),
    "fem_pcg_use_graph": (_I, [_P, _I]),
    "fem_pcg_set_schedule": (_I, [_P, _I]),
    "fem_pcg_set_entries": (_I, [_P, _L]),
    "fem_pcg_get_schedule": (_I, [_P]),
    "fem_pcg_uniform_slices": (_I, [_P, _L, _L, _P, _P, _P]),
    "fem_pcg_persist_build": (_I, [_P, ctypes.POINTER(_I), ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "fem_pcg_pipelined": (_I, [_P, ctypes.POINTER(_I)]),
    "fem_sell_sl_pattern": (_I, [_L, _P, _P, _I, _P, _P, _P, _P, _P]),
    "fem_assemble_tet4_sl": (_I, [_P, _P, _D, _D, _I, _P, _P, _L, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P]),
    "fem_assemble_from_ke_sl": (_I, [_P, _P, _I, _P, _P, _L, _P, _P, _P, _I, _I, _P, _P]),
    "fem_jacobi_sl": (_I, [_P, _I, _P, _P, _P, _P, _P, _L, _P, _P, _P]),
    "fem_spmv_sl": (_I, [_L, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "fem_sell_sl_unpair": (_I, [_L, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "fem_pcg_set_layout": (_I, [_P, _P, _P, _P, _P, _P, _I]),
    "fem_pcg_persist_profile": (_I, [_P, _I, _P, ctypes.POINTER(_I)]),
    "fem_pcg_set_constraints": (_I, [_P, _I, _L, _P, _P, _L, _P, _P, _L, _P, _P, _P, _P, _P]),
    "fem_enforce_constraints": (_I, [_P, _P, _L, _I, _L, _P, _P, _L, _P, _P, _L, _P, _P, _P, _P, _P, _P]),
    "fem_pcg_finish": (_I, [_P]),
    "fem_pcg_profile": (_I, [_P, _I, _I, ctypes.POINTER(_D), ctypes.POINTER(_I)]),
    "fem_pcg_destroy": (None, [_P]),
    "fem_pcg_release_cache": (_I, []),
    "fem_release_scratch": (_I, []),
    "fem_pcg_set_rows": (_I, [_P, _I, _I, _P, _I]),
    "fem_pcg_comm_block": (_I, [_P, ctypes.POINTER(_P), ctypes.POINTER(_L)]),
    "fem_pcg_col_window": (_I, [_P, ctypes.POINTER(_L), ctypes.POINTER(_L)]),
    "fem_pcg_set_peers": (_I, [_P, _P, _P, _P]),
    "fem_pcg_dist_debug": (_I, [_P, _I, _P, _L]),
    "fem_stream_create_cu": (_I, [_I, _I, ctypes.POINTER(_P)]),
    "fem_stream_destroy": (_I, [_P]),
    "fem_pcg_set_prof": (_I, [_P, _P]),
    "fem_ipc_handle": (_I, [_P, ctypes.c_char_p]),
    "fem_ipc_open": (_I, [ctypes.c_char_p, ctypes.POINTER(_P)]),
    "fem_ipc_close": (_I, [_P]),
    "fem_sell_diag": (_I, [_P, _I, _P, _P, _L, _P, _P]),
    "fem_jacobi_from_diag": (_I, [_P, _L, _P, _P, _P]),
    "fem_mf_create": (_I, [_P, _P, _L, _L, _I, _D, _D, ctypes.POINTER(_L), _P, ctypes.POINTER(_P)]),
    "fem_mf_destroy": (_I, [_P]),
    "fem_mf_apply": (_I, [_P, _P, _P, _P]),
    "fem_mf_diag": (_I, [_P, _P, _P]),
    "fem_mf_info": (_I, [_P, ctypes.POINTER(_L)]),
    "fem_mf_spcheck": (_I, [_P]),
    "fem_mf_order": (_I, [_P, _P, _P, _P, _P, _P]),
    "fem_pcg_set_operator_mf": (_I, [_P, _P]),
    "fem_comm_unique_id": (_I, [ctypes.c_char_p]),
    "fem_comm_init": (_I, [_I, _I, ctypes.c_char_p, ctypes.POINTER(_P)]),
    "fem_comm_destroy": (_I, [_P]),
    "fem_allreduce_sum": (_I, [_P, _P, _L, _P]),
    "fem_halo_sum": (_I, [_P, _P, _I, _P, _L, _P, _L, _P, _P]),
    "fem_halo_pack": (_I, [_P, _I, _P, _L, _P, _P]),
    "fem_halo_unpack": (_I, [_P, _I, _P, _L, _P, _P]),
    "fem_pcg_set_dist": (_I, [_P, _I, _P, _L, _P, _P, _P]),
    "fem_pcg_set_dist_variant": (_I, [_P, _I]),
    "fem_pcg_set_p2p": (_I, [_P, _I, _I, _P, _P, _P, _P]),
    "fem_pcg_p2p_buffers": (_I, [_P, ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_L)]),
    "fem_p2p_deliver": (_I, [_P, _I, _P]),
    "fem_pcg_dist_phase": (_I, [_P, _I]),
    "fem_pcg_dist_buffer": (_I, [_P, _I, ctypes.POINTER(_P), ctypes.POINTER(_L)]),
    "fem_group_allreduce": (_I, [_P, _I, _L, _P]),
}

_lib = None
_lock = threading.Lock()


class FemError(RuntimeError):
    pass


def load_library(path: str = LIB_PATH):
    """Load the shared library and bind every symbol of SIGNATURES (no device needed)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise FemError(f"fem355: HIP library not built: {path} (run `python -c 'import __graft_entry__ as g; g.build()'`)")
            lib = ctypes.CDLL(path)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def lib():
    """The library, on a HIP device. Raises when there is no GPU: the package has no CPU path."""
    if not torch.cuda.is_available():
        raise FemError("fem355 requires a HIP (MI355X) device; none is visible. There is no CPU fallback.")
    return load_library()


def check(rc: int, what: str = ""):
    if rc == FEM_OK:
        return
    msg = (_lib.fem_last_error() or b"").decode(errors="replace") if _lib else ""
    if rc == FEM_EBADTYPE:
        raise ValueError(f"{what}: {msg}")
    if rc == FEM_ESINGULAR:
        raise ValueError("Singular matrix encountered while computing B matrix.")
    raise FemError(f"fem355 {what} failed (code {rc}): {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL). A host tensor is refused here: its address handed to a kernel
    would be a memory fault (XNACK off), not an exception."""
    if t is None:
        return None
    if not t.is_cuda:
        raise FemError(f"fem355: a {t.device} tensor was passed where device memory is required")
    return ctypes.c_void_p(t.data_ptr())


def stream(dev=None):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def compute_device(device=None) -> torch.device:
    """The HIP device the work runs on: `device` itself when it is a cuda device, else the current one."""
    if device is not None:
        d = torch.device(device)
        if d.type == "cuda":
            return d if d.index is not None else torch.device("cuda", torch.cuda.current_device())
    return torch.device("cuda", torch.cuda.current_device())


def device_scope(dev):
    """Context that makes `dev` the current HIP device for the calls inside it: the library allocates its
    workspace on, and launches on the null stream of, the CURRENT device, so every public entry point runs its
    C calls inside the scope of the device its tensors live on."""
    d = torch.device(dev)
    if d.type != "cuda" or d.index is None or d.index == torch.cuda.current_device():
        return _NULL_SCOPE
    return torch.cuda.device(d)


class _NullScope:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NULL_SCOPE = _NullScope()


def on_device(fn):
    """Decorator for the reference-named public functions: run `fn` with the current HIP device set to the one
    its `device` argument names (`device="cuda:1"` with current device 0 must not launch on GPU 0)."""
    sig = inspect.signature(fn)
    if "device" not in sig.parameters:
        return fn
    default = sig.parameters["device"].default

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        if not torch.cuda.is_available():
            return fn(*args, **kwargs)
        dev = kwargs.get("device", default)
        if "device" not in kwargs:
            try:
                dev = sig.bind_partial(*args, **kwargs).arguments.get("device", default)
            except TypeError:
                return fn(*args, **kwargs)   # let the call itself raise the reference's TypeError
        try:
            d = compute_device(dev)
        except Exception:
            return fn(*args, **kwargs)
        with device_scope(d):
            return fn(*args, **kwargs)

    return wrapper


def scope_module(namespace: dict):
    """Wrap every public function with a `device` parameter defined in `namespace` (a module's globals())."""
    mod = namespace.get("__name__")
    for name, obj in list(namespace.items()):
        if name.startswith("_") or not inspect.isfunction(obj) or obj.__module__ != mod:
            continue
        namespace[name] = on_device(obj)


def release_cache() -> int:
    """Free the solver buffers the library keeps for reuse (MB released), and its per-stream scratch."""
    if _lib is None:
        return 0
    mb = int(_lib.fem_pcg_release_cache())
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        _lib.fem_release_scratch()
    return mb


atexit.register(release_cache)
