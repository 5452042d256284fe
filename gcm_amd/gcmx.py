"""ctypes binding of the gcmx C-ABI (``include/gcmx.h``).

This is the Python side of the drop-in boundary: a thin, typed wrapper around
``gcm_amd/lib/libgcmx.so``.  There is no fallback: if the HIP library is
missing or no GPU is present, construction fails loudly.
"""
from __future__ import annotations

import ctypes
import weakref
import os
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libgcmx.so")
# Tuning experiments only (scripts/tune.sh): load an alternative build.
if os.environ.get("GCMX_LIB"):
    LIB_PATH = os.path.abspath(os.environ["GCMX_LIB"])

# include/gcmx.h
GCMX_OK = 0
STATUS_NAMES = {0: "GCMX_OK", 1: "GCMX_ERR_INVALID_ARG", 2: "GCMX_ERR_CFL", 3: "GCMX_ERR_HIP",
                4: "GCMX_ERR_OOM", 5: "GCMX_ERR_STATE", 6: "GCMX_ERR_UNSUPPORTED",
                7: "GCMX_ERR_COMM"}
PATH_AUTO, PATH_GENERIC, PATH_SPLIT, PATH_FUSED = 0, 1, 2, 3
PATH_NAMES = {0: "auto", 1: "generic", 2: "split", 3: "fused"}
SCHED_AUTO, SCHED_SINGLE, SCHED_XSLAB, SCHED_BFIRST = 0, 1, 2, 3
FP_FMA, FP_EXACT = 0, 1
UNIQUE_ID_BYTES = 128
MAX_BORDER_Q = 16
QUANTITY_CODES = {"Vx": 2, "Vy": 3, "Vz": 4, "Sxx": 5, "Sxy": 6, "Sxz": 7, "Syy": 8, "Syz": 9,
                  "Szz": 10, "PRESSURE": 12}

# Exported symbols, in header order (checked by tests/test_abi.py).
SYMBOLS = [
    "gcmx_abi_version", "gcmx_last_error", "gcmx_pde_size", "gcmx_status_string",
    "gcmx_create", "gcmx_destroy", "gcmx_set_materials", "gcmx_set_material_ids",
    "gcmx_upload", "gcmx_download", "gcmx_fill_random", "gcmx_stage", "gcmx_step",
    "gcmx_set_kernel_path", "gcmx_set_step_schedule", "gcmx_set_fp_mode", "gcmx_get_fp_mode", "gcmx_effective_path", "gcmx_last_step_path",
    "gcmx_border_fill",
    "gcmx_border_nodes_create", "gcmx_border_apply", "gcmx_border_nodes_destroy", "gcmx_step_faces",
    "gcmx_face_map_create", "gcmx_face_map_destroy", "gcmx_step_face_map",
    "gcmx_copy_box",
    "gcmx_ode_maxwell", "gcmx_step_ode", "gcmx_last_ode_fused",
    "gcmx_comm_unique_id", "gcmx_comm_init_opts", "gcmx_comm_init", "gcmx_comm_channels_per_peer",
    "gcmx_comm_channels_rule", "gcmx_comm_posted_calls", "gcmx_comm_test_stall", "gcmx_halo_exchange", "gcmx_halo_exchange_group",
    "gcmx_comm_init_local", "gcmx_local_group_steps", "gcmx_comm_init_loopback",
    "gcmx_sync", "gcmx_stream",
    "gcmx_profile_enable", "gcmx_profile_reset", "gcmx_profile_read", "gcmx_profile_kernel",
    "gcmx_inner_nodes",
    "gcmx_all_nodes", "gcmx_device_bytes", "gcmx_copy_ceiling", "gcmx_layer_info", "gcmx_geometry",
    "gcmx_clock_probe_start", "gcmx_clock_probe_read",
    "gsx_create", "gsx_destroy", "gsx_set_matrices", "gsx_set_gradient_plan",
    "gsx_set_stage_plan", "gsx_set_border_plan", "gsx_set_border_values",
    "gsx_plain_correction", "gsx_upload", "gsx_download", "gsx_stage", "gsx_sync",
    "gsx_stage_nodes", "gsx_stage_finish", "gsx_contact_create", "gsx_contact_destroy",
    "gsx_contact_plain", "gsx_contact_correct", "gsx_step", "gsx_set_node_lanes",
    "gsx_set_stage_fusion", "gsx_last_stage_fused", "gsx_launch_count", "gsx_stage_plan_info",
    "gsx_set_wait_budget",
    "gsx_test_interpolate",
]


class GcmxError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class Face(ctypes.Structure):
    """gcmx_face: one face's uniform cubic border condition."""
    _fields_ = [("enabled", ctypes.c_int), ("n_quantities", ctypes.c_int),
                ("quantities", ctypes.c_int * MAX_BORDER_Q),
                ("values", ctypes.c_double * MAX_BORDER_Q)]


class CommOptions(ctypes.Structure):
    """gcmx_comm_options."""
    _fields_ = [("global_x", ctypes.c_int), ("channels_per_peer", ctypes.c_int),
                ("min_ctas", ctypes.c_int), ("max_ctas", ctypes.c_int), ("timeout_s", ctypes.c_double)]


class GridDesc(ctypes.Structure):
    _fields_ = [("dim", ctypes.c_int), ("border_size", ctypes.c_int),
                ("sizes", ctypes.c_int * 3), ("start", ctypes.c_int * 3),
                ("h", ctypes.c_double * 3)]


_lib = None


def lib() -> ctypes.CDLL:
    """Load libgcmx.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run __graft_entry__.build() "
                          "(make -C gcm_amd/csrc)")
    L = ctypes.CDLL(LIB_PATH)
    dp = ctypes.POINTER(ctypes.c_double)
    ip = ctypes.POINTER(ctypes.c_int)
    vp = ctypes.c_void_p
    st = ctypes.c_int
    L.gcmx_abi_version.restype = ctypes.c_int
    L.gcmx_last_error.restype = ctypes.c_char_p
    L.gcmx_pde_size.argtypes = [ctypes.c_int]
    L.gcmx_status_string.argtypes = [st]
    L.gcmx_status_string.restype = ctypes.c_char_p
    L.gcmx_create.argtypes = [ctypes.POINTER(GridDesc), ctypes.c_int, ctypes.POINTER(vp)]
    L.gcmx_create.restype = st
    L.gcmx_destroy.argtypes = [vp]
    L.gcmx_destroy.restype = None
    L.gcmx_set_materials.argtypes = [vp, ctypes.c_int, dp, dp, dp]
    L.gcmx_set_material_ids.argtypes = [vp, ctypes.POINTER(ctypes.c_uint8)]
    L.gcmx_upload.argtypes = [vp, dp]
    L.gcmx_download.argtypes = [vp, dp]
    L.gcmx_fill_random.argtypes = [vp, ip, ctypes.c_uint64]
    L.gcmx_stage.argtypes = [vp, ctypes.c_int, ctypes.c_double]
    L.gcmx_step.argtypes = [vp, ctypes.c_double]
    L.gcmx_set_kernel_path.argtypes = [vp, ctypes.c_int]
    L.gcmx_set_step_schedule.argtypes = [vp, ctypes.c_int, ctypes.c_int]
    L.gcmx_set_fp_mode.argtypes = [vp, ctypes.c_int]
    L.gcmx_get_fp_mode.argtypes = [vp, ip]
    L.gcmx_effective_path.argtypes = [vp]
    L.gcmx_last_step_path.argtypes = [vp]
    L.gcmx_border_fill.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ip, ctypes.c_int,
                                   ip, dp]
    L.gcmx_border_nodes_create.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ip,
                                           ctypes.POINTER(vp)]
    L.gcmx_border_apply.argtypes = [vp, vp, ctypes.c_int, ip, dp]
    L.gcmx_border_nodes_destroy.argtypes = [vp]
    L.gcmx_border_nodes_destroy.restype = None
    L.gcmx_step_faces.argtypes = [vp, ctypes.c_double, ctypes.POINTER(Face)]
    L.gcmx_face_map_create.argtypes = [vp, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(vp)]
    L.gcmx_face_map_destroy.argtypes = [vp]
    L.gcmx_face_map_destroy.restype = None
    L.gcmx_step_face_map.argtypes = [vp, ctypes.c_double, vp, ctypes.c_int, ctypes.POINTER(Face)]
    L.gcmx_copy_box.argtypes = [vp, ip, ip, vp, ip]
    L.gcmx_ode_maxwell.argtypes = [vp, ctypes.c_double, dp, ctypes.c_int]
    L.gcmx_step_ode.argtypes = [vp, ctypes.c_double, ctypes.POINTER(Face), dp, ctypes.c_int]
    L.gcmx_last_ode_fused.argtypes = [vp]
    L.gcmx_comm_unique_id.argtypes = [ctypes.POINTER(ctypes.c_uint8)]
    L.gcmx_comm_init.argtypes = [vp, ctypes.POINTER(ctypes.c_uint8), ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int]
    L.gcmx_comm_init_opts.argtypes = [vp, ctypes.POINTER(ctypes.c_uint8), ctypes.c_int, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int, ctypes.POINTER(CommOptions)]
    L.gcmx_comm_channels_per_peer.argtypes = [vp]
    L.gcmx_comm_channels_per_peer.restype = ctypes.c_int
    # (ABI additions of round 5: bound when present, so that A/B timing runs can
    # load an older build; tests/test_abi.py checks this build exports them)
    if hasattr(L, "gcmx_comm_channels_rule"):
        L.gcmx_comm_channels_rule.argtypes = [ctypes.c_int] * 8
        L.gcmx_comm_channels_rule.restype = ctypes.c_int
        L.gcmx_comm_posted_calls.argtypes = [vp]
        L.gcmx_comm_posted_calls.restype = ctypes.c_longlong
    L.gcmx_comm_test_stall.argtypes = [vp, ctypes.c_int]
    L.gcmx_halo_exchange.argtypes = [vp]
    L.gcmx_halo_exchange_group.argtypes = [ctypes.POINTER(vp), ctypes.c_int]
    L.gcmx_comm_init_local.argtypes = [ctypes.POINTER(vp), ctypes.c_int]
    L.gcmx_comm_init_loopback.argtypes = [vp, ctypes.c_double, ctypes.c_int]
    L.gcmx_local_group_steps.argtypes = [ctypes.POINTER(vp), ctypes.c_int, ctypes.c_double, ctypes.c_int]
    L.gcmx_sync.argtypes = [vp]
    L.gcmx_stream.argtypes = [vp]
    L.gcmx_stream.restype = vp
    L.gcmx_profile_enable.argtypes = [vp, ctypes.c_int]
    L.gcmx_profile_reset.argtypes = [vp]
    L.gcmx_profile_read.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), dp,
                                    ctypes.POINTER(ctypes.c_longlong), dp]
    L.gcmx_profile_read.restype = ctypes.c_int
    L.gcmx_profile_kernel.argtypes = [vp, ctypes.c_int]
    L.gcmx_profile_kernel.restype = ctypes.c_char_p
    L.gcmx_inner_nodes.argtypes = [vp]
    L.gcmx_inner_nodes.restype = ctypes.c_longlong
    L.gcmx_all_nodes.argtypes = [vp]
    L.gcmx_all_nodes.restype = ctypes.c_longlong
    L.gcmx_device_bytes.argtypes = [vp]
    L.gcmx_device_bytes.restype = ctypes.c_size_t
    L.gcmx_copy_ceiling.argtypes = [vp, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
    L.gcmx_copy_ceiling.restype = ctypes.c_int
    L.gsx_test_interpolate.argtypes = [ctypes.c_int, ctypes.c_int, dp, dp, dp, dp, dp, dp]
    u64p = ctypes.POINTER(ctypes.c_uint64)
    L.gcmx_layer_info.argtypes = [vp, u64p]
    L.gcmx_geometry.argtypes = [vp, ctypes.POINTER(ctypes.c_int64)]
    L.gcmx_clock_probe_start.argtypes = [vp, ctypes.c_double, ctypes.c_double]
    L.gcmx_clock_probe_read.argtypes = [vp, u64p, ctypes.c_int]
    L.gcmx_clock_probe_read.restype = ctypes.c_int
    _lib = L
    return L


def _check(status: int):
    if status != GCMX_OK:
        raise GcmxError(status, lib().gcmx_last_error().decode())


def _dp(a: np.ndarray):
    if a.dtype != np.float64 or not a.flags["C_CONTIGUOUS"]:
        raise TypeError("expected a C-contiguous float64 array")
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _ip(seq) -> ctypes.Array:
    seq = list(seq)
    return (ctypes.c_int * max(1, len(seq)))(*seq)


def pde_size(dim: int) -> int:
    return dim + dim * (dim + 1) // 2


class Context:
    """One body (or one X-slab of a body) resident on one GPU."""

    def __init__(self, dim: int, border_size: int, sizes: Sequence[int],
                 start: Optional[Sequence[int]] = None, h: Optional[Sequence[float]] = None,
                 device: int = 0):
        start = list(start) if start is not None else [0] * dim
        h = list(h) if h is not None else [1.0] * dim
        self.dim, self.bs, self.M = dim, border_size, pde_size(dim)
        self.sizes = list(sizes)[:dim]
        self.start = start[:dim]
        self.h = h[:dim]
        d = GridDesc(dim, border_size, (ctypes.c_int * 3)(*(self.sizes + [1] * (3 - dim))),
                     (ctypes.c_int * 3)(*(self.start + [0] * (3 - dim))),
                     (ctypes.c_double * 3)(*(list(self.h) + [0.0] * (3 - dim))))
        self._ptr = ctypes.c_void_p()
        _check(lib().gcmx_create(ctypes.byref(d), device, ctypes.byref(self._ptr)))
        self.shape_all = tuple(s + 2 * border_size for s in self.sizes)
        self.n_all = int(np.prod(self.shape_all))

    def _adopt(self, child):
        """FaceMap / BorderNodes of this context: closed before the context is
        (their native destroy reads the context's device and stream)."""
        if not hasattr(self, "_children"):
            self._children = weakref.WeakSet()
        self._children.add(child)

    def close(self):
        for ch in list(getattr(self, "_children", ())):
            ch.close()
        if getattr(self, "_ptr", None) and self._ptr.value:
            lib().gcmx_destroy(self._ptr)
            self._ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ptr(self):
        return self._ptr

    # -- set-up -----------------------------------------------------------
    def set_materials(self, U: np.ndarray, U1: np.ndarray, L: np.ndarray):
        """U/U1: [n_mat, dim, M, M], L: [n_mat, dim, M] (GcmMatrices per material)."""
        U = np.ascontiguousarray(U, dtype=np.float64)
        U1 = np.ascontiguousarray(U1, dtype=np.float64)
        L = np.ascontiguousarray(L, dtype=np.float64)
        n = U.shape[0]
        assert U.shape == (n, self.dim, self.M, self.M) and U1.shape == U.shape
        assert L.shape == (n, self.dim, self.M)
        _check(lib().gcmx_set_materials(self._ptr, n, _dp(U), _dp(U1), _dp(L)))

    def set_material_ids(self, ids_all: Optional[np.ndarray]):
        if ids_all is None:
            _check(lib().gcmx_set_material_ids(self._ptr, None))
            return
        ids = np.ascontiguousarray(ids_all, dtype=np.uint8).reshape(-1)
        assert ids.size == self.n_all
        _check(lib().gcmx_set_material_ids(self._ptr, ids.ctypes.data_as(
            ctypes.POINTER(ctypes.c_uint8))))

    def upload(self, aos: np.ndarray):
        a = np.ascontiguousarray(aos, dtype=np.float64).reshape(-1)
        assert a.size == self.n_all * self.M
        _check(lib().gcmx_upload(self._ptr, _dp(a)))

    def download(self) -> np.ndarray:
        out = np.empty((self.n_all, self.M))
        _check(lib().gcmx_download(self._ptr, _dp(out)))
        return out

    def fill_random(self, global_sizes: Sequence[int], seed: int):
        gs = list(global_sizes) + [1] * (3 - len(global_sizes))
        _check(lib().gcmx_fill_random(self._ptr, _ip(gs), seed))

    # -- hot path ---------------------------------------------------------
    def stage(self, axis: int, tau: float):
        _check(lib().gcmx_stage(self._ptr, axis, tau))

    def step(self, tau: float):
        _check(lib().gcmx_step(self._ptr, tau))

    def set_path(self, path: int):
        _check(lib().gcmx_set_kernel_path(self._ptr, path))

    def set_schedule(self, sched: int, rows_per_block: int = 0):
        """gcmx_set_step_schedule: SCHED_AUTO / SCHED_SINGLE / SCHED_XSLAB / SCHED_BFIRST."""
        _check(lib().gcmx_set_step_schedule(self._ptr, sched, rows_per_block))

    @property
    def fp_mode(self) -> int:
        """gcmx_get_fp_mode: FP_FMA (default) or FP_EXACT."""
        m = ctypes.c_int(0)
        _check(lib().gcmx_get_fp_mode(self._ptr, ctypes.byref(m)))
        return m.value

    @fp_mode.setter
    def fp_mode(self, mode: int):
        """gcmx_set_fp_mode: the one-pass step's floating-point build."""
        _check(lib().gcmx_set_fp_mode(self._ptr, mode))

    @property
    def effective_path(self) -> str:
        return PATH_NAMES[lib().gcmx_effective_path(self._ptr)]

    @property
    def last_path(self) -> str:
        """The path the last step / stage ran (gcmx_last_step_path)."""
        return PATH_NAMES[lib().gcmx_last_step_path(self._ptr)]

    def border_fill(self, axis: int, side: int, nodes: np.ndarray, quantities: Sequence[int],
                    values: Sequence[float]):
        nodes = np.ascontiguousarray(nodes, dtype=np.int32).reshape(-1, self.dim)
        q = _ip(quantities)
        v = (ctypes.c_double * max(1, len(values)))(*values)
        _check(lib().gcmx_border_fill(self._ptr, axis, side, nodes.shape[0],
                                      nodes.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                      len(quantities), q, v))

    def border_nodes(self, axis: int, side: int, nodes: np.ndarray) -> "BorderNodes":
        """gcmx_border_nodes_create: a device-resident face-node list."""
        return BorderNodes(self, axis, side, nodes)

    def border_apply(self, handle: "BorderNodes", quantities: Sequence[int], values: Sequence[float]):
        q = _ip(quantities)
        v = (ctypes.c_double * max(1, len(values)))(*values)
        _check(lib().gcmx_border_apply(self._ptr, handle.ptr, len(quantities), q, v))

    def _faces(self, faces):
        arr = (Face * (2 * self.dim))()
        for f, lst in enumerate(faces[:2 * self.dim]):
            if lst is None:
                continue
            arr[f].enabled = 1
            arr[f].n_quantities = len(lst)
            for k, (q, v) in enumerate(lst):
                arr[f].quantities[k] = q
                arr[f].values[k] = v
        return arr

    def step_faces(self, tau: float, faces: Sequence[Optional[Sequence[tuple]]]):
        """gcmx_step_faces: faces[2*axis + (side > 0)] is None (no condition) or a
        list of (quantity code, value) in the reference's application order."""
        _check(lib().gcmx_step_faces(self._ptr, tau, self._faces(faces)))

    def face_map(self, node_condition: Sequence[Optional[np.ndarray]]) -> "FaceMap":
        """gcmx_face_map_create: per face (2*axis + (side > 0)) None or one uint8
        per face node (other axes increasing, last fastest): condition index or
        255 (GCMX_NO_FACE_CONDITION)."""
        return FaceMap(self, node_condition)

    def step_face_map(self, tau: float, fmap: "FaceMap", conditions: Sequence[Sequence[tuple]]):
        """gcmx_step_face_map: conditions[k] = [(quantity code, value), ...] at Clock::Time()."""
        arr = (Face * max(1, len(conditions)))()
        for k, lst in enumerate(conditions):
            arr[k].enabled = 1
            arr[k].n_quantities = len(lst)
            for i, (q, v) in enumerate(lst):
                arr[k].quantities[i] = q
                arr[k].values[i] = v
        _check(lib().gcmx_step_face_map(self._ptr, tau, fmap.ptr, len(conditions), arr))

    def step_ode(self, tau: float, tau0: Sequence[float], faces=None):
        """gcmx_step_ode: the step (gcmx_step, or gcmx_step_faces with `faces`) then
        MaxwellViscosityOde, folded into the one-pass step's stores where it can be."""
        t0 = np.ascontiguousarray(tau0, dtype=np.float64).reshape(-1)
        arr = self._faces(faces) if faces is not None else None
        _check(lib().gcmx_step_ode(self._ptr, tau, arr, _dp(t0), t0.shape[0]))

    @property
    def last_ode_fused(self) -> bool:
        return bool(lib().gcmx_last_ode_fused(self._ptr))

    def copy_box(self, dst_min, dst_max, src: "Context", src_min):
        pad = lambda s: list(s) + [0] * (3 - len(s))
        _check(lib().gcmx_copy_box(self._ptr, _ip(pad(dst_min)), _ip(pad(dst_max)), src._ptr,
                                   _ip(pad(src_min))))

    def ode_maxwell(self, tau: float, tau0: Sequence[float]):
        """MaxwellViscosityOde::apply: sigma *= exp(-tau / tau0[material])."""
        t0 = np.ascontiguousarray(tau0, dtype=np.float64).reshape(-1)
        _check(lib().gcmx_ode_maxwell(self._ptr, tau, _dp(t0), t0.shape[0]))

    def comm_init(self, unique_id: bytes, nranks: int, rank: int, left: int, right: int,
                  global_x: Optional[int] = None, channels_per_peer: int = -1, timeout_s: float = 0.0):
        """gcmx_comm_init / gcmx_comm_init_opts (non-blocking RCCL communicator;
        global_x = the whole grid's X extent, equal on every rank, for the
        rank-consistent automatic channels-per-peer rule)."""
        buf = (ctypes.c_uint8 * UNIQUE_ID_BYTES)(*unique_id)
        if global_x is None and channels_per_peer == -1 and timeout_s == 0:
            _check(lib().gcmx_comm_init(self._ptr, buf, nranks, rank, left, right))
            return
        o = CommOptions(int(global_x or 0), int(channels_per_peer), -1, -1, float(timeout_s))
        _check(lib().gcmx_comm_init_opts(self._ptr, buf, nranks, rank, left, right, ctypes.byref(o)))

    @property
    def comm_channels_per_peer(self) -> int:
        return lib().gcmx_comm_channels_per_peer(self._ptr)

    @property
    def comm_posted_calls(self) -> int:
        """ncclSend + ncclRecv calls the exchange groups posted (gcmx_comm_posted_calls)."""
        return lib().gcmx_comm_posted_calls(self._ptr)

    def comm_test_stall(self, on: bool = True):
        """Tests only: exchange groups post sends but never receives."""
        _check(lib().gcmx_comm_test_stall(self._ptr, 1 if on else 0))

    def comm_init_loopback(self, gbps_per_direction: float = 64.0, blocks: int = 8):
        """gcmx_comm_init_loopback: x-periodic self-exchange through the RCCL
        post / wait points, held for the bytes' time at the given link rate."""
        _check(lib().gcmx_comm_init_loopback(self._ptr, gbps_per_direction, blocks))

    def halo_exchange(self):
        _check(lib().gcmx_halo_exchange(self._ptr))

    def copy_ceiling_ms(self, nbytes: int, reps: int = 5) -> float:
        """Median duration (ms) of a flat device copy moving `nbytes` (half read,
        half written) on this context's device (gcmx_copy_ceiling)."""
        ms = ctypes.c_float(0.0)
        _check(lib().gcmx_copy_ceiling(self._ptr, int(nbytes), int(reps), ctypes.byref(ms)))
        return float(ms.value)

    def geometry(self) -> dict:
        """gcmx_geometry: the device layout's element strides (tests)."""
        out = (ctypes.c_int64 * 6)()
        _check(lib().gcmx_geometry(self._ptr, out))
        return {"stride": [int(out[0]), int(out[1]), int(out[2])], "cs": int(out[3]),
                "origin": int(out[4]), "row": int(out[5])}

    def layer_info(self) -> dict:
        """gcmx_layer_info: the two time layers' device addresses (measurement)."""
        out = (ctypes.c_uint64 * 4)()
        _check(lib().gcmx_layer_info(self._ptr, out))
        k = int(out[3])
        alloc = {0: "two hipMalloc", 1: "one hipMalloc", 2: "one contiguous block"}.get(
            k, f"shuffled {k >> 20} MiB chunks")
        return {"a": int(out[0]), "b": int(out[1]), "layer_bytes": int(out[2]),
                "one_allocation": k != 0, "alloc": alloc}

    def clock_probe_start(self, seconds: float, period_us: float = 200.0):
        """gcmx_clock_probe_start: one co-resident wave samples the shader clock."""
        _check(lib().gcmx_clock_probe_start(self._ptr, float(seconds), float(period_us)))

    def clock_probe_read(self, cap: int = 65536) -> np.ndarray:
        """(n, 2) array of (100 MHz ticks, shader cycles) samples."""
        buf = np.zeros(2 * cap, dtype=np.uint64)
        n = lib().gcmx_clock_probe_read(self._ptr, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), cap)
        if n < 0:
            raise GcmxError(3, "clock probe read failed")
        return buf[:2 * min(n, cap)].reshape(-1, 2)

    def sync(self):
        _check(lib().gcmx_sync(self._ptr))

    @property
    def stream(self) -> int:
        return lib().gcmx_stream(self._ptr) or 0

    # -- timing -----------------------------------------------------------
    def profile(self, enable: bool = True):
        _check(lib().gcmx_profile_enable(self._ptr, 1 if enable else 0))

    def profile_reset(self):
        _check(lib().gcmx_profile_reset(self._ptr))

    def profile_read(self) -> dict:
        n = lib().gcmx_profile_read(self._ptr, -1, None, None, None, None)
        out = {}
        for i in range(n):
            name = ctypes.c_char_p(); tot = ctypes.c_double(); cnt = ctypes.c_longlong()
            byt = ctypes.c_double()
            lib().gcmx_profile_read(self._ptr, i, ctypes.byref(name), ctypes.byref(tot),
                                    ctypes.byref(cnt), ctypes.byref(byt))
            kern = lib().gcmx_profile_kernel(self._ptr, i) or b""
            out[name.value.decode()] = {"total_ms": tot.value, "launches": cnt.value,
                                        "bytes_per_launch": byt.value, "kernel": kern.decode()}
        return out

    @property
    def inner_nodes(self) -> int:
        return lib().gcmx_inner_nodes(self._ptr)

    @property
    def device_bytes(self) -> int:
        return lib().gcmx_device_bytes(self._ptr)


class FaceMap:
    """gcmx_face_map: per-node face conditions, uploaded once."""

    def __init__(self, ctx: "Context", node_condition):
        self._ctx = ctx  # keeps the context alive
        self._maps = [None if m is None else np.ascontiguousarray(m, dtype=np.uint8).reshape(-1)
                      for m in list(node_condition) + [None] * (6 - len(node_condition))]
        ptrs = (ctypes.c_void_p * 6)(*[None if m is None else m.ctypes.data for m in self._maps])
        self.ptr = ctypes.c_void_p()
        _check(lib().gcmx_face_map_create(ctx.ptr, ptrs, ctypes.byref(self.ptr)))
        ctx._adopt(self)

    def close(self):
        # the native destroy reads the context: after Context.close (which closes
        # its children first) there is nothing left to free here
        if self.ptr and self.ptr.value and self._ctx.ptr.value:
            lib().gcmx_face_map_destroy(self.ptr)
        self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BorderNodes:
    """gcmx_border_nodes: face nodes uploaded once, applied without host sync."""

    def __init__(self, ctx: Context, axis: int, side: int, nodes: np.ndarray):
        nodes = np.ascontiguousarray(nodes, dtype=np.int32).reshape(-1, ctx.dim)
        self.ptr = ctypes.c_void_p()
        self._ctx = ctx  # keeps the context alive
        _check(lib().gcmx_border_nodes_create(ctx.ptr, axis, side, nodes.shape[0],
                                              nodes.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
                                              ctypes.byref(self.ptr)))
        ctx._adopt(self)

    def close(self):
        if self.ptr and self.ptr.value and self._ctx.ptr.value:
            lib().gcmx_border_nodes_destroy(self.ptr)
        self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def halo_exchange_group(slabs: Sequence["Context"]):
    """Refresh X ghosts of in-process X slabs (ordered by increasing X)."""
    arr = (ctypes.c_void_p * len(slabs))(*[c.ptr.value for c in slabs])
    _check(lib().gcmx_halo_exchange_group(arr, len(slabs)))


def comm_init_local(slabs: Sequence["Context"]):
    """Make `slabs` (ordered by increasing X) the ranks of one in-process group:
    the RCCL X-slab exchange with device copies (gcmx_comm_init_local).  Drive
    them concurrently: local_group_steps, or one thread per context."""
    arr = (ctypes.c_void_p * len(slabs))(*[c.ptr.value for c in slabs])
    _check(lib().gcmx_comm_init_local(arr, len(slabs)))


def local_group_steps(slabs: Sequence["Context"], tau: float, steps: int):
    """`steps` gcmx_step calls on every context of an in-process group, one host
    thread per context, then gcmx_sync (gcmx_local_group_steps)."""
    arr = (ctypes.c_void_p * len(slabs))(*[c.ptr.value for c in slabs])
    _check(lib().gcmx_local_group_steps(arr, len(slabs), float(tau), int(steps)))


def test_interpolate(v, g, c, q, lam, device: int = 0):
    """gsx_test_interpolate (tests only): the simplex kernels' device interpolation
    on given cases; returns (hybrid, linear) arrays."""
    v = np.ascontiguousarray(v, dtype=np.float64).reshape(-1, 4)
    n = v.shape[0]
    g = np.ascontiguousarray(g, dtype=np.float64).reshape(n, 4, 3)
    c = np.ascontiguousarray(c, dtype=np.float64).reshape(n, 4, 3)
    q = np.ascontiguousarray(q, dtype=np.float64).reshape(n, 3)
    lam = np.ascontiguousarray(lam, dtype=np.float64).reshape(n, 4)
    out = np.zeros((n, 2), dtype=np.float64)
    _check(lib().gsx_test_interpolate(device, n, _dp(v), _dp(g), _dp(c), _dp(q), _dp(lam), _dp(out)))
    return out[:, 0].copy(), out[:, 1].copy()


def channels_rule(global_x: int, nranks: int, local_x: int, Y: int, Z: int, bs: int = 2,
                  rows_per_block: int = 0, cus: int = 256) -> int:
    """gcmx_comm_channels_rule: the automatic RCCL channels per peer (pure; no GPU
    call for cus > 0)."""
    return lib().gcmx_comm_channels_rule(int(global_x), int(nranks), int(local_x), int(Y), int(Z),
                                         int(bs), int(rows_per_block), int(cus))


def unique_id() -> bytes:
    buf = (ctypes.c_uint8 * UNIQUE_ID_BYTES)()
    _check(lib().gcmx_comm_unique_id(buf))
    return bytes(buf)
