"""ctypes binding of libmaxcover.so (include/maxcover.h).

This is the Python stand-in for the Julia ``ccall`` shim (julia/MaxCoverAMD.jl): same entry
points, same array layouts, same error behaviour. There is no CPU fallback: if the shared
library is missing or cannot be loaded, every entry point raises ``MaxCoverError``.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MAXCOVER_LIB") or os.path.join(_HERE, "libmaxcover.so")

MAC_OK = 0
MAC_E_INVAL = 1
MAC_E_SIZE = 2
MAC_E_NOPOINTS = 3
MAC_E_HIP = 4
MAC_E_NOMEM = 5
MAC_E_LOSSY = 6
MAC_E_NODEVICE = 7

MAC_OPT_ALGO = 1
MAC_OPT_STORAGE = 2
MAC_OPT_TILE_POINTS = 3
MAC_OPT_PROFILE = 4
MAC_OPT_SHARED = 5
MAC_OPT_CHAIN = 6
SHARED_MODES = {"auto": 0, "fp64": 1, "bits": 2}
CHAINS = {"auto": 0, "five": 1, "fused": 2}
MAC_ALGO_AUTO = 0
MAC_ALGO_SCAN = 1
MAC_ALGO_TILED = 2
MAC_ALGO_POLL = 3
MAC_STORE_F64 = 0
MAC_STORE_F32 = 1

# mac_profile_kernels launch roles (include/maxcover.h MAC_PROF_ROLES). Role 5 is one stamp slot
# for the crowded-poll shared-entry pass: the union pass (shared_or_kernel) on equal weights — every
# reference data set — else the bit-word kernel (shared_bits_kernel)
PROF_ROLES = ("prep_kernel",  # (role 0: the prep launch, prep_kernel or prep_x_kernel)
              "disk_index_kernel", "walk_setup_kernel", "coverage_tiled_poll_kernel",
              "coverage_poll_kernel", "shared_or_kernel", "finalize_kernel", "fiw_kernel",
              "fin2_kernel")

ALGOS = {"auto": MAC_ALGO_AUTO, "scan": MAC_ALGO_SCAN, "tiled": MAC_ALGO_TILED,
         "poll": MAC_ALGO_POLL}

# Every symbol include/maxcover.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "mac_last_error", "mac_version", "mac_device_count", "mac_ctx_create", "mac_ctx_destroy",
    "mac_set_option", "mac_set_points_f64", "mac_set_points_records_f64",
    "mac_set_points_dev_f64", "mac_num_points", "mac_get_points_f64",
    "mac_remove_covered_f64", "mac_covered_flags_f64", "mac_area_f64", "mac_area_batch_f64",
    "mac_objective_batch_f64", "mac_poll_best_f64", "mac_area_batch_dev_f64",
    "mac_poll_best_dev_f64", "mac_best_fetch", "mac_poll_arm_dev_f64", "mac_poll_fire",
    "mac_cover_threshold", "mac_profile_read",
    "mac_profile_split", "mac_profile_kernels",
    "mac_append_points_f64", "mac_append_points_dev_f64", "mac_mads_run",
    "mac_fire_last_error", "mac_fire_thresholds", "mac_fire_create", "mac_fire_destroy",
    "mac_fire_initial_points", "mac_fire_step", "mac_fire_last_points", "mac_fire_get_grid",
    "mac_fire_set_grid",
    "mac_set_points_f32", "mac_set_points_dev_f32", "mac_area_f32", "mac_area_batch_f32",
    "mac_poll_best_f32", "mac_poll_best_dev_f32",
    "mac_mads_begin", "mac_mads_poll", "mac_mads_update", "mac_mads_result", "mac_mads_destroy",
    "mac_mads_poll_ahead", "mac_mads_advance",
    "mac_mads_best_buffer", "mac_best_reduce_dev", "mac_poll_basis_f64",
    "mac_comm_unique_id", "mac_comm_init", "mac_poll_exchange", "mac_exchange_records",
)


class MadsParams(ctypes.Structure):
    """mac_mads_params (include/maxcover.h)."""
    _fields_ = [("n_iter", ctypes.c_int64), ("ell0", ctypes.c_int32), ("ell_max", ctypes.c_int32),
                ("seed", ctypes.c_uint64)]


class MadsStats(ctypes.Structure):
    """mac_mads_stats (include/maxcover.h)."""
    _fields_ = [("f", ctypes.c_double), ("iterations", ctypes.c_int64),
                ("evaluations", ctypes.c_int64), ("status", ctypes.c_int32),
                ("feasible", ctypes.c_int32), ("seconds", ctypes.c_double),
                ("host_enqueue_s", ctypes.c_double), ("host_perm_s", ctypes.c_double),
                ("wait_s", ctypes.c_double), ("host_post_s", ctypes.c_double),
                ("feasible_evaluations", ctypes.c_int64), ("rejected_polls", ctypes.c_int64),
                ("successes", ctypes.c_int64), ("slot_fallbacks", ctypes.c_int64)]


class FireParams(ctypes.Structure):
    """mac_fire_params (include/maxcover.h)."""
    _fields_ = [("nx", ctypes.c_int64), ("ny", ctypes.c_int64), ("dx", ctypes.c_double),
                ("dy", ctypes.c_double), ("forest_density", ctypes.c_double),
                ("prob_spread", ctypes.c_double), ("wind_speed", ctypes.c_double),
                ("wind_direction", ctypes.c_double), ("ix0", ctypes.c_int64),
                ("ix1", ctypes.c_int64), ("iy0", ctypes.c_int64), ("iy1", ctypes.c_int64),
                ("seed", ctypes.c_uint64)]


class MaxCoverError(RuntimeError):
    """Non-zero status from libmaxcover (message from mac_last_error)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"libmaxcover error {code}: {msg}")
        self.code = code


class InexactError(MaxCoverError, ValueError):
    """Julia's InexactError from Int(length(circles)/3) (src/AreaCoverageCalculation.jl:65)."""


_dp = ctypes.POINTER(ctypes.c_double)
_fp = ctypes.POINTER(ctypes.c_float)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64

_lib = None
_lib_lock = threading.Lock()


def _declare(L: ctypes.CDLL) -> None:
    sig = {
        "mac_last_error": ([], ctypes.c_char_p),
        "mac_version": ([], ctypes.c_char_p),
        "mac_device_count": ([ctypes.POINTER(_i32)], _i32),
        "mac_ctx_create": ([ctypes.POINTER(_vp), _i32], _i32),
        "mac_ctx_destroy": ([_vp], None),
        "mac_set_option": ([_vp, _i32, _i64], _i32),
        "mac_set_points_f64": ([_vp, _dp, _dp, _dp, _i64], _i32),
        "mac_set_points_records_f64": ([_vp, _dp, _i64, _i64], _i32),
        "mac_set_points_dev_f64": ([_vp, _vp, _vp, _vp, _i64], _i32),
        "mac_num_points": ([_vp, _i64p], _i32),
        "mac_get_points_f64": ([_vp, _dp, _dp, _dp], _i32),
        "mac_remove_covered_f64": ([_vp, _dp, _i64, _i64p, _i64p], _i32),
        "mac_covered_flags_f64": ([_vp, _dp, _i64, _u8p], _i32),
        "mac_area_f64": ([_vp, _dp, _i64, _dp], _i32),
        "mac_area_batch_f64": ([_vp, _dp, _i64, _i64, _dp], _i32),
        "mac_objective_batch_f64": ([_vp, _dp, _i64, _i64, _dp, ctypes.c_double, _dp], _i32),
        "mac_poll_best_f64": ([_vp, _dp, _i64, _i64, _dp, ctypes.c_double, _dp, _dp,
                               ctypes.c_double, _dp, _dp, _i64p], _i32),
        "mac_area_batch_dev_f64": ([_vp, _vp, _i64, _i64, _vp, _vp], _i32),
        "mac_poll_best_dev_f64": ([_vp, _vp, _i64, _i64, _vp, ctypes.c_double, _vp, _vp,
                                   ctypes.c_double, _i64, _vp, _vp, _vp], _i32),
        "mac_best_fetch": ([_vp, _vp, _vp, _dp, _i64p], _i32),
        "mac_best_reduce_dev": ([_vp, _vp, _i32, _vp, _vp], _i32),
        "mac_comm_unique_id": ([ctypes.c_char_p, _vp], _i32),
        "mac_comm_init": ([_vp, ctypes.c_char_p, _vp, _i32, _i32], _i32),
        "mac_poll_exchange": ([_vp, _vp, _vp, _vp, _dp, _i64p], _i32),
        "mac_exchange_records": ([_vp, _vp, _i32, _vp, _vp], _i32),
        "mac_poll_basis_f64": ([_vp, _dp, _i64, ctypes.POINTER(ctypes.c_int16),
                                ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                ctypes.c_double, _dp, ctypes.c_double, _dp, _dp, ctypes.c_double,
                                _dp, _dp, _i64p], _i32),
        "mac_poll_arm_dev_f64": ([_vp, _vp, _i64, _i64, _vp, ctypes.c_double, _vp, _vp,
                                  ctypes.c_double, _i64, _vp, _vp, _vp,
                                  ctypes.POINTER(ctypes.c_uint64)], _i32),
        "mac_poll_fire": ([_vp, ctypes.c_uint64], _i32),
        "mac_cover_threshold": ([ctypes.c_double], ctypes.c_double),
        "mac_profile_read": ([_vp, _dp, _i64p, _i64p, ctypes.POINTER(_i32), _i32], _i32),
        "mac_profile_split": ([_vp, _dp, _dp, _dp, _i64p], _i32),
        "mac_profile_kernels": ([_vp, _dp, _i64p, _i32], _i32),
        "mac_append_points_f64": ([_vp, _dp, _dp, _dp, _i64], _i32),
        "mac_mads_run": ([_vp, _dp, _i64, _dp, ctypes.c_double, _dp, _dp, ctypes.c_double,
                          ctypes.POINTER(MadsParams), _dp, ctypes.POINTER(MadsStats)], _i32),
        "mac_append_points_dev_f64": ([_vp, _vp, _vp, _vp, _i64], _i32),
        "mac_fire_last_error": ([], ctypes.c_char_p),
        "mac_fire_thresholds": ([ctypes.POINTER(FireParams), _dp], None),
        "mac_fire_create": ([ctypes.POINTER(_vp), _i32, ctypes.POINTER(FireParams)], _i32),
        "mac_fire_destroy": ([_vp], None),
        "mac_fire_initial_points": ([_vp, _dp, _i64, _i64p], _i32),
        "mac_fire_step": ([_vp, _vp, _i64p], _i32),
        "mac_fire_last_points": ([_vp, _dp, _i64, _i64p], _i32),
        "mac_fire_get_grid": ([_vp, _u8p], _i32),
        "mac_fire_set_grid": ([_vp, _u8p], _i32),
        "mac_mads_begin": ([_vp, _dp, _i64, _dp, ctypes.c_double, _dp, _dp, ctypes.c_double,
                            ctypes.POINTER(MadsParams), _i64, _i64, ctypes.POINTER(_vp)], _i32),
        "mac_mads_poll": ([_vp, ctypes.POINTER(_i32), _dp, _i64p], _i32),
        "mac_mads_update": ([_vp, ctypes.c_double, _i64], _i32),
        "mac_mads_poll_ahead": ([_vp, _i32, ctypes.POINTER(_i32), _dp, _i64p, _i64p], _i32),
        "mac_mads_advance": ([_vp, ctypes.c_double, _i64, ctypes.POINTER(_i32)], _i32),
        "mac_mads_result": ([_vp, _dp, ctypes.POINTER(MadsStats)], _i32),
        "mac_mads_destroy": ([_vp], None),
        "mac_mads_best_buffer": ([_vp, _vp], _i32),
        "mac_set_points_f32": ([_vp, _fp, _fp, _fp, _i64], _i32),
        "mac_set_points_dev_f32": ([_vp, _vp, _vp, _vp, _i64], _i32),
        "mac_area_f32": ([_vp, _fp, _i64, _dp], _i32),
        "mac_area_batch_f32": ([_vp, _fp, _i64, _i64, _dp], _i32),
        "mac_poll_best_f32": ([_vp, _fp, _i64, _i64, _dp, ctypes.c_double, _fp, _dp,
                               ctypes.c_double, _dp, _dp, _i64p], _i32),
        "mac_poll_best_dev_f32": ([_vp, _vp, _i64, _i64, _vp, ctypes.c_double, _vp, _vp,
                                   ctypes.c_double, _i64, _vp, _vp, _vp], _i32),
    }
    for name, (args, res) in sig.items():
        # (an older build lacks the newer symbols: bound as far as it has them, so A/B tools can
        # load it; tests/test_abi.py checks that the in-tree library exports every one)
        f = getattr(L, name, None)
        if f is None:
            continue
        f.argtypes = args
        f.restype = res


_loaded_before_torch = False


def _one_hip_runtime() -> None:
    """PyTorch-ROCm ships its own HIP and HSA runtimes, which its libraries load by file name. If
    libmaxcover.so (NEEDED libamdhip64.so.7) is loaded first, it binds the system runtime and a
    later torch import loads a second one in the same process, whose device initialisation fails
    ("No HIP GPUs are available"; measured on the MI355X box). With torch loaded first, libmaxcover
    shares torch's runtime: one context for torch tensors, streams, RCCL and the library.

    So a process that uses both must import torch first. The library does not
    import torch itself — a CPU-only user does not pay for it, and which runtime binds does not
    depend silently on whether torch is importable — unless MAXCOVER_TORCH_FIRST=1 asks for it.
    Whether torch was already loaded is recorded: `check_one_runtime` (called by dist.py before
    its device collectives) fails loudly instead of letting two runtimes meet."""
    global _loaded_before_torch
    import sys
    if "torch" not in sys.modules and os.environ.get("MAXCOVER_TORCH_FIRST") == "1":
        import torch  # noqa: F401
    _loaded_before_torch = "torch" not in sys.modules


def check_one_runtime() -> None:
    """Raise if libmaxcover was loaded before torch in this process (two HIP runtimes: torch's
    device work and the library's would not share a context; see _one_hip_runtime)."""
    if _lib is not None and _loaded_before_torch:
        raise MaxCoverError(MAC_E_HIP, "libmaxcover was loaded before torch: import torch before the "
                            "first libmaxcover call (one HIP runtime per process, INTEGRATION.md)")


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load libmaxcover.so (raises MaxCoverError if absent: there is no fallback path)."""
    global _lib
    with _lib_lock:
        if _lib is not None and path is None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise MaxCoverError(MAC_E_HIP, f"{p} not built (run __graft_entry__.build())")
        _one_hip_runtime()
        try:
            L = ctypes.CDLL(p)
        except OSError as e:  # pragma: no cover - depends on the host
            raise MaxCoverError(MAC_E_HIP, f"cannot load {p}: {e}") from e
        _declare(L)
        if path is None:
            _lib = L
        return L


def _check(rc: int) -> None:
    if rc != MAC_OK:
        msg = load_library().mac_last_error().decode(errors="replace")
        if rc == MAC_E_SIZE:
            raise InexactError(rc, msg)
        raise MaxCoverError(rc, msg)


def version() -> str:
    return load_library().mac_version().decode()


def device_count() -> int:
    n = _i32()
    _check(load_library().mac_device_count(ctypes.byref(n)))
    return int(n.value)


def cover_threshold(r: float) -> float:
    return float(load_library().mac_cover_threshold(float(r)))


def _f64(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_dp)


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(_fp)


def _devptr(t) -> int:
    """Device address of a torch tensor / int / None."""
    if t is None:
        return 0
    if isinstance(t, int):
        return t
    return int(t.data_ptr())


def _stream(stream, device: int) -> int:
    """hipStream_t handle for a *_dev call. An int is a raw handle (0: HIP's null stream, the C
    ABI's NULL); a torch stream gives its handle; None follows torch's convention — the current
    torch stream of the context's device when this process has initialised torch's GPU side (so a
    poll is ordered after the torch ops that produced its inputs), else HIP's null stream."""
    if stream is None:
        import sys
        torch = sys.modules.get("torch")
        if torch is not None and torch.cuda.is_initialized():
            return int(torch.cuda.current_stream(device).cuda_stream)
        return 0
    if isinstance(stream, int):
        return stream
    return int(stream.cuda_stream)


class Context:
    """One libmaxcover context = one GPU + one device-resident fire-point list."""

    def __init__(self, device: int = 0, algo: str = "auto", tile_points: int | None = None):
        L = load_library()
        h = _vp()
        _check(L.mac_ctx_create(ctypes.byref(h), int(device)))
        self._h = h
        self.device = int(device)
        self._L = L
        self._steppers = weakref.WeakSet()   # closed before the context (they use its device state)
        self.set_algo(algo)
        if tile_points is not None:
            self.set_option(MAC_OPT_TILE_POINTS, int(tile_points))

    # -- lifetime
    def close(self) -> None:
        if getattr(self, "_h", None):
            for st in list(getattr(self, "_steppers", ())):
                st.close()
            self._L.mac_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- options
    def set_option(self, option: int, value: int) -> None:
        _check(self._L.mac_set_option(self._h, int(option), int(value)))

    def set_shared(self, mode: str) -> None:
        """How the poll walk decides the entries two disks' regions share (MAC_OPT_SHARED):
        "auto" (default), "fp64" (the poll kernel's jobs) or "bits" (the bit-word kernel)."""
        self.set_option(MAC_OPT_SHARED, SHARED_MODES[mode])

    def set_chain(self, chain: str) -> None:
        """The poll chain (MAC_OPT_CHAIN): "auto" (default: the fused three-launch chain unless the
        lane's recent polls were crowded, scattered or off the packed-key grid), "five" (prep, index,
        set-up, walk, finalize) or "fused" (prep, fiw, fin2 whenever it applies)."""
        self.set_option(MAC_OPT_CHAIN, CHAINS[chain])

    def set_algo(self, algo: str) -> None:
        if algo not in ALGOS:
            raise ValueError(f"algo must be one of {sorted(ALGOS)}")
        self.set_option(MAC_OPT_ALGO, ALGOS[algo])

    def profile(self, on: bool = True) -> None:
        self.set_option(MAC_OPT_PROFILE, 1 if on else 0)

    def profile_read(self, reset: bool = True):
        """(coverage-kernel ms summed over launches, launches, candidates evaluated, walk used
        by the last launch: 'scan' | 'tiled' | 'poll' | None)."""
        ms = ctypes.c_double()
        n = _i64()
        k = _i64()
        a = _i32()
        _check(self._L.mac_profile_read(self._h, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(k),
                                        ctypes.byref(a), 1 if reset else 0))
        name = {MAC_ALGO_SCAN: "scan", MAC_ALGO_TILED: "tiled", MAC_ALGO_POLL: "poll"}.get(a.value)
        return ms.value, int(n.value), int(k.value), name

    def profile_split(self):
        """Poll chains since the last reset: (prep ms, walk ms, after-walk ms, polls), summed.
        Call before profile_read(reset=True)."""
        p1, p2, gap = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        n = _i64()
        _check(self._L.mac_profile_split(self._h, ctypes.byref(p1), ctypes.byref(p2),
                                         ctypes.byref(gap), ctypes.byref(n)))
        return p1.value, p2.value, gap.value, int(n.value)

    def profile_kernels(self):
        """Poll chains since the last reset, per launch role (mac_profile_kernels): {kernel name:
        (summed launch spans in ms, launches)}. Call before profile_read(reset=True)."""
        n = len(PROF_ROLES)
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_int64 * n)()
        _check(self._L.mac_profile_kernels(self._h, ms, cnt, n))
        return {name: (ms[r], int(cnt[r])) for r, name in enumerate(PROF_ROLES)}

    # -- point list
    def set_points(self, x, y, w) -> None:
        x, y, w = _f64(x), _f64(y), _f64(w)
        if not (x.shape == y.shape == w.shape) or x.ndim != 1:
            raise ValueError("x, y, w must be 1-D arrays of equal length")
        _check(self._L.mac_set_points_f64(self._h, _ptr(x), _ptr(y), _ptr(w), x.size))

    def set_points_f32(self, x, y, w) -> None:
        """fp32 SoA arrays (mac_set_points_f32): widened exactly to the fp64 list."""
        x, y, w = _f32(x), _f32(y), _f32(w)
        if not (x.shape == y.shape == w.shape) or x.ndim != 1:
            raise ValueError("x, y, w must be 1-D arrays of equal length")
        _check(self._L.mac_set_points_f32(self._h, _fptr(x), _fptr(y), _fptr(w), x.size))

    def set_points_device_f32(self, x, y, w, M: int | None = None) -> None:
        """x, y, w: torch float32 tensors on this context's device (widened copies)."""
        n = int(M if M is not None else x.numel())
        _check(self._L.mac_set_points_dev_f32(self._h, _devptr(x), _devptr(y), _devptr(w), n))

    def set_points_records(self, rec) -> None:
        r = _f64(rec)
        if r.ndim == 1:
            r = r.reshape(-1, 5)
        if r.ndim != 2 or (r.shape[0] and r.shape[1] < 4):
            raise ValueError("records must be M x >=4 ([x, y, area, importance, covered])")
        _check(self._L.mac_set_points_records_f64(self._h, _ptr(r), r.shape[0],
                                                  r.shape[1] if r.shape[0] else 5))

    def set_points_device(self, x, y, w, M: int | None = None) -> None:
        """x, y, w: torch float64 tensors on this context's device (copied)."""
        n = int(M if M is not None else x.numel())
        _check(self._L.mac_set_points_dev_f64(self._h, _devptr(x), _devptr(y), _devptr(w), n))

    def append_points(self, x, y, w) -> None:
        """update_POI (src/CellFunctions.jl:59-79): entries appended at the end of the list."""
        x, y, w = _f64(x), _f64(y), _f64(w)
        if not (x.size == y.size == w.size):
            raise ValueError("x, y, w lengths differ")
        _check(self._L.mac_append_points_f64(self._h, _ptr(x), _ptr(y), _ptr(w), x.size))

    def append_points_device(self, x, y, w, m: int | None = None) -> None:
        m = int(x.numel() if m is None else m)
        _check(self._L.mac_append_points_dev_f64(self._h, _devptr(x), _devptr(y), _devptr(w), m))

    @property
    def num_points(self) -> int:
        m = _i64()
        _check(self._L.mac_num_points(self._h, ctypes.byref(m)))
        return int(m.value)

    def get_points(self):
        M = self.num_points
        x = np.empty(M)
        y = np.empty(M)
        w = np.empty(M)
        _check(self._L.mac_get_points_f64(self._h, _ptr(x), _ptr(y), _ptr(w)))
        return x, y, w

    def covered_flags(self, circles) -> np.ndarray:
        c = _f64(circles)
        out = np.zeros(max(self.num_points, 1), dtype=np.uint8)
        _check(self._L.mac_covered_flags_f64(self._h, _ptr(c), c.size,
                                             out.ctypes.data_as(_u8p)))
        return out[: self.num_points].astype(bool)

    def remove_covered(self, circles) -> np.ndarray:
        """rmvCoveredPOI on the device list; returns the kept original indices (list order)."""
        c = _f64(circles)
        M = self.num_points
        kept = np.zeros(max(M, 1), dtype=np.int64)
        m = _i64()
        _check(self._L.mac_remove_covered_f64(self._h, _ptr(c), c.size,
                                              kept.ctypes.data_as(_i64p), ctypes.byref(m)))
        return kept[: m.value].copy()

    # -- objective
    def area(self, circles) -> float:
        c = _f64(circles)
        out = ctypes.c_double()
        _check(self._L.mac_area_f64(self._h, _ptr(c), c.size, ctypes.byref(out)))
        return out.value

    def area_batch(self, cands) -> np.ndarray:
        """cands: K x 3N (row k = candidate k, i.e. the 3N x K column-major matrix)."""
        c = _f64(cands)
        if c.ndim != 2:
            raise ValueError("cands must be K x 3N")
        K, three_n = c.shape
        out = np.empty(K)
        _check(self._L.mac_area_batch_f64(self._h, _ptr(c), three_n, K, _ptr(out)))
        return out

    def objective_batch(self, cands, r_max, penalty: float = 1e5) -> np.ndarray:
        c = _f64(cands)
        K, three_n = c.shape
        rm = _f64(r_max)
        out = np.empty(K)
        _check(self._L.mac_objective_batch_f64(self._h, _ptr(c), three_n, K, _ptr(rm),
                                               float(penalty), _ptr(out)))
        return out

    def poll_best(self, cands, r_max, penalty: float = 1e5, prev=None, d_lim=None,
                  tan_half_fov: float = 1.0, want_all: bool = False):
        """Returns (best_obj, best_idx[, objectives]); best_idx = -1 if none feasible."""
        c = _f64(cands)
        K, three_n = c.shape
        rm = _f64(r_max)
        pv = _f64(prev) if prev is not None else None
        dl = _f64(d_lim) if d_lim is not None else None
        objs = np.empty(K) if want_all else None
        bo = ctypes.c_double()
        bi = _i64()
        _check(self._L.mac_poll_best_f64(
            self._h, _ptr(c), three_n, K, _ptr(rm), float(penalty),
            _ptr(pv) if pv is not None else None, _ptr(dl) if dl is not None else None,
            float(tan_half_fov), _ptr(objs) if objs is not None else None,
            ctypes.byref(bo), ctypes.byref(bi)))
        if want_all:
            return bo.value, int(bi.value), objs
        return bo.value, int(bi.value)

    def poll_basis(self, x_inc, L, rp, cp, delta: float, r_max, penalty: float = 1e5, prev=None,
                   d_lim=None, tan_half_fov: float = 1.0, want_all: bool = False):
        """mac_poll_basis_f64: the 2n-candidate poll x +- delta * B[:, k], B = L[rp][:, cp],
        expanded on the device. L: n x n lower-triangular integers (|L| < 2^15; its lower triangle
        is packed here) or the packed int16 triangle itself. Returns (best_obj, best_idx[, objs])."""
        x = _f64(x_inc)
        n = x.size
        Lp = np.asarray(L)
        if Lp.ndim == 2:
            if Lp.shape != (n, n):
                raise ValueError("L must be n x n")
            if np.abs(Lp).max(initial=0) > 32767:
                raise ValueError("|L| must fit int16")
            Lp = Lp[np.tril_indices(n)]
        tri = np.ascontiguousarray(Lp, dtype=np.int16)
        if tri.size != n * (n + 1) // 2:
            raise ValueError("packed L must hold n(n+1)/2 entries")
        r = np.ascontiguousarray(rp, dtype=np.int32)
        c = np.ascontiguousarray(cp, dtype=np.int32)
        if r.size != n or c.size != n:
            raise ValueError("rp / cp must hold n entries")
        rm = _f64(r_max)
        pv = _f64(prev) if prev is not None else None
        dl = _f64(d_lim) if d_lim is not None else None
        objs = np.empty(2 * n) if want_all else None
        bo = ctypes.c_double()
        bi = _i64()
        _check(self._L.mac_poll_basis_f64(
            self._h, _ptr(x), n, tri.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)),
            r.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), c.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
            float(delta), _ptr(rm), float(penalty), _ptr(pv) if pv is not None else None,
            _ptr(dl) if dl is not None else None, float(tan_half_fov),
            _ptr(objs) if objs is not None else None, ctypes.byref(bo), ctypes.byref(bi)))
        if want_all:
            return bo.value, int(bi.value), objs
        return bo.value, int(bi.value)

    # -- fp32 candidates (*_f32: widened exactly on the device, fp64 decisions)
    def area_f32(self, circles) -> float:
        c = _f32(circles)
        out = ctypes.c_double()
        _check(self._L.mac_area_f32(self._h, _fptr(c), c.size, ctypes.byref(out)))
        return out.value

    def area_batch_f32(self, cands) -> np.ndarray:
        c = _f32(cands)
        if c.ndim != 2:
            raise ValueError("cands must be K x 3N")
        K, three_n = c.shape
        out = np.empty(K)
        _check(self._L.mac_area_batch_f32(self._h, _fptr(c), three_n, K, _ptr(out)))
        return out

    def poll_best_f32(self, cands, r_max, penalty: float = 1e5, prev=None, d_lim=None,
                      tan_half_fov: float = 1.0, want_all: bool = False):
        c = _f32(cands)
        K, three_n = c.shape
        rm = _f64(r_max)
        pv = _f32(prev) if prev is not None else None
        dl = _f64(d_lim) if d_lim is not None else None
        objs = np.empty(K) if want_all else None
        bo = ctypes.c_double()
        bi = _i64()
        _check(self._L.mac_poll_best_f32(
            self._h, _fptr(c), three_n, K, _ptr(rm), float(penalty),
            _fptr(pv) if pv is not None else None, _ptr(dl) if dl is not None else None,
            float(tan_half_fov), _ptr(objs) if objs is not None else None,
            ctypes.byref(bo), ctypes.byref(bi)))
        if want_all:
            return bo.value, int(bi.value), objs
        return bo.value, int(bi.value)

    def poll_best_dev_f32(self, d_cands, three_n: int, K: int, d_rmax, d_best,
                          penalty: float = 1e5, d_prev=None, d_dlim=None, tan_half_fov: float = 1.0,
                          idx_base: int = 0, d_obj=None, stream=None) -> None:
        _check(self._L.mac_poll_best_dev_f32(
            self._h, _devptr(d_cands), int(three_n), int(K), _devptr(d_rmax), float(penalty),
            _devptr(d_prev), _devptr(d_dlim), float(tan_half_fov), int(idx_base),
            _devptr(d_obj), _devptr(d_best), _stream(stream, self.device)))

    # -- native MADS driver
    def mads_run(self, x0, r_max, penalty: float = 1e5, prev=None, d_lim=None,
                 tan_half_fov: float = 1.0, n_iter: int = 100, ell0: int = 2, ell_max: int = 6,
                 seed: int = 20250216):
        """mac_mads_run: the whole MADS loop in libmaxcover (candidates generated on the device).
        Returns (x, stats dict)."""
        x = _f64(x0)
        rm = _f64(r_max)
        pv = _f64(prev) if prev is not None else None
        dl = _f64(d_lim) if d_lim is not None else None
        out = np.empty_like(x)
        prm = MadsParams(int(n_iter), int(ell0), int(ell_max), int(seed) & (2**64 - 1))
        st = MadsStats()
        _check(self._L.mac_mads_run(self._h, _ptr(x), x.size, _ptr(rm), float(penalty),
                                    _ptr(pv) if pv is not None else None,
                                    _ptr(dl) if dl is not None else None, float(tan_half_fov),
                                    ctypes.byref(prm), _ptr(out), ctypes.byref(st)))
        return out, {k: getattr(st, k) for k, _ in MadsStats._fields_}

    def mads_stepper(self, x0, r_max, penalty: float = 1e5, prev=None, d_lim=None,
                     tan_half_fov: float = 1.0, n_iter: int = 100, ell0: int = 2,
                     ell_max: int = 6, seed: int = 20250216, shard=None) -> "MadsStepper":
        """mac_mads_begin: the native loop one poll at a time over the candidate shard
        ``shard`` = (lo, hi) of each poll's 2n candidates (None: the whole poll)."""
        st = MadsStepper(self, x0, r_max, penalty, prev, d_lim, tan_half_fov, n_iter, ell0,
                         ell_max, seed, shard)
        self._steppers.add(st)
        return st

    # -- device-resident, stream-ordered
    def area_batch_dev(self, d_cands, three_n: int, K: int, d_area, stream=None) -> None:
        _check(self._L.mac_area_batch_dev_f64(self._h, _devptr(d_cands), int(three_n), int(K),
                                              _devptr(d_area), _stream(stream, self.device)))

    def poll_best_dev(self, d_cands, three_n: int, K: int, d_rmax, d_best, penalty: float = 1e5,
                      d_prev=None, d_dlim=None, tan_half_fov: float = 1.0, idx_base: int = 0,
                      d_obj=None, stream=None) -> None:
        _check(self._L.mac_poll_best_dev_f64(
            self._h, _devptr(d_cands), int(three_n), int(K), _devptr(d_rmax), float(penalty),
            _devptr(d_prev), _devptr(d_dlim), float(tan_half_fov), int(idx_base),
            _devptr(d_obj), _devptr(d_best), _stream(stream, self.device)))

    def poll_step(self, d_cands, three_n: int, K: int, d_rmax, d_best, penalty: float = 1e5,
                  d_prev=None, d_dlim=None, tan_half_fov: float = 1.0, idx_base: int = 0,
                  d_obj=None, stream=None, fetch: bool = True):
        """A bound device poll: returns a zero-argument callable that enqueues the poll
        (mac_poll_best_dev_f64) and returns its (objective, index) (mac_best_fetch). The ctypes
        arguments are built once, so a step costs two foreign calls and nothing else on the
        host — the next poll of a MADS loop cannot start before this one's result is known."""
        h = _vp(self._h.value if isinstance(self._h, _vp) else self._h)
        poll_args = (h, _vp(_devptr(d_cands)), _i64(int(three_n)), _i64(int(K)),
                     _vp(_devptr(d_rmax)), ctypes.c_double(float(penalty)),
                     _vp(_devptr(d_prev)), _vp(_devptr(d_dlim)),
                     ctypes.c_double(float(tan_half_fov)), _i64(int(idx_base)),
                     _vp(_devptr(d_obj)), _vp(_devptr(d_best)), _vp(_stream(stream, self.device)))
        bo, bi = ctypes.c_double(), ctypes.c_int64()
        fetch_args = (h, _vp(_devptr(d_best)), _vp(_stream(stream, self.device)), ctypes.byref(bo),
                      ctypes.byref(bi))
        poll, fetch_f = self._L.mac_poll_best_dev_f64, self._L.mac_best_fetch

        def step():
            rc = poll(*poll_args)
            if rc != MAC_OK:
                _check(rc)
            rc = fetch_f(*fetch_args)
            if rc != MAC_OK:
                _check(rc)
            return bo.value, bi.value

        def enqueue():
            rc = poll(*poll_args)
            if rc != MAC_OK:
                _check(rc)

        return step if fetch else enqueue

    def poll_arm(self, d_cands, three_n: int, K: int, d_rmax, d_best, penalty: float = 1e5,
                 d_prev=None, d_dlim=None, tan_half_fov: float = 1.0, idx_base: int = 0,
                 d_obj=None, stream=None) -> int:
        """mac_poll_arm_dev_f64: the device poll enqueued behind the context's doorbell; returns
        its ticket (poll_fire releases it). See include/maxcover.h for the rules."""
        t = ctypes.c_uint64()
        _check(self._L.mac_poll_arm_dev_f64(
            self._h, _devptr(d_cands), int(three_n), int(K), _devptr(d_rmax), float(penalty),
            _devptr(d_prev), _devptr(d_dlim), float(tan_half_fov), int(idx_base),
            _devptr(d_obj), _devptr(d_best), _stream(stream, self.device), ctypes.byref(t)))
        return int(t.value)

    def poll_fire(self, ticket: int) -> None:
        _check(self._L.mac_poll_fire(self._h, int(ticket)))

    def armed_steps(self, polls, stream=None):
        """Bound armed polls for a loop of dependent polls: ``polls`` = a list of dicts of
        poll_best_dev arguments (d_cands, three_n, K, d_rmax, d_best, ...; consecutive polls on
        different d_best buffers). Returns (arm(j), fire(j), fetch(j)): arm enqueues poll j
        behind the doorbell, fire releases it, fetch returns its (objective, index) — with
        prebuilt ctypes arguments, so a loop step is fire(j), arm(j + 1) (enqueued while poll j
        runs), fetch(j)."""
        h = _vp(self._h.value if isinstance(self._h, _vp) else self._h)
        arm_f, fire_f, fetch_f = (self._L.mac_poll_arm_dev_f64, self._L.mac_poll_fire,
                                  self._L.mac_best_fetch)
        tickets = [ctypes.c_uint64() for _ in polls]
        bo, bi = ctypes.c_double(), ctypes.c_int64()
        sv = _vp(_stream(stream, self.device))
        arm_args, fetch_args = [], []
        for p, t in zip(polls, tickets):
            arm_args.append((h, _vp(_devptr(p["d_cands"])), _i64(int(p["three_n"])), _i64(int(p["K"])),
                             _vp(_devptr(p["d_rmax"])), ctypes.c_double(float(p.get("penalty", 1e5))),
                             _vp(_devptr(p.get("d_prev"))), _vp(_devptr(p.get("d_dlim"))),
                             ctypes.c_double(float(p.get("tan_half_fov", 1.0))),
                             _i64(int(p.get("idx_base", 0))), _vp(_devptr(p.get("d_obj"))),
                             _vp(_devptr(p["d_best"])), sv, ctypes.byref(t)))
            fetch_args.append((h, _vp(_devptr(p["d_best"])), sv, ctypes.byref(bo), ctypes.byref(bi)))

        def arm(j):
            rc = arm_f(*arm_args[j])
            if rc != MAC_OK:
                _check(rc)

        def fire(j):
            rc = fire_f(h, tickets[j].value)
            if rc != MAC_OK:
                _check(rc)

        def fetch(j):
            rc = fetch_f(*fetch_args[j])
            if rc != MAC_OK:
                _check(rc)
            return bo.value, bi.value

        return arm, fire, fetch

    def best_reduce_dev(self, d_records, n_records: int, d_best, stream=None) -> None:
        """mac_best_reduce_dev: the lexicographic minimum of n_records 16-B {objective, index}
        records (device) into d_best and its mapped slot, on ``stream`` (read it with best_fetch)."""
        _check(self._L.mac_best_reduce_dev(self._h, _devptr(d_records), int(n_records), _devptr(d_best),
                                           _stream(stream, self.device)))

    # -- the multi-GPU poll exchange over RCCL on the poll's stream (mac_comm_*, mac_poll_exchange)
    @staticmethod
    def comm_unique_id(rccl_path: str | None = None) -> bytes:
        """mac_comm_unique_id: a fresh 128-byte communicator id (rank 0 makes it)."""
        buf = ctypes.create_string_buffer(128)
        _check(load_library().mac_comm_unique_id(rccl_path.encode() if rccl_path else None, buf))
        return buf.raw

    def comm_init(self, uid: bytes, rank: int, world: int, rccl_path: str | None = None) -> None:
        """mac_comm_init (collective over the ranks)."""
        if len(uid) != 128:
            raise ValueError("communicator id must be 128 bytes")
        buf = ctypes.create_string_buffer(bytes(uid), 128)
        _check(self._L.mac_comm_init(self._h, rccl_path.encode() if rccl_path else None, buf,
                                     int(rank), int(world)))

    def exchange_step(self, d_best, d_out, stream=None):
        """A bound mac_poll_exchange (prebuilt ctypes arguments): returns a zero-argument callable
        giving the node's (objective, index) over every rank's 16-B d_best."""
        h = _vp(self._h.value if isinstance(self._h, _vp) else self._h)
        bo, bi = ctypes.c_double(), ctypes.c_int64()
        args = (h, _vp(_devptr(d_best)), _vp(_devptr(d_out)), _vp(_stream(stream, self.device)),
                ctypes.byref(bo), ctypes.byref(bi))
        f = self._L.mac_poll_exchange

        def step():
            rc = f(*args)
            if rc != MAC_OK:
                _check(rc)
            return bo.value, bi.value

        return step

    def exchange_records(self, rec: np.ndarray, out: np.ndarray, stream=None) -> None:
        """mac_exchange_records: rec (this rank's record, a contiguous array of 8-B words) gathered
        from every rank into out (world rows of the same size)."""
        _check(self._L.mac_exchange_records(self._h, rec.ctypes.data, int(rec.nbytes), out.ctypes.data,
                                            _stream(stream, self.device)))

    def reduce_step(self, d_records, n_records: int, d_best, stream=None):
        """A bound mac_best_reduce_dev + mac_best_fetch (prebuilt ctypes arguments): returns a
        zero-argument callable giving the reduced (objective, index)."""
        h = _vp(self._h.value if isinstance(self._h, _vp) else self._h)
        sv = _vp(_stream(stream, self.device))
        red_args = (h, _vp(_devptr(d_records)), _i32(int(n_records)), _vp(_devptr(d_best)), sv)
        bo, bi = ctypes.c_double(), ctypes.c_int64()
        fetch_args = (h, _vp(_devptr(d_best)), sv, ctypes.byref(bo), ctypes.byref(bi))
        red, fetch = self._L.mac_best_reduce_dev, self._L.mac_best_fetch

        def step():
            rc = red(*red_args)
            if rc != MAC_OK:
                _check(rc)
            rc = fetch(*fetch_args)
            if rc != MAC_OK:
                _check(rc)
            return bo.value, bi.value

        return step

    def best_fetch(self, d_best, stream=None):
        """The (objective, index) the latest device poll on d_best wrote (mac_best_fetch).
        Thread-safe: the output words are per call.

        Returns as soon as the poll's mapped result slot lands, while the poll's finalize launch
        may still be retiring: d_best itself is then valid for device work on any stream, but
        later host reads of d_obj / d_area, and reuse of the poll's inputs (candidates, d_prev,
        d_rmax), must be ordered on ``stream`` or follow a synchronisation of it."""
        bo, bi = ctypes.c_double(), ctypes.c_int64()
        _check(self._L.mac_best_fetch(self._h, _devptr(d_best), _stream(stream, self.device),
                                      ctypes.byref(bo), ctypes.byref(bi)))
        return bo.value, bi.value


class MadsStepper:
    """mac_mads_begin / _poll / _update / _result (include/maxcover.h): poll() -> (done,
    best_obj, best_idx) over this stepper's shard; update(obj, idx) with the best over all
    shards; result() -> (x, stats). dist.mads_loop drives it."""

    def __init__(self, ctx: Context, x0, r_max, penalty, prev, d_lim, tan_half_fov, n_iter,
                 ell0, ell_max, seed, shard):
        self._L = ctx._L
        self._ctx = ctx   # keeps the context alive while the stepper lives
        x = _f64(x0)
        rm = _f64(r_max)
        pv = _f64(prev) if prev is not None else None
        dl = _f64(d_lim) if d_lim is not None else None
        self.n = x.size
        lo, hi = (0, 2 * x.size) if shard is None else (int(shard[0]), int(shard[1]))
        self.shard = (lo, hi)
        prm = MadsParams(int(n_iter), int(ell0), int(ell_max), int(seed) & (2**64 - 1))
        h = _vp()
        _check(self._L.mac_mads_begin(ctx._h, _ptr(x), x.size, _ptr(rm), float(penalty),
                                      _ptr(pv) if pv is not None else None,
                                      _ptr(dl) if dl is not None else None, float(tan_half_fov),
                                      ctypes.byref(prm), lo, hi, ctypes.byref(h)))
        self._h = h
        self._done, self._bo, self._bi = _i32(), ctypes.c_double(), _i64()

    def poll(self):
        _check(self._L.mac_mads_poll(self._h, ctypes.byref(self._done), ctypes.byref(self._bo),
                                     ctypes.byref(self._bi)))
        return bool(self._done.value), self._bo.value, int(self._bi.value)

    def update(self, best_obj: float, best_idx: int) -> None:
        _check(self._L.mac_mads_update(self._h, float(best_obj), int(best_idx)))

    def poll_ahead(self, ahead: int):
        """mac_mads_poll_ahead: (done, best_obj, best_idx, feasible) of the poll that follows
        `ahead` failures of the current iteration, the stepper unchanged; feasible = its
        candidates that passed cons3."""
        fe = _i64()
        _check(self._L.mac_mads_poll_ahead(self._h, int(ahead), ctypes.byref(self._done),
                                           ctypes.byref(self._bo), ctypes.byref(self._bi),
                                           ctypes.byref(fe)))
        return bool(self._done.value), self._bo.value, int(self._bi.value), int(fe.value)

    def advance(self, best_obj: float, best_idx: int) -> bool:
        """mac_mads_advance: apply one iteration's result; True when the incumbent moved."""
        mv = _i32()
        _check(self._L.mac_mads_advance(self._h, float(best_obj), int(best_idx), ctypes.byref(mv)))
        return bool(mv.value)

    def best_buffer(self, d_best16) -> None:
        """Later polls also write their 16-B shard best into ``d_best16`` (a device tensor of
        2 float64, or None to stop): mac_mads_best_buffer."""
        self._best_buf = d_best16   # kept alive while the stepper writes it
        _check(self._L.mac_mads_best_buffer(self._h, _devptr(d_best16) if d_best16 is not None
                                            else None))

    def result(self):
        out = np.empty(self.n)
        st = MadsStats()
        _check(self._L.mac_mads_result(self._h, _ptr(out), ctypes.byref(st)))
        return out, {k: getattr(st, k) for k, _ in MadsStats._fields_}

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.mac_mads_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _fcheck(rc: int) -> None:
    if rc != MAC_OK:
        raise MaxCoverError(rc, load_library().mac_fire_last_error().decode(errors="replace"))


class Fire:
    """The GPU cellular-automaton fire of src/DynamicArea.jl (mac_fire_*, include/maxcover.h).

    ``ignition`` = (ix0, ix1, iy0, iy1): 1-based inclusive cell block set on fire (:35)."""

    def __init__(self, nx: int, ny: int, dx: float, dy: float, forest_density: float,
                 prob_spread: float, wind_speed: float, wind_direction: float, ignition,
                 seed: int, device: int = 0):
        L = load_library()
        self._L = L
        ix0, ix1, iy0, iy1 = (int(v) for v in ignition)
        self.params = FireParams(int(nx), int(ny), float(dx), float(dy), float(forest_density),
                                 float(prob_spread), float(wind_speed), float(wind_direction),
                                 ix0, ix1, iy0, iy1, int(seed) & (2**64 - 1))
        h = _vp()
        _fcheck(L.mac_fire_create(ctypes.byref(h), int(device), ctypes.byref(self.params)))
        self._h = h
        self.nx, self.ny = int(nx), int(ny)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.mac_fire_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def thresholds(self) -> np.ndarray:
        out = np.zeros(9)
        self._L.mac_fire_thresholds(ctypes.byref(self.params), _ptr(out))
        return out

    def initial_points(self) -> np.ndarray:
        n = _i64()
        _fcheck(self._L.mac_fire_initial_points(self._h, None, 0, ctypes.byref(n)))
        rec = np.zeros((max(n.value, 1), 5))
        _fcheck(self._L.mac_fire_initial_points(self._h, _ptr(rec), n.value, ctypes.byref(n)))
        return rec[: n.value]

    def step(self, append_to: Context | None = None) -> int:
        """One update_grid step (:52-72); the new points are appended to ``append_to``'s list
        (update_POI) when given. Returns how many points were pushed."""
        n = _i64()
        ctx = append_to._h if append_to is not None else None
        _fcheck(self._L.mac_fire_step(self._h, ctx, ctypes.byref(n)))
        return int(n.value)

    def last_points(self) -> np.ndarray:
        """The last step's points as (n, 5) records, in the reference's push order."""
        n = _i64()
        _fcheck(self._L.mac_fire_last_points(self._h, None, 0, ctypes.byref(n)))
        rec = np.zeros((max(n.value, 1), 5))
        _fcheck(self._L.mac_fire_last_points(self._h, _ptr(rec), n.value, ctypes.byref(n)))
        return rec[: n.value]

    def grid(self) -> np.ndarray:
        g = np.empty(self.nx * self.ny, dtype=np.uint8)
        _fcheck(self._L.mac_fire_get_grid(self._h, g.ctypes.data_as(_u8p)))
        return g.reshape(self.nx, self.ny)

    def set_grid(self, g) -> None:
        g = np.ascontiguousarray(np.asarray(g, dtype=np.uint8).reshape(-1))
        if g.size != self.nx * self.ny:
            raise ValueError("grid size mismatch")
        _fcheck(self._L.mac_fire_set_grid(self._h, g.ctypes.data_as(_u8p)))


_default_ctx = None
_default_lock = threading.Lock()


def default_context() -> Context:
    """Process-wide context on LOCAL_RANK's GPU (device 0 by default)."""
    global _default_ctx
    with _default_lock:
        if _default_ctx is None:
            _default_ctx = Context(int(os.environ.get("LOCAL_RANK", "0")))
        return _default_ctx
