"""ctypes binding of liborpcd_hip.so (include/orpcd.h).

The product path has exactly one backend: the HIP library built for gfx950.
If it is missing or cannot find a GPU, calls fail loudly — there is no CPU
fallback (the CPU oracle under oracle/ is test infrastructure only).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ORPCD_HIP_LIB", os.path.join(_HERE, "_lib", "liborpcd_hip.so"))

ORPCD_OK, ORPCD_EINVAL, ORPCD_ENOCORR, ORPCD_EDEVICE = 0, 1, 2, 3

_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_i64p = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")


class NativeError(RuntimeError):
    """A HIP runtime / kernel failure or a missing native library."""


class GicpParams(ctypes.Structure):
    _fields_ = [("max_correspondence_distance", ctypes.c_double), ("max_iteration", ctypes.c_int32),
                ("relative_fitness", ctypes.c_double), ("relative_rmse", ctypes.c_double),
                ("epsilon", ctypes.c_double)]


class FgrParams(ctypes.Structure):
    _fields_ = [("division_factor", ctypes.c_double), ("tuple_scale", ctypes.c_double),
                ("maximum_correspondence_distance", ctypes.c_double), ("iteration_number", ctypes.c_int32),
                ("decrease_mu", ctypes.c_int32), ("maximum_tuple_count", ctypes.c_int32),
                ("seed", ctypes.c_uint64)]


try:
    from xxhash import xxh3_64_intdigest as _xxh3
except ImportError:  # pragma: no cover - xxhash is in the image; hashlib is the slower stand-in
    import hashlib

    def _xxh3(buf):
        return hashlib.blake2b(buf, digest_size=8).digest()

_lib = None
_lib_lock = threading.Lock()

# every symbol include/orpcd.h declares (checked by tests/test_abi.py)
EXPORTED = ("orpcd_abi_version", "orpcd_build_id", "orpcd_build_flags", "orpcd_device_count", "orpcd_ctx_create", "orpcd_ctx_destroy",
            "orpcd_last_error", "orpcd_set_target", "orpcd_set_source", "orpcd_gicp_batch",
            "orpcd_set_source_rows", "orpcd_gicp_shard_begin", "orpcd_gicp_shard_pass", "orpcd_gicp_shard_update",
            "orpcd_gicp_shard_result", "orpcd_comm_unique_id", "orpcd_comm_init", "orpcd_comm_destroy",
            "orpcd_gicp_shard_run", "orpcd_gicp_batch_window", "orpcd_set_target_rows", "orpcd_target_cov_width", "orpcd_target_cov_rows",
            "orpcd_set_target_cov", "orpcd_target_layout_bytes", "orpcd_get_target_layout", "orpcd_set_target_layouts",
            "orpcd_device_alloc", "orpcd_device_free",
            "orpcd_nn1_radius", "orpcd_estimate_normals", "orpcd_fpfh", "orpcd_fpfh_from_normals", "orpcd_fgr", "orpcd_feature_nn",
            "orpcd_fgr_optimize", "orpcd_fgr_optimize_batch", "orpcd_set_source_points", "orpcd_icp_p2p_batch",
            "orpcd_sor", "orpcd_voxel_down_sample", "orpcd_farthest_downsample",
            "orpcd_set_option", "orpcd_set_targets", "orpcd_gicp_batch_targets", "orpcd_test_solve6",
            "orpcd_gicp_correspondences",
            "orpcd_profiling", "orpcd_stats", "orpcd_reset_stats", "orpcd_rng_draw_attempts", "orpcd_rigid_residual",
            "orpcd_source_ties", "orpcd_set_posed_tie_rows", "orpcd_tie_sets", "orpcd_pose_rows")


class LegacyDraws:
    """numpy's legacy MT19937 RandomState, advanced by orpcd_rng_draw_attempts:
    ``draw(n, low, high)`` returns (theta (n, 3), normal (n, 3)) exactly as n
    consecutive ``(uniform(low, high, 3), randn(3))`` calls on the RandomState
    whose ``get_state()`` tuple it was built from; ``state()`` is the tuple
    after them (for ``set_state``)."""

    def __init__(self, state):
        name, key, pos, has_gauss, gauss = state
        if name != "MT19937":
            raise ValueError(f"legacy RandomState state expected, got {name}")
        self._key = np.array(key, dtype=np.uint32)
        self._pos = np.array([pos], dtype=np.int32)
        self._hg = np.array([has_gauss], dtype=np.int32)
        self._g = np.array([gauss], dtype=np.float64)
        self._L = load_library()

    def draw(self, n: int, low: float, high: float):
        theta = np.empty((n, 3))
        normal = np.empty((n, 3))
        rc = self._L.orpcd_rng_draw_attempts(self._key, self._pos, self._hg, self._g, int(n), float(low),
                                             float(high), theta, normal)
        if rc != ORPCD_OK:
            raise NativeError(f"orpcd_rng_draw_attempts failed (status {rc})")
        return theta, normal

    def state(self):
        return ("MT19937", self._key.copy(), int(self._pos[0]), int(self._hg[0]), float(self._g[0]))


class _MissingSymbol:
    """An entry point a variant library (ORPCD_HIP_LIB: another commit's build,
    for A/B runs) does not export: its ctypes set-up is accepted, a call raises."""

    def __init__(self, name):
        self.__dict__["name"] = name

    def __setattr__(self, key, value):
        pass

    def __call__(self, *args):
        raise NativeError(f"{self.name} is not exported by the variant library {LIB_PATH}")


class _VariantLib:
    def __init__(self, lib):
        self.__dict__["_lib"] = lib

    def __getattr__(self, name):
        try:
            return getattr(self._lib, name)
        except AttributeError:
            m = _MissingSymbol(name)
            self.__dict__[name] = m
            return m


def load_library():
    """Load liborpcd_hip.so (raises NativeError if it is not built)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"liborpcd_hip.so not found at {LIB_PATH}; build it with "
                              "`python multi-scale-pointcloud-registration_amd/build_native.py` "
                              "(or __graft_entry__.build()).  There is no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH)
        if "ORPCD_HIP_LIB" in os.environ:  # a variant of another commit may lack newer entry points
            L = _VariantLib(L)
        vp, c_int, c_i64, c_dbl = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double
        L.orpcd_abi_version.restype = c_int
        L.orpcd_device_count.argtypes = [ctypes.POINTER(c_int)]
        L.orpcd_ctx_create.argtypes = [c_int, ctypes.POINTER(vp)]
        L.orpcd_ctx_destroy.argtypes = [vp]
        L.orpcd_last_error.argtypes = [vp]
        L.orpcd_last_error.restype = ctypes.c_char_p
        L.orpcd_set_target.argtypes = [vp, _f64p, c_i64, c_dbl]
        L.orpcd_set_source.argtypes = [vp, _f64p, c_i64]
        L.orpcd_gicp_batch.argtypes = [vp, _f64p, _f64p, ctypes.c_int32, ctypes.POINTER(GicpParams), _f64p, _f64p,
                                       _f64p, _i32p, _i64p]
        L.orpcd_set_targets.argtypes = [vp, _f64p, _i64p, ctypes.c_int32, c_dbl]
        L.orpcd_gicp_batch_targets.argtypes = [vp, _f64p, _f64p, _i32p, ctypes.c_int32, ctypes.POINTER(GicpParams),
                                               _f64p, _f64p, _f64p, _i32p, _i64p]
        L.orpcd_test_solve6.argtypes = [vp, _f64p, ctypes.c_int32, _f64p, _f64p]
        L.orpcd_gicp_correspondences.argtypes = [vp, ctypes.c_int32, _i32p]
        L.orpcd_set_source_rows.argtypes = [vp, _f64p, c_i64, c_i64, c_i64]
        L.orpcd_gicp_shard_begin.argtypes = [vp, _f64p, _f64p, ctypes.POINTER(GicpParams), c_i64]
        L.orpcd_gicp_shard_pass.argtypes = [vp, _f64p, _i32p]
        L.orpcd_gicp_shard_update.argtypes = [vp, _f64p, _i32p]
        L.orpcd_gicp_shard_result.argtypes = [vp, _f64p, _f64p, _f64p, _i32p, _i64p]
        _u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
        L.orpcd_comm_unique_id.argtypes = [_u8p]
        L.orpcd_comm_init.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, _u8p]
        L.orpcd_comm_destroy.argtypes = [vp]
        L.orpcd_gicp_shard_run.argtypes = [vp, _i32p]
        L.orpcd_gicp_batch_window.argtypes = [vp, _f64p, _f64p, vp, ctypes.c_int32, ctypes.POINTER(GicpParams),
                                              ctypes.c_int32, ctypes.c_int32, vp, _f64p, _i32p, _f64p, _f64p, _f64p,
                                              _i32p, _i64p]
        L.orpcd_set_target_rows.argtypes = [vp, _f64p, c_i64, c_dbl, ctypes.c_int32, ctypes.c_int32, _i64p, _i64p]
        L.orpcd_target_cov_width.restype = ctypes.c_int32
        L.orpcd_target_cov_width.argtypes = []
        L.orpcd_target_cov_rows.argtypes = [vp, c_i64, c_i64, _f64p]
        L.orpcd_set_target_cov.argtypes = [vp, _f64p]
        L.orpcd_target_layout_bytes.argtypes = [vp, ctypes.c_int32]
        L.orpcd_target_layout_bytes.restype = c_i64
        L.orpcd_get_target_layout.argtypes = [vp, ctypes.c_int32, vp, c_i64]
        L.orpcd_set_target_layouts.argtypes = [vp, ctypes.POINTER(vp), ctypes.c_int32]
        L.orpcd_device_alloc.argtypes = [vp, c_i64, ctypes.POINTER(vp)]
        L.orpcd_device_free.argtypes = [vp, vp]
        L.orpcd_nn1_radius.argtypes = [vp, _f64p, c_i64, _f64p, c_i64, c_dbl, _i32p, _f64p]
        L.orpcd_estimate_normals.argtypes = [vp, _f64p, c_i64, ctypes.c_int32, c_dbl, c_dbl, vp, vp, vp]
        L.orpcd_fpfh.argtypes = [vp, _f64p, c_i64, c_dbl, ctypes.c_int32, c_dbl, ctypes.c_int32, _f64p, _f64p]
        L.orpcd_fpfh_from_normals.argtypes = [vp, _f64p, _f64p, c_i64, c_dbl, ctypes.c_int32, _f64p]
        L.orpcd_fgr.argtypes = [vp, _f64p, c_i64, _f64p, c_i64, _f64p, _f64p, ctypes.POINTER(FgrParams), _f64p,
                                _f64p, _f64p, _i64p, _i64p]
        L.orpcd_feature_nn.argtypes = [vp, _f64p, c_i64, _f64p, c_i64, ctypes.c_int32, _i32p]
        L.orpcd_fgr_optimize.argtypes = [vp, _f64p, c_i64, _f64p, c_i64, c_dbl, ctypes.c_int32, c_dbl,
                                         ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(FgrParams), _f64p, _f64p,
                                         _f64p, _i64p, _i64p]
        L.orpcd_fgr_optimize_batch.argtypes = [vp, _f64p, c_i64, _f64p, _i64p, ctypes.c_int32, _f64p, _f64p,
                                               vp, ctypes.c_int32, c_dbl, ctypes.c_int32, c_dbl, ctypes.c_int32,
                                               ctypes.c_int32, ctypes.POINTER(FgrParams), _f64p, _f64p, _f64p, _i64p,
                                               _i64p]
        L.orpcd_set_source_points.argtypes = [vp, _f64p, c_i64]
        L.orpcd_icp_p2p_batch.argtypes = [vp, _f64p, ctypes.c_int32, ctypes.POINTER(GicpParams), _f64p, _f64p,
                                          _f64p, _i32p, _i64p]
        L.orpcd_sor.argtypes = [vp, _f64p, c_i64, ctypes.c_int32, c_dbl, _i64p, _i64p, vp]
        L.orpcd_voxel_down_sample.argtypes = [vp, _f64p, c_i64, c_dbl, vp, _i64p]
        L.orpcd_farthest_downsample.argtypes = [vp, _f64p, c_i64, ctypes.c_int32, c_i64, _i64p]
        L.orpcd_set_option.argtypes = [vp, ctypes.c_char_p, c_dbl]
        L.orpcd_profiling.argtypes = [vp, ctypes.c_int32]
        L.orpcd_stats.argtypes = [vp, _f64p, ctypes.c_int32]
        L.orpcd_reset_stats.argtypes = [vp]
        L.orpcd_rng_draw_attempts.argtypes = [np.ctypeslib.ndpointer(dtype=np.uint32, flags="C_CONTIGUOUS"),
                                              _i32p, _i32p, _f64p, c_i64, c_dbl, c_dbl, _f64p, _f64p]
        L.orpcd_rigid_residual.argtypes = [_f64p, _f64p, c_i64, _f64p, _f64p, _f64p]
        L.orpcd_source_ties.argtypes = [vp, ctypes.POINTER(c_i64), ctypes.POINTER(c_i64), ctypes.POINTER(ctypes.c_int32),
                                        vp]
        L.orpcd_set_posed_tie_rows.argtypes = [vp, ctypes.c_int32, vp]
        L.orpcd_tie_sets.argtypes = [vp, ctypes.c_int32, vp, _i32p]
        L.orpcd_pose_rows.argtypes = [_f64p, vp, c_i64, _f64p, _f64p, _f64p]
        if L.orpcd_abi_version() != 1:
            raise NativeError("liborpcd_hip.so ABI mismatch")
        if hasattr(L, "orpcd_build_id"):
            L.orpcd_build_id.restype = ctypes.c_char_p
            L.orpcd_build_flags.restype = ctypes.c_char_p
        elif "ORPCD_HIP_LIB" not in os.environ:  # a variant built from an older commit may predate it
            raise NativeError(f"{LIB_PATH} has no orpcd_build_id: stale library; rebuild it")
        _check_build_id(L)
        _lib = L
        return L


def build_id() -> tuple:
    """(source id embedded in the loaded library, its extra compile flags)."""
    L = load_library()
    return L.orpcd_build_id().decode(), L.orpcd_build_flags().decode()


def _check_build_id(L):
    """The default library must have been built from the sources beside it
    (csrc/, include/; they travel with it).  A variant named by ORPCD_HIP_LIB
    (A/B builds of other commits or flags) is exempt."""
    if "ORPCD_HIP_LIB" in os.environ:
        return
    pkg = os.path.dirname(_HERE)
    bn = os.path.join(pkg, "build_native.py")
    if not os.path.exists(bn):  # an installed copy without sources: nothing to compare with
        return
    import importlib.util

    spec = importlib.util.spec_from_file_location("_orpcd_build_native", bn)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    want, have = mod.source_id(), L.orpcd_build_id().decode()
    if want != have:
        raise NativeError(f"{LIB_PATH} was built from other sources (library {have}, tree {want}); rebuild it "
                          "with __graft_entry__.build() or multi-scale-pointcloud-registration_amd/build_native.py")
    flags = L.orpcd_build_flags().decode()
    if flags:  # an instrumented / A-B variant (ORPCD_EXTRA_FLAGS) must be named by ORPCD_HIP_LIB, never the default
        raise NativeError(f"{LIB_PATH} was built with extra flags {flags!r}; the default library must be the "
                          "plain build (rebuild it, or name the variant with ORPCD_HIP_LIB)")


def rigid_residual(base: np.ndarray, src: np.ndarray, R: np.ndarray, t: np.ndarray):
    """(max |src - (base R + t)|, max |src|) for (n, 3) float64 clouds (host only)."""
    out = np.zeros(2)
    rc = load_library().orpcd_rigid_residual(base, src, len(src), np.ascontiguousarray(R, dtype=np.float64),
                                             np.ascontiguousarray(t, dtype=np.float64), out)
    if rc != ORPCD_OK:
        raise NativeError(f"orpcd_rigid_residual failed (status {rc})")
    return float(out[0]), float(out[1])


def pose_rows(xyz: np.ndarray, R: np.ndarray, t: np.ndarray, idx=None) -> np.ndarray:
    """xyz[idx] @ R + t as numpy's np.dot + add forms it (orpcd_pose_rows, host only)."""
    xyz = np.ascontiguousarray(xyz, dtype=np.float64)
    ix = None if idx is None else np.ascontiguousarray(idx, dtype=np.int64)
    n = len(xyz) if ix is None else len(ix)
    out = np.zeros((n, 3))
    rc = load_library().orpcd_pose_rows(xyz, None if ix is None else ix.ctypes.data, n,
                                        np.ascontiguousarray(R, dtype=np.float64),
                                        np.ascontiguousarray(t, dtype=np.float64), out)
    if rc != ORPCD_OK:
        raise NativeError(f"orpcd_pose_rows failed (status {rc})")
    return out


def device_count() -> int:
    n = ctypes.c_int(0)
    load_library().orpcd_device_count(ctypes.byref(n))
    return int(n.value)


def _c3(a) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float64)
    if a.ndim != 2 or a.shape[1] != 3:
        raise ValueError(f"expected an (N, 3) point array, got shape {a.shape}")
    return a


def _consecutive(ts):
    """The (sum M_k, 3) array covering C-contiguous (M_k, 3) float64 clouds that
    lie back to back in one buffer (the Aligner's scaled candidates), else
    None (the caller concatenates)."""
    addr = ts[0].ctypes.data
    for t in ts:
        if t.ctypes.data != addr or not t.flags.c_contiguous:
            return None
        addr += t.nbytes
    return np.lib.stride_tricks.as_strided(ts[0], shape=(sum(len(t) for t in ts), 3), strides=ts[0].strides,
                                           writeable=False)


class Context:
    """One device context (stream + device-resident clouds).  Not thread-safe."""

    def __init__(self, device: Optional[int] = None):
        L = load_library()
        if device is None:
            device = int(os.environ.get("LOCAL_RANK", "0")) if device_count() > 1 else 0
        h = ctypes.c_void_p()
        rc = L.orpcd_ctx_create(int(device), ctypes.byref(h))
        if rc != ORPCD_OK:
            raise NativeError(f"orpcd_ctx_create(device={device}) failed with status {rc} "
                              f"({device_count()} HIP device(s) visible)")
        self._h = h
        self._L = L
        self.device = device
        self._target_key = None
        self._source_key = None

    def close(self):
        if getattr(self, "_h", None):
            self._L.orpcd_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str):
        if rc == ORPCD_OK:
            return
        msg = self._L.orpcd_last_error(self._h)
        msg = msg.decode() if msg else ""
        if rc == ORPCD_EINVAL:
            raise ValueError(f"{what}: {msg}")
        raise NativeError(f"{what} failed (status {rc}): {msg}")

    # ------------------------------------------------------------- clouds
    @staticmethod
    def _key(a: np.ndarray):
        # content fingerprint of the cloud (xxh3 over the buffer, no copy): a
        # cloud re-sent unchanged is not re-uploaded, a changed one always is
        return (a.shape, _xxh3(memoryview(a).cast("B")))

    def set_target(self, xyz: np.ndarray, epsilon: float = 1e-3, cache: bool = True):
        xyz = _c3(xyz)
        # cache=False: no fingerprint (xxh3 reads the whole cloud: ~0.6 ms at 1M points)
        key = (self._key(xyz), float(epsilon)) if cache else None
        if cache and key == self._target_key:
            return
        self._target_key = None
        self._check(self._L.orpcd_set_target(self._h, xyz, len(xyz), float(epsilon)), "orpcd_set_target")
        self._target_key = key

    def set_targets(self, targets, epsilon: float = 1e-3, cache: bool = True):
        """Up to 16 targets for gicp_batch_targets (target k = targets[k])."""
        ts = [_c3(t) for t in targets]
        key = (tuple(self._key(t) for t in ts), float(epsilon), "multi")
        if cache and key == self._target_key:
            return
        self._target_key = None
        m = np.array([len(t) for t in ts], np.int64)
        xyz = _consecutive(ts)
        if xyz is None:
            xyz = np.ascontiguousarray(np.concatenate(ts, axis=0))
        self._check(self._L.orpcd_set_targets(self._h, xyz, m, len(ts), float(epsilon)), "orpcd_set_targets")
        self._target_key = key if len(ts) > 1 else (self._key(ts[0]), float(epsilon))

    # ------------------------------- target layouts as device buffers (re-deal)
    def target_layout_bytes(self, k: int = 0) -> int:
        """Size of target k's device-state buffer (orpcd_target_layout_bytes)."""
        n = int(self._L.orpcd_target_layout_bytes(self._h, int(k)))
        if n < 0:
            msg = self._L.orpcd_last_error(self._h)
            raise ValueError(f"orpcd_target_layout_bytes: {msg.decode() if msg else ''}")
        return n

    def device_alloc(self, nbytes: int) -> int:
        """Device memory on this context's device (orpcd_device_alloc); free with device_free."""
        p = ctypes.c_void_p()
        self._check(self._L.orpcd_device_alloc(self._h, int(nbytes), ctypes.byref(p)), "orpcd_device_alloc")
        return int(p.value)

    def device_free(self, dev_ptr: int):
        self._check(self._L.orpcd_device_free(self._h, ctypes.c_void_p(int(dev_ptr))), "orpcd_device_free")

    def get_target_layout(self, k: int, dev_ptr: int, nbytes: int):
        """Write target k's device state to device memory at dev_ptr (>= target_layout_bytes(k), 256-byte
        aligned, on this context's device; e.g. a torch uint8 tensor's data_ptr())."""
        self._check(self._L.orpcd_get_target_layout(self._h, int(k), ctypes.c_void_p(int(dev_ptr)), int(nbytes)),
                    "orpcd_get_target_layout")

    def set_target_layouts(self, dev_ptrs, key=None):
        """Adopt up to 16 target buffers written by get_target_layout (on any context) as targets 0..n-1, as
        set_targets would have built them.  `key`: the set_targets cache key of the same clouds, if known."""
        arr = (ctypes.c_void_p * len(dev_ptrs))(*[ctypes.c_void_p(int(p)) for p in dev_ptrs])
        self._target_key = None
        self._check(self._L.orpcd_set_target_layouts(self._h, arr, len(dev_ptrs)), "orpcd_set_target_layouts")
        self._target_key = key

    def set_target_points(self, xyz: np.ndarray, cache: bool = True):
        """The target's search layout (covariances skipped) for PointToPoint ICP."""
        xyz = _c3(xyz)
        k = self._key(xyz)
        if cache and self._target_key is not None and self._target_key[0] == k:
            return  # any current layout of the same points serves
        self.set_target(xyz, -1.0, cache=False)
        self._target_key = (k, -1.0)

    def set_source(self, xyz: np.ndarray, cache: bool = True):
        xyz = _c3(xyz)
        key = (self._key(xyz), "cov") if cache else None
        if cache and key == self._source_key:
            return
        self._source_key = None
        self._check(self._L.orpcd_set_source(self._h, xyz, len(xyz)), "orpcd_set_source")
        self._source_key = key

    def set_source_points(self, xyz: np.ndarray, cache: bool = True):
        """The source's search layout only (PointToPoint ICP needs no covariances)."""
        xyz = _c3(xyz)
        key = (self._key(xyz), "points")
        if cache and self._source_key is not None and self._source_key[0] == key[0]:
            return  # a source with covariances serves PointToPoint as well
        self._source_key = None
        self._check(self._L.orpcd_set_source_points(self._h, xyz, len(xyz)), "orpcd_set_source_points")
        self._source_key = key

    # ------------------------------------------------ source boundary ties
    def source_ties(self) -> dict:
        """The current source's KNN-20 boundary ties (orpcd_source_ties): the
        number of listed points, the input indices of every row involved
        (`rows`), and whether every tie was listed."""
        nt, nr, comp = ctypes.c_int64(0), ctypes.c_int64(0), ctypes.c_int32(1)
        self._check(self._L.orpcd_source_ties(self._h, ctypes.byref(nt), ctypes.byref(nr), ctypes.byref(comp), None),
                    "orpcd_source_ties")
        rows = np.zeros(nr.value, np.int64)
        if nr.value:
            self._check(self._L.orpcd_source_ties(self._h, ctypes.byref(nt), ctypes.byref(nr), ctypes.byref(comp),
                                                  rows.ctypes.data), "orpcd_source_ties")
        return dict(n_ties=int(nt.value), rows=rows, complete=bool(comp.value))

    def set_posed_tie_rows(self, xyz):
        """Posed coordinates of the tie rows for each start of the next batch
        ((B, n_rows, 3); a start whose block is NaN uses numpy's product).
        None clears."""
        if xyz is None:
            self._check(self._L.orpcd_set_posed_tie_rows(self._h, 0, None), "orpcd_set_posed_tie_rows")
            return
        xyz = np.ascontiguousarray(xyz, dtype=np.float64)
        self._posed_keep = xyz
        self._check(self._L.orpcd_set_posed_tie_rows(self._h, xyz.shape[0], xyz.ctypes.data), "orpcd_set_posed_tie_rows")

    def tie_sets(self, b: int = -1, posed_rows=None, n_ties: Optional[int] = None) -> np.ndarray:
        """(n_ties, 20) neighbour sets of the ties: from posed_rows ((n_rows, 3))
        if given, else those start b of the last batch used."""
        n = self.source_ties()["n_ties"] if n_ties is None else int(n_ties)
        out = np.zeros((n, 20), np.int32)
        if n == 0:
            return out
        pr = None if posed_rows is None else np.ascontiguousarray(posed_rows, dtype=np.float64)
        self._check(self._L.orpcd_tie_sets(self._h, int(b), None if pr is None else pr.ctypes.data, out),
                    "orpcd_tie_sets")
        return out

    # --------------------------------------------------------------- GICP
    def gicp_batch(self, R0: np.ndarray, t0: np.ndarray, max_correspondence_distance=0.5, max_iteration=100,
                   relative_fitness=1e-6, relative_rmse=1e-6, epsilon=1e-3) -> dict:
        R0 = np.ascontiguousarray(R0, dtype=np.float64).reshape(-1, 3, 3)
        B = R0.shape[0]
        t0 = np.ascontiguousarray(t0, dtype=np.float64).reshape(B, 3)
        p = GicpParams(float(max_correspondence_distance), int(max_iteration), float(relative_fitness),
                       float(relative_rmse), float(epsilon))
        T = np.zeros((B, 4, 4))
        rmse, fit = np.zeros(B), np.zeros(B)
        iters = np.zeros(B, np.int32)
        ncorr = np.zeros(B, np.int64)
        self._check(self._L.orpcd_gicp_batch(self._h, R0.reshape(-1), t0.reshape(-1), B, ctypes.byref(p),
                                             T.reshape(-1), rmse, fit, iters, ncorr), "orpcd_gicp_batch")
        return dict(T=T, rmse=rmse, fitness=fit, iters=iters, ncorr=ncorr)

    def gicp_batch_targets(self, R0: np.ndarray, t0: np.ndarray, target_of_start, max_correspondence_distance=0.5,
                           max_iteration=100, relative_fitness=1e-6, relative_rmse=1e-6, epsilon=1e-3) -> dict:
        """gicp_batch with start b against target target_of_start[b] (set_targets)."""
        R0 = np.ascontiguousarray(R0, dtype=np.float64).reshape(-1, 3, 3)
        B = R0.shape[0]
        t0 = np.ascontiguousarray(t0, dtype=np.float64).reshape(B, 3)
        tids = np.ascontiguousarray(target_of_start, dtype=np.int32).reshape(B)
        p = GicpParams(float(max_correspondence_distance), int(max_iteration), float(relative_fitness),
                       float(relative_rmse), float(epsilon))
        T = np.zeros((B, 4, 4))
        rmse, fit = np.zeros(B), np.zeros(B)
        iters = np.zeros(B, np.int32)
        ncorr = np.zeros(B, np.int64)
        self._check(self._L.orpcd_gicp_batch_targets(self._h, R0.reshape(-1), t0.reshape(-1), tids, B,
                                                     ctypes.byref(p), T.reshape(-1), rmse, fit, iters, ncorr),
                    "orpcd_gicp_batch_targets")
        return dict(T=T, rmse=rmse, fitness=fit, iters=iters, ncorr=ncorr)

    STATE_W = 18  # a running start's state: T (4x4, row-major), previous fitness and rmse

    def gicp_batch_window(self, R0: np.ndarray, t0: np.ndarray, target_of_start=None, pass_begin: int = 0,
                          pass_end: int = 1 << 30, state=None, max_correspondence_distance=0.5, max_iteration=100,
                          relative_fitness=1e-6, relative_rmse=1e-6, epsilon=1e-3) -> dict:
        """gicp_batch_targets over passes [pass_begin, pass_end) (orpcd_gicp_batch_window):
        `done` marks the starts that finished (their outputs are set); `state`
        (B, 18) is where the others stand at pass_end, to resume them from
        (pass_begin = pass_end, state) in any batch."""
        R0 = np.ascontiguousarray(R0, dtype=np.float64).reshape(-1, 3, 3)
        B = R0.shape[0]
        t0 = np.ascontiguousarray(t0, dtype=np.float64).reshape(B, 3)
        tids = None if target_of_start is None else np.ascontiguousarray(target_of_start, dtype=np.int32).reshape(B)
        st_in = None if state is None else np.ascontiguousarray(state, dtype=np.float64).reshape(B, self.STATE_W)
        p = GicpParams(float(max_correspondence_distance), int(max_iteration), float(relative_fitness),
                       float(relative_rmse), float(epsilon))
        T = np.zeros((B, 4, 4))
        rmse, fit = np.zeros(B), np.zeros(B)
        iters = np.zeros(B, np.int32)
        ncorr = np.zeros(B, np.int64)
        done = np.zeros(B, np.int32)
        st_out = np.zeros((B, self.STATE_W))
        ptr = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        self._check(self._L.orpcd_gicp_batch_window(self._h, R0.reshape(-1), t0.reshape(-1), ptr(tids), B,
                                                    ctypes.byref(p), int(pass_begin), int(pass_end), ptr(st_in),
                                                    st_out.reshape(-1), done, T.reshape(-1), rmse, fit, iters,
                                                    ncorr), "orpcd_gicp_batch_window")
        return dict(T=T, rmse=rmse, fitness=fit, iters=iters, ncorr=ncorr, done=done.astype(bool), state=st_out)

    def gicp_correspondences(self, B: int, N: int) -> np.ndarray:
        """(B, N) input index of each source point's nearest target in the
        last pass of each start of the last single-target batch (-1: none)."""
        out = np.zeros((int(B), int(N)), dtype=np.int32)
        self._check(self._L.orpcd_gicp_correspondences(self._h, int(B), out), "orpcd_gicp_correspondences")
        return out

    def test_solve6(self, sums27: np.ndarray):
        """(serial, wave) results of orpcd_test_solve6: (n, 23) each."""
        sums27 = np.ascontiguousarray(sums27, dtype=np.float64).reshape(-1, 27)
        n = len(sums27)
        a, b = np.zeros((n, 23)), np.zeros((n, 23))
        self._check(self._L.orpcd_test_solve6(self._h, sums27, n, a, b), "orpcd_test_solve6")
        return a, b

    def icp_p2p_batch(self, init: np.ndarray, max_correspondence_distance=0.5, max_iteration=200,
                      relative_fitness=1e-6, relative_rmse=1e-6) -> dict:
        """registration_icp(PointToPoint) of the current source / target from
        each init[b] (column convention, applied as Open3D applies `init`).
        Returns Open3D's result.transformation per init (init included)."""
        init = np.ascontiguousarray(init, dtype=np.float64).reshape(-1, 4, 4)
        B = init.shape[0]
        p = GicpParams(float(max_correspondence_distance), int(max_iteration), float(relative_fitness),
                       float(relative_rmse), -1.0)
        T = np.zeros((B, 4, 4))
        rmse, fit = np.zeros(B), np.zeros(B)
        iters = np.zeros(B, np.int32)
        ncorr = np.zeros(B, np.int64)
        self._check(self._L.orpcd_icp_p2p_batch(self._h, init.reshape(-1), B, ctypes.byref(p), T.reshape(-1), rmse,
                                                fit, iters, ncorr), "orpcd_icp_p2p_batch")
        return dict(T=T, rmse=rmse, fitness=fit, iters=iters, ncorr=ncorr)

    # ------------------------------------------------------ preprocessing
    def sor(self, xyz: np.ndarray, nb_neighbors: int = 64, std_ratio: float = 2.0, return_avg: bool = False):
        """remove_statistical_outlier: kept indices (increasing) [, per-point mean distances]."""
        xyz = _c3(xyz)
        n = len(xyz)
        idx = np.empty(max(n, 1), np.int64)
        k = np.zeros(1, np.int64)
        avg = np.empty(n) if return_avg else None
        self._check(self._L.orpcd_sor(self._h, xyz if n else np.zeros((1, 3)), n, int(nb_neighbors),
                                      float(std_ratio), idx, k, avg.ctypes.data_as(ctypes.c_void_p)
                                      if avg is not None else None), "orpcd_sor")
        kept = idx[:int(k[0])].copy()
        return (kept, avg) if return_avg else kept

    def voxel_down_sample(self, xyz: np.ndarray, voxel_size: float, count_only: bool = False):
        """voxel_down_sample: averaged points, voxels in (ix, iy, iz) order (or their count)."""
        xyz = _c3(xyz)
        n = len(xyz)
        k = np.zeros(1, np.int64)
        out = None if count_only else np.empty((max(n, 1), 3))
        self._check(self._L.orpcd_voxel_down_sample(self._h, xyz if n else np.zeros((1, 3)), n, float(voxel_size),
                                                    out.ctypes.data_as(ctypes.c_void_p) if out is not None else None,
                                                    k), "orpcd_voxel_down_sample")
        return int(k[0]) if count_only else out[:int(k[0])].copy()

    def farthest_downsample(self, xyz: np.ndarray, sample_size: int, first: int) -> np.ndarray:
        """Farthest-point sampling from index ``first``: the chosen indices."""
        xyz = _c3(xyz)
        idx = np.empty(max(int(sample_size), 1), np.int64)
        self._check(self._L.orpcd_farthest_downsample(self._h, xyz, len(xyz), int(sample_size), int(first), idx),
                    "orpcd_farthest_downsample")
        return idx[:int(sample_size)]

    # ------------------------------------------ one start, rows over ranks
    def set_source_rows(self, xyz: np.ndarray, row_begin: int, row_end: int):
        xyz = _c3(xyz)
        self._check(self._L.orpcd_set_source_rows(self._h, xyz, len(xyz), int(row_begin), int(row_end)),
                    "orpcd_set_source_rows")
        self._source_key = None

    def shard_begin(self, R0, t0, n_total: int, max_correspondence_distance=0.5, max_iteration=100,
                    relative_fitness=1e-6, relative_rmse=1e-6, epsilon=1e-3):
        p = GicpParams(float(max_correspondence_distance), int(max_iteration), float(relative_fitness),
                       float(relative_rmse), float(epsilon))
        R0 = np.ascontiguousarray(R0, dtype=np.float64).reshape(9)
        t0 = np.ascontiguousarray(t0, dtype=np.float64).reshape(3)
        self._check(self._L.orpcd_gicp_shard_begin(self._h, R0, t0, ctypes.byref(p), int(n_total)),
                    "orpcd_gicp_shard_begin")

    def shard_pass(self):
        """(local sums (29,), active)"""
        sums = np.zeros(29)
        act = np.zeros(1, np.int32)
        self._check(self._L.orpcd_gicp_shard_pass(self._h, sums, act), "orpcd_gicp_shard_pass")
        return sums, bool(act[0])

    def shard_update(self, sums: np.ndarray) -> bool:
        sums = np.ascontiguousarray(sums, dtype=np.float64).reshape(29)
        done = np.zeros(1, np.int32)
        self._check(self._L.orpcd_gicp_shard_update(self._h, sums, done), "orpcd_gicp_shard_update")
        return bool(done[0])

    def shard_result(self) -> dict:
        T, rmse, fit = np.zeros(16), np.zeros(1), np.zeros(1)
        it, nc = np.zeros(1, np.int32), np.zeros(1, np.int64)
        self._check(self._L.orpcd_gicp_shard_result(self._h, T, rmse, fit, it, nc), "orpcd_gicp_shard_result")
        return dict(T=T.reshape(4, 4), rmse=float(rmse[0]), fitness=float(fit[0]), iters=int(it[0]),
                    ncorr=int(nc[0]))

    def set_target_rows(self, xyz: np.ndarray, rank: int, nranks: int, epsilon: float = 1e-3):
        """This rank's share of the target's covariance pass (orpcd_set_target_rows);
        returns its Morton rows (lo, hi).  Complete at once with a communicator
        of nranks ranks; otherwise complete it with set_target_cov."""
        xyz = _c3(xyz)
        lo, hi = np.zeros(1, np.int64), np.zeros(1, np.int64)
        self._check(self._L.orpcd_set_target_rows(self._h, xyz, len(xyz), float(epsilon), int(rank), int(nranks),
                                                  lo, hi), "orpcd_set_target_rows")
        self._target_key = None
        self._target_rows_n = len(xyz)
        return int(lo[0]), int(hi[0])

    def target_cov_rows(self, lo: int, hi: int) -> np.ndarray:
        """The target's covariance rows [lo, hi) in Morton order, (hi - lo, width)."""
        w = int(self._L.orpcd_target_cov_width())
        out = np.zeros((max(int(hi) - int(lo), 0), w))
        self._check(self._L.orpcd_target_cov_rows(self._h, int(lo), int(hi), out.reshape(-1) if out.size else
                                                  np.zeros(1)), "orpcd_target_cov_rows")
        return out

    def set_target_cov(self, cov: np.ndarray):
        """Complete a target begun with set_target_rows: every rank's rows, in order (m, width)."""
        cov = np.ascontiguousarray(cov, dtype=np.float64)
        n = getattr(self, "_target_rows_n", None)
        if n is None or cov.size != n * int(self._L.orpcd_target_cov_width()):
            raise ValueError("set_target_cov: needs set_target_rows first and (m, width) rows")
        self._check(self._L.orpcd_set_target_cov(self._h, cov.reshape(-1)), "orpcd_set_target_cov")

    # ------------------------------------------- device collectives (RCCL)
    def comm_unique_id(self) -> bytes:
        """A new RCCL unique id (128 bytes) for orpcd_comm_init on every rank."""
        uid = np.zeros(128, np.uint8)
        if self._L.orpcd_comm_unique_id(uid) != ORPCD_OK:
            raise NativeError("orpcd_comm_unique_id failed (librccl.so missing or no device)")
        return uid.tobytes()

    def comm_init(self, nranks: int, rank: int, uid: bytes):
        buf = np.frombuffer(bytes(uid), np.uint8).copy()
        if buf.size != 128:
            raise ValueError("comm_init: the RCCL id is 128 bytes")
        self._check(self._L.orpcd_comm_init(self._h, int(nranks), int(rank), buf), "orpcd_comm_init")

    def comm_destroy(self):
        self._check(self._L.orpcd_comm_destroy(self._h), "orpcd_comm_destroy")

    def shard_run(self) -> int:
        """Every pass of the begun row-sharded start, the per-pass all-reduce
        on the device (orpcd_gicp_shard_run); returns the passes enqueued."""
        n = np.zeros(1, np.int32)
        self._check(self._L.orpcd_gicp_shard_run(self._h, n), "orpcd_gicp_shard_run")
        return int(n[0])

    # -------------------------------------------------------- kernel level
    def nn1_radius(self, q: np.ndarray, t: np.ndarray, radius: float):
        q, t = _c3(q), _c3(t)
        idx = np.empty(len(q), np.int32)
        d2 = np.empty(len(q))
        self._check(self._L.orpcd_nn1_radius(self._h, q, len(q), t, len(t), float(radius), idx, d2),
                    "orpcd_nn1_radius")
        return idx, d2

    def estimate_normals(self, xyz: np.ndarray, knn: int = 20, radius: float = -1.0, epsilon: float = 1e-3):
        xyz = _c3(xyz)
        n = len(xyz)
        normals = np.empty((n, 3))
        raw = np.empty((n, 3, 3))
        cov = np.empty((n, 3, 3))
        ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        self._check(self._L.orpcd_estimate_normals(self._h, xyz, n, int(knn), float(radius), float(epsilon),
                                                   ptr(normals), ptr(raw), ptr(cov) if epsilon >= 0 else None),
                    "orpcd_estimate_normals")
        return normals, raw, (cov if epsilon >= 0 else None)

    def fpfh(self, xyz: np.ndarray, normal_radius=0.1, normal_knn=20, fpfh_radius=0.1, fpfh_knn=20):
        xyz = _c3(xyz)
        normals = np.empty((len(xyz), 3))
        feat = np.empty((len(xyz), 33))
        self._check(self._L.orpcd_fpfh(self._h, xyz, len(xyz), float(normal_radius), int(normal_knn),
                                       float(fpfh_radius), int(fpfh_knn), normals, feat.reshape(-1)), "orpcd_fpfh")
        return normals, feat

    def fpfh_from_normals(self, xyz: np.ndarray, normals: np.ndarray, fpfh_radius=0.1, fpfh_knn=20):
        xyz, normals = _c3(xyz), _c3(normals)
        if len(normals) != len(xyz):
            raise ValueError("fpfh_from_normals: one normal per point")
        feat = np.empty((len(xyz), 33))
        self._check(self._L.orpcd_fpfh_from_normals(self._h, xyz, normals, len(xyz), float(fpfh_radius),
                                                    int(fpfh_knn), feat.reshape(-1)), "orpcd_fpfh_from_normals")
        return feat

    def feature_nn(self, q: np.ndarray, t: np.ndarray) -> np.ndarray:
        """Nearest row of ``t`` for every row of ``q`` (squared L2, ties -> lowest index)."""
        q = np.ascontiguousarray(q, dtype=np.float64)
        t = np.ascontiguousarray(t, dtype=np.float64)
        if q.ndim != 2 or t.ndim != 2 or q.shape[1] != t.shape[1]:
            raise ValueError(f"feature_nn: expected (Nq, D) and (Nt, D), got {q.shape} and {t.shape}")
        idx = np.empty(len(q), np.int32)
        self._check(self._L.orpcd_feature_nn(self._h, q.reshape(-1), len(q), t.reshape(-1), len(t), q.shape[1],
                                             idx), "orpcd_feature_nn")
        return idx

    def fgr(self, src, tgt, src_feat, tgt_feat, division_factor=1.4, tuple_scale=0.9,
            maximum_correspondence_distance=0.5, iteration_number=100, decrease_mu=True,
            maximum_tuple_count=1000, seed=0) -> dict:
        src, tgt = _c3(src), _c3(tgt)
        fs = np.ascontiguousarray(src_feat, dtype=np.float64)
        ft = np.ascontiguousarray(tgt_feat, dtype=np.float64)
        if fs.shape != (len(src), 33) or ft.shape != (len(tgt), 33):
            raise ValueError(f"features must be (N, 33) per cloud, got {fs.shape} and {ft.shape}")
        p = self._fgr_params(division_factor, tuple_scale, maximum_correspondence_distance, iteration_number,
                             decrease_mu, maximum_tuple_count, seed)
        T = np.zeros(16)
        fit, rmse = np.zeros(1), np.zeros(1)
        nc, nm = np.zeros(1, np.int64), np.zeros(2, np.int64)
        self._check(self._L.orpcd_fgr(self._h, src, len(src), tgt, len(tgt), fs.reshape(-1), ft.reshape(-1),
                                      ctypes.byref(p), T, fit, rmse, nc, nm), "orpcd_fgr")
        return dict(T=T.reshape(4, 4), fitness=float(fit[0]), rmse=float(rmse[0]), ncorr=int(nc[0]),
                    n_mutual=int(nm[0]), n_tuple_corr=int(nm[1]))

    @staticmethod
    def _fgr_params(division_factor, tuple_scale, maximum_correspondence_distance, iteration_number, decrease_mu,
                    maximum_tuple_count, seed):
        return FgrParams(float(division_factor), float(tuple_scale), float(maximum_correspondence_distance),
                         int(iteration_number), int(bool(decrease_mu)), int(maximum_tuple_count),
                         int(seed) & 0xFFFFFFFFFFFFFFFF)

    def fgr_optimize(self, src, tgt, normal_radius=0.1, normal_knn=20, fpfh_radius=0.1, fpfh_knn=20,
                     target_features_from_source=True, division_factor=1.4, tuple_scale=0.9,
                     maximum_correspondence_distance=0.5, iteration_number=100, decrease_mu=True,
                     maximum_tuple_count=1000, seed=0) -> dict:
        """FPFH of both clouds + FGR in one device pass (orpcd_fgr_optimize)."""
        src, tgt = _c3(src), _c3(tgt)
        p = self._fgr_params(division_factor, tuple_scale, maximum_correspondence_distance, iteration_number,
                             decrease_mu, maximum_tuple_count, seed)
        T = np.zeros(16)
        fit, rmse = np.zeros(1), np.zeros(1)
        nc, nm = np.zeros(1, np.int64), np.zeros(2, np.int64)
        self._check(self._L.orpcd_fgr_optimize(self._h, src, len(src), tgt, len(tgt), float(normal_radius),
                                               int(normal_knn), float(fpfh_radius), int(fpfh_knn),
                                               int(bool(target_features_from_source)), ctypes.byref(p), T, fit,
                                               rmse, nc, nm), "orpcd_fgr_optimize")
        return dict(T=T.reshape(4, 4), fitness=float(fit[0]), rmse=float(rmse[0]), ncorr=int(nc[0]),
                    n_mutual=int(nm[0]), n_tuple_corr=int(nm[1]))

    def fgr_optimize_batch(self, src, targets, R0, t0, target_of_start=None, normal_radius=0.1, normal_knn=20,
                           fpfh_radius=0.1, fpfh_knn=20, target_features_from_source=True, division_factor=1.4,
                           tuple_scale=0.9, maximum_correspondence_distance=0.5, iteration_number=100,
                           decrease_mu=True, maximum_tuple_count=1000, seed=0) -> dict:
        """``fgr_optimize(src @ R0[b] + t0[b], targets[target_of_start[b]])``
        for every start b as ONE call (orpcd_fgr_optimize_batch), bit for bit
        the per-call results.  Returns per-start arrays T (B, 4, 4; Open3D's
        column convention), fitness, rmse, ncorr, n_mutual, n_tuple_corr."""
        src = _c3(src)
        tg = [_c3(t) for t in targets]
        if not 1 <= len(tg) <= 16:
            raise ValueError("fgr_optimize_batch: 1..16 targets")
        m = np.array([len(t) for t in tg], np.int64)
        tcat = np.ascontiguousarray(np.concatenate(tg)).reshape(-1)
        R0 = np.ascontiguousarray(R0, dtype=np.float64).reshape(-1, 3, 3)
        t0 = np.ascontiguousarray(t0, dtype=np.float64).reshape(-1, 3)
        B = len(R0)
        if len(t0) != B or B == 0:
            raise ValueError(f"fgr_optimize_batch: R0 {R0.shape} and t0 {t0.shape} must hold the same B >= 1 starts")
        tos = None
        if target_of_start is not None:
            tos = np.ascontiguousarray(target_of_start, dtype=np.int32)
            if tos.shape != (B,):
                raise ValueError("fgr_optimize_batch: one target index per start")
        p = self._fgr_params(division_factor, tuple_scale, maximum_correspondence_distance, iteration_number,
                             decrease_mu, maximum_tuple_count, seed)
        T = np.zeros(16 * B)
        fit, rmse = np.zeros(B), np.zeros(B)
        nc, nm = np.zeros(B, np.int64), np.zeros(2 * B, np.int64)
        self._check(self._L.orpcd_fgr_optimize_batch(
            self._h, src, len(src), tcat, m, len(tg), R0.reshape(-1), t0.reshape(-1),
            None if tos is None else tos.ctypes.data_as(ctypes.c_void_p), B, float(normal_radius), int(normal_knn),
            float(fpfh_radius), int(fpfh_knn), int(bool(target_features_from_source)), ctypes.byref(p), T, fit, rmse,
            nc, nm), "orpcd_fgr_optimize_batch")
        return dict(T=T.reshape(B, 4, 4), fitness=fit, rmse=rmse, ncorr=nc, n_mutual=nm[0::2].copy(),
                    n_tuple_corr=nm[1::2].copy())

    def set_option(self, key: str, value: float):
        self._check(self._L.orpcd_set_option(self._h, key.encode(), float(value)), "orpcd_set_option")

    # ---------------------------------------------------------- measuring
    def profiling(self, enable: bool = True):
        self._check(self._L.orpcd_profiling(self._h, int(bool(enable))), "orpcd_profiling")

    def stats(self) -> dict:
        out = np.zeros(20)
        self._check(self._L.orpcd_stats(self._h, out, 20), "orpcd_stats")
        return dict(launches=out[0], ms=out[1], pairs=out[2], iterations=out[3], passes=out[4], tiles=out[5],
                    accum_ms=out[6], sched_launches=out[7], exact_filed=out[8], exact_queries=out[9],
                    host_batch_ms=out[10], host_launch_ms=out[11], host_sync_ms=out[12], host_batches=out[13],
                    feat_pass1_ms=out[14], feat_pass2_ms=out[15], feat_pass1_pairs=out[16],
                    feat_pass2_pairs=out[17], feat_calls=out[18], tie_gaps=out[19])

    def reset_stats(self):
        self._check(self._L.orpcd_reset_stats(self._h), "orpcd_reset_stats")


_default_ctx = {}


def default_context(device: Optional[int] = None) -> Context:
    """Process-wide context per device (one process per GPU)."""
    key = device
    if key not in _default_ctx:
        _default_ctx[key] = Context(device)
    return _default_ctx[key]
