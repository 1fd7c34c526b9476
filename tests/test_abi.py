"""The C-ABI library loads and exports every symbol include/orpcd.h declares
(no compute calls: runs on a host without a GPU)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REPO


def _declared():
    src = open(os.path.join(REPO, "include", "orpcd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(orpcd_[a-z0-9_]+)\s*\(", src)))


def test_header_lists_the_python_binding_symbols():
    from orpcd_amd import _native
    assert sorted(_native.EXPORTED) == _declared()


def test_library_exports_every_declared_symbol():
    from orpcd_amd import _native
    lib = _native.LIB_PATH
    assert os.path.exists(lib), "run __graft_entry__.build() first"
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (orpcd_[a-z0-9_]+)", out))
    missing = [s for s in _declared() if s not in exported]
    assert not missing, missing
    L = _native.load_library()
    assert L.orpcd_abi_version() == 1


def test_library_is_gfx950_code_object(tmp_path):
    import shutil
    from orpcd_amd import _native
    lib = shutil.copy(_native.LIB_PATH, tmp_path)     # --offloading extracts the bundles next to its input
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", lib],
                         capture_output=True, text=True, cwd=tmp_path)
    text = out.stdout + out.stderr
    if "gfx" not in text:  # older objdump: fall back to scanning the bundle
        text = open(_native.LIB_PATH, "rb").read().decode("latin1")
    assert "gfx950" in text


def test_no_gpu_fails_loudly_not_silently():
    from orpcd_amd import _native
    if _native.device_count() > 0:
        pytest.skip("a GPU is visible")
    L = _native.load_library()
    h = ctypes.c_void_p()
    assert L.orpcd_ctx_create(0, ctypes.byref(h)) == _native.ORPCD_EDEVICE
    with pytest.raises(_native.NativeError):
        _native.Context(0)


def test_null_context_is_rejected():
    from orpcd_amd import _native
    L = _native.load_library()
    assert L.orpcd_ctx_destroy(None) == _native.ORPCD_EINVAL
    assert L.orpcd_set_source(None, np.zeros(3), 1) == _native.ORPCD_EINVAL
    assert L.orpcd_last_error(None) == b"null context"


def test_product_package_never_imports_the_oracle():
    pkg = os.path.join(REPO, "multi-scale-pointcloud-registration_amd")
    for root, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                text = open(os.path.join(root, f)).read()
                assert "import oracle" not in text and "liborpcd_oracle" not in text, f


def test_library_was_built_from_these_sources():
    """The shipped .so embeds the sha256 of csrc/ + include/ (orpcd_build_id);
    the binding compares it with the tree, so a stale prebuilt library cannot
    run silently on the GPU box."""
    import importlib.util
    from orpcd_amd import _native
    if "ORPCD_HIP_LIB" in os.environ:
        pytest.skip("a variant library is selected")
    spec = importlib.util.spec_from_file_location(
        "bn", os.path.join(REPO, "multi-scale-pointcloud-registration_amd", "build_native.py"))
    bn = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bn)
    sid, flags = _native.build_id()
    assert sid == bn.source_id() and flags == ""


def test_stale_library_is_refused(monkeypatch):
    from orpcd_amd import _native

    class Stale:
        @staticmethod
        def orpcd_build_id():
            return b"0000000000000000"

    monkeypatch.delenv("ORPCD_HIP_LIB", raising=False)
    with pytest.raises(_native.NativeError, match="built from other sources"):
        _native._check_build_id(Stale)
