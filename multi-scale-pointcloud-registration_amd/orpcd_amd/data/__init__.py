"""Point-cloud loading (reference: or_pcd/data/__init__.py:5-18, which reads
the packaged sample PLYs through Open3D's ``read_point_cloud``).

``read_ply_points`` parses PLY files without Open3D: ascii,
binary_little_endian and binary_big_endian; the ``vertex`` element's x, y, z
(any scalar type) become an (N, 3) float64 array as ``np.asarray(cloud.points)``
gives; other vertex properties and other elements (including list properties
such as the range scans' ``range_grid``) are skipped.  Host-side I/O: the
points are handed to the device paths afterwards.

``load_sample_cloud(name)`` looks for ``<name>.ply`` in ``data_dir``, then
``$ORPCD_DATA``, then this package directory.  The reference's sample scans
(ArmadilloBack_*.ply, Stanford 3D scanning repository) are not redistributed
with this package; point ``ORPCD_DATA`` at a copy.
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import numpy as np

_SCALARS = {
    "char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1",
    "short": "i2", "int16": "i2", "ushort": "u2", "uint16": "u2",
    "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
    "float": "f4", "float32": "f4", "double": "f8", "float64": "f8",
}


class PlyError(ValueError):
    pass


def _header(f) -> Tuple[str, List[tuple], int]:
    if f.readline().strip() != b"ply":
        raise PlyError("not a PLY file (missing 'ply' magic)")
    fmt = None
    elements: List[tuple] = []  # (name, count, [(prop, type) | (prop, ("list", count_t, item_t))])
    while True:
        line = f.readline()
        if not line:
            raise PlyError("truncated PLY header")
        tok = line.decode("ascii", "replace").split()
        if not tok or tok[0] in ("comment", "obj_info"):
            continue
        if tok[0] == "format":
            fmt = tok[1]
        elif tok[0] == "element":
            elements.append((tok[1], int(tok[2]), []))
        elif tok[0] == "property":
            if not elements:
                raise PlyError("property before any element")
            if tok[1] == "list":
                elements[-1][2].append((tok[4], ("list", _SCALARS[tok[2]], _SCALARS[tok[3]])))
            else:
                if tok[1] not in _SCALARS:
                    raise PlyError(f"unknown PLY type {tok[1]!r}")
                elements[-1][2].append((tok[2], _SCALARS[tok[1]]))
        elif tok[0] == "end_header":
            break
    if fmt not in ("ascii", "binary_little_endian", "binary_big_endian"):
        raise PlyError(f"unsupported PLY format {fmt!r}")
    return fmt, elements, f.tell()


def _skip_binary(buf: memoryview, off: int, count: int, props, endian: str) -> int:
    if all(not isinstance(t, tuple) for _, t in props):
        return off + count * sum(np.dtype(t).itemsize for _, t in props)
    for _ in range(count):
        for _, t in props:
            if isinstance(t, tuple):
                ct = np.dtype(endian + t[1])
                n = int(np.frombuffer(buf, ct, 1, off)[0])
                off += ct.itemsize + n * np.dtype(t[2]).itemsize
            else:
                off += np.dtype(t).itemsize
    return off


def read_ply_points(path: str) -> np.ndarray:
    """The vertex positions of a PLY file as an (N, 3) float64 array."""
    with open(path, "rb") as f:
        fmt, elements, start = _header(f)
        data = f.read()
    names = [e[0] for e in elements]
    if "vertex" not in names:
        raise PlyError("PLY has no vertex element")
    vprops = [p for p, _ in elements[names.index("vertex")][2]]
    if not all(a in vprops for a in "xyz"):
        raise PlyError("vertex element lacks x, y, z")
    if fmt == "ascii":
        lines = data.decode("ascii", "replace").split("\n")
        li = 0
        for name, count, props in elements:
            if name != "vertex":
                li += count
                continue
            if any(isinstance(t, tuple) for _, t in props):
                raise PlyError("list properties in an ascii vertex element are not supported")
            rows = np.array([ln.split() for ln in lines[li:li + count]], dtype=np.float64).reshape(count, len(props))
            return np.ascontiguousarray(rows[:, [vprops.index(a) for a in "xyz"]])
    endian = "<" if fmt == "binary_little_endian" else ">"
    buf = memoryview(data)
    off = 0
    for name, count, props in elements:
        if name == "vertex":
            if any(isinstance(t, tuple) for _, t in props):
                raise PlyError("list properties in the vertex element are not supported")
            dt = np.dtype([(p, endian + t) for p, t in props])
            if off + count * dt.itemsize > len(data):
                raise PlyError("truncated PLY vertex data")
            v = np.frombuffer(data, dt, count, off)
            return np.stack([v[a].astype(np.float64) for a in "xyz"], axis=1)
        off = _skip_binary(buf, off, count, props, endian)
    raise PlyError("unreachable")


def load_sample_cloud(name: str = "ArmadilloBack_180", data_dir: Optional[str] = None) -> np.ndarray:
    """data/__init__.py:5-18: the sample cloud ``name`` as an (N, 3) float64 array."""
    dirs = [d for d in (data_dir, os.environ.get("ORPCD_DATA"), os.path.dirname(os.path.abspath(__file__))) if d]
    for d in dirs:
        path = os.path.join(d, name + ".ply")
        if os.path.exists(path):
            return read_ply_points(path)
    raise FileNotFoundError(f"{name}.ply not found in {dirs}; set ORPCD_DATA to a directory holding the "
                            "sample scans")
