"""PLY loading without Open3D (reference: or_pcd/data/__init__.py:5-18 →
o3d.io.read_point_cloud).  Pinned against the reference's own sample scans
when /root/reference is present (the committed armadillo.npz was parsed from
them), and on synthetic files in every PLY encoding."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from orpcd_amd.data import PlyError, load_sample_cloud, read_ply_points

REF_DATA = "/root/reference/src/or_pcd/data"


@pytest.mark.skipif(not os.path.isdir(REF_DATA), reason="reference sample scans not present")
def test_reference_scans_match_committed_points():
    z = np.load(os.path.join(GOLDEN, "armadillo.npz"))
    for name in ("ArmadilloBack_330", "ArmadilloBack_0"):
        p = load_sample_cloud(name, REF_DATA)
        assert p.dtype == np.float64 and p.shape == z[name].shape
        assert np.array_equal(p, z[name].astype(np.float64))


def _write(path, fmt, pts, extra_list=True):
    n = len(pts)
    hdr = ["ply", f"format {fmt} 1.0", "comment synthetic", "obj_info test 1",
           "element camera 1", "property float px", "property uchar flag"]
    hdr += [f"element vertex {n}", "property double x", "property float nx", "property double y",
            "property double z", "property uchar red"]
    if extra_list:
        hdr += ["element range_grid 4", "property list uchar int vertex_indices"]
    hdr += ["end_header"]
    with open(path, "wb") as f:
        f.write(("\n".join(hdr) + "\n").encode())
        if fmt == "ascii":
            f.write(b"1.5 3\n")
            for p in pts:
                f.write(f"{float(p[0])!r} 0.25 {float(p[1])!r} {float(p[2])!r} 7\n".encode())
            if extra_list:
                f.write(b"0\n1 5\n2 6 7\n0\n")
            return
        e = "<" if fmt == "binary_little_endian" else ">"
        f.write(np.array([1.5], e + "f4").tobytes() + np.array([3], "u1").tobytes())
        dt = np.dtype([("x", e + "f8"), ("nx", e + "f4"), ("y", e + "f8"), ("z", e + "f8"), ("r", "u1")])
        v = np.zeros(n, dt)
        v["x"], v["y"], v["z"], v["nx"], v["r"] = pts[:, 0], pts[:, 1], pts[:, 2], 0.25, 7
        f.write(v.tobytes())
        if extra_list:
            for row in ([], [5], [6, 7], []):
                f.write(np.array([len(row)], "u1").tobytes() + np.array(row, e + "i4").tobytes())


@pytest.mark.parametrize("fmt", ["ascii", "binary_little_endian", "binary_big_endian"])
def test_synthetic_ply_all_encodings(tmp_path, fmt):
    pts = np.random.default_rng(0).normal(size=(37, 3))
    p = tmp_path / "c.ply"
    _write(p, fmt, pts)
    got = read_ply_points(str(p))
    assert got.shape == (37, 3) and np.array_equal(got, pts)


def test_list_element_before_vertex(tmp_path):
    """A binary element with list properties ahead of the vertices is skipped."""
    pts = np.arange(12.0).reshape(4, 3)
    p = tmp_path / "l.ply"
    with open(p, "wb") as f:
        f.write(b"ply\nformat binary_big_endian 1.0\nelement face 2\nproperty list uchar int vi\n"
                b"element vertex 4\nproperty float x\nproperty float y\nproperty float z\nend_header\n")
        f.write(bytes([3]) + np.array([0, 1, 2], ">i4").tobytes() + bytes([1]) + np.array([3], ">i4").tobytes())
        f.write(pts.astype(">f4").tobytes())
    assert np.array_equal(read_ply_points(str(p)), pts)


def test_errors(tmp_path):
    bad = tmp_path / "x.ply"
    bad.write_bytes(b"not a ply\n")
    with pytest.raises(PlyError):
        read_ply_points(str(bad))
    trunc = tmp_path / "t.ply"
    trunc.write_bytes(b"ply\nformat binary_little_endian 1.0\nelement vertex 10\nproperty float x\n"
                      b"property float y\nproperty float z\nend_header\n" + b"\0" * 20)
    with pytest.raises(PlyError):
        read_ply_points(str(trunc))
    with pytest.raises(FileNotFoundError):
        load_sample_cloud("NoSuchCloud", str(tmp_path))
