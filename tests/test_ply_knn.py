"""§8f "next" rows 3-4: the PLY model format (scene/gaussian_model.py:218-318,
scene/dataset_readers.py:156-185) and distCUDA2 (mean squared distance to the 3
nearest neighbours, scene/gaussian_model.py:153-155).

PLY: CPU tests pinned to the reference's own save_ply / load_ply, run in the build
container under a recording ``plyfile`` stand-in (tests/golden/ply.npz, made by
tests/golden/make_golden.py:capture_ply): the vertex array's names, formats and
bytes, and the parameters load_ply rebuilds (also from a shuffled property order).
Plus bit-exact round trips and ascii / big-endian / uchar reading.  The header text
itself is plyfile's (absent here): "property float <name>" for an 'f4' field.
kNN: the C ABI's argument checks on CPU; exactness against scipy's cKDTree on GPU
(simple-knn itself is an absent submodule: its published contract is the exact
mean of the three smallest squared distances to other points)."""
import numpy as np
import pytest
import torch

import ply_io
import synthetic


# ------------------------------------------------------------------ PLY (CPU)
def test_attribute_names_follow_reference_order():
    names = ply_io.attribute_names(3, 45)
    assert len(names) == 62
    assert names[:9] == ["x", "y", "z", "nx", "ny", "nz", "f_dc_0", "f_dc_1", "f_dc_2"]
    assert names[9] == "f_rest_0" and names[53] == "f_rest_44"
    assert names[54:] == ["opacity", "scale_0", "scale_1", "scale_2", "rot_0", "rot_1", "rot_2", "rot_3"]


@pytest.mark.parametrize("degree", [0, 1, 3])
def test_save_load_round_trip_is_bit_exact(tmp_path, degree):
    g = synthetic.make_gaussians(777, degree, seed=degree)
    path = str(tmp_path / "pc" / "point_cloud.ply")
    ply_io.save_ply(path, g)
    raw = open(path, "rb").read()
    head, body = raw.split(b"end_header\n", 1)
    lines = head.decode().split("\n")
    assert lines[:3] == ["ply", "format binary_little_endian 1.0", "element vertex 777"]
    n_rest = 3 * ((degree + 1) ** 2 - 1)
    names = ply_io.attribute_names(3, n_rest)
    assert lines[3:-1] == [f"property float {n}" for n in names]
    assert len(body) == 777 * len(names) * 4
    # the channel-major SH layout of the reference: f_dc_c = features_dc[:, 0, c],
    # f_rest_(c * (M-1) + j) = features_rest[:, j, c]
    rec = np.frombuffer(body, dtype="<f4").reshape(777, len(names))
    np.testing.assert_array_equal(rec[:, 6:9], g.features_dc[:, 0, :].numpy())
    if degree:
        M1 = (degree + 1) ** 2 - 1
        np.testing.assert_array_equal(rec[:, 9 + 1 * M1 + 2], g.features_rest[:, 2, 1].numpy())
    np.testing.assert_array_equal(rec[:, 3:6], 0)
    h = ply_io.load_ply(path, degree)
    assert h.active_sh_degree == degree and h.max_sh_degree == degree
    for a, b in zip(g.params(), h.params()):
        assert a.shape == b.shape
        assert torch.equal(a, b)


_PARAMS = ("xyz", "features_dc", "features_rest", "opacity", "scaling", "rotation")


def _golden_ply():
    from pathlib import Path

    return np.load(Path(__file__).parent / "golden" / "ply.npz")


def _golden_model(z, key):
    deg = int(key[1])
    t = {n: torch.from_numpy(z[key + "in_" + n]) for n in _PARAMS}
    return synthetic.SynthGaussians(t["xyz"], t["features_dc"], t["features_rest"], t["scaling"], t["rotation"],
                                    t["opacity"], deg, deg)


@pytest.mark.parametrize("degree", [0, 1, 3])
def test_save_ply_equals_reference_save_ply(tmp_path, degree):
    """The body save_ply writes is, byte for byte, the structured array the reference's
    own save_ply (scene/gaussian_model.py:240-258) hands PlyElement.describe, with the
    same property names, order and formats (tests/golden/make_golden.py:capture_ply)."""
    z, key = _golden_ply(), f"d{degree}_"
    path = str(tmp_path / "point_cloud.ply")
    ply_io.save_ply(path, _golden_model(z, key))
    head, body = open(path, "rb").read().split(b"end_header\n", 1)
    props = [ln.split() for ln in head.decode().split("\n")[3:-1]]
    assert [p[2] for p in props] == list(z[key + "names"])
    # plyfile names an f4 field "float"
    assert all(p[1] == "float" for p in props) and set(z[key + "formats"]) == {"<f4"}
    assert body == z[key + "body"].tobytes()


@pytest.mark.parametrize("degree", [0, 1, 3])
@pytest.mark.parametrize("order", ["canonical", "shuffled"])
def test_load_ply_equals_reference_load_ply(tmp_path, degree, order):
    """load_ply rebuilds the parameters the reference's own load_ply (scene/
    gaussian_model.py:267-318) rebuilt from the same vertex data, bit for bit — also
    from a file whose properties come in a shuffled order (its numeric-suffix sorts)."""
    z, key = _golden_ply(), f"d{degree}_"
    names = list(z[key + "names"])
    rec = np.frombuffer(z[key + "body"].tobytes(), dtype=[(n, "<f4") for n in names])
    if order == "shuffled":
        names = list(z[key + "shuffled_names"])
    hdr = ["ply", "format binary_little_endian 1.0", f"element vertex {rec.shape[0]}"]
    hdr += [f"property float {n}" for n in names]
    body = np.empty(rec.shape[0], dtype=[(n, "<f4") for n in names])
    for n in names:
        body[n] = rec[n]
    path = tmp_path / "m.ply"
    _write(path, hdr, body.tobytes())
    h = ply_io.load_ply(str(path), degree)
    tag = "load_" if order == "canonical" else "load_shuffled_"
    for n in _PARAMS:
        want = z[key + tag + n]
        got = getattr(h, n).numpy()
        assert got.shape == want.shape and got.dtype == want.dtype, n
        np.testing.assert_array_equal(got, want, err_msg=n)
    # and the reference's round trip is the identity on the parameters it saved
    for n in _PARAMS:
        np.testing.assert_array_equal(z[key + tag + n], z[key + "in_" + n], err_msg=n)


def test_load_rejects_wrong_sh_degree(tmp_path):
    g = synthetic.make_gaussians(10, 1, seed=0)
    path = str(tmp_path / "m.ply")
    ply_io.save_ply(path, g)
    with pytest.raises(ValueError, match="f_rest"):
        ply_io.load_ply(path, 3)


def _write(path, header, body):
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\nend_header\n").encode())
        f.write(body)


def test_read_ascii_big_endian_and_extra_elements(tmp_path):
    rows = np.array([[1.5, -2.0, 3.25], [0.0, 7.0, -1.0]], dtype=np.float32)
    hdr = ["ply", "format ascii 1.0", "comment made by hand", "element vertex 2", "property float x",
           "property double y", "property int z", "element face 1", "property float w"]
    _write(tmp_path / "a.ply", hdr, b"1.5 -2.0 3\n0 7 -1\n9\n")
    v = ply_io.read_ply_vertices(str(tmp_path / "a.ply"))
    np.testing.assert_array_equal(v["x"], rows[:, 0])
    np.testing.assert_array_equal(v["y"], rows[:, 1])
    assert v["z"].dtype == np.int32 and list(v["z"]) == [3, -1]
    hdr = ["ply", "format binary_big_endian 1.0", "element vertex 2", "property float x", "property float y",
           "property float z"]
    _write(tmp_path / "b.ply", hdr, rows.astype(">f4").tobytes())
    v = ply_io.read_ply_vertices(str(tmp_path / "b.ply"))
    for k, n in enumerate("xyz"):
        np.testing.assert_array_equal(v[n], rows[:, k])
    with pytest.raises(ValueError, match="not a PLY"):
        _write(tmp_path / "c.ply", ["nope"], b"")
        ply_io.read_ply_vertices(str(tmp_path / "c.ply"))


def test_points_ply_round_trip(tmp_path):
    rng = np.random.default_rng(0)
    xyz = rng.standard_normal((300, 3)).astype(np.float32)
    rgb = rng.integers(0, 256, (300, 3))
    path = str(tmp_path / "points3D.ply")
    ply_io.store_points_ply(path, xyz, rgb)
    head = open(path, "rb").read().split(b"end_header\n")[0].decode().split("\n")
    assert head[-4:-1] == ["property uchar red", "property uchar green", "property uchar blue"]
    pos, col, nrm = ply_io.fetch_points_ply(path)
    np.testing.assert_array_equal(pos, xyz)
    np.testing.assert_array_equal(col, rgb / 255.0)
    np.testing.assert_array_equal(nrm, 0)


# ------------------------------------------------------------------ kNN ABI (CPU)
def test_knn_abi_validation():
    from diff_gaussian_rasterization import _C

    lib = _C.load_library()
    assert lib.gsr_knn_mean_dist2(-1, None, None, None, None) != 0
    assert "P must be" in lib.gsr_last_error().decode()
    assert lib.gsr_knn_mean_dist2(0, None, None, None, None) == 0
    assert lib.gsr_knn_mean_dist2(5, None, None, None, None) != 0
    assert "NULL" in lib.gsr_last_error().decode()
    assert lib.gsr_knn_scratch_bytes(1000) >= 1000 * 20
    assert lib.gsr_knn_scratch_bytes(0) == 0


# ------------------------------------------------------------------ kNN (GPU)
def _knn_ref(pts):
    from scipy.spatial import cKDTree

    p64 = pts.astype(np.float64)
    k = min(4, len(pts))
    d, _ = cKDTree(p64).query(p64, k=k)
    d = np.asarray(d).reshape(len(pts), k)[:, 1:] ** 2
    out = np.full((len(pts), 3), np.finfo(np.float32).max, dtype=np.float64)
    out[:, : d.shape[1]] = d
    return out


def _clouds():
    rng = np.random.default_rng(7)
    yield "uniform", rng.uniform(-3, 3, (200_000, 3))
    centers = rng.normal(0, 10, (40, 3))
    blob = centers[rng.integers(0, 40, 100_000)] + rng.normal(0, 0.05, (100_000, 3))
    yield "clustered+outliers", np.concatenate([blob, rng.uniform(-500, 500, (200, 3))])
    plane = rng.uniform(-1, 1, (50_000, 3))
    plane[:, 2] = 0.25
    yield "planar", plane
    base = rng.uniform(0, 1, (5000, 3))
    yield "duplicates", np.concatenate([base, base, base[:100]])
    yield "line", np.stack([np.linspace(0, 1, 3000), np.zeros(3000), np.zeros(3000)], 1)


@pytest.mark.gpu
@pytest.mark.parametrize("name,pts", list(_clouds()), ids=[c[0] for c in _clouds()])
def test_knn_is_exact(dev, name, pts):
    import train_ops

    p32 = pts.astype(np.float32)
    got = train_ops.dist_knn3(torch.from_numpy(p32).to(dev)).cpu().numpy()
    # the 3 nearest squared distances from float32 coordinates (rounding of the
    # float32 difference products: relative 1e-6 plus an absolute floor)
    want = _knn_ref(p32).mean(axis=1)
    np.testing.assert_allclose(got, want, rtol=2e-6, atol=1e-12 * max(1.0, float(np.abs(p32).max()) ** 2))


@pytest.mark.gpu
@pytest.mark.parametrize("P", [1, 2, 3, 4, 5, 64])
def test_knn_small_point_counts(dev, P):
    import train_ops

    p = np.random.default_rng(P).uniform(-1, 1, (P, 3)).astype(np.float32)
    got = train_ops.dist_knn3(torch.from_numpy(p).to(dev)).cpu().numpy().astype(np.float64)
    ref = _knn_ref(p)
    want = ref.sum(axis=1) / 3.0
    big = ~np.isfinite(np.float32(want)) | (want > 1e37)
    assert np.all(np.isinf(got[big]) | (got[big] > 1e37))
    np.testing.assert_allclose(got[~big], want[~big], rtol=2e-6)
    assert train_ops.dist_knn3(torch.zeros(0, 3, device=dev)).shape == (0,)


@pytest.mark.gpu
def test_create_from_pcd_matches_reference_formula(dev):
    import train_ops

    rng = np.random.default_rng(3)
    pts = rng.uniform(-2, 2, (20_000, 3)).astype(np.float32)
    col = rng.uniform(0, 1, (20_000, 3))
    g = train_ops.create_from_pcd(pts, col, 3, dev)
    assert g.features_rest.shape == (20_000, 15, 3) and torch.all(g.features_rest == 0)
    torch.testing.assert_close(g.features_dc[:, 0, :].cpu(), ((torch.tensor(col).float() - 0.5) / 0.28209479177387814))
    d2 = np.maximum(_knn_ref(pts).mean(axis=1), 1e-7)
    want = np.log(np.sqrt(d2))
    np.testing.assert_allclose(g.scaling.cpu().numpy(), np.repeat(want[:, None], 3, 1), rtol=0, atol=2e-6)
    assert torch.all(g.rotation.cpu() == torch.tensor([1.0, 0, 0, 0]))
    torch.testing.assert_close(torch.sigmoid(g.opacity).cpu(), torch.full((20_000, 1), 0.1))
