"""PLY model format of the trained Gaussians (SURVEY.md §8f "next" row 3).

Mirrors scene/gaussian_model.py:218-318 (construct_list_of_attributes, save_ply,
load_ply) without the ``plyfile`` dependency (absent here): one ``vertex``
element of little-endian float32 properties in the order
    x y z nx ny nz f_dc_0..2 f_rest_0..(3(D+1)^2-4) opacity scale_0..2 rot_0..3
where f_dc / f_rest are the SH coefficients transposed to channel-major
(``features.transpose(1, 2).flatten(start_dim=1)``), normals are zero, and all
values are the pre-activation parameters (log scale, opacity logit, raw
quaternion).  The header is the one ``plyfile`` writes for that element, so the
files interchange with the reference's.  Reading accepts binary little/big
endian and ascii PLY with float/double/int properties, like ``PlyData.read``.
"""
from __future__ import annotations

import os

import numpy as np
import torch

_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
          "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
          "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}


def attribute_names(n_dc: int, n_rest: int, n_scale: int = 3, n_rot: int = 4) -> list:
    """construct_list_of_attributes (scene/gaussian_model.py:218-231)."""
    names = ["x", "y", "z", "nx", "ny", "nz"]
    names += [f"f_dc_{i}" for i in range(n_dc)]
    names += [f"f_rest_{i}" for i in range(n_rest)]
    names.append("opacity")
    names += [f"scale_{i}" for i in range(n_scale)]
    names += [f"rot_{i}" for i in range(n_rot)]
    return names


def save_ply(path: str, g) -> None:
    """save_ply (scene/gaussian_model.py:233-258) for a GaussianModel-like object with
    xyz [P,3], features_dc [P,1,3], features_rest [P,M-1,3], opacity [P,1],
    scaling [P,3], rotation [P,4]."""
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    xyz = g.xyz.detach().float().cpu().numpy()
    f_dc = g.features_dc.detach().transpose(1, 2).flatten(start_dim=1).contiguous().float().cpu().numpy()
    f_rest = g.features_rest.detach().transpose(1, 2).flatten(start_dim=1).contiguous().float().cpu().numpy()
    cols = [xyz, np.zeros_like(xyz), f_dc, f_rest, g.opacity.detach().float().cpu().numpy(),
            g.scaling.detach().float().cpu().numpy(), g.rotation.detach().float().cpu().numpy()]
    data = np.ascontiguousarray(np.concatenate(cols, axis=1), dtype="<f4")
    names = attribute_names(f_dc.shape[1], f_rest.shape[1], cols[5].shape[1], cols[6].shape[1])
    assert data.shape[1] == len(names)
    header = ["ply", "format binary_little_endian 1.0", f"element vertex {data.shape[0]}"]
    header += [f"property float {n}" for n in names]
    header.append("end_header")
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\n").encode("ascii"))
        f.write(data.tobytes())


def store_points_ply(path: str, xyz: np.ndarray, rgb: np.ndarray) -> None:
    """storePly (scene/dataset_readers.py:164-185): x y z nx ny nz as float (zero
    normals), red green blue as uchar, one binary little-endian vertex element."""
    xyz = np.asarray(xyz, dtype="<f4")
    rgb = np.asarray(rgb)
    rec = np.empty(xyz.shape[0], dtype=[(n, "<f4") for n in ("x", "y", "z", "nx", "ny", "nz")] +
                   [(n, "u1") for n in ("red", "green", "blue")])
    for k, n in enumerate(("x", "y", "z")):
        rec[n] = xyz[:, k]
    for n in ("nx", "ny", "nz"):
        rec[n] = 0.0
    for k, n in enumerate(("red", "green", "blue")):
        rec[n] = rgb[:, k].astype(np.uint8)
    header = ["ply", "format binary_little_endian 1.0", f"element vertex {xyz.shape[0]}"]
    header += [f"property float {n}" for n in ("x", "y", "z", "nx", "ny", "nz")]
    header += [f"property uchar {n}" for n in ("red", "green", "blue")]
    header.append("end_header")
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\n").encode("ascii"))
        f.write(rec.tobytes())


def fetch_points_ply(path: str):
    """fetchPly (scene/dataset_readers.py:156-162) -> (positions [N,3], colors [N,3] in
    [0,1], normals [N,3]) as float64 like the reference's np.vstack(...).T / 255."""
    v = read_ply_vertices(path)
    pos = np.vstack([v["x"], v["y"], v["z"]]).T
    col = np.vstack([v["red"], v["green"], v["blue"]]).T / 255.0
    nrm = np.vstack([v["nx"], v["ny"], v["nz"]]).T
    return pos, col, nrm


def read_ply_vertices(path: str) -> dict:
    """The ``vertex`` element of a PLY file as {property name: numpy array}."""
    with open(path, "rb") as f:
        if f.readline().strip() != b"ply":
            raise ValueError(f"{path}: not a PLY file")
        fmt, elements, cur = None, [], None
        while True:
            line = f.readline()
            if not line:
                raise ValueError(f"{path}: truncated header")
            tok = line.decode("ascii").split()
            if not tok or tok[0] in ("comment", "obj_info"):
                continue
            if tok[0] == "format":
                fmt = tok[1]
            elif tok[0] == "element":
                cur = {"name": tok[1], "count": int(tok[2]), "props": []}
                elements.append(cur)
            elif tok[0] == "property":
                if tok[1] == "list":
                    raise ValueError(f"{path}: list properties are not supported")
                cur["props"].append((tok[2], _TYPES[tok[1]]))
            elif tok[0] == "end_header":
                break
        out = None
        for el in elements:
            if fmt == "ascii":
                rows = [f.readline().split() for _ in range(el["count"])]
                arr = np.array(rows, dtype=np.float64).reshape(el["count"], len(el["props"]))
                cols = {n: arr[:, i].astype(t) for i, (n, t) in enumerate(el["props"])}
            else:
                end = "<" if fmt == "binary_little_endian" else ">"
                dt = np.dtype([(n, end + t) for n, t in el["props"]])
                rec = np.frombuffer(f.read(dt.itemsize * el["count"]), dtype=dt, count=el["count"])
                cols = {n: rec[n].astype(rec[n].dtype.newbyteorder("=")) for n, _ in el["props"]}
            if el["name"] == "vertex":
                out = cols
        if out is None:
            raise ValueError(f"{path}: no vertex element")
        return out


def load_ply(path: str, max_sh_degree: int, device="cpu"):
    """load_ply (scene/gaussian_model.py:267-318) -> SynthGaussians (active degree = max)."""
    from synthetic import SynthGaussians

    v = read_ply_vertices(path)
    xyz = np.stack((v["x"], v["y"], v["z"]), axis=1)
    opacities = np.asarray(v["opacity"])[..., None]
    features_dc = np.stack([v[f"f_dc_{c}"] for c in range(3)], axis=1)[..., None]  # [P,3,1]
    rest = sorted((n for n in v if n.startswith("f_rest_")), key=lambda n: int(n.split("_")[-1]))
    if len(rest) != 3 * (max_sh_degree + 1) ** 2 - 3:
        raise ValueError(f"{path}: {len(rest)} f_rest properties, degree {max_sh_degree} needs "
                         f"{3 * (max_sh_degree + 1) ** 2 - 3}")
    features_extra = np.zeros((xyz.shape[0], 0), dtype=np.float32)
    if rest:
        features_extra = np.stack([v[n] for n in rest], axis=1)
    features_extra = features_extra.reshape(xyz.shape[0], 3, (max_sh_degree + 1) ** 2 - 1)
    scales = np.stack([v[n] for n in sorted((n for n in v if n.startswith("scale_")),
                                            key=lambda n: int(n.split("_")[-1]))], axis=1)
    rots = np.stack([v[n] for n in sorted((n for n in v if n.startswith("rot")),
                                          key=lambda n: int(n.split("_")[-1]))], axis=1)

    def t(a):
        return torch.tensor(a, dtype=torch.float, device=device)

    return SynthGaussians(t(xyz), t(features_dc).transpose(1, 2).contiguous(),
                          t(features_extra).transpose(1, 2).contiguous(), t(scales), t(rots), t(opacities),
                          max_sh_degree, max_sh_degree)
