"""On-disk formats of a trained model.

* `point_cloud.ply` -- binary little-endian PLY, one `vertex` element with float32 properties
  x y z nx ny nz f_dc_0..2 f_rest_0..(3K-4) opacity scale_0..2 rot_0..3, in that order
  (scene/gaussian_model.py:214-226 construct_list_of_attributes, :250-267 save_ply).  f_dc / f_rest
  are the SH coefficients channel-major (features.transpose(1, 2).flatten), normals are zero,
  opacity / scale / rot are the raw (pre-activation) parameters.  load_ply (:274-314) reads them
  back, sorting f_rest_ / scale_ / rot names by their numeric suffix.
* `deformation.pth`, `deformation_table.pth`, `deformation_accum.pth` -- torch.save of the
  deformation network's state dict and the two per-Gaussian tensors (gaussian_model.py:233-249);
  loaded with weights_only=True (tensors only, nothing executed from the file).
* scene/__init__.py:143-150 lays them out as <model>/point_cloud/iteration_<i>/{point_cloud.ply, *.pth}.

The PLY codec is self-contained (the reference uses the `plyfile` package, absent here); it writes
the header plyfile writes for 'f4' properties and reads binary_little_endian / binary_big_endian /
ascii files with float, double, int and uchar properties.
"""
import os

import numpy as np
import torch
import torch.nn as nn

_PLY_TYPES = {"char": "i1", "int8": "i1", "uchar": "u1", "uint8": "u1", "short": "i2", "int16": "i2",
              "ushort": "u2", "uint16": "u2", "int": "i4", "int32": "i4", "uint": "u4", "uint32": "u4",
              "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}


def attribute_names(n_dc, n_rest, n_scale=3, n_rot=4):
    """gaussian_model.py:214-226"""
    return (["x", "y", "z", "nx", "ny", "nz"] + [f"f_dc_{i}" for i in range(n_dc)] +
            [f"f_rest_{i}" for i in range(n_rest)] + ["opacity"] + [f"scale_{i}" for i in range(n_scale)] +
            [f"rot_{i}" for i in range(n_rot)])


def write_ply(path, columns):
    """columns: ordered dict name -> float32 (N,) arrays.  Binary little-endian, float properties."""
    names = list(columns)
    n = len(columns[names[0]]) if names else 0
    rec = np.empty(n, dtype=[(k, "<f4") for k in names])
    for k in names:
        rec[k] = np.asarray(columns[k], np.float32)
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    header = "ply\nformat binary_little_endian 1.0\nelement vertex %d\n" % n
    header += "".join("property float %s\n" % k for k in names) + "end_header\n"
    with open(path, "wb") as f:
        f.write(header.encode("ascii"))
        f.write(rec.tobytes())


def read_ply(path):
    """Returns {property name: (N,) array} of the first element (the vertex element)."""
    with open(path, "rb") as f:
        if f.readline().strip() != b"ply":
            raise ValueError(f"{path}: not a PLY file")
        fmt, elements, cur = None, [], None
        while True:
            line = f.readline()
            if not line:
                raise ValueError(f"{path}: truncated header")
            tok = line.decode("ascii").strip().split()
            if not tok or tok[0] in ("comment", "obj_info"):
                continue
            if tok[0] == "format":
                fmt = tok[1]
            elif tok[0] == "element":
                cur = [tok[1], int(tok[2]), []]
                elements.append(cur)
            elif tok[0] == "property":
                if tok[1] == "list":
                    raise ValueError(f"{path}: list properties are not supported")
                cur[2].append((tok[2], _PLY_TYPES[tok[1]]))
            elif tok[0] == "end_header":
                break
        name, n, props = elements[0]
        if fmt == "ascii":
            data = np.loadtxt(f, max_rows=n, ndmin=2)
            return {p: data[:, i].astype(t) for i, (p, t) in enumerate(props)}
        endian = "<" if fmt == "binary_little_endian" else ">"
        dt = np.dtype([(p, endian + t) for p, t in props])
        rec = np.frombuffer(f.read(dt.itemsize * n), dtype=dt, count=n)
        return {p: rec[p].astype(rec[p].dtype.newbyteorder("=")) for p, _ in props}


def save_gaussians(path, g):
    """gaussian_model.py:250-267 save_ply"""
    xyz = g._xyz.detach().cpu().numpy()
    f_dc = g._features_dc.detach().transpose(1, 2).flatten(start_dim=1).contiguous().cpu().numpy()
    f_rest = g._features_rest.detach().transpose(1, 2).flatten(start_dim=1).contiguous().cpu().numpy()
    opac = g._opacity.detach().cpu().numpy()
    scale = g._scaling.detach().cpu().numpy()
    rot = g._rotation.detach().cpu().numpy()
    names = attribute_names(f_dc.shape[1], f_rest.shape[1], scale.shape[1], rot.shape[1])
    attrs = np.concatenate((xyz, np.zeros_like(xyz), f_dc, f_rest, opac, scale, rot), axis=1)
    write_ply(path, {k: attrs[:, i] for i, k in enumerate(names)})


def load_gaussians(path, g, device="cuda"):
    """gaussian_model.py:274-314 load_ply"""
    el = read_ply(path)
    xyz = np.stack((el["x"], el["y"], el["z"]), axis=1)
    opac = np.asarray(el["opacity"])[..., None]
    fdc = np.zeros((xyz.shape[0], 3, 1))
    for c in range(3):
        fdc[:, c, 0] = el[f"f_dc_{c}"]
    by_suffix = lambda prefix: sorted([k for k in el if k.startswith(prefix)], key=lambda x: int(x.split("_")[-1]))
    extra = by_suffix("f_rest_")
    assert len(extra) == 3 * (g.max_sh_degree + 1) ** 2 - 3
    fextra = np.stack([el[k] for k in extra], axis=1).reshape(xyz.shape[0], 3, (g.max_sh_degree + 1) ** 2 - 1)
    scales = np.stack([el[k] for k in by_suffix("scale_")], axis=1)
    rots = np.stack([el[k] for k in by_suffix("rot")], axis=1)
    t = lambda a: torch.tensor(a, dtype=torch.float, device=device)
    g._xyz = nn.Parameter(t(xyz).requires_grad_(True))
    g._features_dc = nn.Parameter(t(fdc).transpose(1, 2).contiguous().requires_grad_(True))
    g._features_rest = nn.Parameter(t(fextra).transpose(1, 2).contiguous().requires_grad_(True))
    g._opacity = nn.Parameter(t(opac).requires_grad_(True))
    g._scaling = nn.Parameter(t(scales).requires_grad_(True))
    g._rotation = nn.Parameter(t(rots).requires_grad_(True))
    g.active_sh_degree = g.max_sh_degree


def save_deformation(path, g):
    """gaussian_model.py:246-249"""
    os.makedirs(path, exist_ok=True)
    torch.save(g._deformation.state_dict(), os.path.join(path, "deformation.pth"))
    torch.save(g._deformation_table, os.path.join(path, "deformation_table.pth"))
    torch.save(g._deformation_accum, os.path.join(path, "deformation_accum.pth"))


def load_deformation(path, g, device="cuda"):
    """gaussian_model.py:233-245 load_model, with tensor-only (weights_only) loading."""
    sd = torch.load(os.path.join(path, "deformation.pth"), map_location=device, weights_only=True)
    g._deformation.load_state_dict(sd)
    g._deformation = g._deformation.to(device)
    P = g.get_xyz.shape[0]
    g._deformation_table = torch.gt(torch.ones((P), device=device), 0)
    g._deformation_accum = torch.zeros((P, 3), device=device)
    for name in ("deformation_table", "deformation_accum"):
        f = os.path.join(path, name + ".pth")
        if os.path.exists(f):
            setattr(g, "_" + name, torch.load(f, map_location=device, weights_only=True))
    g.max_radii2D = torch.zeros((P), device=device)


def save_model(model_path, iteration, g, stage="fine"):
    """scene/__init__.py:143-150: <model>/point_cloud/iteration_<i>/ (coarse saves go to coarse_iteration_<i>)."""
    d = os.path.join(model_path, "point_cloud", ("coarse_iteration_{}" if stage == "coarse" else "iteration_{}").format(iteration))
    save_gaussians(os.path.join(d, "point_cloud.ply"), g)
    save_deformation(d, g)
    return d


def load_model(model_path, iteration, g, device="cuda"):
    d = os.path.join(model_path, "point_cloud", "iteration_{}".format(iteration))
    load_gaussians(os.path.join(d, "point_cloud.ply"), g, device)
    load_deformation(d, g, device)
    return d
