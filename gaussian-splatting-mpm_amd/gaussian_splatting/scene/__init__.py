"""GaussianModel: the subset of the upstream 3DGS model main.py uses.

PLY layout (Appendix C of SURVEY.md; verified on the reference's real
models/udon/point_cloud/iteration_30000/point_cloud4.ply): binary little-endian
float32 vertex properties x y z nx ny nz f_dc_0..2 f_rest_0..44 opacity
scale_0..2 rot_0..3.  Getters as upstream: opacity = sigmoid, scaling = exp,
rotation = normalised quaternion (w,x,y,z), features = [dc | rest] (N,16,3),
covariance = upper-6 of (R S)(R S)^T.
"""
from __future__ import annotations

import os

import numpy as np
import torch


def _read_ply(path):
    with open(path, "rb") as f:
        head = b""
        while not head.endswith(b"end_header\n"):
            line = f.readline()
            if not line:
                raise ValueError(f"{path}: truncated PLY header")
            head += line
        lines = head.decode("ascii").splitlines()
        if lines[0] != "ply":
            raise ValueError(f"{path}: not a PLY file")
        fmt = next(l for l in lines if l.startswith("format"))
        if "binary_little_endian" not in fmt:
            raise ValueError(f"{path}: only binary_little_endian PLY is supported")
        n = int(next(l for l in lines if l.startswith("element vertex")).split()[-1])
        props = []
        for l in lines:
            if l.startswith("property"):
                t, name = l.split()[1:3]
                if t not in ("float", "float32"):
                    raise ValueError(f"{path}: property {name} has type {t}, expected float")
                props.append(name)
        data = np.frombuffer(f.read(4 * n * len(props)), dtype="<f4").reshape(n, len(props))
    return {p: data[:, i] for i, p in enumerate(props)}, n


def _sorted_names(cols, prefix):
    return sorted([k for k in cols if k.startswith(prefix)], key=lambda s: int(s.split("_")[-1]))


def _build_rotation(r):
    q = r / torch.sqrt(r[:, 0] ** 2 + r[:, 1] ** 2 + r[:, 2] ** 2 + r[:, 3] ** 2)[:, None]
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], dim=1)
    return R.reshape(-1, 3, 3)


class GaussianModel:
    def __init__(self, sh_degree: int, device="cuda"):
        self.max_sh_degree = sh_degree
        self.active_sh_degree = 0
        self.device = device
        z = lambda *s: torch.empty(*s, device=device)
        self._xyz = z(0, 3)
        self._features_dc = z(0, 1, 3)
        self._features_rest = z(0, (sh_degree + 1) ** 2 - 1, 3)
        self._opacity = z(0, 1)
        self._scaling = z(0, 3)
        self._rotation = z(0, 4)

    # ------------------------------------------------------------- getters --
    @property
    def get_xyz(self):
        return self._xyz

    @property
    def get_scaling(self):
        return torch.exp(self._scaling)

    @property
    def get_rotation(self):
        return torch.nn.functional.normalize(self._rotation)

    @property
    def get_opacity(self):
        return torch.sigmoid(self._opacity)

    @property
    def get_features(self):
        return torch.cat((self._features_dc, self._features_rest), dim=1)

    def get_covariance(self, scaling_modifier=1):
        s = scaling_modifier * self.get_scaling
        L = _build_rotation(self._rotation) * s[:, None, :]  # R @ diag(s)
        S = L @ L.transpose(1, 2)
        return torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], dim=1)

    # ------------------------------------------------------------------ io --
    def _arrays_from_ply(self, path):
        cols, n = _read_ply(path)
        xyz = np.stack([cols["x"], cols["y"], cols["z"]], axis=1)
        dc = np.stack([cols["f_dc_0"], cols["f_dc_1"], cols["f_dc_2"]], axis=1)[:, None, :]  # (N,1,3)
        rest_names = _sorted_names(cols, "f_rest_")
        k = (self.max_sh_degree + 1) ** 2 - 1
        assert len(rest_names) == 3 * k, f"expected {3 * k} f_rest_* properties, found {len(rest_names)}"
        rest = np.stack([cols[nm] for nm in rest_names], axis=1).reshape(n, 3, k).transpose(0, 2, 1)  # (N,k,3)
        opa = cols["opacity"][:, None]
        scl = np.stack([cols[nm] for nm in _sorted_names(cols, "scale_")], axis=1)
        rot = np.stack([cols[nm] for nm in _sorted_names(cols, "rot")], axis=1)
        return xyz, dc, rest, opa, scl, rot

    def _set(self, xyz, dc, rest, opa, scl, rot):
        t = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float, device=self.device)
        self._xyz, self._features_dc, self._features_rest = t(xyz), t(dc), t(rest)
        self._opacity, self._scaling, self._rotation = t(opa), t(scl), t(rot)
        self.active_sh_degree = self.max_sh_degree

    def load_ply(self, path):
        self._set(*self._arrays_from_ply(path))

    def load_multiple_plys(self, paths):
        """Concatenate several PLYs (the reference's fork, main.py:47); missing
        files are skipped (lego has no point_cloud2.ply)."""
        parts = [self._arrays_from_ply(p) for p in paths if os.path.exists(p)]
        if not parts:
            raise FileNotFoundError(f"none of {paths} exists")
        self._set(*[np.concatenate([p[i] for p in parts], axis=0) for i in range(6)])

    def save_ply(self, path):
        os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
        n = self._xyz.shape[0]
        k = self._features_rest.shape[1]
        cols = [self._xyz, torch.zeros_like(self._xyz),
                self._features_dc.transpose(1, 2).flatten(start_dim=1),
                self._features_rest.transpose(1, 2).flatten(start_dim=1),
                self._opacity, self._scaling, self._rotation]
        data = torch.cat([c.detach().float().reshape(n, -1) for c in cols], dim=1).cpu().numpy().astype("<f4")
        names = (["x", "y", "z", "nx", "ny", "nz"] + [f"f_dc_{i}" for i in range(3)] +
                 [f"f_rest_{i}" for i in range(3 * k)] + ["opacity"] + [f"scale_{i}" for i in range(3)] +
                 [f"rot_{i}" for i in range(4)])
        head = "ply\nformat binary_little_endian 1.0\nelement vertex %d\n" % n
        head += "".join(f"property float {nm}\n" for nm in names) + "end_header\n"
        with open(path, "wb") as f:
            f.write(head.encode("ascii"))
            f.write(data.tobytes())

    # ----------------------------------------------------------- synthetic --
    def init_synthetic(self, n, seed=0, box=((-0.65, -0.65, -0.55), (0.65, 0.65, 0.55))):
        """Lego-like synthetic Gaussians: the lego PLY in the
        reference is a git-LFS pointer, not data."""
        rng = np.random.default_rng(seed)
        lo, hi = np.asarray(box[0]), np.asarray(box[1])
        k = (self.max_sh_degree + 1) ** 2 - 1
        xyz = rng.uniform(lo, hi, size=(n, 3))
        scl = rng.normal(-4.5, 0.5, size=(n, 3))
        rot = rng.normal(0.0, 1.0, size=(n, 4))
        rot /= np.linalg.norm(rot, axis=1, keepdims=True)
        opa = rng.normal(2.0, 1.5, size=(n, 1))
        dc = rng.normal(0.5, 0.5, size=(n, 1, 3))
        rest = rng.normal(0.0, 0.05, size=(n, k, 3))
        self._set(xyz, dc, rest, opa, scl, rot)
        return self
