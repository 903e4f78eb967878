"""Cut a 64-Gaussian PLY fixture out of the reference's real 3DGS data file
models/udon/point_cloud/iteration_30000/point_cloud4.ply (MIT, LICENSE:1;
2,153 Gaussians) and record the upstream getter values computed with plain
numpy, independent of gaussian_splatting/scene.

The PLY is read as data (header + little-endian f32 records); no reference
code runs.  Run in the build container only; outputs are committed:
  udon64.ply, udon64_expected.npz, and the whole file as udon_point_cloud4.ply
  (round 5: the GPU path's one real 3DGS scene, tests/test_gpu_udon.py)
"""
import os

import numpy as np

SRC = "/root/reference/models/udon/point_cloud/iteration_30000/point_cloud4.ply"
HERE = os.path.dirname(os.path.abspath(__file__))
N = 64


def main():
    with open(SRC, "rb") as f:
        raw = f.read()
    with open(os.path.join(HERE, "udon_point_cloud4.ply"), "wb") as f:  # the whole scene, byte for byte
        f.write(raw)
    end = raw.index(b"end_header\n") + len(b"end_header\n")
    lines = raw[:end].decode("ascii").splitlines()
    props = [l.split()[2] for l in lines if l.startswith("property")]
    n = int(next(l for l in lines if l.startswith("element vertex")).split()[-1])
    data = np.frombuffer(raw[end:end + 4 * n * len(props)], "<f4").reshape(n, len(props))[:N]
    head = "\n".join(l if not l.startswith("element vertex") else f"element vertex {N}" for l in lines) + "\n"
    with open(os.path.join(HERE, "udon64.ply"), "wb") as f:
        f.write(head.encode("ascii"))
        f.write(data.astype("<f4").tobytes())

    col = {p: data[:, i].astype(np.float64) for i, p in enumerate(props)}
    xyz = np.stack([col["x"], col["y"], col["z"]], 1)
    opacity = 1.0 / (1.0 + np.exp(-col["opacity"]))
    s = np.exp(np.stack([col[f"scale_{i}"] for i in range(3)], 1))
    q = np.stack([col[f"rot_{i}"] for i in range(4)], 1)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    w, x, y, z = q.T
    R = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                  2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                  2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], 1).reshape(-1, 3, 3)
    L = R * s[:, None, :]
    S = L @ L.transpose(0, 2, 1)
    cov6 = np.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], 1)
    dc = np.stack([col[f"f_dc_{i}"] for i in range(3)], 1)[:, None, :]
    rest = np.stack([col[f"f_rest_{i}"] for i in range(45)], 1).reshape(N, 3, 15).transpose(0, 2, 1)
    feats = np.concatenate([dc, rest], 1)
    np.savez(os.path.join(HERE, "udon64_expected.npz"), xyz=xyz, opacity=opacity, cov6=cov6, features=feats,
             scaling=s, rotation=q)
    print("wrote udon64.ply, udon64_expected.npz, udon_point_cloud4.ply")


if __name__ == "__main__":
    main()
