"""Material codes (mpm_solver/utils.py:5-10).

The reference's Taichi kernels that lived here (stress, p2g, grid update, g2p,
postprocess, mu/lam, mass) are replaced by the HIP kernels in
gaussian-splatting-mpm_amd/csrc/mpm.hip; see DESIGN.md for the mapping.
"""
material_types = {
    "jelly": 0,
    "metal": 1,
    "sand": 2,
    "foam": 3,
}
