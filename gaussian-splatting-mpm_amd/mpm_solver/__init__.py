"""Drop-in for the reference's ``mpm_solver`` package (mpm_solver/*.py).

``MPM_Simulator`` keeps the reference's constructor, methods and state
attributes; the substep itself runs as three fused HIP kernels in
libgsmpm.so (gsmpm_mpm_step), replayed from a cached hipGraph.
"""
