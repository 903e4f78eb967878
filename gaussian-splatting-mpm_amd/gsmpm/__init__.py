"""gsmpm -- MI355X-native runtime behind the PhysGaussian drop-in modules.

``gsmpm._lib`` binds libgsmpm.so (HIP kernels + C-ABI, include/gsmpm.h).
``gsmpm.sim`` / ``gsmpm.raster`` are the thin torch-facing wrappers the
reference-shaped packages (``mpm_solver``, ``diff_gaussian_rasterization``,
``internel_filling``) are built on.  ``gsmpm.bc`` holds the host-side
boundary-condition scheduling (f64 clock), ``gsmpm.dist`` the
spatial-slab multi-GPU driver.
"""
__all__ = ["sim", "raster", "bc", "dist"]
