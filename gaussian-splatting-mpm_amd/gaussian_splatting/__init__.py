"""Minimal stand-in for the graphdeco ``gaussian_splatting`` submodule.

The reference's submodule directory is empty (.gitmodules:1-3); main.py only
uses GaussianModel's PLY loader/getters, graphics_utils camera math and
system_utils.searchForMaxIteration (main.py:17-22,37-47,64,74,100-101,135-137,235).
Those are restated here from the public 3DGS code; training code is out of scope.
"""
