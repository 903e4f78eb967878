"""The host debug build of the oracle: grid-index bounds checks.

The reference runs Taichi without debug=True (/root/reference/main.py:28), so
an out-of-range grid index there is undefined behaviour nobody reports.  The
oracle's debug build (oracle/Makefile `debug` / `asan`, -DOM_DEBUG) checks
every grid index, counts the stencil nodes the restatement skips because they
lie outside the grid, and with GSMPM_ORACLE_STRICT=1 aborts on the first one,
as Taichi's debug mode would stop.  The ASan/UBSan run of the whole CPU suite
is tools/oracle_asan.sh (log under profiles/)."""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

_SCRIPT = r"""
import sys, numpy as np
sys.path.insert(0, {oracle!r})
import oracle as O
L = O.lib()
L.om_debug_skipped.restype = __import__("ctypes").c_long
assert L.om_debug_build() == 1
rng = np.random.default_rng(0)
n, ng = 200, 16
x = rng.uniform({lo}, {hi}, size=(n, 3)).astype(np.float32)
cov = np.tile(np.array([1e-4, 0, 0, 1e-4, 0, 1e-4], np.float32), (n, 1))
vol = np.full(n, 1e-6, np.float32)
sim = O.OracleMPM(x, cov, vol, n_grid=ng, grid_extent=1.0, material="jelly", E=2e4, nu=0.3, density=100.0,
                  gravity=(0.0, 0.0, -9.8))
for _ in range(3):
    sim.substep(1e-4, None, [])
print("SKIPPED", L.om_debug_skipped())
"""


def _run(lo, hi, strict=False):
    env = dict(os.environ, GSMPM_ORACLE_VARIANT="debug", OMP_NUM_THREADS="1")
    env.pop("GSMPM_ORACLE_STRICT", None)
    if strict:
        env["GSMPM_ORACLE_STRICT"] = "1"
    code = _SCRIPT.format(oracle=os.path.join(ROOT, "oracle"), lo=lo, hi=hi)
    return subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)


def _skipped(p):
    assert p.returncode == 0, p.stderr[-2000:]
    return int(p.stdout.split("SKIPPED")[1])


def test_debug_build_interior_scene_has_no_out_of_grid_access():
    assert _skipped(_run(0.3, 0.7)) == 0


def test_debug_build_counts_stencils_outside_the_grid():
    # particles in the last cell: base = trunc(x / dx - 0.5) = 15, so nodes 16 and 17 fall outside
    assert _skipped(_run(0.97, 0.999)) > 0


def test_debug_build_strict_stops_at_the_first_out_of_grid_node():
    p = _run(0.97, 0.999, strict=True)
    assert p.returncode != 0
    assert "outside the 16^3 grid (strict)" in p.stderr


def test_release_build_reports_no_debug():
    import oracle as O
    import ctypes
    L = O.lib()
    L.om_debug_skipped.restype = ctypes.c_long
    if os.environ.get("GSMPM_ORACLE_VARIANT"):
        assert L.om_debug_build() == 1
    else:
        assert L.om_debug_build() == 0 and L.om_debug_skipped() == -1
    assert np.isfinite(1.0)
