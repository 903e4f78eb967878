"""The committed oracle goldens (tests/golden/make_oracle_goldens.py) are
reproduced bit for bit by the current oracle build (CPU, no GPU)."""
import os
import sys

import numpy as np

from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
import make_oracle_goldens as G  # noqa: E402


def _check(path, fresh):
    gold = np.load(path)
    assert set(gold.files) == set(fresh)
    for k in gold.files:
        np.testing.assert_array_equal(gold[k], np.asarray(fresh[k]), err_msg=k)


def test_lego_A_golden_reproduces():
    _check(os.path.join(GOLDEN, "oracle_lego_A.npz"), G.lego_A())


def test_raster_golden_reproduces():
    _check(os.path.join(GOLDEN, "oracle_raster.npz"), G.raster())
