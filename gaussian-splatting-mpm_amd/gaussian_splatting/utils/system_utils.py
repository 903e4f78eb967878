"""searchForMaxIteration (upstream gaussian-splatting utils/system_utils.py)."""
import os


def searchForMaxIteration(folder):
    its = [int(name.split("_")[-1]) for name in os.listdir(folder)]
    return max(its)
