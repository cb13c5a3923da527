"""CPU side of the C shim test: the program compiles with gcc -Wall -Wextra -Werror against
include/hmsc_amd.h alone, and the TD model file round-trips through model_io."""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(HERE, "capi"))
from model_io import model_arrays, read_results, write_model  # noqa: E402


def test_shim_compiles_with_gcc(tmp_path):
    obj = str(tmp_path / "shim.o")
    p = subprocess.run(["gcc", "-std=c99", "-Wall", "-Wextra", "-Werror", "-c", "-I", os.path.join(ROOT, "include"),
                        os.path.join(HERE, "capi", "shim_run.c"), "-o", obj], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr


def test_model_file_round_trip(tmp_path):
    from test_golden_td import td_model
    hM = td_model()
    path = str(tmp_path / "m.bin")
    write_model(hM, path)
    back = read_results(path)
    ref = model_arrays(hM)
    assert set(back) == set(ref)
    for k, v in ref.items():
        np.testing.assert_array_equal(back[k], v)
    # what the shim marshals for TD: phylogeny spectral form and the spatial plot level
    assert back["C_values"].size == hM.ns and back["rhopw"].size == 2 * hM.rhopw.shape[0]
    assert back["spatialMethod"].tolist() == [0, 1] and back["sCoord1"].size == 2 * int(hM.np[1])
