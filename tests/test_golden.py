"""The oracle still reproduces the committed golden fixtures, CPU only.

tests/golden/make_golden.py wrote each fixture from fixed seeds with injected randomness; here
every case is rebuilt the same way and its inputs and outputs are compared with the stored
arrays.  This freezes the restatement for the configurations pinned only by reading the
reference (NeRFLE at 64 / 256 depths and with the envmap light, PlainNeRF, Path with and without
shadow rays, FoV camera + PointLights + Diffuse / Conductor, DTU camera + render)."""
import os

import numpy as np
import pytest
import torch

from tests.golden import make_golden as G

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name", sorted(G.CASES))
def test_oracle_reproduces_golden(name):
    path = os.path.join(HERE, name + ".npz")
    assert os.path.exists(path), f"missing fixture {path}: run tests/golden/make_golden.py"
    want = np.load(path)  # allow_pickle=False (default): plain arrays only
    threads = torch.get_num_threads()
    torch.set_num_threads(1)  # the summation order the fixtures were written with
    try:
        got = G.to_numpy(G.CASES[name]())
    finally:
        torch.set_num_threads(threads)
    assert set(got) == set(want.files)
    # construction order (same seeds -> same weights)
    assert abs(float(got["weights"]) - float(want["weights"])) <= 1e-9 * float(want["weights"])
    for k in want.files:
        if k == "weights":
            continue
        a, b = np.asarray(got[k]), want[k]
        assert a.shape == b.shape, k
        if a.dtype == np.bool_:
            assert np.array_equal(a, b), k
        else:
            np.testing.assert_allclose(a, b, rtol=0, atol=1e-6, err_msg=f"{name}:{k}")
    out = want["out"]
    assert np.isfinite(out).all() and out.std() > 0  # a non-trivial image
