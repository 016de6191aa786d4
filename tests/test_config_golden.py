"""TCI2 on the BASELINE configurations against committed golden results
(tests/golden/config_golden.json, made by tests/golden/make_config_golden.py from the oracle).

CPU: the oracle reproduces the fixture bitwise (the fixture is pinned data, not re-derived).
GPU: the product reproduces ranks, link dimensions and pivot sets exactly; errors bitwise for the
integer-exact Lorentzian and within 1e-10 (relative to maxsample) otherwise; interpolated values
within 1e-9 of maxsample at 64 fixed random points.
"""
import json
import os

import numpy as np
import pytest

import oracle_lib as O

GOLDEN = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                     "config_golden.json")))
NAMES = [c["name"] for c in GOLDEN]


def _cfg(name):
    return next(c for c in GOLDEN if c["name"] == name)


@pytest.mark.parametrize("name", [c["name"] for c in GOLDEN if c.get("cpu_check", True)])
def test_oracle_reproduces_config_golden(name):
    c = _cfg(name)
    t, ranks, errors = O.crossinterpolate2(c["kind"], c["params"], c["localdims"], c["initialpivots"], **c["kw"])
    r = c["result"]
    assert [int(x) for x in ranks] == r["ranks"]
    assert [float(e) for e in errors] == r["errors"]
    assert t.linkdims() == r["linkdims"]
    for p in range(len(c["localdims"])):
        assert t.Iset(p).tolist() == r["Iset"][p] and t.Jset(p).tolist() == r["Jset"][p]


@pytest.mark.gpu
@pytest.mark.parametrize("name", NAMES)
def test_gpu_matches_config_golden(name):
    T = pytest.importorskip("tci_amd")
    c = _cfg(name)
    r = c["result"]
    f = T.GPUBatchEvaluator(c["kind"], c["params"], c["localdims"])
    tci, ranks, errors = T.crossinterpolate2(f, c["localdims"], c["initialpivots"], nsearchglobalpivot=0,
                                             **c["kw"])
    assert list(ranks) == r["ranks"]
    assert tci.linkdims() == r["linkdims"]
    if c["kind"] == 1:
        # integer-exact integrand: the whole run is bitwise the oracle's
        for p in range(len(c["localdims"])):
            assert tci.Iset[p].tolist() == r["Iset"][p] and tci.Jset[p].tolist() == r["Jset"][p]
        assert list(errors) == r["errors"]
    else:
        # device exp/sin/pow differ from glibc by ulps, and quantics / Gaussian Pi matrices are
        # full of near-ties (the last legs move f by ~2^-40), so individual pivots may differ
        # while ranks, errors and the interpolant agree
        np.testing.assert_allclose(errors, r["errors"], rtol=0, atol=1e-10)
    got = tci.evaluate_many(np.asarray(r["points"], np.int32))
    np.testing.assert_allclose(got, r["values"], rtol=0, atol=1e-9 * r["maxsamplevalue"])
