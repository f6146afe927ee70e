"""GPU replicant coalesce (hsc_coalesce_readsets, comdb2_amd/csrc/hsc_coalesce.hip)
against oracle/coalesce_oracle.c (itself cross-checked against the Python
model in tests/test_coalesce.py): random read sets full of corner cases,
many small sets and a few very large ones."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
from coalesce_model import as_rows, random_readsets  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,ntxn,maxr", [(1, 300, 40), (2, 2000, 12), (3, 4, 3000),
                                            (4, 1, 20000)])
def test_gpu_coalesce_matches_oracle(validator, oracle_mod, seed, ntxn, maxr):
    rs = random_readsets(seed, ntxn=ntxn, max_ranges=maxr)
    want = oracle_mod.coalesce(rs)
    got = validator.coalesce(rs)
    assert list(got.txn_off) == list(want.txn_off)
    assert as_rows(got) == as_rows(want)
    assert len(got.table) < len(rs.table)  # something merged


def test_gpu_coalesce_empty(validator, oracle_mod):
    rs = random_readsets(5, ntxn=10, max_ranges=1)  # every set empty
    got = validator.coalesce(rs)
    assert list(got.txn_off) == [0] * 11
