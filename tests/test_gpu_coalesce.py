"""GPU replicant coalesce (hsc_coalesce_readsets, comdb2_amd/csrc/hsc_coalesce.hip)
against oracle/coalesce_oracle.c (itself cross-checked against the Python
model in tests/test_coalesce.py): random read sets full of corner cases,
many small sets and a few very large ones."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(__file__))
from coalesce_model import as_rows, long_run_readsets, random_readsets  # noqa: E402

from comdb2_amd.hsc import PATH_CO_RUN_THREAD, PATH_CO_SERIAL  # noqa: E402

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


@pytest.mark.parametrize("seed,ntxn,lo,hi,null_lo,ntables", [
    (11, 6, 256, 3000, 0.0, 3),      # every set on the level-parallel path
    (12, 40, 200, 700, 0.0, 3),      # sizes either side of the threshold
    (13, 8, 300, 2000, 0.002, 3),    # some sets hold a tie-with-everything (NULL) lower key
    (14, 1, 60000, 60001, 0.0, 3),   # one deep set (16 merge levels)
    (15, 4, 3000, 9000, 0.0, 60),  # ~180 (table, index) runs per set, many locked tables
    (16, 4, 2000, 8000, 0.05, 3),    # NULL lower keys everywhere: glibc's merge tree replayed
    (17, 1, 60000, 60001, 0.03, 3),  # one deep set with ties (16 levels)
    (18, 3, 5000, 9000, 0.3, 2),     # ties dominate
])
def test_gpu_coalesce_large_sets(validator, oracle_mod, monkeypatch, seed, ntxn, lo, hi, null_lo,
                                 ntables):
    """Large sets take the level-parallel sort (hsc_coalesce.hip, CoBig; with
    NULL lower keys the replay of glibc's merge tree, CoTie): equal to the
    oracle and to the per-thread glibc-msort path (PATH_CO_SERIAL)."""
    rs = random_readsets(seed, ntxn=ntxn, max_ranges=hi, min_ranges=lo, null_lo=null_lo,
                         tables=tuple(f"t{i:02d}" for i in range(ntables)))
    want = oracle_mod.coalesce(rs)
    got = validator.coalesce(rs)
    assert list(got.txn_off) == list(want.txn_off)
    assert as_rows(got) == as_rows(want)
    validator.set_paths(PATH_CO_SERIAL)
    try:
        ser = validator.coalesce(rs)
    finally:
        validator.set_paths(0)
    assert as_rows(ser) == as_rows(want)


def test_gpu_coalesce_empty(validator, oracle_mod):
    rs = random_readsets(5, ntxn=10, max_ranges=1)  # every set empty
    got = validator.coalesce(rs)
    assert list(got.txn_off) == [0] * 11


@pytest.mark.parametrize("seed,ntxn,n,overlap", [(21, 2, 30000, 0.2), (22, 3, 5000, 0.9),
                                                 (23, 1, 70000, 0.0)])
def test_gpu_coalesce_long_runs(validator, oracle_mod, monkeypatch, seed, ntxn, n, overlap):
    """Sets that are one long (table, index) run: the merge scan splits into
    chunks stitched per run (k_run_local / k_run_stitch / k_run_pack); equal
    to the oracle, to one thread per run (PATH_CO_RUN_THREAD) and to the
    per-thread msort path (PATH_CO_SERIAL)."""
    rs = long_run_readsets(seed, ntxn=ntxn, n=n, overlap=overlap)
    want = oracle_mod.coalesce(rs)
    got = validator.coalesce(rs)
    assert list(got.txn_off) == list(want.txn_off)
    assert as_rows(got) == as_rows(want)
    try:
        for flags in (PATH_CO_RUN_THREAD, PATH_CO_SERIAL):
            validator.set_paths(flags)
            assert as_rows(validator.coalesce(rs)) == as_rows(want), flags
    finally:
        validator.set_paths(0)
