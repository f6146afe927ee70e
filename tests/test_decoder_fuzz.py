"""Untrusted-bytes robustness of the host decoders (host-only contexts):
the raw log decoder (hsc_logdec.cpp, bdb/llog.src layouts, and the physical
records its index-key reconstruction walks, berkdb/db/db.src) and the
OSQL_SERIAL wire decoder (hsc_wire.cpp, db/osqlcomm.c:909-993) fed valid
streams with random byte flips, truncations and length-field damage must
either decode or return an error -- never read out of bounds.  Run plainly
here and under ASan + UBSan by tests/test_sanitize.py."""
import numpy as np
import pytest

from comdb2_amd import formats as F
from comdb2_amd.hsc import HscError, Validator
from comdb2_amd.workloads import random_case


@pytest.fixture(scope="module")
def host():
    v = Validator(-1)
    yield v
    v.close()


def mutate(buf: np.ndarray, rng, n_flips: int) -> np.ndarray:
    b = buf.copy()
    for _ in range(n_flips):
        i = int(rng.integers(0, len(b)))
        b[i] = rng.integers(0, 256)
    return b


@pytest.mark.parametrize("seed", range(6))
def test_raw_log_mutations(host, seed):
    log, _ = random_case(500 + seed, n_commits=40)
    raw = F.encode_raw(log)
    rng = np.random.default_rng(seed)
    for k in range(60):
        r = F.RawLog(lsn=raw.lsn, off=raw.off.copy(), len=raw.len.copy(),
                     buf=mutate(raw.buf, rng, int(rng.integers(1, 16))), end_lsn=raw.end_lsn,
                     recon_lsn=raw.recon_lsn, recon_off=raw.recon_off, recon_len=raw.recon_len,
                     recon_keys=raw.recon_keys)
        if k % 3 == 0:  # shorten some records (a DBT or field running past the end)
            i = rng.integers(0, len(r.len), size=4)
            r.len[i] = np.maximum(r.len[i] // 2, 0)
        try:
            host.decode_raw(r)
        except HscError:
            pass


@pytest.mark.parametrize("seed", range(6))
def test_physical_log_mutations(host, seed):
    """Raw logs whose keyless index keys come from the physical records
    (formats.encode_raw_physical: addrem / big / pg_free chains walked by the
    key reconstruction, bdb/rowlocks.c:209-617), with byte flips inside the
    physical records' headers, item headers (BKEYDATA / BOVERFLOW lengths) and
    chain LSNs, and shortened records."""
    log, _ = random_case(550 + seed, n_commits=40, keylens=(9, 30))
    raw = F.encode_raw_physical(log, seed=seed, overflow=0.5)
    phys = np.nonzero(np.isin([int.from_bytes(bytes(raw.buf[int(o):int(o) + 4]), "big")
                               for o in raw.off], [41, 43, 47, 49, 50, 52]))[0]
    rng = np.random.default_rng(seed)
    for k in range(60):
        b = raw.buf.copy()
        for _ in range(int(rng.integers(1, 8))):  # flips inside physical records
            i = int(phys[int(rng.integers(0, len(phys)))])
            o = int(raw.off[i]) + int(rng.integers(0, int(raw.len[i])))
            b[o] = rng.integers(0, 256)
        r = F.RawLog(lsn=raw.lsn, off=raw.off.copy(), len=raw.len.copy(), buf=b,
                     end_lsn=raw.end_lsn, recon_lsn=raw.recon_lsn, recon_off=raw.recon_off,
                     recon_len=raw.recon_len, recon_keys=raw.recon_keys)
        if k % 3 == 0:
            i = phys[rng.integers(0, len(phys), size=3)]
            r.len[i] = np.maximum(r.len[i] - rng.integers(1, 12, size=3).astype(np.uint32), 16)
        try:
            host.decode_raw(r)
        except HscError:
            pass


@pytest.mark.parametrize("seed", range(6))
def test_wire_mutations(host, seed):
    _, rs = random_case(600 + seed, n_txn=30)
    buf, off, ln = F.encode_serial(rs)
    rng = np.random.default_rng(seed)
    for k in range(60):
        b = mutate(buf, rng, int(rng.integers(1, 24)))
        ln2 = ln.copy()
        if k % 4 == 0:
            i = rng.integers(0, len(ln2), size=3)
            ln2[i] = ln2[i] // 3
        try:
            host.decode_serial((b, off, ln2))
        except HscError:
            pass
