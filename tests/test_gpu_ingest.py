"""GPU: the window build's sort + dedupe (hsc_ingest.hip packed-key sort and
the generic whole-row radix sort of hsc_kernels.hip) against numpy: every
version in stable (gid, key words) order and the newest version per key,
read back through hsc_window_export.  Cases cover one and several words,
several groups, varying bits scattered over the words, heavy duplication,
unsorted LSNs, block-boundary row counts and a window whose varying bits
plus row index do not fit 64 bits (the packed path declines it: the
compact-code merge sort of hsc_csort.hip takes it, config-3-like keys too);
the packed sort runs with its dedupe fused into the unpack and with the
separate flag / scan / compaction dedupe."""

import numpy as np
import pytest

from comdb2_amd.hsc import PATH_NO_PACKED_SORT, Validator

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _reference(gid, words, lsn):
    order = np.lexsort(tuple(words[j] for j in range(words.shape[0] - 1, -1, -1)) + (gid,))
    g, w, l = gid[order], words[:, order], lsn[order]
    same_next = np.ones(len(g), bool)
    same_next[-1] = False
    same_next[:-1] = (g[1:] == g[:-1]) & np.all(w[:, 1:] == w[:, :-1], axis=0)
    last = ~same_next
    return (g, w, l), (g[last], w[:, last], l[last])


def _case(rng, n, W, ngroups, pattern):
    gid = rng.integers(0, ngroups, n).astype(np.uint32)
    words = np.zeros((W, n), np.uint64)
    base = rng.integers(0, 1 << 63, W, dtype=np.uint64)
    for j in range(W):
        words[j] = base[j]
    if pattern == "low40":
        words[W - 1] = base[W - 1] & ~np.uint64((1 << 40) - 1) | rng.integers(0, 1 << 40, n, dtype=np.uint64)
    elif pattern == "dups":
        words[W - 1] = rng.integers(0, 97, n).astype(np.uint64) << np.uint64(17)
    elif pattern == "scattered":  # a few bits in every word
        for j in range(W):
            m = np.uint64(0x8000_0100_0040_1001 >> j)
            r = rng.integers(0, 1 << 63, n, dtype=np.uint64)
            words[j] = (base[j] & ~m) | (r & m)
    elif pattern == "wide":  # > 64 varying bits: the code sort (or the radix sort)
        for j in range(W):
            words[j] = rng.integers(0, 1 << 63, n, dtype=np.uint64)
    elif pattern == "c3":  # config-3-like: per-group key lengths, lumpy bytes, repeats
        klen = rng.integers(9, min(8 * W, 32) + 1, ngroups)  # <= 160 varying bits: 3 code words
        letters = np.array([0x41, 0x43, 0x47, 0x4B, 0x52, 0x53, 0x5A], np.uint8)
        pool = rng.integers(0, max(2, n // 3), n)  # about 3 versions per key
        kb = np.zeros((n, 8 * W), np.uint8)
        for g in range(ngroups):
            sel = gid == g
            r = np.random.default_rng(1000 + g)
            keys_g = letters[r.integers(0, 7, (max(2, n // 3), int(klen[g])))]
            kb[sel, :klen[g]] = keys_g[pool[sel] % len(keys_g)]
        words = np.ascontiguousarray(kb.view(">u8").astype(np.uint64).T)
    lsn = np.sort(rng.integers(1, 1 << 40, n, dtype=np.uint64))
    if pattern in ("dups", "scattered"):
        rng.shuffle(lsn)  # not in log order
    if pattern == "log":  # 24 varying key bits (with repeats), commit LSNs of a log:
        # file << 32 | 28 + 64 k, four rows per commit -- the LSNs' varying bits
        # fit beside the key's, so they ride in the sort key (no gather)
        words[W - 1] = (base[W - 1] & ~np.uint64((1 << 24) - 1)) | rng.integers(0, 1 << 20, n, dtype=np.uint64)
        k = np.arange(n, dtype=np.uint64) // np.uint64(4)
        lsn = (np.uint64(3) << np.uint64(32)) | (np.uint64(28) + np.uint64(64) * k)
    return gid, words, lsn


def _build(gid, words, lsn, ngroups, packed, path=None):
    # packed: the packed sort with the dedupe fused into its unpack (the
    # default when the varying bits fit) or, for wider varying bits, the
    # compact-code merge sort; False the whole-row radix sort
    try:
        v = Validator(0)
        v.set_paths(0 if packed else PATH_NO_PACKED_SORT)
        W = words.shape[0]
        for g in range(ngroups):
            assert v.register_group(f"t{g}", 0, 8 * W) == g
        dev = torch.device("cuda", 0)
        tg = torch.from_numpy(gid.copy()).to(dev)
        tw = torch.from_numpy(np.ascontiguousarray(words).reshape(-1).view(np.int64)).to(dev)
        tl = torch.from_numpy(lsn.view(np.int64)).to(dev)
        v.ingest_device(len(lsn), W, tg.data_ptr(), tw.data_ptr(), tl.data_ptr(), int(lsn.max()) + 1)
        torch.cuda.synchronize()
        out = v.export_window(True), v.export_window(False)
        if path is not None:
            path.append(v.sort_path)
        v.close()
        return out
    finally:
        pass


CASES = [
    (1, 1, 1, "low40"), (2, 1, 1, "dups"), (1000, 1, 1, "low40"), (8191, 1, 3, "dups"),
    (8192, 2, 1, "low40"), (8193, 1, 2, "scattered"), (100_000, 3, 5, "scattered"),
    (300_000, 1, 1, "dups"), (1 << 20, 1, 1, "low40"), (50_000, 2, 3, "wide"),
    (70_000, 5, 2, "scattered"), (300_000, 8, 32, "c3"), (5000, 8, 3, "c3"), (1025, 4, 2, "wide"),
    # the LSN in the sort key; >= 2M rows: the one-sweep passes (index / LSN in the low bits)
    (300_000, 1, 2, "log"), (2_500_000, 1, 1, "log"), (2_200_000, 1, 1, "low40"), (2_100_000, 2, 3, "scattered"),
]


@pytest.mark.parametrize("n,W,ngroups,pattern", CASES)
def test_build_rows_match_numpy(n, W, ngroups, pattern):
    rng = np.random.default_rng(n * 31 + W * 7 + ngroups)
    gid, words, lsn = _case(rng, n, W, ngroups, pattern)
    want_all, want_u = _reference(gid, words, lsn)
    for packed in (True, False):
        path = []
        got_all, got_u = _build(gid, words, lsn, ngroups, packed, path)
        if pattern in ("wide", "c3") and n > 1:  # codes when the varying bits fit 3 words
            fits = pattern == "c3" or W <= 2
            assert path == ["codes" if packed and fits else "radix"], path
        for got, want in ((got_all, want_all), (got_u, want_u)):
            np.testing.assert_array_equal(got[0], want[0])
            np.testing.assert_array_equal(got[1], want[1])
            np.testing.assert_array_equal(got[2], want[2])
