"""Device-resident batches (hsc_probe_device) on several HIP streams.

The context keeps one probe lane (scratch buffers) per stream, so batches on
different streams run concurrently; a stream that takes over another
stream's lane first waits for the lane's last batch.  Every verdict must
still equal the oracle's (oracle/serial_oracle.c): batches are interleaved
over 2 streams with no synchronisation between launches, and over more
streams than there are lanes."""
import numpy as np
import pytest

from comdb2_amd import formats as F
from comdb2_amd import hsc
from comdb2_amd.formats import LogBuilder, Range, ReadSets

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def one_log_two_batches(seed, n_commits=20000, per_commit=6, n_txn=3000, ranges=8):
    """One index of int64 keys and two independent read-set batches over it."""
    rng = np.random.default_rng(seed)
    lb = LogBuilder()
    commits = [lb.next_lsn()]
    for c in range(n_commits):
        lb.begin(c)
        for _ in range(per_commit):
            lb.write(c, F.REC_UNDO_UPD_IX, "t1", 0, F.enc_int64(int(rng.integers(0, 1 << 30))))
        commits.append(lb.commit(c))
    log = lb.build()
    recent = max(1, len(commits) // 20)
    batches = []
    for _ in range(2):
        sets, snaps = [], []
        for _ in range(n_txn):
            rs = []
            for _ in range(ranges):
                a = int(rng.integers(0, 1 << 30))
                w = int(rng.integers(0, 1 << 16)) if rng.random() < 0.5 else 0
                rs.append(Range("t1", 0, F.enc_int64(a), F.enc_int64(a + w)))
            sets.append(rs)
            snaps.append(commits[len(commits) - 1 - int(rng.integers(0, recent))])
        batches.append(ReadSets.from_lists(sets, snaps, tbnames=lb.tbnames))
    return log, batches


def upload(dev, m):
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return dict(lo=t(m["lo"]), hi=t(m["hi"]), gid=t(m["gid"]), snap=t(m["snap"]),
                txn=t(m["txn"]), n=m["n"], lock_table=t(m["lock_table"]),
                lock_snap=t(m["lock_snap"]), lock_txn=t(m["lock_txn"]), n_lock=m["n_lock"],
                n_txn=m["n_txn"], forced=m["forced"])


def probe_struct(b, verdict, bitmap):
    return hsc.ProbeBatch(b["n"], b["lo"].data_ptr(), b["hi"].data_ptr(), b["gid"].data_ptr(),
                          b["snap"].data_ptr(), b["txn"].data_ptr(), b["n_lock"],
                          b["lock_table"].data_ptr(), b["lock_snap"].data_ptr(),
                          b["lock_txn"].data_ptr(), b["n_txn"], verdict.data_ptr(),
                          bitmap.data_ptr())


@pytest.mark.parametrize("nstreams", [1, 2, 6])
def test_streams_interleaved_match_oracle(validator, oracle_mod, nstreams):
    dev = torch.device("cuda", 0)
    log, batches = one_log_two_batches(7 + nstreams)
    want = [oracle_mod.check(log, rs, nthreads=8)[0] != 0 for rs in batches]
    v = validator
    v.ingest_log(log)
    ms = [v.marshal(rs) for rs in batches]
    ups = [upload(dev, m) for m in ms]
    streams = [torch.cuda.Stream(device=dev) for _ in range(nstreams)]
    # outputs per (stream, batch) so that nothing but the lanes is shared
    outs = {}
    for si in range(nstreams):
        for bi, u in enumerate(ups):
            T = u["n_txn"]
            outs[si, bi] = (torch.full((T,), 7, dtype=torch.uint8, device=dev),
                            torch.zeros((T + 63) // 64, dtype=torch.int64, device=dev))
    torch.cuda.synchronize()
    try:
        order = [(k % nstreams, (k // nstreams + k) % 2) for k in range(6 * nstreams)]
        for si, bi in order:
            v.set_stream(streams[si].cuda_stream)
            v.probe_device(probe_struct(ups[bi], *outs[si, bi]))
        torch.cuda.synchronize()
    finally:
        v.set_stream(0)
    ran = {key for key in order}
    for si, bi in ran:
        verdict, bitmap = outs[si, bi]
        got = np.maximum(verdict.cpu().numpy(), ms[bi]["forced"]) != 0
        np.testing.assert_array_equal(got, want[bi], err_msg=f"stream {si} batch {bi}")
        bits = np.unpackbits(bitmap.cpu().numpy().view(np.uint8), bitorder="little")[:len(got)]
        np.testing.assert_array_equal(bits.astype(bool), verdict.cpu().numpy() != 0)
    assert sum(int(w.sum()) for w in want) > 0


@pytest.mark.parametrize("layout", ["tiles", "auto"])
def test_tile_path_bitmap_equals_verdict(validator, oracle_mod, layout):
    """The tile pipeline builds the verdict bitmap itself (k_plan_s writes the
    locate's flags as whole words, the join ORs its hits in; no pack pass):
    a bitmap holding garbage from before must come back equal to the verdict
    bytes, and the bytes to the oracle's verdicts."""
    from comdb2_amd.hsc import LAYOUT_AUTO, LAYOUT_NARROW_TILES
    dev = torch.device("cuda", 0)
    log, batches = one_log_two_batches(31, n_txn=4000, ranges=10)
    want = [oracle_mod.check(log, rs, nthreads=8)[0] != 0 for rs in batches]
    v = validator
    v.set_layout(LAYOUT_NARROW_TILES if layout == "tiles" else LAYOUT_AUTO)
    try:
        v.ingest_log(log)
        for bi, rs in enumerate(batches):
            m = v.marshal(rs)
            u = upload(dev, m)
            T = u["n_txn"]
            verdict = torch.full((T,), 7, dtype=torch.uint8, device=dev)
            bitmap = torch.full(((T + 63) // 64,), -1, dtype=torch.int64, device=dev)
            for _ in range(2):  # the second pass over the first one's outputs
                v.probe_device(probe_struct(u, verdict, bitmap))
                torch.cuda.synchronize()
                got = np.maximum(verdict.cpu().numpy(), m["forced"]) != 0
                np.testing.assert_array_equal(got, want[bi])
                bits = np.unpackbits(bitmap.cpu().numpy().view(np.uint8), bitorder="little")[:T]
                np.testing.assert_array_equal(bits.astype(bool), verdict.cpu().numpy() != 0)
    finally:
        v.set_layout(LAYOUT_AUTO)


def test_window_change_waits_for_other_streams(validator, oracle_mod):
    """Lane fences are recorded when the context leaves a stream: a batch
    probed on stream A, then a switch to stream B and a window rebuild there,
    must still finish against the old window (the rebuild waits on A's lane),
    and probes after the rebuild see the new one -- on A and on B."""
    dev = torch.device("cuda", 0)
    log1, b1 = one_log_two_batches(101)
    log2, b2 = one_log_two_batches(202)
    want1 = [oracle_mod.check(log1, rs, nthreads=8)[0] != 0 for rs in b1]
    want2 = [oracle_mod.check(log2, rs, nthreads=8)[0] != 0 for rs in b2]
    v = validator
    sa, sb = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    try:
        v.ingest_log(log1)
        ms = [v.marshal(rs) for rs in b1]
        ups = [upload(dev, m) for m in ms]
        outs = [(torch.zeros(u["n_txn"], dtype=torch.uint8, device=dev),
                 torch.zeros((u["n_txn"] + 63) // 64, dtype=torch.int64, device=dev)) for u in ups]
        torch.cuda.synchronize()
        v.set_stream(sa.cuda_stream)
        v.probe_device(probe_struct(ups[0], *outs[0]))
        v.probe_device(probe_struct(ups[1], *outs[1]))
        v.set_stream(sb.cuda_stream)      # leaves A: its lane's fence goes onto A
        v.ingest_log(log2)                # the rebuild on B waits for A's batches
        ms2 = [v.marshal(rs) for rs in b2]
        ups2 = [upload(dev, m) for m in ms2]
        outs2 = [(torch.zeros(u["n_txn"], dtype=torch.uint8, device=dev),
                  torch.zeros((u["n_txn"] + 63) // 64, dtype=torch.int64, device=dev)) for u in ups2]
        torch.cuda.synchronize()
        v.probe_device(probe_struct(ups2[0], *outs2[0]))  # on B
        v.set_stream(sa.cuda_stream)
        v.probe_device(probe_struct(ups2[1], *outs2[1]))  # on A, after the rebuild
        torch.cuda.synchronize()
        for i in range(2):
            got = np.maximum(outs[i][0].cpu().numpy(), ms[i]["forced"]) != 0
            np.testing.assert_array_equal(got, want1[i], err_msg=f"old window batch {i}")
            got2 = np.maximum(outs2[i][0].cpu().numpy(), ms2[i]["forced"]) != 0
            np.testing.assert_array_equal(got2, want2[i], err_msg=f"new window batch {i}")
    finally:
        v.set_stream(0)
