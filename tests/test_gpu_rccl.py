"""GPU: the RCCL branches of comdb2_amd/shard.py on a one-rank "nccl"
process group (the multi-GPU runs belong to the driver; the gloo rehearsals
in test_dist_gloo.py cover the N > 1 data flow): the device all_gather of
sampled_splitters, the all_to_all_single of exchange_rows, the all_reduce of
allreduce_table_max and the all_gather_into_tensor of gather_bitmaps, then a
config-5 check over the exchanged rows with the bitmap merged through
hsc_or_bitmaps equals the unsharded verdicts."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def nccl_group():
    import torch.distributed as dist
    torch.cuda.set_device(0)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


def test_world1_collectives_run_on_rccl(nccl_group):
    dist = nccl_group
    from comdb2_amd import shard
    from comdb2_amd.workloads import config5_scaled, int64_words
    from comdb2_amd.hsc import Validator
    assert dist.get_backend() == "nccl"
    c5 = config5_scaled(keys_per_gpu=200_000, n_txn=2000)
    sp = shard.sampled_splitters(c5.keys, c5.range_keys, 1, 0, shard.ROW_COST, shard.RANGE_COST,
                                 samples=1024)
    assert len(sp["splitters"]) == 0
    keys, lsn = shard.exchange_rows(c5.keys, c5.lsn, sp["splitters"])
    # one rank owns everything: the exchange keeps every row (order kept: one owner)
    np.testing.assert_array_equal(keys, c5.keys)
    np.testing.assert_array_equal(lsn, c5.lsn)
    tmax = shard.allreduce_table_max(np.array([lsn.max()], np.uint64))
    assert int(tmax[0]) == int(lsn.max())

    dev = torch.device("cuda", 0)
    v = Validator(0)
    try:
        assert v.register_group("t1", 0, 9) == 0
        words = int64_words(keys)
        tg = torch.from_numpy(np.zeros(len(keys), np.uint32)).to(dev)
        tw = torch.from_numpy(np.ascontiguousarray(words).reshape(-1).view(np.int64)).to(dev)
        tl = torch.from_numpy(lsn.view(np.int64)).to(dev)
        v.ingest_device(len(lsn), words.shape[0], tg.data_ptr(), tw.data_ptr(), tl.data_ptr(),
                        c5.end_lsn)
        torch.cuda.synchronize()
        v.merge_table_max(tmax)
        want = v.check_readsets(c5.readsets) != 0
        assert 0 < int(want.sum()) < len(want)
        # the bench's N > 1 merge at world 1: verdict bits packed, all-gathered
        # into the [world x words] tensor, OR-ed on the device
        T = c5.readsets.ntxn
        W64 = (T + 63) // 64
        bits = np.zeros(W64 * 8, np.uint8)
        bits[: (T + 7) // 8] = np.packbits(want, bitorder="little")
        lb = torch.from_numpy(bits.view(np.int64).copy()).to(dev)
        gath = torch.zeros(W64, dtype=torch.int64, device=dev)
        shard.gather_bitmaps(lb, gath)
        out = torch.zeros(W64, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        v.or_bitmaps(gath.data_ptr(), 1, W64, out.data_ptr())
        v.synchronize()
        got = np.unpackbits(out.cpu().numpy().view(np.uint8), bitorder="little")[:T] != 0
        np.testing.assert_array_equal(got, want)
    finally:
        v.close()
