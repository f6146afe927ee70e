"""Multi-GPU verdict merge primitive (hsc_or_bitmaps): the OR of N per-shard
verdict bitmaps after the all-gather, on the device, against numpy."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("nparts,words", [(1, 1), (2, 1563), (8, 12500), (3, 0)])
def test_or_bitmaps_matches_numpy(validator, nparts, words):
    rng = np.random.default_rng(nparts * 1000 + words)
    parts = rng.integers(0, 1 << 62, size=(nparts, words), dtype=np.int64)
    parts &= rng.integers(0, 1 << 62, size=(nparts, words), dtype=np.int64)  # sparse-ish bits
    dev = torch.device("cuda", 0)
    src = torch.from_numpy(parts.reshape(-1).copy()).to(dev)
    out = torch.full((max(words, 1),), -1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    validator.set_stream(0)
    validator.or_bitmaps(src.data_ptr(), nparts, words, out.data_ptr())
    validator.synchronize()
    want = np.bitwise_or.reduce(parts, axis=0) if words else np.zeros(0, np.int64)
    np.testing.assert_array_equal(out.cpu().numpy()[:words], want)
