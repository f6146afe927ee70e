"""Host submission cost of hsc_probe_device: time to enqueue K config-2
batches (no synchronisation inside the loop) vs. the device time of the same
K batches."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bench import upload_batch, probe_struct
from comdb2_amd import hsc
from comdb2_amd.workloads import config2, config2_device_window

dev = torch.device("cuda", 0)
v = hsc.Validator(0)
v.register_group("t1", 0, 9)
c2 = config2(build_log=False)
gid, words, lsn = config2_device_window(c2)
tg = torch.from_numpy(gid).to(dev); tw = torch.from_numpy(words.reshape(-1).view(np.int64)).to(dev)
tl = torch.from_numpy(lsn.view(np.int64)).to(dev)
v.ingest_device(len(lsn), 2, tg.data_ptr(), tw.data_ptr(), tl.data_ptr(), c2.params["end_lsn"])
b = upload_batch(torch, dev, v.marshal(c2.readsets))
T = c2.readsets.ntxn
streams = [torch.cuda.current_stream(), torch.cuda.Stream(device=dev)]
outs = [(torch.zeros(T, dtype=torch.uint8, device=dev), torch.zeros((T + 63) // 64, dtype=torch.int64, device=dev)) for _ in streams]
structs = [probe_struct(hsc, b, *o, T) for o in outs]
for K in (10, 200):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        v.set_stream(streams[k % 2].cuda_stream)
        v.probe_device(structs[k % 2])
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"K={K}: submit {1e6 * (t1 - t0) / K:.1f} us/batch, total {1e6 * (t2 - t0) / K:.1f} us/batch")
