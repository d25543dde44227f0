import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import torch, bench, maxio_amd
ctx = maxio_amd.Context(device_mask=1)
dev = torch.device("cuda", 0)
s = torch.cuda.Stream(device=dev)
w = bench.Mixed(torch, ctx, dev, s.cuda_stream, 24 << 30, bench.SEED)
torch.cuda.synchronize()
for _ in range(2): w.step()
torch.cuda.synchronize()
# host enqueue time of the encode half and the reconstruct half
t0 = time.perf_counter()
for (k, m, S, n, t, dl, pres) in w.classes:
    ctx.encode_strided_device(k, m, S, n, t.data_ptr(), (k + m) * S, S, t[:, k:].data_ptr(), (k + m) * S, S, data_len=dl, stream=s.cuda_stream)
t1 = time.perf_counter()
torch.cuda.synchronize(); t2 = time.perf_counter()
for (k, m, S, n, t, dl, pres) in w.classes:
    pr = pres.copy()
    ctx.reconstruct_strided_device(k, m, S, n, t.data_ptr(), (k + m) * S, S, pr, shard_len=dl + [S] * m, stream=s.cuda_stream)
t3 = time.perf_counter()
torch.cuda.synchronize(); t4 = time.perf_counter()
print("encode enqueue ms", (t1-t0)*1e3, "encode total ms", (t2-t0)*1e3)
print("recon enqueue ms", (t3-t2)*1e3, "recon total ms", (t4-t2)*1e3)
for (k, m, S, n, t, dl, pres) in w.classes: print(k, m, S, n)
