"""GPU plumbing check of batch.ChunkedGather at world size 1 over RCCL (side
stream, event waits, pinned size copies, all_gather on the side stream); the
point-to-point part needs two GPUs and is covered by the gloo tests."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "yuv-manipulations-2_amd")]
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import batch  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29533")
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
s1 = torch.cuda.Stream(dev)
pay = torch.randint(0, 256, (10, 4096), dtype=torch.uint8, device=dev)
sizes = torch.tensor([100 + 37 * i for i in range(10)], dtype=torch.int32, device=dev)
g = batch.ChunkedGather(dist, 1, 0, dev)
for i0 in range(0, 10, 3):
    with torch.cuda.stream(s1):
        pay[i0:i0 + 3].add_(1)  # "compression" of the chunk on another stream
    ev = torch.cuda.Event()
    ev.record(s1)
    local = list(range(i0, min(i0 + 3, 10)))
    g.add(local, [pay[i] for i in local], sizes[i0:i0 + 3], [ev])
out = g.finish(10)
torch.cuda.synchronize(dev)
ok = all(torch.equal(out[i], pay[i][: 100 + 37 * i]) for i in range(10))
print("chunked gather world=1:", "OK" if ok else "MISMATCH")
dist.destroy_process_group()
sys.exit(0 if ok else 1)
