"""Pin and free 8 x 8000 MiB of host memory (what the N = 8 rehearsal's configs[4] leaves behind), so a
following run can show whether fragmented pinned memory slows zero-copy reads (round 5: it does not)."""
import torch, time
bufs = []
for i in range(8):
    t = torch.empty(8000 << 20, dtype=torch.uint8, pin_memory=True)
    t.fill_(1)
    bufs.append(t)
del bufs
print("pinned 8 x 8000 MiB and freed", flush=True)
