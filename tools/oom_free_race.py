"""Run tools/oom_free_race.hip's phases inside a process that has initialised torch on the GPU
(the round-4 segfault's setting: torch's HIP with libroctracer64 loaded).  Usage on the box:
    timeout -k 10 120 python -u tools/oom_free_race.py [phase_mask]   (1 oom, 2 race, 4 locked)"""
import ctypes
import os
import sys

import torch

torch.cuda.init()
x = torch.ones(1 << 20, device="cuda")      # torch's allocator and context are live
torch.cuda.synchronize()
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "liboom_free_race.so"))
rc = lib.oom_free_race(int(sys.argv[1]) if len(sys.argv) > 1 else 7)
print(f"oom_free_race rc={rc}", flush=True)
sys.exit(rc)
