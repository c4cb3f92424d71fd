import os, sys
sys.path.insert(0, os.getcwd())
import hwbloomradixjoin_amd as hw
L = hw.lib()
import torch
print("torch avail", torch.cuda.is_available(), torch.cuda.device_count(), flush=True)
t = torch.empty((1000, 2), dtype=torch.int32, device="cuda")
print("devcount lib", L.hwbrj_device_count(), flush=True)
try:
    hw.generate_device(t, 2, 1000, 1000, 1.0, 1)
    print("gen ok", flush=True)
except Exception as e:
    print("gen fail", e, flush=True)
