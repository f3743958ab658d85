"""Diagnose HIP runtime sharing between torch and libmrt (order given by argv[1])."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
order = sys.argv[1] if len(sys.argv) > 1 else "torch-first"


def maps():
    return sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip" in l or "hsa-runtime" in l})


if order == "torch-first":
    import torch
    print("torch devices", torch.cuda.device_count(), torch.cuda.is_available())
    L = ctypes.CDLL(os.path.join(ROOT, "rendering-algorithms-raytracer_amd/lib/libmrt.so"))
    print("mrt devices", L.mrt_device_count())
else:
    L = ctypes.CDLL(os.path.join(ROOT, "rendering-algorithms-raytracer_amd/lib/libmrt.so"))
    print("mrt devices", L.mrt_device_count())
    import torch
    print("torch devices", torch.cuda.device_count(), torch.cuda.is_available())
    x = torch.ones(4, device="cuda")
    print("torch alloc ok", float(x.sum()))
print(order, maps())
