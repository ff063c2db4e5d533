"""Which order of HIP runtime users works in one process: torch first or libbfz first."""
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "zkvm-brainfuck_amd"))
order = sys.argv[1]
if order == "torch_first":
    import torch
    x = torch.ones(4, device="cuda")
    print("torch ok", x.sum().item())
    from bfz import _lib
    _lib.init(0)
    print("bfz ok")
else:
    from bfz import _lib
    _lib.init(0)
    print("bfz ok")
    import torch
    x = torch.ones(4, device="cuda")
    print("torch ok", x.sum().item())
import ctypes
for l in open("/proc/self/maps"):
    if "amdhip64" in l:
        print(l.split()[-1])
        break
