"""Probe: does RCCL accept two ranks on one device in one process
(fa_comm_init(2, [0, 0]))?  If it does, the native 2-rank round is run and
compared with the single-GPU reduction (max |diff| in ULP-ish terms)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from feddct_amd import _lib  # noqa: E402
from feddct_amd import comm as C  # noqa: E402

torch.cuda.set_device(0)
devs = (ctypes.c_int * 2)(0, 0)
hs = (ctypes.c_void_p * 2)()
rc = C.lib().fa_comm_init(2, devs, hs)
print("fa_comm_init(2,[0,0]) rc", rc, _lib.lib.fa_last_error().decode(), flush=True)
