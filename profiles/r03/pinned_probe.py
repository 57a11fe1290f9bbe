"""Does hipPointerGetAttributes call a pageable buffer host memory once another buffer is registered?
(diagnosis of the pageable frame-verify rate)"""
import ctypes
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import annety_amd  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


class Attr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def attr(a):
    at = Attr()
    rc = hip.hipPointerGetAttributes(ctypes.byref(at), ctypes.c_void_p(a.ctypes.data))
    return rc, at.type


torch.zeros(1, device="cuda")
page = np.ones(1 << 30, dtype=np.uint8)
print("pageable alone:", attr(page), flush=True)
pin = annety_amd.PinnedHostBuffer(1 << 30)
print("pageable with a registered buffer alive:", attr(page), "registered:", attr(pin.array), flush=True)
d = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
for name in ("pageable", "registered"):
    src = page if name == "pageable" else pin.array
    t = torch.from_numpy(src)
    d.copy_(t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        d.copy_(t)
    torch.cuda.synchronize()
    print(name, "H2D", round(5 / (time.perf_counter() - t0), 2), "GiB/s", flush=True)
pin.close()
print("pageable after unregister:", attr(page), flush=True)
