"""Dev probe (GPU box): is a strided (2-D) host-to-device copy of fixed slots
as fast per useful byte as a contiguous one?  1M slots of 2,048 B in pinned
host memory, 1,358 used bytes per slot (a Salamander datagram of 1,350 B),
copied (a) whole, contiguous (2 GiB), (b) as hipMemcpy2DAsync rows of 1,358
B into a 1,408-byte device pitch, (c) 1.4 GB contiguous (the packed bytes).
Also the device-to-host direction."""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpy2DAsync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                 ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                 ctypes.c_int, ctypes.c_void_p]
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                               ctypes.c_void_p]
H2D, D2H = 1, 2
n, slot, used, pitch = 1 << 20, 2048, 1358, 1408
host = torch.empty(n * slot, dtype=torch.uint8).pin_memory()
dev = torch.empty(n * slot, dtype=torch.uint8, device="cuda")
s = torch.cuda.current_stream().cuda_stream


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


for name, kind in (("H2D", H2D), ("D2H", D2H)):
    def whole():
        a, b = (dev, host) if kind == H2D else (host, dev)
        assert hip.hipMemcpyAsync(a.data_ptr(), b.data_ptr(), n * slot, kind, s) == 0

    def packed():
        a, b = (dev, host) if kind == H2D else (host, dev)
        assert hip.hipMemcpyAsync(a.data_ptr(), b.data_ptr(), n * pitch, kind, s) == 0

    def rows():
        if kind == H2D:
            assert hip.hipMemcpy2DAsync(dev.data_ptr(), pitch, host.data_ptr(), slot, used, n,
                                        kind, s) == 0
        else:
            assert hip.hipMemcpy2DAsync(host.data_ptr(), slot, dev.data_ptr(), pitch, used, n,
                                        kind, s) == 0
    tw, tp, tr = t(whole), t(packed), t(rows)
    print(f"{name}: whole 2,048 B slots {tw * 1e3:7.2f} ms ({n * slot / tw / 1e9:5.1f} GB/s), "
          f"packed 1,408 B {tp * 1e3:7.2f} ms ({n * pitch / tp / 1e9:5.1f} GB/s), "
          f"2-D rows of 1,358 B {tr * 1e3:7.2f} ms ({n * used / tr / 1e9:5.1f} GB/s useful)",
          flush=True)
