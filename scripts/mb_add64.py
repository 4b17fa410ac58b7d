"""Dev microbenchmark: cycles per instruction group for 64-bit add forms."""
import ctypes, os
import torch
L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "libmb.so"))
out = torch.zeros(1 << 20, dtype=torch.int64, device="cuda")
cyc = torch.zeros(4096, dtype=torch.int64, device="cuda")
for waves_per_simd in (1, 4):
    for mode, name in ((0, "lshl_add_u64"), (1, "add_co+addc"), (2, "xor64"), (3, "rot64")):
        blocks = 256 * waves_per_simd
        L.mb_run(mode, blocks, 256, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cyc.data_ptr()))
        L.mb_run(mode, blocks, 256, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(cyc.data_ptr()))
        c = cyc[:blocks].double().mean().item()
        print(f"waves/SIMD {waves_per_simd} {name:14s} {c / (256 * 8):6.2f} cycles per 64-bit op (per wave)")
