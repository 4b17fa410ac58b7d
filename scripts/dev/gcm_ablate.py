"""Dev (container): ablation builds of the AES-128-GCM kernel -- each drops
one piece of the cooperative payload pass (the output is wrong; only the
time matters), so the GPU run of scripts/dev/gcm_ablate_run.sh attributes the
kernel's time: the Shoup multiply by H^m per chunk, the GHASH multiply per
block, the AES keystream per block pair.  Builds
build/ablate/<name>/libsqobfs.so from the in-tree objects plus a modified
copy of sq_quic_gcm.hip (nothing here ships; SQOBFS_LIB selects a build).
usage: python3 scripts/dev/gcm_ablate.py [set]   (set: ablate, the default;
occupancy: workgroup size / packets per wave variants, correct output)"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
PKG = os.path.join(REPO, "sing-quic_amd")
SRC = os.path.join(PKG, "csrc", "sq_quic_gcm.hip")
VARIANTS = {
    "base": [],
    "no_shoup": [("      if (m) KB.mul_pow(yb, m);", "")],
    "no_ghash": [("      ghash_absorb(y, g);\n      gmul_pos<KM == 1>(y, K.hpos);", "      ghash_absorb(y, g);")],
    "no_aes": [("    aes_encrypt_n<KM, 2>(K.rk, tT, tcol, s2);", "")],
}
SETS = {
    "ablate": VARIANTS,
    "occupancy": {
        "base": [],
        "w16p16": [("constexpr uint32_t kGBlock = 768;", "constexpr uint32_t kGBlock = 1024;"),
                   ("constexpr uint32_t kGPpw = 32;", "constexpr uint32_t kGPpw = 16;")],
        "w16p32": [("constexpr uint32_t kGBlock = 768;", "constexpr uint32_t kGBlock = 1024;")],
    },
}
SETS["shoup"] = {"e_sunroll": [("""#pragma unroll 1
  for (int i = 0; i < 4; i++) {
    const uint32_t w4 = w << 4;
    uint32_t z4 = 0;""", """#pragma unroll
  for (int i = 0; i < 4; i++) {
    asm volatile("" : "+v"(w), "+v"(z0), "+v"(z1), "+v"(z2), "+v"(z3));
    const uint32_t w4 = w << 4;
    uint32_t z4 = 0;""")]}
VARIANTS = SETS[sys.argv[1] if len(sys.argv) > 1 else "ablate"]
if not os.environ.get("KEEP"):  # (KEEP=1: add to scripts/dev/ab_head.sh's builds)
    shutil.rmtree(os.path.join(REPO, "build", "ablate"), ignore_errors=True)
objs = [os.path.join(PKG, "build", "obj", f + ".o")
        for f in ("sq_kernels", "sq_quic", "sq_api", "packet_conn", "udp_batch", "pconn", "sq_cpu")]
src = open(SRC).read()
for name, subs in VARIANTS.items():
    d = os.path.join(REPO, "build", "ablate", name)
    os.makedirs(d, exist_ok=True)
    s = src
    for a, b in subs:
        assert a in s, (name, a)
        s = s.replace(a, b)
    p = os.path.join(d, "sq_quic_gcm.hip")
    open(p, "w").write(s)
    flags = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-I" + os.path.join(REPO, "include"),
             "-I" + os.path.join(PKG, "csrc"), "-I" + os.path.join(PKG, "host")]
    subprocess.run(["/opt/rocm/bin/hipcc"] + flags + ["-c", "-o", os.path.join(d, "gcm.o"), p], check=True)
    subprocess.run(["/opt/rocm/bin/hipcc"] + flags + ["-shared", "-o", os.path.join(d, "libsqobfs.so"),
                    os.path.join(d, "gcm.o")] + objs + ["-lpthread"], check=True)
    print(name, "built", flush=True)
