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
# round 6, late: more LDS lookups in flight at 3 waves per SIMD (the kernels
# hold 140-167 VGPRs of the 170 that occupancy allows): the multiply by H
# with its 8 lookups of a word issued together (4 groups, not 8), the Shoup
# multiply by H^m likewise, and both (correct output)
_POS4 = """    for (int h = 0; h < 8; h += 4) {
      // (an empty asm the next reads' addresses depend on, after the last
      // XORs: keeps the unrolled reads from being hoisted into 128 VGPRs)
      asm volatile("" : "+v"(w), "+v"(z0), "+v"(z1), "+v"(z2), "+v"(z3));
      const uint32_t w4 = w << 4;
      u32x4 e[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int jj = h + j;
        const uint32_t off = (((jj & 1) ? w : w4) >> (8 * (jj >> 1))) & 0xF0u;
        const char *p = base + 256 * (8 * i + jj) + off;
        e[j] = *(const u32x4 *)p;
      }
#pragma unroll
      for (int j = 0; j < 4; j += 2) {"""
_POS8 = _POS4.replace("h += 4", "h += 8").replace("u32x4 e[4];", "u32x4 e[8];").replace(
    "j < 4; j++", "j < 8; j++").replace("j < 4; j += 2", "j < 8; j += 2")
_SH4 = """    for (int h = 0; h < 8; h += 4) {  // (4 reads in flight: 8 made the kernels spill)
      u32x4 e[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int jj = h + j;
        const uint32_t off = ((((jj & 1) ? w : w4) >> (8 * (jj >> 1))) & 0xF0u) ^ sw16;
        if (GLOBAL) e[j] = gld<u32x4>((uint64_t)(t + off));
        else e[j] = *(const u32x4 *)(t + off);
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {"""
_SH8 = _SH4.replace("h += 4", "h += 8").replace("u32x4 e[4];", "u32x4 e[8];").replace(
    "j < 4; j++) {\n        const int jj", "j < 8; j++) {\n        const int jj").replace(
    "#pragma unroll\n      for (int j = 0; j < 4; j++) {\n        if", "#pragma unroll\n      for (int j = 0; j < 8; j++) {\n        if")
_SH8 = _SH8.replace("      for (int j = 0; j < 4; j++) {\n        const int jj", "      for (int j = 0; j < 8; j++) {\n        const int jj")
_SH8 = _SH8[:_SH8.rindex("j < 4; j++) {")] + "j < 8; j++) {"
SETS["ilp"] = {"base": [], "pos8": [(_POS4, _POS8)], "shoup8": [(_SH4, _SH8)],
               "both8": [(_POS4, _POS8), (_SH4, _SH8)]}
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
