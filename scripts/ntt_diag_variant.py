"""Builds a DIAGNOSTIC variant of libbfz.so into zkvm-brainfuck_amd/variants/<name>/libbfz.so by
patching a scratch copy of csrc/ (the product sources stay untouched).  Diagnostic outputs are
wrong by construction: they exist to time one ingredient of the NTT kernels.

  twconst  every twiddle-table load of the NTT windows (r16_window's table loads, the base
           twiddle of the strided passes, load_window_tw's prefetch) is replaced by an opaque
           register value: bounds what the table loads cost
  noexch   the 2^14 / small tile passes skip the LDS exchanges between windows (every window
           works on the registers the previous one left): compute + HBM only
  reps0    the tile passes do no butterflies at all: HBM -> (LDS) -> HBM data movement only
  syncmalloc  the device pool waits for the GPU to go idle before every hipMalloc: tests whether
           the first proof's long launches (kernel_outliers.py) are stalls caused by the pool
           growing while kernels run

usage: python3 scripts/ntt_diag_variant.py <name> [<name> ...]
Then run a program against it with LD_LIBRARY_PATH=zkvm-brainfuck_amd/variants/<name>
(scripts/ubench_ntt has a RUNPATH, which LD_LIBRARY_PATH overrides).
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "zkvm-brainfuck_amd")

DIAG_TW = ("__device__ __forceinline__ uint32_t diag_tw(int l) {\n"
           "  uint32_t z = 0x2345671u * (uint32_t)(l + 1) % 0x7f000001u;\n"
           "  asm volatile(\"\" : \"+v\"(z));\n"
           "  return z;\n"
           "}\n")

PATCHES = {
    "twconst": [
        ("ntt_dev.h", "constexpr uint32_t G24 = cpow(3, 127);", DIAG_TW + "constexpr uint32_t G24 = cpow(3, 127);"),
        ("ntt_dev.h", "tws[l] = ld_b(rt, off, ((1u << (s0 + g0 + kk)) + ((uint32_t)l << (g0 + s0))) * 4u);",
         "tws[l] = diag_tw(l); (void)rt; (void)off;"),
        ("ntt_dev.h", "const uint32_t wb = tw[(1u << (s0 + t)) + (m_low << s0) + lo_g];",
         "const uint32_t wb = diag_tw(t);"),
        ("ntt_dev.h", "pre[(1 << kk) - 1 + l] = ld_b(rsrc_of(tw), m_low * 4u, ((1u << (g0 + kk)) + ((uint32_t)l << g0)) * 4u);",
         "pre[(1 << kk) - 1 + l] = diag_tw(l);"),
    ],
    "noexch": [
        ("ntt.hip", "    if (!DIN || w > 0) {\n      if (WS && w > 0",
         "    if (!DIN && w == 0) {\n      if (WS && w > 0"),
        ("ntt.hip", "    } else {\n#pragma unroll\n      for (int i = 0; i < E; i++) lds[pb + (i << g0) + ((i << g0) >> R)] = x[i];",
         "    } else if (w == NW - 1) {\n#pragma unroll\n      for (int i = 0; i < E; i++) lds[pb + (i << g0) + ((i << g0) >> R)] = x[i];"),
    ],
    "syncmalloc": [
        ("gpu.h", "    void* p = nullptr;\n    HIP_CHECK(hipMalloc(&p, bytes));",
         "    void* p = nullptr;\n    HIP_CHECK(hipDeviceSynchronize());\n    HIP_CHECK(hipMalloc(&p, bytes));"),
    ],
    "reps0": [
        ("ntt.hip", "    if (g0 == 0)\n      r16_window<DIF, true, false, R>",
         "    if (kk_lo > 99)\n      r16_window<DIF, true, false, R>"),
        ("ntt.hip", "    else if (TWPF)\n      r16_window<DIF, false, true, R, true>",
         "    else if (TWPF && kk_lo > 99)\n      r16_window<DIF, false, true, R, true>"),
        ("ntt.hip", "    else\n      r16_window<DIF, false, true, R>(x, g0, kk_lo, kk_hi, 0, m_low, 0, tw);",
         "    else if (kk_lo > 99)\n      r16_window<DIF, false, true, R>(x, g0, kk_lo, kk_hi, 0, m_low, 0, tw);"),
    ],
}


def build(name):
    if name not in PATCHES:
        raise SystemExit(f"unknown variant {name}: {sorted(PATCHES)}")
    tmp = os.path.join(ROOT, ".scratch", f"diag_{name}")
    shutil.rmtree(tmp, ignore_errors=True)
    os.makedirs(os.path.join(tmp, "zkvm-brainfuck_amd"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    for d in ("csrc", "bfz"):
        shutil.copytree(os.path.join(PKG, d), os.path.join(tmp, "zkvm-brainfuck_amd", d))
    shutil.copy(os.path.join(PKG, "Makefile"), os.path.join(tmp, "zkvm-brainfuck_amd"))
    for fname, old, new in PATCHES[name]:
        path = os.path.join(tmp, "zkvm-brainfuck_amd", "csrc", fname)
        src = open(path).read()
        if src.count(old) != 1:
            raise SystemExit(f"{name}: patch anchor not found exactly once in {fname}: {old[:60]!r}")
        open(path, "w").write(src.replace(old, new))
    subprocess.run(["make", "-s", "-j16", "-C", os.path.join(tmp, "zkvm-brainfuck_amd"), "libbfz.so"],
                   check=True)
    out = os.path.join(PKG, "variants", name)
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(tmp, "zkvm-brainfuck_amd", "libbfz.so"), os.path.join(out, "libbfz.so"))
    shutil.rmtree(tmp)
    print(f"built {out}/libbfz.so")


if __name__ == "__main__":
    for n in sys.argv[1:]:
        build(n)
