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
  nohbm    the 2^14 tiles read and write only four tiles' worth of addresses (L2-resident; output
           wrong): the butterflies + LDS exchanges + L2 traffic without HBM, to set against the
           full pass and reps0 (HBM only) -- how much of compute and data movement overlaps
  desync1/2/3  the first blocks on each CU (one launch's first wave) start staggered: block k of a
           CU (its arrival order, from a per-CU atomic counter) sleeps k x 1/2/3 x 8128 cycles, so
           co-resident blocks of the tile / mid kernels leave the load -> compute -> store lockstep
           they start in (tests whether compute and HBM phases of co-resident blocks overlap)

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

DESYNC = ("__device__ uint32_t g_cu_arrivals[4096];\n"
          "__device__ __forceinline__ void desync_first_wave(uint32_t* word) {\n"
          "  const uint32_t per_cu = 2048u / blockDim.x;\n"
          "  if (blockIdx.y * gridDim.x + blockIdx.x >= 256u * per_cu) return;\n"
          "  if (threadIdx.x == 0) {\n"
          "    uint32_t hw, xcc;\n"
          "    asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\" : \"=s\"(hw));\n"
          "    asm volatile(\"s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)\" : \"=s\"(xcc));\n"
          "    const uint32_t cu = ((xcc & 15u) << 8) | ((hw >> 8) & 0xffu);\n"
          "    word[0] = atomicAdd(&g_cu_arrivals[cu], 1u) % per_cu;\n"
          "  }\n"
          "  __syncthreads();\n"
          "  const uint32_t k = word[0];\n"
          "  __syncthreads();\n"
          "  for (uint32_t i = 0; i < k * DESYNC_UNIT; i++) __builtin_amdgcn_s_sleep(127);\n"
          "}\n")


def desync(unit):
    return [
        ("ntt.hip", "constexpr int TILE_LOG = 12;", f"constexpr uint32_t DESYNC_UNIT = {unit};\n" + DESYNC + "constexpr int TILE_LOG = 12;"),
        ("ntt.hip", "  uint32_t x[E];\n  if constexpr (DIN) {", "  uint32_t x[E];\n  desync_first_wave(lds);\n  if constexpr (DIN) {"),
        ("ntt.hip", "  uint32_t x[16];\n  int done_lo = 0;", "  uint32_t x[16];\n  desync_first_wave(lds);\n  int done_lo = 0;"),
    ]


PATCHES = {
    "nohbm": [
        ("ntt.hip", "  const uint32_t* S = src + (size_t)blockIdx.y * src_stride + ((size_t)blockIdx.x << B);\n"
                    "  uint32_t* D = dst + (size_t)blockIdx.y * dst_stride + ((size_t)blockIdx.x << B);",
         "  const uint32_t* S = src + ((size_t)(blockIdx.x & 3) << B);\n"
         "  uint32_t* D = dst + ((size_t)(blockIdx.x & 3) << B);  (void)src_stride; (void)dst_stride;"),
    ],
    "desync1": desync(1),
    "desync2": desync(2),
    "desync3": desync(3),
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
