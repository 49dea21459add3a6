#!/usr/bin/env python3
"""Generate scripts/ubench/asm_mix.hip: the point loop of k_pnp_score_mf as hand-scheduled inline
asm, operands in registers, no memory.  One wave-iteration = 4 MFMA groups x
(2 v_mfma_f32_32x32x16_f16 + the VALU test of 4 slots x 2 pairs + each slot's band flag on the
scalar unit), the same instruction multiset as the compiler's loop (scripts/ubench/mf_mix.hip), in
an order chosen here:

  pipe  : group t + 1's two MFMAs issued at the start of group t's VALU (outputs ping-pong between
          two 32-register sets), so each result is read one group (64 VALU) after its MFMA
  now   : the compiler's order: a group's MFMAs, the 18 wait states a 16-pass XDL result needs
          before a VALU reads it, then the group's VALU
  nomfma: pipe without the MFMAs (the VALU/SALU ceiling of the same order)
  nosalu: nomfma without the scalar flag instructions (v_cmp kept)
  fma   : 256 independent v_fma_f32 per wave-iteration (the issue peak of this register layout)

Within a group the 4 slots' 64 VALU run stage by stage (q1 q2 of all 8 pairs, then q2^2, ...), so
consecutive instructions are independent.  Registers are fixed (v0-v155 clobbered): 168 VGPRs,
3 waves per SIMD, as the kernel.  Cycles come from s_memtime around the loop in every wave.
"""
import os
import sys

OUT = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "asm_mix.hip")

AR = 0        # v[0:15]   A operands of the 4 groups
BA, BB = 16, 20  # v[16:19], v[20:23] B operands of the two point tiles
UA, VA, UB, VB = 24, 25, 26, 27
AP = 28       # v[28:43]  a' of (t, g)
BP = 44       # v[44:59]  b' of (t, g)
VC = 60       # v[60:75]  255 x counts of (t, g)
X = (76, 108)  # two sets of 32: tile a outputs [0:16), tile b [16:32)
T = 140       # v[140:155] temporaries: 4 per slot
NV = 156


def mfma(t, par):
    x = X[par]
    return [f"v_mfma_f32_32x32x16_f16 v[{x}:{x + 15}], v[{AR + 4 * t}:{AR + 4 * t + 3}], v[{BA}:{BA + 3}], 0",
            f"v_mfma_f32_32x32x16_f16 v[{x + 16}:{x + 31}], v[{AR + 4 * t}:{AR + 4 * t + 3}], v[{BB}:{BB + 3}], 0"]


def group_valu(t, par, salu=True):
    """The 64 VALU (+ scalar flag ops) of group t reading output set `par`, stage by stage."""
    x = X[par]
    out = []
    za = lambda g: x + 4 * g + 2
    zb = lambda g: x + 16 + 4 * g + 2
    tmp = lambda g, k: T + 4 * g + k
    # q1, q2 of both pairs of every slot: T0 = q1a, T1 = q2a, T2 = q1b, T3 = q2b
    for g in range(4):
        out.append(f"v_fma_f32 v{tmp(g, 0)}, v{UA}, v{za(g)}, v{x + 4 * g}")
        out.append(f"v_fma_f32 v{tmp(g, 1)}, v{VA}, v{za(g)}, v{x + 4 * g + 1}")
        out.append(f"v_fma_f32 v{tmp(g, 2)}, v{UB}, v{zb(g)}, v{x + 16 + 4 * g}")
        out.append(f"v_fma_f32 v{tmp(g, 3)}, v{VB}, v{zb(g)}, v{x + 16 + 4 * g + 1}")
    for g in range(4):  # q2^2
        out.append(f"v_mul_f32_e32 v{tmp(g, 1)}, v{tmp(g, 1)}, v{tmp(g, 1)}")
        out.append(f"v_mul_f32_e32 v{tmp(g, 3)}, v{tmp(g, 3)}, v{tmp(g, 3)}")
    for g in range(4):  # + q1^2
        out.append(f"v_fmac_f32_e32 v{tmp(g, 1)}, v{tmp(g, 0)}, v{tmp(g, 0)}")
        out.append(f"v_fmac_f32_e32 v{tmp(g, 3)}, v{tmp(g, 2)}, v{tmp(g, 2)}")
    for g in range(4):  # D = . - z^2
        out.append(f"v_fma_f32 v{tmp(g, 1)}, -v{za(g)}, v{za(g)}, v{tmp(g, 1)}")
        out.append(f"v_fma_f32 v{tmp(g, 3)}, -v{zb(g)}, v{zb(g)}, v{tmp(g, 3)}")
    for g in range(4):  # t = |D| - a'|z|
        a = AP + 4 * t + g
        out.append(f"v_fma_f32 v{tmp(g, 0)}, -v{a}, |v{za(g)}|, |v{tmp(g, 1)}|")
        out.append(f"v_fma_f32 v{tmp(g, 2)}, -v{a}, |v{zb(g)}|, |v{tmp(g, 3)}|")
    for g in range(4):  # the count: sign bytes of Da, Db summed onto vc
        out.append(f"v_perm_b32 v{tmp(g, 1)}, v{tmp(g, 1)}, v{tmp(g, 3)}, s10")
    for g in range(4):
        out.append(f"v_sad_u8 v{VC + 4 * t + g}, v{tmp(g, 1)}, 0, v{VC + 4 * t + g}")
    for g in range(4):  # the band: min(ta, tb) <= b'
        out.append(f"v_min_f32_e32 v{tmp(g, 0)}, v{tmp(g, 0)}, v{tmp(g, 2)}")
    for g in range(4):
        out.append(f"v_cmp_ngt_f32_e64 s[{20 + 2 * g}:{21 + 2 * g}], v{tmp(g, 0)}, v{BP + 4 * t + g}")
    if salu:
        for g in range(4):
            bit = 1 << (4 * t + g)
            out.append(f"s_cmp_lg_u64 s[{20 + 2 * g}:{21 + 2 * g}], 0")
            out.append(f"s_cselect_b32 s{28 + g}, {bit}, 0")
            out.append(f"s_or_b32 s11, s11, s{28 + g}")
    return out


def body(mode):
    lines = []
    if mode == "fma":
        for k in range(256):
            d = T + (k % 16)
            lines.append(f"v_fma_f32 v{d}, v{UA}, v{X[0] + (k % 32)}, v{d}")
        return lines
    if mode in ("pipe", "nomfma", "nosalu"):
        for t in range(4):
            par = t & 1
            if mode == "pipe":
                lines += mfma((t + 1) % 4, par ^ 1)  # the next group's (iteration t = 3: group 0 of the next)
            lines += group_valu(t, par, salu=mode != "nosalu")
        return lines
    if mode == "now":
        for t in range(4):
            lines += mfma(t, 0)
            lines += ["s_nop 7", "s_nop 7", "s_nop 1"]
            lines += group_valu(t, 0)
        return lines
    raise ValueError(mode)


MODES = ["pipe", "now", "nomfma", "nosalu", "fma"]


def count_valu(lines):
    return sum(1 for l in lines if l.startswith("v_"))


def asm_block(mode):
    init = []
    for r in range(NV):
        init.append(f"v_mov_b32 v{r}, %[seed]")
    for r in range(AP, AP + 16):
        init.append(f"v_mul_f32 v{r}, 0x358637bd, v{r}")  # small slopes
    for r in range(BP, BP + 16):
        init.append(f"v_mov_b32 v{r}, 0xff800000")  # b' = -inf: no flags
    init += ["s_mov_b32 s10, 0x0c0c0b09", "s_mov_b32 s11, 0"]
    if mode == "pipe":
        init += mfma(0, 0)
    loop = ["s_mov_b32 s12, %[iters]", "s_memtime %[t0]", "s_waitcnt lgkmcnt(0)", "1:"]
    loop += body(mode)
    loop += ["s_sub_u32 s12, s12, 1", "s_cmp_lg_u32 s12, 0", "s_cbranch_scc1 1b", "s_memtime %[t1]",
             "s_waitcnt lgkmcnt(0)"]
    loop += [f"v_add_u32 %[res], v{VC}, v{VC + 5}", f"v_add_u32 %[res], %[res], v{T}"]
    text = "\\n\\t".join(init + loop)
    clob = ", ".join(f'"v{r}"' for r in range(NV)) + ', "s10", "s11", "s12", ' + \
        ", ".join(f'"s{r}"' for r in range(20, 32)) + ', "vcc", "scc"'
    return text, clob


def main():
    src = [f"// GENERATED by scripts/ubench/gen_asm_mix.py -- do not edit.\n{__doc__.replace('*/', '')}".replace(
        "\n", "\n// ").rstrip("/ ") + "\n",
           "#include <hip/hip_runtime.h>", "#include <cstdio>", "#include <cstdint>", "",
           "static constexpr int kIters = 2000;", ""]
    for i, m in enumerate(MODES):
        text, clob = asm_block(m)
        src += [f"// mode {m}: {count_valu(body(m))} VALU per wave-iteration (MFMA included)",
                f"__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_{m}("
                "uint32_t *out, uint64_t *cyc, float seedf) {",
                "    uint32_t res;", "    uint64_t t0, t1;",
                "    const float seed = seedf * (float)(threadIdx.x + 1);",
                f'    asm volatile("{text}"',
                '                 : [res] "=v"(res), [t0] "=s"(t0), [t1] "=s"(t1)',
                '                 : [seed] "v"(seed), [iters] "s"(kIters)',
                f"                 : {clob});",
                "    out[blockIdx.x * 256 + threadIdx.x] = res;",
                "    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;",
                "}", ""]
    src += ["int main() {",
            "    int cus = 0;",
            "    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);",
            "    uint32_t *out;", "    uint64_t *cyc;",
            "    (void)hipMalloc(&out, sizeof(uint32_t) * 256 * cus * 4);",
            "    (void)hipMalloc(&cyc, sizeof(uint64_t) * 4 * cus * 4);",
            "    uint64_t *h = new uint64_t[4 * cus * 4];",
            "    hipEvent_t e0, e1;", "    (void)hipEventCreate(&e0);", "    (void)hipEventCreate(&e1);",
            f"    const char *names[{len(MODES)}] = {{{', '.join(chr(34) + m + chr(34) for m in MODES)}}};",
            f"    const int valu[{len(MODES)}] = {{{', '.join(str(count_valu(body(m))) for m in MODES)}}};",
            f"    for (int m = 0; m < {len(MODES)}; ++m)",
            "        for (int bpc : {1, 2, 3}) {",
            "            const int blocks = cus * bpc;  // 4 waves per block, one per SIMD",
            "            auto launch = [&]() {",
            "                switch (m) {"]
    for i, m in enumerate(MODES):
        src.append(f"                    case {i}: hipLaunchKernelGGL(k_{m}, dim3(blocks), dim3(256), 0, 0, out, cyc, "
                   "0.999f); break;")
    src += ["                }",
            "            };",
            "            launch();",
            "            (void)hipDeviceSynchronize();",
            "            (void)hipEventRecord(e0);",
            "            for (int r = 0; r < 5; ++r) launch();",
            "            (void)hipEventRecord(e1);",
            "            (void)hipEventSynchronize(e1);",
            "            float ms = 0;",
            "            (void)hipEventElapsedTime(&ms, e0, e1);",
            "            ms /= 5;",
            "            (void)hipMemcpy(h, cyc, sizeof(uint64_t) * 4 * blocks, hipMemcpyDeviceToHost);",
            "            double s = 0;",
            "            for (int i = 0; i < 4 * blocks; ++i) s += (double)h[i];",
            "            const double wave_cyc = s / (4 * blocks) / kIters;  // one wave's cycles per iteration",
            "            const double simd_cyc = wave_cyc / bpc;  // per SIMD and wave-iteration (waves overlap)",
            "            const double per_quad = valu[m] / (simd_cyc / 4.0);",
            "            printf(\"%-7s waves/SIMD %d: %.3f ms, wave %6.0f cyc/iter, SIMD %6.0f cyc per wave-iteration, \"",
            "                   \"%.3f VALU per quad-cycle (%.3f of 2; %d VALU)\\n\",",
            "                   names[m], bpc, ms, wave_cyc, simd_cyc, per_quad, per_quad / 2, valu[m]);",
            "        }",
            "    return 0;",
            "}"]
    open(OUT, "w").write("\n".join(src) + "\n")


if __name__ == "__main__":
    main()
