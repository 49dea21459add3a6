"""Phase stamps of the EPnP-5 latency chain (k_epnp5_a / k_epnp5_jacobi_b / k_epnp5_c, first
hypothesis of the round): copies the library sources to /tmp, inserts s_memrealtime stamps (100 MHz)
at fixed anchors, builds build/ab/librsac_eptrace.so; k_epnp5_c's thread 0 prints the deltas.
The product sources stay unchanged.

    python3 scripts/ubench/epnp_trace.py
    RSAC_LIB_PATH=$PWD/build/ab/librsac_eptrace.so python3 scripts/trace_ms_to_best.py epnp5 opencv
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
T = "/tmp/eptrace"

MATH = [
    ("#define RSAC_TRACE_MARK(red, phase) ((void)0)\n#endif\n",
     "#define RSAC_TRACE_MARK(red, phase) ((void)0)\n#endif\n"
     "static __device__ unsigned long long g_ep_ts[64];\n"
     "#if defined(__HIP_DEVICE_COMPILE__)\n"
     "#define EPM(i) do { if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) "
     "g_ep_ts[i] = __builtin_amdgcn_s_memrealtime(); } while (0)\n"
     "#else\n#define EPM(i) ((void)0)\n#endif\n"),
    ("    const double n = s4[3];\n", "    const double n = s4[3];\n    EPM(3);\n"),
    ("    }, cov);\n", "    }, cov);\n    EPM(4);\n"),
    ("    const EpnpAlpha af = epnp_alpha_frame(f);\n    red.template sum<kEpnpPairSums / 2>",
     "    EPM(5);\n    const EpnpAlpha af = epnp_alpha_frame(f);\n    red.template sum<kEpnpPairSums / 2>"),
    ("    }, s1.pairs + kEpnpPairSums / 2);\n", "    }, s1.pairs + kEpnpPairSums / 2);\n    EPM(7);\n"),
    ("    householder_ls<6, 5>(A, b, x);\n    if (approx == 1) {",
     "    EPM(18);\n    householder_ls<6, 5>(A, b, x);\n    EPM(19);\n    if (approx == 1) {"),
    ("    if (ok) epnp_gauss_newton(L, rho, be);\n    return ok;",
     "    EPM(20);\n    if (ok) epnp_gauss_newton(L, rho, be);\n    EPM(21);\n    return ok;"),
    ("    }, H);\n    if (!epnp_rotation(H, Rk)) return false;",
     "    }, H);\n    EPM(23);\n    if (!epnp_rotation(H, Rk)) return false;\n    EPM(24);"),
    ("    err = es / n;\n    return true;", "    err = es / n;\n    EPM(25);\n    return true;"),
]
KERN = [
    ("    const int8_t st = epnp5_sample(a, rec, h, n, idx);\n    EpnpStage1 s1;",
     "    EPM(0);\n    const int8_t st = epnp5_sample(a, rec, h, n, idx);\n    EPM(1);\n    EpnpStage1 s1;"),
    ("        epnp5_reducer(q, red, c);\n", "        epnp5_reducer(q, red, c);\n        EPM(2);\n"),
    ("    *reinterpret_cast<EpnpStage1 *>(a.epnp + ((int64_t)prob * H + hl) * kEpnpRec) = s1;\n",
     "    *reinterpret_cast<EpnpStage1 *>(a.epnp + ((int64_t)prob * H + hl) * kEpnpRec) = s1;\n    EPM(8);\n"),
    ("    const bool live = hl < H && a.status[rec] > 0 && s1->ok != 0.0;  // wave-uniform\n    if (!live) return;\n"
     "    double *LA = L.A[hb], *LV = L.V[hb], *LP = L.part[hb];",
     "    EPM(10);\n    const bool live = hl < H && a.status[rec] > 0 && s1->ok != 0.0;  // wave-uniform\n"
     "    if (!live) return;\n    double *LA = L.A[hb], *LV = L.V[hb], *LP = L.part[hb];"),
    ("    ep_wave_sync();\n    for (int sweep = 0; sweep < 60; ++sweep) {\n        {  // row tr's",
     "    ep_wave_sync();\n    EPM(11);\n    int nsw = 0;\n    for (int sweep = 0; sweep < 60; ++sweep) {\n"
     "        nsw = sweep;\n        {  // row tr's"),
    ("        if (!(off > 1e-32 * diag)) break;\n        epnp_blk_sweep<0>",
     "        if (!(off > 1e-32 * diag)) break;\n        if (sweep == 0) EPM(12);\n        epnp_blk_sweep<0>"),
    ("        epnp_blk_sweep<0>(sweep, ba, bb, vr0, LA, LV, L.cs[hb]);\n",
     "        epnp_blk_sweep<0>(sweep, ba, bb, vr0, LA, LV, L.cs[hb]);\n        if (sweep == 0) EPM(13);\n"),
    ("    int *O = L.ord[hb];\n    if (lane == 0) {  // eig_order_desc<12> on the diagonal",
     "    EPM(14);\n    if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) g_ep_ts[40] = nsw;\n"
     "    int *O = L.ord[hb];\n    if (lane == 0) {  // eig_order_desc<12> on the diagonal"),
    ("        E[64 + lane] = LV[kEpR * j + O[11 - i]];\n    }\n}",
     "        E[64 + lane] = LV[kEpR * j + O[11 - i]];\n    }\n    EPM(15);\n}"),
    ("        epnp5_gather(a, p0, idx, q);\n        const EpnpStage1 s1",
     "        EPM(16);\n        epnp5_gather(a, p0, idx, q);\n        const EpnpStage1 s1"),
    ("            epnp_l_rho(s1, s2, L, rho);\n", "            EPM(17);\n            epnp_l_rho(s1, s2, L, rho);\n"),
    ("                epnp5_reducer(q, red, cen);\n", "                epnp5_reducer(q, red, cen);\n                EPM(22);\n"),
    ("    const int src = base + (win < 0 ? 0 : win);", "    EPM(26);\n    const int src = base + (win < 0 ? 0 : win);"),
    ("        if (ok && a.rvec_rt) rodrigues_roundtrip(R);\n        st = ok ? 1 : 0;",
     "        EPM(27);\n        if (ok && a.rvec_rt) rodrigues_roundtrip(R);\n        EPM(28);\n        st = ok ? 1 : 0;"),
    ("                     a.fconst + (int64_t)prob * kFconstStride, a.fmodels + rec * kFModelStride, a.fform);\n}\n\n"
     "// Small rounds",
     "                     a.fconst + (int64_t)prob * kFconstStride, a.fmodels + rec * kFModelStride, a.fform);\n"
     "    EPM(29);\n"
     "    if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) {\n"
     "        for (int i = 0; i < 30; ++i) if (g_ep_ts[i]) printf(\"ep %d %lld\\n\", i, (long long)(g_ep_ts[i] - g_ep_ts[0]));\n"
     "        printf(\"ep sweeps %llu\\n\", g_ep_ts[40]);\n"
     "        for (int i = 0; i < 64; ++i) g_ep_ts[i] = 0;\n    }\n}\n\n// Small rounds"),
]


def patch(path, edits):
    s = open(path).read()
    for old, new in edits:
        if s.count(old) != 1:
            sys.exit(f"anchor not found once in {os.path.basename(path)}: {old[:60]!r}")
        s = s.replace(old, new)
    open(path, "w").write(s)


shutil.rmtree(T, ignore_errors=True)
shutil.copytree(os.path.join(ROOT, "code-reproduction-ransac_amd", "csrc"), os.path.join(T, "x", "csrc"),
                ignore=shutil.ignore_patterns("build"))
shutil.copytree(os.path.join(ROOT, "include"), os.path.join(T, "include"))
patch(os.path.join(T, "x", "csrc", "rsac_math.h"), MATH)
patch(os.path.join(T, "x", "csrc", "rsac_kernels.hip"), KERN)
os.makedirs(os.path.join(ROOT, "build", "ab"), exist_ok=True)
out = os.path.join(ROOT, "build", "ab", "librsac_eptrace.so")
subprocess.run(["make", "-s", "-j8", "-C", os.path.join(T, "x", "csrc"), f"OUT={out}"], check=True,
               stderr=subprocess.DEVNULL)
print(out)
